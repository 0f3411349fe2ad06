#!/bin/bash
# Effective shader clock during the C5 in-batch passes: GRBM_GUI_ACTIVE (GPU
# busy cycles per dispatch) next to the kernel-trace durations, plus MFMA busy.
#   tools/ib16_clock.sh TAG [lib]
TAG=$1; LIB=${2:-}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
[ -n "$LIB" ] && export RTREC_HIP_LIB=$R/$LIB
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES -d $P/c1 -o c -- python3 $R/tools/microbench_inbatch.py --c5 > $P/c1.log 2>&1 || { tail -5 $P/c1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 $R/tools/microbench_inbatch.py --c5 > $P/kt.log 2>&1 || { tail -5 $P/kt.log; exit 1; }
python3 $R/tools/pmc_dump.py $(find $P/c1 -name "*.db") --filter ib16 > $O/clock_pmc.txt
python3 $R/tools/prof_summary.py $(find $P/kt -name "*.db" | head -1) --title "ib16 clock run" > $O/clock_kt.md
cat $O/clock_pmc.txt; grep ib16 $O/clock_kt.md | cut -c1-150
