#!/bin/bash
# GPU-box attribution of the C4 top-K kernel: kernel-trace durations at
# k = 1, 10, 100 and SQ/TCC counter passes (one rocprofv3 --pmc run each) at
# k = 1 and k = 100. Summaries land in gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-topk_pmc}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/prof_topk.py 100 1 > /dev/null || exit 1
for K in 1 10 100; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $P/kt$K -o kt -- python3 $R/tools/prof_topk.py $K 3 > $P/kt$K.log 2>&1 || { tail -20 $P/kt$K.log; exit 1; }
  python3 $R/tools/prof_summary.py $(find $P/kt$K -name "*.db" | head -1) --by-base --title "top-K k=$K" > $O/kt_k$K.md || exit 1
done
PASSES=(
  "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
  "SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_LDS_IDX_ACTIVE"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
for K in 1 100; do
  i=0
  for C in "${PASSES[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $C -d $P/pk${K}_$i -o p -- python3 $R/tools/prof_topk.py $K 2 > $P/p${K}_$i.log 2>&1 || { tail -20 $P/p${K}_$i.log; exit 1; }
  done
  python3 $R/tools/pmc_dump.py $(find $P/pk${K}_* -name "*.db") --filter topk > $O/pmc_k$K.txt || exit 1
done
