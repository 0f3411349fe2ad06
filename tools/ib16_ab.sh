#!/bin/bash
# A/B of librtrec_hip.so variants on the C5 in-batch CE (tools/microbench_inbatch.py
# --c5), interleaved, then one kernel trace per variant (per-pass times).
#   tools/ib16_ab.sh TAG ROUNDS lib1.so lib2.so ...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    echo "== $lib round $r" >> $O/ab.txt
    RTREC_HIP_LIB=$R/$lib timeout -k 10 120 python3 $R/tools/microbench_inbatch.py --c5 >> $O/ab.txt 2> $O/ab_err.log || { tail -20 $O/ab_err.log; exit 1; }
  done
done
cat $O/ab.txt
cd /tmp && export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1))
  RTREC_HIP_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $P/kt$i -o kt -- python3 $R/tools/microbench_inbatch.py --c5 > $P/kt$i.log 2>&1 || { tail -20 $P/kt$i.log; exit 1; }
  python3 $R/tools/prof_summary.py $(find $P/kt$i -name "*.db" | head -1) --title "$lib" > $O/kt$i.md || exit 1
  grep -E "ib16" $O/kt$i.md | cut -c1-160
done
