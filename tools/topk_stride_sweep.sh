#!/bin/bash
# Sample-stride sweep of the v4 plan on the probe binary (k = 100 lines are the
# ones the (stride, rank) pairs are sized for): tools/topk_stride_sweep.sh TAG
# ROUNDS "NX" "ST:R ST:R ...". Output under gpurun_out/$TAG/sweep.txt.
set -o pipefail
TAG=$1; ROUNDS=$2; NXS=$3; PAIRS=$4
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for NX in $NXS; do
    for P in $PAIRS; do
      echo "== stride:rank $P nx=$NX round=$r" >> $O/sweep.txt
      timeout -k 10 120 $R/tools/hip_probe/topk_probe_BASE 65536 $NX 2 ${P%:*} ${P#*:} >> $O/sweep.txt 2>&1 || { echo "FAIL $P rc=$?" >> $O/sweep.txt; cat $O/sweep.txt; exit 1; }
    done
  done
done
grep -E "^==|k=100" $O/sweep.txt
