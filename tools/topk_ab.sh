#!/bin/bash
# Interleaved A/B of top-K probe binaries (tools/hip_probe/topk_probe_<V>) on the
# GPU box: each variant at each corpus size, ROUNDS times, mode 2 (v4 forced).
# Output (times per k and output hashes) under gpurun_out/$TAG/ab.txt.
# Usage: topk_ab.sh TAG ROUNDS "NX1 NX2" V1 V2 ...  (V@MODE: that probe at
# rt_flatip_topk_tuning mode MODE instead of 2, e.g. NEW@18 = v4 without presample)
set -o pipefail
TAG=$1; ROUNDS=$2; NXS=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
for r in $(seq $ROUNDS); do
  for NX in $NXS; do
    for V in "$@"; do
      B=${V%@*}; M=2; [ "$B" != "$V" ] && M=${V#*@}
      echo "== $V nx=$NX round=$r" >> $O/ab.txt
      timeout -k 10 120 $R/tools/hip_probe/topk_probe_$B 65536 $NX $M >> $O/ab.txt 2>&1 || { echo "FAIL $V rc=$?" >> $O/ab.txt; cat $O/ab.txt; exit 1; }
    done
  done
done
cat $O/ab.txt
