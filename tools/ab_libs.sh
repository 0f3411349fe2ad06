#!/bin/bash
# A/B of librtrec_hip.so variants on the C2 bench line (GPU box), interleaved:
#   tools/ab_libs.sh TAG ROUNDS lib1.so lib2.so ...
# Each variant runs `bench.py --no-extras --no-cpu-baseline` through
# RTREC_HIP_LIB; one JSON line per run lands in gpurun_out/TAG/ab.jsonl.
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    line=$(RTREC_HIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-extras --no-cpu-baseline 2> $O/ab_err.log) || { tail -20 $O/ab_err.log; exit 1; }
    ms=$(echo "$line" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "{\"lib\": \"$lib\", \"round\": $r, \"ms_per_step\": $ms}" | tee -a $O/ab.jsonl
  done
done
