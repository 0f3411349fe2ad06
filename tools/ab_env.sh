#!/bin/bash
# A/B of environment switches on the C2 bench line (GPU box), interleaved:
#   tools/ab_env.sh TAG ROUNDS "VAR=a" "VAR=b" ...
# Each variant runs `bench.py --steps 200 --warmup 20 --no-extras --no-cpu-baseline`
# under `env <variant>`; one JSON line per run lands in gpurun_out/TAG/ab.jsonl.
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    line=$(env $v timeout -k 10 120 python -u bench.py --steps 200 --warmup 20 --no-extras --no-cpu-baseline 2> $O/ab_err.log) || { tail -20 $O/ab_err.log; exit 1; }
    ms=$(echo "$line" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "{\"env\": \"$v\", \"round\": $r, \"ms_per_step\": $ms}" | tee -a $O/ab.jsonl
  done
done
