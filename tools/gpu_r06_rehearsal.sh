#!/bin/bash
# bench.py --gpus 2 / 4 rehearsed on a one-GPU box: every rank on cuda:0
# (RTREC_BENCH_SAME_GPU=1), collectives through gloo (RCCL refuses two ranks on
# one device). Times are not meaningful; the run checks that every N > 1 leg
# executes through the round-6 code (the index-class C4 leg included).
set -o pipefail
TAG=${1:-r06reh}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for N in 2 4; do
  RTREC_BENCH_SAME_GPU=1 RTREC_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_n$N.json 2> $O/bench_n$N.err || { tail -30 $O/bench_n$N.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_n$N.json').read().strip().splitlines()[-1]); e=d.get('extras',{}); print($N, d['ms_per_step'], json.dumps({k: (v.get('error') or v.get('ms_per_launch') or v.get('ms_per_step')) for k, v in e.items()}), json.dumps(e.get('topk_c4_1m_sharded',{}).get('global_threshold')))"
done
