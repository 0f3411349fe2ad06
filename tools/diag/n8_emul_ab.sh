#!/bin/bash
# The C4 N = 8 per-rank emulation (bench.topk_c4_n8_emulated) under several
# library builds, interleaved: tools/diag/n8_emul_ab.sh TAG ROUNDS lib1.so lib2.so ...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    RTREC_HIP_LIB=$R/$lib timeout -k 10 240 python -u -c "
import json, torch, bench
e = bench.topk_c4_n8_emulated(torch.device('cuda:0'))
print(json.dumps({'lib': '$lib', 'round': $r, **{k: round(v, 3) for k, v in e.items() if isinstance(v, float)}}))
" >> $O/n8.jsonl 2> $O/n8_err.log || { tail -20 $O/n8_err.log; exit 1; }
  done
done
cat $O/n8.jsonl
