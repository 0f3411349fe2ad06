#!/bin/bash
# GPU-box check used during development: the 16-bit top-K parity tests first
# (fail fast), then the rest of the GPU suite, then the top-K A/B timing.
# Output under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-chk}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk16.py -x -v --timeout 200 --timeout-method thread > $O/pytest_topk16.log 2>&1 || { tail -40 $O/pytest_topk16.log; exit 1; }
tail -2 $O/pytest_topk16.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread --deselect tests/test_gpu_topk16.py > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u tools/topk_v4_bench.py 2 > $O/topk_bench.log 2>&1 || { tail -20 $O/topk_bench.log; exit 1; }
cat $O/topk_bench.log
