#!/bin/bash
# round-6 GPU check: the new/changed GPU tests first (fail fast), then the
# whole GPU suite and a default bench line. Output under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-r06}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest ${FIRST:-tests/test_gpu_dist.py tests/test_gpu_graph.py tests/test_gpu_c5_scale.py} -x -v --timeout 250 --timeout-method thread > $O/pytest_first.log 2>&1 || { tail -60 $O/pytest_first.log; exit 1; }
tail -3 $O/pytest_first.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
