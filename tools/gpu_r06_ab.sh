#!/bin/bash
# round-6 development check: the changed GPU tests, the dropout diagnostic,
# then interleaved A/Bs: RTREC_W_PLANES on the C2 bench line, and the v4
# top-K scan with shared per-query candidate regions (BASE) against the
# per-half regions of round 5 (RT_TOPK_V4_PER_HALF). Output under gpurun_out/$TAG/.
set -o pipefail
TAG=${1:-r06ab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/diag/dropout_det.py > $O/dropout_det.txt 2>&1 || { tail -20 $O/dropout_det.txt; exit 1; }
cat $O/dropout_det.txt
timeout -k 10 600 python -u -m pytest ${FIRST:-tests/test_gpu_graph.py tests/test_gpu_c2_fullsize.py tests/test_gpu_model.py tests/test_gpu_dist.py tests/test_gpu_c5_scale.py} -x -v --timeout 250 --timeout-method thread $DESEL > $O/pytest_first.log 2>&1 || { tail -60 $O/pytest_first.log; exit 1; }
tail -3 $O/pytest_first.log
bash tools/ab_env.sh $TAG 3 RTREC_W_PLANES=0 RTREC_W_PLANES=1 || exit 1
bash tools/topk_ab.sh $TAG 2 "125000 1000000" BASE RT_TOPK_V4_PER_HALF > /dev/null || exit 1
grep -E "^==|k=100" $O/ab.txt | head -40
