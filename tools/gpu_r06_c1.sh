#!/bin/bash
# C1 dz column split: parity tests, then an interleaved epoch-time A/B
# (RT_DZ_KSPLIT=1: no split; unset: automatic = split at C1) and a kernel trace.
set -o pipefail
TAG=${1:-r06c1}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_c1.py tests/test_gpu_c2_fullsize.py tests/test_gpu_graph.py tests/test_gpu_wplanes.py -x -q --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  RT_DZ_KSPLIT=1 timeout -k 10 200 python -u tools/c1_time.py 2 2>> $O/err.log | tee -a $O/ab.jsonl || exit 1
  timeout -k 10 200 python -u tools/c1_time.py 2 2>> $O/err.log | tee -a $O/ab.jsonl || exit 1
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d /tmp/c1kt -o kt -- python3 $R/tools/c1_time.py 1 > /tmp/c1kt.log 2>&1 || { tail -20 /tmp/c1kt.log; exit 1; }
python3 $R/tools/prof_summary.py $(find /tmp/c1kt -name "*.db" | head -1) --by-grid --title "C1 epoch, dz column split (auto)" > $O/c1_trace.md
grep -E "linear_bwd_dz|linear_fwd|linear_bwd_dw" $O/c1_trace.md | head -20
