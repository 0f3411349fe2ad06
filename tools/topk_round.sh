#!/bin/bash
# GPU-box check of a top-K change: the top-K parity tests, an interleaved A/B of
# probe binaries (tools/hip_probe/topk_probe_<V>, built beforehand on the CPU
# side), and the FETCH_SIZE / WRITE_SIZE passes of the C4 shard call.
# Usage: topk_round.sh TAG ROUNDS "NX1 NX2" V1 V2 ...
set -o pipefail
TAG=$1; ROUNDS=$2; NXS=$3; shift 3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_topk16.py tests/test_gpu_topk_bench_dist.py tests/test_gpu_retrieval.py tests/test_gpu_topk_dense.py tests/test_gpu_model.py \
  -s > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed|separated" $O/pytest.log | tail -5
bash $R/tools/topk_ab.sh $TAG $ROUNDS "$NXS" "$@" > /dev/null || { tail -20 $O/ab.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/prof_topk.py 100 2 > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 $R/tools/prof_topk.py 100 3 > $P/kt.log 2>&1 || { tail -20 $P/kt.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $P/kt -name "*.db" | head -1) --by-grid --title "C4 shard k=100, 3 calls" > $O/kt.md || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/tf -o tf -- python3 $R/tools/prof_topk.py 100 2 > $P/tf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/tw -o tw -- python3 $R/tools/prof_topk.py 100 2 > $P/tw.log 2>&1 || exit 1
python3 $R/tools/pmc_dump.py $(find $P/tf $P/tw -name "*.db") --filter topk --calls 2 > $O/topk_c4_traffic_pmc.txt
cat $O/ab.txt | grep -v "^$" | tail -40
cat $O/kt.md | head -30
cat $O/topk_c4_traffic_pmc.txt
