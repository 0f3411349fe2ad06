#!/bin/bash
# GPU-box round profile: parity tests, the default bench line, a rocprofv3
# kernel trace of the same bench, and the HBM-traffic PMC passes (FETCH_SIZE,
# WRITE_SIZE in separate runs) of a short C2 bench. Small summaries land in
# gpurun_out/$TAG/ (copied into profiles/ by hand).
set -o pipefail
TAG=${1:-prof}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 $R/bench.py --cpu-budget 2 > $P/kt.log 2>&1 || { tail -20 $P/kt.log; exit 1; }
DB=$(find $P/kt -name "*.db" | head -1)
python3 $R/tools/prof_summary.py $DB --by-base --title "kernel families, full bench.py run incl. extras" > $O/kernel_families.md
python3 $R/tools/prof_summary.py $DB --by-grid --title "per launch shape, full bench.py run incl. extras" > $O/kernel_shapes.md
B="python3 $R/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/f -o f -- $B > $P/f.log 2>&1 || { tail -20 $P/f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/w -o w -- $B > $P/w.log 2>&1 || { tail -20 $P/w.log; exit 1; }
python3 $R/tools/pmc_dump.py $(find $P/f $P/w -name "*.db") --filter rt:: > $O/c2_traffic_pmc.txt
python3 $R/tools/prof_topk.py 100 3 > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/tf -o tf -- python3 $R/tools/prof_topk.py 100 2 > $P/tf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/tw -o tw -- python3 $R/tools/prof_topk.py 100 2 > $P/tw.log 2>&1 || exit 1
python3 $R/tools/pmc_dump.py $(find $P/tf $P/tw -name "*.db") --filter topk --calls 2 > $O/topk_c4_traffic_pmc.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $P/gf -o gf -- python3 $R/tools/prof_gather.py 2 > $P/gf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $P/gw -o gw -- python3 $R/tools/prof_gather.py 2 > $P/gw.log 2>&1 || exit 1
python3 $R/tools/pmc_dump.py $(find $P/gf $P/gw -name "*.db") --filter gather > $O/gather_c5_traffic_pmc.txt
TOPK_CALLS=2 python3 $R/tools/traffic_json.py $O/c2_traffic_pmc.txt $O/topk_c4_traffic_pmc.txt $O/gather_c5_traffic_pmc.txt > $O/traffic.json || true
ls -la $O
