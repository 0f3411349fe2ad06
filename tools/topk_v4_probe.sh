#!/bin/bash
# v4 top-K attribution on the GPU box: kernel trace of the library build (scan vs
# finish per launch), per-phase s_memtime cycles (RT_TOPK_PROBE_TIMING) and the
# scan with selection disabled (RT_TOPK_PROBE_NOSEL). Args: TAG NQ NX.
set -o pipefail
TAG=${1:-v4probe}; NQ=${2:-65536}; NX=${3:-125000}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
H=$R/tools/hip_probe
timeout -k 10 120 $H/topk_probe_BASE $NQ $NX 2 > $O/base.txt 2>&1 || { cat $O/base.txt; exit 1; }
cat $O/base.txt
timeout -k 10 120 $H/topk_probe_RT_TOPK_PROBE_TIMING $NQ $NX 2 > $O/timing.txt 2>&1 || { cat $O/timing.txt; exit 1; }
cat $O/timing.txt
timeout -k 10 120 $H/topk_probe_RT_TOPK_PROBE_NOSEL $NQ $NX 2 > $O/nosel.txt 2>&1 || { cat $O/nosel.txt; exit 1; }
cat $O/nosel.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- $H/topk_probe_BASE $NQ $NX 2 > $P/kt.log 2>&1 || { tail -20 $P/kt.log; exit 1; }
DB=$(find $P/kt -name "*.db" | head -1)
python3 $R/tools/prof_summary.py $DB --by-grid --title "v4 probe $NQ x $NX" > $O/kernel_shapes.md
cat $O/kernel_shapes.md
