#!/bin/bash
# rocprofv3 kernel trace of tools/emulate_c4_n8.py (the per-rank C4 work at N = 8).
set -o pipefail
TAG=${1:-emu}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $P/kt -o kt -- python3 $R/tools/emulate_c4_n8.py > $O/emu.json 2> $P/kt.log || { tail -20 $P/kt.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $P/kt -name "*.db" | head -1) --by-grid --title "C4 N=8 per-rank emulation" > $O/kt.md
cat $O/emu.json; head -30 $O/kt.md
