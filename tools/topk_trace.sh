#!/bin/bash
# rocprofv3 kernel trace (scan vs finish per launch) of top-K probe binaries
# on the C4 shard shape. Usage: topk_trace.sh TAG V1 V2 ...
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $P/$V -o kt -- $R/tools/hip_probe/topk_probe_$V 65536 125000 2 > $P/$V.log 2>&1 || { tail -20 $P/$V.log; exit 1; }
  DB=$(find $P/$V -name "*.db" | head -1)
  python3 $R/tools/prof_summary.py $DB --by-grid --title "topk_probe_$V 65536 x 125000 (k = 1, 10, 100; 4 calls each)" > $O/trace_$V.md
  cat $O/trace_$V.md
done
