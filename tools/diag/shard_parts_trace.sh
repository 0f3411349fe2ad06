#!/bin/bash
# Kernel traces of tools/diag/shard_parts.py under two library builds.
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for l in "$@"; do
  b=$(basename $l .so)
  RTREC_HIP_LIB=$R/$l timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $P/$b -o kt -- python3 $R/tools/diag/shard_parts.py > $P/$b.log 2>&1 || { tail -20 $P/$b.log; exit 1; }
  tail -1 $P/$b.log
  DB=$(find $P/$b -name "*.db" | head -1)
  python3 $R/tools/prof_summary.py $DB --by-grid --title "shard_parts $b" > $O/trace_$b.md
  grep topk $O/trace_$b.md | head -20
done
