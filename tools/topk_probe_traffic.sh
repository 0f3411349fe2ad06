#!/bin/bash
# FETCH_SIZE / WRITE_SIZE PMC passes (separate runs) over top-K probe binaries
# at the C4 shard shape, v4 forced (k = 1, 10, 100; per-kernel averages).
# Usage: topk_probe_traffic.sh TAG V1 V2 ...
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
P=/tmp/$TAG; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $C -d $P/$V.$C -o p -- $R/tools/hip_probe/topk_probe_$V 65536 125000 2 > $P/$V.$C.log 2>&1
    rc=$?; if [ $rc -ne 0 ]; then echo "$V $C rc=$rc"; tail -3 $P/$V.$C.log; exit 1; fi
  done
  python3 $R/tools/pmc_dump.py $(find $P -path "*$V.*" -name "*.db") --filter topk > $O/traffic_$V.txt
  echo "== $V"; cat $O/traffic_$V.txt
done
