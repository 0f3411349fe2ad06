#!/bin/bash
# Build librtrec_hip.so from the csrc/ and include/ of a git revision (or the
# working tree with REV=WORKTREE) into OUT, with optional extra hipcc flags —
# the library variants of tools/ab_libs.sh A/B runs.
# Usage: tools/build_lib_at.sh REV OUT [EXTRA_FLAGS...]
set -e
REV=$1; OUT=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/rtlib.XXXX)
PKG=real-time-recommendation-system-with-feature-store_amd
mkdir -p $T/csrc $T/include $T/obj
if [ "$REV" = WORKTREE ]; then
  cp $R/$PKG/csrc/* $T/csrc/; cp $R/include/* $T/include/
else
  git -C $R archive $REV $PKG/csrc include | tar -x -C $T
  mv $T/$PKG/csrc/* $T/csrc/
fi
pids=()
for f in $T/csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-function \
    -I$T/include -I$T/csrc "$@" -c $f -o $T/obj/$(basename $f .hip).o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "compile failed"; exit 1; }; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT.tmp $T/obj/*.o
# a kernel template whose host pass failed leaves its launch stub undefined
if nm -C $OUT.tmp | grep -q " U .*__device_stub__"; then echo "undefined kernel stubs in $OUT"; exit 1; fi
mv -f $OUT.tmp $OUT
rm -rf $T
echo built $OUT
