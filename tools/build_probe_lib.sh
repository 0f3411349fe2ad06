#!/bin/bash
# Diagnostic library: librtrec_hip.so with the MLP phase probe compiled in
# (-DRT_PHASE_PROBE, csrc/mlp.hip), for tools/c2_phase_probe.py. Output:
# tools/hip_probe/librtrec_probe.so (git-ignored; travels to the GPU box).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/real-time-recommendation-system-with-feature-store_amd
make -s -C $P -j8
B=/tmp/rtrec_probe_build; mkdir -p $B
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-function \
  -I$R/include -I$P/csrc -DRT_PHASE_PROBE ${EXTRA_FLAGS} -c $P/csrc/mlp.hip -o $B/mlp.o
OBJS=$(ls $P/build/*.o | grep -v '/mlp.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $R/tools/hip_probe/librtrec_probe.so $OBJS $B/mlp.o
echo built $R/tools/hip_probe/librtrec_probe.so
