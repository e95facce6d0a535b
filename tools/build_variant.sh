#!/bin/bash
# A/B diagnostics: build libkpsim with extra compile flags into tools/ab/<name>.so (objects under /tmp), e.g.
#   tools/build_variant.sh blockscan0 -DKP_TOPO_BLOCK_SCAN=0
set -euo pipefail
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/karpenter-provider-aws_amd
OUT=/tmp/kpvar_$NAME
mkdir -p "$OUT" "$ROOT/tools/ab"
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-result -Wno-unused-value -mllvm --amdgpu-sched-strategy=max-ilp $*"
pids=()
for f in kp_kernels kp_ffd_base kp_ffd_resv kp_ffd_pref kp_ffd_pref_resv kp_ffd_base_topo kp_ffd_resv_topo kp_ffd_pref_topo kp_ffd_pref_resv_topo kp_consolidate kp_launch; do
  /opt/rocm/bin/hipcc $FLAGS -c -o "$OUT/$f.o" "$PKG/csrc/$f.hip" & pids+=($!)
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $* -x hip -c -o "$OUT/kp_host.o" "$PKG/csrc/kp_host.cpp" & pids+=($!)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -c -o "$OUT/kp_ingest.o" "$PKG/csrc/kp_ingest.cpp" & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$ROOT/tools/ab/$NAME.so" "$OUT"/*.o
echo "built tools/ab/$NAME.so"
