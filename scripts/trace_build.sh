#!/bin/bash
# Timing build of libdab with per-wave s_memrealtime stamps in k_eval_bal (-DDAB_TRACE)
# into scripts/trace/libdab.so (git-ignored; OUT= and EXTRA= flags for variants). Run here (hipcc cross-compiles); the .so
# travels with the tree. Used by scripts/trace_fused.py.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
SRC=$HERE/../deeparc-sfm_amd/csrc
OUT=${OUT:-$HERE/trace}
mkdir -p "$OUT"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -DDAB_TRACE $EXTRA"
pids=()
for f in dab_kernels dab_chol dab_pcg dab_solver dab_p2p dab_setup; do
  /opt/rocm/bin/hipcc $F -c "$SRC/$f.hip" -o "$OUT/$f.o" & pids+=($!)
done
for f in errors synth; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -x c++ -c "$SRC/$f.cpp" -o "$OUT/$f.o" & pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$OUT/libdab.so" "$OUT"/*.o -L/opt/rocm/lib -lrccl -lamdhip64 -Wl,-rpath,/opt/rocm/lib
rm -f "$OUT"/*.o
