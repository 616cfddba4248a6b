#!/usr/bin/env bash
# tools/build_variant.sh NAME ["-DMACRO=v ..."] : a lab build of
# libspmv_hip.so (lab/libspmv_hip_NAME.so, for SPMV_HIP_LIB=... A/B runs and
# diagnostics; never the product).  Extra defines apply to every source.
# NAME stamps_sell / stamps_csr / stamps_coo also inject tools/lab_stamps_{sell,csr,coo}.h
# into csrc/{sell,csr,staged}.hip (the per-wave phase stamps of tools/sell_stamps.py).
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
defs=${*:-}
d=build/var_$name
mkdir -p "$d" lab
pids=()
for f in opencl-spmv-algorithms_amd/csrc/*.hip; do
  base=$(basename "$f" .hip)
  inc=()
  if [ "$name" = stamps_sell ] && [ "$base" = sell ]; then inc=(-include tools/lab_stamps_sell.h); fi
  if [ "$name" = stamps_csr ] && [ "$base" = csr ]; then inc=(-include tools/lab_stamps_csr.h); fi
  if [ "$name" = stamps_coo ] && [ "$base" = staged ]; then inc=(-include tools/lab_stamps_coo.h); fi
  # shellcheck disable=SC2086
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude "${inc[@]}" $defs -c "$f" -o "$d/$base.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -O3 -fPIC --offload-arch=gfx950 -shared "$d"/*.o -o "lab/libspmv_hip_$name.so" \
  -Lopencl-spmv-algorithms_amd/lib -lspmv_host -Wl,-rpath,"$PWD/opencl-spmv-algorithms_amd/lib" -ldl
echo "lab/libspmv_hip_$name.so"
