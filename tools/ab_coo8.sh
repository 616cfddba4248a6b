# round-6: COO single pass with 8-bit row keys on 2,048-entry tiles (product) vs the int32-key
# single pass (lab/libspmv_hip_coo32.so = the tree before it), cant-like single, events, one box
set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python tools/cant_single.py --formats coo --flush-mode read > gpurun_out/k8_$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=$PWD/lab/libspmv_hip_coo32.so timeout -k 10 200 python tools/cant_single.py --formats coo --flush-mode read > gpurun_out/k32_$r.log 2>&1 || exit 1
done
echo ok
