# round-6: COO single-pass tile (kCooR pairs per thread: 1,024 / 1,536 / 2,048 entries) on one
# cant-like matrix, product (R = 3) vs lab builds, two interleaved rounds, events, one box
set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python tools/cant_single.py --formats coo,hyb --flush-mode read > gpurun_out/r3_$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=$PWD/lab/libspmv_hip_coor2.so timeout -k 10 200 python tools/cant_single.py --formats coo,hyb --flush-mode read > gpurun_out/r2_$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=$PWD/lab/libspmv_hip_coor4.so timeout -k 10 200 python tools/cant_single.py --formats coo,hyb --flush-mode read > gpurun_out/r4_$r.log 2>&1 || exit 1
done
echo ok
