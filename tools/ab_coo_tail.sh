# round-6: COO single pass, tail x gathered with the tile (product) vs in the products' branch (lab/libspmv_hip_r6base.so)
set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python tools/cant_single.py --formats coo,hyb --flush-mode read > gpurun_out/prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=lab/libspmv_hip_r6base.so timeout -k 10 200 python tools/cant_single.py --formats coo,hyb --flush-mode read > gpurun_out/base$r.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "coo or hyb" > gpurun_out/t.log 2>&1 || exit 1
echo ok
