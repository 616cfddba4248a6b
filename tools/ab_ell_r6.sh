# round-6: ELL small grids with the batched slot loop (product) vs the round-6 start
set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python tools/cant_single.py --formats ell,hyb --flush-mode read --extra 'ell@{"xwin": false}' > gpurun_out/prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=lab/libspmv_hip_r6base.so timeout -k 10 200 python tools/cant_single.py --formats ell,hyb --flush-mode read --extra 'ell@{"xwin": false}' > gpurun_out/base$r.log 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_drivers_gpu.py -m gpu -k "ell or hyb" > gpurun_out/t.log 2>&1 || exit 1
echo ok
