# round-6: CSR x-window kernel chunk size (pairs per lane R) on one cant-like matrix, lab builds xr2/xr5/xr6
set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python tools/cant_single.py --formats csr,csr16 --flush-mode read > gpurun_out/prod$r.log 2>&1 || exit 1
  for v in xr2 xr5 xr6; do
    SPMV_HIP_LIB=lab/libspmv_hip_$v.so timeout -k 10 200 python tools/cant_single.py --formats csr,csr16 --flush-mode read > gpurun_out/$v$r.log 2>&1 || exit 1
  done
done
echo ok
