# round-6: COO lanes per row for long rows (mean >= 48): product L=8 vs lab L=4 / L=16
set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python tools/cant_single.py --formats coo --flush-mode read > gpurun_out/prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=lab/libspmv_hip_cool4.so timeout -k 10 200 python tools/cant_single.py --formats coo --flush-mode read > gpurun_out/l4_$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=lab/libspmv_hip_cool16.so timeout -k 10 200 python tools/cant_single.py --formats coo --flush-mode read > gpurun_out/l16_$r.log 2>&1 || exit 1
done
echo ok
