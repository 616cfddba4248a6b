# round-6: CSR x-window kernel (MODE 3) y stores: store_y (agent-scope relaxed atomic store,
# product) vs plain stores (lab/libspmv_hip_plainy.so), cant-like single, events, one box
set -o pipefail
for r in 1 2 3; do
  timeout -k 10 200 python tools/cant_single.py --formats csr --flush-mode read > gpurun_out/ya_$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=$PWD/lab/libspmv_hip_plainy.so timeout -k 10 200 python tools/cant_single.py --formats csr --flush-mode read > gpurun_out/yp_$r.log 2>&1 || exit 1
done
echo ok
