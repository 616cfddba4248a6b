# round-6: SELL small kernel y stores plain (product) vs sc1 (lab build ysc1): trace + in-process
set -o pipefail
B="--format sell --batch no --per-format no --single no --rmat-strong no --banded-strong no --rmat-per-format no --sell-single no --cpu-seconds 0"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=lab/libspmv_hip_ysc1.so timeout -k 10 300 python bench.py $B > gpurun_out/ysc1$r.log 2>&1 || exit 1
done
SPMV_HIP_LIB=lab/libspmv_hip_stamps_sell.so timeout -k 10 200 python tools/sell_stamps.py --formats sell > gpurun_out/stamps_new.log 2>&1 || exit 1
echo ok
