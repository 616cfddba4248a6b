# round-6: SELL small kernel y stores plain (product) vs non-temporal (lab build ynt)
set -o pipefail
B="--format sell --batch no --per-format no --single no --rmat-strong no --banded-strong no --rmat-per-format no --sell-single no --cpu-seconds 0"
for r in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=lab/libspmv_hip_ynt.so timeout -k 10 300 python bench.py $B > gpurun_out/ynt$r.log 2>&1 || exit 1
done
echo ok
