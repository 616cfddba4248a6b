# round-6: SELL small kernel, waves without x-copy duty issue their head before the window bounds (lab build hfirst)
set -o pipefail
B="--format sell --batch no --per-format no --single no --rmat-strong no --banded-strong no --rmat-per-format no --sell-single no --cpu-seconds 0"
for r in 1 2; do
  timeout -k 10 200 python tools/cant_single.py --formats sell,sell16 --flush-mode read > gpurun_out/cs_prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=lab/libspmv_hip_hfirst.so timeout -k 10 200 python tools/cant_single.py --formats sell,sell16 --flush-mode read > gpurun_out/cs_hf$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py $B > gpurun_out/prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=lab/libspmv_hip_hfirst.so timeout -k 10 300 python bench.py $B > gpurun_out/hf$r.log 2>&1 || exit 1
done
echo ok
