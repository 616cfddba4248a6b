# round-6 SELL A/B: the product library against lab builds (tools/build_variant.sh), then bench's sell line
set -o pipefail
for r in 1 2; do
  timeout -k 10 200 python tools/cant_single.py --formats sell,sell16 --flush-mode read > gpurun_out/new$r.log 2>&1 || exit 1
  for v in r6base xc8 xc2 lb4; do
    SPMV_HIP_LIB=lab/libspmv_hip_$v.so timeout -k 10 200 python tools/cant_single.py --formats sell,sell16 --flush-mode read > gpurun_out/$v$r.log 2>&1 || exit 1
  done
  SPMV_HIP_LIB=lab/libspmv_hip_rb8.so timeout -k 10 200 python tools/cant_single.py --formats sell --flush-mode read --extra 'sell@{"_opt": {"sell_rest": 1}}' --extra 'sell16@{"_opt": {"sell_rest": 1}}' > gpurun_out/rb8$r.log 2>&1 || exit 1
  timeout -k 10 300 python bench.py --format sell --batch no --per-format no --single no --rmat-strong no --banded-strong no --rmat-per-format no --sell-single no --cpu-seconds 0 > gpurun_out/bench$r.log 2>&1 || exit 1
done
echo ok
