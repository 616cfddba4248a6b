# round-6: non-temporal stream loads (each kernel's default: on) vs plain loads
# (spmv_set_option stream_nt = 0) on ONE cant-like matrix: SELL, SELL16, CSR; events, one box
set -o pipefail
for r in 1 2 3; do
  timeout -k 10 300 python tools/cant_single.py --formats sell,sell16,csr --flush-mode read \
    --extra 'sell@{"_opt": {"stream_nt": 0}}' --extra 'sell16@{"_opt": {"stream_nt": 0}}' \
    --extra 'csr@{"_opt": {"stream_nt": 0}}' > gpurun_out/nt_$r.log 2>&1 || exit 1
done
echo ok
