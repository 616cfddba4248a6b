# round-6: HYB ELL width on one cant-like matrix: the byte rule's K = 52 (ELL + COO tail) vs
# wider K (shorter tail) and K = 82 (the longest row: no tail, one kernel), ELL beside
set -o pipefail
for r in 1 2; do
  timeout -k 10 300 python tools/cant_single.py --formats hyb,ell --flush-mode read \
    --extra 'hyb@{"hyb_k": 64}' --extra 'hyb@{"hyb_k": 72}' --extra 'hyb@{"hyb_k": 82}' \
    > gpurun_out/hybk$r.log 2>&1 || exit 1
done
echo ok
