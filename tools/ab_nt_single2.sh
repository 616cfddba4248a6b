# round-6: as ab_nt_single.sh for COO, ELL and CMRS on ONE cant-like matrix
set -o pipefail
for r in 1 2 3; do
  timeout -k 10 300 python tools/cant_single.py --formats coo,ell,cmrs --flush-mode read \
    --extra 'coo@{"_opt": {"stream_nt": 0}}' --extra 'ell@{"_opt": {"stream_nt": 0}}' \
    --extra 'cmrs@{"_opt": {"stream_nt": 0}}' > gpurun_out/nt2_$r.log 2>&1 || exit 1
done
echo ok
