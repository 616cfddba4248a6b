# round-6: COO accumulate mode (HYB tail), product vs lab/libspmv_hip_hybold.so (the
# row loop with y[r] += s), same box, interleaved, rocprofv3 kernel traces
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export SPMV_HIP_LIB=$PWD/lab/libspmv_hip_hybold.so; else unset SPMV_HIP_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/acc_${v}_$r -o run -- \
      python3 tools/cant_single.py --formats ell --flush-mode read --extra 'hyb@{"hyb_k": 52}' \
      > gpurun_out/acc_${v}_$r.log 2>&1 || exit 1
  done
done
echo ok
