# round-6: SELL split plan in one grid (product) vs main kernel then split kernel (lab build nofuse), R-MAT bench layout
set -o pipefail
export TMPDIR=/tmp
S='sell@{"sigma": 16777216, "hot": 0}'
for r in 1 2; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_prod$r -o run -- python3 tools/rmat_formats_lab.py "$S" --rounds 1 --steps 20 > gpurun_out/prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=$PWD/lab/libspmv_hip_nofuse.so timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_nofuse$r -o run -- python3 tools/rmat_formats_lab.py "$S" --rounds 1 --steps 20 > gpurun_out/nofuse$r.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "sell or rmat" > gpurun_out/t.log 2>&1 || exit 1
echo ok
