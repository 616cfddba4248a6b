# round-6: tiled CSR on the R-MAT (bench layout), branch-free offsets + columns pinned before them (product) vs the round-6 start
set -o pipefail
export TMPDIR=/tmp
S='csr@{"hot": 0}'
for r in 1 2; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_prod$r -o run -- python3 tools/rmat_formats_lab.py "$S" 'cmrs@{"hot": 0}' --rounds 1 --steps 20 > gpurun_out/prod$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=$PWD/lab/libspmv_hip_r6base.so timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_base$r -o run -- python3 tools/rmat_formats_lab.py "$S" 'cmrs@{"hot": 0}' --rounds 1 --steps 20 > gpurun_out/base$r.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "tiled or rmat or csr" > gpurun_out/t.log 2>&1 || exit 1
echo ok
