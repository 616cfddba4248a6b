# round-6: carry kernel with the head test first (product) vs the round-6 start — R-MAT bench layout (CSR, CMRS, COO), kernel trace; parity
set -o pipefail
export TMPDIR=/tmp
SP=('csr@{"hot": 0}' 'cmrs@{"hot": 0}' 'coo@{"hot": 0}')
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_prod -o run -- python3 tools/rmat_formats_lab.py "${SP[@]}" --rounds 1 --steps 20 > gpurun_out/prod.log 2>&1 || exit 1
SPMV_HIP_LIB=$PWD/lab/libspmv_hip_r6base.so timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_base -o run -- python3 tools/rmat_formats_lab.py "${SP[@]}" --rounds 1 --steps 20 > gpurun_out/base.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "coo or cmrs or tiled or rmat or hyb" > gpurun_out/t.log 2>&1 || exit 1
echo ok
