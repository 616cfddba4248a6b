# round-6: tiled CMRS with owned strip offsets staged in LDS per pass (product) vs the round-6 start — R-MAT, kernel trace; CMRS parity
set -o pipefail
export TMPDIR=/tmp
SP=('cmrs@{"hot": 0}' 'cmrs@{"hot": 4096}')
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_prod -o run -- python3 tools/rmat_formats_lab.py "${SP[@]}" --rounds 2 --steps 20 > gpurun_out/prod.log 2>&1 || exit 1
SPMV_HIP_LIB=$PWD/lab/libspmv_hip_r6base.so timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_base -o run -- python3 tools/rmat_formats_lab.py "${SP[@]}" --rounds 2 --steps 20 > gpurun_out/base.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_drivers_gpu.py tests/test_build_gpu.py -m gpu -k "cmrs" > gpurun_out/t.log 2>&1 || exit 1
echo ok
