# round-6: tiled CMRS with the plan's tile table (filled once) — R-MAT bench layout, kernel trace; CMRS parity tests
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_prod -o run -- python3 tools/rmat_formats_lab.py 'cmrs@{"hot": 0}' 'cmrs@{"hot": 4096}' --rounds 2 --steps 20 > gpurun_out/prod.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_drivers_gpu.py -m gpu -k "cmrs" > gpurun_out/t.log 2>&1 || exit 1
echo ok
