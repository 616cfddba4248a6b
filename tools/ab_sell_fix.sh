# round-6: SELL split fix kernel with 32 chunks in flight (product) — R-MAT bench layout, kernel trace; SELL parity tests
set -o pipefail
export TMPDIR=/tmp
S='sell@{"sigma": 16777216, "hot": 0}'
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_prod -o run -- python3 tools/rmat_formats_lab.py "$S" --rounds 2 --steps 20 > gpurun_out/prod.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "sell or rmat" > gpurun_out/t.log 2>&1 || exit 1
echo ok
