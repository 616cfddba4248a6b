set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -k "variant5 or variant-5 or bit_identical or stream_load or bitwise or rmat_skewed or ragged" > gpurun_out/t13.log 2>&1; rc=$?; tail -3 gpurun_out/t13.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_job.sh sweepnt
