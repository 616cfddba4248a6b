set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -k "xwin" > gpurun_out/t22.log 2>&1; rc=$?; tail -3 gpurun_out/t22.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/sweep.py --env-only --rounds 3 > gpurun_out/sweep_batch.log 2>&1; rc=$?; grep '^{' gpurun_out/sweep_batch.log; exit $rc
