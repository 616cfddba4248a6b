set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_build_gpu.py -x -q > gpurun_out/t33.log 2>&1; rc=$?; tail -15 gpurun_out/t33.log; exit $rc
