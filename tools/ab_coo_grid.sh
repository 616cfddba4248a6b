# round-6: COO single pass vs carry pass over cant-like prefixes and HYB tails
# (tools/coo_grid_probe.py), product vs lab builds (AB_LIBS name=lib ...), one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for nl in tree ${AB_LIBS:-}; do
  name=${nl%%=*}; lib=${nl#*=}
  if [ "$name" = tree ]; then unset SPMV_HIP_LIB; else export SPMV_HIP_LIB=$PWD/$lib; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gp_$name -o run -- \
    python3 tools/coo_grid_probe.py > gpurun_out/gp_$name.log 2>&1 || exit 1
done
echo ok
