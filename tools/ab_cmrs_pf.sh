# round-6: tiled CMRS on the R-MAT (bench.py --workload rmat --format cmrs), product vs
# lab/libspmv_hip_cmrspf.so (next item's strip offsets prefetched), two interleaved rounds
set -o pipefail
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload rmat --format cmrs --steps 20 --warmup 3 > gpurun_out/cm_tree_$r.log 2>&1 || exit 1
  SPMV_HIP_LIB=$PWD/lab/libspmv_hip_cmrspf.so timeout -k 10 300 python bench.py --workload rmat --format cmrs --steps 20 --warmup 3 > gpurun_out/cm_pf_$r.log 2>&1 || exit 1
done
echo ok
