# round-6: SELL split-chunk kernel unroll on the R-MAT (bench layout), product (U = 4) vs lab builds su8 / su16, kernel trace
set -o pipefail
export TMPDIR=/tmp
S='sell@{"sigma": 16777216, "hot": 0}'
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_prod -o run -- python3 tools/rmat_formats_lab.py "$S" --rounds 1 --steps 20 > gpurun_out/prod.log 2>&1 || exit 1
for v in su8 su16; do
  SPMV_HIP_LIB=$PWD/lab/libspmv_hip_$v.so timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_$v -o run -- python3 tools/rmat_formats_lab.py "$S" --rounds 1 --steps 20 > gpurun_out/$v.log 2>&1 || exit 1
done
echo ok
