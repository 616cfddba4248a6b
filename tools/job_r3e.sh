#!/bin/bash
# COO / CMRS wave-per-long-row: parity tests, then R-MAT and cant-batch A/B against the previous build.
set -u
OUT=gpurun_out/g14
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "coo or cmrs or hyb or rmat or golden or cantlike or reproducible" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 300 python3 -u -m pytest tests/test_drivers_gpu.py -x -q --timeout 200 --timeout-method thread > "$OUT/drivers.log" 2>&1 || { tail -30 "$OUT/drivers.log"; exit 3; }
tail -1 "$OUT/drivers.log"
timeout -k 10 60 ./bin/sigma_c --gen cantlike --reps 50 --index16 > "$OUT/sc16.log" 2>&1 && timeout -k 10 60 ./bin/sigma_c --gen cantlike --reps 50 > "$OUT/sc.log" 2>&1 || exit 4
grep -i "took\|GB/s\|SELL16\|result" "$OUT/sc16.log" "$OUT/sc.log"
for m in rmat cantlike; do
    for v in base new base new; do
        SPMV_HIP_LIB=opencl-spmv-algorithms_amd/lib/ab/libspmv_hip_$v.so timeout -k 10 400 python3 -u tools/time_formats.py \
            --matrix $m --formats coo,cmrs,hyb --rounds 3 > "$OUT/tf_${m}_$v.log" 2>&1 || { tail -20 "$OUT/tf_${m}_$v.log"; exit 2; }
        echo "$m $v"; grep '^{' "$OUT/tf_${m}_$v.log"
    done
done
