#!/bin/bash
# Round-3 GPU job: parity of the changed kernels, R-MAT timings, SELL small-kernel shapes (cold, rocprof).
# usage: bash tools/job_r3.sh OUTDIR
set -u
OUT=${1:-gpurun_out/job}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "tiled or hot or rmat or csrg or empty_row or golden or cantlike or sell16 or sell_small" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 500 python3 -u tools/rmat_split_exp.py --parts 4,8,16 --reps 10 --colmaps zero > "$OUT/rmat.log" 2>&1 || exit 2
grep -v "^W20\|^E20" "$OUT/rmat.log"
for shape in def 16w 8w 16 12w; do
    k=$shape; [ "$shape" = def ] && k=""
    SPMV_SELL_SMALL=$k timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/cs_$shape" -o run -- \
        python3 tools/cant_single.py --formats sell,sell16 --json "$OUT/cs_$shape.json" > "$OUT/cs_$shape.log" 2>&1 || exit 3
    echo "shape $shape done"
done
