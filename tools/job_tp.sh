#!/bin/bash
# A/B of tiled-CSR library builds on the R-MAT (product path, every-column-0 probe, y hash)
# usage: bash tools/job_tp.sh OUTDIR name...   (libs in opencl-spmv-algorithms_amd/lib/ab/<name>.so)
set -u
OUT=$1; shift
mkdir -p "$OUT"
for r in 1 2; do
    for n in "$@"; do
        SPMV_HIP_LIB=$PWD/opencl-spmv-algorithms_amd/lib/ab/$n.so timeout -k 10 240 \
            python3 -u tools/rmat_split_exp.py --parts 4 --colmaps zero --reps 20 > "$OUT/$n$r.log" 2>&1 || exit 3
        echo "$n$r done"
    done
done
