#!/bin/bash
# A/B of two builds of libspmv_hip.so on the cold cant-like single (rocprof), interleaved.
# usage: bash tools/job_ab.sh OUTDIR LIB_A LIB_B [formats]
set -u
OUT=$1; A=$2; B=$3; F=${4:-sell16}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
    for tag in A B; do
        lib=$A; [ $tag = B ] && lib=$B
        SPMV_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${tag}$i" -o run -- \
            python3 tools/cant_single.py --formats "$F" --json "$OUT/${tag}$i.json" > "$OUT/${tag}$i.log" 2>&1 || exit 3
        echo "$tag$i done"
    done
done
