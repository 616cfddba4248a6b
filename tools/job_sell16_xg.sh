#!/bin/bash
# SELL16 on the cold cant-like single against variants given as cant_single --extra runs, twice.
# usage: bash tools/job_sell16_xg.sh OUTDIR 'sell16@{"_params": {"xcap": 0}}' ...
set -u
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
args=()
for e in "$@"; do args+=(--extra "$e"); done
for i in 1 2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/r$i" -o run -- \
        python3 tools/cant_single.py --formats sell16 "${args[@]}" \
        --json "$OUT/r$i.json" > "$OUT/r$i.log" 2>&1 || { tail -20 "$OUT/r$i.log"; exit 3; }
    echo "r$i done"
done
