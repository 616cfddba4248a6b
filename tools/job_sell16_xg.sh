#!/bin/bash
# SELL16 on the cold cant-like single: x window in LDS (product) vs gathers from global memory (xcap 0), twice.
set -u
OUT=gpurun_out/g17
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/r$i" -o run -- \
        python3 tools/cant_single.py --formats sell16 --extra 'sell16@{"_params": {"xcap": 0}}' \
        --json "$OUT/r$i.json" > "$OUT/r$i.log" 2>&1 || { tail -20 "$OUT/r$i.log"; exit 3; }
    echo "r$i done"
done
