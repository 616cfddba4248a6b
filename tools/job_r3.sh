#!/bin/bash
# Round-3 GPU job: parity of the changed kernels, SELL16 cold (rocprof), then the default bench.
# usage: bash tools/job_r3.sh OUTDIR
set -u
OUT=${1:-gpurun_out/job}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "sell16 or sell_small or sell_xwin or golden" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for i in 1 2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/cs$i" -o run -- \
        python3 tools/cant_single.py --formats sell,sell16 --json "$OUT/cs$i.json" > "$OUT/cs$i.log" 2>&1 || exit 3
done
echo cant_single done
timeout -k 10 900 python3 -u bench.py > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 4; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
echo bench done
