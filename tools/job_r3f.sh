#!/bin/bash
# Round-3 closing check at HEAD: full GPU suite, smoke, default bench, R-MAT bench, cold cant-like single.
set -u
OUT=gpurun_out/g16
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 2; }
tail -1 "$OUT/smoke.log"
timeout -k 10 300 python3 -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 4; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"; echo bench done
timeout -k 10 300 python3 -u bench.py --workload rmat --steps 20 > "$OUT/bench_rmat.log" 2>&1 || { tail -20 "$OUT/bench_rmat.log"; exit 5; }
tail -1 "$OUT/bench_rmat.log" > "$OUT/bench_rmat.json"; echo rmat bench done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/cs" -o run -- \
    python3 tools/cant_single.py --formats sell,sell16,ell,csr --json "$OUT/cant_single.json" > "$OUT/cant_single.log" 2>&1 || { tail -20 "$OUT/cant_single.log"; exit 6; }
echo cant_single done
