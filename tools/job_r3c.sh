#!/bin/bash
# Round-3 closing validation: full GPU suite, cold shard rehearsal, default bench, R-MAT bench.
set -u
OUT=gpurun_out/g11
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 400 python3 -u tools/shard_rehearse.py --gpus 1,2,4,8 --flush --graph > "$OUT/shard_rehearse.log" 2>&1 || { tail -20 "$OUT/shard_rehearse.log"; exit 3; }
echo rehearsal done
timeout -k 10 300 python3 -u bench.py > "$OUT/bench.log" 2>&1 || { tail -20 "$OUT/bench.log"; exit 4; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"; echo bench done
timeout -k 10 300 python3 -u bench.py --workload rmat --steps 20 > "$OUT/bench_rmat.log" 2>&1 || { tail -20 "$OUT/bench_rmat.log"; exit 5; }
tail -1 "$OUT/bench_rmat.log" > "$OUT/bench_rmat.json"; echo rmat bench done
