#!/bin/bash
# Round-3 closing job: SELL16 tests, A/B of the SELL16 tail order, cold 1/2/4/8-shard R-MAT rehearsal, bench kernel stats.
set -u
OUT=gpurun_out/g10
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "sell16 or hot_l1" > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 400 python3 -u tools/rmat_split_exp.py --parts 4 --reps 10 --hot-l1 0,2048,4096 > "$OUT/rmat_l1.log" 2>&1 || exit 5
grep -v "^W20\|^E20\|amdgpu.ids" "$OUT/rmat_l1.log"
bash tools/job_ab.sh "$OUT" opencl-spmv-algorithms_amd/lib/ab/libspmv_hip_base.so opencl-spmv-algorithms_amd/lib/ab/libspmv_hip_tail.so sell,sell16 || exit 2
timeout -k 10 600 python3 -u tools/shard_rehearse.py --gpus 1,2,4,8 --flush --graph > "$OUT/shard_rehearse.log" 2>&1 || { tail -20 "$OUT/shard_rehearse.log"; exit 3; }
grep -v "^W20\|^E20\|amdgpu.ids" "$OUT/shard_rehearse.log" | tail -12
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 bench.py --profile --steps 200 > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 4; }
echo prof done
