#!/bin/bash
# Round-3 GPU job: parity of the changed kernels, then R-MAT timings per tiled-CSR tile size.
# usage: bash tools/job_r3.sh OUTDIR
set -u
OUT=${1:-gpurun_out/job}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    -k "tiled or hot or rmat or csrg or empty_row or golden or csrf32 or sell16" > "$OUT/tests.log" 2>&1 || { tail -40 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
for R in 1 2 3; do
    SPMV_TILED_R=$R timeout -k 10 400 python3 -u tools/rmat_split_exp.py --parts 4,8 --reps 10 --colmaps zero > "$OUT/rmat_R$R.log" 2>&1 || exit 2
    echo "R=$R"; grep -v "^W20\|^E20\|amdgpu.ids" "$OUT/rmat_R$R.log"
done
for i in 1 2; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/cs$i" -o run -- \
        python3 tools/cant_single.py --formats sell,sell16 --json "$OUT/cs$i.json" > "$OUT/cs$i.log" 2>&1 || exit 3
done
echo cant_single done
