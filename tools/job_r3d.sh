#!/bin/bash
# Round-3: hub-shard tile size A/B (R = 3 above a mean row of 96, or always R = 2), PMC traffic of the new R-MAT CSR and SELL16 batch.
set -u
OUT=gpurun_out/g12
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
    for v in r3 r2; do
        SPMV_HIP_LIB=opencl-spmv-algorithms_amd/lib/ab/libspmv_hip_$v.so timeout -k 10 300 python3 -u tools/shard_rehearse.py --gpus 1,8 --graph > "$OUT/reh_${v}_$i.log" 2>&1 || { tail -20 "$OUT/reh_${v}_$i.log"; exit 2; }
        echo "$v $i"; grep '"gpus"' "$OUT/reh_${v}_$i.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['gpus'], d['shard_ms'], d['max_ms'])"
    done
done
timeout -k 10 400 python3 -u tools/pmc_traffic.py --formats csr,csrg --workload rmat --kernel tiled_kernel --out traffic_rmat_r3.json > "$OUT/pmc_rmat.log" 2>&1 || { tail -20 "$OUT/pmc_rmat.log"; exit 3; }
echo pmc rmat done
timeout -k 10 400 python3 -u tools/pmc_traffic.py --formats sell16 --kernel sell_xwin_kernel --out traffic_sell16.json > "$OUT/pmc_sell16.log" 2>&1 || { tail -20 "$OUT/pmc_sell16.log"; exit 4; }
echo pmc sell16 done
