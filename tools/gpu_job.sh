#!/usr/bin/env bash
# GPU-box job: smoke, GPU parity tests, bench, rocprofv3 kernel-trace.
# Each GPU step has its own time limit; ANY failing step stops the job (a
# Python process that hit a GPU fault exits 1, like a failed test, so no
# exit code is safe to run past).
# usage: tools/gpu_job.sh [steps...]   steps: see the case list below
# (Round 1-2 A/B jobs over environment knobs that no longer exist were
# removed with the knobs; their logs stay under profiles/round1, round2.)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(smoke tests bench prof)
fatal() { [ "$1" -ne 0 ]; }
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc" | tee -a gpurun_out/job.log
  tail -5 "gpurun_out/$name.log"
  if fatal $rc; then echo "fatal exit $rc in $name: stopping"; exit $rc; fi
  return 0
}
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
for s in "${steps[@]}"; do
  case $s in
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()";;
    tests) run gpu_tests 1500 $PYT tests -m gpu;;
    tests1) run gpu_tests_parity 1200 $PYT tests/test_gpu_parity.py;;
    tests2) run gpu_tests_rest 1200 $PYT tests -m gpu --deselect tests/test_gpu_parity.py;;
    bench) run bench 900 python bench.py;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --profile --steps 200;;
    single) run cant_single 600 python tools/cant_single.py --json gpurun_out/cant_single.json;;
    profsingle) # CS_ARGS: extra cant_single arguments, e.g. --formats csr --extra 'csr@{"small": false}'
                eval "cs_args=(${CS_ARGS:-})"
                run prof_single 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_single -o run -- python3 tools/cant_single.py --json gpurun_out/cant_single_prof.json "${cs_args[@]}" &&
                run attach_single 120 python tools/cant_single.py --json gpurun_out/cant_single_prof.json --attach gpurun_out/prof_single;;
    newtests) run new_tests 900 $PYT tests/test_gpu_parity.py -k "small or sell16_head";;
    sweep) run sweep 600 python tools/sweep.py;;
    benchrmat) run bench_rmat 600 python bench.py --workload rmat --steps 20;;
    benchbanded) run bench_banded_sell 600 python bench.py --workload banded --format sell --steps 20 && run bench_banded_csr 600 python bench.py --workload banded --format csr --steps 20;;
    rehearse8) run shard_rehearse 900 python tools/shard_rehearse.py --gpus 1,2,4,8 --graph --reps 50;;
    rehearsecold) run shard_rehearse_cold 900 python tools/shard_rehearse.py --gpus 1,2,4,8 --graph --reps 50 --flush;;
    spawn2) run spawn2 900 python bench.py --gpus 2 --backend gloo --share-gpu --steps 20 --banded-strong no;;
    rehearse2) run rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --share-gpu --steps 20;;
    rehearse2r) run rehearse2_rmat 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --backend gloo --share-gpu --workload rmat --steps 10;;
    drivers) run drivers 600 $PYT tests/test_drivers_gpu.py;;
    itertests) run iter_tests 600 $PYT tests/test_iterate_gpu.py;;
    lab) run sell_lab 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lab -o run -- python3 tools/sell_lab.py &&
         run lab_medians 60 python tools/trace_medians.py gpurun_out/lab;;
    overlap) run overlap_rmat 600 python tools/iterate_bench.py --rehearse 8 --matrix rmat --reps 20 &&
             run overlap_lap 600 python tools/iterate_bench.py --rehearse 8 --matrix laplacian --k 3000 --reps 20;;
    counters) run counters 120 rocprofv3 -L;;
    probe) [ -x tools/bw_probe ] || hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o tools/bw_probe; run bw_probe 300 tools/bw_probe;;
    pmc) run pmc 1100 python tools/pmc_traffic.py;;
    pmcrmat) run pmc_rmat 1100 python tools/pmc_traffic.py --workload rmat --formats csr --kernel csr_tiled_kernel --out traffic_rmat.json --steps 5;;
    stalls) run pmc_stalls 1150 python tools/pmc_stalls.py --formats csr,sell;;
    iterbench) run iter_power 300 python tools/iterate_bench.py --what power --matrix cantlike --iters 200 &&
               run iter_power_graph 300 python tools/iterate_bench.py --what power --matrix cantlike --iters 200 --graph &&
               run iter_cg 600 python tools/iterate_bench.py --what cg --matrix laplacian --k 2000 --iters 500;;
    *) echo "unknown step $s";;
  esac
done
