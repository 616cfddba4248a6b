#!/usr/bin/env bash
# GPU-box job: every GPU step of this suite as a named subcommand, each with
# its own time limit; ANY failing step stops the job (a Python process that
# hit a GPU fault exits 1, like a failed test, so no exit code is safe to
# run past).  Logs go to gpurun_out/<step>.log.
#
# usage: tools/gpu_job.sh [steps...]      (default: smoke tests bench prof)
#
# Parameters come from the environment:
#   CS_ARGS    extra tools/cant_single.py arguments (single, profsingle,
#              absingle), e.g. CS_ARGS="--formats csr --extra 'csr@{\"small\": false}'"
#   AB_LIBS    name=lib[,name=lib...] builds of libspmv_hip.so to A/B, each
#              run twice, interleaved ("tree" = the in-tree library):
#              absingle (cold cant-like single under rocprofv3), abrmat
#              (R-MAT tiled CSR, tools/rmat_split_exp.py), abreh (1- and
#              8-shard cold R-MAT rehearsal)
#   PMC_ARGS   extra tools/pmc_traffic.py arguments (pmc, pmcsingle)
#   REH_ARGS   extra tools/shard_rehearse.py arguments (abreh), e.g. --relabel
#   TEST_K     pytest -k expression (testk)
#   BENCH_ARGS extra bench.py arguments (bench), BENCH_TAG its log name
#              (gpurun_out/bench_<tag>.log; default bench.log)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
steps=("$@")
[ ${#steps[@]} -eq 0 ] && steps=(smoke tests bench prof)
run() { # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  local t0=$SECONDS
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc ($((SECONDS - t0)) s)" | tee -a gpurun_out/job.log
  tail -5 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ]; then echo "fatal exit $rc in $name: stopping"; exit "$rc"; fi
  return 0
}
lib_of() { # SPMV_HIP_LIB of one AB_LIBS entry ("" = the in-tree library)
  if [ "$1" = tree ]; then echo ""; else echo "$PWD/$1"; fi
}
ab_pairs() { IFS=, read -ra AB <<< "${AB_LIBS:?AB_LIBS=name=lib,... is required}"; }
PYT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
eval "cs_args=(${CS_ARGS:-})"
eval "pmc_args=(${PMC_ARGS:-})"
eval "bench_args=(${BENCH_ARGS:-})"
eval "reh_args=(${REH_ARGS:-})"
for s in "${steps[@]}"; do
  case $s in
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()";;
    tests) run gpu_tests 1500 $PYT tests -m gpu;;
    tests1) run gpu_tests_parity 1200 $PYT tests/test_gpu_parity.py;;
    tests2) run gpu_tests_rest 1200 $PYT tests -m gpu --deselect tests/test_gpu_parity.py;;
    testk) run gpu_tests_k 900 $PYT tests -m gpu -k "${TEST_K:?TEST_K is required}";;
    drivers) run drivers 600 $PYT tests/test_drivers_gpu.py;;
    itertests) run iter_tests 600 $PYT tests/test_iterate_gpu.py;;
    bench) run "bench${BENCH_TAG:+_$BENCH_TAG}" 900 python bench.py "${bench_args[@]}";;
    benchrmat) run bench_rmat 600 python bench.py --workload rmat --steps 20;;
    benchbatch) run bench_batch 600 python bench.py --workload batch --rmat-strong no --banded-strong no;;
    benchbanded) run bench_banded_sell 600 python bench.py --workload banded --format sell --steps 20 &&
                 run bench_banded_csr 600 python bench.py --workload banded --format csr --steps 20;;
    spawn2) run spawn2 900 python bench.py --gpus 2 --backend gloo --share-gpu --steps 20 --banded-strong no;;
    rehearse2) run rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --share-gpu --steps 20;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --profile --steps 200;;
    profbatch) run prof_batch 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_batch -o run -- python3 bench.py --profile --workload batch --steps 200;;
    single) run cant_single 600 python tools/cant_single.py --json gpurun_out/cant_single.json "${cs_args[@]}";;
    profsingle) run prof_single 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_single -o run -- python3 tools/cant_single.py --json gpurun_out/cant_single_prof.json "${cs_args[@]}" &&
                run attach_single 120 python tools/cant_single.py --json gpurun_out/cant_single_prof.json --attach gpurun_out/prof_single;;
    absingle) ab_pairs
              for i in 1 2; do
                for p in "${AB[@]}"; do
                  n=${p%%=*}; d=gpurun_out/ab_single_${n}_$i
                  SPMV_HIP_LIB=$(lib_of "${p#*=}") run "ab_single_${n}_$i" 300 rocprofv3 --kernel-trace --output-format csv -d "$d" -o run -- python3 tools/cant_single.py --json "$d.json" "${cs_args[@]}"
                  run "ab_attach_${n}_$i" 120 python tools/cant_single.py --json "$d.json" --attach "$d"
                done
              done;;
    abrmat) ab_pairs
            for i in 1 2; do
              for p in "${AB[@]}"; do
                SPMV_HIP_LIB=$(lib_of "${p#*=}") run "ab_rmat_${p%%=*}_$i" 300 python3 -u tools/rmat_split_exp.py --parts 4 --reps 20
              done
            done;;
    abreh) ab_pairs
           for i in 1 2; do
             for p in "${AB[@]}"; do
               SPMV_HIP_LIB=$(lib_of "${p#*=}") run "ab_reh_${p%%=*}_$i" 400 python3 -u tools/shard_rehearse.py --gpus 1,8 --graph --flush "${reh_args[@]}"
             done
           done;;
    rehrelabel) run reh_base 500 python -u tools/shard_rehearse.py --gpus 1,8 --graph --flush &&
                run reh_relabel 500 python -u tools/shard_rehearse.py --gpus 1,8 --graph --flush --relabel;;
    rehtrace) run reh_trace 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/reh_trace -o run -- python3 -u tools/shard_rehearse.py --gpus 1,8 --graph --flush --reps 20 "${reh_args[@]}";;
    rehcal) run reh_cal 900 python -u tools/shard_rehearse.py --gpus 8 --graph --flush --calibrate 3 "${reh_args[@]}";;
    sweep) run sweep 600 python tools/sweep.py;;
    rehearse8) run shard_rehearse 900 python tools/shard_rehearse.py --gpus 1,2,4,8 --graph --reps 50;;
    rehearsecold) run shard_rehearse_cold 900 python tools/shard_rehearse.py --gpus 1,2,4,8 --graph --reps 50 --flush;;
    lab) run sell_lab 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lab -o run -- python3 tools/sell_lab.py &&
         run lab_medians 60 python tools/trace_medians.py gpurun_out/lab;;
    overlap) run overlap_rmat 600 python tools/iterate_bench.py --rehearse 8 --matrix rmat --reps 20 &&
             run overlap_lap 600 python tools/iterate_bench.py --rehearse 8 --matrix laplacian --k 3000 --reps 20;;
    iterbench) run iter_power 300 python tools/iterate_bench.py --what power --matrix cantlike --iters 200 &&
               run iter_power_graph 300 python tools/iterate_bench.py --what power --matrix cantlike --iters 200 --graph &&
               run iter_cg 600 python tools/iterate_bench.py --what cg --matrix laplacian --k 2000 --iters 500;;
    counters) run counters 120 rocprofv3 -L;;
    probe) [ -x tools/bw_probe ] || hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o tools/bw_probe; run bw_probe 300 tools/bw_probe;;
    pmc) run pmc 1100 python tools/pmc_traffic.py "${pmc_args[@]}";;
    pmcrmat) run pmc_rmat 1100 python tools/pmc_traffic.py --workload rmat --formats csr --kernel csr_tiled_kernel --out "${PMC_OUT:-traffic_rmat.json}" --steps 5;;
    pmcsingle) run pmc_single 1100 python tools/pmc_traffic.py --workload cant --formats csr --out traffic_single.json --steps 20 "${pmc_args[@]}";;
    stalls) run pmc_stalls 1150 python tools/pmc_stalls.py --formats csr,sell;;
    stallsingle) run pmc_stalls_single 1150 python tools/pmc_stalls.py --workload cant --no-probe --formats "${STALL_FORMATS:-csr,sell16}" --passes "${STALL_PASSES:-sq,sq2,lds,lat,tcc,ta}" --out pmc_stalls_single.json;;
    *) echo "unknown step $s"; exit 2;;
  esac
done
