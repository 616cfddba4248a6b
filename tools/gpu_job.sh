#!/usr/bin/env bash
# GPU-box job: smoke, GPU parity tests, bench, rocprofv3 kernel-trace.
# Each GPU step has its own time limit; ANY failing step stops the job (a
# Python process that hit a GPU fault exits 1, like a failed test, so no
# exit code is safe to run past).
# usage: tools/gpu_job.sh [steps...]   steps: smoke tests bench prof pmc
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
for s in "${steps[@]}"; do
  case $s in
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()";;
    tests) run gpu_tests 1500 python -m pytest tests -m gpu -x -q;;
    testsq) run gpu_tests 1500 python -m pytest tests -m gpu -q;;
    bench) run bench 900 python bench.py;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --profile --steps 200;;
    sweep) run sweep 600 python tools/sweep.py;;
    sweep0) SPMV_XCD_REMAP=0 run sweep_noremap 600 python tools/sweep.py --rounds 2;;
    sweepr3) SPMV_CSR_STAGE_ROUNDS=3 run sweep_r3 300 python tools/sweep.py --rounds 2 --only csr;;
    sweepr8) SPMV_CSR_STAGE_ROUNDS=8 run sweep_r8 300 python tools/sweep.py --rounds 2 --only csr;;
    sweepbt) SPMV_SELL_BT=256 run sweep_bt256 300 python tools/sweep.py --rounds 2 --only sell;;
    sweepu8) SPMV_COO_U=8 run sweep_u8 300 python tools/sweep.py --rounds 2 --only coo,cmrs;;
    sweepu16) SPMV_COO_U=16 run sweep_u16 300 python tools/sweep.py --rounds 2 --only coo,cmrs;;
    sweepcoo) run sweep_coo 300 python tools/sweep.py --rounds 2 --only coo,cmrs;;
    sweepcoo1) SPMV_COO_VARIANT=1 SPMV_CMRS_VARIANT=1 run sweep_coo1 300 python tools/sweep.py --rounds 2 --only coo,cmrs;;
    sweeprmat2) run sweep_rmat 900 python tools/sweep.py --matrix rmat --rounds 1 --reps 20;;
    benchrmat) run bench_rmat 600 python bench.py --workload rmat --steps 20;;
    benchbanded) run bench_banded_sell 600 python bench.py --workload banded --format sell --steps 20 && run bench_banded_csr 600 python bench.py --workload banded --format csr --steps 20;;
    rehearse8) run shard_rehearse 900 python tools/shard_rehearse.py --gpus 1,2,4,8 &&
               run shard_rehearse_sell 900 python tools/shard_rehearse.py --gpus 1,8 --format sell;;
    rehearsew) run shard_rehearse_w 900 python tools/shard_rehearse.py --gpus 1,8 --row-weights 0,2,4 &&
               run shard_rehearse_nohot 600 python tools/shard_rehearse.py --gpus 8 --row-weights 2 --hot 0 &&
               run prof_rehearse 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rehearse -o run -- python3 tools/shard_rehearse.py --gpus 8 --row-weights 2;;
    rehearsew2) run shard_rehearse_w2 900 python tools/shard_rehearse.py --gpus 8 --row-weights 4,6,8;;
    rehearseh) run shard_rehearse_h17 600 python tools/shard_rehearse.py --gpus 8 --row-weights 4 --hot 131072 &&
               run shard_rehearse_h18 600 python tools/shard_rehearse.py --gpus 8 --row-weights 4 --hot 262144;;
    rehearse18) run shard_rehearse_18 900 python tools/shard_rehearse.py --gpus 1,8;;
    testempty) run gpu_tests_empty 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "empty_row_runs or csr_hot";;
    profreh8) run prof_rehearse8 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_reh8 -o run -- python3 tools/shard_rehearse.py --gpus 8;;
    abreh) SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run reh_head 600 python tools/shard_rehearse.py --gpus 1,8 &&
           run reh_new 600 python tools/shard_rehearse.py --gpus 1,8 &&
           SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run reh_head2 600 python tools/shard_rehearse.py --gpus 1,8 &&
           run reh_new2 600 python tools/shard_rehearse.py --gpus 1,8;;
    abcmrs) SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run cmrs_head 600 python tools/shard_rehearse.py --gpus 1,8 --format cmrs &&
            run cmrs_new 600 python tools/shard_rehearse.py --gpus 1,8 --format cmrs;;
    coont) run coo_base 300 python bench.py --format coo --per-format no --cpu-seconds 0 &&
           SPMV_STREAM_NT=1 run coo_nt 300 python bench.py --format coo --per-format no --cpu-seconds 0 &&
           run coo_base2 300 python bench.py --format coo --per-format no --cpu-seconds 0 &&
           SPMV_STREAM_NT=1 run coo_nt2 300 python bench.py --format coo --per-format no --cpu-seconds 0;;
    abcoo) # interleaved on one box: library before NT COO loads vs current (NT on / off)
           for i in 1 2 3; do
             SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_prev.so run coo_prev$i 300 python bench.py --format coo --per-format no --cpu-seconds 0 &&
             run coo_cur_nt$i 300 python bench.py --format coo --per-format no --cpu-seconds 0 &&
             SPMV_STREAM_NT=0 run coo_cur_nt0_$i 300 python bench.py --format coo --per-format no --cpu-seconds 0
           done;;
    abremap) run ab_csr_xwin_remap 600 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_MODE=0,3 --env SPMV_XWIN_REMAP=0,1 --rounds 5;;
    abxr) run ab_csr_xwin_r 600 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_R=2,3,4,6,8 --rounds 5;;
    abx4) run ab_csr_xwin_m34 600 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_MODE=0,3,4 --env SPMV_CSR_XWIN_R=3,4 --rounds 5;;
    abwaves) for i in 1 2; do
               run ab_w1_$i 300 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_R=3,4 --rounds 3 &&
               SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_w7.so run ab_w7_$i 300 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_R=3,4 --rounds 3 &&
               SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_w8.so run ab_w8_$i 300 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_R=3,4 --rounds 3
             done;;
    abprobe) for i in 1 2; do  # (bit 4 = no second barrier faulted: not built any more)
               run abp_base_$i 300 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_R=3,4 --rounds 3
               for p in 1 2 8; do
                 SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_p$p.so run abp_p${p}_$i 300 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_R=3,4 --rounds 3
               done
             done;;
    abflat) run ab_flat_l4 600 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_MODE=3,5 --env SPMV_CSR_XWIN_R=3,4 --rounds 5 &&
            run ab_flat_l2 600 python tools/ab_env.py --format csr --kw '{"lanes": 2}' --env SPMV_CSR_XWIN_MODE=3,5 --env SPMV_CSR_XWIN_R=3,4 --rounds 5 &&
            run ab_flat_l8 600 python tools/ab_env.py --format csr --kw '{"lanes": 8}' --env SPMV_CSR_XWIN_MODE=3,5 --env SPMV_CSR_XWIN_R=3,4 --rounds 5;;
    abformats) for i in 1 2; do  # head = tools/ab/libspmv_hip_head.so
                 SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run abf_head_$i 600 python tools/time_formats.py &&
                 run abf_new_$i 600 python tools/time_formats.py
               done;;
    abformatsr) for i in 1 2; do
                 SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run abfr_head_$i 600 python tools/time_formats.py --matrix rmat --formats csr,cmrs,coo,hyb,sell --rounds 2 --reps 10 &&
                 run abfr_new_$i 600 python tools/time_formats.py --matrix rmat --formats csr,cmrs,coo,hyb,sell --rounds 2 --reps 10
               done;;
    abpre) run ab_csr_xwin_pre 600 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_PRE=0,1 --rounds 6;;
    abrows) for r in 64 128 256 512; do
              run ab_csr_rows$r 300 python tools/ab_env.py --format csr --kw "{\"xwin_rows\": $r}" --env SPMV_CSR_XWIN_MODE=3,5 --rounds 4
            done &&
            run ab_sell_unroll 300 python tools/ab_env.py --format sell --env SPMV_SLOT_UNROLL=4,8 --env SPMV_XWIN_REMAP=0,1 --rounds 4;;
    abpipe) run ab_sell_pipe 300 python tools/ab_env.py --format sell --env SPMV_SLOT_PIPE=0,1 --rounds 5 &&
            run ab_ell_pipe 300 python tools/ab_env.py --format ell --env SPMV_SLOT_PIPE=0,1 --rounds 5;;
    reh2) run reh2_w 900 python tools/shard_rehearse.py --gpus 1,8 --row-weights 2,4,8 &&
          run reh2_trace 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/reh2_trace -o run -- python3 tools/shard_rehearse.py --gpus 8 --row-weights 4 --reps 10;;
    abbanded) run ab_banded_csr 600 python tools/ab_env.py --matrix banded --format csr --env SPMV_CSR_XWIN_MODE=0,3 --env SPMV_XWIN_REMAP=0,1 --rounds 4 --reps 20 &&
              run ab_banded_csr_r 600 python tools/ab_env.py --matrix banded --format csr --env SPMV_CSR_XWIN_MODE=3 --env SPMV_CSR_XWIN_R=3,4 --rounds 4 --reps 20 &&
              run ab_banded_sell 600 python tools/ab_env.py --matrix banded --format sell --kw '{"ki": 1}' --env SPMV_XWIN_REMAP=0,1 --rounds 4 --reps 20;;
    abbanded2) run ab_banded2_csr 600 python tools/ab_env.py --matrix banded --format csr --env SPMV_CSR_XWIN_MODE=0,2,3,auto --rounds 4 --reps 20 &&
               run ab_cant2_csr 600 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_MODE=0,3,auto --rounds 4;;
    absellcopy) for i in 1 2; do
                  SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run ab_sellcopy_head_$i 300 python tools/ab_env.py --matrix banded --format sell --kw '{"ki": 1}' --rounds 3 --reps 20 &&
                  run ab_sellcopy_new_$i 300 python tools/ab_env.py --matrix banded --format sell --kw '{"ki": 1}' --rounds 3 --reps 20 &&
                  SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run ab_sellcopy_cant_head_$i 300 python tools/ab_env.py --format sell --rounds 3 &&
                  run ab_sellcopy_cant_new_$i 300 python tools/ab_env.py --format sell --rounds 3
                done;;
    testxs) run gpu_tests_xstream 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "xstream";;
    abxs) run ab_xstream 600 python tools/ab_env.py --format csr --kw '{}' --kw '{"xwin_rows": 1}' --env SPMV_CSR_XSTREAM=0,1 --rounds 5 &&
          run ab_xstream_banded 600 python tools/ab_env.py --format csr --matrix banded --kw '{}' --kw '{"xwin_rows": 1}' --env SPMV_CSR_XSTREAM=0,1 --rounds 3 --reps 20;;
    abpad) run ab_lds_pad 600 python tools/ab_env.py --format csr --kw '{}' --env SPMV_CSR_LDS_PAD=0,9216,15360,30000 --rounds 5 &&
           run ab_lds_pad_xs 600 python tools/ab_env.py --format csr --kw '{"xwin_rows": 1}' --env SPMV_CSR_XSTREAM=1 --env SPMV_CSR_LDS_PAD=0,12288 --rounds 5;;
    abfused) run gpu_tests_fused 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "fused_carry or csr_hot or empty_row_runs" &&
             run ab_fused_rehearse 900 python tools/shard_rehearse.py --gpus 1,8 --env SPMV_TILED_FUSED_CARRY=0,1 --rounds 3;;
    abtiler) for r in 3 2 1 4 3; do
               SPMV_TILED_R=$r run reh_tiled_r$r 600 python tools/shard_rehearse.py --gpus 1,8 --rounds 2 || exit 1
             done;;
    tiledw) run gpu_tests_tiled 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "tiled or hot or fused or rmat or csrf32" &&
            run reh_tiled_w 900 python tools/shard_rehearse.py --gpus 1,8 --row-weights 1,2,3,4 --rounds 2;;
    tiledh) run reh_tiled_h 900 python tools/shard_rehearse.py --gpus 8 --row-weights 1.5,2,2.5 --hot 131072,262144,-1 --rounds 2;;
    reh3) run reh3_eager 900 python tools/shard_rehearse.py --gpus 1,2,4,8 --rounds 2 &&
          run reh3_graph 900 python tools/shard_rehearse.py --gpus 1,2,4,8 --rounds 2 --graph --reps 50;;
    reh4) SPMV_TILED_R=1 run reh4_r1 900 python tools/shard_rehearse.py --gpus 2,4,8 --graph --reps 50 &&
          run reh4_rule 900 python tools/shard_rehearse.py --gpus 2,4,8 --graph --reps 50 &&
          SPMV_TILED_R=3 run reh4_r3 900 python tools/shard_rehearse.py --gpus 2,4,8 --graph --reps 50;;
    reh5) run reh5_w 1000 python tools/shard_rehearse.py --gpus 1,2,4,8 --row-weights 0.5,1,1.5,2 --graph --reps 50;;
    reh6) run reh6_cal 1000 python tools/shard_rehearse.py --gpus 2,4,8 --row-weights 1,2 --graph --reps 50 --calibrate 2 &&
          run rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --share-gpu --steps 20;;
    abgather) run gpu_tests_gather 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "coo or hot or tiled or hyb or sell or rmat" &&
              for i in 1 2; do
                SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run abg_head_$i 600 python tools/shard_rehearse.py --gpus 1,8 --graph --reps 50 || exit 1
                run abg_new_$i 600 python tools/shard_rehearse.py --gpus 1,8 --graph --reps 50 || exit 1
              done &&
              SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_head.so run abg_coo_head 600 python tools/time_formats.py --formats coo,csr --rounds 2 &&
              run abg_coo_new 600 python tools/time_formats.py --formats coo,csr --rounds 2;;
    rmatfmt) run bench_rmat 600 python bench.py --workload rmat --steps 20 --rmat-strong no &&
             run gpu_tests_cmrs1 600 env SPMV_CMRS_TILED_R=1 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "cmrs" &&
             SPMV_CMRS_TILED_R=1 run reh_cmrs_r1 600 python tools/shard_rehearse.py --format cmrs --gpus 1,8 --graph --reps 30 &&
             run reh_cmrs_r3 600 python tools/shard_rehearse.py --format cmrs --gpus 1,8 --graph --reps 30;;
    rmatfmt2) run gpu_tests_fmt2 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "coo or cmrs or hot or rmat or hyb or tiled" &&
              run bench_rmat2 600 python bench.py --workload rmat --steps 20 --rmat-strong no &&
              SPMV_COO_HOT_R=0 run reh_coo_r3 600 python tools/shard_rehearse.py --format coo --gpus 1,8 --graph --reps 30 &&
              run reh_coo_r1 600 python tools/shard_rehearse.py --format coo --gpus 1,8 --graph --reps 30;;
    proffmt) run prof_fmt 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fmt -o run -- python3 bench.py --steps 50 --rmat-strong no --cpu-seconds 0;;
    abbanded3) run ab_banded3 900 python tools/ab_env.py --matrix banded --format csr --kw '{}' --kw '{"xwin_rows": 256}' --kw '{"xwin_rows": 512}' --kw '{"lanes": 4}' --env SPMV_CSR_XWIN_MODE=0,3 --rounds 3 --reps 20;;
    abp11) for i in 1 2; do
             run abp11_base_$i 300 python tools/ab_env.py --format csr --rounds 3 &&
             SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_p11.so run abp11_probe_$i 300 python tools/ab_env.py --format csr --rounds 3
           done && run bw_probe 300 tools/bw_probe;;
    abp11m) run abmodes_real 300 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_MODE=0,3 --rounds 3 &&
            run abmodes_real_total 300 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_MODE=0,3 --rounds 3 --total &&
            SPMV_HIP_LIB=$PWD/tools/ab/libspmv_hip_p11.so run abp11_total 300 python tools/ab_env.py --format csr --rounds 3 --total &&
            run bw_probe 300 tools/bw_probe;;
    abdata) run ab_stream_probe 300 python tools/ab_env.py --format csr --env SPMV_CSR_STREAM_PROBE=P3,P4,PA,PG,PH,PI,PJ --rounds 5 --total &&

            run bw_probe 300 tools/bw_probe;;
    rehot) run shard_rehearse_hot 1100 python tools/shard_rehearse.py --gpus 1,8 --hot=-1,262144,131072,65536 --reps 10;;
    rew) run shard_rehearse_w3 1100 python tools/shard_rehearse.py --gpus 8 --row-weights 2,3,5 --reps 10 &&
         run shard_rehearse_graph 1100 python tools/shard_rehearse.py --gpus 1,8 --row-weights 4 --reps 10 --graph;;
    absy) run test_sell_ystage 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "sell" &&
          run ab_sell_ystage 300 python tools/ab_env.py --format sell --env SPMV_SELL_YSTAGE=0,1 --rounds 5 --total &&
          run ab_sell_ystage_banded 300 python tools/ab_env.py --format sell --matrix banded --env SPMV_SELL_YSTAGE=0,1 --rounds 3 --reps 20 --total;;
    abr32) run ab_r_csrf32 300 python tools/ab_env.py --format csrf32 --env SPMV_CSR_XWIN_R=0,4,6 --rounds 4 --total &&
           run ab_r_csr16 300 python tools/ab_env.py --format csr16 --env SPMV_CSR_XWIN_R=0,4,6 --rounds 4 --total;;
    abgraph) run ab_graph_events 300 python tools/ab_env.py --format csr --rounds 4 &&
             run ab_graph_span 300 python tools/ab_env.py --format csr --rounds 4 --total &&
             run ab_graph_replay 300 python tools/ab_env.py --format csr --rounds 4 --total --graph;;
    test16) run gpu_tests_csr16 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "csr16 or csrf32 or xwin";;
    abcmrspipe) run ab_cmrs_pipe 300 python tools/ab_env.py --format cmrs --env SPMV_CMRS_PIPE=0,1 --rounds 5 &&
                run ab_cmrs_pipe_h16 300 python tools/ab_env.py --format cmrs --kw '{"h": 16}' --env SPMV_CMRS_PIPE=0,1 --rounds 4;;
    abxwin) run ab_csr_xwin_mode 600 python tools/ab_env.py --format csr --env SPMV_CSR_XWIN_MODE=0,2,3 --rounds 5;;
    cmrsnt) run cmrs_base 300 python bench.py --format cmrs --per-format no --cpu-seconds 0 &&
            SPMV_STREAM_NT=1 run cmrs_nt 300 python bench.py --format cmrs --per-format no --cpu-seconds 0 &&
            run cmrs_base2 300 python bench.py --format cmrs --per-format no --cpu-seconds 0 &&
            SPMV_STREAM_NT=1 run cmrs_nt2 300 python bench.py --format cmrs --per-format no --cpu-seconds 0 &&
            run coo_ntdef 300 python bench.py --format coo --per-format no --cpu-seconds 0;;
    rehearsec) run shard_rehearse_cmrs 900 python tools/shard_rehearse.py --gpus 1,8 --format cmrs;;
    rehearseg) run shard_rehearse_graph 900 python tools/shard_rehearse.py --gpus 1,8 --row-weights 4 --graph;;
    profrmat) run prof_rmat 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rmat -o run -- python3 bench.py --workload rmat --profile --steps 50;;
    testhot) run gpu_tests_hot 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "hot or rmat_skewed or bitwise or split";;
    testpf) run gpu_tests_pf 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "prefetch or xwin";;
    sweeppf) run sweep_pf 600 python tools/sweep.py --rounds 3 --env-only --only csr;;
    drvrmat) run drv_csr_rmat 600 ./bin/csr --gen rmat --reps 20 --no-cpu &&
             run drv_cmrs_rmat 600 ./bin/cmrs --gen rmat --reps 20 --no-cpu &&
             run drv_sell_rmat 600 ./bin/sigma_c --gen rmat --reps 20 --sigma 16777216 &&
             run drv_coo_cant 600 ./bin/coo --gen cantlike --copies 32 --reps 20 --no-cpu;;
    sweepxr) run sweep_xwin_remap 600 python tools/sweep.py --rounds 3 --env-only --only csr,sell;;
    testxr) SPMV_XWIN_REMAP=1 run gpu_tests_xr 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "xwin or cantlike or golden";;
    testhyb) run gpu_tests_hyb 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "hyb";;
    sweephyb) run sweep_hyb_rmat 600 python tools/sweep.py --matrix rmat --rounds 2 --reps 10 --only hyb &&
              run sweep_hyb_cant 600 python tools/sweep.py --rounds 2 --only hyb;;
    testf32) run gpu_tests_f32 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "csrf32 or bitwise";;
    rehearse2r) run rehearse2_rmat 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --backend gloo --share-gpu --workload rmat --steps 10;;
    rehearse2) run rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --backend gloo --share-gpu --steps 20;;
    drivers) run drivers 600 python -m pytest tests/test_drivers_gpu.py -q;;
    sweepremap) SPMV_XCD_REMAP=1 run sweep_remap 600 python tools/sweep.py --rounds 2 --only csr,sell,ell;;
    sweeprmat) run sweep_rmat 600 python tools/sweep.py --matrix rmat --rounds 2 --reps 20;;
    counters) run counters 120 rocprofv3 -L;;
    probe) [ -x tools/bw_probe ] || hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o tools/bw_probe; run bw_probe 300 tools/bw_probe;;
    sweepfast) run sweep_fast 600 python tools/sweep.py --only csr,sell,ell --rounds 2;;
    sweepnopair) SPMV_CSR_PAIR=0 run sweep_nopair 300 python tools/sweep.py --only csr --rounds 2;;
    pmcrmat) run pmc_rmat 1100 python tools/pmc_traffic.py --workload rmat --formats csr --kernel csr_tiled_kernel --out traffic_rmat.json --steps 5;;
    rmatexp) run rmat_exp 600 python tools/rmat_exp.py;;
    testsplit) run gpu_tests_split 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "split or cmrs_variant or rmat_skewed or h8-cmrs or bitwise";;
    benchrmatpf) run bench_rmat_pf 900 python bench.py --workload rmat --steps 20 --per-format yes;;
    sweeprmatenv) run sweep_rmat_env 900 python tools/sweep.py --matrix rmat --rounds 2 --reps 10 --env-only --only csr,sell,coo;;
    sweepcantenv) run sweep_cant_env 600 python tools/sweep.py --rounds 2 --env-only --only coo,cmrs,csr;;
    sweeprmatfmt) run sweep_rmat_fmt 600 python tools/sweep.py --matrix rmat --rounds 1 --reps 10 --only sell,cmrs,coo,hyb;;
    pmc) run pmc 1100 python tools/pmc_traffic.py;;
    pmcvar) run pmc_var 1100 python tools/pmc_traffic.py --out traffic_variants.json --formats "csr,csr@SPMV_XCD_REMAP=1,csr:lanes=16,sell:sigma=256,sell,ell@SPMV_XCD_REMAP=1";;
    sweepnt) run sweep_nt 600 python tools/sweep.py --env-only --rounds 3;;
    pmcnt) run pmc_nt 1100 python tools/pmc_traffic.py --out traffic_nt.json --formats "csr@SPMV_STREAM_NT=1,sell@SPMV_STREAM_NT=1,ell@SPMV_STREAM_NT=1,coo,cmrs";;
    ldsconf) run pmc_lds 600 python tools/pmc_stalls.py --formats csr,sell,cmrs --passes ta,sq,lds --out pmc_lds.json;;
    stalls2) run pmc_stalls2 1150 python tools/pmc_stalls.py --formats "csr,csr@SPMV_CSR_XWIN_MODE=0" --passes sq,sq2,tcc,lat,lds,ta --out pmc_stalls_r2.json;;
    stalls) run pmc_stalls 1150 python tools/pmc_stalls.py --formats csr,sell;;
    iterbench) run iter_power 300 python tools/iterate_bench.py --what power --matrix cantlike --iters 200 &&
               run iter_power_graph 300 python tools/iterate_bench.py --what power --matrix cantlike --iters 200 --graph &&
               run iter_power_sell 300 python tools/iterate_bench.py --what power --matrix cantlike --iters 200 --format sell --graph &&
               run iter_cg 600 python tools/iterate_bench.py --what cg --matrix laplacian --k 2000 --iters 500;;
    *) echo "unknown step $s";;
  esac
done
