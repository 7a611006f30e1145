#!/usr/bin/env bash
# Runs a sequence of GPU steps on the gpurun box, each under its own time
# limit.  Stops at the first step that faults, aborts or times out (exit codes
# other than 0 = pass and 1 = test failures); logs go to gpurun_out/.
# usage: scripts/gpu_session.sh STEP...   (steps: smoke tests bench prof pmc tiles bench512 bench2d)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export NCCL_SOCKET_IFNAME=${NCCL_SOCKET_IFNAME:-lo}
step() {
  local name=$1 limit=$2; shift 2
  echo "=== $name (limit ${limit}s): $*"
  local t0=$(date +%s)
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)"
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step pytest_gpu 1000 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread ;;
    testsq) step pytest_gpu 900 python -m pytest tests -m gpu -q ;;
    bench) step bench 600 python bench.py ;;
    bench512) step bench512 600 python bench.py --workload jacobi3d_512 --no-cpu-baseline ;;
    bench2d) step bench2d 600 python bench.py --workload jacobi2d_8192_f64 ;;
    tiles) step tiles 900 python bench.py --steps 2 --warmup 1 --sweep-tiles --no-cpu-baseline ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc_fetch) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 30 --no-cpu-baseline ;;
    pmc_write) step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 30 --no-cpu-baseline ;;
    sq_tb) step sq_tb 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d gpurun_out/sq_tb -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 20 --no-cpu-baseline ;;
    sq_march) step sq_march 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d gpurun_out/sq_march -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 20 --tb 1 --no-cpu-baseline ;;
    pmc_fetch_tb) step pmc_fetch_tb 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_tb -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 20 --no-cpu-baseline ;;
    pmc_write_tb) step pmc_write_tb 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_tb -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 20 --no-cpu-baseline ;;
    prof_tb) step prof_tb 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_tb -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    slab1) step slab1 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-slab --steps 3 --warmup 1 ;;
    benchch) step benchch 600 python bench.py --workload jacobi3d_channel --no-cpu-baseline ;;
    testsk) step pytest_k 900 python -m pytest tests -m gpu -q -k "k_levels or variants_agree or temporal or full_size" ;;
    ksweep) step ksweep 900 bash -c 'for cfg in ${KSWEEP:-"3 0 1 0" "3 16 2 0" "3 16 1 256" "4 0 1 0" "2 0 1 0"}; do set -- $cfg; echo "K=$1 rows=$2 PD=$3 zchunk=$4"; python bench.py --no-cpu-baseline --steps 5 --tb $1 --tb-rows $2 --tb-prefetch $3 --tb-zchunk $4 | grep -o "\"value\": [0-9.]*\|avg_launch_ms\": [0-9.]*" | tr "\n" " "; echo; done' ;;
    testspred) step pytest_pred 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "predictor or powf or time_step or golden or persistent" ;;
    benchpred) step benchpred 600 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3 ;;
    benchpred64) step benchpred64 600 python bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3 ;;
    benchpredf) step benchpredf 600 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --tau-mode fast ;;
    benchpred64f) step benchpred64f 600 python bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3 --tau-mode fast ;;
    profpredf) step profpredf 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profpredf -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --no-cpu-baseline --tau-mode fast ;;
    profpred64f) step profpred64f 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profpred64f -o run --output-format csv -- python3 bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3 --no-cpu-baseline --tau-mode fast ;;
    pmc_fetch_predf) step pmc_fetch_predf 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_predf -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 12 --warmup 0 --no-cpu-baseline --tau-mode fast ;;
    pmc_write_predf) step pmc_write_predf 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_predf -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 12 --warmup 0 --no-cpu-baseline --tau-mode fast ;;
    pmc_fetch_pred64) step pmc_fetch_pred64 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_pred64 -o run --output-format csv -- python3 bench.py --workload predictor2d_8192_f64 --steps 12 --warmup 0 --no-cpu-baseline ;;
    pmc_write_pred64) step pmc_write_pred64 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_pred64 -o run --output-format csv -- python3 bench.py --workload predictor2d_8192_f64 --steps 12 --warmup 0 --no-cpu-baseline ;;
    sq_predf) step sq_predf 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d gpurun_out/sq_predf -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 12 --warmup 0 --no-cpu-baseline --tau-mode fast ;;
    pmc_fetch_pred64f) step pmc_fetch_pred64f 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_pred64f -o run --output-format csv -- python3 bench.py --workload predictor2d_8192_f64 --steps 12 --warmup 0 --no-cpu-baseline --tau-mode fast ;;
    pmc_write_pred64f) step pmc_write_pred64f 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_pred64f -o run --output-format csv -- python3 bench.py --workload predictor2d_8192_f64 --steps 12 --warmup 0 --no-cpu-baseline --tau-mode fast ;;
    testspred2) step pytest_pred2 900 python -u -m pytest tests/test_gpu_predictor.py -q -x --timeout 300 --timeout-method thread ;;
    benchpredv1) step benchpredv1 600 env CFD_PRED_VARIANT=1 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --no-cpu-baseline ;;
    profpred) step profpred 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profpred -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --no-cpu-baseline ;;
    profpred64) step profpred64 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profpred64 -o run --output-format csv -- python3 bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3 --no-cpu-baseline ;;
    pmc_fetch_pred) step pmc_fetch_pred 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_pred -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 12 --warmup 0 --no-cpu-baseline ;;
    pmc_write_pred) step pmc_write_pred 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_pred -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 12 --warmup 0 --no-cpu-baseline ;;
    predsweep) step predsweep 600 python scripts/pred_sweep.py ;;
    sq_pred) step sq_pred 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d gpurun_out/sq_pred -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 12 --warmup 0 --no-cpu-baseline ;;
    sq_k4a) step sq_k4a 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d gpurun_out/sq_k4a -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 40 --no-cpu-baseline ;;
    sq_k4b) step sq_k4b 300 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES -d gpurun_out/sq_k4b -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 40 --no-cpu-baseline ;;
    tests2d) step pytest_2d 900 python -m pytest tests -m gpu -q -k "jacobi2d or rbgs2d or time_step or golden" ;;
    sweep2d) step sweep2d 900 bash -c 'for K in ${K2D:-8 10 12}; do echo "K=$K"; python bench.py --workload jacobi2d_8192_f64 --no-cpu-baseline --steps 3 --tb $K | grep -o "\"value\": [0-9.]*\|avg_launch_ms\": [0-9.]*" | tr "\n" " "; echo; done' ;;
    testslocal) step pytest_local 900 python -m pytest tests -m gpu -q -x -k "local_group" ;;
    testsgs) step pytest_gs 900 python -m pytest tests -m gpu -q -k "rbgs or slab" ;;
    benchgs) step benchgs 600 python bench.py --workload rbgs3d_1024 ;;
    gssweep) step gssweep 900 bash -c 'for cfg in ${GSSWEEP:-0:0 2:16 4:0 4:16 2:18 2:20 2:28}; do set -- ${cfg/:/ }; echo "tb=$1 rows=$2"; python bench.py --workload rbgs3d_1024 --no-cpu-baseline --steps 3 --tb $1 --tb-rows $2 | grep -o "\"value\": [0-9.]*\|avg_launch_ms\": [0-9.]*\|iterations_done_last_step\": [0-9]*" | tr "\n" " "; echo; done' ;;
    benchgs_inplace) step benchgs_inplace 600 python bench.py --workload rbgs3d_1024 --tb 1 --no-cpu-baseline --steps 3 ;;
    slab1gs) step slab1gs 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 1 --force-slab --workload rbgs3d_1024 --steps 3 --warmup 1 ;;
    prof2d) step prof2d 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2d -o run --output-format csv -- python3 bench.py --workload jacobi2d_8192_f64 --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc_fetch_2d) step pmc_fetch_2d 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_2d -o run --output-format csv -- python3 bench.py --workload jacobi2d_8192_f64 --steps 1 --warmup 0 --iters 80 --no-cpu-baseline ;;
    pmc_write_2d) step pmc_write_2d 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_2d -o run --output-format csv -- python3 bench.py --workload jacobi2d_8192_f64 --steps 1 --warmup 0 --iters 80 --no-cpu-baseline ;;
    prof_gs) step prof_gs 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gs -o run --output-format csv -- python3 bench.py --workload rbgs3d_1024 --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmc_fetch_gs) step pmc_fetch_gs 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_gs -o run --output-format csv -- python3 bench.py --workload rbgs3d_1024 --steps 1 --warmup 0 --iters 20 --no-cpu-baseline ;;
    pmc_write_gs) step pmc_write_gs 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_gs -o run --output-format csv -- python3 bench.py --workload rbgs3d_1024 --steps 1 --warmup 0 --iters 20 --no-cpu-baseline ;;
    rehearse) step rehearse 900 bash -c 'python scripts/slab_rehearsal.py --ranks 1 && python scripts/slab_rehearsal.py --ranks 8 && python scripts/slab_rehearsal.py --ranks 8 --no-overlap && python scripts/slab_rehearsal.py --ranks 1 --nz 134 && python scripts/slab_rehearsal.py --ranks 2 && python scripts/slab_rehearsal.py --ranks 4' ;;
    rehearse_gs) step rehearse_gs 900 bash -c 'python scripts/slab_rehearsal.py --workload rbgs --ranks 1 && python scripts/slab_rehearsal.py --workload rbgs --ranks 8' ;;
    selfr) step selfr 900 bash -c 'for w in jacobi rbgs; do for R in 8 4 2; do python scripts/slab_rehearsal.py --rccl-self --workload $w --ranks $R || exit $?; done; python scripts/slab_rehearsal.py --rccl-self --workload $w --ranks 8 --no-overlap || exit $?; done' ;;
    prof_selfr) step prof_selfr 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_selfr -o run --output-format csv -- python3 scripts/slab_rehearsal.py --rccl-self --ranks 8 --steps 1 ;;
    selfr2) step selfr2 900 bash -c 'for o in "--comm-priority 0" "--comm-priority 1" "--prefetch 2" "--prefetch 2 --no-overlap" "--workload rbgs" "--workload rbgs --prefetch 2"; do python scripts/slab_rehearsal.py --rccl-self --ranks 8 $o || exit $?; done' ;;
    prof_selfr2) step prof_selfr2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_selfr2 -o run --output-format csv -- python3 scripts/slab_rehearsal.py --rccl-self --ranks 8 --steps 1 ;;
    prof_selfr3) step prof_selfr3 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_selfr3 -o run --output-format csv -- python3 scripts/slab_rehearsal.py --rccl-self --ranks 8 --steps 1 --prefetch 2 ;;
    selfr3) step selfr3 900 bash -c 'for o in "" "--workload rbgs"; do python scripts/slab_rehearsal.py --rccl-self --ranks 8 $o && CFD_SLAB_COMM_CUS=0 python scripts/slab_rehearsal.py --rccl-self --ranks 8 $o && python scripts/slab_rehearsal.py --rccl-self --ranks 4 $o && python scripts/slab_rehearsal.py --rccl-self --ranks 2 $o || exit $?; done' ;;
    testsslab) step pytest_slab 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "slab or local_group or rccl" ;;
    prof_selfgs) step prof_selfgs 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_selfgs -o run --output-format csv -- python3 scripts/slab_rehearsal.py --rccl-self --workload rbgs --ranks 8 --steps 1 ;;
    ab2d) step ab2d 600 bash -c 'for e in 0 1; do echo "CFD_J2_RHS_REGS=$e"; CFD_J2_RHS_REGS=$e python bench.py --workload jacobi2d_8192_f64 --no-cpu-baseline --steps 5 | grep -o "\"value\": [0-9.]*\|avg_launch_ms\": [0-9.]*" | tr "\n" " "; echo; done' ;;
    cyl) step cyl 600 bash -c 'python scripts/cylinder_bench.py && python scripts/cylinder_bench.py --jacobi' ;;
    sq_gs) step sq_gs 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES -d gpurun_out/sq_gs -o run --output-format csv -- python3 bench.py --workload rbgs3d_1024 --steps 1 --warmup 0 --iters 12 --no-cpu-baseline ;;
    sq_2d) step sq_2d 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_BUSY_CYCLES -d gpurun_out/sq_2d -o run --output-format csv -- python3 bench.py --workload jacobi2d_8192_f64 --steps 1 --warmup 0 --iters 80 --no-cpu-baseline ;;
    pmc_fetch_512) step pmc_fetch_512 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_512 -o run --output-format csv -- python3 bench.py --workload jacobi3d_512 --steps 1 --warmup 0 --iters 30 --no-cpu-baseline ;;
    pmc_write_512) step pmc_write_512 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_512 -o run --output-format csv -- python3 bench.py --workload jacobi3d_512 --steps 1 --warmup 0 --iters 30 --no-cpu-baseline ;;
    pmc_fetch_ch) step pmc_fetch_ch 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_ch -o run --output-format csv -- python3 bench.py --workload jacobi3d_channel --steps 1 --warmup 0 --iters 30 --no-cpu-baseline ;;
    pmc_write_ch) step pmc_write_ch 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_ch -o run --output-format csv -- python3 bench.py --workload jacobi3d_channel --steps 1 --warmup 0 --iters 30 --no-cpu-baseline ;;
    prof512) step prof512 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof512 -o run --output-format csv -- python3 bench.py --workload jacobi3d_512 --steps 3 --warmup 1 --no-cpu-baseline ;;
    profch) step profch 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profch -o run --output-format csv -- python3 bench.py --workload jacobi3d_channel --steps 3 --warmup 1 --no-cpu-baseline ;;
    benchgs_n) step benchgs_n 600 python bench.py --workload rbgs3d_1024 --steps 5 ;;
    bench512_n) step bench512_n 600 python bench.py --workload jacobi3d_512 ;;
    benchch_n) step benchch_n 600 python bench.py --workload jacobi3d_channel ;;
    benchcav) step benchcav 600 python bench.py --workload cavity2d_128 --steps 50 --warmup 5 ;;
    prof_cyl) step prof_cyl 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cyl -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 3 --warmup 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "=== all steps done"
