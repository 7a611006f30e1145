# r05 closing session: bench lines of every workload with their kernel stats,
# the v5 cylinder step (both branches), the slab rehearsal, PMC traffic of the
# headline and GS passes.  Each step has its own time limit; the first failure
# ends the session (no GPU step after a fault or a time-out).
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step_group=${1:-all}
if [ "$step_group" = all ] || [ "$step_group" = bench ]; then
  run b_default 600 python bench.py
  cp gpurun_out/b_default.log gpurun_out/b_jacobi3d_1024.json
  run b_rbgs 600 python bench.py --workload rbgs3d_1024
  run b_512 300 python bench.py --workload jacobi3d_512 --no-cpu-baseline
  run b_channel 300 python bench.py --workload jacobi3d_channel --no-cpu-baseline
  run b_f64 600 python bench.py --workload jacobi2d_8192_f64
  run b_cavity 600 python bench.py --workload cavity2d_128
  run b_pred 300 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3
  run b_predf 300 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --tau-mode fast
  run b_pred64 300 python bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3
  run b_pred64f 300 python bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3 --tau-mode fast
fi
if [ "$step_group" = all ] || [ "$step_group" = cyl ]; then
  run cyl_gs 300 python scripts/cylinder_bench.py --steps 50
  run cyl_j 300 python scripts/cylinder_bench.py --steps 50 --jacobi
fi
if [ "$step_group" = all ] || [ "$step_group" = prof ]; then
  run prof_k4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k4 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
  run prof_gs 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gs -o run --output-format csv -- python3 bench.py --workload rbgs3d_1024 --steps 10 --warmup 2 --no-cpu-baseline
  run prof_f64 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f64 -o run --output-format csv -- python3 bench.py --workload jacobi2d_8192_f64 --steps 5 --warmup 1 --no-cpu-baseline
  run prof_cylj 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cylj -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 20 --jacobi --cpu-steps 0
  run prof_cylgs 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cylgs -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 20 --cpu-steps 0
  P="--steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
  run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py $P
  run pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py $P
  G="--workload rbgs3d_1024 --steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
  run pmc_fetch_gs 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_gs -o run --output-format csv -- python3 bench.py $G
  run pmc_write_gs 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_gs -o run --output-format csv -- python3 bench.py $G
fi
if [ "$step_group" = all ] || [ "$step_group" = slab ]; then
  run rh_j8 300 python scripts/slab_rehearsal.py --self --ranks 8
  run rh_gs8 300 python scripts/slab_rehearsal.py --self --ranks 8 --workload rbgs
fi
echo "== done"
