# r06 closing session A: bench lines of every workload (CPU baselines
# included, as the driver runs them) and rocprof kernel statistics (with the
# kernel trace, for steady-state averages) of the shipped kernels.  Each step
# has its own time limit; the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run f_default 600 python bench.py
run f_rbgs 600 python bench.py --workload rbgs3d_1024
run f_512 300 python bench.py --workload jacobi3d_512 --no-cpu-baseline
run f_channel 300 python bench.py --workload jacobi3d_channel --no-cpu-baseline
run f_f64 600 python bench.py --workload jacobi2d_8192_f64
run f_cavity 600 python bench.py --workload cavity2d_128
run f_pred 300 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3
run f_predf 300 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --tau-mode fast
run f_pred64 300 python bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3
run f_pred64f 300 python bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3 --tau-mode fast
run f_cyl_gs 300 python scripts/cylinder_bench.py --steps 50
run f_cyl_j 300 python scripts/cylinder_bench.py --steps 50 --jacobi
echo "== done"
