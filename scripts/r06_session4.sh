# r06 session 4: the predictor's packed-pair arithmetic (VEC = 2, f32):
# parity (predictor tests, step fixtures), then the four predictor bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run t_pred 600 python -u -m pytest tests/test_gpu_predictor.py tests/test_gpu_solver.py tests/test_gpu_cavity.py -m gpu -x -q --timeout 300 --timeout-method thread
run b_pred 300 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --no-cpu-baseline
run b_predf 300 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --tau-mode fast --no-cpu-baseline
run b_pred64 300 python bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3 --no-cpu-baseline
run cyl_j 300 python scripts/cylinder_bench.py --steps 50 --jacobi --cpu-steps 0
echo "== done"
