# r06 session 1: the N-rank bench path on the one-GPU lease (--shared-gpu
# lines), the v5 cylinder step after the per-stream failure words and the
# persistent-launch order, the profiled cylinder command of the r05 exit-time
# SIGSEGV (run once; its log is kept), and the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
run cyl_gs 300 python scripts/cylinder_bench.py --steps 50 --cpu-steps 0
run cyl_j 300 python scripts/cylinder_bench.py --steps 50 --jacobi --cpu-steps 0
run prof_cylj 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cylj6 -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 10 --jacobi --cpu-steps 0
run b_default 600 python bench.py --no-cpu-baseline
run sh_j1024 150 python bench.py --gpus 2 --shared-gpu --steps 3 --warmup 1 --no-cpu-baseline
echo "== done"
