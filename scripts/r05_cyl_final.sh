# r05 late: the v5 cylinder step (both branches, CPU baseline included) and the
# GS branch's kernel statistics after the persistent GS's early publish
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run cyl_gs 300 python scripts/cylinder_bench.py --steps 50
run cyl_j 300 python scripts/cylinder_bench.py --steps 50 --jacobi
run prof_cylgs 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cylgs -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 20 --cpu-steps 0
run gs_trace 300 python scripts/gs2d_bench.py --ni 4 --modes 2 --tols 1e-8,0 --trace
echo "== done"
