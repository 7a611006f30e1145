# r05: headline bench, rehearsals, other 3-D benches, rocprof of the default bench
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
run bench 300 python bench.py
run rh_j8 300 python scripts/slab_rehearsal.py --self --ranks 8
run rh_j8g4 300 python scripts/slab_rehearsal.py --self --ranks 8 --ghost 4
run rh_g8 300 python scripts/slab_rehearsal.py --self --workload rbgs --ranks 8
run rh_j4 300 python scripts/slab_rehearsal.py --self --ranks 4
run rh_j2 300 python scripts/slab_rehearsal.py --self --ranks 2
run benchgs 300 python bench.py --workload rbgs3d_1024 --no-cpu-baseline
run bench512 300 python bench.py --workload jacobi3d_512 --no-cpu-baseline
run benchch 300 python bench.py --workload jacobi3d_channel --no-cpu-baseline
run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline
