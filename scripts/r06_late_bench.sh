#!/bin/bash
# r06 (late): bench lines of the workloads the late persistent-solve changes touch
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run lb_cav 300 python bench.py --workload cavity2d_128
run lb_cav_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lb_cav_prof -o run --output-format csv -- python3 bench.py --workload cavity2d_128 --steps 20 --warmup 3 --no-cpu-baseline
grep -h '^{' gpurun_out/lb_cav.log | cut -c1-300
head -n 4 gpurun_out/lb_cav_prof/run_kernel_stats.csv | cut -c1-160
echo "== done"
