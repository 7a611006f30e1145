#!/bin/bash
# r06 (late): the v5 cylinder step after the paired-level persistent Jacobi and
# the 5-iteration padded-LDS persistent RB-GS: bench lines with the CPU
# baselines, and rocprof kernel statistics of both branches.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run c_gs 300 python scripts/cylinder_bench.py --steps 50
run c_j 300 python scripts/cylinder_bench.py --steps 50 --jacobi
run cp_gs 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cp_gs -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 20 --cpu-steps 0
run cp_j 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cp_j -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 20 --jacobi --cpu-steps 0
grep -h '^{' gpurun_out/c_gs.log gpurun_out/c_j.log | cut -c1-400
echo "== done"
