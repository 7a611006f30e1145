#!/bin/bash
# r06: full GPU suite after the paired-level persistent Jacobi, then the v5 cylinder steps
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pairs_gpu_suite.log 2>&1 &&
$T 200 python -u scripts/cylinder_bench.py --steps 50 --jacobi --cpu-steps 0 > gpurun_out/pairs_cyl_jacobi.log 2>&1 &&
$T 200 python -u scripts/cylinder_bench.py --steps 50 --cpu-steps 0 > gpurun_out/pairs_cyl_gs.log 2>&1 &&
$T 120 python -u scripts/j2_trace.py >> gpurun_out/pairs_trace_final.log 2>&1
rc=$?
tail -n 3 gpurun_out/pairs_gpu_suite.log; grep -h '^{' gpurun_out/pairs_cyl_*.log gpurun_out/pairs_trace_final.log
exit $rc
