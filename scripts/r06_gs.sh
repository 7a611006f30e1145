#!/bin/bash
# r06: persistent 2-D RB-GS with 5 iterations per block: parity, trace, cylinder step
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pins.py -k "rbgs2d" > gpurun_out/gs_pins.log 2>&1 &&
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_solver.py tests/test_gpu_cavity.py > gpurun_out/gs_solver.log 2>&1 &&
$T 200 python -u scripts/gs2d_bench.py --ni 5,4 --modes 2 --tols 1e-8,0 --trace > gpurun_out/gs_trace.log 2>&1 &&
$T 200 python -u scripts/cylinder_bench.py --steps 50 --cpu-steps 0 > gpurun_out/gs_cyl.log 2>&1
rc=$?
tail -n 2 gpurun_out/gs_pins.log gpurun_out/gs_solver.log; grep -h '^{' gpurun_out/gs_trace.log gpurun_out/gs_cyl.log
exit $rc
