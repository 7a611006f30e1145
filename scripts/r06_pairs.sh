#!/bin/bash
# r06: the persistent Jacobi's paired levels -- parity (modes 2 and 3, 4..10
# sweeps per block), the block-phase trace and the fixed cost of a solve on the
# v5 cylinder grid, and the cylinder step
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pins.py -k "jacobi2d_persistent" > gpurun_out/pairs_pins.log 2>&1 &&
: > gpurun_out/pairs_trace.log &&
for c in "10 2" "10 3" "8 2"; do
  set -- $c
  $T 120 python -u scripts/j2_trace.py --ni $1 --mode $2 >> gpurun_out/pairs_trace.log 2>&1 || exit 1
done
$T 120 python -u scripts/j2_overhead.py --ni 10 >> gpurun_out/pairs_trace.log 2>&1 &&
$T 200 python -u scripts/cylinder_bench.py --steps 50 --jacobi --cpu-steps 0 > gpurun_out/pairs_cyl.log 2>&1
rc=$?
tail -n 2 gpurun_out/pairs_pins.log; grep -h '^{' gpurun_out/pairs_trace.log gpurun_out/pairs_cyl.log
exit $rc
