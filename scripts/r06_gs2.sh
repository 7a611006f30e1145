#!/bin/bash
# r06: the persistent GS without the workspace init and edge-row launches: parity, cylinder step
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pins.py tests/test_gpu_solver.py tests/test_gpu_integration_binding.py -k "rbgs or gs or persistent or health or solver or binding or step" > gpurun_out/gs2_tests.log 2>&1 &&
$T 200 python -u scripts/cylinder_bench.py --steps 50 --cpu-steps 0 > gpurun_out/gs2_cyl.log 2>&1
rc=$?
tail -n 2 gpurun_out/gs2_tests.log; grep -h '^{' gpurun_out/gs2_cyl.log | cut -c1-300
exit $rc
