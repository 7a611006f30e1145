#!/bin/bash
# r06 (late): the round-end checks on the final tree: the whole -m gpu suite,
# smoke(), the default bench line (N = 1)
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/val_gpu.log 2>&1 &&
$T 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/val_smoke.log 2>&1 &&
$T 400 python -u bench.py > gpurun_out/val_bench.log 2>&1
rc=$?
tail -n 2 gpurun_out/val_gpu.log; tail -n 1 gpurun_out/val_smoke.log
grep -h '^{' gpurun_out/val_bench.log | cut -c1-400
exit $rc
