#!/bin/bash
# r06: streaming policy on the tile rows no neighbour reads (CFD_TBR_NTI) -- A/B of the headline
set -o pipefail
mkdir -p gpurun_out
T="timeout -k 10"
: > gpurun_out/nti.log
for rep in 1 2; do
  $T 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/nti.log 2>&1 || exit 1
  CFDSIM_LIB=$PWD/abvar/libcfdsim_nti.so $T 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline >> gpurun_out/nti.log 2>&1 || exit 1
done
CFDSIM_LIB=$PWD/abvar/libcfdsim_nti.so $T 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "1024 or 512" >> gpurun_out/nti.log 2>&1
rc=$?
grep -h '^{' gpurun_out/nti.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['value'], d['roofline']['frac'], d['roofline'].get('avg_launch_ms'))"
tail -n 2 gpurun_out/nti.log
exit $rc
