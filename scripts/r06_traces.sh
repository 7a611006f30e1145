#!/bin/bash
# r06: block-phase traces of the two persistent small-grid solves on the v5 cylinder grid (committed as profiles)
set -o pipefail
bash scripts/r06_pairs.sh &&
timeout -k 10 200 python -u scripts/gs2d_bench.py --ni 5,4 --modes 2,3 --tols 1e-8,0 --trace > gpurun_out/gs_trace_final.log 2>&1
rc=$?
grep -h '^{' gpurun_out/gs_trace_final.log
exit $rc
