#!/usr/bin/env bash
# A/B timing of in-tree library builds on the GPU box: runs bench.py with each
# CFDSIM_LIB in turn, ROUNDS times, and prints value / launch ms per run.
# usage: scripts/ab.sh ROUNDS "bench args" lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1; args=$2; shift 2
for r in $(seq "$rounds"); do
  for lib in "$@"; do
    out=$(CFDSIM_LIB=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline $args 2>/dev/null)
    rc=$?
    if [ $rc -ne 0 ]; then echo "$lib rc=$rc"; exit $rc; fi
    echo "$lib $(echo "$out" | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | tr '\n' ' ')"
  done
done | tee -a gpurun_out/ab.log
