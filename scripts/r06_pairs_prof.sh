#!/bin/bash
# r06: kernel stats of the cylinder Jacobi step per rows-per-wave setting
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for rw in 2 4; do
  CFD_J2P_NI=10 CFD_J2P_RW=$rw timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rw$rw -o run -- python3 scripts/cylinder_bench.py --steps 30 --jacobi --cpu-steps 0 > gpurun_out/prof_rw$rw.log 2>&1 || exit 1
done
for rw in 2 4; do
  f=$(find gpurun_out/prof_rw$rw -name '*kernel_stats.csv' | head -n 1)
  echo "== rw $rw: $f"; head -n 6 "$f"
done
