set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for R in 8 2; do for g in 0 3; do timeout -k 10 200 python scripts/slab_rehearsal.py --self --ranks $R --ghost $g --steps 3 2>/dev/null | tail -1; done; done
for R in 8 2; do timeout -k 10 200 python scripts/slab_rehearsal.py --self --ranks $R --workload rbgs --steps 3 2>/dev/null | tail -1; done
