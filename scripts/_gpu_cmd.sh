set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread -k "copy_engine" > gpurun_out/t_ce.log 2>&1; rc=$?; tail -25 gpurun_out/t_ce.log; [ $rc -eq 0 ] || exit $rc
for w in jacobi rbgs; do for R in 8 4 2; do timeout -k 10 120 python scripts/slab_rehearsal.py --self --workload $w --ranks $R || exit $?; done; done 2>&1 | tee gpurun_out/reh_ce.log
