set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "rbgs2d or time_step or cylinder or golden or step" > gpurun_out/t_gs2d.log 2>&1; rc=$?; tail -5 gpurun_out/t_gs2d.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/cylinder_bench.py --cpu-steps 0 > gpurun_out/cyl.log 2>&1; rc=$?; tail -3 gpurun_out/cyl.log; echo "cyl rc=$rc"
[ $rc -eq 0 ] || exit $rc
CFD_GS_PERSIST=0 timeout -k 10 300 python scripts/cylinder_bench.py --cpu-steps 0 2>&1 | tail -2
