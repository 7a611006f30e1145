set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "rbgs2d or time_step or cylinder or golden or step" > gpurun_out/t_gs2d.log 2>&1; rc=$?; tail -5 gpurun_out/t_gs2d.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/gs2d_bench.py --ni 2,3,4 --modes 2 --trace > gpurun_out/gs2d.log 2>&1; rc=$?; cat gpurun_out/gs2d.log | grep -v amdgpu.ids; echo "rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/cylinder_bench.py --cpu-steps 0 2>&1 | tail -1
