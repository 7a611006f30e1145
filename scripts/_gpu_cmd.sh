set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo -n "== $*: "; timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" 2>/dev/null | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | sort -u | tr '\n' ' '; echo; }
for rep in 1 2; do run --workload rbgs3d_1024; run; done
timeout -k 10 900 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_parity.py tests/test_gpu_solver.py -x -q --timeout 300 --timeout-method thread -m gpu -k "rbgs or gs or 3d or slab" > gpurun_out/t3d.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t3d.log
