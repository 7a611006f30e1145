set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { lib=$1; shift; if [ -n "$lib" ]; then export CFDSIM_LIB=$PWD/$lib/libcfdsim.so; else unset CFDSIM_LIB; fi
  echo -n "== $lib $*: "; timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline "$@" 2>/dev/null | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | sort -u | tr '\n' ' '; echo; }
for rep in 1 2 3; do for lib in "" build_gsown; do run "$lib" --workload rbgs3d_1024; done; done
export CFDSIM_LIB=$PWD/build_gsown/libcfdsim.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu -k "rbgs3d or slab" > gpurun_out/tgs.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/tgs.log
