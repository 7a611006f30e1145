set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { lib=$1; shift; if [ -n "$lib" ]; then export CFDSIM_LIB=$PWD/$lib/libcfdsim.so; else unset CFDSIM_LIB; fi
  echo -n "== $lib $*: "; timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline "$@" 2>/dev/null | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | sort -u | tr '\n' ' '; echo; }
for rep in 1 2; do for lib in "" build_nosb; do run "$lib"; run "$lib" --tb 3; run "$lib" --workload rbgs3d_1024; done; done
