set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -k "jacobi3d or headline or slab or zero" > gpurun_out/t3d.log 2>&1; rc=$?; tail -3 gpurun_out/t3d.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash scripts/ab.sh 3 "--steps 10 --warmup 3" cfd-simulations_amd/libcfdsim.so ${OLD_LIB:-build_old/libcfdsim.so}
if [ -f build_trace/libcfdsim.so ]; then
  timeout -k 10 300 env CFDSIM_LIB=$PWD/build_trace/libcfdsim.so python scripts/tbr_trace.py > gpurun_out/trace_k4.log 2>&1 || exit $?
  tail -1 gpurun_out/trace_k4.log | cut -c1-200
fi
