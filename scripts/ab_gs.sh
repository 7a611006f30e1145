set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -k "rbgs3d or rbgs_3d or gs3d or slab_rbgs or stop_at_every" > gpurun_out/tgs.log 2>&1; rc=$?; tail -3 gpurun_out/tgs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash scripts/ab.sh 3 "--workload rbgs3d_1024 --steps 6 --warmup 2" cfd-simulations_amd/libcfdsim.so ${OLD_LIB:-build_old/libcfdsim.so}
