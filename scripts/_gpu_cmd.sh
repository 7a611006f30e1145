export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu -k "jacobi3d or rbgs3d" > gpurun_out/t1.log 2>&1; rc=$?
tail -1 gpurun_out/t1.log; grep -E "^FAILED" gpurun_out/t1.log | head -5
[ $rc -eq 0 ] || exit 1
bash scripts/ab.sh 3 "--steps 10 --warmup 2" cfd-simulations_amd/libcfdsim.so build_oldtbr/libcfdsim.so || exit 1
bash scripts/ab.sh 2 "--workload rbgs3d_1024 --steps 4 --warmup 1" cfd-simulations_amd/libcfdsim.so build_oldtbr/libcfdsim.so || exit 1
