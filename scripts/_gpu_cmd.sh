export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu -k "jacobi3d" > gpurun_out/t1.log 2>&1; rc=$?
tail -2 gpurun_out/t1.log; grep -E "^FAILED" gpurun_out/t1.log | head -5
[ $rc -eq 0 ] || exit 1
bash scripts/ab.sh 3 "--steps 10 --warmup 2" cfd-simulations_amd/libcfdsim.so build_rotr0/libcfdsim.so || exit 1
