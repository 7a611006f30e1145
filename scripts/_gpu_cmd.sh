export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu -k "last_jacobi2d_path or cavity or persistent" > gpurun_out/t1.log 2>&1; rc=$?
tail -3 gpurun_out/t1.log; grep -E "^FAILED|Error" gpurun_out/t1.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --workload cavity2d_128 --no-cpu-baseline > gpurun_out/cav.json || exit 1
grep -o '"kernel": "[^"]*"\|avg_launch_ms": [0-9.]*\|"value": [0-9.]*' gpurun_out/cav.json
