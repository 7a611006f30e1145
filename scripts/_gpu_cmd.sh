export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 60 ./scripts/vsqrt_probe || exit 1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "predictor or step or powf or smoke" > gpurun_out/t_main.log 2>&1 || { tail -30 gpurun_out/t_main.log; exit 1; }
tail -1 gpurun_out/t_main.log
B="python bench.py --workload predictor2d_8192 --no-cpu-baseline --steps 30 --warmup 3"
for r in 1 2; do
CFDSIM_LIB=$PWD/build_pq/libcfdsim.so timeout -k 10 200 $B > gpurun_out/bp.json 2>/dev/null || exit 1; echo "pq $(grep -o 'avg_launch_ms": [0-9.]*' gpurun_out/bp.json)"
timeout -k 10 200 $B > gpurun_out/bp.json 2>/dev/null || exit 1; echo "main $(grep -o 'avg_launch_ms": [0-9.]*' gpurun_out/bp.json)"
done
echo ok
