export TMPDIR=/tmp; mkdir -p gpurun_out
CFDSIM_LIB=$PWD/build_pj/libcfdsim.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "predictor or step or powf" > gpurun_out/t_v.log 2>&1 || { tail -30 gpurun_out/t_v.log; exit 1; }
tail -1 gpurun_out/t_v.log
B="python bench.py --workload predictor2d_8192 --no-cpu-baseline --steps 30 --warmup 3"
run() { L=$PWD/build_$1/libcfdsim.so; [ $1 = main ] && L=$PWD/cfd-simulations_amd/libcfdsim.so; CFDSIM_LIB=$L timeout -k 10 200 $B > gpurun_out/bp.json 2>/dev/null || exit 1; echo "$1 $(grep -o 'avg_launch_ms": [0-9.]*' gpurun_out/bp.json)"; }
for r in 1 2 3; do run main; run pbase; run pj; done
echo ok
