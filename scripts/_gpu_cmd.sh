export TMPDIR=/tmp; mkdir -p gpurun_out
CFDSIM_LIB=$PWD/build_q64/libcfdsim.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "jacobi3d or tbr or slab or rbgs3d" > gpurun_out/t_v.log 2>&1 || { tail -30 gpurun_out/t_v.log; exit 1; }
tail -1 gpurun_out/t_v.log
B="python bench.py --no-cpu-baseline --steps 10 --warmup 2"
run() { L=$PWD/build_$1/libcfdsim.so; [ $1 = main ] && L=$PWD/cfd-simulations_amd/libcfdsim.so; CFDSIM_LIB=$L timeout -k 10 300 $B $2 > gpurun_out/bp.json 2>/dev/null || exit 1; echo "$1 $2 $(grep -o '"value": [0-9.]*' gpurun_out/bp.json | head -1) $(grep -o 'avg_launch_ms": [0-9.]*' gpurun_out/bp.json | head -1)"; }
for r in 1 2; do run main ""; run q64 ""; done
for r in 1 2; do run main "--workload rbgs3d_1024"; run q64 "--workload rbgs3d_1024"; done
echo ok
