export TMPDIR=/tmp; mkdir -p gpurun_out
for v in pabl32 pabl64; do
  CFDSIM_LIB=$PWD/build_$v/libcfdsim.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pf_$v -o run --output-format csv -- python3 scripts/pred_fetch.py 1 > /dev/null || exit 1
  CFDSIM_LIB=$PWD/build_$v/libcfdsim.so timeout -k 10 200 python bench.py --workload predictor2d_8192 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/bp.json 2>/dev/null; echo "$v $(grep -o 'avg_launch_ms": [0-9.]*' gpurun_out/bp.json | head -1)"
done
echo ok
