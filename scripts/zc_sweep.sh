set -e
for zc in 0 342 128; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --tb-zchunk $zc | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | tr '\n' ' '; echo " zc=$zc"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/zc_$zc -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 30 --no-cpu-baseline --tb-zchunk $zc > /dev/null 2>&1
done
