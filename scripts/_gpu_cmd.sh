export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do for b in base cur; do
  if [ $b = base ]; then d=build_base; else d=.; fi
  timeout -k 10 300 python $d/bench.py --workload cavity2d_128 --no-cpu-baseline > gpurun_out/cav.json || exit 1
  echo "$b $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' gpurun_out/cav.json | tr '\n' ' ')"
done; done
