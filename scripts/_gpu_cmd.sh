export TMPDIR=/tmp; mkdir -p gpurun_out
: > gpurun_out/r04_slab_rehearsal.jsonl
for R in 8 4 2; do
  timeout -k 10 300 python scripts/slab_rehearsal.py --self --ranks $R --workload jacobi --ghost 3 >> gpurun_out/r04_slab_rehearsal.jsonl || exit 1
  timeout -k 10 300 python scripts/slab_rehearsal.py --self --ranks $R --workload rbgs >> gpurun_out/r04_slab_rehearsal.jsonl || exit 1
done
tail -c 1500 gpurun_out/r04_slab_rehearsal.jsonl
for w in rbgs3d_1024 jacobi2d_8192_f64 jacobi3d_512 jacobi3d_channel cavity2d_128; do
  timeout -k 10 400 python bench.py --workload $w > gpurun_out/r04_bench_${w}_n1.json || exit 1
  echo "$w $(grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|avg_launch_ms": [0-9.]*' gpurun_out/r04_bench_${w}_n1.json | tr '\n' ' ')"
done
timeout -k 10 400 python bench.py > gpurun_out/r04_bench_jacobi3d_1024_n1.json || exit 1
echo "headline $(grep -o '"value": [0-9.]*\|"frac": [0-9.]*\|avg_launch_ms": [0-9.]*' gpurun_out/r04_bench_jacobi3d_1024_n1.json | tr '\n' ' ')"
timeout -k 10 400 python bench.py --workload predictor2d_8192 > gpurun_out/r04_bench_predictor2d_8192_n1.json || exit 1
timeout -k 10 400 python bench.py --workload predictor2d_8192_f64 > gpurun_out/r04_bench_predictor2d_8192_f64_n1.json || exit 1
timeout -k 10 300 python scripts/cylinder_bench.py --steps 30 > gpurun_out/r04_cyl_gs.json || exit 1
timeout -k 10 300 python scripts/cylinder_bench.py --steps 30 --jacobi > gpurun_out/r04_cyl_j.json || exit 1
cat gpurun_out/r04_cyl_gs.json gpurun_out/r04_cyl_j.json
