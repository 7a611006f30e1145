export TMPDIR=/tmp; mkdir -p gpurun_out
B="python bench.py --workload predictor2d_8192 --no-cpu-baseline --steps 30 --warmup 3"
run() { CFD_PRED_ROWS=$1 CFD_PRED_VEC=$2 timeout -k 10 200 $B > gpurun_out/bp.json 2>/dev/null || exit 1; echo "rows $1 vec $2 $(grep -o 'avg_launch_ms": [0-9.]*' gpurun_out/bp.json)"; }
for r in 1 2; do run 16 2; run 16 4; run 8 2; run 12 2; run 16 1; done
echo ok
