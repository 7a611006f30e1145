# r06: predictor cells-per-lane sweep (CFD_PRED_VEC) in both tau modes, f32
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 1 2 4; do
  for m in exact fast; do
    CFD_PRED_VEC=$v timeout -k 10 120 python bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --tau-mode $m --no-cpu-baseline > gpurun_out/ps_${v}_${m}.log 2>&1 || exit 1
    python -c "
import json
d=json.loads([l for l in open('gpurun_out/ps_${v}_${m}.log') if l.startswith('{')][-1])
print('vec $v $m', d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline']['kernel'])
"
  done
done
