export TMPDIR=/tmp; mkdir -p gpurun_out
CFD_J2P_RW=4 timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu -k "jacobi2d or persistent or cavity or time_step or golden" > gpurun_out/t1.log 2>&1; rc=$?
tail -1 gpurun_out/t1.log; grep -E "^FAILED" gpurun_out/t1.log | head -5
[ $rc -eq 0 ] || exit 1
for r in 1 2; do for rw in 2 4; do
  CFD_J2P_RW=$rw timeout -k 10 300 python scripts/cylinder_bench.py --steps 40 --cpu-steps 0 --jacobi > gpurun_out/cyl.json || exit 1
  echo "rw=$rw cyl $(python3 -c "import json; d=json.load(open('gpurun_out/cyl.json')); print(d['ms_per_step'], d['pressure_ms'], d['pressure_us_per_iteration'])")"
  CFD_J2P_RW=$rw timeout -k 10 300 python bench.py --workload cavity2d_128 --no-cpu-baseline > gpurun_out/cav.json || exit 1
  echo "rw=$rw cav $(grep -o '"ms_per_step": [0-9.]*\|avg_launch_ms": [0-9.]*' gpurun_out/cav.json | tr '\n' ' ')"
done; done
