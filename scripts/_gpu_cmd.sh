export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_predictor.py -x -q --timeout 120 --timeout-method thread -k quiescent > gpurun_out/t_q.log 2>&1 || { tail -30 gpurun_out/t_q.log; exit 1; }
tail -1 gpurun_out/t_q.log
for r in 1 2; do
  timeout -k 10 200 python scripts/cylinder_bench.py --cpu-steps 0 --steps 40 > gpurun_out/cy.json 2>/dev/null || exit 1
  timeout -k 10 200 python scripts/cylinder_bench.py --cpu-steps 0 --steps 40 --jacobi > gpurun_out/cyj.json 2>/dev/null || exit 1
  echo "gs $(grep -o 'ms_per_step": [0-9.]*' gpurun_out/cy.json | head -1) jac $(grep -o 'ms_per_step": [0-9.]*' gpurun_out/cyj.json | head -1)"
done
timeout -k 10 200 python bench.py --workload cavity2d_128 --no-cpu-baseline > gpurun_out/cav.json 2>/dev/null || exit 1
grep -o '"value": [0-9.]*\|ms_per_step": [0-9.]*' gpurun_out/cav.json | tr '\n' ' '; echo
echo ok
