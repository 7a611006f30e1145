export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu -k "clean_divergence" > gpurun_out/t1.log 2>&1; rc=$?
tail -3 gpurun_out/t1.log; grep -E "^FAILED|Error" gpurun_out/t1.log | head -10
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu -k "time_step or golden or cavity" > gpurun_out/t2.log 2>&1; rc=$?
tail -2 gpurun_out/t2.log; [ $rc -eq 0 ] || exit 1
for p in 0 1 0 1; do CFD_CLEAN_PIPE=$p timeout -k 10 120 python scripts/lex_bench.py || exit 1; done
for p in 0 1; do for br in "--jacobi" ""; do
  CFD_CLEAN_PIPE=$p timeout -k 10 300 python scripts/cylinder_bench.py --steps 40 --cpu-steps 0 $br > gpurun_out/cyl.json || exit 1
  echo "pipe=$p $br $(python3 -c "import json; d=json.load(open('gpurun_out/cyl.json')); print(d['ms_per_step'], d['pressure_ms'])")"
done; done
