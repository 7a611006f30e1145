export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu -k "clean_divergence or time_step or lex" > gpurun_out/t1.log 2>&1; rc=$?
tail -3 gpurun_out/t1.log; grep -E "^FAILED" gpurun_out/t1.log | head -20
[ $rc -eq 0 ] || exit 1
for r in 1 2; do
for v in "" lexrow; do
  if [ -z "$v" ]; then L=$PWD/cfd-simulations_amd/libcfdsim.so; else L=$PWD/build_$v/libcfdsim.so; fi
  CFDSIM_LIB=$L timeout -k 10 120 python scripts/lex_bench.py || exit 1
done
done
timeout -k 10 300 python scripts/cylinder_bench.py --steps 30 --cpu-steps 0 --jacobi > gpurun_out/cyl_j.json || exit 1
timeout -k 10 300 python scripts/cylinder_bench.py --steps 30 --cpu-steps 0 > gpurun_out/cyl_gs.json || exit 1
cat gpurun_out/cyl_j.json gpurun_out/cyl_gs.json
