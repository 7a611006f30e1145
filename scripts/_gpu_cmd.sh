export TMPDIR=/tmp; mkdir -p gpurun_out
for v in lag5 lag6; do
  CFDSIM_LIB=$PWD/build_$v/libcfdsim.so timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests -m gpu -k "rbgs2d or time_step or persistent" > gpurun_out/t_$v.log 2>&1; rc=$?
  echo "$v tests: $(tail -1 gpurun_out/t_$v.log)"; [ $rc -eq 0 ] || exit 1
done
for r in 1 2; do for v in "" lag5 lag6; do
  if [ -z "$v" ]; then L=$PWD/cfd-simulations_amd/libcfdsim.so; else L=$PWD/build_$v/libcfdsim.so; fi
  CFDSIM_LIB=$L timeout -k 10 300 python scripts/cylinder_bench.py --steps 40 --cpu-steps 0 > gpurun_out/cyl.json || exit 1
  echo "${v:-lag3} $(python3 -c "import json; d=json.load(open('gpurun_out/cyl.json')); print(d['ms_per_step'], d['pressure_ms'], d['pressure_us_per_iteration'])")"
done; done
