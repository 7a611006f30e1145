export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests -m gpu -k "fused_step_tails or workgroup_march or time_step or halo_rows or persistent" > gpurun_out/t1.log 2>&1; rc=$?
tail -3 gpurun_out/t1.log; grep -E "^FAILED" gpurun_out/t1.log | head -20
[ $rc -le 1 ] || exit 1
for w in 0 4; do
  CFD_J2_WGM=$w timeout -k 10 200 python bench.py --workload jacobi2d_8192_f64 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/b64_$w.json || exit 1
  echo "wgm=$w $(grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' gpurun_out/b64_$w.json | tr '\n' ' ')"
done
for h in 1 2 4; do
  CFD_J2P_HR=$h timeout -k 10 300 python scripts/cylinder_bench.py --steps 30 --cpu-steps 0 --jacobi > gpurun_out/cyl_j_$h.json || exit 1
  echo "hr=$h $(cat gpurun_out/cyl_j_$h.json)"
done
timeout -k 10 300 python scripts/cylinder_bench.py --steps 30 --cpu-steps 0 > gpurun_out/cyl_gs.json || exit 1
cat gpurun_out/cyl_gs.json
for v in "" lex1 lex2 lex4 lex16 lex7 lex23; do
  if [ -z "$v" ]; then L=$PWD/cfd-simulations_amd/libcfdsim.so; else L=$PWD/build_$v/libcfdsim.so; fi
  CFDSIM_LIB=$L timeout -k 10 120 python scripts/lex_bench.py || exit 1
done
CFDSIM_LIB=$PWD/build_tbrtrace/libcfdsim.so timeout -k 10 200 python scripts/tbr_trace.py > gpurun_out/r04_tbr_trace_k4.json || exit 1
CFDSIM_LIB=$PWD/build_tbrtrace/libcfdsim.so timeout -k 10 200 python scripts/tbr_trace.py --gs > gpurun_out/r04_tbr_trace_gs4.json || exit 1
head -c 600 gpurun_out/r04_tbr_trace_k4.json
