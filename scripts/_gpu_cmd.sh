export TMPDIR=/tmp; mkdir -p gpurun_out
CFDSIM_LIB=$PWD/build_nt0/libcfdsim.so timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_predictor.py > gpurun_out/t1.log 2>&1 || { tail -5 gpurun_out/t1.log; exit 1; }
tail -1 gpurun_out/t1.log
bash scripts/ab.sh 3 "--workload predictor2d_8192 --steps 10 --warmup 2" cfd-simulations_amd/libcfdsim.so build_nt0/libcfdsim.so || exit 1
for v in nt0; do
  CFDSIM_LIB=$PWD/build_$v/libcfdsim.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pf_$v -o run --output-format csv -- python3 scripts/pred_fetch.py 1 > /dev/null || exit 1
  CFDSIM_LIB=$PWD/build_$v/libcfdsim.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pw_$v -o run --output-format csv -- python3 scripts/pred_fetch.py 1 > /dev/null || exit 1
done
