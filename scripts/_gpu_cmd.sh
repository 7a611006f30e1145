set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "clean_divergence or time_step or step or golden or energy or cavity or diagnostics" > gpurun_out/t_lex.log 2>&1; rc=$?; tail -3 gpurun_out/t_lex.log; echo "tests rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cyl2 -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 10 --warmup 2 --cpu-steps 0 > gpurun_out/prof_cyl2.log 2>&1; echo "prof rc=$?"; tail -1 gpurun_out/prof_cyl2.log
