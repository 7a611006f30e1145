set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "f64 or pow or time_step or solver" > gpurun_out/t_f64.log 2>&1; rc=$?; tail -5 gpurun_out/t_f64.log; echo "tests rc=$rc"
