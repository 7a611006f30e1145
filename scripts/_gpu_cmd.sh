set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_all.log 2>&1; rc=$?; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t_all.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids | tail -2
timeout -k 10 300 python scripts/cylinder_bench.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/cyl_gs.log
timeout -k 10 300 python scripts/cylinder_bench.py --jacobi 2>&1 | grep -v amdgpu.ids | tee gpurun_out/cyl_j.log
