# r06 session 3: the tall-tile kernels after the lane-spill work (GS packed
# constants in VGPRs, DPP `old` halo cells, 32-bit LDS-DMA addresses):
# parity first (the 3-D Jacobi / RB-GS pins and parity tests), then the
# headline and RB-GS bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-900; [ $rc -eq 0 ] || exit $rc; }
run t_tbr 900 python -u -m pytest tests/test_gpu_pins.py tests/test_gpu_parity.py -m gpu -x -q -k "jacobi3d or rbgs3d or slab" --timeout 300 --timeout-method thread
run b_default 600 python bench.py --no-cpu-baseline
run b_rbgs 600 python bench.py --workload rbgs3d_1024 --no-cpu-baseline
run b_default2 600 python bench.py --no-cpu-baseline
run b_rbgs2 600 python bench.py --workload rbgs3d_1024 --no-cpu-baseline
echo "== done"
