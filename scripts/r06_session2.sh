# r06 session 2: the copy-engine landing path (pairs of 2 GiB or more) --
# multiprocess parity with and without landing buffers, then the 1024^3
# two-rank shared-GPU bench lines (Jacobi and RB-GS) that hung in session 1.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-1500; [ $rc -eq 0 ] || exit $rc; }
run mp_tests 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "copy_engine_multiprocess" -v --timeout 300 --timeout-method thread
run sh_j1024 240 python bench.py --gpus 2 --shared-gpu --steps 3 --warmup 1 --no-cpu-baseline
run sh_gs1024 240 python bench.py --gpus 2 --shared-gpu --workload rbgs3d_1024 --steps 2 --warmup 1 --no-cpu-baseline
echo "== done"
