set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "f64 or fixed_dt or copy_engine or zero_start or headline or k_levels or temporal_blocking or full_size or local_group or slab or time_step or snapshot" > gpurun_out/t4.log 2>&1; rc=$?; tail -5 gpurun_out/t4.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/t4.log | head -20; exit $rc; }
for w in jacobi rbgs; do for R in 8 4 2; do timeout -k 10 120 python scripts/slab_rehearsal.py --self --workload $w --ranks $R || exit $?; done; done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/reh4.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline 2>&1 | grep -v amdgpu.ids | tail -1 | cut -c1-300
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-slab --steps 3 --warmup 1 > gpurun_out/bench_slab1.log 2>&1; echo slab1 rc=$?; grep -v amdgpu.ids gpurun_out/bench_slab1.log | tail -1 | cut -c1-600
