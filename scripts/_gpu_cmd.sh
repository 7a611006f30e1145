set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=3 --master-addr 127.0.0.1 --master-port 29611 scripts/multirank_check.py --share-gpu --transport ce --quick --size 48 --repeat 5 > gpurun_out/mr3.log 2>&1; echo mr3 rc=$?; grep -c bit-exact gpurun_out/mr3.log; grep -E "MISMATCH|MULTIRANK" gpurun_out/mr3.log | head
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 29612 scripts/multirank_check.py --share-gpu --transport ce --size 48 > gpurun_out/mr2.log 2>&1; echo mr2 rc=$?; grep -c bit-exact gpurun_out/mr2.log; grep -E "MISMATCH|MULTIRANK" gpurun_out/mr2.log | head
for w in jacobi rbgs; do timeout -k 10 120 python scripts/slab_rehearsal.py --self --workload $w --ranks 8 || exit $?; done 2>&1 | grep -v amdgpu.ids
for e in "" "CFD_TBR_XBW=2" "CFD_TBR_XBW=1" "CFD_TBR_SHIFTQ=1"; do echo "== $e"; env $e timeout -k 10 200 python bench.py --steps 8 --warmup 2 --no-cpu-baseline 2>/dev/null | grep -o '"value": [0-9.]*\|avg_launch_ms": [0-9.]*' | tr '\n' ' '; echo; done
for e in "X=0" "CFD_TBR_XBW=2" "CFD_TBR_SHIFTQ=1"; do echo "== pmc $e"; env $e timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$e -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --iters 30 --no-cpu-baseline > /dev/null 2>&1; echo rc=$?; done
