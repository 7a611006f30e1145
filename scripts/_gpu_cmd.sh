set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > gpurun_out/tall.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/tall.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2>gpurun_out/bench_final.err; echo "bench rc=$?"; cat gpurun_out/bench_final.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_gs -o run -- python3 bench.py --workload rbgs3d_1024 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/p_gs.json 2>gpurun_out/p_gs.err; echo "prof rc=$?"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p_j -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/p_j.json 2>gpurun_out/p_j.err; echo "prof rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_gs -o run -- python3 bench.py --workload rbgs3d_1024 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>gpurun_out/f_gs.err; echo "pmc rc=$?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/w_gs -o run -- python3 bench.py --workload rbgs3d_1024 --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>gpurun_out/w_gs.err; echo "pmc rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f_j -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>gpurun_out/f_j.err; echo "pmc rc=$?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/w_j -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > /dev/null 2>gpurun_out/w_j.err; echo "pmc rc=$?"
