# r05: tall-tile phase traces (trace build), ghost-3 rehearsal, SQ and PMC counters of the shipped K = 4 kernels
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
run trace_k4 300 env CFDSIM_LIB=$PWD/build_trace/libcfdsim.so python scripts/tbr_trace.py
run trace_gs4 300 env CFDSIM_LIB=$PWD/build_trace/libcfdsim.so python scripts/tbr_trace.py --gs
run rh_j8g3 300 python scripts/slab_rehearsal.py --self --ranks 8 --ghost 3
P="--steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
run sq_k4a 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d gpurun_out/sq_k4a -o run --output-format csv -- python3 bench.py $P
run sq_k4b 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES -d gpurun_out/sq_k4b -o run --output-format csv -- python3 bench.py $P
run pmc_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py $P
run pmc_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py $P
G="--workload rbgs3d_1024 --steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
run sq_gsa 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d gpurun_out/sq_gsa -o run --output-format csv -- python3 bench.py $G
run sq_gsb 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES -d gpurun_out/sq_gsb -o run --output-format csv -- python3 bench.py $G
