# r06 closing session B: rocprof kernel statistics (kernel trace kept for the
# steady-state averages), PMC traffic (FETCH_SIZE and WRITE_SIZE in separate
# passes) and SQ counters of the shipped kernels, and the R = 8 slab rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
pmc() { local name=$1; shift; timeout -s KILL 90 rocprofv3 --pmc $1 -d gpurun_out/$name -o run --output-format csv -- "${@:2}" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run p_k4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_k4 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
run p_gs 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_gs -o run --output-format csv -- python3 bench.py --workload rbgs3d_1024 --steps 10 --warmup 2 --no-cpu-baseline
run p_pred 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_pred -o run --output-format csv -- python3 bench.py --workload predictor2d_8192 --steps 20 --warmup 3 --no-cpu-baseline
run p_pred64 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_pred64 -o run --output-format csv -- python3 bench.py --workload predictor2d_8192_f64 --steps 20 --warmup 3 --no-cpu-baseline
run p_cylgs 300 rocprofv3 --kernel-trace --stats -d gpurun_out/p_cylgs -o run --output-format csv -- python3 scripts/cylinder_bench.py --steps 20 --cpu-steps 0
P="--steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
G="--workload rbgs3d_1024 --steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
Q="--workload predictor2d_8192 --steps 10 --warmup 1 --no-cpu-baseline"
Q64="--workload predictor2d_8192_f64 --steps 10 --warmup 1 --no-cpu-baseline"
pmc m_k4f FETCH_SIZE python3 bench.py $P
pmc m_k4w WRITE_SIZE python3 bench.py $P
pmc m_gsf FETCH_SIZE python3 bench.py $G
pmc m_gsw WRITE_SIZE python3 bench.py $G
pmc m_prf FETCH_SIZE python3 bench.py $Q
pmc m_prw WRITE_SIZE python3 bench.py $Q
pmc m_pr64f FETCH_SIZE python3 bench.py $Q64
pmc m_pr64w WRITE_SIZE python3 bench.py $Q64
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
B="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES"
pmc s_pra "$A" python3 bench.py $Q
pmc s_prb "$B" python3 bench.py $Q
pmc s_pr64a "$A" python3 bench.py $Q64
pmc s_pr64b "$B" python3 bench.py $Q64
pmc s_gsa "$A" python3 bench.py $G
run rh_j8 300 python scripts/slab_rehearsal.py --self --ranks 8
run rh_gs8 300 python scripts/slab_rehearsal.py --self --ranks 8 --workload rbgs
echo "== done"
