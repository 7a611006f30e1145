# r05 closing SQ counters of the shipped K = 4 Jacobi and 4-level GS passes
set -u
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
P="--steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
G="--workload rbgs3d_1024 --steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
A="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
B="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES"
run sq_k4a 120 rocprofv3 --pmc $A -d gpurun_out/sq_k4a -o run --output-format csv -- python3 bench.py $P
run sq_k4b 120 rocprofv3 --pmc $B -d gpurun_out/sq_k4b -o run --output-format csv -- python3 bench.py $P
run sq_gsa 120 rocprofv3 --pmc $A -d gpurun_out/sq_gsa -o run --output-format csv -- python3 bench.py $G
run sq_gsb 120 rocprofv3 --pmc $B -d gpurun_out/sq_gsb -o run --output-format csv -- python3 bench.py $G
echo "== done"
