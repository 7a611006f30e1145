export TMPDIR=/tmp; mkdir -p gpurun_out
B="python3 bench.py --workload rbgs3d_1024 --steps 1 --warmup 0 --iters 40 --no-cpu-baseline"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gs -o run --output-format csv -- $B > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_gs -o run --output-format csv -- $B > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_gs -o run --output-format csv -- $B > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES -d gpurun_out/sq_gs_a -o run --output-format csv -- $B > /dev/null || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_WAVES -d gpurun_out/sq_gs_b -o run --output-format csv -- $B > /dev/null || exit 1
echo done
