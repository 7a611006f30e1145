set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for n in 8 10 8 10; do echo -n "NI=$n "; CFD_J2P_NI=$n timeout -k 10 200 python scripts/cylinder_bench.py --jacobi --cpu-steps 0 2>&1 | tail -1 | grep -o '"ms_per_step": [0-9.]*\|"pressure_us_per_iteration": [0-9.]*' | tr '\n' ' '; echo; done
for n in 8 10; do echo -n "cavity NI=$n "; CFD_J2P_NI=$n timeout -k 10 200 python bench.py --workload cavity2d_128 --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o '"ms_per_step": [0-9.]*'; done
