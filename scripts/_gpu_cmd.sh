set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py --workload cavity2d_128 --steps 20 --warmup 3 > gpurun_out/cav.json 2>gpurun_out/cav.err; echo "rc=$?"; cut -c1-300 gpurun_out/cav.json
