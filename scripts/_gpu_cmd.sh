set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for w in jacobi3d_512 jacobi3d_channel; do timeout -k 10 300 python bench.py --workload $w > gpurun_out/b_$w.json 2>gpurun_out/b_$w.err; echo "$w rc=$?"; cut -c1-200 gpurun_out/b_$w.json; done
timeout -k 10 300 python bench.py --workload rbgs3d_1024 > gpurun_out/b_rbgs3d_1024.json 2>gpurun_out/b_rbgs.err; echo "gs rc=$?"; cut -c1-200 gpurun_out/b_rbgs3d_1024.json
timeout -k 10 300 python bench.py --workload jacobi2d_8192_f64 > gpurun_out/b_f64.json 2>gpurun_out/b_f64.err; echo "f64 rc=$?"; cut -c1-200 gpurun_out/b_f64.json
