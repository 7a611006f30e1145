export TMPDIR=/tmp; mkdir -p gpurun_out
for r in 1 2; do
  for b in base cur; do
    if [ $b = base ]; then d=build_base; else d=.; fi
    for br in "--jacobi" ""; do
      timeout -k 10 300 python $d/scripts/cylinder_bench.py --steps 40 --cpu-steps 0 $br > gpurun_out/cyl.json || exit 1
      echo "$b $br $(python3 -c "import json; d=json.load(open('gpurun_out/cyl.json')); print(d['ms_per_step'], d['pressure_ms'])")"
    done
  done
done
