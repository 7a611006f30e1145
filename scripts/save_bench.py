#!/usr/bin/env python3
"""Copy the JSON bench line out of a gpurun step log into profiles/.

    python scripts/save_bench.py gpurun_out/benchpredf.log profiles/r05_bench_predictor2d_8192_fast_n1.json
"""
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
line = [ln for ln in open(src) if ln.startswith("{") and '"metric"' in ln][-1]
d = json.loads(line)
open(dst, "w").write(json.dumps(d, indent=1) + "\n")
print(dst, d["value"], d.get("roofline", {}).get("frac"))
