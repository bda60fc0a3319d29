#!/usr/bin/env python3
"""Table of gpu_ab.sh runs: ms/step and the K3 stage times per variant."""
import glob
import json
import sys

tag = sys.argv[1]
for f in sorted(glob.glob(f"gpurun_out/{tag}_ab_*.log")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "no json", e)
        continue
    s = d["stages"]
    print(f"{f.split('/')[-1]:24s} step {d['ms_per_step']:.3f}  chain {d['roofline']['avg_launch_ms']:.3f}  "
          f"part {s['part_ms']:.3f} agg {s['agg_ms']:.3f} fin {s['finalize_ms']:.3f}  frac {d['roofline']['frac']:.3f}")
