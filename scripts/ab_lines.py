#!/usr/bin/env python3
"""Summarize gpurun_out/<tag>/bench_*.log: per variant and rep, the headline
and each line's ms (and the K3 stages)."""
import glob
import json
import os
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r05"
for f in sorted(glob.glob(os.path.join("gpurun_out", tag, "bench_*.log"))):
    line = [x for x in open(f) if x.startswith("{")]
    if not line:
        print(os.path.basename(f), "no JSON line")
        continue
    d = json.loads(line[-1])
    st = d.get("stages", {})
    out = [f"{os.path.basename(f)[6:-4]:14s} step {d['ms_per_step']:.3f} chain {d['roofline']['avg_launch_ms']:.3f} "
           f"(scat {st.get('part_ms', 0):.3f} agg {st.get('agg_ms', 0):.3f} fin {st.get('finalize_ms', 0):.3f}) "
           f"frac {d['roofline']['frac']:.3f}"]
    for k, v in d.get("lines", {}).items():
        ms = v.get("ms", v.get("ms_per_batch"))
        out.append(f"{k} {ms:.3f}")
    print(" | ".join(out))
