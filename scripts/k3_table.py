"""Summarize K3-only bench logs (gpurun_out/<tag>/k3_*.log): stage times per variant."""
import glob
import json
import sys

for f in sorted(glob.glob(f"gpurun_out/{sys.argv[1]}/k3_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            st, tr = d["stages"], d["triage"]
            print(f.split("/")[-1][:-4].ljust(16), "ms/step %.3f" % d["ms_per_step"],
                  "part %.3f agg %.3f fin %.3f" % (st["part_ms"], st["agg_ms"], st["finalize_ms"]),
                  "frac %.3f" % d["roofline"]["frac"], "changed", tr.get("changed"), "pairs", tr.get("new_pairs"))
