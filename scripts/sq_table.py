"""Summarize rocprofv3 SQ counter CSVs: per kernel, counters summed over
dispatches and divided by the dispatch count (SQ_WAIT*/ACTIVE as a share of
SQ_WAVE_CYCLES).  usage: sq_table.py <dir with */run_counter_collection.csv>..."""
import collections
import csv
import glob
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in glob.glob(d + "/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:34]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((f, r["Dispatch_Id"]))
    print("==", d)
    for k, c in agg.items():
        n = len(disp[k]) / max(1, len({f for f, _ in disp[k]}))
        wc = c.get("SQ_WAVE_CYCLES", 0)
        out = []
        for name, v in sorted(c.items()):
            if name.startswith("SQ_WAIT") or name == "SQ_ACTIVE_INST_ANY":
                out.append(f"{name[3:]}={v / wc:.3f}" if wc else f"{name[3:]}=?")
            else:
                out.append(f"{name[3:]}={v / n:.3g}")
        print(f"  {k}: " + " ".join(out))
