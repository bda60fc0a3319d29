#!/usr/bin/env python3
"""Condense a profile.sh run (gpurun_out/<tag>/) into profiles/<tag>/:

  kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as written)
  summary.json       per kernel: launches, avg duration, and per-launch HBM
                     bytes from the separate PMC passes, corrected as
                     MI355X_MICROARCH.md "HBM [CDNA4]" prescribes:
                       read bytes  = FETCH_SIZE (KiB) * 1024 * 2   (gfx950 tallies
                                     128-B requests at 64 B)
                       write bytes = WRITE_SIZE (KiB) * 1024
                     plus the L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS).

bench.py reads summary.json for roofline.traffic (bytes per k_probe launch).
usage: summarize_prof.py gpurun_out/prof_r01 profiles/r01_prof
"""
import collections
import csv
import json
import os
import shutil
import sys


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").strip()


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    out = collections.OrderedDict()
    if os.path.exists(stats):  # a counter-only run (scripts/pmc_sq.sh) has no trace
        shutil.copy(stats, os.path.join(dst, "kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            out[short(r["Name"])] = {"launches": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                     "pct": float(r["Percentage"])}
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in sorted(os.listdir(src)):
        f = os.path.join(src, d, "run_counter_collection.csv")
        if not d.startswith("pmc") or not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in pmc.items():
        e = out.setdefault(k, {})
        avg = {c: sum(v) / len(v) for c, v in cs.items()}
        if "FETCH_SIZE" in avg:
            e["read_bytes"] = avg["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in avg:
            e["write_bytes"] = avg["WRITE_SIZE"] * 1024
        if "read_bytes" in e and "write_bytes" in e:
            e["traffic_bytes"] = e["read_bytes"] + e["write_bytes"]
        if "SQ_WAVE_CYCLES" in avg and avg["SQ_WAVE_CYCLES"]:
            # quad-cycle counters (MI355X_MICROARCH.md): shares of wave time
            wc = avg["SQ_WAVE_CYCLES"]
            e["sq_shares"] = {c: avg[c] / wc for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                        "SQ_WAIT_INST_LDS") if c in avg}
        if "SQ_LDS_IDX_ACTIVE" in avg and avg["SQ_LDS_IDX_ACTIVE"] and "SQ_LDS_BANK_CONFLICT" in avg:
            e["lds_bank_conflict_share"] = avg["SQ_LDS_BANK_CONFLICT"] / avg["SQ_LDS_IDX_ACTIVE"]
        if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
            t = avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]
            e["l2_hit"] = avg["TCC_HIT_sum"] / t if t else None
        e["pmc_raw"] = avg
    log = os.path.join(src, "trace.log")
    bench = None
    if os.path.exists(log):
        for line in open(log):
            if line.startswith("{"):
                bench = json.loads(line)
    import time

    summary = {"source": src, "bench_args": os.environ.get("BENCH_ARGS", ""), "created": time.time(), "kernels": out}
    if bench:
        summary["bench_config"] = bench.get("config")
        with open(os.path.join(dst, "bench.json"), "w") as f:
            f.write(json.dumps(bench) + "\n")
    with open(os.path.join(dst, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    for k, e in out.items():
        if "traffic_bytes" in e or e.get("pct", 0) > 1:
            print(f"{k:40s} {e.get('avg_ms', 0):9.3f} ms  traffic {e.get('traffic_bytes', 0) / 1e9:7.3f} GB  "
                  f"L2 hit {e.get('l2_hit') or 0:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
