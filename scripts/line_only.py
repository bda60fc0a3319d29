"""Run one of bench.py's extra lines alone (c5, c4, c1, gw, rw, pipe, poll, edge; then the walk: global | region), for
profiling: the line's JSON object on stdout."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from syzkaller_amd.device import Device  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "c5"
WALK = sys.argv[2] if len(sys.argv) > 2 else "global"  # the headline's trace distribution
dev = Device(0)
dev.L.syzsig_ctx_set_timing(dev.eng.h, 1)
pairs = torch.empty(4 * 2048 * 5939 + 64, dtype=torch.int64, device=dev.dev)
if which == "c5":
    out = bench.c5_line(dev, pairs)
elif which == "c1":
    out = bench.c1_line(dev)
elif which == "gw":
    out = bench.c2_walk_line(dev, pairs, 4096, 64, 4096, "global")
elif which == "rw":
    out = bench.c2_walk_line(dev, pairs, 4096, 64, 4096, "region")
elif which == "poll":
    out = bench.poll_line(dev)
elif which == "edge":
    import numpy as np

    from syzkaller_amd._lib import SYZSIG_DEBUG_EDGE_MARKALL, SYZSIG_DEBUG_EDGE_PASSES

    mode = os.environ.get("EDGE_MODE", "")  # force K2's marking mode: markall | passes
    if mode:
        dev.eng.set_debug(SYZSIG_DEBUG_EDGE_MARKALL if mode == "markall" else SYZSIG_DEBUG_EDGE_PASSES)
    P, C, L = 4096, 64, 4096
    cl = torch.full((P * C,), L, dtype=torch.int32)
    pcs, cs, cl, _ = dev.synth_traces(bench.walk_cfg(WALK), 0, P, C, cl)
    pidx = torch.arange(P + 1, dtype=torch.int32, device=dev.dev) * C
    sigs = torch.empty(pcs.numel(), dtype=torch.int32, device=dev.dev)
    cnt = torch.empty(P * C, dtype=torch.int32, device=dev.dev)
    comp = torch.empty(P, dtype=torch.int32, device=dev.dev)
    ms = []
    for i in range(6):
        dev.edge_derive(pcs, cs, cl, pidx, sigs, cnt, comp)
        ms.append(dev.L.syzsig_ctx_last_ms(dev.eng.h))
    out = {"walk": WALK, "edge_dev_ms": float(np.median(ms[1:])), "all": ms,
           "signals": int(cnt.to(torch.int64).sum().item()),
           "checksum": int(sigs.to(torch.int64).sum().item())}
elif which == "pipe":
    out = bench.pipeline_line(dev, pairs, 4096, 64, 4096, WALK)
else:
    P, C, L = 4096, 64, 4096
    sigs, cs, cnt, prio, _, _ = bench.synth_batch(dev, bench.walk_cfg(WALK), 0, P, C, L)
    out = bench.c4_rank_line(dev, sigs, cs, cnt, prio, P, C, L, WALK)
print(json.dumps(out), flush=True)
