"""CPU: bench.py's measurement plumbing -- which PMC summary a line's
roofline.traffic may come from (the same workload, and a profiled chain time
within 15 % of the line's own), and the trace-distribution switch of the
headline (SURVEY.md 8(d)'s global walk by default)."""
import json
import os

import numpy as np
import pytest


def _summary(root, name, cfg, kernels, created):
    d = os.path.join(root, "profiles", name)
    os.makedirs(d)
    with open(os.path.join(d, "summary.json"), "w") as f:
        json.dump({"bench_config": cfg, "created": created, "kernels": kernels}, f)


def test_pmc_traffic_matches_workload_and_time(tmp_path, monkeypatch):
    import bench

    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    cfg = {"workload": "w1"}
    k = {"syz::k_a": {"avg_ms": 1.0, "traffic_bytes": 5e9}, "syz::k_b<4u>": {"avg_ms": 0.5, "traffic_bytes": 1e9}}
    _summary(str(tmp_path), "old", cfg, k, 1.0)
    _summary(str(tmp_path), "other", {"workload": "w2"}, k, 3.0)
    b, src, note = bench.pmc_traffic(["syz::k_a", "syz::k_b"], cfg, ("workload",), expect_ms=1.5)
    assert b == pytest.approx(6e9) and src == os.path.join("profiles", "old", "summary.json") and note is None
    # a newer summary of the same workload wins ...
    k2 = {"syz::k_a": {"avg_ms": 1.2, "traffic_bytes": 4e9}, "syz::k_b": {"avg_ms": 0.4, "traffic_bytes": 1e9}}
    _summary(str(tmp_path), "new", cfg, k2, 2.0)
    b, src, _ = bench.pmc_traffic(["syz::k_a", "syz::k_b"], cfg, ("workload",), expect_ms=1.5)
    assert b == pytest.approx(5e9) and "new" in src
    # ... unless its profiled chain is more than 15 % off the line's own time
    b, src, note = bench.pmc_traffic(["syz::k_a", "syz::k_b"], cfg, ("workload",), expect_ms=1.0)
    assert b is None and src is None and "profiled chain" in note
    # no summary of the workload at all
    b, src, note = bench.pmc_traffic(["syz::k_a"], {"workload": "w3"}, ("workload",), expect_ms=1.0)
    assert b is None and note == "no PMC summary of this workload"


def test_walk_configs():
    import bench
    from syzkaller_amd import synth

    g, r = bench.walk_cfg("global"), bench.walk_cfg("region", skew=1)
    assert g.global_walk == 1 and r.global_walk == 0 and r.skew == 1
    assert bench.KNOWN_SYS == {"global": 1, "region": 2048}
    # SURVEY 8(d)'s walk: PCs at 0xffffffff81000000 + 5 b over all 2^20 blocks,
    # each step b <- (4 b + 1 + r % 4) mod 2^20 (csrc/common.h synth_trace)
    pcs, cs, prio = synth.traces(g, 0, 2, 4, np.full(8, 512, np.uint32))
    b = (pcs - np.uint64(0xFFFFFFFF81000000)) // np.uint64(5)
    assert ((pcs - np.uint64(0xFFFFFFFF81000000)) % np.uint64(5) == 0).all() and (b < (1 << 20)).all()
    for c in range(8):
        x = b[int(cs[c]): int(cs[c]) + 512].astype(np.int64)
        d = (x[1:] - 4 * x[:-1] - 1) % (1 << 20)
        assert (d < 4).all()
    assert len(np.unique(b)) > 3000  # not confined to 256-block regions
