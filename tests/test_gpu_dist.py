"""GPU, world_size 2 and 4 over gloo with every rank on cuda:0: the sharded step of
syzkaller_amd/dist.py driving the real kernels (GpuShardOps: the staircase
aggregation of agg.hip, records-mode triage of triage.hip) -- the N>1 path of
bench.py with gloo standing in for RCCL (RCCL refuses two ranks on one GPU).
Two consecutive batches per rank (the shards carry their state), compared
with sequential checkNewSignal (oracle) over the whole rank-major batch.

Reference: syz-fuzzer/fuzzer.go:494-511; SURVEY.md 8(e).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import oracle as O

pytestmark = pytest.mark.gpu

NPROG, CPP, L, NM0, KNOWN = 24, 32, 2048, 100_000, 1024


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, outdir, want_bits, cap, gate=False, backend="gloo"):
    import torch
    import torch.distributed as dist

    from syzkaller_amd import signal as S
    from syzkaller_amd import synth
    from syzkaller_amd.device import Device
    from syzkaller_amd.dist import GpuShardOps, ShardedTriage

    torch.cuda.set_device(0)
    if backend == "nccl":  # RCCL: its collectives run on RCCL's own streams
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = Device(0)
    dev.L.syzsig_ctx_set_timing(dev.eng.h, 1)
    if gate:  # every owner's LDS records pass reports an overflow: the fix-up path
        from syzkaller_amd._lib import SYZSIG_DEBUG_RECS_GATE

        dev.L.syzsig_ctx_set_debug(dev.eng.h, SYZSIG_DEBUG_RECS_GATE)
    cfg = synth.synth_default(skew=1)
    se, sp = dev.synth_m0_shard(cfg, KNOWN, NM0, world, rank)  # this rank's shard of M0, in index order
    ms = dev.deserialize(se, sp)
    ns = S.Signal.make(1 << 16, dev.eng)
    ops = GpuShardOps(dev)
    sh = ShardedTriage(ops, ms, ns, cap=cap)  # first step: levels agreed by all_reduce
    out = {}
    for step in range(2):
        # batch `step`, rank r's programs: a contiguous range of the global, rank-major order
        p0 = (step * world + rank) * NPROG
        cl = torch.full((NPROG * CPP,), L, dtype=torch.int32)
        pcs, cs, cl, prio = dev.synth_traces(cfg, p0, NPROG, CPP, cl)
        pidx = torch.arange(NPROG + 1, dtype=torch.int32, device=dev.dev) * CPP
        sigs, cnt, _ = dev.edge_derive(pcs, cs, cl, pidx)
        pairs = torch.full((int(cnt.to(torch.int64).sum()) + 1,), -1, dtype=torch.int64, device=dev.dev)
        b, bits, cnew = dev.batch(sigs, cs, cnt, prio, new_pairs=pairs, want_bits=want_bits)
        bits, cnew, st = sh.step((b, bits, cnew), prio, rank * NPROG * CPP)
        if step == 0:
            sh.fixed_levels = sh.levels(prio)  # later steps: no collective
        out[f"redos{step}"] = np.array([sh.redos])
        torch.cuda.synchronize()
        if want_bits:
            out[f"bits{step}"] = bits.cpu().numpy().view(np.uint32)
        out[f"cnew{step}"] = cnew.cpu().numpy()
        out[f"pairs{step}"] = pairs[: st["new_pairs"]].cpu().numpy().view(np.uint64)
        out[f"sent{step}"] = np.array([st["sent"], st["received"]])
    se = ms.Serialize()
    out["ms_e"], out["ms_p"] = se.Elems, se.Prios
    sn = ns.Serialize() if not ns.is_nil() else S.Serial()
    out["ns_e"], out["ns_p"] = sn.Elems, sn.Prios
    out["redos"] = np.array([sh.redos, sh.fixups])
    np.savez(os.path.join(outdir, f"r{rank}.npz"), **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,want_bits,cap,gate,backend", [
    (2, True, None, False, "gloo"), (2, False, None, False, "gloo"), (2, False, 256, False, "gloo"),
    (4, True, None, False, "gloo"), (4, False, 256, False, "gloo"), (2, True, None, True, "gloo"),
    (1, False, None, False, "nccl"), (1, True, 256, True, "nccl")])
def test_gpu_sharded_step_gloo(world, want_bits, cap, gate, backend):
    """The stream-ordered step (syzsig_step_*: staircase buckets, equal-split
    exchanges, the owners' LDS-partitioned replay, flags back) on the real
    kernels, 2 or 4 ranks on one GPU over gloo, two consecutive batches;
    cap=256 overflows the first step's buckets, which is redone with a larger
    cap; gate: every owner skips its LDS pass, so every step takes the owner
    fix-up (per-record redo, a second flags exchange).  backend nccl: one rank
    over RCCL (it refuses two ranks on one GPU) -- the exchanges run on RCCL's
    own streams, so the library's ordering against them (its blocking stream
    against torch's null stream, device.py) is what is checked."""
    from tests.test_gpu_triage import oracle_pairs
    from syzkaller_amd import synth
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(worker, args=(world, _port(), d, want_bits, cap, gate, backend), nprocs=world,
                           start_method="spawn")
        res = [dict(np.load(os.path.join(d, f"r{r}.npz"))) for r in range(world)]
    if gate:
        assert all(int(x["redos"][1]) == 2 for x in res)  # one fix-up per step
    cfg = synth.synth_default(skew=1)
    m0e, m0p = synth.m0(cfg, KNOWN, NM0)
    oms = O.deserialize(m0e, m0p)
    ons = O.OSig()
    cl = synth.call_lengths(NPROG, CPP, L)
    pidx = synth.prog_call_index(NPROG, CPP)
    for step in range(2):
        for r in range(world):  # serial order: batch by batch, rank-major inside a batch
            pcs, cs, prio = synth.traces(cfg, (step * world + r) * NPROG, NPROG, CPP, cl)
            sigs, cnt, _ = O.exec_batch(pcs, cs, cl, pidx)
            ons, obits, ocnew = O.triage_batch_into(oms, sigs, cs, cnt, prio, ons)
            np.testing.assert_array_equal(res[r][f"cnew{step}"], ocnew[: cnt.size])
            if want_bits:
                np.testing.assert_array_equal(res[r][f"bits{step}"], obits[: (sigs.size + 31) // 32])
            np.testing.assert_array_equal(np.sort(res[r][f"pairs{step}"]), oracle_pairs(sigs, cs, cnt, obits))
    assert sum(int(x[f"sent{s}"][0]) for x in res for s in range(2)) == \
        sum(int(x[f"sent{s}"][1]) for x in res for s in range(2))
    # a fresh context's first step may void itself once (its distinct-ratio guess
    # for the LDS partitions is learned by the exact redo); the second never does,
    # and a 256-record cap always overflows the first
    assert all(int(x["redos1"][0]) == int(x["redos0"][0]) for x in res)
    assert all(int(x["redos0"][0]) >= (1 if cap else 0) for x in res)
    ge = np.concatenate([x["ms_e"] for x in res])
    gpr = np.concatenate([x["ms_p"] for x in res])
    oe, op = oms.Serialize()
    o1, o2 = np.argsort(ge), np.argsort(oe)
    np.testing.assert_array_equal(ge[o1], oe[o2])
    np.testing.assert_array_equal(gpr[o1], op[o2])
    ne = np.concatenate([x["ns_e"] for x in res])
    npr = np.concatenate([x["ns_p"] for x in res])
    oe, op = ons.Serialize()
    o1, o2 = np.argsort(ne), np.argsort(oe)
    np.testing.assert_array_equal(ne[o1], oe[o2])
    np.testing.assert_array_equal(npr[o1], op[o2])


def minimize_worker(rank, world, port, outdir):
    import torch
    import torch.distributed as dist

    from syzkaller_amd.device import Device
    from syzkaller_amd.dist import GpuMinimizeOps, sharded_minimize

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = Device(0)
    off, e, p = _min_corpus()
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(dev.dev)  # noqa: E731
    keep, n = sharded_minimize(GpuMinimizeOps(dev), t(off, np.int64), t(e, np.int32), t(p, np.int8),
                               hint_distinct=1 << 16)
    np.save(os.path.join(outdir, f"m{rank}.npy"), keep.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


def _min_corpus():
    rng = np.random.default_rng(77)
    lens = rng.geometric(1 / 200, size=5000)
    off = np.zeros(lens.size + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    U = 1 << 16
    base = rng.integers(0, U, size=lens.size)
    stride = rng.integers(0, U // 2, size=lens.size) * 2 + 1
    ctx = np.repeat(np.arange(lens.size), lens)
    k = np.arange(int(off[-1])) - off[:-1].astype(np.int64)[ctx]
    e = ((base[ctx] + k * stride[ctx]) & (U - 1)).astype(np.uint32)
    p = rng.integers(0, 4, size=e.size).astype(np.int8)
    return off, e, p


def test_gpu_sharded_minimize_gloo_two_ranks():
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(minimize_worker, args=(world, _port(), d), nprocs=world, start_method="spawn")
        keeps = [np.load(os.path.join(d, f"m{r}.npy")) for r in range(world)]
    off, e, p = _min_corpus()
    exp = O.minimize(off, e, p)
    for k in keeps:
        assert np.nonzero(k)[0].tolist() == exp


@pytest.mark.parametrize("nshards", [1, 3, 8])
def test_synth_m0_shard_equals_filtered_m0(gpu, nshards):
    """syzsig_synth_m0_shard_dev (how a rank builds its shard of the 1B-element
    M0) = synth_m0 filtered by owner_of, in index order."""
    import torch

    from syzkaller_amd import synth
    from syzkaller_amd.dist import owner_of_torch

    cfg = synth.synth_default()
    n = 3_000_017
    ge, gp = gpu.synth_m0(cfg, 2048, n)
    own = owner_of_torch(ge, nshards)
    for g in range(nshards):
        e, p = gpu.synth_m0_shard(cfg, 2048, n, nshards, g)
        assert torch.equal(e, ge[own == g]) and torch.equal(p, gp[own == g])
