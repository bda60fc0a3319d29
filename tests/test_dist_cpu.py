"""CPU, world_size 2 over gloo: the sharded step of syzkaller_amd/dist.py
(levels all-reduce, counts + records all-to-all, owner triage, flags back)
equals sequential checkNewSignal over the whole batch.  The device half is
replaced by a numpy restatement (records-mode triage in serial order), so the
exchange logic itself is what is tested here; the device kernels are checked
against unsharded triage in tests/test_gpu_minimize_shard.py."""
import json
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.test_gpu_minimize_shard import _owner

SER = 0xFFFFFF


HDR_VOID, HDR_OVF, HDR_COUNT = 1 << 63, 1 << 62, (1 << 40) - 1


class NumpyStepOps:
    """The stream-ordered sharded step of csrc (syzsig_step_send_dev /
    _own_dev / _back_dev / _finish) restated over torch CPU tensors: buckets of
    cap + 1 words per owner with a header (count | VOID | OVF), the owner's
    records-mode replay in serial order, a status byte per flags bucket.
    stair=True: each element's staircase is sent (agg.hip), else every record.
    fail_owner: this rank's first non-exact owner pass skips its records
    (status 2), as an LDS partition overflow would."""

    device = "cpu"

    def __init__(self, rank, stair=True, fail_owner=False, spill=False, raise_send=False, raise_own=False):
        self.rank, self.stair, self.fail_owner = rank, stair, fail_owner
        self.spill = spill            # every capped (non-exact) run spills a cell: VOID headers, src_void 1
        self.raise_send = raise_send  # send raises (as ERANGE on the serial range would), host side
        self.raise_own = raise_own    # own raises (as a failed reserve would), host side
        self.exact_sends = 0
        self.pairs = set()
        self.st = {"src_void": 0, "global_void": 0, "owners_void": 0, "max_out": 0}

    @staticmethod
    def alloc(n, dtype):
        return torch.zeros(n, dtype=dtype)

    @staticmethod
    def records(batch):
        return int(batch["sigs"].size)

    def send(self, batch, serial_base, levels, nshards, cap, send, exact=False):
        if self.raise_send:
            raise OverflowError("step_send: batch serial order exceeds 2^24 calls")
        self.exact_sends += bool(exact)
        if self.spill and not exact:
            # a void run (k_stair_heads): every bucket VOID with count 0
            sv = send.numpy().view(np.uint64)
            for g in range(nshards):
                sv[g * (cap + 1)] = HDR_VOID
            self.pairs = set()
            self.st = {"src_void": 1, "global_void": 0, "owners_void": 0, "records": int(batch["sigs"].size),
                       "sent": 0, "max_out": 0, "inserted": 0, "changed": 0, "own_distinct": 0, "new_pairs": 0}
            return
        sigs, cs, cl, prio = batch["sigs"], batch["call_start"], batch["call_len"], batch["call_prio"]
        lvl = {(v & 0xFF): i for i, v in enumerate(levels)}
        groups = [[] for _ in range(nshards)]
        first = {}
        for c in range(cl.size):
            lv = lvl[int(prio[c])]
            for j in range(int(cl[c])):
                e = int(sigs[int(cs[c]) + j])
                if not self.stair:
                    groups[_owner(e, nshards)].append((e << 32) | (lv << 24) | ((serial_base + c) & SER))
                else:
                    f = first.setdefault(e, [None] * 4)
                    if f[lv] is None:
                        f[lv] = c
        for e, f in first.items():
            mk, recs = None, []
            for lv in range(3, -1, -1):
                if f[lv] is not None and (mk is None or f[lv] < mk):
                    mk = f[lv]
                    recs.append((e << 32) | (lv << 24) | ((serial_base + f[lv]) & SER))
            groups[_owner(e, nshards)] += recs[::-1]  # serial order, as k_stair_bucket writes them
        mx = max(len(x) for x in groups)
        sv = send.numpy().view(np.uint64)
        for g, recs in enumerate(groups):
            base = g * (cap + 1)
            sv[base] = len(recs) | (HDR_OVF if mx > cap else 0)
            for k, r in enumerate(recs[:cap]):
                sv[base + 1 + k] = r
        self.pairs = set()
        self.st = {"src_void": 0, "global_void": 0, "owners_void": 0, "records": int(sigs.size),
                   "sent": sum(len(x) for x in groups), "max_out": mx, "inserted": 0, "changed": 0,
                   "own_distinct": 0, "new_pairs": 0}

    def own(self, shard, new_signal, recv, nshards, cap, levels, flags, exact=False):
        if self.raise_own:
            raise MemoryError("step_own: out of device memory")
        rv = recv.numpy().view(np.uint64)
        fl = flags.numpy()
        fl[:] = 0
        hdr = [int(rv[g * (cap + 1)]) for g in range(nshards)]
        status = 0
        if any(h & (HDR_VOID | HDR_OVF) for h in hdr):
            status = 1
        elif self.fail_owner and not exact:
            self.fail_owner = False
            status = 2
        else:
            by_k = {}
            for g in range(nshards):
                for j in range(min(hdr[g] & HDR_COUNT, cap)):
                    i = g * (cap + 1) + 1 + j
                    by_k.setdefault(int(rv[i]) & SER, []).append(i)
            seen, changed, inserted = set(), set(), set()
            for k in sorted(by_k):
                upd = {}
                for i in by_k[k]:
                    e, p = int(rv[i]) >> 32, levels[(int(rv[i]) >> 24) & 0xFF]
                    seen.add(e)
                    if e not in shard or p > shard[e]:
                        fl[i] = 1
                        upd[e] = max(p, upd.get(e, -999))
                for e, p in upd.items():
                    if e not in shard:
                        inserted.add(e)
                    changed.add(e)
                    shard[e] = p
                    new_signal[e] = max(p, new_signal.get(e, -999))
            self.st["own_distinct"] += len(seen)
            self.st["inserted"] += len(inserted)
            self.st["changed"] += len(changed)
        for g in range(nshards):
            fl[g * (cap + 1)] = status

    def back(self, batch, serial_base, send, nshards, cap, back):
        sv, bk = send.numpy().view(np.uint64), back.numpy()
        for g in range(nshards):
            base = g * (cap + 1)
            if bk[base] == 1:
                self.st["global_void"] = 1
                continue
            if bk[base] == 2:
                self.st["owners_void"] |= 1 << g
                continue
            for j in range(min(int(sv[base]) & HDR_COUNT, cap)):
                if bk[base + 1 + j]:
                    r = int(sv[base + 1 + j])
                    self.pairs.add(((r & SER) - serial_base, r >> 32))

    def finish(self):
        st = dict(self.st)
        st["new_pairs"] = len(self.pairs)
        self.st["global_void"] = self.st["owners_void"] = 0
        self.st["inserted"] = self.st["changed"] = self.st["own_distinct"] = 0
        return st

    def outputs(self, batch):
        sigs, cs, cl = batch["sigs"], batch["call_start"], batch["call_len"]
        bits = np.zeros(sigs.size, np.uint8)
        cnew = np.zeros(cl.size, np.uint8)
        for c in range(cl.size):
            for j in range(int(cl[c])):
                if (c, int(sigs[int(cs[c]) + j])) in self.pairs:
                    bits[int(cs[c]) + j] = 1
                    cnew[c] = 1
        return bits, cnew


def make_rank_batch(rank, ncalls, seed, universe=300):
    rng = np.random.default_rng(seed + rank)
    cl = rng.integers(0, 40, size=ncalls).astype(np.uint32)
    cs = np.zeros(ncalls, np.uint64)
    cs[1:] = np.cumsum(cl[:-1])
    sigs = rng.integers(0, universe, size=int(cl.sum())).astype(np.uint32)
    prio = rng.choice(np.array([0, 1, 2, 3], np.uint8), size=ncalls)
    return {"sigs": sigs, "call_start": cs, "call_len": cl, "call_prio": prio}


def m0_global(seed, universe=300):
    rng = np.random.default_rng(seed)
    e = rng.choice(universe, size=universe // 2, replace=False)
    return {int(x): int(rng.integers(0, 4)) for x in e}


def rank_calls(rank, ncalls, uneven):
    """Calls of rank r: uneven loads give later ranks more calls."""
    return ncalls + (25 * rank if uneven else 0)


def worker(rank, world, port, outdir, ncalls, seed, stair, uneven, cap, fail_rank):
    from syzkaller_amd.dist import ShardedTriage

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    batch = make_rank_batch(rank, rank_calls(rank, ncalls, uneven), seed)
    base = sum(rank_calls(r, ncalls, uneven) for r in range(rank))
    shard = {e: p for e, p in m0_global(seed).items() if _owner(e, world) == rank}
    news = {}
    ops = NumpyStepOps(rank, stair, fail_owner=rank == fail_rank)
    st = ShardedTriage(ops, shard, news, cap=cap, levels=[0, 1, 2, 3])
    bits, cnew, stats = st.step(batch, torch.from_numpy(batch["call_prio"]), base)
    stats.update(redos=st.redos, fixups=st.fixups, cap_after=st.cap)
    json.dump({"bits": bits.tolist(), "cnew": cnew.tolist(), "shard": shard, "new": news, "stats": stats},
              open(os.path.join(outdir, f"r{rank}.json"), "w"))
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,stair,uneven,cap,fail_rank,seed", [
    (2, False, False, None, -1, 1), (2, True, False, None, -1, 2),
    (2, True, True, 4, -1, 3),       # a cap of 4 records: every bucket overflows, the step is redone
    (4, True, True, None, -1, 4),
    (4, True, True, None, 2, 5),     # owner 2 skips its records (LDS overflow): the fix-up round
    (4, False, True, 16, 1, 6),      # every record routed, both a redo and a fix-up
])
def test_sharded_step_equals_sequential_checknewsignal(world, stair, uneven, cap, fail_rank, seed):
    """The stream-ordered sharded step (dist.ShardedTriage over gloo, the device
    half restated in numpy) against sequential checkNewSignal over the whole
    rank-major batch (syz-fuzzer/fuzzer.go:494-511): bits, call flags, the
    union of the shards and of the newSignal shards."""
    from oracle import oracle as O

    ncalls = 40
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(worker, args=(world, free_port(), d, ncalls, seed, stair, uneven, cap, fail_rank),
                           nprocs=world, start_method="spawn")
        res = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(world)]
    parts = [make_rank_batch(r, rank_calls(r, ncalls, uneven), seed) for r in range(world)]
    sigs = np.concatenate([p["sigs"] for p in parts])
    off, cs = 0, []
    for p in parts:
        cs.append(p["call_start"] + off)
        off += p["sigs"].size
    cs = np.concatenate(cs)
    cl = np.concatenate([p["call_len"] for p in parts])
    prio = np.concatenate([p["call_prio"] for p in parts])
    m0 = m0_global(seed)
    ms, ns, obits, ocnew = O.triage_batch(np.array(list(m0), np.uint32), np.array(list(m0.values()), np.int8),
                                          sigs, cs, cl, prio)
    got_bits = np.concatenate([np.array(r["bits"], np.uint8) for r in res])
    exp_bits = np.array([(obits[i >> 5] >> (i & 31)) & 1 for i in range(sigs.size)], np.uint8)
    np.testing.assert_array_equal(got_bits, exp_bits)
    np.testing.assert_array_equal(np.concatenate([r["cnew"] for r in res]), ocnew)
    merged = {}
    for r in res:
        merged.update({int(k): v for k, v in r["shard"].items()})
    assert merged == ms.to_dict()
    nm = {}
    for r in res:
        nm.update({int(k): v for k, v in r["new"].items()})
    assert nm == ns.to_dict()
    st = [r["stats"] for r in res]
    assert all(x["redos"] == (1 if cap is not None else 0) for x in st), st  # a small cap: one redo
    assert all(x["fixups"] == (1 if fail_rank >= 0 else 0) for x in st), st
    assert sum(x["changed"] for x in st) == len(ns.to_dict())
    assert all(x["cap_after"] == st[0]["cap_after"] for x in st)  # every rank agrees on the cap


# ---- Minimize sharded by element (dist.sharded_minimize) ----

def _owner_np(e, n):
    """syz::owner_of (csrc/common.h) over a u32 array."""
    h = (np.asarray(e, np.uint64) * np.uint64(0x9E3779B1) + np.uint64(0x7F4A7C15)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(0xFFFFFFFF)
    h ^= h >> np.uint64(16)
    return ((h * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


class NumpyMinimizeOps:
    """The data-split Minimize (csrc/minimize.hip syzsig_minimize_split_dev /
    _resolve_dev) restated: the part's range of contexts in sort order (cut at
    about total/nparts entries), per element the winner (prio, -rank) inside the
    range as e << 32 | (prio ^ 0x80) << 24 | (0xFFFFFF - rank), grouped by
    owner; the owner takes the max per element and marks the winners."""

    @staticmethod
    def _order(off):
        lens = np.diff(off.astype(np.int64))
        return np.lexsort((np.arange(lens.size), -lens)), lens

    def split(self, off, elems, prios, nparts, part, nshards, hint_distinct=0):
        order, lens = self._order(off)
        cum = np.concatenate([[0], np.cumsum(lens[order])])  # entries of ranks < r
        total = int(cum[-1])

        def cut(k):  # first rank r with cum[r] >= k * total / nparts (nctx if none)
            if k == 0:
                return 0
            if k >= nparts:
                return order.size
            r = int(np.searchsorted(cum[:-1], total * k // nparts, side="left"))
            return min(r, order.size)

        lo, hi = cut(part), cut(part + 1)
        best = {}
        for r in range(lo, hi):
            c = int(order[r])
            for j in range(int(off[c]), int(off[c + 1])):
                e = int(elems[j])
                v = ((int(prios[j]) & 0xFF) ^ 0x80) << 24 | (0xFFFFFF - r)
                if v > best.get(e, -1):
                    best[e] = v
        groups = [[] for _ in range(nshards)]
        for e, v in best.items():
            groups[int(_owner_np([e], nshards)[0])].append((e << 32) | v)
        send = np.array([x for g in groups for x in g], dtype=np.uint64).view(np.int64)
        return torch.from_numpy(send.copy()), [len(g) for g in groups]

    def resolve(self, off, recs):
        order, _ = self._order(off)
        best = {}
        for x in recs.numpy().view(np.uint64):
            e, v = int(x) >> 32, int(x) & 0xFFFFFFFF
            best[e] = max(v, best.get(e, -1))
        keep = np.zeros(order.size, np.uint8)
        for v in best.values():
            keep[order[0xFFFFFF - (v & 0xFFFFFF)]] = 1
        return torch.from_numpy(keep)


def _corpus(seed, n=300, U=2000):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 60, size=n)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    elems = np.concatenate([rng.choice(U, size=int(L), replace=False) for L in lens]).astype(np.uint32)
    prios = rng.integers(0, 4, size=elems.size).astype(np.int8)
    return off, elems, prios


def minimize_worker(rank, world, port, outdir, seed, hint):
    from syzkaller_amd.dist import sharded_minimize

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    off, elems, prios = _corpus(seed)
    keep, n = sharded_minimize(NumpyMinimizeOps(), off, elems, prios, hint_distinct=hint)
    json.dump({"keep": keep.tolist(), "n": n}, open(os.path.join(outdir, f"m{rank}.json"), "w"))
    dist.destroy_process_group()


@pytest.mark.parametrize("seed,world,hint", [(3, 2, 0), (4, 2, 1500), (5, 3, 0), (6, 4, 1800)])
def test_sharded_minimize_equals_minimize(seed, world, hint):
    """Data-split Minimize over gloo (each rank reads only its range of the
    corpus) against oracle Minimize over the whole corpus."""
    from oracle import oracle as O

    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(minimize_worker, args=(world, free_port(), d, seed, hint), nprocs=world,
                           start_method="spawn")
        res = [json.load(open(os.path.join(d, f"m{r}.json"))) for r in range(world)]
    off, elems, prios = _corpus(seed)
    exp = O.minimize(off, elems, prios)
    for r in res:  # every rank holds the reduced result
        assert np.nonzero(np.array(r["keep"]))[0].tolist() == exp and r["n"] == len(exp)


@pytest.mark.parametrize("nparts", [1, 2, 3, 5])
def test_minimize_split_restatement_parts_cover_corpus(nparts):
    """The part ranges tile the sort order and balance entries; the winners of
    all parts resolved together give oracle Minimize (no collective)."""
    from oracle import oracle as O

    off, elems, prios = _corpus(9, n=500)
    ops = NumpyMinimizeOps()
    sends = [ops.split(off, elems, prios, nparts, k, 3) for k in range(nparts)]
    keep = np.zeros(off.size - 1, np.uint8)
    for g in range(3):
        recv = torch.cat([s[g * 0 + sum(c[:g]): sum(c[: g + 1])] for s, c in sends])
        keep |= ops.resolve(off, recv).numpy()
    assert np.nonzero(keep)[0].tolist() == O.minimize(off, elems, prios)


class FailingMinimizeOps(NumpyMinimizeOps):
    """split raises on rank 1 only (as syzsig_minimize_split_dev can with
    ERANGE on a send buffer too small for its part)."""

    def split(self, off, elems, prios, nparts, part, nshards, hint_distinct=0):
        if part == 1:
            raise ValueError("split failed on part 1")
        return super().split(off, elems, prios, nparts, part, nshards, hint_distinct)


def failing_minimize_worker(rank, world, port, outdir):
    from syzkaller_amd.dist import sharded_minimize

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    off, elems, prios = _corpus(7)
    try:
        sharded_minimize(FailingMinimizeOps(), off, elems, prios)
        msg = None
    except Exception as e:  # noqa: BLE001
        msg = f"{type(e).__name__}: {e}"
    json.dump({"err": msg}, open(os.path.join(outdir, f"f{rank}.json"), "w"))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_sharded_minimize_split_failure_raises_on_every_rank():
    """A split that fails on one rank makes every rank raise before the
    all-to-all instead of leaving the others blocked in it."""
    world = 3
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(failing_minimize_worker, args=(world, free_port(), d), nprocs=world, start_method="spawn")
        res = [json.load(open(os.path.join(d, f"f{r}.json")))["err"] for r in range(world)]
    assert res[1] == "ValueError: split failed on part 1"
    assert res[0] and res[2] and "another rank" in res[0] and "another rank" in res[2]


def mode_worker(rank, world, port, outdir, seed, cap, mode):
    """One step with a per-rank failure mode: {"spill": [ranks], "raise_send":
    [ranks], "raise_own": [ranks]}."""
    from syzkaller_amd.dist import ShardedTriage

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    ncalls = mode.get("ncalls", [40] * world)
    batch = make_rank_batch(rank, ncalls[rank], seed)
    shard = {e: p for e, p in m0_global(seed).items() if _owner(e, world) == rank}
    ops = NumpyStepOps(rank, True, spill=rank in mode.get("spill", ()),
                       raise_send=rank in mode.get("raise_send", ()), raise_own=rank in mode.get("raise_own", ()))
    st = ShardedTriage(ops, shard, {}, cap=cap, levels=[0, 1, 2, 3])
    out = {"err": None}
    try:
        bits, cnew, stats = st.step(batch, torch.from_numpy(batch["call_prio"]), sum(ncalls[:rank]))
        out.update(bits=bits.tolist(), redos=st.redos, exact_sends=ops.exact_sends)
    except Exception as e:  # noqa: BLE001
        out["err"] = f"{type(e).__name__}: {e}"
    json.dump(out, open(os.path.join(outdir, f"x{rank}.json"), "w"))
    dist.destroy_process_group()


def _run_mode(world, seed, cap, mode):
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(mode_worker, args=(world, free_port(), d, seed, cap, mode), nprocs=world,
                           start_method="spawn")
        return [json.load(open(os.path.join(d, f"x{r}.json"))) for r in range(world)]


@pytest.mark.timeout(120)
def test_sharded_step_spill_and_cap_overflow_same_step():
    """Rank 1's capped run spills (a void source: it must take its exact path)
    while rank 0's one call fits the cap of 64 records: attempt 1 is void (the
    spill), attempt 2 is void again (rank 1 exact, but over the cap), attempt
    3 succeeds.  Rank 1 stays exact across attempts 2 and 3 -- it must not return
    to the capped cells after the overflow -- and the bits equal
    sequential checkNewSignal."""
    from oracle import oracle as O

    world, seed = 2, 11
    ncalls = [1, 40]
    res = _run_mode(world, seed, 64, {"spill": [1], "ncalls": ncalls})
    assert all(r["err"] is None for r in res), res
    assert res[1]["exact_sends"] == 2 and res[0]["exact_sends"] == 0, res
    assert all(r["redos"] == 2 for r in res), res
    parts = [make_rank_batch(r, ncalls[r], seed) for r in range(world)]
    sigs = np.concatenate([p["sigs"] for p in parts])
    cs = np.concatenate([parts[0]["call_start"], parts[1]["call_start"] + parts[0]["sigs"].size])
    cl = np.concatenate([p["call_len"] for p in parts])
    prio = np.concatenate([p["call_prio"] for p in parts])
    m0 = m0_global(seed)
    _, _, obits, _ = O.triage_batch(np.array(list(m0), np.uint32), np.array(list(m0.values()), np.int8),
                                    sigs, cs, cl, prio)
    exp = np.array([(obits[i >> 5] >> (i & 31)) & 1 for i in range(sigs.size)], np.uint8)
    np.testing.assert_array_equal(np.concatenate([np.array(r["bits"], np.uint8) for r in res]), exp)


@pytest.mark.timeout(120)
@pytest.mark.parametrize("mode,own_err", [({"raise_send": [2]}, "OverflowError"), ({"raise_own": [1]}, "MemoryError")])
def test_sharded_step_failure_raises_on_every_rank(mode, own_err):
    """A host-side failure of send or own on one rank travels in-band (VOID
    headers / a void status byte), so every rank raises at the redo's
    agreement instead of its peers blocking in the all-to-all:
    the failing rank its own error, the others a RuntimeError."""
    world = 3
    res = _run_mode(world, 12, None, mode)
    bad = (mode.get("raise_send") or mode.get("raise_own"))[0]
    for r, x in enumerate(res):
        assert x["err"] is not None, (r, x)
        assert x["err"].startswith(own_err if r == bad else "RuntimeError"), (r, x)


class _FakeNs:
    def __init__(self, n):
        self.n = n

    def Len(self):
        return self.n

    def clear(self):
        pass


class _FakeSharded:
    """What bench.dist_parity needs from dist.ShardedTriage: one step of the
    rank's batch returning (bits, call_new, stats), the pairs written into the
    batch's pairs buffer.  The fake computes rank 0's result with the oracle
    over the whole M0 (what the real step must return for its calls), and
    `corrupt` flips one call flag so the check must fail."""

    def __init__(self, rank, m0e, m0p, pool0, pairs, ns, corrupt):
        self.rank, self.m0e, self.m0p, self.pool0 = rank, m0e, m0p, pool0
        self.pairs, self.ns, self.corrupt = pairs, ns, corrupt

    def step(self, batch, call_prio, serial_base):
        from oracle import oracle as O

        sigs, cs, cnt, prio = (t.numpy() for t in self.pool0[:4])
        if self.rank == 0:
            _, ons, obits, ocnew = O.triage_batch(self.m0e, self.m0p, sigs.view(np.uint32), cs.view(np.uint64),
                                                  cnt.view(np.uint32), prio.view(np.uint8))
            r = np.nonzero(np.unpackbits(obits.view(np.uint8), bitorder="little"))[0].astype(np.uint64)
            call = np.searchsorted(cs.view(np.uint64) + cnt.view(np.uint32).astype(np.uint64), r, side="right")
            pp = np.unique((call.astype(np.uint64) << np.uint64(32)) | sigs.view(np.uint32)[r].astype(np.uint64))
            self.pairs[: pp.size] = torch.from_numpy(pp.view(np.int64))
            cnew = torch.from_numpy(ocnew.copy())
            if self.corrupt:
                cnew[0] ^= 1
            self.ns.n = ons.Len()
            return None, cnew, {"changed": ons.Len(), "new_pairs": int(pp.size)}
        self.ns.n = 0
        return None, torch.zeros(int(cnt.size), dtype=torch.uint8), {"changed": 0, "new_pairs": 0}


def parity_worker(rank, world, port, outdir, corrupt):
    import bench
    from syzkaller_amd.dist import owner_of_torch

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    rng = np.random.default_rng(7)
    P, C, L = 10, 4, 60
    ncalls = P * C
    cs = (np.arange(ncalls, dtype=np.uint64) * L)
    cnt = rng.integers(0, L + 1, ncalls).astype(np.uint32)
    sigs = rng.integers(0, 400, ncalls * L).astype(np.uint32)
    prio = rng.integers(0, 4, ncalls).astype(np.uint8)
    e_all = np.arange(0, 400, 2, dtype=np.uint32)  # M0: every even element, prio 0..3
    p_all = rng.integers(0, 4, e_all.size).astype(np.int8)
    own = owner_of_torch(torch.from_numpy(e_all.view(np.int32)), world).numpy() == rank
    m0e = torch.from_numpy(e_all[own].view(np.int32).copy())
    m0p = torch.from_numpy(p_all[own].copy())
    pool0 = (torch.from_numpy(sigs.view(np.int32)), torch.from_numpy(cs.view(np.int64)),
             torch.from_numpy(cnt.view(np.int32)), torch.from_numpy(prio))
    pairs = torch.zeros(ncalls * L + 8, dtype=torch.int64)
    ns = _FakeNs(0)
    sharded = _FakeSharded(rank, e_all, p_all, pool0, pairs, ns, corrupt)

    class _Dev:
        dev = torch.device("cpu")

    out = bench.dist_parity(_Dev(), sharded, None, pool0, pairs, lambda: None, ns, m0e, m0p, rank, world, P, C,
                            "gloo", nprog=8)
    if rank == 0:
        json.dump(out, open(os.path.join(outdir, "parity.json"), "w"))
    dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [False, True])
def test_bench_dist_parity_plumbing(corrupt):
    """bench.py's parity object for N > 1 (verdict round 5, item 3) over gloo at
    world size 2: rank 0's prefix keys broadcast, M0 gathered from both
    shards, the oracle on the prefix, the union check -- green on a correct
    step, red when one call flag is wrong."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(parity_worker, args=(2, free_port(), d, corrupt), nprocs=2, start_method="spawn")
        out = json.load(open(os.path.join(d, "parity.json")))
    assert out["world_size"] == 2 and out["backend"] == "gloo" and out["checked_programs"] == 8
    assert out["union_ok"] and out["pairs_ok"]
    assert out["call_new_ok"] is (not corrupt)
    assert out["ok"] is (not corrupt)
    assert out["m0_keys_gathered"] > 0
