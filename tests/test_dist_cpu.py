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


class NumpyShardOps:
    def partition(self, batch, serial_base, levels, nshards):
        sigs, cs, cl, prio = batch["sigs"], batch["call_start"], batch["call_len"], batch["call_prio"]
        lvl = {(v & 0xFF): i for i, v in enumerate(levels)}
        recs, owners, pos_of = [], [], []
        for c in range(cl.size):
            for j in range(int(cl[c])):
                e = int(sigs[int(cs[c]) + j])
                recs.append((e << 32) | (lvl[int(prio[c])] << 24) | ((serial_base + c) & SER))
                owners.append(_owner(e, nshards))
                pos_of.append(int(cs[c]) + j)
        order = sorted(range(len(recs)), key=lambda i: owners[i])
        send = np.array([recs[i] for i in order], dtype=np.uint64).view(np.int64)
        send_pos = np.zeros(sigs.size, np.int64)
        for k, i in enumerate(order):
            send_pos[pos_of[i]] = k
        counts = [owners.count(g) for g in range(nshards)]
        return torch.from_numpy(send.copy()), send_pos, counts

    def triage_records(self, shard, new_signal, recs, levels):
        r = recs.numpy().view(np.uint64)
        flags = np.zeros(r.size, np.uint8)
        by_k = {}
        for i, x in enumerate(r):
            by_k.setdefault(int(x) & SER, []).append(i)
        for k in sorted(by_k):
            upd = {}
            for i in by_k[k]:
                e, p = int(r[i]) >> 32, levels[(int(r[i]) >> 24) & 0xFF]
                if e not in shard or p > shard[e]:
                    flags[i] = 1
                    upd[e] = max(p, upd.get(e, -999))
            for e, p in upd.items():
                shard[e] = p
                new_signal[e] = max(p, new_signal.get(e, -999))
        return torch.from_numpy(flags), {"records": int(r.size)}

    def unpartition(self, batch, send_pos, back):
        b = back.numpy()
        bits = np.array([b[send_pos[i]] for i in range(send_pos.size)], np.uint8)
        cs, cl = batch["call_start"], batch["call_len"]
        cnew = np.array([bits[int(cs[c]): int(cs[c]) + int(cl[c])].any() for c in range(cl.size)], np.uint8)
        return bits, cnew


class NumpyStairOps(NumpyShardOps):
    """The aggregated routing of agg.hip restated: per element, the first call
    at each level; only the staircase (a level's first call precedes every
    higher level's) is sent; flags come back as (call, elem) pairs."""

    def partition(self, batch, serial_base, levels, nshards):
        sigs, cs, cl, prio = batch["sigs"], batch["call_start"], batch["call_len"], batch["call_prio"]
        lvl = {(v & 0xFF): i for i, v in enumerate(levels)}
        first = {}
        for c in range(cl.size):
            lv = lvl[int(prio[c])]
            for j in range(int(cl[c])):
                f = first.setdefault(int(sigs[int(cs[c]) + j]), [None] * 4)
                if f[lv] is None:
                    f[lv] = c
        groups = [[] for _ in range(nshards)]
        for e, f in first.items():
            mk = None
            for lv in range(3, -1, -1):
                if f[lv] is not None and (mk is None or f[lv] < mk):
                    mk = f[lv]
                    groups[_owner(e, nshards)].append((e << 32) | (lv << 24) | ((serial_base + f[lv]) & SER))
        send = np.array([r for g in groups for r in g], dtype=np.uint64)
        return torch.from_numpy(send.view(np.int64).copy()), (send, serial_base), [len(g) for g in groups]

    def unpartition(self, batch, token, back):
        send, serial_base = token
        pairs = {((int(send[i]) & SER) - serial_base, int(send[i]) >> 32) for i in np.nonzero(back.numpy())[0]}
        sigs, cs, cl = batch["sigs"], batch["call_start"], batch["call_len"]
        bits = np.zeros(sigs.size, np.uint8)
        cnew = np.zeros(cl.size, np.uint8)
        for c in range(cl.size):
            for j in range(int(cl[c])):
                if (c, int(sigs[int(cs[c]) + j])) in pairs:
                    bits[int(cs[c]) + j] = 1
                    cnew[c] = 1
        return bits, cnew


def make_rank_batch(rank, ncalls, seed):
    rng = np.random.default_rng(seed + rank)
    cl = rng.integers(0, 40, size=ncalls).astype(np.uint32)
    cs = np.zeros(ncalls, np.uint64)
    cs[1:] = np.cumsum(cl[:-1])
    sigs = rng.integers(0, 300, size=int(cl.sum())).astype(np.uint32)
    prio = rng.choice(np.array([0, 1, 2, 3], np.uint8), size=ncalls)
    return {"sigs": sigs, "call_start": cs, "call_len": cl, "call_prio": prio}


def m0_global(seed):
    rng = np.random.default_rng(seed)
    e = rng.choice(300, size=150, replace=False)
    return {int(x): int(rng.integers(0, 4)) for x in e}


def worker(rank, world, port, outdir, ncalls, seed, stair):
    from syzkaller_amd.dist import ShardedTriage

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    batch = make_rank_batch(rank, ncalls, seed)
    shard = {e: p for e, p in m0_global(seed).items() if _owner(e, world) == rank}
    news = {}
    st = ShardedTriage(NumpyStairOps() if stair else NumpyShardOps(), shard, news)
    bits, cnew, stats = st.step(batch, torch.from_numpy(batch["call_prio"]), rank * ncalls)
    json.dump({"bits": bits.tolist(), "cnew": cnew.tolist(), "shard": shard, "new": news, "stats": stats},
              open(os.path.join(outdir, f"r{rank}.json"), "w"))
    dist.destroy_process_group()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("stair", [False, True])
@pytest.mark.parametrize("seed", [1, 2])
def test_sharded_step_equals_sequential_checknewsignal(seed, stair):
    """stair: route only each element's staircase (the aggregated routing)."""
    from oracle import oracle as O

    world, ncalls = 2, 60
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(worker, args=(world, free_port(), d, ncalls, seed, stair), nprocs=world,
                           start_method="spawn")
        res = [json.load(open(os.path.join(d, f"r{r}.json"))) for r in range(world)]
    # sequential reference over the concatenated batch (rank-major serial order)
    parts = [make_rank_batch(r, ncalls, seed) for r in range(world)]
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
    sent = sum(r["stats"]["sent"] for r in res)
    assert sent == sum(r["stats"]["received"] for r in res)
    assert sent < sigs.size if stair else sent == sigs.size


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
