"""CPU: K2's parallel round algorithm (csrc/edge.hip, SYZ_EDGE_DEC 4) restated
in Python and checked against the executor's sequential lossy dedup
(executor/executor.h:687-706, restated as `seq_dedup`) on the reference
executor's fixtures, chunk by chunk: every chunk's emitted flags and the
table after it.  This pins the exactness argument of the conflict test on
CPU; tests/test_gpu_edge.py pins the kernel.

Per round, every pending lane evaluates dedup() on the current table: its
decision slot d (first match or zero of its window, or h when forced), its
write slots now or after a re-run (h and the window's empty slots).  Writers
mark those slots; a lane is blocked when an earlier lane marked the bin of d
and some other lane marked d itself; a blocked lane marks its write slots and
d.  Unblocked writers store; blocked lanes run again next round.

sig == 0 is the one write that empties a slot: its forced overwrite stores 0
at slot 0 (executor.h:704), which changes the predicates of every later lane
whose window holds slot 0 (h in 8189..8191, 0).  Such a lane's decision slot
lies in 8189..8191, 0..3, so a sig-0 lane marks all seven of those slots
(ZERO_SLOTS) instead of its window.  And inside a window that holds slot 0
the rest of the argument fails too: a slot there can hold sig while an earlier
slot (slot 0) is empty, so once slot 0 fills again the lane decides at a slot
after today's decision slot, and a later zero write changes a slot it has
read.  A lane whose window holds slot 0 (h in 8189..8191, 0) therefore marks
its whole window, so that every later write into it waits while it is
pending."""
import os

import numpy as np
import pytest

M = 8192
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def exec_hash(a):
    a &= 0xFFFFFFFF
    a = (a ^ 61) ^ (a >> 16)
    a = (a + (a << 3)) & 0xFFFFFFFF
    a ^= a >> 4
    a = (a * 0x27D4EB2D) & 0xFFFFFFFF
    return a ^ (a >> 15)


def seq_dedup(T, s):
    for i in range(4):
        p = (s + i) % M
        if T[p] == s:
            return False
        if T[p] == 0:
            T[p] = s
            return True
    T[s % M] = s
    return True


ZERO_SLOTS = [M - 3, M - 2, M - 1, 0, 1, 2, 3]


def write_slots(s, ps, h):
    """Slots a pending lane marks: those it can write, now or after a re-run
    (h and its window's empty slots); its whole window when that holds slot 0;
    for sig == 0, every decision slot of a window that holds slot 0 (its
    forced overwrite makes slot 0 empty again)."""
    if s == 0:
        return list(ZERO_SLOTS)
    if h >= M - 3 or h == 0:  # the window holds slot 0: all of it
        ps = 15
    return [(h + k) % M for k in range(4) if ps >> k & 1]


def round_chunk(T, ch, binsh=3, seq_max=0, mark_all=False):
    """One chunk through the rounds; returns (emitted flags, rounds).  Once a
    round leaves at most seq_max lanes pending, they go to edge.hip's tail
    (SYZ_EDGE_SEQ): in passes, a pending signal whose window no earlier pending
    window overlaps runs dedup() on the table as it stands.  That is exact
    because every write lies in its writer's window, given the rounds'
    invariant that the pending lanes, run in order on the table as it stands,
    give the sequential outcome.  mark_all (SYZ_EDGE_MARKALL): every pending
    lane marks in the first pass, so one pass is the fixed point."""
    n, pend, emit, rounds = len(ch), list(range(len(ch))), [False] * len(ch), 0
    while pend:
        if rounds and len(pend) <= seq_max:
            while pend:
                go = [i for j, i in enumerate(pend)
                      if all((ch[i] - ch[k] + 3) % M > 6 for k in pend[:j])]
                for i in go:  # disjoint windows: any order
                    emit[i] = seq_dedup(T, ch[i])
                pend = [i for i in pend if i not in go]
            break
        rounds += 1
        ev = {}
        for i in pend:
            s = ch[i]
            h = s % M
            eqm = zm = 0
            for k in range(4):
                t = T[(h + k) % M]
                eqm |= (t == s) << k
                zm |= (t == 0) << k
            m = eqm | zm
            first = (m & -m).bit_length() - 1 if m else 4
            writer = first == 4 or not (eqm >> first) & 1
            ev[i] = (writer, (h + (first & 3)) % M, 1 | zm, h)
        stamp, once, twice, marked, blocked = {}, set(), set(), set(), {}

        def mark(i, slots):
            marked.add(i)
            for sl in slots:
                b = sl >> binsh
                stamp[b] = min(stamp.get(b, n), i)
                (twice if sl in once else once).add(sl)

        for i in pend:
            w, d, ps, h = ev[i]
            if w:
                mark(i, write_slots(ch[i], ps, h))
            elif mark_all:
                mark(i, write_slots(ch[i], ps, h) + [d])
        while True:
            new = []
            for i in pend:
                w, d, ps, h = ev[i]
                other = d in (twice if i in marked else once)
                blocked[i] = stamp.get(d >> binsh, n) < i and other
                if blocked[i] and i not in marked:
                    new.append(i)
            if not new:
                break
            for i in new:
                w, d, ps, h = ev[i]
                mark(i, write_slots(ch[i], ps, h) + [d])
        nxt = []
        for i in pend:
            if blocked[i]:
                nxt.append(i)
            elif ev[i][0]:
                T[ev[i][1]] = ch[i]
                emit[i] = True
        assert len(nxt) < len(pend)  # the earliest pending lane always finishes
        pend = nxt
    return emit, rounds


def _golden_names():
    return sorted(f[:-4] for f in os.listdir(HERE) if f.startswith("executor_") and f.endswith(".npz"))


SEQ_MAX = [0, 24, 256]  # rounds only; the kernel's tail; one round then sequential


@pytest.mark.parametrize("seq_max", SEQ_MAX)
@pytest.mark.parametrize("name", _golden_names())
def test_rounds_equal_sequential_dedup(name, seq_max):
    """Every program of every reference-executor fixture, chunk by chunk.
    A program aborted by cover_check is replayed over all its calls: the
    rounds are checked against sequential dedup, not against the abort."""
    d = np.load(os.path.join(HERE, name + ".npz"))
    pcs, cs, cl, pc = d["pcs"], d["call_start"], d["call_len"], d["prog_call"]
    for p in range(pc.size - 1):
        Tp, Ts = [0] * M, [0] * M
        for c in range(int(pc[p]), int(pc[p + 1])):
            trace = pcs[int(cs[c]): int(cs[c]) + int(cl[c])].tolist()
            prev, sigs = 0, []
            for x in trace:
                sigs.append((x & 0xFFFFFFFF) ^ prev)
                prev = exec_hash(x & 0xFFFFFFFF)
            for c0 in range(0, len(sigs), 256):
                ch = sigs[c0: c0 + 256]
                got, _ = round_chunk(Tp, ch, seq_max=seq_max)
                want = [seq_dedup(Ts, s) for s in ch]
                assert got == want, (name, p, c, c0)
                assert Tp == Ts


@pytest.mark.parametrize("seq_max", SEQ_MAX)
@pytest.mark.parametrize("global_walk,region_log2", [(1, 8), (0, 8), (0, 12)])
def test_rounds_equal_sequential_dedup_synthetic(global_walk, region_log2, seq_max):
    """The bench's trace distributions (SURVEY 8(d)'s global walk: the table
    thrashes, almost every signal a forced overwrite; region walks: mostly
    duplicates), 16 calls of 4096 PCs of one program."""
    from syzkaller_amd import synth

    cfg = synth.synth_default(global_walk=global_walk, region_log2=region_log2)
    pcs, cs, _ = synth.traces(cfg, 77, 1, 16, np.full(16, 4096, np.uint32))
    Tp, Ts = [0] * M, [0] * M
    for c in range(16):
        prev, sigs = 0, []
        for x in pcs[int(cs[c]): int(cs[c]) + 4096].tolist():
            sigs.append((x & 0xFFFFFFFF) ^ prev)
            prev = exec_hash(x & 0xFFFFFFFF)
        for c0 in range(0, len(sigs), 256):
            ch = sigs[c0: c0 + 256]
            got, _ = round_chunk(Tp, ch, seq_max=seq_max)
            assert got == [seq_dedup(Ts, s) for s in ch], (c, c0)
            assert Tp == Ts


def _zero_stress_chunk(rng, n):
    """A chunk dense in sig == 0 and in signals whose window holds slot 0 (or
    neighbours it), over a few values each, so that forced overwrites, zero
    writes and re-inserts meet inside one round."""
    homes = [M - 4, M - 3, M - 2, M - 1, 0, 1, 2, 3, 4]
    vals = [0] + [k * M + h for h in homes for k in range(1, 4)]
    p = np.full(len(vals), 1.0)
    p[0] = 6.0
    p /= p.sum()
    return [int(vals[j]) for j in rng.choice(len(vals), n, p=p)]


@pytest.mark.parametrize("seq_max", SEQ_MAX)
@pytest.mark.parametrize("seed", range(8))
def test_rounds_zero_writer_stress(seed, seq_max):
    """Randomized: chunks seeded with zero signals over a table whose slots
    8188..4 start full, empty or mixed; every chunk's flags and the table
    after it equal sequential dedup (executor.h:693-706)."""
    rng = np.random.default_rng(seed)
    for trial in range(40):
        T = [0] * M
        fill = trial % 3  # 0: full near slot 0, 1: empty, 2: mixed
        for sl in list(range(M - 6, M)) + list(range(0, 7)):
            if fill == 0 or (fill == 2 and rng.random() < 0.6):
                T[sl] = int(rng.integers(1, 5)) * M + sl
        Tp, Ts = list(T), list(T)
        for _ in range(3):
            ch = _zero_stress_chunk(rng, int(rng.integers(8, 257)))
            got, _ = round_chunk(Tp, ch, seq_max=seq_max)
            want = [seq_dedup(Ts, s) for s in ch]
            assert got == want, (seed, trial)
            assert Tp == Ts, (seed, trial)


@pytest.mark.parametrize("seq_max", [0, 16])
@pytest.mark.parametrize("name", _golden_names())
def test_rounds_mark_all_equal_sequential_dedup(name, seq_max):
    """The one-pass marking variant (SYZ_EDGE_MARKALL) on every fixture."""
    d = np.load(os.path.join(HERE, name + ".npz"))
    pcs, cs, cl, pc = d["pcs"], d["call_start"], d["call_len"], d["prog_call"]
    for p in range(pc.size - 1):
        Tp, Ts = [0] * M, [0] * M
        for c in range(int(pc[p]), int(pc[p + 1])):
            trace = pcs[int(cs[c]): int(cs[c]) + int(cl[c])].tolist()
            prev, sigs = 0, []
            for x in trace:
                sigs.append((x & 0xFFFFFFFF) ^ prev)
                prev = exec_hash(x & 0xFFFFFFFF)
            for c0 in range(0, len(sigs), 256):
                ch = sigs[c0: c0 + 256]
                got, _ = round_chunk(Tp, ch, seq_max=seq_max, mark_all=True)
                assert got == [seq_dedup(Ts, s) for s in ch], (name, p, c, c0)
                assert Tp == Ts


@pytest.mark.parametrize("seed", range(4))
def test_rounds_mark_all_zero_writer_stress(seed):
    rng = np.random.default_rng(100 + seed)
    for trial in range(40):
        T = [0] * M
        for sl in list(range(M - 6, M)) + list(range(0, 7)):
            if trial % 3 == 0 or (trial % 3 == 2 and rng.random() < 0.6):
                T[sl] = int(rng.integers(1, 5)) * M + sl
        Tp, Ts = list(T), list(T)
        for _ in range(3):
            ch = _zero_stress_chunk(rng, int(rng.integers(8, 257)))
            got, _ = round_chunk(Tp, ch, seq_max=16, mark_all=True)
            assert got == [seq_dedup(Ts, s) for s in ch], (seed, trial)
            assert Tp == Ts, (seed, trial)


def test_rounds_zero_writer_verdict_case():
    """The round-4 verdict's trace: after 8192, 8193, 16384, 8195 fill slots
    0..3, sig 0 is emitted and empties slot 0, so the following 16384 (then at
    slot 2) is a NEW insert at slot 0 -- 7 signals, as the reference executor
    emits (golden executor_zero2)."""
    sigs = [0x81000005, 8192, 8193, 16384, 8195, 0, 16384]
    Tp, Ts = [0] * M, [0] * M
    got, _ = round_chunk(Tp, sigs)
    assert got == [seq_dedup(Ts, s) for s in sigs] == [True] * 7
    assert Tp == Ts


def clear_race_trace(nprog, nchunks=16, seed=0):
    """Programs of one call whose 256-signal chunks alternate between a chunk
    that every lane finishes in its first round with nothing left pending
    (homes 32 apart: disjoint windows, no shared marks) and a chunk of
    colliding pairs (lanes 2j and 2j+1 share a home: the second is blocked).
    In edge.hip's mark-all mode the first kind leaves its round through the
    `!more` path, and the next chunk of the same prefetch group marks with no
    K1 barrier in front of it: the ADVICE round-5 race of the mark clear.
    Returns (pcs, call_start, call_len, prog_call) in the golden layout."""
    rng = np.random.default_rng(seed)
    n = nchunks * 256

    def vhash(a):  # exec_hash over a uint64 array of u32 values
        a = (a ^ 61) ^ (a >> 16)
        a = (a + (a << 3)) & 0xFFFFFFFF
        a ^= a >> 4
        a = (a * 0x27D4EB2D) & 0xFFFFFFFF
        return a ^ (a >> 15)

    pcs = np.zeros((nprog, n), np.uint64)
    prev = np.zeros(nprog, np.uint64)
    for q in range(nchunks):
        base = rng.integers(0, M, nprog).astype(np.uint64)
        for i in range(256):
            home = (base + 32 * (i if q % 2 == 0 else i // 2)) % M
            lo = np.zeros(nprog, np.uint64)
            todo = np.ones(nprog, bool)
            while todo.any():  # a signal with this home whose PC passes cover_check
                k = int(todo.sum())
                sig = (rng.integers(1, 1 << 19, k).astype(np.uint64) << 13) | home[todo]
                cand = sig ^ prev[todo]
                ok = (cand >= 0x80000000) & (cand < 0xFF000000)
                idx = np.flatnonzero(todo)[ok]
                lo[idx] = cand[ok]
                todo[idx] = False
            pcs[:, q * 256 + i] = np.uint64(0xFFFFFFFF00000000) | lo
            prev = vhash(lo)
    pcs = pcs.reshape(-1)
    cs = np.arange(nprog, dtype=np.uint64) * n
    cl = np.full(nprog, n, np.uint32)
    return pcs, cs, cl, np.arange(nprog + 1, dtype=np.uint32)


def test_clear_race_trace_shape():
    """The trace clear_race_trace builds does what its GPU test needs: in the
    mark-all mode, even chunks end after one round with no lane pending, odd
    chunks leave lanes pending; and the rounds still equal sequential dedup."""
    pcs, cs, cl, pc = clear_race_trace(2, nchunks=6, seed=3)
    for p in range(2):
        Tp, Ts = [0] * M, [0] * M
        trace = pcs[int(cs[p]): int(cs[p]) + int(cl[p])].tolist()
        prev, sigs = 0, []
        for x in trace:
            sigs.append((x & 0xFFFFFFFF) ^ prev)
            prev = exec_hash(x & 0xFFFFFFFF)
        for q, c0 in enumerate(range(0, len(sigs), 256)):
            ch = sigs[c0: c0 + 256]
            got, rounds = round_chunk(Tp, ch, seq_max=0, mark_all=True)
            assert got == [seq_dedup(Ts, s) for s in ch]
            assert (rounds == 1) == (q % 2 == 0), (p, q, rounds)
