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
d.  Unblocked writers store; blocked lanes run again next round."""
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


def round_chunk(T, ch, binsh=3):
    """One chunk through the rounds; returns (emitted flags, rounds)."""
    n, pend, emit, rounds = len(ch), list(range(len(ch))), [False] * len(ch), 0
    while pend:
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
                mark(i, [(h + k) % M for k in range(4) if ps >> k & 1])
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
                mark(i, [(h + k) % M for k in range(4) if ps >> k & 1] + [d])
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


@pytest.mark.parametrize("name,progs", [("executor_wide", (0, 5)), ("executor_synth", (1, 3)),
                                        ("executor_big", (0,))])
def test_rounds_equal_sequential_dedup(name, progs):
    d = np.load(os.path.join(HERE, name + ".npz"))
    pcs, cs, cl, pc = d["pcs"], d["call_start"], d["call_len"], d["prog_call"]
    for p in progs:
        Tp, Ts = [0] * M, [0] * M
        for c in range(int(pc[p]), int(pc[p + 1])):
            trace = pcs[int(cs[c]): int(cs[c]) + int(cl[c])].tolist()
            prev, sigs = 0, []
            for x in trace:
                sigs.append((x & 0xFFFFFFFF) ^ prev)
                prev = exec_hash(x & 0xFFFFFFFF)
            for c0 in range(0, len(sigs), 256):
                ch = sigs[c0: c0 + 256]
                got, _ = round_chunk(Tp, ch)
                want = [seq_dedup(Ts, s) for s in ch]
                assert got == want, (name, p, c, c0)
                assert Tp == Ts


@pytest.mark.parametrize("global_walk,region_log2", [(1, 8), (0, 8), (0, 12)])
def test_rounds_equal_sequential_dedup_synthetic(global_walk, region_log2):
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
            got, _ = round_chunk(Tp, ch)
            assert got == [seq_dedup(Ts, s) for s in ch], (c, c0)
            assert Tp == Ts
