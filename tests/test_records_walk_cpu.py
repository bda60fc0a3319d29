"""CPU: the records-mode algorithm of the owner side, restated with numpy,
against the oracle's sequential checkNewSignal (oracle/oracle.c
orc_triage_batch over the calls in serial order; syz-fuzzer/fuzzer.go:494-511,
pkg/signal/signal.go:90-131).

Round 4's kernels (csrc/recs.hip k_rp_agg / k_rp_elems / k_rp_flags) use the
closed form: with first[l] = the smallest serial among an element's records
at level l, record (s, l) is new iff prio(l) > M0[e], first[l] == s and
first[l'] > s for every l' > l; the final prio is max(M0[e], the top level
present).  `closed_form` restates that.  `sorted_walk` is round 3's
equivalent (sort by (element, serial), replay each run from M0[e]); both are
checked against the sequential loop.  tests/test_gpu_triage.py
test_records_mode_vs_oracle pins the kernels."""
import numpy as np
import pytest

from oracle import oracle as O


def sorted_walk(rec, m0, rng=None):
    """rec: u64 records (e << 32 | level << 24 | serial), level = prio here.
    Returns (flags per record, {e: final prio} of the changed elements).
    The runs are walked from their compacted heads (k_recs_heads), in a random
    order when rng is given: k_recs_heads compacts them in no particular
    order, and no run's replay depends on another's."""
    e = (rec >> np.uint64(32)).astype(np.uint64)
    serial = rec & np.uint64(0xFFFFFF)
    key = (e << np.uint64(24)) | serial
    order = np.argsort(key, kind="stable")
    es = e[order]
    heads = np.flatnonzero(np.r_[True, es[1:] != es[:-1]]) if rec.size else np.zeros(0, np.int64)
    if rng is not None:
        heads = rng.permutation(heads)
    flags = np.zeros(rec.size, np.uint8)
    changed = {}
    n = rec.size
    for i in heads.tolist():
        el = int(es[i])
        m0v = m0.get(el, -1000)
        m = m0v
        last_new = -1
        j = i
        while j < n and int(es[j]) == el:
            r = int(rec[order[j]])
            p = (r >> 24) & 0xFF
            k = r & 0xFFFFFF
            if p > m or k == last_new:
                flags[order[j]] = 1
                m = max(m, p)
                last_new = k
            j += 1
        if m > m0v:
            changed[el] = m
    return flags, changed


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_sorted_walk_equals_sequential_checknewsignal(seed):
    rng = np.random.default_rng(seed)
    pool = np.unique(rng.integers(0, 1 << 32, 3000, dtype=np.uint64).astype(np.uint32))
    ncall = 900
    clen = rng.integers(0, 9, ncall).astype(np.uint32)
    cs = np.zeros(ncall, np.uint64)
    cs[1:] = np.cumsum(clen[:-1].astype(np.uint64))
    nrec = int(clen.sum())
    # distinct elements inside a call (DiffRaw of a call's raw signal), repeats across calls
    sigs = np.concatenate([rng.choice(pool, int(c), replace=False) for c in clen]).astype(np.uint32)
    lvl = rng.integers(0, 4, ncall).astype(np.uint8)
    m0e = np.unique(rng.choice(pool, 800))
    m0p = rng.integers(0, 4, m0e.size).astype(np.int8)
    serial = np.repeat(np.arange(ncall, dtype=np.uint64), clen)
    rec = (sigs.astype(np.uint64) << np.uint64(32)) | (np.repeat(lvl, clen).astype(np.uint64) << np.uint64(24)) | serial
    perm = rng.permutation(nrec)  # the owner receives the records in no particular order
    flags, changed = sorted_walk(rec[perm], dict(zip(m0e.tolist(), m0p.tolist())), rng if seed else None)
    oms, ons, obits, _ = O.triage_batch(m0e, m0p, sigs, cs, clen, lvl)
    onew = np.unpackbits(obits.view(np.uint8), bitorder="little")[:nrec].astype(np.uint8)
    np.testing.assert_array_equal(flags, onew[perm])
    final = dict(zip(m0e.tolist(), m0p.tolist()))
    final.update(changed)
    assert final == oms.to_dict()
    assert changed == ons.to_dict()


def closed_form(rec, m0):
    """rec: u64 records (e << 32 | level << 24 | serial), level = prio here.
    The k_rp_* closed form, vectorised: no ordering of the records at all."""
    e = (rec >> np.uint64(32)).astype(np.int64)
    lv = ((rec >> np.uint64(24)) & np.uint64(0xFF)).astype(np.int64)
    ser = (rec & np.uint64(0xFFFFFF)).astype(np.int64)
    ue, inv = np.unique(e, return_inverse=True)
    none = np.int64(1 << 40)
    first = np.full((ue.size, 4), none, np.int64)
    np.minimum.at(first, (inv, lv), ser)  # k_rp_agg: ds_min per (element, level)
    m0v = np.array([m0.get(int(x), -1000) for x in ue], np.int64)  # k_rp_elems: one probe per element
    mine = first[inv, lv] == ser
    later = np.zeros(rec.size, bool)
    for l in range(4):
        later |= (l > lv) & (first[inv, l] <= ser)
    flags = ((lv > m0v[inv]) & mine & ~later).astype(np.uint8)  # k_rp_flags
    top = np.where(first < none, np.arange(4), -1).max(axis=1)
    fin = np.maximum(m0v, top)
    changed = {int(x): int(f) for x, f, m in zip(ue, fin, m0v) if f > m}
    return flags, changed


@pytest.mark.parametrize("seed,dups", [(0, False), (1, False), (2, True), (3, True)])
def test_closed_form_equals_sequential_checknewsignal(seed, dups):
    """dups: a call's raw signal repeats elements (DiffRaw collapses them: the
    copies of a new element are flagged together)."""
    rng = np.random.default_rng(seed)
    pool = np.unique(rng.integers(0, 1 << 32, 2000, dtype=np.uint64).astype(np.uint32))
    ncall = 1200
    clen = rng.integers(0, 12, ncall).astype(np.uint32)
    cs = np.zeros(ncall, np.uint64)
    cs[1:] = np.cumsum(clen[:-1].astype(np.uint64))
    nrec = int(clen.sum())
    sigs = np.concatenate([rng.choice(pool, int(c), replace=dups) for c in clen]).astype(np.uint32)
    lvl = rng.integers(0, 4, ncall).astype(np.uint8)
    m0e = np.unique(rng.choice(pool, 700))
    m0p = rng.integers(0, 4, m0e.size).astype(np.int8)
    serial = np.repeat(np.arange(ncall, dtype=np.uint64), clen)
    rec = (sigs.astype(np.uint64) << np.uint64(32)) | (np.repeat(lvl, clen).astype(np.uint64) << np.uint64(24)) | serial
    perm = rng.permutation(nrec)
    flags, changed = closed_form(rec[perm], dict(zip(m0e.tolist(), m0p.tolist())))
    oms, ons, obits, _ = O.triage_batch(m0e, m0p, sigs, cs, clen, lvl)
    onew = np.unpackbits(obits.view(np.uint8), bitorder="little")[:nrec].astype(np.uint8)
    np.testing.assert_array_equal(flags, onew[perm])
    final = dict(zip(m0e.tolist(), m0p.tolist()))
    final.update(changed)
    assert final == oms.to_dict()
    assert changed == ons.to_dict()
