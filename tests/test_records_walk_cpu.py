"""CPU: the records-mode algorithm of the owner side (csrc/triage.hip
k_recs_keys / radix sort / k_recs_heads / k_recs_walk), restated with numpy, against the
oracle's sequential checkNewSignal (oracle/oracle.c orc_triage_batch over the
calls in serial order; syz-fuzzer/fuzzer.go:494-511, pkg/signal/signal.go:90-131).

Sorting the records by (element, serial) makes each element's records one run
in serial order; replaying the run from M0[e] -- a record is new iff its prio
exceeds the running maximum, or it repeats a new record's serial -- gives
exactly the per-record new flags and the final maxSignal of the sequential
loop.  This pins the design on CPU; tests/test_gpu_triage.py
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
