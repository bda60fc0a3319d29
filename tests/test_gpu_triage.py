"""GPU: K3 batch triage (triage.hip) bit-exact against the sequential oracle
(checkNewSignal over every call of the batch in serial order), plus
size-independent properties at the BASELINE config-2 size."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _u(t, dt):
    return t.cpu().numpy().view(dt)


def host_batch(cfg, nprog, cpp, call_len, prog_base=0):
    """host traces -> oracle executor -> per-call raw signal (sparse layout)"""
    from syzkaller_amd import synth

    pcs, cs, prio = synth.traces(cfg, prog_base, nprog, cpp, call_len)
    sigs, cnt, comp = O.exec_batch(pcs, cs, call_len, synth.prog_call_index(nprog, cpp))
    return sigs, cs, cnt, prio


def dev_batch(gpu, cfg, nprog, cpp, call_len, prog_base=0):
    """device traces -> K1+K2 -> per-call raw signal, all resident in HBM"""
    from syzkaller_amd import synth

    cl = torch.from_numpy(np.ascontiguousarray(call_len).view(np.int32))
    pcs, cs, cl, prio = gpu.synth_traces(cfg, prog_base, nprog, cpp, cl)
    pidx = torch.from_numpy(synth.prog_call_index(nprog, cpp).view(np.int32)).to(gpu.dev)
    sigs, cnt, comp = gpu.edge_derive(pcs, cs, cl, pidx)
    del pcs
    return sigs, cs, cnt, prio


def oracle_pairs(hs, hcs, hcnt, obits):
    """Every call's DiffRaw result as sorted unique (call << 32 | elem)."""
    r = np.nonzero(np.unpackbits(obits.view(np.uint8), bitorder="little"))[0].astype(np.uint64)
    ends = hcs.astype(np.uint64) + hcnt.astype(np.uint64)
    call = np.searchsorted(ends, r, side="right").astype(np.uint64)
    return np.unique((call << np.uint64(32)) | hs[r].astype(np.uint64))


def compare(gpu, m0, hb, db, new0=None, ms_hint=None, agg=1, parts=0, reset=True, want_bits=True, pairs_cap=None):
    """agg: 0 = per-call path, 1 = auto, 2 = aggregation path (parts fixed if > 0).
    reset=False keeps the engine's path settings (and its adaptive state) as they are.
    want_bits=False: no per-record bits (what checkNewSignal returns; a large
    batch then takes the one-sync optimistic run); pairs_cap: the new_pairs
    buffer's size (default: one per record)."""
    from syzkaller_amd import signal as S

    hs, hcs, hcnt, hprio = hb
    ds, dcs, dcnt, dprio = db
    np.testing.assert_array_equal(_u(dcnt, np.uint32), hcnt)
    np.testing.assert_array_equal(_u(dprio, np.uint8), hprio)
    ms = S.Serial(*m0).Deserialize(gpu.eng) if m0[0].size else S.Signal.make(ms_hint or 0, gpu.eng)
    ns = S.Serial(*new0).Deserialize(gpu.eng) if new0 is not None else S.Signal(None, gpu.eng)
    pairs = torch.full((pairs_cap or int(hcnt.sum()) + 1,), -1, dtype=torch.int64, device=gpu.dev)
    if reset:
        gpu.eng.set_agg(agg, parts)
    try:
        bits, cnew, st = gpu.triage(ms, ns, ds, dcs, dcnt, dprio, new_pairs=pairs, want_bits=want_bits)
    finally:
        if reset:
            gpu.eng.set_agg(1, 0)
    oms, ons, obits, ocnew = O.triage_batch(m0[0], m0[1], hs, hcs, hcnt, hprio, new0)
    np.testing.assert_array_equal(_u(cnew, np.uint8), ocnew)
    if want_bits:
        np.testing.assert_array_equal(_u(bits, np.uint32), obits)
    op = oracle_pairs(hs, hcs, hcnt, obits)
    assert st["new_pairs"] == op.size
    np.testing.assert_array_equal(np.sort(_u(pairs[: op.size], np.uint64)), op)
    assert ms.Len() == oms.Len()
    assert ms.to_dict() == oms.to_dict()
    assert (ns.to_dict() if not ns.is_nil() else {}) == ons.to_dict()
    assert ns.is_nil() == ons.is_nil()
    return st


@pytest.mark.parametrize("agg", [0, 2])
@pytest.mark.parametrize("over,known,nm0", [({}, 2048, 200000), ({"skew": 1}, 1024, 100000),
                                             ({"region_log2": 11}, 4096, 300000), ({}, 0, 0)])
def test_triage_c1_vs_oracle(gpu, over, known, nm0, agg):
    """Config 1: 64 programs x 32 calls x 2k PCs, through K1+K2+K3, on the
    per-call path (agg=0) and the LDS aggregation path (agg=2)."""
    from syzkaller_amd import synth

    cfg = synth.synth_default(**over)
    nprog, cpp = 64, 32
    cl = synth.call_lengths(nprog, cpp, 2048)
    m0 = synth.m0(cfg, known, nm0)
    st = compare(gpu, m0, host_batch(cfg, nprog, cpp, cl), dev_batch(gpu, cfg, nprog, cpp, cl), agg=agg)
    assert st["candidates"] > 0 and st["runs"] == 1
    assert (st["parts"] > 0) == (agg == 2)


@pytest.mark.parametrize("want_bits,direct", [(True, False), (False, False), (False, True)])
@pytest.mark.parametrize("skew", [0, 1])
def test_triage_agg_auto_vs_oracle(gpu, skew, want_bits, direct):
    """A 5M-element maxSignal and a batch big enough (128 x 32 x 2k) to take
    the aggregation path by itself; without per-record bits it is the one-sync
    optimistic run, and with a new_pairs buffer of 4 entries per record its
    pairs are written there directly."""
    from syzkaller_amd import synth

    cfg = synth.synth_default(skew=skew)
    nprog, cpp = 128, 32
    cl = synth.call_lengths(nprog, cpp, 2048)
    m0 = synth.m0(cfg, 2048, 5_000_000)
    hb = host_batch(cfg, nprog, cpp, cl)
    st = compare(gpu, m0, hb, dev_batch(gpu, cfg, nprog, cpp, cl), want_bits=want_bits,
                 pairs_cap=4 * int(hb[2].sum()) + 64 if direct else None)
    assert st["parts"] >= 8 and st["overflow_parts"] == 0, st


@pytest.mark.parametrize("case", ["prio7", "prio_neg", "five_levels"])
def test_triage_optimistic_assumptions_fail(gpu, case):
    """The one-sync run assumes prios 0..3; a batch with another prio (a
    DiffRaw prio is any uint8, compared as int8: signal.go:90-102) voids it on
    device before anything is written, and the planned path (presence pass,
    level runs) must give the oracle's result."""
    from syzkaller_amd import synth

    cfg = synth.synth_default()
    nprog, cpp = 128, 32
    cl = synth.call_lengths(nprog, cpp, 2048)
    m0 = synth.m0(cfg, 2048, 2_000_000)
    hs, hcs, hcnt, hprio = host_batch(cfg, nprog, cpp, cl)
    hprio = hprio.copy()
    rng = np.random.default_rng(3)
    pick = rng.choice(hprio.size, 40, replace=False)
    hprio[pick] = {"prio7": 7, "prio_neg": 0xFF, "five_levels": 4}[case]
    if case == "five_levels":
        hprio[pick[:20]] = 0x80  # -128
    ds, dcs, dcnt, _ = dev_batch(gpu, cfg, nprog, cpp, cl)
    dprio = torch.from_numpy(hprio).to(gpu.dev)
    st = compare(gpu, m0, (hs, hcs, hcnt, hprio), (ds, dcs, dcnt, dprio), want_bits=False)
    assert st["records"] == int(hcnt.sum()) and st["runs"] >= 1


def test_triage_optimistic_bad_range_leaves_state(gpu):
    """A call range outside the record space, in a batch large enough for the
    optimistic run: EINVAL (triage.hip batch_total_records), and maxSignal,
    newSignal and the pairs are untouched."""
    from syzkaller_amd import _lib
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth

    cfg = synth.synth_default()
    nprog, cpp = 128, 32
    cl = synth.call_lengths(nprog, cpp, 2048)
    m0 = synth.m0(cfg, 2048, 1_000_000)
    ds, dcs, dcnt, dprio = dev_batch(gpu, cfg, nprog, cpp, cl)
    dcs = dcs.clone()
    dcs[77] = ds.numel() - 3  # runs past the end
    ms = S.Serial(*m0).Deserialize(gpu.eng)
    ns = S.Signal(None, gpu.eng)
    before = ms.to_dict()
    pairs = torch.full((1024,), -1, dtype=torch.int64, device=gpu.dev)
    with pytest.raises(_lib.SyzsigError):
        gpu.triage(ms, ns, ds, dcs, dcnt, dprio, new_pairs=pairs, want_bits=False)
    assert ms.to_dict() == before and ns.is_nil()
    assert bool((pairs == -1).all())


AGG_LIMIT = 7424 * 4 // 5  # csrc/agg.hip kAggLimit (kAggSlots * 4 / 5): distinct elements an LDS partition holds


@pytest.mark.parametrize("case", ["tight_tables", "nil_new_signal"])
def test_triage_finalize_deferred_path(gpu, case):
    """The finalize's slice-exclusive fast path and its deferred (atomic) path:
    with SYZSIG_DEBUG_FIN_DEFER every element whose probe sequence leaves its
    home bucket takes the deferred path; results must equal the oracle's.
    tight_tables: maxSignal and newSignal loaded close to their growth limit,
    so probe chains are long and slice ends are reached."""
    from syzkaller_amd import synth
    from syzkaller_amd._lib import SYZSIG_DEBUG_FIN_DEFER

    cfg = synth.synth_default()
    nprog, cpp = 128, 32
    cl = synth.call_lengths(nprog, cpp, 2048)
    m0 = synth.m0(cfg, 2048, 700_000 if case == "tight_tables" else 50_000)
    new0 = None
    if case == "tight_tables":
        e = np.unique(np.random.default_rng(5).integers(0, 1 << 32, 300_000, dtype=np.uint64).astype(np.uint32))
        new0 = (e, np.zeros(e.size, np.int8))
    for dbg in (0, SYZSIG_DEBUG_FIN_DEFER):
        gpu.eng.set_debug(dbg)
        try:
            st = compare(gpu, m0, host_batch(cfg, nprog, cpp, cl), dev_batch(gpu, cfg, nprog, cpp, cl), new0=new0,
                         agg=2)
        finally:
            gpu.eng.set_debug(0)
        assert st["parts"] >= 8 and st["overflow_parts"] == 0, st


@pytest.mark.parametrize("mode", ["capped", "capped_split", "counted", "spill", "idx64", "counted_idx64", "edge_passes",
                                  "hot"])
def test_triage_cell_layouts(gpu, mode):
    """Both record layouts of the aggregation path against the oracle: capped
    cells (default; capped_split: at 2048 partitions), counted cells (SYZSIG_DEBUG_EXACT_CELLS), capped cells that
    overflow and are redone counted (SYZSIG_DEBUG_CAP_SPILL), k_agg's 64-bit
    record indices (SYZSIG_DEBUG_AGG_IDX64: the path of runs past record 2^32,
    both layouts), K2's marking-mode flag left set (SYZSIG_DEBUG_EDGE_PASSES:
    its bit once reached the scatter as a timing-only "drop the records"
    switch), and a batch whose calls repeat one hot element hundreds of times, so that one cell of every
    chunk overflows its capacity: each batch is redone with counted cells and
    the slack doubles until capped cells are given up -- every batch exact."""
    from syzkaller_amd import synth
    from syzkaller_amd._lib import (SYZSIG_DEBUG_AGG_IDX64, SYZSIG_DEBUG_CAP_SPILL, SYZSIG_DEBUG_EDGE_PASSES,
                                    SYZSIG_DEBUG_EXACT_CELLS)

    if mode == "hot":
        rng = np.random.default_rng(21)
        pool = rng.integers(0, 1 << 32, 200_000, dtype=np.uint64).astype(np.uint32)
        ncalls, per = 2048, 600
        calls = [np.concatenate([rng.choice(pool, per - 300), np.full(300, 0x12345, np.uint32)]) for _ in range(ncalls)]
        calls = [rng.permutation(c) for c in calls]
        hs = np.concatenate(calls).astype(np.uint32)
        hcnt = np.full(ncalls, per, np.uint32)
        hcs = (np.arange(ncalls, dtype=np.uint64) * per).astype(np.uint64)
        hprio = rng.integers(0, 4, ncalls).astype(np.uint8)
        m0e = np.unique(rng.choice(pool, 20_000))
        m0 = (m0e, rng.integers(0, 4, m0e.size).astype(np.int8))
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu.dev)  # noqa: E731
        db = (t(hs, np.int32), t(hcs, np.int64), t(hcnt, np.int32), t(hprio, np.uint8))
        retries = []
        gpu.eng.set_agg(2, 128)  # resets the capped-cell slack too
        for _ in range(4):  # sd 6 -> 12 -> 24 -> counted cells only
            st = compare(gpu, m0, (hs, hcs, hcnt, hprio), db, agg=2, reset=False)
            retries.append(st["retries"])
        gpu.eng.set_agg(1, 0)
        assert retries[0] == 1 and retries[-1] == 0, retries
        return
    cfg = synth.synth_default(skew=1)
    nprog, cpp = 128, 32
    cl = synth.call_lengths(nprog, cpp, 2048)
    m0 = synth.m0(cfg, 2048, 1_000_000)
    dbg = {"counted": SYZSIG_DEBUG_EXACT_CELLS, "spill": SYZSIG_DEBUG_CAP_SPILL, "idx64": SYZSIG_DEBUG_AGG_IDX64,
           "counted_idx64": SYZSIG_DEBUG_EXACT_CELLS | SYZSIG_DEBUG_AGG_IDX64,
           "edge_passes": SYZSIG_DEBUG_EDGE_PASSES}.get(mode, 0)
    # capped_split: 2048 partitions (the LDS write-combining buffers at their largest)
    parts = 2048 if mode == "capped_split" else 0
    gpu.eng.set_debug(dbg)
    try:
        st = compare(gpu, m0, host_batch(cfg, nprog, cpp, cl), dev_batch(gpu, cfg, nprog, cpp, cl), agg=2,
                     parts=parts)
    finally:
        gpu.eng.set_debug(0)
    assert st["parts"] >= 8 and st["overflow_parts"] == 0, st
    assert st["retries"] == (1 if mode == "spill" else 0), st


def fmix32_inv_np(h):
    """Inverse of murmur3 fmix32 (csrc/agg.hip fmix32_inv), on a u32 array."""
    h = np.asarray(h, np.uint32).copy()
    h ^= h >> np.uint32(16)
    h *= np.uint32(0x7ED1B41D)
    h ^= (h >> np.uint32(13)) ^ (h >> np.uint32(26))
    h *= np.uint32(0xA5CB9243)
    h ^= h >> np.uint32(16)
    return h


@pytest.mark.parametrize("over", [(0,) * 8, (1, 0, 0, 1, 0, 1, 1, 0), (1,) * 8])
def test_triage_agg_lds_overflow_fallback(gpu, over):
    """8 partitions (the top 3 bits of h = fmix32(e)); partition p gets
    kAggLimit + 300 distinct elements when over[p] (it overflows the LDS table
    and is redone in the HBM table) or kAggLimit - 300.  h = 0 and
    h = 0xFFFFFFFF (the HBM table's extra slot) are among the elements."""
    rng = np.random.default_rng(sum(over) + 11)
    pools = []
    for p, o in enumerate(over):
        n = AGG_LIMIT + 300 if o else AGG_LIMIT - 300
        low = rng.choice(1 << 29, size=n, replace=False).astype(np.uint32)
        pools.append((np.uint32(p) << np.uint32(29)) | low)
    pools[0][0] = 0
    pools[7][0] = 0xFFFFFFFF
    h = np.concatenate(pools)
    assert np.unique(h).size == h.size
    elems = fmix32_inv_np(h)
    # calls: every element once in a shuffled pass, then random repeats
    ncalls = 600
    stream = np.concatenate([rng.permutation(elems), rng.choice(elems, size=elems.size * 2)])
    cuts = np.sort(rng.choice(np.arange(1, stream.size), size=ncalls - 1, replace=False))
    hcs = np.concatenate([[0], cuts]).astype(np.uint64)
    hcnt = np.diff(np.concatenate([hcs, [stream.size]])).astype(np.uint32)
    hprio = rng.integers(0, 4, size=ncalls).astype(np.uint8)
    hs = stream.astype(np.uint32)
    m0e = np.concatenate([rng.choice(elems, size=5000, replace=False), rng.integers(0, 1 << 32, 3000, np.uint64)])
    m0e = np.unique(m0e.astype(np.uint32))
    m0p = rng.integers(0, 4, size=m0e.size).astype(np.int8)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu.dev)  # noqa: E731
    db = (t(hs, np.int32), t(hcs, np.int64), t(hcnt, np.int32), t(hprio, np.uint8))
    st = compare(gpu, (m0e, m0p), (hs, hcs, hcnt, hprio), db, agg=2, parts=8)
    assert st["parts"] == 8 and st["distinct"] == elems.size
    assert st["overflow_parts"] == sum(over), st


@pytest.mark.parametrize("big", [AGG_LIMIT + 300, 9 * AGG_LIMIT])
def test_triage_one_sync_direct_pairs_lds_overflow(gpu, big):
    """The one-sync run (want_bits=False) writing its pairs straight into the
    caller's new_pairs (capacity 4 x 8 partitions x kAggLimit, the least that
    path accepts) while one of its 8 partitions overflows the LDS table and is
    committed from the HBM table after the sync: the pairs already written must
    survive.  With 9 x kAggLimit elements in that partition the run's pairs no
    longer all fit the caller's buffer, so they move to the workspace first."""
    rng = np.random.default_rng(big)
    per_part = 2 * big  # records of every partition alike, so that no capped cell spills
    parts = []
    for p in range(8):
        n = big if p == 2 else 400
        low = rng.choice(1 << 29, size=n, replace=False).astype(np.uint32)
        e = fmix32_inv_np((np.uint32(p) << np.uint32(29)) | low)
        parts.append(np.concatenate([e, rng.choice(e, size=per_part - n)]))
    elems = np.concatenate(parts)
    ncalls = 500
    stream = rng.permutation(elems)
    cuts = np.sort(rng.choice(np.arange(1, stream.size), size=ncalls - 1, replace=False))
    hcs = np.concatenate([[0], cuts]).astype(np.uint64)
    hcnt = np.diff(np.concatenate([hcs, [stream.size]])).astype(np.uint32)
    hprio = rng.integers(0, 4, size=ncalls).astype(np.uint8)
    hs = stream.astype(np.uint32)
    m0e = np.unique(rng.choice(np.unique(elems), size=2000, replace=False))
    m0p = rng.integers(0, 4, size=m0e.size).astype(np.int8)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu.dev)  # noqa: E731
    db = (t(hs, np.int32), t(hcs, np.int64), t(hcnt, np.int32), t(hprio, np.uint8))
    st = compare(gpu, (m0e, m0p), (hs, hcs, hcnt, hprio), db, agg=2, parts=8, want_bits=False,
                 pairs_cap=4 * 8 * AGG_LIMIT)
    assert st["parts"] == 8 and st["overflow_parts"] == 1 and st["retries"] == 0, st


@pytest.mark.parametrize("agg", [0, 2])
def test_triage_overflow_retry(gpu, agg):
    """maxSignal starts as make(Signal) with 16 slots: the per-call path
    overflows and restarts on bigger tables, the aggregation path reserves from
    its distinct count; results must not change."""
    from syzkaller_amd import synth

    cfg = synth.synth_default()
    cl = synth.call_lengths(32, 16, 0, ragged=(0, 3000), seed=3)
    m0 = (np.empty(0, np.uint32), np.empty(0, np.int8))
    st = compare(gpu, m0, host_batch(cfg, 32, 16, cl), dev_batch(gpu, cfg, 32, 16, cl), ms_hint=0, agg=agg)
    assert st["retries"] > 0 or agg == 2


@pytest.mark.parametrize("agg", [0, 2])
def test_triage_many_prios_and_existing_new_signal(gpu, agg):
    """Arbitrary uint8 prios (int8 order, > 4 distinct -> several runs) and a
    non-empty newSignal before the batch."""
    from syzkaller_amd import synth

    cfg = synth.synth_default(region_log2=10)
    nprog, cpp = 16, 16
    cl = synth.call_lengths(nprog, cpp, 0, ragged=(0, 2500), seed=8)
    hs, hcs, hcnt, _ = host_batch(cfg, nprog, cpp, cl)
    ds, dcs, dcnt, _ = dev_batch(gpu, cfg, nprog, cpp, cl)
    rng = np.random.default_rng(1)
    prio = rng.choice(np.array([0, 1, 2, 3, 7, 127, 128, 200, 255], np.uint8), size=nprog * cpp)
    m0 = synth.m0(cfg, 512, 50000)
    new0 = synth.m0(cfg, 0, 1000)
    st = compare(gpu, m0, (hs, hcs, hcnt, prio), (ds, dcs, dcnt, torch.from_numpy(prio).to(gpu.dev)), new0=new0,
                 agg=agg)
    assert st["runs"] > 1


@pytest.mark.parametrize("agg", [0, 2])
def test_triage_empty_and_degenerate(gpu, agg):
    from syzkaller_amd import signal as S

    gpu.eng.set_agg(agg, 0)
    ms = S.Signal.make(0, gpu.eng)
    ns = S.Signal(None, gpu.eng)
    z = lambda n, dt: torch.zeros(n, dtype=dt, device=gpu.dev)  # noqa: E731
    bits, cnew, st = gpu.triage(ms, ns, z(0, torch.int32), z(0, torch.int64), z(0, torch.int32), z(0, torch.uint8))
    assert ns.is_nil() and ms.Len() == 0
    # calls that are all empty
    bits, cnew, st = gpu.triage(ms, ns, z(4, torch.int32), z(3, torch.int64), z(3, torch.int32), z(3, torch.uint8))
    assert int(cnew.sum()) == 0 and ns.is_nil()
    # only element 0xFFFFFFFF (the LDS table's special slot) and element 0
    sigs = torch.tensor([-1, 0, -1, 0, 5], dtype=torch.int32, device=gpu.dev)
    cs = torch.tensor([0, 2, 4], dtype=torch.int64, device=gpu.dev)
    cl = torch.tensor([2, 2, 1], dtype=torch.int32, device=gpu.dev)
    pr = torch.tensor([1, 3, 2], dtype=torch.uint8, device=gpu.dev)
    pairs = torch.zeros(8, dtype=torch.int64, device=gpu.dev)
    bits, cnew, st = gpu.triage(ms, ns, sigs, cs, cl, pr, new_pairs=pairs)
    gpu.eng.set_agg(1, 0)
    assert cnew.tolist() == [1, 1, 1] and int(bits[0]) == 0b11111 and st["new_pairs"] == 5
    got = sorted(int(v) & ((1 << 64) - 1) for v in pairs[:5].tolist())
    assert got == sorted([0xFFFFFFFF, 0, (1 << 32) | 0xFFFFFFFF, 1 << 32, (2 << 32) | 5])
    assert ms.to_dict() == {0xFFFFFFFF: 3, 0: 3, 5: 2} and ns.to_dict() == ms.to_dict()


def test_triage_rejects_out_of_range_calls(gpu):
    from syzkaller_amd import signal as S
    from syzkaller_amd._lib import SyzsigError

    ms = S.Signal.make(0, gpu.eng)
    ns = S.Signal(None, gpu.eng)
    sigs = torch.arange(100, dtype=torch.int32, device=gpu.dev)
    cs = torch.tensor([0, 90], dtype=torch.int64, device=gpu.dev)
    cl = torch.tensor([10, 20], dtype=torch.int32, device=gpu.dev)
    with pytest.raises(SyzsigError):
        gpu.triage(ms, ns, sigs, cs, cl, torch.zeros(2, dtype=torch.uint8, device=gpu.dev))


def test_triage_c2_properties(gpu):
    """Config 2 size (4096 programs x 64 calls x 4k PCs vs a 10M maxSignal):
    the whole batch in one launch equals the same batch as two sequential halves
    (bit-exact bits, flags, maxSignal); replaying the batch finds nothing new;
    every changed element is in newSignal."""
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth

    cfg = synth.synth_default()
    nprog, cpp = 4096, 64
    cl = synth.call_lengths(nprog, cpp, 4096)
    ds, dcs, dcnt, dprio = dev_batch(gpu, cfg, nprog, cpp, cl)
    e0, p0 = gpu.synth_m0(cfg, 2048, 10_000_000)
    ms = gpu.deserialize(e0, p0)
    ms2 = ms.clone()
    ns = S.Signal(None, gpu.eng)
    pairs = torch.empty(16 << 20, dtype=torch.int64, device=gpu.dev)
    bits, cnew, st = gpu.triage(ms, ns, ds, dcs, dcnt, dprio, new_pairs=pairs)
    assert st["changed"] == ns.Len() and st["records"] == int(dcnt.to(torch.int64).sum()) and st["parts"] > 0
    assert st["overflow_parts"] == 0 and st["new_pairs"] <= pairs.numel()
    # pairs <-> bits: one pair per distinct (call, elem) among the marked records
    npair = st["new_pairs"]
    assert npair == int(torch.unique(pairs[:npair]).numel())
    assert int(cnew.sum()) == int(torch.unique(pairs[:npair] >> 32).numel())
    h = nprog * cpp // 2
    ns2 = S.Signal(None, gpu.eng)
    b1, c1, _ = gpu.triage(ms2, ns2, ds, dcs[:h].contiguous(), dcnt[:h].contiguous(), dprio[:h].contiguous())
    b2, c2, _ = gpu.triage(ms2, ns2, ds, dcs[h:].contiguous(), dcnt[h:].contiguous(), dprio[h:].contiguous())
    assert torch.equal(cnew, torch.cat([c1, c2]))
    assert torch.equal(bits, b1 | b2)
    assert ms.Len() == ms2.Len() and ns.Len() == ns2.Len()
    ser, ser2 = ms.Serialize(), ms2.Serialize()
    o, o2 = np.argsort(ser.Elems), np.argsort(ser2.Elems)
    np.testing.assert_array_equal(ser.Elems[o], ser2.Elems[o2])
    np.testing.assert_array_equal(ser.Prios[o], ser2.Prios[o2])
    # replay: nothing is new any more, maxSignal unchanged
    ns3 = S.Signal(None, gpu.eng)
    n_before = ms.Len()
    bits3, cnew3, st3 = gpu.triage(ms, ns3, ds, dcs, dcnt, dprio)
    assert int(cnew3.sum()) == 0 and int(bits3.count_nonzero()) == 0 and ns3.is_nil() and ms.Len() == n_before


@pytest.mark.parametrize("agg,npool", [(1, 2_500_000), (0, 2_500_000), (1, 200_000), (1, 20_000), (1, 200)])
def test_records_mode_vs_oracle(gpu, agg, npool):
    """Records mode (the owner side of a sharded step, triage.hip
    triage_records_impl): ~1.2M records (e, level, serial) in a shuffled order,
    each serial one call of up to 6 distinct elements at one level, against a
    shard holding part of the pool.  agg=1 takes the LDS-partitioned path
    (recs.hip: records grouped by element hash, each partition sorted by
    (element, serial) in LDS, one thread per element run), agg=0 the per-record
    probe path.  npool=200k gives ~6 records per element, 20k ~60; npool=200
    puts ~6000 records on each element, so partitions overflow the LDS
    capacity and the run falls back to the per-record path before committing.
    All must flag exactly the records the oracle's sequential checkNewSignal
    over the calls in serial order marks new, and leave the same shard and
    newSignal."""
    from syzkaller_amd import signal as S

    rng = np.random.default_rng(77)
    pool = np.unique(rng.integers(0, 1 << 32, npool, dtype=np.uint64).astype(np.uint32))
    assert all((7919 * k) % pool.size for k in range(1, 7))  # a call's elements are distinct
    ncall = 300_000
    clen = rng.integers(1, 7, ncall).astype(np.uint32)
    nrec = int(clen.sum())
    assert nrec >= 1 << 20
    cs = np.zeros(ncall, np.uint64)
    cs[1:] = np.cumsum(clen[:-1].astype(np.uint64))
    # distinct elements inside a call: consecutive picks of a random walk through the pool
    start = rng.integers(0, pool.size, ncall)
    idx = (np.repeat(start, clen) + (np.arange(nrec) - np.repeat(cs.astype(np.int64), clen)) * 7919) % pool.size
    sigs = pool[idx]
    lvl = rng.integers(0, 4, ncall).astype(np.uint8)
    serial = np.repeat(np.arange(ncall, dtype=np.uint64), clen)
    rec = (sigs.astype(np.uint64) << np.uint64(32)) | (np.repeat(lvl, clen).astype(np.uint64) << np.uint64(24)) | serial
    perm = rng.permutation(nrec)
    m0e = np.unique(rng.choice(pool, 1_000_000))
    m0p = rng.integers(0, 4, m0e.size).astype(np.int8)
    ms = S.Serial(m0e, m0p).Deserialize(gpu.eng)
    ns = S.Signal(None, gpu.eng)
    drec = torch.from_numpy(rec[perm].view(np.int64)).to(gpu.dev)
    flags = torch.zeros(nrec, dtype=torch.uint8, device=gpu.dev)
    gpu.eng.set_agg(0 if agg == 0 else 1, 0)
    try:
        st = gpu.triage_records(ms, ns, drec, [0, 1, 2, 3], flags)
    finally:
        gpu.eng.set_agg(1, 0)
    oms, ons, obits, _ = O.triage_batch(m0e, m0p, sigs, cs, clen, lvl)
    onew = np.unpackbits(obits.view(np.uint8), bitorder="little")[:nrec].astype(np.uint8)
    np.testing.assert_array_equal(_u(flags, np.uint8), onew[perm])
    assert ms.to_dict() == oms.to_dict()
    assert ns.to_dict() == ons.to_dict()
    assert (st["parts"] > 0) == (agg != 0 and npool > 1000), st  # the LDS path reports its partitions


def test_restore_keys_brings_back_the_snapshot(gpu):
    """syzsig_set_restore_keys: after a batch on the one-sync aggregation path
    and one in records mode, copying back only newSignal's slots from the
    snapshot gives the snapshot exactly (slot for slot); a table that grew
    since is refused."""
    from syzkaller_amd import _lib
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth

    cfg = synth.synth_default()
    nprog, cpp = 128, 32
    cl = synth.call_lengths(nprog, cpp, 2048)
    m0e, m0p = synth.m0(cfg, 2048, 1_000_000)
    ms = S.Signal.make(16_000_000, gpu.eng)  # room for the batches' growth: no rehash after the snapshot
    ms.Merge(S.Serial(m0e, m0p).Deserialize(gpu.eng))
    snap = ms.clone()
    ds, dcs, dcnt, dprio = dev_batch(gpu, cfg, nprog, cpp, cl)
    ns = S.Signal.make(100_000, gpu.eng)
    for _ in range(2):
        gpu.triage(ms, ns, ds, dcs, dcnt, dprio, want_bits=False)
        assert ns.Len() > 0 and not ms.equal(snap)
        ms.restore_keys(snap, ns)
        assert ms.equal(snap)
        ns.clear()
    # records mode (the owner side), >= 2^20 records: the sorted path
    rng = np.random.default_rng(5)
    e = rng.choice(np.unique(np.concatenate([m0e, rng.integers(0, 1 << 32, 600_000, dtype=np.uint64).astype(np.uint32)])),
                   1_200_000)
    rec = (e.astype(np.uint64) << np.uint64(32)) | (rng.integers(0, 4, e.size).astype(np.uint64) << np.uint64(24)) | \
        rng.integers(0, 1 << 20, e.size).astype(np.uint64)
    flags = torch.zeros(e.size, dtype=torch.uint8, device=gpu.dev)
    gpu.triage_records(ms, ns, torch.from_numpy(rec.view(np.int64)).to(gpu.dev), [0, 1, 2, 3], flags)
    assert ns.Len() > 0
    ms.restore_keys(snap, ns)
    assert ms.equal(snap)
    big = S.Signal.make(100_000_000, gpu.eng)  # (a different capacity)
    with pytest.raises(_lib.SyzsigError):
        big.restore_keys(snap, ns)


def test_one_sync_run_geometry_miss_redo(gpu):
    """The one-sync run sizes its partitions from the distinct/records ratio of
    the previous large batch.  After a batch of a few hot elements (ratio ~0),
    a batch of all-distinct elements overflows most LDS partitions: the run
    must commit nothing, redo itself once with partitions for what it counted,
    and give the oracle's result."""
    from syzkaller_amd import signal as S

    rng = np.random.default_rng(9)
    ncalls, per = 1024, 1100
    hot = rng.integers(0, 1 << 32, 64, dtype=np.uint64).astype(np.uint32)
    cs = (np.arange(ncalls, dtype=np.uint64) * per).astype(np.uint64)
    cnt = np.full(ncalls, per, np.uint32)
    prio = rng.integers(0, 4, ncalls).astype(np.uint8)
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu.dev)  # noqa: E731
    for kind in ("hot", "distinct"):
        if kind == "hot":
            sigs = rng.choice(hot, ncalls * per)
        else:
            sigs = np.unique(rng.integers(0, 1 << 32, ncalls * per * 2, dtype=np.uint64).astype(np.uint32))
            sigs = rng.permutation(sigs)[: ncalls * per]
        m0e = np.unique(rng.integers(0, 1 << 32, 50_000, dtype=np.uint64).astype(np.uint32))
        m0p = rng.integers(0, 4, m0e.size).astype(np.int8)
        st = compare(gpu, (m0e, m0p), (sigs, cs, cnt, prio),
                     (t(sigs, np.int32), t(cs, np.int64), t(cnt, np.int32), t(prio, np.uint8)), want_bits=False,
                     reset=False)
        if kind == "distinct":
            assert st["retries"] >= 1 and st["overflow_parts"] == 0, st
