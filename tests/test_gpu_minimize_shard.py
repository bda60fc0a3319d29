"""GPU: K5 Minimize (minimize.hip) vs the oracle, and the shard routing
(shard.hip + records-mode triage) vs unsharded triage on one GPU."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def corpus(rng, n, mean, universe, distinct_len=False):
    if distinct_len:
        lens = rng.permutation(np.arange(1, n * 3))[:n]
    else:
        lens = rng.geometric(1.0 / mean, size=n)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    elems = np.concatenate([rng.choice(universe, size=int(L), replace=False) for L in lens]).astype(np.uint32)
    prios = rng.integers(0, 4, size=elems.size).astype(np.int8)
    return off, elems, prios


@pytest.mark.parametrize("path", ["agg", "atomic"])
@pytest.mark.parametrize("seed,n,mean,U,distinct", [(0, 300, 50, 4000, True), (1, 2000, 200, 100000, False),
                                                     (2, 5000, 30, 500, False)])
def test_minimize_vs_oracle(gpu, seed, n, mean, U, distinct, path):
    """Both K5 paths: the aggregation path (default: entries partitioned by
    element, LDS winners per partition) and the per-entry atomicMax path."""
    from syzkaller_amd._lib import SYZSIG_DEBUG_MIN_ATOMIC

    rng = np.random.default_rng(seed)
    off, e, p = corpus(rng, n, mean, U, distinct)
    exp = O.minimize(off, e, p)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(gpu.dev)  # noqa: E731
    gpu.eng.set_debug(SYZSIG_DEBUG_MIN_ATOMIC if path == "atomic" else 0)
    try:
        keep, cnt = gpu.minimize(t(off, np.int64), t(e, np.int32), t(p, np.int8))
    finally:
        gpu.eng.set_debug(0)
    got = np.nonzero(keep.cpu().numpy())[0].tolist()
    assert got == exp and cnt == len(exp)


def test_minimize_many_prios_takes_atomic_path(gpu):
    """8 distinct prios (incl. negative ones) exceed the aggregation records'
    2 level bits: the atomic path runs, same result as the oracle."""
    rng = np.random.default_rng(11)
    off, e, _ = corpus(rng, 1500, 80, 30000)
    p = rng.integers(-4, 4, size=e.size).astype(np.int8)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(gpu.dev)  # noqa: E731
    keep, cnt = gpu.minimize(t(off, np.int64), t(e, np.int32), t(p, np.int8))
    assert np.nonzero(keep.cpu().numpy())[0].tolist() == O.minimize(off, e, p)


def test_minimize_negative_prios_agg_path(gpu):
    """4 prios spanning the sign (signed order -2 < -1 < 0 < 3) on the
    aggregation path."""
    rng = np.random.default_rng(12)
    off, e, _ = corpus(rng, 1500, 80, 30000)
    p = rng.choice(np.array([-2, -1, 0, 3], np.int8), size=e.size)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(gpu.dev)  # noqa: E731
    keep, cnt = gpu.minimize(t(off, np.int64), t(e, np.int32), t(p, np.int8))
    assert np.nonzero(keep.cpu().numpy())[0].tolist() == O.minimize(off, e, p)


def test_minimize_agg_partition_overflow(gpu):
    """8 fixed partitions for ~98k distinct elements: every partition overflows
    its LDS table and is aggregated in the HBM fallback table."""
    rng = np.random.default_rng(13)
    off, e, p = corpus(rng, 2000, 200, 100000)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(gpu.dev)  # noqa: E731
    gpu.eng.set_agg(1, 8)
    try:
        keep, cnt = gpu.minimize(t(off, np.int64), t(e, np.int32), t(p, np.int8))
    finally:
        gpu.eng.set_agg(1, 0)
    exp = O.minimize(off, e, p)
    assert np.nonzero(keep.cpu().numpy())[0].tolist() == exp and cnt == len(exp)


def test_minimize_host_api(gpu):
    from syzkaller_amd import signal as S

    rng = np.random.default_rng(4)
    off, e, p = corpus(rng, 500, 40, 3000)
    ctxs = [S.Context(S.Serial(e[off[i]:off[i + 1]], p[off[i]:off[i + 1]]).Deserialize(gpu.eng) if off[i + 1] > off[i]
                      else S.Signal.make(0, gpu.eng), i) for i in range(500)]
    got = sorted(S.Minimize(ctxs, gpu.eng))
    assert got == O.minimize(off, e, p)


@pytest.mark.parametrize("nshards", [2, 3, 8])
@pytest.mark.parametrize("bits", [False, True])
def test_step_routing_equals_unsharded(gpu, nshards, bits):
    """The sharded step's device API on one GPU (what dist.ShardedTriage
    drives, the all-to-alls replaced by tensor copies): G sources (program
    ranges of one batch) each send their staircase records into fixed buckets
    (syzsig_step_send_dev), the G owner shards triage what they receive
    (syzsig_step_own_dev), the flags come back (syzsig_step_back_dev); the
    sources' call flags, record bits (when asked for) and pairs, the union of
    the shards and of the newSignal shards equal plain triage of the whole
    batch against the unsharded maxSignal, and the pairs equal the oracle's."""
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth
    from tests.test_gpu_triage import dev_batch, oracle_pairs

    cfg = synth.synth_default(skew=1)
    nprog, cpp = 48, 32
    cl = synth.call_lengths(nprog, cpp, 0, ragged=(0, 3000), seed=nshards + 7)
    ds, dcs, dcnt, dprio = dev_batch(gpu, cfg, nprog, cpp, cl)
    m0e, m0p = synth.m0(cfg, 1024, 80000)
    ms = S.Serial(m0e, m0p).Deserialize(gpu.eng)
    ns = S.Signal(None, gpu.eng)
    ref_bits, cnew, _ = gpu.triage(ms, ns, ds, dcs, dcnt, dprio)
    owner = np.array([_owner(int(x), nshards) for x in m0e], np.uint32)
    shards = [S.Serial(m0e[owner == g], m0p[owner == g]).Deserialize(gpu.eng) for g in range(nshards)]
    news = [S.Signal.make(1 << 12, gpu.eng) for _ in range(nshards)]
    levels = sorted(set(int(x) for x in dprio.cpu().numpy().astype(np.int8)))
    ncalls = nprog * cpp
    bounds = [ncalls * s // nshards for s in range(nshards + 1)]
    cap = int(dcnt.to(torch.int64).sum()) + 64  # generous: no step is void
    W = cap + 1
    src = []
    for s in range(nshards):
        a, z = bounds[s], bounds[s + 1]
        # (room for the whole batch's pairs: the pairs counter keeps running
        # over the sources' step_back calls, see below)
        pairs = torch.full((int(dcnt.to(torch.int64).sum()) + 1,), -1, dtype=torch.int64, device=gpu.dev)
        b, sbits, scnew = gpu.batch(ds, dcs[a:z].contiguous(), dcnt[a:z].contiguous(), dprio[a:z].contiguous(),
                                    new_pairs=pairs, want_bits=bits)
        send = torch.empty(nshards * W, dtype=torch.int64, device=gpu.dev)
        gpu.step_send(b, a, levels, nshards, cap, send)
        st = gpu.step_finish()
        assert not st["global_void"] and not st["src_void"] and st["max_out"] <= cap, st
        src.append((b, sbits, scnew, pairs, send))
    flags = []
    for g in range(nshards):  # owner g's bucket s is source s's bucket g
        recv = torch.cat([x[4][g * W: (g + 1) * W] for x in src])
        f = torch.empty(nshards * W, dtype=torch.uint8, device=gpu.dev)
        gpu.step_own(shards[g], news[g], recv, nshards, cap, levels, f)
        ost = gpu.step_finish()
        assert not ost["global_void"] and not ost["owners_void"], ost
        flags.append(f)
    got_bits = torch.zeros_like(ref_bits)
    got_pairs, before = [], 0
    for s, (b, sbits, scnew, pairs, send) in enumerate(src):
        back = torch.cat([flags[g][s * W: (s + 1) * W] for g in range(nshards)])
        gpu.step_back(b, bounds[s], send, nshards, cap, back)
        bst = gpu.step_finish()
        assert not bst["global_void"] and not bst["owners_void"], bst
        assert torch.equal(scnew, cnew[bounds[s]: bounds[s + 1]])
        if bits:
            got_bits |= sbits
        # (one context plays every source: the pairs counter keeps running
        # over the step_back calls, so source s's pairs are [before, after))
        p = pairs[before: bst["new_pairs"]].cpu().numpy().view(np.uint64)
        got_pairs.append(p + (np.uint64(bounds[s]) << np.uint64(32)))
        before = bst["new_pairs"]
    torch.cuda.synchronize()
    if bits:
        assert torch.equal(got_bits, ref_bits)
    hs, hcs, hc = ds.cpu().numpy().view(np.uint32), dcs.cpu().numpy().view(np.uint64), dcnt.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(np.sort(np.concatenate(got_pairs)),
                                  oracle_pairs(hs, hcs, hc, ref_bits.cpu().numpy().view(np.uint32)))
    merged = {}
    for g in range(nshards):
        merged.update(shards[g].to_dict())
    assert merged == ms.to_dict()
    nmerged = {}
    for g in range(nshards):
        nmerged.update(news[g].to_dict() if not news[g].is_nil() else {})
    assert nmerged == ns.to_dict()


def _owner(e, n):
    """syz::owner_of (csrc/common.h) restated for the test."""
    def fmix(h):
        h ^= h >> 16
        h = (h * 0x85EBCA6B) & 0xFFFFFFFF
        h ^= h >> 13
        h = (h * 0xC2B2AE35) & 0xFFFFFFFF
        h ^= h >> 16
        return h
    h = fmix((e * 0x9E3779B1 + 0x7F4A7C15) & 0xFFFFFFFF)
    return (h * n) >> 32


@pytest.mark.parametrize("nshards", [2, 3, 8])
def test_minimize_sharded_by_element_equals_unsharded(gpu, nshards):
    """G element shards on one GPU (syzsig_minimize_shard_dev): the OR of
    their keep flags equals unsharded Minimize and the oracle."""
    rng = np.random.default_rng(40 + nshards)
    off, e, p = corpus(rng, 3000, 120, 20000)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(gpu.dev)  # noqa: E731
    doff, de, dp = t(off, np.int64), t(e, np.int32), t(p, np.int8)
    keep1, n1 = gpu.minimize(doff, de, dp)
    acc = torch.zeros_like(keep1)
    tot = 0
    for g in range(nshards):
        k, n = gpu.minimize_shard(doff, de, dp, nshards, g)
        acc = torch.maximum(acc, k)
        tot += n
    assert torch.equal(acc, keep1)
    assert tot >= n1
    assert np.nonzero(acc.cpu().numpy())[0].tolist() == O.minimize(off, e, p)


def _split_emulated(gpu, doff, de, dp, nparts, nshards, hint=0):
    """The data-split Minimize's exchange on one GPU: every part's winner
    records routed to their owners, each owner resolved, keep flags OR-ed."""
    sends = [gpu.minimize_split(doff, de, dp, nparts, k, nshards, hint) for k in range(nparts)]
    keep = None
    for g in range(nshards):
        recv = torch.cat([s[sum(c[:g]): sum(c[: g + 1])] for s, c in sends])
        k, _ = gpu.minimize_resolve(doff, recv)
        keep = k if keep is None else torch.maximum(keep, k)
    return keep, sends


@pytest.mark.parametrize("nparts,nshards", [(1, 1), (2, 2), (3, 5), (8, 8)])
def test_minimize_data_split_equals_unsharded(gpu, nparts, nshards):
    """syzsig_minimize_split_dev / _resolve_dev (each part reads only its range
    of the corpus) equal unsharded Minimize and the oracle."""
    rng = np.random.default_rng(70 + nparts)
    off, e, p = corpus(rng, 3000, 120, 20000)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(gpu.dev)  # noqa: E731
    doff, de, dp = t(off, np.int64), t(e, np.int32), t(p, np.int8)
    keep1, _ = gpu.minimize(doff, de, dp)
    keep, sends = _split_emulated(gpu, doff, de, dp, nparts, nshards)
    assert torch.equal(keep, keep1)
    assert np.nonzero(keep.cpu().numpy())[0].tolist() == O.minimize(off, e, p)
    # every part sends at most one record per distinct element of its range
    assert all(sum(c) <= np.unique(e).size for _, c in sends)


@pytest.mark.parametrize("case", ["many_prios", "forced_atomic"])
@pytest.mark.parametrize("nparts,nshards", [(2, 2), (3, 5)])
def test_minimize_data_split_atomic_fallback(gpu, case, nparts, nshards):
    """A part with more than 4 distinct prios (any int8 is a valid prio:
    signal.go:138-166) takes the split's per-entry atomicMax table instead of
    failing (which would have left its peers blocked in the all-to-all);
    forced_atomic runs that table on 0..3 prios.  Equal to the oracle."""
    from syzkaller_amd._lib import SYZSIG_DEBUG_MIN_ATOMIC

    rng = np.random.default_rng(90 + nparts)
    off, e, p = corpus(rng, 2000, 100, 20000)
    if case == "many_prios":
        p = rng.integers(-4, 4, size=e.size).astype(np.int8)
    t = lambda a, dt: torch.from_numpy(a.view(dt)).to(gpu.dev)  # noqa: E731
    doff, de, dp = t(off, np.int64), t(e, np.int32), t(p, np.int8)
    gpu.eng.set_debug(SYZSIG_DEBUG_MIN_ATOMIC if case == "forced_atomic" else 0)
    try:
        keep, sends = _split_emulated(gpu, doff, de, dp, nparts, nshards)
    finally:
        gpu.eng.set_debug(0)
    assert np.nonzero(keep.cpu().numpy())[0].tolist() == O.minimize(off, e, p)
    assert all(sum(c) <= np.unique(e).size for _, c in sends)


def test_minimize_data_split_c3_eight_parts(gpu):
    """BASELINE config 3 (200k contexts, ~400M entries) split over 8 parts and
    8 owners on one GPU (the N=8 exchange emulated) against unsharded Minimize
    and the oracle."""
    from tests.test_gpu_configs import _corpus_dev

    rng = np.random.default_rng(2018)
    n, U = 200_000, 1 << 22
    lens = np.minimum(rng.geometric(1.0 / 2000, size=n), U)
    doff, de, dp = _corpus_dev(gpu.dev, n, lens, U, seed=n)
    keep1, _ = gpu.minimize(doff, de, dp, hint_distinct=U)
    keep, _ = _split_emulated(gpu, doff, de, dp, 8, 8, hint=U)
    assert torch.equal(keep, keep1)
    exp = np.array(O.minimize(doff.cpu().numpy().view(np.uint64), de.cpu().numpy().view(np.uint32),
                              dp.cpu().numpy().view(np.int8)), np.int64)
    np.testing.assert_array_equal(np.nonzero(keep.cpu().numpy())[0], exp)
