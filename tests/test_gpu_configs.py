"""GPU: BASELINE.json's configs at their full sizes, checked against the oracle.

  C2  the whole 4096 x 64 x 4096 batch vs a 10M-element maxSignal on the
      aggregation path the bench runs (2048 partitions), against sequential
      checkNewSignal (oracle/oracle.c orc_triage_batch) over the same records.
  C3  signal.Minimize over a 200k-context corpus (geometric lengths, mean 2k,
      ~400M entries), against orc_minimize; plus a distinct-length corpus where
      the reference's unstable sort.Slice order cannot matter.
  C4  a 1B-element maxSignal: hash-sharded into 8 shard tables on one GPU, one
      C2 batch (the global walk's 1.07e9 records) split into 8 source program
      ranges routed through the stream-ordered step API (syzsig_step_*) that
      `bench.py --gpus 8` runs, against the same batch on the unsharded 1B
      table; plus the oracle on a program prefix (M0 restricted to the
      prefix's keys).
  C5  streaming, skewed: two consecutive batches of 8192 programs x 64 x 1k
      (one rank's share of 64k programs per batch on 8 GPUs; SURVEY 8(d)'s
      global walks from Zipf(1.1) entries, and rounds 1-4's power-skewed
      region walks) triaged against the state the previous batch left,
      against the oracle over both batches in order.

References: syz-fuzzer/fuzzer.go:494-511 (checkNewSignal), pkg/signal/signal.go
:73-166 (Diff/DiffRaw/Merge/Minimize).
"""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _u(t, dt):
    return t.cpu().numpy().view(dt)


def _sorted_ser(elems, prios):
    o = np.argsort(elems, kind="stable")
    return elems[o], prios[o]


def assert_same_set(dev_set, osig):
    """Device Signal == oracle Signal, compared as sorted (elem, prio) arrays."""
    ge, gp = _sorted_ser(*(lambda s: (s.Elems, s.Prios))(dev_set.Serialize()))
    oe, op = _sorted_ser(*osig.Serialize())
    np.testing.assert_array_equal(ge, oe)
    np.testing.assert_array_equal(gp, op)


def pairs_from_bits(sigs, cs, cnt, bits):
    """Every call's DiffRaw result as sorted unique (call << 32 | elem) from
    per-record new bits (sparse record layout)."""
    r = np.nonzero(np.unpackbits(bits.view(np.uint8), bitorder="little"))[0].astype(np.uint64)
    ends = cs.astype(np.uint64) + cnt.astype(np.uint64)
    call = np.searchsorted(ends, r, side="right").astype(np.uint64)
    return np.unique((call << np.uint64(32)) | sigs[r].astype(np.uint64))


def device_batch(gpu, cfg, prog_base, nprog, cpp, pcs_per_call):
    """synthetic traces -> K1+K2 on device; returns (sigs, call_start, sig_cnt, prio)."""
    from syzkaller_amd import synth

    cl = torch.full((nprog * cpp,), pcs_per_call, dtype=torch.int32)
    pcs, cs, cl, prio = gpu.synth_traces(cfg, prog_base, nprog, cpp, cl)
    pidx = torch.from_numpy(synth.prog_call_index(nprog, cpp).view(np.int32)).to(gpu.dev)
    sigs, cnt, comp = gpu.edge_derive(pcs, cs, cl, pidx)
    del pcs
    return sigs, cs, cnt, prio


def test_c2_full_batch_vs_oracle(gpu):
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth

    cfg = synth.synth_default()
    P, C, L = 4096, 64, 4096
    sigs, cs, cnt, prio = device_batch(gpu, cfg, 0, P, C, L)
    m0e, m0p = gpu.synth_m0(cfg, 2048, 10_000_000)
    ms = gpu.deserialize(m0e, m0p)
    ns = S.Signal(None, gpu.eng)
    nrec = int(cnt.to(torch.int64).sum())
    pairs = torch.full((16 << 20,), -1, dtype=torch.int64, device=gpu.dev)
    _, cnew, st = gpu.triage(ms, ns, sigs, cs, cnt, prio, new_pairs=pairs, want_bits=False)
    torch.cuda.synchronize()
    # the geometry the bench reports: one run on the aggregation path, 2048 partitions, no overflow
    assert st["records"] == nrec and st["runs"] == 1
    assert st["parts"] == 2048 and st["overflow_parts"] == 0
    hs, hcs, hcnt, hprio = _u(sigs, np.uint32), _u(cs, np.uint64), _u(cnt, np.uint32), _u(prio, np.uint8)
    oms, ons, obits, ocnew = O.triage_batch(_u(m0e, np.uint32), _u(m0p, np.int8), hs, hcs, hcnt, hprio)
    np.testing.assert_array_equal(_u(cnew, np.uint8), ocnew)
    op = pairs_from_bits(hs, hcs, hcnt, obits)
    assert st["new_pairs"] == op.size <= pairs.numel()
    np.testing.assert_array_equal(np.sort(_u(pairs[: op.size], np.uint64)), op)
    assert ms.Len() == oms.Len() and ns.Len() == ons.Len()
    assert_same_set(ms, oms)
    assert_same_set(ns, ons)


def _corpus_dev(dev, n, lens, U, seed):
    """Minimize corpus on device: context c has lens[c] distinct elements
    (base_c + k * stride_c) mod U (stride odd, U a power of two) and prio
    uniform 0..3 per entry."""
    g = torch.Generator(device=dev).manual_seed(seed)
    lens_t = torch.as_tensor(lens, dtype=torch.int64, device=dev)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(lens_t, 0)
    N = int(off[-1])
    base = torch.randint(0, U, (n,), generator=g, device=dev, dtype=torch.int64)
    stride = torch.randint(0, U // 2, (n,), generator=g, device=dev, dtype=torch.int64) * 2 + 1
    ctx = torch.repeat_interleave(torch.arange(n, device=dev), lens_t)
    k = torch.arange(N, device=dev, dtype=torch.int64) - off[:-1][ctx]
    elems = ((base[ctx] + k * stride[ctx]) & (U - 1)).to(torch.int32)
    del ctx, k
    prios = torch.randint(0, 4, (N,), generator=g, device=dev, dtype=torch.int8)
    return off, elems, prios


@pytest.mark.parametrize("n,mean,U,distinct", [(200_000, 2000, 1 << 22, False), (4000, 2000, 1 << 16, True)],
                         ids=["c3_200k", "distinct_len"])
def test_c3_minimize_vs_oracle(gpu, n, mean, U, distinct):
    rng = np.random.default_rng(2018)
    if distinct:
        lens = rng.permutation(np.arange(1, 2 * mean + 1))[:n]  # distinct Len: sort order is unambiguous
    else:
        lens = np.minimum(rng.geometric(1.0 / mean, size=n), U)
    off, elems, prios = _corpus_dev(gpu.dev, n, lens, U, seed=n)
    keep, cnt = gpu.minimize(off, elems, prios, hint_distinct=U)
    torch.cuda.synchronize()
    got = np.nonzero(keep.cpu().numpy())[0]
    exp = np.array(O.minimize(_u(off, np.uint64), _u(elems, np.uint32), _u(prios, np.int8)), np.int64)
    assert cnt == exp.size
    np.testing.assert_array_equal(got, exp)


def _owner_split(gpu, m0e, m0p, G, chunk=1 << 27):
    """M0 entries per owner shard (order kept), computed on device in chunks."""
    from syzkaller_amd.dist import owner_of_torch

    parts = [[] for _ in range(G)]
    for a in range(0, m0e.numel(), chunk):
        e, p = m0e[a:a + chunk], m0p[a:a + chunk]
        own = owner_of_torch(e, G)
        for g in range(G):
            m = own == g
            parts[g].append((e[m], p[m]))
        del own
    return [(torch.cat([x[0] for x in q]), torch.cat([x[1] for x in q])) for q in parts]


@pytest.mark.parametrize("walk", ["global", "region"])
def test_c5_streaming_skewed_vs_oracle(gpu, walk):
    """BASELINE config 5 at one rank's share of 8 GPUs, two consecutive
    batches, the second against the state the first left.  global: SURVEY
    8(d)'s C5 input (walks over all 2^20 blocks from Zipf(1.1)-chosen entries,
    skew=2; M0 holds the edge universe); region: rounds 1-4's power-skewed
    region walks (skew=1)."""
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth

    if walk == "global":
        cfg = synth.synth_default(global_walk=1, skew=2)
        P, C, L, known = 8192, 64, 1024, 1  # one rank's share of C5's 64k programs per batch on 8 GPUs
    else:
        cfg = synth.synth_default(skew=1)
        P, C, L, known = 4096, 64, 1024, 1024
    m0e, m0p = gpu.synth_m0(cfg, known, 10_000_000)
    ms = gpu.deserialize(m0e, m0p)
    ns = S.Signal(None, gpu.eng)
    oms = O.deserialize(_u(m0e, np.uint32), _u(m0p, np.int8))
    ons = O.OSig()
    for batch in range(2):  # the second batch sees the state the first one left
        sigs, cs, cnt, prio = device_batch(gpu, cfg, batch * P, P, C, L)
        pairs = torch.full((32 << 20,), -1, dtype=torch.int64, device=gpu.dev)
        _, cnew, st = gpu.triage(ms, ns, sigs, cs, cnt, prio, new_pairs=pairs, want_bits=False)
        hs, hcs, hcnt, hprio = _u(sigs, np.uint32), _u(cs, np.uint64), _u(cnt, np.uint32), _u(prio, np.uint8)
        ons, obits, ocnew = O.triage_batch_into(oms, hs, hcs, hcnt, hprio, ons)
        ocnew = ocnew[: hcnt.size]
        np.testing.assert_array_equal(_u(cnew, np.uint8), ocnew)
        op = pairs_from_bits(hs, hcs, hcnt, obits[: (hs.size + 31) // 32])
        assert st["new_pairs"] == op.size
        np.testing.assert_array_equal(np.sort(_u(pairs[: op.size], np.uint64)), op)
        assert ms.Len() == oms.Len() and ns.Len() == ons.Len()
        del sigs, cs, cnt, prio, pairs
    assert_same_set(ms, oms)
    assert_same_set(ns, ons)


def test_c4_step_api_1b_global_walk_vs_unsharded(gpu):
    """BASELINE config 4 through the API `bench.py --gpus 8` runs: the
    stream-ordered step (syzsig_step_send_dev / _own_dev / _back_dev /
    syzsig_step_finish, dist.ShardedTriage's device half) for 8 sources and 8
    owner shards of a 1B-element maxSignal on one GPU, the two all-to-alls
    replaced by tensor copies, on the C2 batch of SURVEY 8(d)'s global walk
    (1.07e9 records).  Against the same batch on the unsharded 1B table (the
    path test_c2 pins to the oracle): call_new, the DiffRaw pairs, the union
    of the shards and of the newSignal shards; and the oracle on a program
    prefix (syz-fuzzer/fuzzer.go:494-511)."""
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth
    from syzkaller_amd._lib import STEP_HDR_COUNT
    from syzkaller_amd.dist import SIGNAL_PRIO_LEVELS

    G, NM0 = 8, 1_000_000_000
    cfg = synth.synth_default(global_walk=1)
    P, C, L = 4096, 64, 4096
    sigs, cs, cnt, prio = device_batch(gpu, cfg, 0, P, C, L)
    nrec = int(cnt.to(torch.int64).sum())
    assert nrec > 1_000_000_000  # the global walk: almost every PC emits a signal
    m0e, m0p = gpu.synth_m0(cfg, 1, NM0)
    ms = gpu.deserialize(m0e, m0p)
    ns = S.Signal(None, gpu.eng)
    pairs = torch.full((32 << 20,), -1, dtype=torch.int64, device=gpu.dev)
    _, cnew, st = gpu.triage(ms, ns, sigs, cs, cnt, prio, new_pairs=pairs, want_bits=False)
    ref_pairs = np.sort(_u(pairs[: st["new_pairs"]], np.uint64))
    ref_cnew = cnew.clone()
    del pairs
    split = _owner_split(gpu, m0e, m0p, G)
    shards = [gpu.deserialize(e, p) for e, p in split]
    del split
    news = [S.Signal.make(1 << 20, gpu.eng) for _ in range(G)]
    levels = list(SIGNAL_PRIO_LEVELS)
    ncalls = P * C
    bounds = [ncalls * s // G for s in range(G + 1)]
    cap = nrec // (G * G) + 4096  # generous: no step is void
    W = cap + 1
    src = []
    for s in range(G):  # 1. every source's staircase into fixed buckets
        a, z = bounds[s], bounds[s + 1]
        sp = torch.full((32 << 20,), -1, dtype=torch.int64, device=gpu.dev)
        b, _, scnew = gpu.batch(sigs, cs[a:z].contiguous(), cnt[a:z].contiguous(), prio[a:z].contiguous(),
                                new_pairs=sp, want_bits=False)
        send = torch.empty(G * W, dtype=torch.int64, device=gpu.dev)
        gpu.step_send(b, a, levels, G, cap, send)
        sst = gpu.step_finish()
        assert not sst["global_void"] and not sst["src_void"] and sst["max_out"] <= cap, sst
        src.append((b, scnew, sp, send))
    flags = []
    for g in range(G):  # 2. the all-to-all: owner g's bucket s is source s's bucket g; 3. the owners
        recv = torch.cat([x[3][g * W: (g + 1) * W] for x in src])
        f = torch.empty(G * W, dtype=torch.uint8, device=gpu.dev)
        gpu.step_own(shards[g], news[g], recv, G, cap, levels, f)
        ost = gpu.step_finish()
        assert not ost["global_void"] and not ost["owners_void"], ost
        hdr = recv.view(G, W)[:, 0].cpu().numpy().view(np.uint64) & np.uint64(STEP_HDR_COUNT)
        assert ost["received"] == int(hdr.sum())
        flags.append(f)
        del recv
    got_pairs = []
    # (one context plays all 8 ranks: the pairs counter a rank's step_send
    # resets keeps running over these 8 step_back calls, so source s's pairs
    # are the ones it added, at [before, after) of its own buffer)
    before = 0
    for s, (b, scnew, sp, send) in enumerate(src):  # 4. the flags back; 5. each source's outputs
        back = torch.cat([flags[g][s * W: (s + 1) * W] for g in range(G)])
        gpu.step_back(b, bounds[s], send, G, cap, back)
        bst = gpu.step_finish()
        assert not bst["global_void"] and not bst["owners_void"], bst
        assert torch.equal(scnew, ref_cnew[bounds[s]: bounds[s + 1]])
        got_pairs.append(_u(sp[before: bst["new_pairs"]], np.uint64) + (np.uint64(bounds[s]) << np.uint64(32)))
        before = bst["new_pairs"]
    np.testing.assert_array_equal(np.sort(np.concatenate(got_pairs)), ref_pairs)
    del src, flags
    assert sum(x.Len() for x in shards) == ms.Len()
    U = S.Signal(None, gpu.eng)
    for x in shards:
        U.Merge(x)
    assert U.Len() == ms.Len() and ms.Diff(U).is_nil() and U.Diff(ms).is_nil()
    NU = S.Signal(None, gpu.eng)
    for x in news:
        NU.Merge(x)
    assert NU.Len() == ns.Len() and ns.Diff(NU).is_nil() and NU.Diff(ns).is_nil()
    del U, NU, shards
    # the oracle on a program prefix (M0 restricted to the prefix's elements)
    npre = 8 * C
    end = int(cs[npre - 1]) + int(cnt[npre - 1])
    hs, hcs, hcnt, hprio = (_u(sigs[:end], np.uint32), _u(cs[:npre], np.uint64), _u(cnt[:npre], np.uint32),
                            _u(prio[:npre], np.uint8))
    keys = np.unique(np.concatenate([hs[int(a): int(a) + int(n)] for a, n in zip(hcs, hcnt)]))
    fe, fp = O.filter_keys(_u(m0e, np.uint32), _u(m0p, np.int8), keys)
    _, _, obits, ocnew = O.triage_batch(fe, fp, hs, hcs, hcnt, hprio)
    np.testing.assert_array_equal(_u(ref_cnew[:npre], np.uint8), ocnew)
    op = pairs_from_bits(hs, hcs, hcnt, obits)
    np.testing.assert_array_equal(ref_pairs[ref_pairs < (np.uint64(npre) << np.uint64(32))], op)
