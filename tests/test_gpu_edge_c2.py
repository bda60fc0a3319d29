"""GPU: K1+K2 (edge.hip) and K3 at BASELINE config 2's full shape -- 4096
programs x 64 calls x 4096 PCs, 1.07e9 PCs -- against the oracle.

  * the bench's workload (syscall-region walk): every program's sig_cnt,
    completed and emitted signals against oracle.exec_batch, in slices of 256
    programs synthesized on the host (the same generator the device runs);
  * SURVEY 8(d)'s global walk (every call walks b <- (4b + 1 + r%4) mod 2^20
    from a uniform block, no restarts: almost every PC is a new edge for the
    program's lossy dedup table, so K2 writes on nearly every signal): the same
    edge check, then checkNewSignal over the whole 1.07e9-record batch against
    a 10M-element M0 drawn from that walk's edge universe, against the
    sequential oracle run per element shard (see _triage_oracle_sharded).

References: executor/executor.h:492-512 (write_coverage_signal), :687-706
(dedup), syz-fuzzer/fuzzer.go:494-511 (checkNewSignal).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu

NPROG, CPP, PCS = 4096, 64, 4096
SLICE = 256  # programs per host oracle slice (67M PCs)


def _u(t, dt):
    return t.cpu().numpy().view(dt)


def _device_edge(gpu, cfg):
    from syzkaller_amd import synth

    cl = torch.full((NPROG * CPP,), PCS, dtype=torch.int32)
    pcs, cs, cl, prio = gpu.synth_traces(cfg, 0, NPROG, CPP, cl)
    pidx = torch.from_numpy(synth.prog_call_index(NPROG, CPP).view(np.int32)).to(gpu.dev)
    sigs, cnt, comp = gpu.edge_derive(pcs, cs, cl, pidx)
    torch.cuda.synchronize()
    del pcs
    return sigs, cs, cnt, comp, prio


def _check_edge_slices(cfg, sigs, cnt, comp):
    """Device K1+K2 output of the full batch vs oracle.exec_batch, slice by slice."""
    from syzkaller_amd import synth

    hcnt, hcomp = _u(cnt, np.uint32), _u(comp, np.uint32)
    pidx = synth.prog_call_index(SLICE, CPP)
    pos = np.arange(PCS, dtype=np.uint32)[None, :]
    for p0 in range(0, NPROG, SLICE):
        cl = synth.call_lengths(SLICE, CPP, PCS)
        pcs, cs, _ = synth.traces(cfg, p0, SLICE, CPP, cl)
        es, ec, ed = O.exec_batch(pcs, cs, cl, pidx)
        del pcs
        c0, c1 = p0 * CPP, (p0 + SLICE) * CPP
        np.testing.assert_array_equal(hcomp[p0: p0 + SLICE], ed, err_msg=f"completed, programs {p0}+")
        np.testing.assert_array_equal(hcnt[c0:c1], ec, err_msg=f"sig_cnt, programs {p0}+")
        dev = _u(sigs[c0 * PCS: c1 * PCS], np.uint32).reshape(-1, PCS)
        live = pos < ec[:, None]
        np.testing.assert_array_equal(dev[live], es.reshape(-1, PCS)[live], err_msg=f"signals, programs {p0}+")


@pytest.mark.parametrize("mode", ["markall", "passes"])
def test_edge_c2_full_batch_vs_oracle(gpu, mode):
    """The region walk (mostly duplicates) under both of K2's marking modes."""
    from syzkaller_amd import synth
    from syzkaller_amd._lib import SYZSIG_DEBUG_EDGE_MARKALL, SYZSIG_DEBUG_EDGE_PASSES

    cfg = synth.synth_default()
    gpu.eng.set_debug(SYZSIG_DEBUG_EDGE_MARKALL if mode == "markall" else SYZSIG_DEBUG_EDGE_PASSES)
    try:
        sigs, cs, cnt, comp, prio = _device_edge(gpu, cfg)
    finally:
        gpu.eng.set_debug(0)
    _check_edge_slices(cfg, sigs, cnt, comp)


def test_edge_c2_global_walk_vs_oracle(gpu):
    from syzkaller_amd import synth

    cfg = synth.synth_default(global_walk=1)
    sigs, cs, cnt, comp, prio = _device_edge(gpu, cfg)
    assert int(cnt.to(torch.int64).sum()) > 0.9 * NPROG * CPP * PCS  # almost every edge is emitted
    _check_edge_slices(cfg, sigs, cnt, comp)


def _owner16(e):
    return ((e.astype(np.uint32) * np.uint32(0x9E3779B1)) >> np.uint32(28)).astype(np.uint8)


def _triage_oracle_sharded(m0e, m0p, rec_sig, rec_call, ncalls, call_prio, T=16):
    """Sequential checkNewSignal (oracle.c orc_triage_batch) run on T element
    shards in parallel threads.  Exact: an element's new records, M_final and
    newSignal entry depend only on that element's own records in serial order
    and on M0[e] ("Batch restatement"), so running the sequential
    loop on each shard's records -- serial order kept, every call present --
    and taking the union is the same computation as one loop over the batch.
    Returns (max-final (elems, prios), newSignal (elems, prios), sorted unique
    new pairs call << 32 | elem, call_new u8[ncalls])."""
    own = _owner16(rec_sig)
    order = np.argsort(own, kind="stable")  # radix sort: serial order kept per shard
    bounds = np.searchsorted(own[order], np.arange(T + 1))
    own_m0 = _owner16(m0e)

    def shard(g):
        idx = order[bounds[g]: bounds[g + 1]]
        s_sig, s_call = rec_sig[idx], rec_call[idx]
        s_cnt = np.bincount(s_call, minlength=ncalls).astype(np.uint32)
        s_cs = np.zeros(ncalls, np.uint64)
        np.cumsum(s_cnt[:-1], out=s_cs[1:])
        m = own_m0 == g
        ms, ns, bits, cnew = O.triage_batch(m0e[m], m0p[m], s_sig, s_cs, s_cnt, call_prio)
        r = np.nonzero(np.unpackbits(bits.view(np.uint8), bitorder="little")[: s_sig.size])[0]
        pairs = (s_call[r].astype(np.uint64) << np.uint64(32)) | s_sig[r].astype(np.uint64)
        return ms.Serialize(), ns.Serialize(), pairs, cnew

    with ThreadPoolExecutor(T) as ex:
        res = list(ex.map(shard, range(T)))
    cat = lambda k, j: np.concatenate([r[k][j] for r in res])  # noqa: E731
    cnew = np.zeros(ncalls, np.uint8)
    for r in res:
        cnew |= r[3]
    return (cat(0, 0), cat(0, 1)), (cat(1, 0), cat(1, 1)), np.unique(np.concatenate([r[2] for r in res])), cnew


def _sorted(e, p):
    o = np.argsort(e, kind="stable")
    return e[o], p[o]


def test_triage_c2_global_walk_vs_oracle(gpu):
    """checkNewSignal over the whole global-walk C2 batch (1.07e9 records,
    ~5M distinct elements, most of them in M0) on the bench's aggregation
    path, against the element-sharded sequential oracle."""
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth

    cfg = synth.synth_default(global_walk=1)
    sigs, cs, cnt, comp, prio = _device_edge(gpu, cfg)
    m0e, m0p = gpu.synth_m0(cfg, 1, 10_000_000)
    ms = gpu.deserialize(m0e, m0p)
    ns = S.Signal(None, gpu.eng)
    pairs = torch.full((32 << 20,), -1, dtype=torch.int64, device=gpu.dev)
    _, cnew, st = gpu.triage(ms, ns, sigs, cs, cnt, prio, new_pairs=pairs, want_bits=False)
    torch.cuda.synchronize()
    nrec = int(cnt.to(torch.int64).sum())
    assert st["records"] == nrec and st["runs"] == 1 and st["overflow_parts"] == 0
    # the batch's records in serial order, compacted on the host
    hcnt = _u(cnt, np.uint32)
    live = (np.arange(PCS, dtype=np.uint32)[None, :] < hcnt[:, None]).ravel()
    rec_sig = _u(sigs, np.uint32)[live]
    rec_call = np.repeat(np.arange(NPROG * CPP, dtype=np.int64), hcnt)
    del live
    (oe, op), (ne, np_), opairs, ocnew = _triage_oracle_sharded(_u(m0e, np.uint32), _u(m0p, np.int8), rec_sig,
                                                                rec_call, NPROG * CPP, _u(prio, np.uint8))
    del rec_sig, rec_call
    np.testing.assert_array_equal(_u(cnew, np.uint8), ocnew)
    assert st["new_pairs"] == opairs.size <= pairs.numel()
    np.testing.assert_array_equal(np.sort(_u(pairs[: opairs.size], np.uint64)), opairs)
    ge, gp = _sorted(*(lambda s: (s.Elems, s.Prios))(ms.Serialize()))
    oe, op = _sorted(oe, op)
    np.testing.assert_array_equal(ge, oe)
    np.testing.assert_array_equal(gp, op)
    ge, gp = _sorted(*(lambda s: (s.Elems, s.Prios))(ns.Serialize()))
    ne, np_ = _sorted(ne, np_)
    np.testing.assert_array_equal(ge, ne)
    np.testing.assert_array_equal(gp, np_)
