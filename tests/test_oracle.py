"""CPU: the oracle (oracle/oracle.c) pinned against (a) golden vectors written
by the reference executor itself and (b) hand-derived pkg/signal KATs."""
import os

import numpy as np
import pytest

from oracle import oracle as O
from tests import kat_runner as KR
from tests.conftest import golden_names, load_golden


@pytest.mark.parametrize("name", golden_names())
def test_oracle_matches_reference_executor_goldens(name):
    fx = load_golden(name)
    sigs, cnt, comp = O.exec_batch(fx["pcs"], fx["call_start"], fx["call_len"], fx["prog_call"])
    np.testing.assert_array_equal(comp, fx["exp_completed"])
    np.testing.assert_array_equal(cnt, fx["exp_cnt"])
    for c in range(fx["call_len"].size):
        s, n = int(fx["call_start"][c]), int(fx["exp_cnt"][c])
        np.testing.assert_array_equal(sigs[s: s + n], fx["exp_sigs"][s: s + n], err_msg=f"call {c}")


def test_goldens_cover_corner_cases():
    zero = load_golden("executor_zero")
    assert 0 in set(zero["exp_sigs"][zero["call_start"][1]: zero["call_start"][1] + zero["exp_cnt"][1]].tolist())
    abort = load_golden("executor_abort")
    assert (abort["exp_completed"] < np.diff(abort["prog_call"])).any()
    big = load_golden("executor_big")
    assert big["call_len"].max() == 262143
    assert (load_golden("executor_synth")["call_len"] == 0).any()


@pytest.mark.skipif(not os.path.exists(O.REF_HARNESS), reason="reference harness not built (no /root/reference)")
def test_oracle_matches_live_reference_on_fresh_programs():
    from syzkaller_amd import synth

    cfg = synth.synth_default(region_log2=10, bad_pc_ppm=50)
    nprog, cpp = 4, 6
    cl = synth.call_lengths(nprog, cpp, 0, ragged=(0, 5000), seed=99)
    pcs, cs, prio = synth.traces(cfg, 777, nprog, cpp, cl)
    pidx = synth.prog_call_index(nprog, cpp)
    sigs, cnt, comp = O.exec_batch(pcs, cs, cl, pidx)
    progs = [[(((prio[c] >> 1) & 1) == 0, pcs[cs[c]: cs[c] + cl[c]]) for c in range(pidx[p], pidx[p + 1])]
             for p in range(nprog)]
    for p, (completed, calls) in enumerate(O.run_reference_executor(progs)):
        assert completed == comp[p]
        for idx, err, rs in calls:
            c = pidx[p] + idx
            np.testing.assert_array_equal(sigs[cs[c]: cs[c] + cnt[c]], rs)


class OracleImpl(KR.Impl):
    corrupt_exc = ValueError

    def nil(self):
        return O.OSig()

    def empty(self):
        return O.OSig(O.lib().orc_sig_new(0))

    def from_dict(self, d):
        return O.deserialize(np.array(list(d.keys()), np.uint32), np.array(list(d.values()), np.int8))

    def from_raw(self, raw, prio):
        return O.from_raw(raw, prio)

    def deserialize(self, e, p):
        return O.deserialize(e, p)

    def minimize(self, ctxs):
        off = np.zeros(len(ctxs) + 1, np.uint64)
        off[1:] = np.cumsum([len(c) for c in ctxs]) if ctxs else []
        e = np.array([k for c in ctxs for k in c], np.uint32)
        p = np.array([v for c in ctxs for v in c.values()], np.int8)
        return O.minimize(off, e, p)

    def check_new(self, m0, calls):
        sigs, starts, lens, prios = KR.flatten_calls(calls)
        me = np.array(list(m0.keys()), np.uint32)
        mp = np.array(list(m0.values()), np.int8)
        ms, ns, bits, cnew = O.triage_batch(me, mp, sigs, starts, lens, prios)
        return ([i for i, f in enumerate(cnew) if f], ms.to_dict(), ns.to_dict(),
                KR.rec_sets_from_bits(bits, starts, lens))


@pytest.mark.parametrize("run", KR.ALL, ids=[f.__name__ for f in KR.ALL])
def test_oracle_kat(run):
    run(OracleImpl())


def test_oracle_minimize_matches_literal_python():
    """Cross-check orc_minimize against a literal Python transcription of
    signal.go:138-166 on random corpora with distinct Len values."""
    rng = np.random.default_rng(5)
    for trial in range(20):
        n = int(rng.integers(1, 40))
        lens = rng.permutation(np.arange(1, 200))[:n]
        ctxs = []
        for L in lens:
            el = rng.choice(300, size=int(L), replace=False)
            ctxs.append({int(e): int(rng.integers(-2, 4)) for e in el})
        order = sorted(range(n), key=lambda i: (-len(ctxs[i]), i))
        covered = {}
        for si, ci in enumerate(order):
            for e, p in ctxs[ci].items():
                if e not in covered or p > covered[e][0]:
                    covered[e] = (p, si)
        exp = sorted(order[si] for si in {v[1] for v in covered.values()})
        assert sorted(OracleImpl().minimize(ctxs)) == exp


@pytest.mark.parametrize("threads", [1, 4])
def test_oracle_mt_baseline_matches_sequential(threads):
    """orc_triage_batch_mt (the bench's nproc-core CPU baseline: Procs under
    one rwlock, fuzzer.go:494-511) ends in the same maxSignal and newSignal
    as sequential checkNewSignal; which calls report new signal depends on the
    thread interleaving, so only its bounds are checked."""
    from syzkaller_amd import synth

    cfg = synth.synth_default(skew=1)
    nprog, cpp = 24, 16
    cl = synth.call_lengths(nprog, cpp, 600)
    pidx = synth.prog_call_index(nprog, cpp)
    pcs, cs, prio = synth.traces(cfg, 0, nprog, cpp, cl)
    sigs, cnt, _ = O.exec_batch(pcs, cs, cl, pidx)
    m0e, m0p = synth.m0(cfg, 64, 20000)
    ms, ns, _, cnew = O.triage_batch(m0e, m0p, sigs, cs, cnt, prio)
    ms2 = O.deserialize(m0e, m0p)
    ns2, ncalls = O.triage_batch_mt(ms2, sigs, cs, cnt, prio, cpp, threads)
    assert ms2.to_dict() == ms.to_dict()
    assert ns2.to_dict() == ns.to_dict()
    assert 0 < ncalls <= cnt.size
    if threads == 1:
        assert ncalls == int(cnew.sum())
