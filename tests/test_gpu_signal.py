"""GPU: pkg/signal's algebra on device (table.hip) through the C ABI, against the
known answers and differentially against the oracle on random sets."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import kat_runner as KR

pytestmark = pytest.mark.gpu


class GpuImpl(KR.Impl):
    def __init__(self, dev):
        from syzkaller_amd import signal as S
        from syzkaller_amd._lib import CorruptedSerial

        self.S, self.eng = S, dev.eng
        self.corrupt_exc = CorruptedSerial

    def nil(self):
        return self.S.Signal(None, self.eng)

    def empty(self):
        return self.S.Signal.make(0, self.eng)

    def from_dict(self, d):
        return self.S.Serial(list(d.keys()), list(d.values())).Deserialize(self.eng)

    def from_raw(self, raw, prio):
        return self.S.FromRaw(raw, prio, self.eng)

    def deserialize(self, e, p):
        return self.S.Serial(e, p).Deserialize(self.eng)

    def minimize(self, ctxs):
        corpus = [self.S.Context(self.make(c) if c else self.empty(), i) for i, c in enumerate(ctxs)]
        return self.S.Minimize(corpus, self.eng)

    def check_new(self, m0, calls):
        ms = self.make(m0) if m0 else self.empty()
        ns = self.nil()
        idx, bits = self.S.check_new_signal(ms, ns, calls, self.eng, want_bits=True)
        _, starts, lens, _ = KR.flatten_calls(calls)
        return idx, ms.to_dict(), (ns.to_dict() if not ns.is_nil() else {}), KR.rec_sets_from_bits(bits, starts, lens)


@pytest.mark.parametrize("run", KR.ALL, ids=[f.__name__ for f in KR.ALL])
def test_gpu_kat(gpu, run):
    run(GpuImpl(gpu))


def _rand_sig(rng, n, universe, prio_lo=-3, prio_hi=4):
    e = rng.choice(universe, size=min(n, universe), replace=False).astype(np.uint32)
    p = rng.integers(prio_lo, prio_hi, size=e.size).astype(np.int8)
    return e, p


@pytest.mark.parametrize("seed", range(4))
def test_gpu_algebra_random_vs_oracle(gpu, seed):
    from syzkaller_amd import signal as S

    rng = np.random.default_rng(seed)
    U = 1 << int(rng.integers(8, 20))
    for _ in range(6):
        a = _rand_sig(rng, int(rng.integers(0, 5000)), U)
        b = _rand_sig(rng, int(rng.integers(0, 5000)), U)
        ga, gb = S.Serial(*a).Deserialize(gpu.eng), S.Serial(*b).Deserialize(gpu.eng)
        oa, ob = O.deserialize(*a), O.deserialize(*b)
        assert KR.as_result(ga) == KR.as_result(oa)
        assert KR.as_result(ga.Diff(gb)) == KR.as_result(oa.Diff(ob))
        assert KR.as_result(ga.Intersection(gb)) == KR.as_result(oa.Intersection(ob))
        raw = rng.integers(0, U, size=int(rng.integers(0, 8000))).astype(np.uint32)
        prio = int(rng.integers(0, 256))
        assert KR.as_result(ga.DiffRaw(raw, prio)) == KR.as_result(oa.DiffRaw(raw, prio))
        assert KR.as_result(S.FromRaw(raw, prio, gpu.eng)) == KR.as_result(O.from_raw(raw, prio))
        ga.Merge(gb)
        oa.Merge(ob)
        assert ga.to_dict() == oa.to_dict()
        assert ga.Len() == oa.Len()


def test_gpu_merge_growth_and_serialize_roundtrip(gpu):
    from syzkaller_amd import signal as S

    rng = np.random.default_rng(7)
    acc, oacc = S.Signal(None, gpu.eng), O.OSig()
    for step in range(8):
        e, p = _rand_sig(rng, 20000 * (step + 1), 1 << 22)
        g, o = S.Serial(e, p).Deserialize(gpu.eng), O.deserialize(e, p)
        acc.Merge(g)
        oacc.Merge(o)
    assert acc.Len() == oacc.Len()
    ser = acc.Serialize()
    assert len(set(ser.Elems.tolist())) == ser.Elems.size == acc.Len()
    back = ser.Deserialize(gpu.eng)
    assert back.to_dict() == oacc.to_dict()


def test_gpu_deserialize_last_duplicate_wins(gpu):
    from syzkaller_amd import signal as S

    rng = np.random.default_rng(3)
    e = rng.integers(0, 1000, size=50000).astype(np.uint32)
    p = rng.integers(-128, 128, size=e.size).astype(np.int8)
    assert S.Serial(e, p).Deserialize(gpu.eng).to_dict() == O.deserialize(e, p).to_dict()


def test_gpu_serialize_many_vs_serialize(gpu):
    """syzsig_serialize_batch (the Poll replies' Serialize, manager.go:1049)
    against one Serialize per set: nil, empty-after-Subtract, small and
    multi-block sets in one call; set i's entries in [offs[i], offs[i+1])."""
    import ctypes

    from syzkaller_amd import signal as S
    from syzkaller_amd._lib import SyzsigError

    rng = np.random.default_rng(7)
    sets = [None]
    for n in (1, 5, 300, 70_000, 0, 2_000_000, 17):
        e = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
        p = rng.integers(-128, 128, n).astype(np.int8)
        sets.append(S.Serial(e, p).Deserialize(gpu.eng) if n else S.Signal.make(0, gpu.eng))
    sets.append(None)
    got = S.serialize_many(sets, gpu.eng)
    assert len(got) == len(sets)
    for s, g in zip(sets, got):
        want = s.Serialize() if s is not None else S.Serial()
        assert g.Elems.size == want.Elems.size
        o1, o2 = np.argsort(g.Elems), np.argsort(want.Elems)
        np.testing.assert_array_equal(g.Elems[o1], want.Elems[o2])
        np.testing.assert_array_equal(g.Prios[o1], want.Prios[o2])
    # a cap below the total is refused, with the offsets filled
    hs = (ctypes.c_void_p * len(sets))(*[(x.handle.value or 0) if x is not None else 0 for x in sets])
    offs = np.zeros(len(sets) + 1, np.uint64)
    e = np.empty(10, np.uint32)
    p = np.empty(10, np.int8)
    rc = gpu.eng.L.syzsig_serialize_batch(gpu.eng.h, hs, len(sets), e.ctypes.data, p.ctypes.data, 10,
                                          offs.ctypes.data)
    assert rc != 0 and int(offs[-1]) == sum(g.Elems.size for g in got)
    with pytest.raises(SyzsigError):
        from syzkaller_amd._lib import check
        check(rc)
