"""GPU: the manager's Poll over a batch of polls (csrc/poll.hip,
syzsig_manager_poll_batch) against the reference's sequential loop restated
over the oracle's Signal ops (oracle.poll: syz-manager/manager.go:1027-1052)."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _serial(rng, n, U, dup=True):
    e = rng.integers(0, U, size=n).astype(np.uint32)  # duplicates inside a Serial: the later one wins
    if not dup:
        e = np.unique(e)
    p = rng.integers(-3, 5, size=e.size).astype(np.int8)
    return e, p


@pytest.mark.parametrize("seed,F,K,U,n,limits", [(0, 5, 40, 3000, 400, None), (1, 1, 8, 500, 100, None),
                                                 (2, 16, 200, 50_000, 3000, None), (3, 3, 30, 200, 50, None),
                                                 (4, 5, 40, 3000, 400, (24, 4000))])
def test_poll_batch_vs_sequential_oracle(gpu, monkeypatch, seed, F, K, U, n, limits):
    """limits: (polls x fuzzers, entries x fuzzers) per library call lowered so
    that signal.manager_poll applies the batch as several consecutive calls."""
    from syzkaller_amd import signal as S

    if limits:
        monkeypatch.setattr(S, "POLL_MAX_NEXT", limits[0])
        monkeypatch.setattr(S, "POLL_MAX_FANOUT", limits[1])
    rng = np.random.default_rng(seed)
    m0 = _serial(rng, 4 * n, U, dup=False)
    pre = [None if rng.random() < 0.3 else _serial(rng, int(rng.integers(0, n)), U, dup=False) for _ in range(F)]
    polls = [(int(rng.integers(0, F)), _serial(rng, int(rng.integers(0, 2 * n)), U)) for _ in range(K)]
    # device
    ms = S.Serial(*m0).Deserialize(gpu.eng)
    nm = [S.Serial(*p).Deserialize(gpu.eng) if p is not None else S.Signal(None, gpu.eng) for p in pre]
    replies = S.manager_poll(ms, nm, [(f, S.Serial(e, p)) for f, (e, p) in polls], gpu.eng)
    # oracle: one poll after the other
    oms = O.deserialize(*m0)
    onm = [O.deserialize(*p) if p is not None else O.OSig() for p in pre]
    for i, (f, ser) in enumerate(polls):
        re, rp = O.poll(oms, onm, f, ser)
        got = dict(zip(replies[i].Elems.tolist(), replies[i].Prios.tolist()))
        assert got == dict(zip(re.tolist(), rp.tolist())), f"reply {i}"
    assert ms.to_dict() == oms.to_dict()
    for g in range(F):
        assert (nm[g].to_dict() if not nm[g].is_nil() else {}) == onm[g].to_dict(), f"fuzzer {g}"
        assert nm[g].is_nil() == onm[g].is_nil() or onm[g].Len() == 0


def test_poll_batch_empty_and_nil_max(gpu):
    from syzkaller_amd import signal as S

    ms = S.Signal(None, gpu.eng)
    nm = [S.Signal(None, gpu.eng) for _ in range(3)]
    rep = S.manager_poll(ms, nm, [(0, S.Serial()), (1, S.Serial([7, 8, 7], [1, 2, 0])), (0, S.Serial())], gpu.eng)
    assert [r.Elems.size for r in rep] == [0, 0, 2]
    assert dict(zip(rep[2].Elems.tolist(), rep[2].Prios.tolist())) == {7: 0, 8: 2}
    assert ms.to_dict() == {7: 0, 8: 2}
    assert nm[0].is_nil() and nm[1].is_nil() and nm[2].to_dict() == {7: 0, 8: 2}


@pytest.mark.parametrize("case", ["forced_sequential", "hot_element"])
def test_poll_batch_sequential_path_vs_oracle(gpu, case):
    """The batch's exact fallback (csrc/poll.hip poll_sequential: the
    reference loop over the set ops) -- forced (SYZSIG_DEBUG_RECS_GATE gates
    every element partition), or taken because one element is in every one of
    3000 polls (its partition holds more than 2048 entries) -- against the
    oracle's sequential loop."""
    from syzkaller_amd import signal as S
    from syzkaller_amd._lib import SYZSIG_DEBUG_RECS_GATE

    rng = np.random.default_rng(11)
    F, U = 6, 4000
    K, n = (40, 300) if case == "forced_sequential" else (3000, 20)
    m0 = _serial(rng, 1000, U, dup=False)
    pre = [None if g % 3 == 0 else _serial(rng, 50, U, dup=False) for g in range(F)]
    polls = []
    for _ in range(K):
        e, p = _serial(rng, int(rng.integers(0, n)), U)
        if case == "hot_element":
            e, p = np.append(e, np.uint32(7)), np.append(p, np.int8(rng.integers(-3, 5)))
        polls.append((int(rng.integers(0, F)), (e, p)))
    ms = S.Serial(*m0).Deserialize(gpu.eng)
    nm = [S.Serial(*p).Deserialize(gpu.eng) if p is not None else S.Signal(None, gpu.eng) for p in pre]
    gpu.eng.set_debug(SYZSIG_DEBUG_RECS_GATE if case == "forced_sequential" else 0)
    try:
        replies = S.manager_poll(ms, nm, [(f, S.Serial(e, p)) for f, (e, p) in polls], gpu.eng)
    finally:
        gpu.eng.set_debug(0)
    oms = O.deserialize(*m0)
    onm = [O.deserialize(*p) if p is not None else O.OSig() for p in pre]
    for i, (f, ser) in enumerate(polls):
        re, rp = O.poll(oms, onm, f, ser)
        got = dict(zip(replies[i].Elems.tolist(), replies[i].Prios.tolist()))
        assert got == dict(zip(re.tolist(), rp.tolist())), f"reply {i}"
    assert ms.to_dict() == oms.to_dict()
    for g in range(F):
        assert (nm[g].to_dict() if not nm[g].is_nil() else {}) == onm[g].to_dict(), f"fuzzer {g}"


def test_poll_batch_sequential_failure_leaves_sets(gpu):
    """the sequential fallback is all or nothing like
    the batched path -- a failure before its last poll (injected,
    SYZSIG_DEBUG_POLL_FAIL) leaves maxSignal and every fuzzer's newMaxSignal
    as they were (nil ones nil), and hands out no reply."""
    from syzkaller_amd import signal as S
    from syzkaller_amd._lib import SYZSIG_DEBUG_POLL_FAIL, SYZSIG_DEBUG_RECS_GATE, SyzsigError

    rng = np.random.default_rng(5)
    F, U, K = 4, 3000, 12
    m0 = _serial(rng, 800, U, dup=False)
    pre = [None if g % 2 == 0 else _serial(rng, 40, U, dup=False) for g in range(F)]
    polls = [(int(rng.integers(0, F)), S.Serial(*_serial(rng, 200, U))) for _ in range(K)]
    ms = S.Serial(*m0).Deserialize(gpu.eng)
    nm = [S.Serial(*p).Deserialize(gpu.eng) if p is not None else S.Signal(None, gpu.eng) for p in pre]
    before = (ms.to_dict(), [None if s.is_nil() else s.to_dict() for s in nm])
    gpu.eng.set_debug(SYZSIG_DEBUG_RECS_GATE | SYZSIG_DEBUG_POLL_FAIL)
    try:
        with pytest.raises(SyzsigError):
            S.manager_poll(ms, nm, polls, gpu.eng)
    finally:
        gpu.eng.set_debug(0)
    assert (ms.to_dict(), [None if s.is_nil() else s.to_dict() for s in nm]) == before
    # and the same batch then goes through, against the oracle
    replies = S.manager_poll(ms, nm, polls, gpu.eng)
    oms = O.deserialize(*m0)
    onm = [O.deserialize(*p) if p is not None else O.OSig() for p in pre]
    for i, (f, ser) in enumerate(polls):
        re, rp = O.poll(oms, onm, f, (np.asarray(ser.Elems), np.asarray(ser.Prios)))
        assert dict(zip(replies[i].Elems.tolist(), replies[i].Prios.tolist())) == dict(zip(re.tolist(), rp.tolist()))
    assert ms.to_dict() == oms.to_dict()
