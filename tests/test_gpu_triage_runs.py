"""GPU: triageInput's signal re-runs (syz-fuzzer/proc.go:107-140) over a batch
of triage items, against the restatement built from the oracle's Signal ops
(Deserialize / FromRaw / Intersection), covering skipped runs (not executed,
empty signal, failed after success), the give-up rule, minimized items and
prio ordering (Intersection keeps e only when the run's prio >= e's prio)."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def make_items(rng, nitems, runs):
    item_off, elems, prios, flags = [0], [], [], []
    run_off, run_sigs, run_prio, run_errno, run_exec = [0], [], [], [], []
    for i in range(nitems):
        n = int(rng.integers(0, 120)) if i % 11 else 0
        e = np.unique(rng.integers(0, 5000, n).astype(np.uint32) + np.uint32(i * 10000))
        elems.append(e)
        prios.append(rng.integers(-1, 4, e.size).astype(np.int8))
        item_off.append(item_off[-1] + e.size)
        flags.append(int(rng.integers(0, 4)))
        for r in range(runs):
            keep_frac = rng.choice([1.0, 0.97, 0.6, 0.0])
            sig = e[rng.random(e.size) < keep_frac]
            noise = rng.integers(0, 5000, int(rng.integers(0, 50))).astype(np.uint32) + np.uint32(i * 10000)
            sig = np.concatenate([sig, noise]) if rng.random() < 0.9 else np.empty(0, np.uint32)
            rng.shuffle(sig)
            run_sigs.append(sig)
            run_off.append(run_off[-1] + sig.size)
            run_prio.append(int(rng.integers(0, 4)))
            run_errno.append(int(rng.choice([0, 0, 0, 22])))
            run_exec.append(int(rng.random() < 0.9))
    cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.empty(0, dt)  # noqa: E731
    return (np.array(item_off, np.uint64), cat(elems, np.uint32), cat(prios, np.int8), np.array(flags, np.uint8),
            np.array(run_off, np.uint64), cat(run_sigs, np.uint32), np.array(run_prio, np.uint8),
            np.array(run_errno, np.int32), np.array(run_exec, np.uint8))


def _t(gpu, a, dt):
    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu.dev)


@pytest.mark.parametrize("runs,seed", [(3, 1), (3, 2), (1, 3), (5, 4), (0, 5)])
def test_triage_runs_vs_restatement(gpu, runs, seed):
    rng = np.random.default_rng(seed)
    io, el, pr, fl, ro, rs, rp, re, rx = make_items(rng, 400, runs)
    ik, ek = gpu.triage_runs(_t(gpu, io, np.int64), _t(gpu, el, np.int32), _t(gpu, pr, np.int8),
                             _t(gpu, fl, np.uint8), runs, _t(gpu, ro, np.int64), _t(gpu, rs, np.int32),
                             _t(gpu, rp, np.uint8), _t(gpu, re, np.int32), _t(gpu, rx, np.uint8))
    okeep, finals = O.triage_runs(io, el, pr, fl, runs, ro, rs, rp, re, rx)
    ik, ek = ik.cpu().numpy(), ek.cpu().numpy()
    np.testing.assert_array_equal(ik, okeep)
    assert 0 < okeep.sum() < okeep.size or runs == 0
    for i in range(io.size - 1):
        a, b = int(io[i]), int(io[i + 1])
        got = {int(e): int(p) for e, p, k in zip(el[a:b], pr[a:b], ek[a:b]) if k}
        assert got == (finals[i] or {}), i


def test_triage_runs_empty_batch(gpu):
    z64 = torch.zeros(1, dtype=torch.int64, device=gpu.dev)
    e = torch.empty(0, dtype=torch.int32, device=gpu.dev)
    u8 = torch.empty(0, dtype=torch.uint8, device=gpu.dev)
    ik, ek = gpu.triage_runs(z64, e, u8.view(torch.int8), u8, 3, z64, e, u8, e, u8)
    assert ik.numel() == 0 and ek.numel() == 0


@pytest.mark.parametrize("attempts,seed", [(3, 11), (1, 12), (4, 13)])
def test_minimize_pred_vs_restatement(gpu, attempts, seed):
    rng = np.random.default_rng(seed)
    io, el, pr, fl, ro, rs, rp, re, rx = make_items(rng, 400, attempts)
    pred = gpu.minimize_pred(_t(gpu, io, np.int64), _t(gpu, el, np.int32), _t(gpu, pr, np.int8),
                             _t(gpu, fl, np.uint8), attempts, _t(gpu, ro, np.int64), _t(gpu, rs, np.int32),
                             _t(gpu, rp, np.uint8), _t(gpu, re, np.int32), _t(gpu, rx, np.uint8))
    exp = O.minimize_pred(io, el, pr, fl, attempts, ro, rs, rp, re, rx)
    np.testing.assert_array_equal(pred.cpu().numpy(), exp)
    assert 0 < exp.sum() < exp.size
