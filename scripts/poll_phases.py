"""Where the Poll line's wall time goes (host phases of signal.manager_poll)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from syzkaller_amd import signal as S  # noqa: E402
from syzkaller_amd.device import Device  # noqa: E402

dev = Device(0)
rng = np.random.default_rng(1027)
F, K, per, m0 = 16, 256, 16384, 10_000_000
e0 = rng.integers(0, 1 << 32, m0, dtype=np.uint64).astype(np.uint32)
p0 = rng.integers(0, 4, m0).astype(np.int8)
polls = []
for _ in range(K):
    known = rng.random(per) >= 0.05
    pick = rng.integers(0, m0, per)
    e = np.where(known, e0[pick], rng.integers(0, 1 << 32, per, dtype=np.uint64).astype(np.uint32))
    p = np.where(known, np.minimum(p0[pick], rng.integers(0, 4, per)), rng.integers(0, 4, per)).astype(np.int8)
    polls.append((int(rng.integers(0, F)), S.Serial(e.astype(np.uint32), p)))
pristine = S.Serial(e0, p0).Deserialize(dev.eng)
orig_many = S.serialize_many
T = {}


def timed_many(sets, eng=None):
    t = time.perf_counter()
    r = orig_many(sets, eng)
    T["serialize_many"] = time.perf_counter() - t
    return r


S.serialize_many = timed_many
for r in range(4):
    ms = pristine.clone()
    nm = [S.Signal(None, dev.eng) for _ in range(F)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    el = np.concatenate([np.asarray(s.Elems, np.uint32) for _, s in polls])
    pr = np.concatenate([np.asarray(s.Prios, np.int8) for _, s in polls])
    t1 = time.perf_counter()
    replies = S.manager_poll(ms, nm, polls, dev.eng)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    del replies
    t3 = time.perf_counter()
    print(f"concat {1e3*(t1-t0):.2f} ms  manager_poll {1e3*(t2-t1):.2f} ms (serialize_many "
          f"{1e3*T['serialize_many']:.2f}, stream {dev.L.syzsig_ctx_last_ms(dev.eng.h):.2f})  del replies "
          f"{1e3*(t3-t2):.2f} ms", flush=True)
    del ms, nm
