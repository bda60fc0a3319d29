"""Debug: C1 batch on the aggregation path, stats + call_new vs oracle."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_gpu_triage import dev_batch, host_batch  # noqa: E402
from oracle import oracle as O  # noqa: E402
from syzkaller_amd import signal as S  # noqa: E402
from syzkaller_amd import synth  # noqa: E402
from syzkaller_amd.device import Device  # noqa: E402

gpu = Device(0)
cfg = synth.synth_default()
nprog, cpp = 64, 32
cl = synth.call_lengths(nprog, cpp, 2048)
m0 = synth.m0(cfg, 2048, 200000)
hs, hcs, hcnt, hprio = host_batch(cfg, nprog, cpp, cl)
ds, dcs, dcnt, dprio = dev_batch(gpu, cfg, nprog, cpp, cl)
for wb in (True, False):
    ms = S.Serial(*m0).Deserialize(gpu.eng)
    ns = S.Signal(None, gpu.eng)
    pairs = torch.full((int(hcnt.sum()) + 1,), -1, dtype=torch.int64, device=gpu.dev)
    gpu.eng.set_agg(2, 0)
    bits, cnew, st = gpu.triage(ms, ns, ds, dcs, dcnt, dprio, new_pairs=pairs, want_bits=wb)
    gpu.eng.set_agg(1, 0)
    oms, ons, obits, ocnew = O.triage_batch(m0[0], m0[1], hs, hcs, hcnt, hprio, None)
    print("want_bits", wb, st, flush=True)
    print("  call_new gpu", int(cnew.sum()), "oracle", int(ocnew.sum()), "ms", ms.Len(), oms.Len(), flush=True)
