"""Run only bench.py's Minimize line (BASELINE config 3), for profiling."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from syzkaller_amd.device import Device  # noqa: E402

dev = Device(0)
dev.L.syzsig_ctx_set_timing(dev.eng.h, 1)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
print(json.dumps(bench.minimize_line(dev, n)), flush=True)
