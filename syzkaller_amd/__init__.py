"""syzkaller_amd -- MI355X coverage-signal triage engine for syzkaller.

The product is libsyzsig.so (HIP kernels for gfx950 behind the C ABI in
include/syzsig.h).  This package is its Python host side:
  signal  -- pkg/signal's API (Signal, Serial, FromRaw, Minimize, ...)
  device  -- the batch path over device tensors (triage, edge derivation,
             minimize, shard routing)
  dist    -- hash-sharded maxSignal over one process per GPU
  synth   -- host-side synthetic KCOV workload (same generator as on device)
"""
from ._lib import LIB_PATH, SyzsigError, CorruptedSerial  # noqa: F401

__version__ = "0.1.0"
