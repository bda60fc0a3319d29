"""Host-side synthetic KCOV workload (numpy), produced by libsyzsig's host
generator -- the same code the device generator runs (csrc/common.h), so host
checkers and GPU kernels see identical traces.  Needs no GPU."""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, synth_default

__all__ = ["synth_default", "call_lengths", "traces", "m0", "prog_call_index"]


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


def call_lengths(nprog, calls_per_prog, length, ragged=None, seed=0):
    """Per-call PC counts: fixed `length`, or uniform in [ragged[0], ragged[1]]."""
    n = nprog * calls_per_prog
    if ragged is None:
        return np.full(n, length, dtype=np.uint32)
    rng = np.random.default_rng(seed)
    return rng.integers(ragged[0], ragged[1] + 1, size=n).astype(np.uint32)


def prog_call_index(nprog, calls_per_prog):
    return (np.arange(nprog + 1, dtype=np.uint32) * calls_per_prog).astype(np.uint32)


def traces(cfg, prog_base, nprog, calls_per_prog, call_len):
    """-> pcs u64[sum(call_len)], call_start u64[n], call_prio u8[n]"""
    call_len = np.ascontiguousarray(call_len, dtype=np.uint32)
    call_start = np.zeros(call_len.size, dtype=np.uint64)
    if call_len.size > 1:
        np.cumsum(call_len[:-1], out=call_start[1:])
    total = int(call_len.sum())
    pcs = np.empty(max(total, 1), dtype=np.uint64)  # never NULL: empty calls are legal
    prio = np.empty(call_len.size, dtype=np.uint8)
    check(_lib.lib().syzsig_synth_traces_host(ctypes.byref(cfg), prog_base, nprog, calls_per_prog, _p(call_start),
                                              _p(call_len), _p(pcs), _p(prio)))
    return pcs[:total], call_start, prio


def m0(cfg, known_sys, n):
    elems = np.empty(n, dtype=np.uint32)
    prios = np.empty(n, dtype=np.int8)
    check(_lib.lib().syzsig_synth_m0_host(ctypes.byref(cfg), known_sys, n, _p(elems), _p(prios)))
    return elems, prios


def frame_exec_output(sigs, call_start, sig_cnt, completed, prog_call, call_errno, order_seed=None):
    """Frame per-call signals as executor output regions (executor.h:566-604
    handle_completion records: callIndex, callNum = call index, errno,
    faultInjected = 0, nsig, ncover = 0, ncomps = 0, sig[nsig]) -- the synthetic
    stand-in for a batch of executors' shmem out files.  Program p published
    its first completed[p] calls; order_seed shuffles the record order inside a
    program (calls completing out of order).  Returns (out u32[], prog_off u64[nprog+1])."""
    sigs = np.asarray(sigs, np.uint32)
    rng = np.random.default_rng(order_seed) if order_seed is not None else None
    parts, off = [], [0]
    for p in range(len(prog_call) - 1):
        c0 = int(prog_call[p])
        idx = np.arange(int(completed[p]))
        if rng is not None:
            rng.shuffle(idx)
        words = [np.array([idx.size], np.uint32)]
        for i in idx:
            c = c0 + int(i)
            n, s = int(sig_cnt[c]), int(call_start[c])
            words.append(np.array([i, i, np.uint32(np.int64(call_errno[c]) & 0xFFFFFFFF), 0, n, 0, 0], np.uint32))
            words.append(sigs[s:s + n])
        w = np.concatenate(words)
        parts.append(w)
        off.append(off[-1] + w.size)
    return np.concatenate(parts) if parts else np.empty(0, np.uint32), np.array(off, np.uint64)
