"""ctypes wrapper of liboracle.so -- the CPU restatement (oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker / the timed CPU baseline,
never by the product path.  See oracle.h for the parity status.
"""
import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_int8, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")

_L = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


def lib():
    global _L
    if _L is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        P = c_void_p
        sig = {
            "orc_exec_hash": (c_uint32, [c_uint32]),
            "orc_cover_check": (c_int, [c_uint64]),
            "orc_exec_program": (None, [P, P, P, c_uint32, P, P, POINTER(c_uint32)]),
            "orc_sig_new": (P, [c_uint64]),
            "orc_sig_free": (None, [P]),
            "orc_sig_len": (c_uint64, [P]),
            "orc_sig_get": (c_int, [P, c_uint32, POINTER(c_int8)]),
            "orc_from_raw": (P, [P, c_uint64, c_uint8]),
            "orc_serialize": (c_uint64, [P, P, P]),
            "orc_deserialize": (c_int, [P, c_uint64, P, c_uint64, POINTER(c_void_p)]),
            "orc_diff": (P, [P, P]),
            "orc_diff_raw": (P, [P, P, c_uint64, c_uint8]),
            "orc_intersection": (P, [P, P]),
            "orc_merge": (None, [POINTER(c_void_p), P]),
            "orc_minimize": (c_uint64, [P, P, P, c_uint64, P]),
            "orc_triage_batch": (None, [POINTER(c_void_p), POINTER(c_void_p), P, P, P, P, c_uint64, P, P]),
        }
        for k, (r, a) in sig.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _L = L
    return _L


def _p(a):
    return c_void_p(a.ctypes.data) if a.size else c_void_p(0)


class OSig:
    """Oracle Signal (Go map restated); None handle == nil."""

    def __init__(self, h=None):
        self.h = h if h else None

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_sig_free(self.h)
            self.h = None

    @property
    def ptr(self):
        return c_void_p(self.h) if self.h else c_void_p(0)

    def is_nil(self):
        return self.h is None

    def Len(self):
        return int(lib().orc_sig_len(self.ptr))

    def to_dict(self):
        n = self.Len()
        e = np.empty(n, np.uint32)
        p = np.empty(n, np.int8)
        lib().orc_serialize(self.ptr, _p(e), _p(p))
        return {int(a): int(b) for a, b in zip(e, p)}

    def Diff(self, s1):
        return OSig(lib().orc_diff(self.ptr, s1.ptr))

    def DiffRaw(self, raw, prio):
        raw = np.ascontiguousarray(raw, np.uint32)
        return OSig(lib().orc_diff_raw(self.ptr, _p(raw), raw.size, int(prio) & 0xFF))

    def Intersection(self, s1):
        return OSig(lib().orc_intersection(self.ptr, s1.ptr))

    def Merge(self, s1):
        h = c_void_p(self.h or 0)
        lib().orc_merge(ctypes.byref(h), s1.ptr)
        self.h = h.value

    def Serialize(self):
        n = self.Len()
        e = np.empty(n, np.uint32)
        p = np.empty(n, np.int8)
        lib().orc_serialize(self.ptr, _p(e), _p(p))
        return e, p


def from_raw(raw, prio):
    raw = np.ascontiguousarray(raw, np.uint32)
    return OSig(lib().orc_from_raw(_p(raw), raw.size, int(prio) & 0xFF))


def deserialize(elems, prios):
    """Returns OSig, or raises ValueError('corrupted Serial')."""
    e = np.ascontiguousarray(elems, np.uint32)
    p = np.ascontiguousarray(prios, np.int8)
    h = c_void_p()
    if lib().orc_deserialize(_p(e), e.size, _p(p), p.size, ctypes.byref(h)) != 0:
        raise ValueError("corrupted Serial")
    return OSig(h.value)


def exec_program(pcs, call_start, call_len):
    """One program through write_coverage_signal.  Returns (sigs, cnt, completed)."""
    pcs = np.ascontiguousarray(pcs, np.uint64)
    cs = np.ascontiguousarray(call_start, np.uint64)
    cl = np.ascontiguousarray(call_len, np.uint32)
    out = np.zeros(max(pcs.size, 1), np.uint32)
    cnt = np.zeros(cl.size, np.uint32)
    done = c_uint32()
    lib().orc_exec_program(_p(pcs), _p(cs), _p(cl), cl.size, _p(out), _p(cnt), ctypes.byref(done))
    return out[: pcs.size], cnt, int(done.value)


def exec_batch(pcs, call_start, call_len, prog_call):
    """Every program of a batch (calls [prog_call[p], prog_call[p+1])), each with a
    fresh dedup table.  Returns (sigs in pcs indexing, sig_cnt per call, completed per prog)."""
    pcs = np.ascontiguousarray(pcs, np.uint64)
    call_start = np.ascontiguousarray(call_start, np.uint64)
    call_len = np.ascontiguousarray(call_len, np.uint32)
    sigs = np.zeros(pcs.size, np.uint32)
    cnt = np.zeros(call_len.size, np.uint32)
    comp = np.zeros(len(prog_call) - 1, np.uint32)
    L = lib()
    for p in range(len(prog_call) - 1):
        a, b = int(prog_call[p]), int(prog_call[p + 1])
        if a == b:
            continue
        cs = call_start[a:b]
        cnt_p = np.zeros(b - a, np.uint32)
        done = c_uint32()
        # program-local view: starts relative to the global pcs array
        L.orc_exec_program(_p(pcs), _p(np.ascontiguousarray(cs)), _p(np.ascontiguousarray(call_len[a:b])), b - a,
                           _p(sigs), _p(cnt_p), ctypes.byref(done))
        cnt[a:b] = cnt_p
        comp[p] = done.value
    return sigs, cnt, comp


def triage_batch(m0_elems, m0_prios, sigs, call_start, call_len, call_prio, new0=None):
    """Sequential checkNewSignal over a batch.  Returns
    (max_final dict, new_signal dict or None, new_bits u32[], call_new u8[])."""
    ms = deserialize(m0_elems, m0_prios)
    ns = deserialize(*new0) if new0 is not None else OSig()
    sigs = np.ascontiguousarray(sigs, np.uint32)
    cs = np.ascontiguousarray(call_start, np.uint64)
    cl = np.ascontiguousarray(call_len, np.uint32)
    cp = np.ascontiguousarray(call_prio, np.uint8)
    bits = np.zeros((sigs.size + 31) // 32 or 1, np.uint32)
    cnew = np.zeros(max(cl.size, 1), np.uint8)
    mh, nh = c_void_p(ms.h or 0), c_void_p(ns.h or 0)
    lib().orc_triage_batch(ctypes.byref(mh), ctypes.byref(nh), _p(sigs), _p(cs), _p(cl), _p(cp), cl.size, _p(bits),
                           _p(cnew))
    ms.h, ns.h = mh.value, nh.value
    return ms, ns, bits[: (sigs.size + 31) // 32], cnew[: cl.size]


def minimize(off, elems, prios):
    off = np.ascontiguousarray(off, np.uint64)
    e = np.ascontiguousarray(elems, np.uint32)
    p = np.ascontiguousarray(prios, np.int8)
    n = off.size - 1
    out = np.empty(max(n, 1), np.uint64)
    k = lib().orc_minimize(_p(off), _p(e), _p(p), n, _p(out))
    return [int(x) for x in out[:k]]


def run_reference_executor(programs):
    """Run the REFERENCE executor's signal code (oracle/_ref/ref_harness, built
    from /root/reference by oracle/Makefile) on programs = [[(failed, pcs u64[]), ...], ...].
    Returns per program (completed, [(call_index, errno, sigs u32[]), ...])."""
    import struct

    data = [struct.pack("<I", len(programs))]
    for prog in programs:
        data.append(struct.pack("<I", len(prog)))
        for failed, pcs in prog:
            pcs = np.ascontiguousarray(pcs, np.uint64)
            data.append(struct.pack("<II", int(failed), pcs.size))
            data.append(pcs.tobytes())
    out = subprocess.run([REF_HARNESS], input=b"".join(data), capture_output=True, check=True).stdout
    res, pos = [], 0
    for _ in programs:
        (nw,) = struct.unpack_from("<I", out, pos)
        words = np.frombuffer(out, np.uint32, nw, pos + 4)
        pos += 4 + 4 * nw
        completed = int(words[0])
        calls, q = [], 1
        for _ in range(completed):
            idx, num, err, fault, nsig, ncover, ncomps = (int(x) for x in words[q: q + 7])
            calls.append((idx, err, np.array(words[q + 7: q + 7 + nsig], np.uint32)))
            q += 7 + nsig + ncover
        res.append((completed, calls))
    return res


def triage_batch_into(ms, sigs, call_start, call_len, call_prio, ns=None):
    """orc_triage_batch on an existing maxSignal (the timed CPU baseline)."""
    ns = ns if ns is not None else OSig()
    sigs = np.ascontiguousarray(sigs, np.uint32)
    cs = np.ascontiguousarray(call_start, np.uint64)
    cl = np.ascontiguousarray(call_len, np.uint32)
    cp = np.ascontiguousarray(call_prio, np.uint8)
    bits = np.zeros((sigs.size + 31) // 32 or 1, np.uint32)
    cnew = np.zeros(max(cl.size, 1), np.uint8)
    mh, nh = c_void_p(ms.h or 0), c_void_p(ns.h or 0)
    lib().orc_triage_batch(ctypes.byref(mh), ctypes.byref(nh), _p(sigs), _p(cs), _p(cl), _p(cp), cl.size, _p(bits),
                           _p(cnew))
    ms.h, ns.h = mh.value, nh.value
    return ns, bits, cnew
