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
            "orc_triage_batch_mt": (c_uint64, [POINTER(c_void_p), POINTER(c_void_p), P, P, P, P, c_uint64, c_uint64,
                                               c_uint32]),
            "orc_filter_keys": (c_uint64, [P, P, c_uint64, P, c_uint64, P, P]),
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
            try:
                lib().orc_sig_free(self.h)
            except TypeError:  # interpreter shutdown: module globals are gone, the process frees everything
                pass
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


def run_reference_executor(programs, raw=False):
    """Run the REFERENCE executor's signal code (oracle/_ref/ref_harness, built
    from /root/reference by oracle/Makefile) on programs = [[(failed, pcs u64[]), ...], ...].
    Returns per program (completed, [(call_index, errno, sigs u32[]), ...]), or with raw=True the program's
    output region words as the executor wrote them (executor.h:566-604)."""
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
        if raw:
            res.append(words.copy())
            continue
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


def triage_batch_mt(ms, sigs, call_start, call_len, call_prio, calls_per_prog, nthreads, ns=None):
    """orc_triage_batch_mt: checkNewSignal as `nthreads` Procs run it under
    signalMu (fuzzer.go:494-511) -- the multi-core CPU baseline.  Returns
    (newSignal, number of calls with new signal)."""
    ns = ns if ns is not None else OSig()
    sigs = np.ascontiguousarray(sigs, np.uint32)
    cs = np.ascontiguousarray(call_start, np.uint64)
    cl = np.ascontiguousarray(call_len, np.uint32)
    cp = np.ascontiguousarray(call_prio, np.uint8)
    mh, nh = c_void_p(ms.h or 0), c_void_p(ns.h or 0)
    n = lib().orc_triage_batch_mt(ctypes.byref(mh), ctypes.byref(nh), _p(sigs), _p(cs), _p(cl), _p(cp),
                                  cl.size // calls_per_prog, calls_per_prog, int(nthreads))
    ms.h, ns.h = mh.value, nh.value
    return ns, int(n)


def filter_keys(elems, prios, keys):
    """The Serial entries (elems, prios) whose element is in keys, input order kept."""
    e = np.ascontiguousarray(elems, np.uint32)
    p = np.ascontiguousarray(prios, np.int8)
    k = np.ascontiguousarray(keys, np.uint32)
    oe = np.empty(max(e.size, 1), np.uint32)
    op = np.empty(max(e.size, 1), np.int8)
    n = lib().orc_filter_keys(_p(e), _p(p), e.size, _p(k), k.size, _p(oe), _p(op))
    return oe[:n].copy(), op[:n].copy()


def poll(max_signal, new_max, fuzzer, serial):
    """syz-manager/manager.go:1027-1052 Manager.Poll restated over oracle sets:
    new_max = list of every fuzzer's newMaxSignal (OSig), `fuzzer` the caller's
    index, serial its a.MaxSignal.  Returns the reply's MaxSignal (elems, prios)
    and updates max_signal / new_max in place."""
    nm = max_signal.Diff(deserialize(*serial))
    if nm.Len():
        max_signal.Merge(nm)
        for i, f1 in enumerate(new_max):
            if i != fuzzer:
                f1.Merge(nm)
    reply = (np.empty(0, np.uint32), np.empty(0, np.int8))
    if new_max[fuzzer].Len():
        reply = new_max[fuzzer].Serialize()
        new_max[fuzzer] = OSig()
    return reply


# ---- pkg/ipc/ipc.go:328-468 readOutCoverage (restated; test infrastructure only) ----
INGEST_OK, INGEST_ENCMD, INGEST_EHEADER, INGEST_EINDEX, INGEST_ECALLNUM, INGEST_EDOUBLE = 0, 1, 2, 3, 4, 5
INGEST_ESIGNAL, INGEST_ECOVER, INGEST_ECOMPS, INGEST_ECOMPTYPE = 6, 7, 8, 9


def read_out_coverage(words, ncalls, call_num=None):
    """One executor output region -> (status, info) with info[i] = (errno, sig_off, sig_len, cov_off, cov_len) or
    None for a call without a record (Errno = -1, Signal = nil; ipc.go:362-365).  Offsets are word indices into
    `words`.  status != 0 names the ipc.go error branch taken (see include/syzsig.h SYZSIG_INGEST_*)."""
    out = [int(x) for x in words]
    pos, n = 0, len(out)
    info = [None] * ncalls
    if n == 0:  # ipc.go:356-359
        return INGEST_ENCMD, info
    ncmd = out[0]
    pos = 1
    for _ in range(ncmd):
        if n - pos < 7:  # ipc.go:378-383
            return INGEST_EHEADER, info
        idx, num, err, _fault, nsig, ncover, ncomps = out[pos:pos + 7]
        pos += 7
        if idx >= ncalls:  # ipc.go:384-388
            return INGEST_EINDEX, info
        if call_num is not None and int(call_num[idx]) != num:  # ipc.go:389-395
            return INGEST_ECALLNUM, info
        if info[idx] is not None:  # ipc.go:396-400
            return INGEST_EDOUBLE, info
        if nsig > n - pos:  # ipc.go:403-407
            return INGEST_ESIGNAL, info
        so = pos
        pos += nsig
        if ncover > n - pos:  # ipc.go:411-415
            return INGEST_ECOVER, info
        info[idx] = (err - (1 << 32) if err >= 1 << 31 else err, so, nsig, pos, ncover)
        pos += ncover
        for _j in range(ncomps):  # ipc.go:420-458
            if pos >= n:
                return INGEST_ECOMPS, info
            typ = out[pos]
            pos += 1
            if typ > (1 | 6):  # compConstMask | compSizeMask
                return INGEST_ECOMPTYPE, info
            w = 4 if (typ & 6) == 6 else 2
            if n - pos < w:
                return INGEST_ECOMPS, info
            pos += w
    return INGEST_OK, info


def signal_prio(errno, any_):
    """syz-fuzzer/fuzzer.go:513-521"""
    return (2 if errno == 0 else 0) | (0 if any_ else 1)


def ingest_batch(regions, ncalls, call_any, call_num=None):
    """readOutCoverage over a batch; regions = list of u32 arrays, ncalls[p] = len(p.Calls).  Returns flat
    (out_words, prog_off, prog_call, call_start, call_len, call_prio, call_errno, status) with the expected
    result: a failed program (status != 0) contributes no signal (syz-fuzzer/proc.go:269-278)."""
    prog_off, prog_call = [0], [0]
    for r, nc in zip(regions, ncalls):
        prog_off.append(prog_off[-1] + len(r))
        prog_call.append(prog_call[-1] + int(nc))
    out = np.concatenate([np.asarray(r, np.uint32) for r in regions]) if regions else np.empty(0, np.uint32)
    nct = prog_call[-1]
    cs = np.zeros(nct, np.uint64)
    cl = np.zeros(nct, np.uint32)
    ce = np.full(nct, -1, np.int32)
    st = np.zeros(len(regions), np.int32)
    for p, r in enumerate(regions):
        c0 = prog_call[p]
        nums = None if call_num is None else call_num[c0:prog_call[p + 1]]
        s, info = read_out_coverage(r, int(ncalls[p]), nums)
        st[p] = s
        for i, inf in enumerate(info):
            cs[c0 + i] = prog_off[p]
            if s == INGEST_OK and inf is not None:
                ce[c0 + i] = inf[0]
                cs[c0 + i] = prog_off[p] + inf[1]
                cl[c0 + i] = inf[2]
    cp = np.array([signal_prio(int(e), int(a)) for e, a in zip(ce, call_any)], np.uint8)
    return (out, np.array(prog_off, np.uint64), np.array(prog_call, np.uint32), cs, cl, cp, ce, st)


class OCover:
    """pkg/cover/cover.go:7-30 restated: Cover = map[uint32]struct{} (None = nil map)."""

    def __init__(self):
        self.c = None

    def Merge(self, raw):  # cover.go:9-18
        if self.c is None:
            self.c = set()
        self.c.update(int(x) for x in np.asarray(raw, np.uint32))

    def Serialize(self):  # cover.go:20-26
        return sorted(self.c or ())


def triage_runs(item_off, elems, prios, item_flags, runs, run_off, run_sigs, run_prio, run_errno, run_exec):
    """syz-fuzzer/proc.go:107-140 restated per item with the oracle Signal ops.  Returns (item_keep u8[],
    final newSignal per item as a dict elem -> prio, or None if dropped)."""
    keep, finals = [], []
    for i in range(len(item_off) - 1):
        a, b = int(item_off[i]), int(item_off[i + 1])
        ns = deserialize(elems[a:b], prios[a:b])
        minimized, orig_ok = bool(item_flags[i] & 1), bool(item_flags[i] & 2)
        ok = ns.Len() > 0  # proc.go:109-111
        notexec = 0
        for r in range(runs):
            if not ok:
                break
            rr = i * runs + r
            ra, rb = int(run_off[rr]), int(run_off[rr + 1])
            if not run_exec[rr] or rb == ra or (orig_ok and run_errno[rr] != 0):  # proc.go:122-128
                notexec += 1
                if notexec > runs // 2 + 1:
                    ok = False
                continue
            ns = ns.Intersection(from_raw(run_sigs[ra:rb], int(run_prio[rr])))  # proc.go:131-132
            if ns.Len() == 0 and not minimized:  # proc.go:133-137
                ok = False
        keep.append(int(ok))
        finals.append(ns.to_dict() if ok else None)
    return np.array(keep, np.uint8), finals


def minimize_pred(item_off, elems, prios, item_flags, attempts, run_off, run_sigs, run_prio, run_errno, run_exec):
    """The prog.Minimize predicate of syz-fuzzer/proc.go:141-160, restated per item."""
    out = []
    for i in range(len(item_off) - 1):
        a, b = int(item_off[i]), int(item_off[i + 1])
        ns = deserialize(elems[a:b], prios[a:b])
        orig_ok = bool(item_flags[i] & 2)
        res = 0
        for r in range(attempts):
            rr = i * attempts + r
            ra, rb = int(run_off[rr]), int(run_off[rr + 1])
            if not run_exec[rr] or rb == ra:  # proc.go:146-148
                continue
            if orig_ok and run_errno[rr] != 0:  # proc.go:150-154
                break
            this = from_raw(run_sigs[ra:rb], int(run_prio[rr]))
            if ns.Intersection(this).Len() == ns.Len():  # proc.go:155-159
                res = 1
                break
        out.append(res)
    return np.array(out, np.uint8)
