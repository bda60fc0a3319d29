"""pkg/signal's API over the MI355X engine.

Mirrors pkg/signal/signal.go (the whole package, :11-166) so code written
against the reference reads the same:

    s := signal.FromRaw(raw, prio)          s = FromRaw(raw, prio)
    d := max.DiffRaw(raw, prio)             d = max_.DiffRaw(raw, prio)
    max.Merge(d)                            max_.Merge(d)
    ser := s.Serialize(); ser.Deserialize() ser = s.Serialize(); ser.Deserialize()
    signal.Minimize(corpus)                 Minimize(corpus)

Every Signal lives in HBM as a libsyzsig table; ``Signal()`` is Go's nil
Signal (Len 0, valid receiver, allocated by Merge).  Host arrays are numpy.
"""
import ctypes
import threading

import numpy as np

from . import _lib
from ._lib import check

__all__ = ["Engine", "engine", "Signal", "Cover", "Serial", "Context", "FromRaw", "Minimize", "signal_prio",
           "check_new_signal", "manager_poll"]


class Engine:
    """One libsyzsig context (device + stream) per process and GPU."""

    def __init__(self, device=0):
        self.L = _lib.lib()
        h = ctypes.c_void_p()
        check(self.L.syzsig_ctx_create(int(device), ctypes.byref(h)))
        self.h = h
        self.device = int(device)
        self._pin, self._pin_bytes = None, 0  # page-locked staging (syzsig_host_alloc)

    def staging(self, nbytes):
        """A page-locked host buffer of at least nbytes (uint8 numpy view),
        reused across calls: arrays built in it upload by DMA.  Its contents
        are the caller's until the next staging() call."""
        if nbytes > self._pin_bytes:
            self._free_staging()
            want = max(int(nbytes), 2 * self._pin_bytes, 1 << 20)
            p = ctypes.c_void_p()
            check(self.L.syzsig_host_alloc(self.h, want, ctypes.byref(p)))
            self._pin, self._pin_bytes = p, want
        return np.ctypeslib.as_array(ctypes.cast(self._pin, ctypes.POINTER(ctypes.c_uint8)), shape=(self._pin_bytes,))

    def _free_staging(self):
        if self._pin is not None and self.h:
            self.L.syzsig_host_free(self.h, self._pin)
        self._pin, self._pin_bytes = None, 0

    def set_stream(self, stream_handle):
        check(self.L.syzsig_ctx_set_stream(self.h, ctypes.c_void_p(stream_handle)))

    def set_agg(self, mode=1, parts=0):
        """Large-batch triage path: 0 per-call, 1 auto (default), 2 aggregation always."""
        check(self.L.syzsig_ctx_set_agg(self.h, int(mode), int(parts)))

    def set_debug(self, flags):
        """Result-preserving code-path knobs (include/syzsig.h SYZSIG_DEBUG_*), for tests."""
        check(self.L.syzsig_ctx_set_debug(self.h, int(flags)))

    def close(self):
        if self.h:
            self._free_staging()
            self.L.syzsig_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_engines = {}
_engines_lock = threading.Lock()


def engine(device=0):
    with _engines_lock:
        e = _engines.get(device)
        if e is None:
            e = _engines[device] = Engine(device)
        return e


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else ctypes.c_void_p(0)


class Signal:
    """type Signal map[elemType]prioType (signal.go:17), device-resident."""

    __slots__ = ("_h", "_e")

    def __init__(self, handle=None, eng=None):
        self._h = handle if (handle is not None and handle.value) else None
        self._e = eng or engine()

    # -- ownership
    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        # at interpreter shutdown the engine may be finalized first (cycles from
        # tracebacks): its context -- and every set's memory with it -- is gone then
        if h is not None and getattr(getattr(self, "_e", None), "h", None):
            try:
                self._e.L.syzsig_set_free(h)
            except Exception:
                pass

    @property
    def handle(self):
        return self._h if self._h is not None else ctypes.c_void_p(0)

    def is_nil(self):
        return self._h is None

    @classmethod
    def make(cls, hint=0, eng=None):
        """make(Signal, hint)"""
        eng = eng or engine()
        h = ctypes.c_void_p()
        check(eng.L.syzsig_set_make(eng.h, int(hint), ctypes.byref(h)))
        return cls(h, eng)

    def _wrap(self, h):
        return Signal(h, self._e)

    # -- signal.go:23-29
    def Len(self):
        return int(self._e.L.syzsig_len(self.handle))

    def Empty(self):
        return self.Len() == 0

    def __len__(self):
        return self.Len()

    def capacity(self):
        return int(self._e.L.syzsig_capacity(self.handle))

    # -- signal.go:42-57
    def Serialize(self):
        n = self.Len()
        if n == 0:
            return Serial()
        elems = np.empty(n, dtype=np.uint32)
        prios = np.empty(n, dtype=np.int8)
        out = ctypes.c_uint64()
        check(self._e.L.syzsig_serialize(self._e.h, self.handle, _ptr(elems), _ptr(prios), n, ctypes.byref(out)))
        return Serial(elems, prios)

    # -- signal.go:73-88
    def Diff(self, s1):
        h = ctypes.c_void_p()
        check(self._e.L.syzsig_diff(self._e.h, self.handle, s1.handle, ctypes.byref(h)))
        return self._wrap(h)

    # -- signal.go:90-102
    def DiffRaw(self, raw, prio):
        raw = np.ascontiguousarray(raw, dtype=np.uint32)
        h = ctypes.c_void_p()
        check(self._e.L.syzsig_diff_raw(self._e.h, self.handle, _ptr(raw), raw.size, int(prio) & 0xFF,
                                        ctypes.byref(h)))
        return self._wrap(h)

    # -- signal.go:104-115
    def Intersection(self, s1):
        h = ctypes.c_void_p()
        check(self._e.L.syzsig_intersection(self._e.h, self.handle, s1.handle, ctypes.byref(h)))
        return self._wrap(h)

    # -- signal.go:117-131 (pointer receiver: allocates a nil receiver)
    def Merge(self, s1):
        h = ctypes.c_void_p(self._h.value if self._h is not None else 0)
        check(self._e.L.syzsig_merge(self._e.h, ctypes.byref(h), s1.handle))
        if h.value and self._h is None:
            self._h = h

    # -- helpers for tests / tools
    def to_dict(self):
        ser = self.Serialize()
        return {int(e): int(p) for e, p in zip(ser.Elems, ser.Prios)}

    def clear(self):
        if self._h is not None:
            check(self._e.L.syzsig_set_clear(self._e.h, self._h))

    def clone(self):
        h = ctypes.c_void_p()
        check(self._e.L.syzsig_set_clone(self._e.h, self.handle, ctypes.byref(h)))
        return self._wrap(h)

    def copy_from(self, src):
        check(self._e.L.syzsig_set_copy_from(self._e.h, self.handle, src.handle))

    def restore_keys(self, src, keys):
        """Back to the snapshot src this set was copied from, copying only the
        slots of the elements in `keys` (every element changed since: the
        newSignal of the batches since, if it was empty at the snapshot)."""
        check(self._e.L.syzsig_set_restore_keys(self._e.h, self.handle, src.handle, keys.handle))

    def reserve(self, extra):
        """Room for `extra` more elements (syzsig_set_reserve)."""
        check(self._e.L.syzsig_set_reserve(self._e.h, self.handle, int(extra)))

    def equal(self, other):
        """Same capacity, length and slot words (a snapshot check)."""
        eq = ctypes.c_int(0)
        check(self._e.L.syzsig_set_equal(self._e.h, self.handle, other.handle, ctypes.byref(eq)))
        return bool(eq.value)


class Cover:
    """type Cover map[uint32]struct{} (pkg/cover/cover.go:7), device-resident;
    the zero value is nil, as in Go."""

    __slots__ = ("_s",)

    def __init__(self, eng=None):
        self._s = Signal(None, eng)

    def is_nil(self):
        return self._s.is_nil()

    def Merge(self, raw):
        """cover.go:9-18 (allocates a nil receiver, even for an empty raw)."""
        raw = np.ascontiguousarray(raw, dtype=np.uint32)
        e = self._s._e
        h = ctypes.c_void_p(self._s.handle.value or 0)
        check(e.L.syzsig_cover_merge(e.h, ctypes.byref(h), _ptr(raw), raw.size))
        if self._s.is_nil() and h.value:
            self._s._h = h

    def Serialize(self):
        """cover.go:20-26: the PCs in unspecified order."""
        return self._s.Serialize().Elems if not self._s.is_nil() else np.empty(0, np.uint32)

    def __len__(self):
        return self._s.Len()


class Serial:
    """type Serial struct{Elems []elemType; Prios []prioType} (signal.go:19-22)."""

    __slots__ = ("Elems", "Prios")

    def __init__(self, elems=None, prios=None):
        self.Elems = np.asarray(elems if elems is not None else [], dtype=np.uint32)
        self.Prios = np.asarray(prios if prios is not None else [], dtype=np.int8)

    def Deserialize(self, eng=None):
        """signal.go:59-71; raises CorruptedSerial on a length mismatch."""
        eng = eng or engine()
        e = np.ascontiguousarray(self.Elems, dtype=np.uint32)
        p = np.ascontiguousarray(self.Prios, dtype=np.int8)
        h = ctypes.c_void_p()
        check(eng.L.syzsig_deserialize(eng.h, _ptr(e), e.size, _ptr(p), p.size, ctypes.byref(h)))
        return Signal(h, eng)


def serialize_many(sets, eng=None):
    """Serialize (signal.go:42-57) of every set in `sets` (Signal objects; a
    nil one is empty) with one library call (syzsig_serialize_batch): the
    manager serializes every Poll reply (manager.go:1049).  Returns a Serial
    per set; their arrays are views of one buffer."""
    n = len(sets)
    if n == 0:
        return []
    eng = eng or next((x._e for x in sets if x is not None), None) or engine()
    hs = (ctypes.c_void_p * n)(*[(x.handle.value or 0) if x is not None else 0 for x in sets])
    offs = np.zeros(n + 1, dtype=np.uint64)
    check(eng.L.syzsig_serialize_batch(eng.h, hs, n, None, None, 0, _ptr(offs)))
    tot = int(offs[-1])
    if tot == 0:
        return [Serial() for _ in range(n)]
    elems = np.empty(tot, dtype=np.uint32)
    prios = np.empty(tot, dtype=np.int8)
    check(eng.L.syzsig_serialize_batch(eng.h, hs, n, _ptr(elems), _ptr(prios), tot, _ptr(offs)))
    return [Serial(elems[a:b], prios[a:b]) for a, b in zip(offs[:-1].tolist(), offs[1:].tolist())]


def FromRaw(raw, prio, eng=None):
    """signal.go:31-40"""
    eng = eng or engine()
    raw = np.ascontiguousarray(raw, dtype=np.uint32)
    h = ctypes.c_void_p()
    check(eng.L.syzsig_from_raw(eng.h, _ptr(raw), raw.size, int(prio) & 0xFF, ctypes.byref(h)))
    return Signal(h, eng)


class Context:
    """type Context struct{Signal Signal; Context interface{}} (signal.go:133-136)."""

    __slots__ = ("Signal", "Context")

    def __init__(self, signal, context):
        self.Signal = signal
        self.Context = context


def Minimize(corpus, eng=None, hint_distinct=0):
    """signal.go:138-166.  Like sort.Slice in the reference, reorders `corpus`
    in place (Len desc; ties keep input order) and returns the surviving
    contexts' Context values (in sorted order)."""
    eng = eng or engine()
    n = len(corpus)
    if n == 0:
        return []
    sers = [c.Signal.Serialize() for c in corpus]
    lens = np.array([s.Elems.size for s in sers], dtype=np.uint64)
    off = np.zeros(n + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    elems = np.concatenate([s.Elems for s in sers]) if off[-1] else np.empty(0, np.uint32)
    prios = np.concatenate([s.Prios for s in sers]) if off[-1] else np.empty(0, np.int8)
    out_idx = np.empty(n, dtype=np.uint64)
    cnt = ctypes.c_uint64()
    check(eng.L.syzsig_minimize(eng.h, _ptr(off), _ptr(elems), _ptr(prios), n, int(hint_distinct),
                                _ptr(out_idx), ctypes.byref(cnt)))
    keep = set(int(i) for i in out_idx[: cnt.value])
    order = sorted(range(n), key=lambda i: (-int(lens[i]), i))
    corpus[:] = [corpus[i] for i in order]
    return [corpus[r].Context for r, i in enumerate(order) if i in keep]


def signal_prio(errno, contains_any):
    """syz-fuzzer/fuzzer.go:513-521 signalPrio."""
    prio = 0
    if errno == 0:
        prio |= 1 << 1
    if not contains_any:
        prio |= 1 << 0
    return prio


def check_new_signal(max_signal, new_signal, calls, eng=None, want_bits=False):
    """syz-fuzzer/fuzzer.go:494-511 checkNewSignal for one program.

    calls: sequence of (raw signal u32[], prio) in call-index order (the
    CallInfo.Signal slices and their signalPrio).  Merges into max_signal and
    new_signal (nil ones are allocated, as Merge does) and returns the indices
    of calls with new signal; with want_bits also the per-record new bitmap."""
    eng = eng or max_signal._e
    raws = [np.ascontiguousarray(r, dtype=np.uint32) for r, _ in calls]
    lens = np.array([r.size for r in raws], dtype=np.uint32)
    starts = np.zeros(len(raws), dtype=np.uint64)
    if len(raws) > 1:
        np.cumsum(lens[:-1], out=starts[1:])
    sigs = np.concatenate(raws) if raws and lens.sum() else np.empty(0, np.uint32)
    prios = np.array([int(p) & 0xFF for _, p in calls], dtype=np.uint8)
    out = np.empty(max(len(raws), 1), dtype=np.uint32)
    n = ctypes.c_uint32()
    bits = np.zeros(max((sigs.size + 31) // 32, 1), dtype=np.uint32)
    mh = ctypes.c_void_p(max_signal.handle.value or 0)
    nh = ctypes.c_void_p(new_signal.handle.value or 0)
    check(eng.L.syzsig_check_new_signal(eng.h, ctypes.byref(mh), ctypes.byref(nh), _ptr(sigs), sigs.size,
                                        _ptr(starts), _ptr(lens), _ptr(prios), len(raws), _ptr(out),
                                        ctypes.byref(n), _ptr(bits) if want_bits else ctypes.c_void_p(0)))
    if mh.value and max_signal.is_nil():
        max_signal._h = mh
    if nh.value and new_signal.is_nil():
        new_signal._h = nh
    idx = [int(i) for i in out[: n.value]]
    return (idx, bits[: (sigs.size + 31) // 32]) if want_bits else idx


# limits of one syzsig_manager_poll_batch call (csrc/poll.hip kPollMax*)
POLL_MAX_TARGETS = (1 << 24) - 2
POLL_MAX_NEXT = 1 << 28
POLL_MAX_FANOUT = 1 << 31
POLL_MAX_ENTRIES = 1 << 23  # past it one call takes the sequential loop (csrc/poll.hip kPollMaxEntries)


def manager_poll(max_signal, new_max, polls, eng=None):
    """syz-manager/manager.go:1027-1052 Manager.Poll for a batch of polls, in
    order: polls = [(fuzzer index, Serial a.MaxSignal)], new_max = every
    fuzzer's newMaxSignal (Signal objects, updated in place; a polling
    fuzzer's becomes nil).  max_signal is merged (a nil one is allocated).
    Returns each poll's reply r.MaxSignal as a Serial (empty if none)."""
    eng = eng or max_signal._e
    F, K = len(new_max), len(polls)
    lens = [np.asarray(s.Elems).size for _, s in polls]
    # one library call holds at most POLL_MAX_NEXT polls x fuzzers and
    # POLL_MAX_FANOUT entries x fuzzers (include/syzsig.h): a larger batch is
    # applied as consecutive sub-batches, which is the same sequential loop
    cuts, k0, n_acc = [], 0, 0
    for k in range(K):
        if k > k0 and ((k + 1 - k0) * F > POLL_MAX_NEXT or (n_acc + lens[k]) * F > POLL_MAX_FANOUT
                       or (k + 1 - k0) + F > POLL_MAX_TARGETS or n_acc + lens[k] > POLL_MAX_ENTRIES):
            cuts.append((k0, k))
            k0, n_acc = k, 0
        n_acc += lens[k]
    if cuts:
        out = []
        for a, z in cuts + [(k0, K)]:
            out += manager_poll(max_signal, new_max, polls[a:z], eng)
        return out
    pf = np.array([int(f) for f, _ in polls], dtype=np.uint32)
    lens = np.array([np.asarray(s.Elems).size for _, s in polls], dtype=np.uint64)
    for _, s in polls:
        if np.asarray(s.Elems).size != np.asarray(s.Prios).size:
            raise _lib.CorruptedSerial(_lib.SYZSIG_ECORRUPT, "corrupted Serial")  # signal.go:60-62
    off = np.zeros(K + 1, dtype=np.uint64)
    np.cumsum(lens, out=off[1:])
    # the Serials back to back in page-locked memory (the upload is a DMA)
    n = int(off[-1])
    if n:
        buf = eng.staging(5 * n + 64)
        elems = buf[: 4 * n].view(np.uint32)
        prios = buf[4 * n: 5 * n].view(np.int8)
        np.concatenate([np.asarray(s.Elems, np.uint32) for _, s in polls], out=elems)
        np.concatenate([np.asarray(s.Prios, np.int8) for _, s in polls], out=prios)
    else:
        elems, prios = np.empty(0, np.uint32), np.empty(0, np.int8)
    nm = (ctypes.c_void_p * max(F, 1))(*[s.handle.value or 0 for s in new_max])
    rep = (ctypes.c_void_p * max(K, 1))()
    mh = ctypes.c_void_p(max_signal.handle.value or 0)
    try:
        check(eng.L.syzsig_manager_poll_batch(eng.h, ctypes.byref(mh), nm, F, _ptr(pf), _ptr(off), _ptr(elems),
                                              _ptr(prios), K, rep))
    finally:
        # the library replaces the polled fuzzers' sets only on success, and
        # leaves every handle as it was on an error: mirror nm[] either way
        if mh.value and max_signal.is_nil():
            max_signal._h = mh
        for g, s in enumerate(new_max):
            s._h = ctypes.c_void_p(nm[g]) if nm[g] else None
    reps = [Signal(ctypes.c_void_p(rep[i]) if rep[i] else None, eng) for i in range(K)]
    return serialize_many(reps, eng)
