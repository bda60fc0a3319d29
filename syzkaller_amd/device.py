"""Batch (device-resident) API of the engine over torch tensors.

torch is plumbing here: it owns HBM buffers and the stream; every computation
runs in libsyzsig's HIP kernels.  All tensors must live on this Device's GPU.
"""
import ctypes

import torch

from . import _lib
from ._lib import Batch, BatchStats, StepStatus, check
from .signal import Signal, engine

__all__ = ["Device", "call_layout"]


def _p(t):
    return ctypes.c_void_p(t.data_ptr() if (t is not None and t.numel()) else 0)


def call_layout(call_len, device=None):
    """Exclusive prefix sum of per-call lengths -> call_start (u64 as int64)."""
    call_len = torch.as_tensor(call_len, device=device)
    start = torch.zeros(call_len.numel(), dtype=torch.int64, device=call_len.device)
    if call_len.numel() > 1:
        start[1:] = torch.cumsum(call_len[:-1].to(torch.int64), 0)
    return start


class Device:
    def __init__(self, device=0):
        if not torch.cuda.is_available():
            raise RuntimeError("syzkaller_amd.device needs a ROCm GPU (no CPU fallback)")
        self.index = int(device)
        self.dev = torch.device("cuda", self.index)
        self.eng = engine(self.index)
        self.sync_stream()

    def sync_stream(self):
        """Run library work on torch's current stream of this device.  torch's
        default stream is HIP's null stream (handle 0); the library's own
        stream (selected by 0) is a blocking stream, ordered against the null
        stream both ways, so inputs torch (or a synchronous RCCL collective)
        produced there are complete when a library kernel reads them."""
        self.eng.set_stream(torch.cuda.current_stream(self.dev).cuda_stream)

    @property
    def L(self):
        return self.eng.L

    def _check_dev(self, *ts):
        for t in ts:
            if t is not None and t.device != self.dev:
                raise ValueError(f"tensor on {t.device}, expected {self.dev}")
            if t is not None and not t.is_contiguous():
                raise ValueError("tensors must be contiguous")

    def copy_bw(self, dst, src, nbytes):
        """Device time (ms) of a plain 16-B-per-lane copy of nbytes from src to
        dst (syzsig_copy_bw_dev): the achievable-bandwidth companion of the
        bench's rooflines."""
        self._check_dev(dst, src)
        if nbytes > min(dst.numel() * dst.element_size(), src.numel() * src.element_size()):
            raise ValueError("copy_bw: nbytes exceeds a buffer")
        ms = ctypes.c_double()
        check(self.L.syzsig_copy_bw_dev(self.eng.h, _p(dst), _p(src), int(nbytes), ctypes.byref(ms)))
        return ms.value

    # ---------------------------------------------------------------- sets
    def new_set(self, hint=0):
        return Signal.make(hint, self.eng)

    def deserialize(self, elems, prios):
        self._check_dev(elems, prios)
        assert elems.dtype == torch.int32 or elems.dtype == torch.uint32
        h = ctypes.c_void_p()
        check(self.L.syzsig_deserialize_dev(self.eng.h, _p(elems), _p(prios), elems.numel(), ctypes.byref(h)))
        return Signal(h, self.eng)

    # ---------------------------------------------------------------- K3
    def batch(self, sigs, call_start, call_len, call_prio, new_bits=None, call_new=None, new_pairs=None,
              want_bits=True):
        """A syzsig_batch over device tensors.  new_bits is allocated when
        want_bits (else NULL: not computed); new_pairs (int64) is optional."""
        self._check_dev(sigs, call_start, call_len, call_prio, new_bits, call_new, new_pairs)
        nrec, ncalls = sigs.numel(), call_len.numel()
        if new_bits is None and want_bits:
            new_bits = torch.empty((nrec + 31) // 32, dtype=torch.int32, device=self.dev)
        if call_new is None:
            call_new = torch.empty(ncalls, dtype=torch.uint8, device=self.dev)
        b = Batch(sigs=_p(sigs).value, call_start=_p(call_start).value, call_len=_p(call_len).value,
                  call_prio=_p(call_prio).value, ncalls=ncalls, nrec=nrec, new_bits=_p(new_bits).value,
                  call_new=_p(call_new).value, new_pairs=_p(new_pairs).value,
                  new_pairs_cap=0 if new_pairs is None else new_pairs.numel())
        return b, new_bits, call_new

    def triage(self, max_signal, new_signal, sigs, call_start, call_len, call_prio, new_bits=None, call_new=None,
               new_pairs=None, want_bits=True):
        """checkNewSignal over a whole batch (syz-fuzzer/fuzzer.go:494-511).
        Returns (new_bits int32[ceil(nrec/32)] or None, call_new uint8[ncalls], stats);
        stats["new_pairs"] = number of (call << 32 | elem) DiffRaw entries, the
        first min(that, new_pairs.numel()) of which are written to new_pairs."""
        b, new_bits, call_new = self.batch(sigs, call_start, call_len, call_prio, new_bits, call_new, new_pairs,
                                           want_bits)
        return new_bits, call_new, self.triage_b(max_signal, new_signal, b)

    def triage_b(self, max_signal, new_signal, b):
        """syzsig_triage_batch on a prepared Batch; returns the stats dict."""
        st = BatchStats()
        nh = ctypes.c_void_p(new_signal.handle.value or 0)
        check(self.L.syzsig_triage_batch(self.eng.h, max_signal.handle, ctypes.byref(nh), ctypes.byref(b),
                                         ctypes.byref(st)))
        if nh.value and new_signal.is_nil():
            new_signal._h = nh
        return st.as_dict()

    # ---------------------------------------------------------------- K1+K2
    def edge_derive(self, pcs, call_start, call_len, prog_call, sigs=None, sig_cnt=None, completed=None):
        """executor write_coverage_signal for every program of a batch."""
        self._check_dev(pcs, call_start, call_len, prog_call, sigs, sig_cnt, completed)
        nprog = prog_call.numel() - 1
        if sigs is None:
            sigs = torch.empty(pcs.numel(), dtype=torch.int32, device=self.dev)
        if sig_cnt is None:
            sig_cnt = torch.empty(call_len.numel(), dtype=torch.int32, device=self.dev)
        if completed is None:
            completed = torch.empty(max(nprog, 0), dtype=torch.int32, device=self.dev)
        check(self.L.syzsig_edge_derive_dev(self.eng.h, _p(pcs), pcs.numel(), _p(call_start), _p(call_len),
                                            call_len.numel(), _p(prog_call), max(nprog, 0), _p(sigs), _p(sig_cnt),
                                            _p(completed)))
        return sigs, sig_cnt, completed

    # ---------------------------------------------------------------- executor output ingest
    def ingest_exec_output(self, out, prog_off, prog_call, call_any, call_num=None, want_cover=False):
        """pkg/ipc/ipc.go:328-468 readOutCoverage over a batch of executor output
        regions (program p's at out[prog_off[p]:prog_off[p+1]]).  Returns a dict of
        device tensors call_start (int64), call_len (int32), call_prio (uint8),
        call_errno (int32), prog_status (int32), cover_start/cover_len (if
        want_cover), and n_failed.  call_start/len index `out`, so
        triage(max, new, out, call_start, call_len, call_prio) runs checkNewSignal
        on the batch without copying the signal."""
        self._check_dev(out, prog_off, prog_call, call_any, call_num)
        nprog, ncalls = prog_off.numel() - 1, call_any.numel()
        if prog_call.numel() != prog_off.numel():
            raise ValueError("prog_call and prog_off need nprog + 1 entries")
        if call_num is not None and call_num.numel() != ncalls:
            raise ValueError("call_num needs one entry per call")
        r = {"call_start": torch.empty(ncalls, dtype=torch.int64, device=self.dev),
             "call_len": torch.empty(ncalls, dtype=torch.int32, device=self.dev),
             "call_prio": torch.empty(ncalls, dtype=torch.uint8, device=self.dev),
             "call_errno": torch.empty(ncalls, dtype=torch.int32, device=self.dev),
             "prog_status": torch.empty(max(nprog, 0), dtype=torch.int32, device=self.dev)}
        if want_cover:
            r["cover_start"] = torch.empty(ncalls, dtype=torch.int64, device=self.dev)
            r["cover_len"] = torch.empty(ncalls, dtype=torch.int32, device=self.dev)
        nf = ctypes.c_uint64()
        check(self.L.syzsig_ingest_exec_output_dev(
            self.eng.h, _p(out), out.numel(), _p(prog_off), max(nprog, 0), _p(prog_call), ncalls, _p(call_num),
            _p(call_any), _p(r["call_start"]), _p(r["call_len"]), _p(r["call_prio"]), _p(r["call_errno"]),
            _p(r.get("cover_start")), _p(r.get("cover_len")), _p(r["prog_status"]), ctypes.byref(nf)))
        r["n_failed"] = int(nf.value)
        return r

    # ---------------------------------------------------------------- triageInput re-runs
    def triage_runs(self, item_off, elems, prios, item_flags, runs, run_off, run_sigs, run_prio, run_errno,
                    run_exec):
        """syz-fuzzer/proc.go:107-140 over a batch of triage items (see
        include/syzsig.h syzsig_triage_runs_dev).  Returns (item_keep, elem_keep)
        as uint8 device tensors."""
        self._check_dev(item_off, elems, prios, item_flags, run_off, run_sigs, run_prio, run_errno, run_exec)
        nitems = item_off.numel() - 1
        if run_off.numel() != nitems * runs + 1 and nitems > 0:
            raise ValueError("run_off needs nitems * runs + 1 entries")
        item_keep = torch.empty(max(nitems, 0), dtype=torch.uint8, device=self.dev)
        elem_keep = torch.empty(elems.numel(), dtype=torch.uint8, device=self.dev)
        check(self.L.syzsig_triage_runs_dev(self.eng.h, _p(item_off), max(nitems, 0), _p(elems), _p(prios),
                                            _p(item_flags), int(runs), _p(run_off), _p(run_sigs), _p(run_prio),
                                            _p(run_errno), _p(run_exec), _p(item_keep), _p(elem_keep)))
        return item_keep, elem_keep

    def minimize_pred(self, item_off, elems, prios, item_flags, attempts, run_off, run_sigs, run_prio, run_errno,
                      run_exec):
        """triageInput's minimize predicate (proc.go:141-160) per item; uint8 tensor."""
        self._check_dev(item_off, elems, prios, item_flags, run_off, run_sigs, run_prio, run_errno, run_exec)
        nitems = item_off.numel() - 1
        if run_off.numel() != nitems * attempts + 1 and nitems > 0:
            raise ValueError("run_off needs nitems * attempts + 1 entries")
        pred = torch.empty(max(nitems, 0), dtype=torch.uint8, device=self.dev)
        check(self.L.syzsig_minimize_pred_dev(self.eng.h, _p(item_off), max(nitems, 0), _p(elems), _p(prios),
                                              _p(item_flags), int(attempts), _p(run_off), _p(run_sigs),
                                              _p(run_prio), _p(run_errno), _p(run_exec), _p(pred)))
        return pred

    # ---------------------------------------------------------------- K5
    def minimize(self, ctx_off, elems, prios, hint_distinct=0):
        self._check_dev(ctx_off, elems, prios)
        n = ctx_off.numel() - 1
        keep = torch.empty(max(n, 0), dtype=torch.uint8, device=self.dev)
        cnt = ctypes.c_uint64()
        check(self.L.syzsig_minimize_dev(self.eng.h, _p(ctx_off), _p(elems), _p(prios), max(n, 0),
                                         int(hint_distinct), _p(keep), ctypes.byref(cnt)))
        return keep, int(cnt.value)

    def minimize_shard(self, ctx_off, elems, prios, nshards, shard, hint_distinct=0):
        """Minimize over the elements this shard owns (owner_of); OR the keep
        arrays of all shards for the corpus result (see dist.sharded_minimize)."""
        self._check_dev(ctx_off, elems, prios)
        n = ctx_off.numel() - 1
        keep = torch.empty(max(n, 0), dtype=torch.uint8, device=self.dev)
        cnt = ctypes.c_uint64()
        check(self.L.syzsig_minimize_shard_dev(self.eng.h, _p(ctx_off), _p(elems), _p(prios), max(n, 0),
                                               int(nshards), int(shard), int(hint_distinct), _p(keep),
                                               ctypes.byref(cnt)))
        return keep, int(cnt.value)

    def minimize_split(self, ctx_off, elems, prios, nparts, part, nshards, hint_distinct=0, send=None):
        """Data-split Minimize, source side (syzsig_minimize_split_dev): this
        part's contexts aggregated, one winner record per distinct element,
        grouped by owner.  -> (send int64[sum(counts)], counts)."""
        self._check_dev(ctx_off, elems, prios, send)
        n = ctx_off.numel() - 1
        if send is None:
            send = torch.empty(max(elems.numel(), 1), dtype=torch.int64, device=self.dev)
        counts = (ctypes.c_uint64 * nshards)()
        check(self.L.syzsig_minimize_split_dev(self.eng.h, _p(ctx_off), _p(elems), _p(prios), max(n, 0), int(nparts),
                                               int(part), int(nshards), int(hint_distinct), _p(send), send.numel(),
                                               counts))
        counts = [int(c) for c in counts]
        return send[: sum(counts)], counts

    def minimize_resolve(self, ctx_off, recs):
        """Data-split Minimize, owner side (syzsig_minimize_resolve_dev): the
        winner records sent to this owner -> keep uint8[nctx]."""
        self._check_dev(ctx_off, recs)
        n = ctx_off.numel() - 1
        keep = torch.empty(max(n, 0), dtype=torch.uint8, device=self.dev)
        cnt = ctypes.c_uint64()
        check(self.L.syzsig_minimize_resolve_dev(self.eng.h, _p(ctx_off), max(n, 0), _p(recs), recs.numel(),
                                                 _p(keep), ctypes.byref(cnt)))
        return keep, int(cnt.value)

    # ---------------------------------------------------------------- sharding (records mode: the owner side)
    def triage_records(self, shard, new_signal, recs, levels, new_flags):
        self._check_dev(recs, new_flags)
        lv = (ctypes.c_int8 * len(levels))(*levels)
        st = BatchStats()
        nh = ctypes.c_void_p(new_signal.handle.value or 0)
        check(self.L.syzsig_triage_records_dev(self.eng.h, shard.handle, ctypes.byref(nh), _p(recs), recs.numel(),
                                               lv, len(levels), _p(new_flags), ctypes.byref(st)))
        if nh.value and new_signal.is_nil():
            new_signal._h = nh
        return st.as_dict()

    # ---------------------------------------------------------------- the stream-ordered sharded step
    def step_send(self, b, serial_base, levels, nshards, cap, send, exact=False):
        """Source side (syzsig_step_send_dev): b's staircase records into
        nshards buckets of cap + 1 words (send, int64).  Enqueues only."""
        self._check_dev(send)
        if send.numel() < nshards * (cap + 1):
            raise ValueError("send needs nshards * (cap + 1) words")
        lv = (ctypes.c_int8 * len(levels))(*levels)
        check(self.L.syzsig_step_send_dev(self.eng.h, ctypes.byref(b), int(serial_base), lv, len(levels), int(nshards),
                                          int(cap), _p(send), int(bool(exact))))

    def step_own(self, shard, new_signal, recv, nshards, cap, levels, flags, exact=False):
        """Owner side (syzsig_step_own_dev): the received buckets against this
        owner's shard; flags (uint8, nshards * (cap + 1)).  Enqueues only
        (exact: the per-record path, synchronous)."""
        self._check_dev(recv, flags)
        if recv.numel() < nshards * (cap + 1) or flags.numel() < nshards * (cap + 1):
            raise ValueError("recv / flags need nshards * (cap + 1) entries")
        if new_signal.is_nil():
            raise ValueError("step_own needs a non-nil newSignal shard (make(Signal, hint))")
        lv = (ctypes.c_int8 * len(levels))(*levels)
        check(self.L.syzsig_step_own_dev(self.eng.h, shard.handle, new_signal.handle, _p(recv), int(nshards),
                                         int(cap), lv, len(levels), _p(flags), int(bool(exact))))

    def step_back(self, b, serial_base, send, nshards, cap, back):
        """Source side again (syzsig_step_back_dev): the owners' flags -> b's
        call_new / new_pairs (/ new_bits).  Enqueues only unless bits are wanted."""
        self._check_dev(send, back)
        check(self.L.syzsig_step_back_dev(self.eng.h, ctypes.byref(b), int(serial_base), _p(send), int(nshards),
                                          int(cap), _p(back)))

    def step_finish(self):
        """The step's one host synchronisation -> the status dict."""
        st = StepStatus()
        check(self.L.syzsig_step_finish(self.eng.h, ctypes.byref(st)))
        return st.as_dict()

    # ---------------------------------------------------------------- synthetic data
    def synth_traces(self, cfg, prog_base, nprog, calls_per_prog, call_len):
        """-> (pcs int64[sum], call_start int64[n], call_prio uint8[n]) for nprog programs."""
        call_len = call_len.to(self.dev, torch.int32).contiguous()
        call_start = call_layout(call_len)
        total = int(call_len.to(torch.int64).sum().item())
        pcs = torch.empty(total, dtype=torch.int64, device=self.dev)
        prio = torch.empty(call_len.numel(), dtype=torch.uint8, device=self.dev)
        check(self.L.syzsig_synth_traces_dev(self.eng.h, ctypes.byref(cfg), int(prog_base), int(nprog),
                                             int(calls_per_prog), _p(call_start), _p(call_len), _p(pcs), _p(prio)))
        return pcs, call_start, call_len, prio

    def synth_m0_shard(self, cfg, known_sys, n, nshards, shard):
        """This shard's elements of synth_m0(cfg, known_sys, n), in index order
        (owner_of), without materialising the whole M0."""
        cap = n // nshards + 8 * int(n ** 0.5) + 1024 if nshards > 1 else n
        for _ in range(2):
            elems = torch.empty(max(cap, 1), dtype=torch.int32, device=self.dev)
            prios = torch.empty(max(cap, 1), dtype=torch.int8, device=self.dev)
            got = ctypes.c_uint64()
            rc = self.L.syzsig_synth_m0_shard_dev(self.eng.h, ctypes.byref(cfg), int(known_sys), int(n), int(nshards),
                                                  int(shard), _p(elems), _p(prios), cap, ctypes.byref(got))
            if rc == _lib.SYZSIG_ERANGE and got.value > cap:
                cap = got.value
                continue
            check(rc)
            return elems[: got.value], prios[: got.value]
        raise RuntimeError("synth_m0_shard: size changed between calls")

    def synth_m0(self, cfg, known_sys, n):
        elems = torch.empty(n, dtype=torch.int32, device=self.dev)
        prios = torch.empty(n, dtype=torch.int8, device=self.dev)
        check(self.L.syzsig_synth_m0_dev(self.eng.h, ctypes.byref(cfg), int(known_sys), int(n), _p(elems),
                                         _p(prios)))
        return elems, prios
