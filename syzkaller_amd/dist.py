"""Hash-sharded maxSignal across GPUs: one process per GPU, torch.distributed
(RCCL over xGMI on MI355X; gloo in CPU tests).

A batch is split by program range: rank r triages programs
[r*P, (r+1)*P), so the global serial order is rank-major (the order a single
fuzzer would see them).  maxSignal is partitioned by element:
shard(e) = owner_of(e, world) (csrc/common.h).  One step (ShardedTriage.step),
stream-ordered with ONE host synchronisation:

  1. source: aggregate the rank's records per element and write each
     element's staircase into fixed buckets, one per owner, each with a
     header word (count, void / overflow flags)       (syzsig_step_send_dev)
  2. equal-split all_to_all_single of the buckets        (RCCL, no split sizes
                                                          needed on the host)
  3. owner: the received buckets, LDS-partitioned by
     element, replayed against the shard               (syzsig_step_own_dev)
  4. equal-split all_to_all_single of the flags back (a status byte per bucket)
  5. source: flags -> call_new / pairs                   (syzsig_step_back_dev)
  6. syzsig_step_finish: the one synchronisation; reads the step's status.

Every owner sees every source's header, so all ranks agree, without another
collective, whether the step is void (nothing committed anywhere: redone with
a larger bucket cap or the exact source path) or which owners skipped their
records (redone by those owners on the exact path, one more flags exchange).
Each element's whole history in the batch lands on one owner, which applies
the exact serial semantics via the serial index carried in every record.
"""
import torch
import torch.distributed as dist

# include/syzsig.h SYZSIG_STEP_HDR_VOID (bit 63) as an int64 bucket word
HDR_VOID = -(1 << 63)

__all__ = ["owner_of_torch", "ShardedTriage", "GpuShardOps", "GpuMinimizeOps", "SIGNAL_PRIO_LEVELS",
           "sharded_minimize"]

_M32 = 0xFFFFFFFF


def _fmix32(h):
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & _M32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & _M32
    h = h ^ (h >> 16)
    return h


def owner_of_torch(elems, nshards):
    """syz::owner_of over an int32/int64 tensor of elements (as u32)."""
    e = elems.to(torch.int64) & _M32
    h = _fmix32((e * 0x9E3779B1 + 0x7F4A7C15) & _M32)
    return (h * nshards) >> 32


class GpuShardOps:
    """The device half of a sharded step, on libsyzsig (syzsig_step_*):
    stream-ordered, one host synchronisation in finish()."""

    def __init__(self, dev):
        self.dev = dev
        self.device = dev.dev
        self.last = {}

    def alloc(self, n, dtype):
        return torch.empty(n, dtype=dtype, device=self.device)

    @staticmethod
    def records(batch):
        return int(batch[0].nrec)

    def send(self, batch, serial_base, levels, nshards, cap, send, exact=False):
        self.dev.step_send(batch[0], serial_base, levels, nshards, cap, send, exact)

    def own(self, shard, new_signal, recv, nshards, cap, levels, flags, exact=False):
        self.dev.step_own(shard, new_signal, recv, nshards, cap, levels, flags, exact)

    def back(self, batch, serial_base, send, nshards, cap, back):
        self.dev.step_back(batch[0], serial_base, send, nshards, cap, back)

    def finish(self):
        self.last = self.dev.step_finish()
        return self.last

    @staticmethod
    def outputs(batch):
        return batch[1], batch[2]


# The prios signalPrio can produce (syz-fuzzer/fuzzer.go:513-521): a fixed
# level set for batches of real executions, so no collective is needed to
# agree on one (a superset of the prios present is exact: unused levels are
# never compared).
SIGNAL_PRIO_LEVELS = (0, 1, 2, 3)


class ShardedTriage:
    """One rank's side of a sharded checkNewSignal step (syz-fuzzer/fuzzer.go:494-511
    over the rank-major batch).

    ops: GpuShardOps(dev) or a restatement with the same send / own / back /
    finish / alloc methods.  levels: the prio levels of every rank's calls,
    ascending as int8 (<= 4); None = agree on them with an all_reduce each step.
    The bucket cap (records per source and owner) is agreed by all ranks: on the
    first step from the batch sizes, then tightened once to what the first step
    needed; a step that overflows it is redone with a larger one."""

    CAP_SLACK = 1.25

    def __init__(self, ops, shard, new_signal, group=None, device=None, levels=None, cap=None):
        self.ops = ops
        self.shard = shard            # this rank's maxSignal shard
        self.new_signal = new_signal  # this rank's newSignal shard (non-nil)
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device
        self.fixed_levels = sorted(levels) if levels is not None else None
        self.cap = cap
        self._tightened = cap is not None
        self._exact = False
        self._bufs = {}
        self.redos = 0
        self.fixups = 0

    def levels(self, call_prio):
        """Union of the prios of all ranks' calls, ascending as int8."""
        if self.fixed_levels is not None:
            return self.fixed_levels
        present = torch.zeros(256, dtype=torch.int32, device=call_prio.device)
        if call_prio.numel():
            present[call_prio.to(torch.int64)] = 1
        dist.all_reduce(present, op=dist.ReduceOp.MAX, group=self.group)
        vals = [v if v < 128 else v - 256 for v in torch.nonzero(present).flatten().tolist()]
        return sorted(vals)

    def _agree(self, vals):
        t = torch.tensor(vals, dtype=torch.int64, device=self.ops.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return [int(x) for x in t.tolist()]

    def _cap_for(self, need):
        return int(need * self.CAP_SLACK) + 4096

    def _buffers(self, cap):
        n = self.world * (cap + 1)
        if self._bufs.get("n", 0) < n:
            self._bufs = {"n": n, "send": self.ops.alloc(n, torch.int64), "recv": self.ops.alloc(n, torch.int64),
                          "flags": self.ops.alloc(n, torch.uint8), "back": self.ops.alloc(n, torch.uint8)}
        return [self._bufs[k][:n] for k in ("send", "recv", "flags", "back")]

    def step(self, batch, call_prio, serial_base):
        """batch: what ops.send takes for this rank's calls (GpuShardOps: the
        (Batch, new_bits, call_new) triple of Device.batch).  Returns
        (new_bits, call_new, stats)."""
        levels = self.levels(call_prio)
        if len(levels) > 4:
            raise ValueError("sharded triage supports <= 4 distinct prios per batch (signalPrio gives 0..3)")
        if not levels:
            levels = [0]
        W, g = self.world, self.group
        if self.cap is None:
            # first step: a guess every rank agrees on (a step that overflows it
            # is redone with what the sources counted)
            self.cap = self._cap_for(self._agree([min(self.ops.records(batch) // (4 * W) + 1, 1 << 21)])[0])
        for attempt in range(4):
            cap = self.cap
            send, recv, flags, back = self._buffers(cap)
            # A rank whose send or own fails (a host-side check: ERANGE on its
            # serial range, EINVAL, an allocation) must not leave its peers in
            # the exchange, and the steady state has no host collective to
            # agree on errors.  So the failure travels in-band: a failed send
            # puts VOID headers in every bucket, a failed own the "void" status
            # (1) in every flags bucket; every rank then sees a void step and
            # the redo's agreement below raises on every rank alike.
            err = None
            try:
                self.ops.send(batch, serial_base, levels, W, cap, send, self._exact)
            except Exception as e:  # noqa: BLE001 -- raised on every rank below
                err = e
                send.view(W, cap + 1)[:, 0] = HDR_VOID
            dist.all_to_all_single(recv, send, group=g)
            try:
                self.ops.own(self.shard, self.new_signal, recv, W, cap, levels, flags)
            except Exception as e:  # noqa: BLE001
                err = err or e
                flags.view(W, cap + 1)[:, 0] = 1
            dist.all_to_all_single(back, flags, group=g)
            self.ops.back(batch, serial_base, send, W, cap, back)
            st = self.ops.finish()  # the step's one host synchronisation
            if not st["global_void"]:
                if err is not None:  # (not reachable: the failing rank's VOID reaches everyone)
                    raise err
                break
            # nothing was committed on any rank (every owner saw the same headers):
            # agree on a cap for what the sources counted, a void source takes its
            # exact path, and the step runs again
            self.redos += 1
            need, bad, failed = self._agree([st["max_out"] if err is None else 0,
                                             1 if err is None and st["src_void"] == 2 else 0,
                                             1 if err is not None else 0])
            if failed:
                if err is not None:
                    raise err
                raise RuntimeError("sharded step: the step failed on another rank")
            if bad:  # a call's prio outside the agreed levels: an error on every rank alike
                raise ValueError("sharded step: a call's prio is not among the step's levels")
            self.cap = max(self.cap, self._cap_for(need)) if need > cap else self.cap
            # a source that voided its run stays on its exact path for the rest of
            # the step (a later cap overflow must not send it back to the capped
            # cells, which would spill again)
            self._exact = self._exact or st["src_void"] != 0
        else:
            raise RuntimeError("sharded step: still void after 4 attempts")
        self._exact = False
        if st["owners_void"]:
            # owners whose records overflowed the LDS partitions skipped them:
            # they redo them on the per-record path, the flags go back once more
            self.fixups += 1
            err = None
            if (st["owners_void"] >> self.rank) & 1:
                try:
                    self.ops.own(self.shard, self.new_signal, recv, W, cap, levels, flags, True)
                except Exception as e:  # noqa: BLE001 -- raised on every rank below
                    err = e
                    flags.view(W, cap + 1)[:, 0] = 1
            else:
                flags.zero_()
            dist.all_to_all_single(back, flags, group=g)
            self.ops.back(batch, serial_base, send, W, cap, back)
            st2 = self.ops.finish()
            if err is not None:
                raise err
            if st2["global_void"]:  # an owner's fix-up failed: every source sees its status
                raise RuntimeError("sharded step: an owner's exact fix-up failed on another rank")
            for k in ("inserted", "changed", "own_distinct"):
                st[k] += st2[k]
            st["new_pairs"] = st2["new_pairs"]
        if not self._tightened:
            # once: the cap this workload needs (all ranks agree on it)
            self._tightened = True
            need = self._agree([st["max_out"]])[0]
            self.cap = min(self.cap, self._cap_for(need))
        st = dict(st)
        st["cap"] = cap
        new_bits, call_new = self.ops.outputs(batch)
        return new_bits, call_new, st


class GpuMinimizeOps:
    """The device halves of the data-split Minimize (csrc/minimize.hip)."""

    def __init__(self, dev):
        self.dev = dev

    def split(self, ctx_off, elems, prios, nparts, part, nshards, hint_distinct=0):
        return self.dev.minimize_split(ctx_off, elems, prios, nparts, part, nshards, hint_distinct)

    def resolve(self, ctx_off, recs):
        return self.dev.minimize_resolve(ctx_off, recs)[0]


def sharded_minimize(ops, ctx_off, elems, prios, group=None, hint_distinct=0):
    """signal.Minimize (pkg/signal/signal.go:138-166) split by data over the
    ranks of `group`: rank r takes a contiguous range of the
    contexts in sort order (Len desc, index asc; ~total/world entries) and reads
    only its own entries; it aggregates them to one winner record
    (e, prio, rank) per distinct element (ops.split), the records go to
    owner_of(e) with all_to_all_single, the owner keeps the max per element and
    marks the winning contexts (ops.resolve), and the keep bytes are OR-reduced
    (all_reduce MAX).  ops = GpuMinimizeOps(dev) or a restatement with the same
    methods.  Every rank holds the corpus description (ctx_off); elems/prios
    need only hold its own range.  Returns (keep u8[nctx], survivors)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    err = None
    try:
        send, counts = ops.split(ctx_off, elems, prios, world, rank, world, hint_distinct)
    except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
        err = e
    # every rank agrees on the split's success before entering the exchange: a
    # rank that raised alone would leave its peers blocked in all_to_all_single
    dev = ctx_off.device if isinstance(ctx_off, torch.Tensor) else "cpu"
    bad = torch.tensor([1 if err is not None else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(bad, op=dist.ReduceOp.MAX, group=group)
    if err is not None:
        raise err
    if int(bad.item()):
        raise RuntimeError("sharded_minimize: the split failed on another rank")
    dev = send.device
    cnt_out = torch.tensor(counts, dtype=torch.int64, device=dev)
    cnt_in = torch.empty_like(cnt_out)
    dist.all_to_all_single(cnt_in, cnt_out, group=group)
    recv_counts = cnt_in.tolist()
    recv = torch.empty(sum(recv_counts), dtype=torch.int64, device=dev)
    dist.all_to_all_single(recv, send, recv_counts, counts, group=group)
    keep = ops.resolve(ctx_off, recv)
    dist.all_reduce(keep, op=dist.ReduceOp.MAX, group=group)
    return keep, int(keep.to(torch.int64).sum().item())
