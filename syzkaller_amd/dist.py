"""Hash-sharded maxSignal across GPUs: one process per GPU, torch.distributed
(RCCL over xGMI on MI355X; gloo in CPU tests).

A batch is split by program range: rank r triages programs
[r*P, (r+1)*P), so the global serial order is rank-major (the order a single
fuzzer would see them).  maxSignal is partitioned by element:
shard(e) = owner_of(e, world) (csrc/common.h).  One step:

  1. levels  = union of every rank's call prios          (all_reduce, 256 ints)
  2. aggregate the rank's records per element and keep
     each element's staircase, grouped by owner           (agg.hip; shard.hip
                                                           routes every record)
  3. exchange counts, then records                       (all_to_all_single)
  4. owner triages the records it received               (triage.hip, records mode)
  5. new-flags travel back to the sources                (all_to_all_single)
  6. sources turn flags into call flags / pairs / bits   (agg.hip or shard.hip)

Only step 3/5 move data between GPUs; each element's whole history in the
batch lands on one owner, which applies the exact serial semantics via the
serial index carried in every record (see triage.hip).
"""
import torch
import torch.distributed as dist

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
    """The device half of a sharded step, on libsyzsig.

    aggregate=True (default): the source aggregates its batch per element and
    sends only the staircase records (agg.hip, <= 4 per distinct element);
    False: every record is sent (shard.hip).  Both give the same result."""

    def __init__(self, dev, aggregate=True):
        self.dev = dev
        self.aggregate = aggregate
        self._send = None
        self._flags = None
        self.last_source_stats = {}

    def partition(self, batch, serial_base, levels, nshards):
        b, new_bits, call_new = batch
        n = b.nrec
        if self.aggregate:
            if self._send is None or self._send.numel() < max(n, 1):
                self._send = torch.empty(max(n, 1), dtype=torch.int64, device=self.dev.dev)
            counts, st = self.dev.shard_agg_partition(b, serial_base, levels, nshards, self._send)
            self.last_source_stats = st
            send = self._send[: sum(counts)]
            return send, (send, serial_base), counts
        send = torch.empty(n, dtype=torch.int64, device=self.dev.dev)
        send_pos = torch.empty(n, dtype=torch.int32, device=self.dev.dev)
        counts = self.dev.shard_partition(b, serial_base, levels, nshards, send, send_pos)
        return send, send_pos, counts

    def triage_records(self, shard, new_signal, recs, levels):
        if self._flags is None or self._flags.numel() < recs.numel():
            self._flags = torch.empty(max(recs.numel(), 1) * 5 // 4 + 1, dtype=torch.uint8, device=self.dev.dev)
        flags = self._flags[: recs.numel()]
        st = self.dev.triage_records(shard, new_signal, recs, levels, flags)
        return flags, st

    def unpartition(self, batch, token, back):
        b, new_bits, call_new = batch
        if self.aggregate:
            send, serial_base = token
            self.dev.shard_agg_unpartition(b, serial_base, send, back)
        else:
            self.dev.shard_unpartition(b, token, back)
        return new_bits, call_new


# The prios signalPrio can produce (syz-fuzzer/fuzzer.go:513-521): a fixed
# level set for batches of real executions, so no collective is needed to
# agree on one (a superset of the prios present is exact: unused levels are
# never compared).
SIGNAL_PRIO_LEVELS = (0, 1, 2, 3)


class ShardedTriage:
    """One rank's side of a sharded checkNewSignal step.

    levels: the prio levels of every rank's calls, ascending as int8 (<= 4);
    None = agree on them with an all_reduce each step.  Per step the only host
    synchronisation is the exchange of the per-owner record counts (the split
    sizes all_to_all_single needs); the receive and flag buffers are reused."""

    def __init__(self, ops, shard, new_signal, group=None, device=None, levels=None):
        self.ops = ops
        self.shard = shard            # this rank's maxSignal shard
        self.new_signal = new_signal  # this rank's newSignal shard
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device
        self.fixed_levels = sorted(levels) if levels is not None else None
        self._recv = None
        self._back = None

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

    @staticmethod
    def _buffer(buf, n, dtype, dev):
        if buf is None or buf.numel() < n or buf.device != dev:
            buf = torch.empty(max(n, 1) + max(n, 1) // 4, dtype=dtype, device=dev)
        return buf

    def step(self, batch, call_prio, serial_base):
        """batch = (Batch, new_bits, call_new) for this rank's calls."""
        levels = self.levels(call_prio)
        if len(levels) > 4:
            raise ValueError("sharded triage supports <= 4 distinct prios per batch (signalPrio gives 0..3)")
        if not levels:
            levels = [0]
        send, token, counts = self.ops.partition(batch, serial_base, levels, self.world)
        dev = send.device
        cnt_out = torch.tensor(counts, dtype=torch.int64, device=dev)
        cnt_in = torch.empty_like(cnt_out)
        dist.all_to_all_single(cnt_in, cnt_out, group=self.group)
        recv_counts = cnt_in.tolist()  # the step's one host sync: split sizes
        nrecv = sum(recv_counts)
        self._recv = self._buffer(self._recv, nrecv, torch.int64, dev)
        recv = self._recv[:nrecv]
        dist.all_to_all_single(recv, send, recv_counts, counts, group=self.group)
        flags, st = self.ops.triage_records(self.shard, self.new_signal, recv, levels)
        self._back = self._buffer(self._back, send.numel(), torch.uint8, dev)
        back = self._back[: send.numel()]
        dist.all_to_all_single(back, flags, counts, recv_counts, group=self.group)
        new_bits, call_new = self.ops.unpartition(batch, token, back)
        st = dict(st)
        st["sent"] = int(send.numel())
        st["received"] = int(nrecv)
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
    send, counts = ops.split(ctx_off, elems, prios, world, rank, world, hint_distinct)
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
