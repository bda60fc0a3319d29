#!/usr/bin/env python3
"""Benchmark: signal elements triaged per second (batched DiffRaw+Merge of
checkNewSignal against maxSignal), BASELINE.json config 2 per GPU:

  4096 programs x 64 calls x 4096 PCs (synthetic KCOV traces)
  -> K1+K2 edge derivation (setup, timed separately as `stages.edge_ms`)
  -> one step = restore maxSignal to the 10M-element M0, then triage the whole
     batch (K3 probe + decide), outputs: per-record new bits, per-call flags,
     updated maxSignal and newSignal.

N=1: one GPU, one process.  N>1 (torchrun, one rank per GPU): maxSignal is
hash-sharded over the ranks (10M elements per rank), each rank owns its own
4096-program slice of the batch (weak scaling), records are routed to their
owner with RCCL all-to-all (syzkaller_amd/dist.py).

Prints one JSON line on rank 0.  Beside the headline K3 line it carries, as
their own objects with their own roofline, `lines.edge` (K1+K2: KCOV PCs ->
edge signals, 12 B/PC) and `lines.minimize` (BASELINE config 3: Minimize over
a 200k-context corpus, 5 B/entry + 4 B/distinct element); `cpu_baseline` is
the oracle on one core plus `multi_core` (--cpu-threads Procs under one
rwlock, as syz-fuzzer runs checkNewSignal), with nproc and the CPU model.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
PROBE_BYTES_PER_REC = 12.0  # 4 B element read + 8 B maxSignal slot read
# the K3 pipeline of one step on one GPU (csrc/agg.hip); roofline.avg_launch_ms is
# their summed device time (HIP events), roofline.traffic their summed PMC bytes
# (two scatters over one run, each taking the work items the other skips: csrc/agg.hip scatter_triage)
K3_KERNELS = "k_fast_prep+k_cell_plan_fast+k_scat3+k_agg_scatter_blk+k_agg+k_agg_finalize_x+k_fin_deferred"
EDGE_BYTES_PER_PC = 12.0  # K1+K2: 8 B u64 PC in + 4 B u32 signal out
# Minimize's chain on its aggregation path (csrc/minimize.hip header); the
# keys sort and k_min_calls are negligible (200k contexts)
MIN_KERNELS = ("k_min_calls+k_chunk_sizes+k_cell_plan+k_scat3+k_agg_scatter_blk+k_agg"
               "+k_min_from_dist+k_count_u8")
MIN_BYTES_PER_ENTRY, MIN_BYTES_PER_DISTINCT = 5.0, 4.0  # Minimize: (elem, prio) entry + covered[e]
# N > 1: the source's aggregation, then the owner's records-mode triage of the staircases
K3_DIST_KERNELS = ("k_fast_prep+k_cell_plan_fast+k_scat3+k_agg_scatter_blk+k_agg+k_stair_bucket+k_stair_heads"
                   "+k_step_heads+k_rp_count+k_rp_colsum+k_rp_scan+k_rp_coloffs+k_rp_scatter+k_rp_agg+k_rp_elems+k_rp_reduce+k_rp_flags+k_step_status"
                   "+k_step_back")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--programs", type=int, default=4096, help="programs per GPU")
    ap.add_argument("--calls", type=int, default=64)
    ap.add_argument("--pcs", type=int, default=4096)
    ap.add_argument("--m0", type=int, default=10_000_000, help="maxSignal elements (N=1)")
    ap.add_argument("--m0-total", type=int, default=1_000_000_000,
                    help="N>1: maxSignal elements over all ranks, hash-sharded (BASELINE config 4: 1B)")
    ap.add_argument("--skew", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample time (s)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (= RCCL over xGMI, the product path); gloo only to rehearse N>1 ranks "
                         "sharing fewer GPUs (rank r uses GPU r mod device_count)")
    ap.add_argument("--ns-hint", type=int, default=4_000_000, help="newSignal size hint (make(Signal, hint))")
    ap.add_argument("--table-hint", type=int, default=0,
                    help="size maxSignal's table for this many entries (default: the library's policy)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the multi-core CPU baseline (the GPU box's CPU share is 16 per GPU)")
    ap.add_argument("--min-contexts", type=int, default=200_000, help="Minimize line: corpus size (BASELINE config 3)")
    ap.add_argument("--no-min", action="store_true", help="skip the Minimize line")
    ap.add_argument("--no-c5", action="store_true", help="skip the C5 streaming line")
    ap.add_argument("--no-c4", action="store_true", help="skip the C4 per-rank line")
    ap.add_argument("--no-c1", action="store_true", help="skip the C1 line")
    ap.add_argument("--no-gw", action="store_true", help="skip the C2 line on the other trace distribution")
    ap.add_argument("--walk", default="global", choices=("global", "region"),
                    help="trace distribution: SURVEY 8(d)'s walk over all 2^20 blocks (global), or walks inside "
                         "per-syscall 256-block regions (region, rounds 1-3's headline)")
    ap.add_argument("--batches", type=int, default=4, help="distinct batches the steps cycle through")
    ap.add_argument("--no-pipe", action="store_true", help="skip the K1+K2 -> K3 pipeline line")
    ap.add_argument("--no-poll", action="store_true", help="skip the manager Poll line")
    return ap.parse_args()


TRIAGE_KEYS = ("programs_per_gpu", "calls", "pcs_per_call", "m0_per_gpu", "skew", "parallelism", "walk", "batches")
# M0's known part per trace distribution (synth_m0 known_sys): the global walk's
# whole edge universe, or every edge of syscalls 0..2047 of the region walk
KNOWN_SYS = {"global": 1, "region": 2048}


def walk_cfg(walk, **over):
    from syzkaller_amd import synth

    return synth.synth_default(global_walk=1 if walk == "global" else 0, **over)
MIN_KEYS = ("workload", "contexts", "entries", "mean_len")


def pmc_traffic(kernel_prefixes, cfg, keys=TRIAGE_KEYS, expect_ms=None, tol=0.15):
    """HBM bytes per launch of the dominant kernel chain from the newest
    committed rocprofv3 PMC summary (profiles/*/summary.json, written by
    scripts/summarize_prof.py from separate FETCH_SIZE / WRITE_SIZE passes of
    this same workload: scripts/profile.sh) whose workload matches.  expect_ms:
    the line's own chain time; a summary whose matched kernels' summed average
    duration differs from it by more than `tol` profiled other code and is not
    used.  Returns (bytes or None, source path or None, reason or None)."""
    import glob

    best, rejected = None, []
    for f in glob.glob(os.path.join(ROOT, "profiles", "*", "summary.json")):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        bc = d.get("bench_config") or {}
        if any(bc.get(k) != cfg.get(k) for k in keys):
            continue
        tot, ms, hit = 0.0, 0.0, False
        for name, e in d.get("kernels", {}).items():
            if any(name == k or name.startswith(k + "<") for k in kernel_prefixes) and "traffic_bytes" in e:
                tot += e["traffic_bytes"]
                ms += e.get("avg_ms", 0.0)
                hit = True
        if not hit:
            continue
        rel = os.path.relpath(f, ROOT)
        if expect_ms and abs(ms / expect_ms - 1.0) > tol:
            rejected.append(f"{rel}: profiled chain {ms:.3f} ms vs this line's {expect_ms:.3f} ms")
            continue
        t = (d.get("created", 0), f)  # the newest summary (created stamp), then name
        if best is None or t > best[0]:
            best = (t, tot, rel)
    if best:
        return best[1], best[2], None
    return None, None, ("no PMC summary of this workload and code: " + "; ".join(rejected)) if rejected else \
        "no PMC summary of this workload"


def achievable_bw(dev, nbytes=1 << 30, reps=5):
    """the achievable HBM bandwidth beside the spec peak -- a plain
    device copy (csrc/runtime.hip k_copy16, 16 B per lane, nontemporal) of
    `nbytes` between two HBM buffers, read + write bytes / device time (HIP
    events), median of `reps` after one warm-up."""
    src = torch.ones(nbytes // 8, dtype=torch.int64, device=dev.dev)
    dst = torch.empty_like(src)
    ms = [dev.copy_bw(dst, src, nbytes) for _ in range(reps + 1)][1:]
    ok = bool(torch.equal(dst, src))
    t = float(np.median(ms))
    del src, dst
    return {"value": 2 * nbytes / (t * 1e-3) / 1e9, "unit": "GB/s", "ms": t, "bytes_copied": nbytes,
            "kernel": "k_copy16 (one 16-B element per lane, nontemporal loads and stores)", "check": ok}


def with_achievable(roof, ach):
    """roofline + the achievable bandwidth and the fraction of it."""
    if roof and ach and roof.get("unit") == "GB/s":
        roof["achievable"] = ach["value"]
        roof["frac_achievable"] = roof["achieved"] / ach["value"]
    return roof


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(dev, sigs, cs, cnt, prio, m0e, m0p, calls_per_prog, target_s, threads):
    """The oracle (plain-C restatement of checkNewSignal/pkg/signal,
    oracle/oracle.c) on a bounded sample: the first S programs of this batch
    against the same M0.  1 core: the sequential loop; N cores: `threads`
    Procs running fuzzer.go:494-511 concurrently (DiffRaw under the reader
    lock, Merge under the writer lock, orc_triage_batch_mt)."""
    from oracle import oracle as O

    h_cs = cs.cpu().numpy().view(np.uint64)
    h_cnt = cnt.cpu().numpy().view(np.uint32)
    h_prio = prio.cpu().numpy()
    e = m0e.cpu().numpy().view(np.uint32)
    p = m0p.cpu().numpy()
    nprog_total = h_cnt.size // calls_per_prog

    def run(nprog, nthreads):
        nc = nprog * calls_per_prog
        end = int(h_cs[nc - 1]) + int(h_cnt[nc - 1])
        h_sigs = sigs[:end].cpu().numpy().view(np.uint32)
        ms = O.deserialize(e, p)
        t = time.perf_counter()
        if nthreads == 1:
            O.triage_batch_into(ms, h_sigs, h_cs[:nc], h_cnt[:nc], h_prio[:nc])
        else:
            O.triage_batch_mt(ms, h_sigs, h_cs[:nc], h_cnt[:nc], h_prio[:nc], calls_per_prog, nthreads)
        dt = time.perf_counter() - t
        return int(h_cnt[:nc].sum()), dt

    def sample(nthreads, budget):
        n = 8
        recs, dt = run(n, nthreads)
        est = max(1, min(nprog_total, int(n * budget / max(dt, 1e-3))))
        if est > n:
            n = est
            recs, dt = run(n, nthreads)
        return n, recs, dt

    n, recs, dt = sample(1, target_s)
    out = {"value": recs / dt, "unit": "elems/s", "cores": 1, "kind": "port",
           "sample": f"first {n} programs ({recs} signal elements) of the same batch vs the same M0, "
                     f"oracle/oracle.c single thread, {dt:.2f} s",
           "nproc": os.cpu_count(), "cpu_model": cpu_model()}
    if threads > 1:
        n2, recs2, dt2 = sample(threads, target_s / 2)
        out["multi_core"] = {"value": recs2 / dt2, "unit": "elems/s", "cores": threads, "kind": "port",
                             "sample": f"first {n2} programs ({recs2} signal elements), {threads} threads as Procs "
                                       f"under one rwlock (fuzzer.go:494-511, oracle.c orc_triage_batch_mt), "
                                       f"{dt2:.2f} s"}
    return out


def minimize_cpu(off, elems, prios, target_s):
    """Minimize's CPU leg: the oracle (plain-C restatement of
    pkg/signal/signal.go:138-166: sort by Len desc, then the per-element
    strictly-greater replacement over a Go-map-like hash) on one core, over
    the first S contexts of the same corpus (a smaller corpus of the same
    length and element distribution), S calibrated to ~target_s."""
    from oracle import oracle as O

    h_off = off.cpu().numpy().view(np.uint64)
    n = h_off.size - 1

    def run(k):
        z = int(h_off[k])
        e = elems[:z].cpu().numpy().view(np.uint32)
        p = prios[:z].cpu().numpy().view(np.int8)
        t = time.perf_counter()
        O.minimize(h_off[: k + 1], e, p)
        return z, time.perf_counter() - t

    k = min(n, 2000)
    z, dt = run(k)
    est = max(1, min(n, int(k * target_s / max(dt, 1e-3))))
    if est > k:
        k = est
        z, dt = run(k)
    return {"value": z / dt, "unit": "entries/s", "cores": 1, "kind": "port", "ms": dt * 1e3,
            "sample": f"first {k} of the {n} contexts ({z} entries), oracle/oracle.c orc_minimize single thread, "
                      f"{dt:.2f} s"}


def minimize_line(dev, n, mean=2000, U=1 << 22, seed=2018, reps=3, cpu_s=0.0):
    """BASELINE config 3: signal.Minimize (pkg/signal/signal.go:138-166) over a
    synthetic n-context corpus (geometric lengths, mean `mean`, elements from a
    2^22 universe, distinct inside a context, prio 0..3), resident in HBM;
    device time of syzsig_minimize_dev (HIP events)."""
    g = torch.Generator(device=dev.dev).manual_seed(seed)
    rng = np.random.default_rng(seed)
    lens = torch.as_tensor(np.minimum(rng.geometric(1.0 / mean, size=n), U), dtype=torch.int64, device=dev.dev)
    off = torch.zeros(n + 1, dtype=torch.int64, device=dev.dev)
    off[1:] = torch.cumsum(lens, 0)
    N = int(off[-1])
    base = torch.randint(0, U, (n,), generator=g, device=dev.dev, dtype=torch.int64)
    stride = torch.randint(0, U // 2, (n,), generator=g, device=dev.dev, dtype=torch.int64) * 2 + 1
    ctx = torch.repeat_interleave(torch.arange(n, device=dev.dev), lens)
    k = torch.arange(N, device=dev.dev, dtype=torch.int64) - off[:-1][ctx]
    elems = ((base[ctx] + k * stride[ctx]) & (U - 1)).to(torch.int32)
    del ctx, k
    prios = torch.randint(0, 4, (N,), generator=g, device=dev.dev, dtype=torch.int8)
    distinct = int(torch.unique(elems).numel())
    ms = []
    for _ in range(reps):
        keep, cnt = dev.minimize(off, elems, prios, hint_distinct=U)
        ms.append(dev.L.syzsig_ctx_last_ms(dev.eng.h))
    t = float(np.median(ms))
    cpu = minimize_cpu(off, elems, prios, cpu_s) if cpu_s > 0 else None
    byts = MIN_BYTES_PER_ENTRY * N + MIN_BYTES_PER_DISTINCT * distinct
    cfg = {"workload": f"BASELINE config 3: Minimize over a {n}-program synthetic corpus, 1 GPU",
           "contexts": n, "entries": N, "distinct": distinct, "mean_len": mean, "survivors": cnt}
    traffic, src, note = pmc_traffic(["syz::" + k for k in MIN_KERNELS.split("+")], cfg, MIN_KEYS, expect_ms=t)
    achieved = byts / (t * 1e-3) / 1e9
    return {"metric": "signal.Minimize corpus entries/sec", "value": N / (t * 1e-3), "unit": "entries/s",
            "higher_is_better": True, "ms": t, "dtype": "u32",
            "config": cfg, "cpu": cpu,
            "roofline": {"bound": "hbm", "kernel": MIN_KERNELS,
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
                         "traffic_note": note,
                         "bytes_per_unit": f"{MIN_BYTES_PER_ENTRY} B/entry + {MIN_BYTES_PER_DISTINCT} B/distinct",
                         "avg_launch_ms": t}}


POLL_BYTES_PER_ENTRY = 5.0  # Poll: a polled (elem u32, prio i8) entry (SURVEY 8(d)'s Minimize-style figure)
# the batch's kernels (csrc/poll.hip, and recs.hip's grouping); the Serialize of the replies is not among them
POLL_KERNELS = ("k_poll_recpoll+k_poll_x+k_rp_one_seg+k_rp_count+k_rp_colsum+k_rp_scan+k_rp_coloffs+k_rp_scatter_idx"
                "+k_poll_part_walk+k_poll_fanout+k_poll_pre+k_poll_count+k_poll_commit+k_poll_scatter")


def poll_cpu(e0, p0, polls, F, target_s):
    """Poll's CPU leg: the reference loop (manager.go:1027-1052) restated over
    the oracle's sets (oracle.poll: Diff into maxSignal, Merge, fan-out into
    every other fuzzer's newMaxSignal, the reply) on one core, poll after poll
    over the first polls of the same batch against the same maxSignal."""
    from oracle import oracle as O

    oms = O.deserialize(e0, p0)
    onm = [O.OSig() for _ in range(F)]
    t0, k, n = time.perf_counter(), 0, 0
    for f, ser in polls:
        O.poll(oms, onm, f, (np.asarray(ser.Elems), np.asarray(ser.Prios)))
        k += 1
        n += int(np.asarray(ser.Elems).size)
        if time.perf_counter() - t0 > target_s:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "entries/s", "cores": 1, "kind": "port", "ms": dt * 1e3,
            "sample": f"first {k} of the {len(polls)} polls ({n} entries) against the same {e0.size}-element "
                      f"maxSignal, oracle.poll single thread (manager.go:1027-1052), {dt:.2f} s"}


def poll_line(dev, F=16, K=256, per=16384, fresh=0.05, m0=10_000_000, reps=3, seed=1027, cpu_s=0.0):
    """syz-manager's Poll (manager.go:1027-1052) over a
    batch of K polls from F fuzzers, each carrying a Serial of `per` entries,
    against a 10M-element maxSignal (random u32, prio 0..3): a steady-state
    manager, where a fuzzer's newSignal since its last poll is mostly signal
    the manager already has -- a (1 - fresh) share of the entries are
    elements of maxSignal at a prio no higher than maxSignal's, the rest
    random u32 at prio 0..3 (new).  Every fuzzer starts with an empty
    newMaxSignal.  One signal.manager_poll call (syzsig_manager_poll_batch: the
    Serials are host arrays, i.e. RPC payloads, so the time includes their
    upload and the replies' Serialize); wall time, median of `reps`, state
    restored between reps."""
    from syzkaller_amd import signal as S

    rng = np.random.default_rng(seed)
    e0 = rng.integers(0, 1 << 32, m0, dtype=np.uint64).astype(np.uint32)
    p0 = rng.integers(0, 4, m0).astype(np.int8)
    polls = []
    for _ in range(K):
        known = rng.random(per) >= fresh
        pick = rng.integers(0, m0, per)
        e = np.where(known, e0[pick], rng.integers(0, 1 << 32, per, dtype=np.uint64).astype(np.uint32))
        p = np.where(known, np.minimum(p0[pick], rng.integers(0, 4, per)), rng.integers(0, 4, per)).astype(np.int8)
        polls.append((int(rng.integers(0, F)), S.Serial(e.astype(np.uint32), p)))
    pristine = S.Serial(e0, p0).Deserialize(dev.eng)
    walls, devs = [], []
    for r in range(reps + 1):
        ms = pristine.clone()
        nm = [S.Signal(None, dev.eng) for _ in range(F)]
        torch.cuda.synchronize()
        t = time.perf_counter()
        replies = S.manager_poll(ms, nm, polls, dev.eng)
        torch.cuda.synchronize()
        if r:
            walls.append(time.perf_counter() - t)
            devs.append(dev.L.syzsig_ctx_last_ms(dev.eng.h))
        nrep = sum(int(np.asarray(x.Elems).size) for x in replies)
        del ms, nm, replies
    wall, dms = float(np.median(walls)), float(np.median(devs))
    cpu = poll_cpu(e0, p0, polls, F, cpu_s) if cpu_s > 0 else None
    n = K * per
    achieved = POLL_BYTES_PER_ENTRY * n / (dms * 1e-3) / 1e9
    wl = (f"{K} polls from {F} fuzzers x {per} entries ({fresh:.0%} new, the rest already in maxSignal) vs a "
          f"{m0}-element maxSignal, one batch (host Serials: upload and replies' Serialize included)")
    # HBM bytes of the batch's kernels from the newest PMC summary of this line
    # (the stream time also holds copies and host round trips, so the
    # profiled kernels' time is not compared with it)
    traffic, src, note = pmc_traffic(["syz::" + k for k in POLL_KERNELS.split("+")], {"workload": wl}, ("workload",))
    return {"metric": "manager Poll: polled entries/sec (Diff into maxSignal, Merge, fan-out)",
            "value": n / wall, "unit": "entries/s", "higher_is_better": True, "ms": wall * 1e3, "dtype": "u32",
            "library_stream_ms": dms, "cpu": cpu,
            "config": {"workload": wl, "entries": n, "reply_entries": nrep},
            "roofline": {"bound": "hbm", "kernel": "syzsig_manager_poll_batch's stream work (uploads, kernels, the "
                                                    "host round trips between; HIP events); traffic: " + POLL_KERNELS,
                         "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_source": src, "traffic_note": note,
                         "bytes_per_unit": POLL_BYTES_PER_ENTRY, "units_per_launch": n,
                         "avg_launch_ms": dms}}


def synth_batch(dev, cfg, prog_base, P, C, L):
    """Synthetic KCOV traces of P programs x C calls x L PCs -> K1+K2 on device.
    Returns (sigs, call_start, sig_cnt, prio, records, pcs)."""
    cl = torch.full((P * C,), L, dtype=torch.int32)
    pcs, cs, cl, prio = dev.synth_traces(cfg, prog_base, P, C, cl)
    pidx = torch.arange(P + 1, dtype=torch.int32, device=dev.dev) * C
    sigs, cnt, comp = dev.edge_derive(pcs, cs, cl, pidx)
    npc = pcs.numel()
    del pcs
    return sigs, cs, cnt, prio, int(cnt.to(torch.int64).sum().item()), npc


def chain_ms(st):
    return st["part_ms"] + st["probe_ms"] + st["decide_ms"]


def c5_line(dev, pairs, programs=8192, calls=64, pcs=1024, nbatches=4, reps=3, m0=10_000_000, walk="global",
            cpu_s=0.0, cpu_threads=16):
    """BASELINE config 5 (sustained streaming triage, skewed PC distribution)
    at one rank's share of an 8-GPU node: batches of `programs` x `calls` x
    `pcs`, each triaged against the maxSignal/newSignal state the previous
    batch left (syz-fuzzer/proc.go:230-247 -> fuzzer.go:494-511 per
    execution, batched).  walk="global" is SURVEY 8(d)'s C5 input: every
    call a walk over all 2^20 blocks started from the entry of a
    Zipf(1.1)-chosen syscall (skew=2, csrc/common.h synth_zipf4096), so the
    walks' first edges are hot across the batch, against a 10M-element M0
    holding the edge universe; walk="region" is rounds 1-4's line (power-skewed
    syscalls, u^4, walking their 256-block regions).  The sequence of
    `nbatches` batches starts from M0 and is replayed `reps` times (state
    restored between replays, outside the timed region); value = records /
    wall time of the sequence, chain = device time of the K3 kernels."""
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth

    cfg = walk_cfg(walk, skew=2 if walk == "global" else 1)
    keep, bs = [], []
    total = 0
    for i in range(nbatches):
        sigs, cs, cnt, prio, nrec, _ = synth_batch(dev, cfg, i * programs, programs, calls, pcs)
        b, _, cnew = dev.batch(sigs, cs, cnt, prio, new_pairs=pairs, want_bits=False)
        keep.append((sigs, cs, cnt, prio, cnew))
        bs.append(b)
        total += nrec
    m0e, m0p = dev.synth_m0(cfg, KNOWN_SYS[walk], m0)
    pristine = dev.deserialize(m0e, m0p)
    # CPU leg: the first programs of batch 1 against the same M0 (the oracle's
    # sequential checkNewSignal on one core, and `cpu_threads` Procs under one
    # rwlock as fuzzer.go:494-511 runs them)
    cpu = cpu_baseline(dev, *keep[0][:4], m0e, m0p, calls, cpu_s, cpu_threads) if cpu_s > 0 else None
    del m0e, m0p
    walls, chains, sts = [], [], []
    for r in range(reps + 1):
        ms = pristine.clone()
        ns = S.Signal.make(4_000_000, dev.eng)
        torch.cuda.synchronize()
        t = time.perf_counter()
        st = [dev.triage_b(ms, ns, b) for b in bs]
        torch.cuda.synchronize()
        if r:  # the first replay warms up
            walls.append(time.perf_counter() - t)
            chains.append(sum(chain_ms(x) for x in st))
            sts = st
    wall, chain = float(np.median(walls)), float(np.median(chains))
    achieved = PROBE_BYTES_PER_REC * total / (chain * 1e-3) / 1e9
    wl = (f"BASELINE config 5 at one rank's share of 8 GPUs: {nbatches} consecutive batches of {programs} programs "
          f"x {calls} calls x {pcs} PCs, " +
          ("SURVEY 8(d)'s global walks from Zipf(1.1) entries" if walk == "global" else "skew=1") +
          f", each against the state the previous one left (M0 {m0})")
    traffic, src, note = pmc_traffic(["syz::" + k for k in K3_KERNELS.split("+")], {"workload": wl}, ("workload",),
                                     expect_ms=chain / nbatches)
    return {"metric": "signal elems triaged/sec (Diff+Merge), streaming skewed batches",
            "value": total / wall, "unit": "elems/s", "higher_is_better": True,
            "ms_per_batch": wall * 1e3 / nbatches, "dtype": "u32", "cpu": cpu,
            "config": {"workload": wl,
                       "records": total, "batches": nbatches,
                       "retries": [x["retries"] for x in sts], "runs": [x["runs"] for x in sts],
                       "new_per_batch": [x["changed"] for x in sts], "distinct": [x["distinct"] for x in sts],
                       "note": ("SURVEY 8(d)'s global walk reaches every edge of the universe in the first "
                                "batch, so the later batches find almost nothing new: they time checkNewSignal's "
                                "DiffRaw with next to no Merge (new_per_batch)") if walk == "global" else None},
            "roofline": {"bound": "hbm", "kernel": K3_KERNELS, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
                         "traffic_note": note,
                         "bytes_per_unit": PROBE_BYTES_PER_REC, "units_per_launch": total // nbatches,
                         "avg_launch_ms": chain / nbatches}}


def c2_walk_line(dev, pairs, P, C, L, walk, reps=5, m0=10_000_000):
    """BASELINE config 2 on one trace distribution (the one the headline does
    not use): `global` is SURVEY 8(d)'s own input -- every call a walk
    b <- (4b + 1 + r%4) mod B over all B = 2^20 blocks from a uniform block
    (csrc/common.h synth_trace, global_walk=1), so almost every PC emits a
    signal (~1.07e9 records per batch), against a 10M-element M0 that holds the
    whole 5.2M-edge universe (prio uniform 0..3) plus random elements; `region`
    walks inside per-syscall 256-block regions (rounds 1-3's headline: 321M
    records, a 70 % K2 drop rate) against every edge of syscalls 0..2047 plus
    random elements.  Same step as the headline: maxSignal back to M0, then the
    whole batch (syz-fuzzer/fuzzer.go:494-511 per call, batched)."""
    from syzkaller_amd import signal as S

    cfg = walk_cfg(walk)
    sigs, cs, cnt, prio, nrec, npc = synth_batch(dev, cfg, 0, P, C, L)
    m0e, m0p = dev.synth_m0(cfg, KNOWN_SYS[walk], m0)
    pristine = dev.deserialize(m0e, m0p)
    del m0e, m0p
    b, _, _ = dev.batch(sigs, cs, cnt, prio, new_pairs=pairs, want_bits=False)
    ms = pristine.clone()
    ns = S.Signal.make(4_000_000, dev.eng)
    walls, chains, st = [], [], None
    for r in range(reps + 1):
        if ms.capacity() != pristine.capacity():
            ms = pristine.clone()
        else:
            ms.copy_from(pristine)
        ns.clear()
        torch.cuda.synchronize()
        t = time.perf_counter()
        st = dev.triage_b(ms, ns, b)
        torch.cuda.synchronize()
        if r:
            walls.append(time.perf_counter() - t)
            chains.append(chain_ms(st))
    wall, chain = float(np.median(walls)), float(np.median(chains))
    achieved = PROBE_BYTES_PER_REC * nrec / (chain * 1e-3) / 1e9
    wl = (f"BASELINE config 2 on SURVEY 8(d)'s global walk: {P} programs x {C} calls x {L} PCs over all 2^20 blocks "
          f"vs a {m0}-element maxSignal holding the edge universe") if walk == "global" else \
         (f"BASELINE config 2 on per-syscall region walks: {P} programs x {C} calls x {L} PCs in 256-block regions "
          f"vs a {m0}-element maxSignal holding every edge of syscalls 0..2047, one batch")
    traffic, src, note = pmc_traffic(["syz::" + k for k in K3_KERNELS.split("+")], {"workload": wl}, ("workload",),
                                     expect_ms=chain)
    del sigs, cs, cnt, prio, b
    return {"metric": "signal elems triaged/sec (Diff+Merge), " +
                      ("SURVEY 8(d) global-walk traces" if walk == "global" else "per-syscall region-walk traces"),
            "value": nrec / wall, "unit": "elems/s", "higher_is_better": True, "ms": wall * 1e3, "dtype": "u32",
            "config": {"workload": wl, "records": nrec, "pcs": npc, "distinct": st["distinct"],
                       "changed": st["changed"], "retries": st["retries"], "runs": st["runs"],
                       "parts": st["parts"], "overflow_parts": st["overflow_parts"]},
            "roofline": {"bound": "hbm", "kernel": K3_KERNELS, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
                         "traffic_note": note, "bytes_per_unit": PROBE_BYTES_PER_REC, "units_per_launch": nrec,
                         "avg_launch_ms": chain}}


def c4_rank_line(dev, sigs, cs, cnt, prio, P, C, L, walk, world=8, m0_total=1_000_000_000, reps=3):
    """BASELINE config 4 seen from one rank of an 8-GPU node, on one GPU, with
    the stream-ordered step's own calls (syzsig_step_*): (1) the source side --
    this rank's C2 batch aggregated per element, each element's staircase into
    one fixed bucket per owner (syzsig_step_send_dev); (2) the owner side --
    owner 0's LDS-partitioned replay of the buckets all 8 sources send it
    (syzsig_step_own_dev; the 8 sources' batches are synthesized here one
    after another, program ranges r*P..) against owner 0's shard of a
    1B-element maxSignal (125M elements, built with synth_m0_shard); (3) the
    flags back at this rank's source (syzsig_step_back_dev).  The two
    equal-split all-to-alls between them are not on one GPU: their bytes are
    reported.  value = this rank's records / (source + owner + back device time)."""
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth
    from syzkaller_amd._lib import STEP_HDR_COUNT
    from syzkaller_amd.dist import SIGNAL_PRIO_LEVELS

    cfg = walk_cfg(walk)
    levels = list(SIGNAL_PRIO_LEVELS)
    nrec0 = int(cnt.to(torch.int64).sum().item())

    def ev_time(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        return out, a.elapsed_time(b)

    # every source's bucket for owner 0 (a generous cap first; the step's cap is
    # then what all sources needed, as ShardedTriage agrees on it)
    cap_big = nrec0 // world + 4096
    send_big = torch.empty(world * (cap_big + 1), dtype=torch.int64, device=dev.dev)
    parts, max_out, sent_per_owner, b0 = [], 0, None, None
    for r in range(world):
        if r == 0:
            s_sigs, s_cs, s_cnt, s_prio = sigs, cs, cnt, prio
        else:
            s_sigs, s_cs, s_cnt, s_prio, _, _ = synth_batch(dev, cfg, r * P, P, C, L)
        b, _, _ = dev.batch(s_sigs, s_cs, s_cnt, s_prio, want_bits=False)
        dev.step_send(b, r * P * C, levels, world, cap_big, send_big)
        st = dev.step_finish()
        if st["global_void"] or st["src_void"] or st["max_out"] > cap_big:
            raise RuntimeError(f"c4_rank: source {r} bucket pass failed: {st}")
        max_out = max(max_out, st["max_out"])
        hdr = send_big.view(world, cap_big + 1)[:, 0].cpu().numpy().view(np.uint64) & np.uint64(STEP_HDR_COUNT)
        if r == 0:
            sent_per_owner, src_st, b0 = [int(x) for x in hdr], st, (b, s_sigs, s_cs, s_cnt, s_prio)
        parts.append(send_big[1: 1 + int(hdr[0])].clone())
        if r:
            del s_sigs, s_cs, s_cnt, s_prio, b
    del send_big
    cap = int(max_out * 1.25) + 4096
    n = world * (cap + 1)
    recv = torch.zeros(n, dtype=torch.int64, device=dev.dev)
    rv = recv.view(world, cap + 1)
    for r, x in enumerate(parts):
        rv[r, 0] = x.numel()
        rv[r, 1: 1 + x.numel()] = x
    received = sum(x.numel() for x in parts)
    del parts
    # owner 0's shard of the 1B-element M0
    se, sp = dev.synth_m0_shard(cfg, KNOWN_SYS[walk], m0_total, world, 0)
    pristine = dev.deserialize(se, sp)
    shard_len = int(se.numel())
    del se, sp
    b, s_sigs, s_cs, s_cnt, s_prio = b0
    send = torch.empty(n, dtype=torch.int64, device=dev.dev)
    flags = torch.empty(n, dtype=torch.uint8, device=dev.dev)
    back = torch.zeros(n, dtype=torch.uint8, device=dev.dev)
    src_ms, own_ms, back_ms, ost = [], [], [], None
    for rep in range(reps + 1):
        _, t_src = ev_time(lambda: dev.step_send(b, 0, levels, world, cap, send))
        dev.step_finish()
        shard = pristine.clone()
        ns = S.Signal.make(4_000_000, dev.eng)
        _, t_own = ev_time(lambda: dev.step_own(shard, ns, recv, world, cap, levels, flags))
        ost = dev.step_finish()
        # this source's flags back: owner 0's from the replay, the other owners' none
        back.view(world, cap + 1)[0].copy_(flags.view(world, cap + 1)[0])
        _, t_back = ev_time(lambda: dev.step_back(b, 0, send, world, cap, back))
        dev.step_finish()
        if rep:
            src_ms.append(t_src)
            own_ms.append(t_own)
            back_ms.append(t_back)
        del shard, ns
    if ost["global_void"] or ost["owners_void"] or ost["received"] != received:
        raise RuntimeError(f"c4_rank: the owner pass failed: {ost}")
    s_ms, o_ms, k_ms = float(np.median(src_ms)), float(np.median(own_ms)), float(np.median(back_ms))
    step = s_ms + o_ms + k_ms
    achieved = PROBE_BYTES_PER_REC * nrec0 / (step * 1e-3) / 1e9
    xbytes = 8 * (world - 1) * (cap + 1) + (world - 1) * (cap + 1)  # records out + flags back per rank
    wl = (f"BASELINE config 4, one rank of {world}: this rank's {P} x {C} x {L} {walk}-walk batch (source aggregation into "
          f"staircase buckets), owner 0's LDS-partitioned replay of what all {world} sources send it against its "
          f"{shard_len}-element shard of a {m0_total}-element maxSignal, the flags back")
    traffic, src, note = pmc_traffic(["syz::" + k for k in K3_DIST_KERNELS.split("+")], {"workload": wl},
                                     ("workload",), expect_ms=step)
    return {"metric": "signal elems triaged/sec (Diff+Merge) per rank of a 1B-element maxSignal over 8 GPUs",
            "value": nrec0 / (step * 1e-3), "unit": "elems/s", "higher_is_better": True, "dtype": "u32",
            "ms": step, "source_ms": s_ms, "owner_ms": o_ms, "back_ms": k_ms,
            "config": {"workload": wl,
                       "records": nrec0, "staircase_sent": src_st["sent"], "sent_per_owner": sent_per_owner,
                       "bucket_cap": cap, "owner_received": received, "shard_elems": shard_len,
                       "owner_parts": ost["own_parts"], "owner_distinct": ost["own_distinct"],
                       "xgmi_bytes_out": xbytes,
                       "xgmi_ms_at_7x153GBps": xbytes / (7 * 153e9) * 1e3,
                       "source_distinct": src_st["distinct"], "owner_changed": ost["changed"]},
            "roofline": {"bound": "hbm", "kernel": K3_DIST_KERNELS, "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
                         "traffic_note": note,
                         "bytes_per_unit": PROBE_BYTES_PER_REC, "units_per_launch": nrec0, "avg_launch_ms": step}}


def pipeline_line(dev, pairs, P, C, L, walk, reps=3, m0=10_000_000):
    """The per-execution path end to end on one C2 batch: raw KCOV traces in
    HBM -> K1+K2 (executor write_coverage_signal + dedup, executor.h:492-512)
    -> K3 (checkNewSignal over the batch, fuzzer.go:494-511; proc.go:230-247
    calls one after the other), timed as one sequence with HIP events, maxSignal
    back to M0 and newSignal cleared before each (outside the events)."""
    from syzkaller_amd import signal as S
    from syzkaller_amd import synth

    cfg = walk_cfg(walk)
    cl = torch.full((P * C,), L, dtype=torch.int32)
    pcs, cs, cl, prio = dev.synth_traces(cfg, 0, P, C, cl)
    pidx = torch.arange(P + 1, dtype=torch.int32, device=dev.dev) * C
    sigs = torch.empty(pcs.numel(), dtype=torch.int32, device=dev.dev)
    cnt = torch.empty(P * C, dtype=torch.int32, device=dev.dev)
    comp = torch.empty(P, dtype=torch.int32, device=dev.dev)
    m0e, m0p = dev.synth_m0(cfg, KNOWN_SYS[walk], m0)
    pristine = dev.deserialize(m0e, m0p)
    del m0e, m0p
    ms = pristine.clone()
    ns = S.Signal.make(4_000_000, dev.eng)
    b, _, _ = dev.batch(sigs, cs, cnt, prio, new_pairs=pairs, want_bits=False)
    times, st = [], None
    for r in range(reps + 1):
        if ms.capacity() != pristine.capacity():
            ms = pristine.clone()
        else:
            ms.copy_from(pristine)
        ns.clear()
        a, z = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        dev.edge_derive(pcs, cs, cl, pidx, sigs, cnt, comp)
        st = dev.triage_b(ms, ns, b)
        z.record()
        torch.cuda.synchronize()
        if r:
            times.append(a.elapsed_time(z))
    t = float(np.median(times))
    npc = pcs.numel()
    nrec = int(cnt.to(torch.int64).sum().item())
    del pcs, sigs
    return {"metric": "KCOV PCs -> checkNewSignal result per second (K1+K2 then K3 on one batch)",
            "value": npc / (t * 1e-3), "unit": "PCs/s", "higher_is_better": True, "ms": t, "dtype": "u64->u32",
            "records_per_s": nrec / (t * 1e-3),
            "config": {"workload": f"BASELINE config 2 batch: {P} programs x {C} calls x {L} PCs from raw "
                                   f"{walk}-walk traces, vs a {m0}-element maxSignal",
                       "pcs": npc, "records": nrec, "changed": st["changed"]}}


def c1_line(dev, reps=20):
    """BASELINE config 1 (64 programs x 32 calls x 2k PCs): the reference's
    CPU-runnable case, FromRaw/DiffRaw+Merge per call (checkNewSignal,
    fuzzer.go:494-511) against a 200k-element maxSignal -- the oracle on one
    core beside the GPU path on the same batch and M0."""
    from oracle import oracle as O
    from syzkaller_amd import synth

    cfg = synth.synth_default()
    P, C, L = 64, 32, 2048
    sigs, cs, cnt, prio, nrec, _ = synth_batch(dev, cfg, 0, P, C, L)
    m0e, m0p = dev.synth_m0(cfg, 2048, 200_000)
    pristine = dev.deserialize(m0e, m0p)
    b, _, _ = dev.batch(sigs, cs, cnt, prio, want_bits=False)
    from syzkaller_amd import signal as S

    wall = []
    ns = S.Signal.make(1 << 20, dev.eng)  # newSignal grabbed before every batch (storage kept: syzsig_set_clear)
    for r in range(reps + 2):
        ms = pristine.clone()  # (the batch grows maxSignal's table: a fresh copy of M0 each time)
        ns.clear()
        torch.cuda.synchronize()
        t = time.perf_counter()
        dev.triage_b(ms, ns, b)
        torch.cuda.synchronize()
        if r >= 2:
            wall.append(time.perf_counter() - t)
    g = float(np.median(wall))
    h_sigs = sigs.cpu().numpy().view(np.uint32)
    h_cs, h_cnt, h_prio = cs.cpu().numpy().view(np.uint64), cnt.cpu().numpy().view(np.uint32), prio.cpu().numpy()
    e, p = m0e.cpu().numpy().view(np.uint32), m0p.cpu().numpy()
    cpu = []
    for _ in range(3):
        oms = O.deserialize(e, p)
        t = time.perf_counter()
        O.triage_batch_into(oms, h_sigs, h_cs, h_cnt, h_prio)
        cpu.append(time.perf_counter() - t)
    c = float(np.median(cpu))
    return {"metric": "signal elems triaged/sec (Diff+Merge), BASELINE config 1", "value": nrec / g,
            "unit": "elems/s", "higher_is_better": True, "ms": g * 1e3, "dtype": "u32",
            "config": {"workload": f"BASELINE config 1: {P} programs x {C} calls x {L} PCs vs a 200000-element "
                                   "maxSignal (GPU path, wall time per batch incl. host sync)", "records": nrec},
            "cpu": {"value": nrec / c, "unit": "elems/s", "cores": 1, "kind": "port", "ms": c * 1e3,
                    "sample": "the whole C1 batch, oracle/oracle.c single thread (sequential checkNewSignal)"}}


def frame_regions(sigs, cs, cnt, prio, comp, P, C):
    """The batch as executor output regions (executor.h:566-604 records, one
    region per program; errno 22 for failed calls), built with torch ops on
    the batch's device.  Returns (out int32, prog_off int64, call index,
    published-call mask)."""
    d = sigs.device
    n = P * C
    ar = torch.arange(n, device=d)
    callidx, progidx = ar % C, ar // C
    done = callidx < comp.to(torch.int64)[progidx]
    c64 = cnt.to(torch.int64)
    L = torch.where(done, c64 + 7, torch.zeros_like(c64)).view(P, C)
    poff = torch.zeros(P + 1, dtype=torch.int64, device=d)
    poff[1:] = (L.sum(1) + 1).cumsum(0)
    roff = (poff[:-1].unsqueeze(1) + 1 + L.cumsum(1) - L).view(-1)
    out = torch.zeros(int(poff[-1].item()), dtype=torch.int32, device=d)
    out[poff[:-1]] = comp.to(torch.int32)
    p64 = prio.to(torch.int64)
    errno = torch.where(((p64 >> 1) & 1) == 0, 22, 0)
    z = torch.zeros_like(c64)
    hdr = torch.stack([callidx, callidx, errno, z, c64, z, z], 1)[done]
    out[(roff[done].unsqueeze(1) + torch.arange(7, device=d)).view(-1)] = hdr.view(-1).to(torch.int32)
    rep = c64[done]
    call_of = torch.repeat_interleave(torch.arange(rep.numel(), device=d), rep)
    within = torch.arange(call_of.numel(), device=d) - (rep.cumsum(0) - rep)[call_of]
    out[(roff[done] + 7)[call_of] + within] = sigs[cs[done][call_of] + within]
    return out, poff, callidx, done


def ingest_stage(dev, sigs, cs, cnt, prio, comp, P, C, reps=5):
    """Frame the batch as executor output regions on device (frame_regions),
    then time readOutCoverage on device (syzsig_ingest_exec_output_dev,
    pkg/ipc/ipc.go:328-468) over all of them.  Not part of `value`; reported
    as stages.ingest_ms.  Returns (ms, check_ok)."""
    d = sigs.device
    out, poff, callidx, done = frame_regions(sigs, cs, cnt, prio, comp, P, C)
    c64 = cnt.to(torch.int64)
    z = torch.zeros_like(c64)
    p64 = prio.to(torch.int64)
    any_ = ((p64 & 1) == 0).to(torch.uint8)
    pc = (torch.arange(P + 1, device=d, dtype=torch.int32) * C)
    ms = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        r = dev.ingest_exec_output(out, poff, pc, any_, callidx.to(torch.int32))
        torch.cuda.synchronize()
        ms.append((time.perf_counter() - t) * 1e3)
    exp_prio = torch.where(done, p64, p64 & 1)
    ok = (r["n_failed"] == 0 and bool((r["call_len"].to(torch.int64) == torch.where(done, c64, z)).all())
          and bool((r["call_prio"].to(torch.int64) == exp_prio).all()))
    del out
    return float(np.median(ms)), ok


def dist_parity(dev, sharded, batch, pool0, pairs, reset, ns, m0e, m0p, rank, world, P, C, backend, nprog=8):
    """Parity evidence from the sharded run itself (outside the timed region):
    one more step of batch 0 from M0 on every rank, then
      * rank 0's first `nprog` programs -- the head of the rank-major serial
        order, so their checkNewSignal result depends on M0 and their own
        records only -- against the oracle (plain-C sequential checkNewSignal,
        syz-fuzzer/fuzzer.go:494-511) over M0 restricted to their elements,
        gathered from every rank's shard: call_new and the DiffRaw pairs;
      * the newSignal shards: their union (the shards are disjoint by owner)
        holds exactly the elements the owners changed.
    The oracle is the checker here, never the thing measured."""
    import torch.distributed as dist

    from oracle import oracle as O

    cdev = dev.dev if backend == "nccl" else torch.device("cpu")
    reset()
    ns.clear()
    _, cnew, st = sharded.step(batch, pool0[3], rank * P * C)
    if dev.dev.type == "cuda":
        torch.cuda.synchronize()
    tot = torch.tensor([ns.Len(), st["changed"], st["new_pairs"], int(cnew.to(torch.int64).sum().item())],
                       dtype=torch.int64, device=cdev)
    dist.all_reduce(tot)
    ns_union, changed, npairs_all, cnew_all = (int(x) for x in tot.tolist())
    sigs, cs, cnt, prio = pool0[:4]
    npre = nprog * C
    keys = None
    if rank == 0:
        end = int(cs[npre - 1].item()) + int(cnt[npre - 1].item())
        hs = sigs[:end].cpu().numpy().view(np.uint32)
        hcs, hcnt = cs[:npre].cpu().numpy().view(np.uint64), cnt[:npre].cpu().numpy().view(np.uint32)
        hprio = prio[:npre].cpu().numpy().view(np.uint8)
        keys = np.unique(np.concatenate([hs[int(a): int(a) + int(n)] for a, n in zip(hcs, hcnt)]))
        nk = torch.tensor([keys.size], dtype=torch.int64, device=cdev)
    else:
        nk = torch.zeros(1, dtype=torch.int64, device=cdev)
    dist.broadcast(nk, 0)
    kt = torch.from_numpy(keys.view(np.int32)).to(cdev) if rank == 0 else \
        torch.empty(int(nk.item()), dtype=torch.int32, device=cdev)
    dist.broadcast(kt, 0)
    mask = torch.isin(m0e, kt.to(m0e.device))
    fe, fp = m0e[mask], m0p[mask].to(torch.int32)  # (int32 for the gather; prios are int8 values)
    n_here = torch.tensor([fe.numel()], dtype=torch.int64, device=cdev)
    ns_all = [torch.zeros_like(n_here) for _ in range(world)]
    dist.all_gather(ns_all, n_here)
    width = max(1, max(int(x.item()) for x in ns_all))
    pad_e = torch.zeros(width, dtype=torch.int32, device=cdev)
    pad_p = torch.zeros(width, dtype=torch.int32, device=cdev)
    pad_e[: fe.numel()] = fe.to(cdev)
    pad_p[: fp.numel()] = fp.to(cdev)
    ge = [torch.zeros_like(pad_e) for _ in range(world)]
    gp = [torch.zeros_like(pad_p) for _ in range(world)]
    dist.all_gather(ge, pad_e)
    dist.all_gather(gp, pad_p)
    out = {"world_size": world, "backend": backend, "checked_programs": nprog,
           "newsignal_union": ns_union, "owners_changed": changed, "union_ok": ns_union == changed,
           "new_pairs_all_ranks": npairs_all, "calls_with_new_all_ranks": cnew_all}
    if rank == 0:
        e = np.concatenate([g[: int(n.item())].cpu().numpy().view(np.uint32) for g, n in zip(ge, ns_all)])
        pr = np.concatenate([g[: int(n.item())].cpu().numpy().astype(np.int8) for g, n in zip(gp, ns_all)])
        _, _, obits, ocnew = O.triage_batch(e, pr, hs, hcs, hcnt, hprio)
        r = np.nonzero(np.unpackbits(obits.view(np.uint8), bitorder="little"))[0].astype(np.uint64)
        call = np.searchsorted(hcs.astype(np.uint64) + hcnt.astype(np.uint64), r, side="right").astype(np.uint64)
        opairs = np.unique((call << np.uint64(32)) | hs[r].astype(np.uint64))
        gpairs = pairs[: st["new_pairs"]].cpu().numpy().view(np.uint64)
        gpairs = np.unique(gpairs[gpairs < (np.uint64(npre) << np.uint64(32))])
        cnew_ok = bool(np.array_equal(cnew[:npre].cpu().numpy().view(np.uint8), ocnew))
        pairs_ok = bool(np.array_equal(gpairs, opairs))
        out.update({"m0_keys_gathered": int(e.size), "prefix_records": int(hcnt.sum()),
                    "call_new_ok": cnew_ok, "pairs_ok": pairs_ok, "pairs_checked": int(opairs.size),
                    "ok": cnew_ok and pairs_ok and ns_union == changed})
    return out


def progress(rank, msg):
    """One line per setup phase on stderr (a silent multi-minute setup looks hung)."""
    print(f"[bench rank {rank}] {msg} (t={time.perf_counter() - T0:.1f}s)", file=sys.stderr, flush=True)


T0 = time.perf_counter()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if a.gpus != 1 or world != 1:
            raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    if a.dist_backend == "gloo":
        local = local % torch.cuda.device_count()
    torch.cuda.set_device(local)
    distributed = world > 1
    if distributed:
        import torch.distributed as dist

        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    from syzkaller_amd import signal as S
    from syzkaller_amd import synth
    from syzkaller_amd.device import Device

    progress(rank, f"device {local}, world {world}")
    dev = Device(local)
    dev.L.syzsig_ctx_set_timing(dev.eng.h, 1)
    ach = achievable_bw(dev)
    cfg = walk_cfg(a.walk, skew=a.skew)
    known = KNOWN_SYS[a.walk]
    P, C, L = a.programs, a.calls, a.pcs
    NB = max(1, min(a.batches, a.steps + a.warmup))
    # ---- setup: traces -> K1+K2 (timed as a stage, not part of `value`)
    progress(rank, f"traces {P} x {C} x {L} ({a.walk} walk), batch 1 of {NB}")
    cl = torch.full((P * C,), L, dtype=torch.int32)
    pcs, cs, cl, prio = dev.synth_traces(cfg, rank * P, P, C, cl)
    pidx = torch.arange(P + 1, dtype=torch.int32, device=dev.dev) * C
    sigs = torch.empty(pcs.numel(), dtype=torch.int32, device=dev.dev)
    cnt = torch.empty(P * C, dtype=torch.int32, device=dev.dev)
    comp = torch.empty(P, dtype=torch.int32, device=dev.dev)
    edge_ms, edge_dev_ms = [], []
    for i in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        dev.edge_derive(pcs, cs, cl, pidx, sigs, cnt, comp)
        torch.cuda.synchronize()
        edge_ms.append((time.perf_counter() - t) * 1e3)
        edge_dev_ms.append(dev.L.syzsig_ctx_last_ms(dev.eng.h))
    npc = pcs.numel()
    del pcs
    nrec = int(cnt.to(torch.int64).sum().item())
    # the other batches the steps cycle through: batch j of rank r holds
    # programs (j * world + r) * P .. + P, so no step replays the previous one
    pool = [(sigs, cs, cnt, prio, nrec)]
    for j in range(1, NB):
        progress(rank, f"traces, batch {j + 1} of {NB}")
        clj = torch.full((P * C,), L, dtype=torch.int32)
        pj, csj, clj, prj = dev.synth_traces(cfg, (j * world + rank) * P, P, C, clj)
        sj, cj, _ = dev.edge_derive(pj, csj, clj, pidx)
        del pj
        pool.append((sj, csj, cj, prj, int(cj.to(torch.int64).sum().item())))
    # ---- M0 (maxSignal before the batch): 10M elements per GPU
    if distributed:
        from syzkaller_amd.dist import SIGNAL_PRIO_LEVELS, GpuShardOps, ShardedTriage

        # BASELINE config 4: one maxSignal of m0_total elements, hash-sharded;
        # each rank generates only its own shard (in index order)
        progress(rank, f"M0 shard of {a.m0_total} elements")
        m0e, m0p = dev.synth_m0_shard(cfg, known, a.m0_total, world, rank)
    else:
        m0e, m0p = dev.synth_m0(cfg, known, a.m0)
    progress(rank, f"maxSignal of {m0e.numel()} elements")
    ms = dev.deserialize(m0e, m0p)
    if a.table_hint:
        sized = S.Signal.make(a.table_hint, dev.eng)
        sized.Merge(ms)
        ms = sized
    pristine = ms.clone()
    ns = S.Signal.make(a.ns_hint, dev.eng)
    # checkNewSignal's outputs: the calls with new signal, every call's DiffRaw
    # result (pairs), maxSignal and newSignal (per-record bits are not part of
    # the reference's result and are not computed)
    # room for every pair the run can emit (4 per distinct element, <= 2048 x 5939 distinct):
    # the library writes them here directly instead of copying them after the run
    pairs = torch.empty(4 * 2048 * 5939 + 64, dtype=torch.int64, device=dev.dev)
    batches = [dev.batch(x[0], x[1], x[2], x[3], new_pairs=pairs, want_bits=False) for x in pool]
    if distributed:
        ops = GpuShardOps(dev)
        # the prio levels are fixed for the workload (signalPrio gives 0..3,
        # fuzzer.go:513-521), not agreed with a collective every step
        sharded = ShardedTriage(ops, ms, ns, levels=SIGNAL_PRIO_LEVELS)

    def reset():
        # back to M0: a copy of the whole table, or -- when that moves more bytes,
        # as for a 1B/N-element shard -- only the slots of the elements the
        # previous step changed (exactly newSignal's, cleared after each step);
        # a table that grew in the step is replaced by a fresh copy of M0
        nonlocal ms
        if ms.capacity() != pristine.capacity():
            ms = pristine.clone()
            if distributed:
                sharded.shard = ms
        elif ms.capacity() * 16 <= ns.capacity() * 16 + ns.Len() * 256:
            ms.copy_from(pristine)
        else:
            ms.restore_keys(pristine, ns)

    def step(i):
        # batch i % NB: serial base of rank r = its programs' place in the step's
        # rank-major batch
        reset()
        ns.clear()
        j = i % NB
        if distributed:
            st = dict(sharded.step(batches[j], pool[j][3], rank * P * C)[2])
            # source aggregation + staircase buckets, the owner's replay, the flags back
            st["part_ms"], st["probe_ms"], st["decide_ms"] = st["src_ms"], st["own_ms"], st["back_ms"]
        else:
            st = dev.triage_b(ms, ns, batches[j][0])
        st["nrec"] = pool[j][4]
        return st

    progress(rank, f"warmup {a.warmup}")
    for i in range(a.warmup):
        step(i)
        if distributed and ms.capacity() != pristine.capacity():
            # the owner reserved its shard for a step's worst case (bucket cap x
            # ranks): the snapshot gets the same room, so that the state reset
            # stays a restore of the changed slots
            pristine.reserve(world * sharded.cap)
    progress(rank, f"timed {a.steps}")
    stats = []
    if distributed:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        stats.append(step(a.warmup + i))
    torch.cuda.synchronize()
    if distributed:
        dist.barrier()
    dt = time.perf_counter() - t0
    total_rec = sum(s["nrec"] for s in stats)  # this rank's records over the timed steps
    reset()  # (outside the timed region: the reset brought back M0 exactly)
    restore_ok = ms.equal(pristine)
    if not restore_ok:
        raise SystemExit("bench: maxSignal was not restored to M0 between steps")
    if distributed:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev.dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        tr = torch.tensor([total_rec], dtype=torch.int64, device=dev.dev)
        dist.all_reduce(tr)
        total_rec = int(tr.item())
    parity = dist_parity(dev, sharded, batches[0], pool[0], pairs, reset, ns, m0e, m0p, rank, world, P, C,
                         a.dist_backend) if distributed else None
    ingest_ms, ingest_ok = ingest_stage(dev, sigs, cs, cnt, prio, comp, P, C) if not distributed else (None, None)
    ms_per_step = dt / a.steps * 1e3
    value = total_rec / dt
    s0 = stats[-1]
    probe_ms = float(np.mean([s["probe_ms"] for s in stats]))
    decide_ms = float(np.mean([s["decide_ms"] for s in stats]))
    part_ms = float(np.mean([s["part_ms"] for s in stats]))
    k3_ms = part_ms + probe_ms + decide_ms
    probe_units = float(np.mean([s["nrec"] for s in stats]))  # records per launch (this rank)
    # roofline over the whole K3 pipeline (every kernel between the records in
    # HBM and the updated sets), not one kernel of it
    achieved = PROBE_BYTES_PER_REC * probe_units / (k3_ms * 1e-3) / 1e9
    out = None
    if rank == 0:
        out = {
            "metric": "signal elems triaged/sec (Diff+Merge)",
            "value": value,
            "unit": "elems/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {"workload": ("BASELINE config 2: 1xMI355X batch triage, "
                                    f"{P} programs x {C} calls x {L} PCs vs a {a.m0}-element maxSignal, "
                                    + ("SURVEY 8(d)'s global-walk traces" if a.walk == "global" else
                                       "per-syscall region-walk traces") + f", {NB} distinct batches in turn")
                       if not distributed else
                       (f"BASELINE config 4: a {a.m0_total}-element maxSignal hash-sharded over {world} GPUs "
                        f"({m0e.numel()} elements on rank 0), each rank triaging {P} programs x {C} calls x {L} PCs "
                        f"(BASELINE config 2 per GPU, {a.walk}-walk traces, {NB} distinct batches in turn), staircase "
                        "records routed with RCCL all-to-all"),
                       "programs_per_gpu": P, "calls": C, "pcs_per_call": L,
                       "m0_per_gpu": a.m0 if not distributed else int(m0e.numel()),
                       "records_per_gpu": probe_units, "records_per_batch": [x[4] for x in pool],
                       "pcs_per_gpu": npc, "skew": a.skew, "walk": a.walk, "batches": NB,
                       "table_slots": ms.capacity(),
                       "parallelism": f"shard{world}" if distributed else "single",
                       **({"dist_backend": a.dist_backend, "world_size": world} if distributed else {})},
            "roofline": {"bound": "hbm",
                         "kernel": K3_KERNELS if not distributed else K3_DIST_KERNELS,
                         "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "bytes_per_unit": PROBE_BYTES_PER_REC, "units_per_launch": probe_units,
                         "avg_launch_ms": k3_ms},
            "stages": {"edge_ms": float(np.median(edge_ms)), "edge_dev_ms": float(np.median(edge_dev_ms)), "part_ms": part_ms, "agg_ms": probe_ms,
                       "finalize_ms": decide_ms,
                       "edge_pcs_per_s": npc / (np.median(edge_ms) * 1e-3),
                       "ingest_ms": ingest_ms, "ingest_check": ingest_ok},
            "triage": {k: v for k, v in s0.items() if k not in ("probe_ms", "decide_ms", "part_ms", "nrec")},
            "state_reset": "maxSignal back to M0 before every step: a table copy, or the slots of the previous "
                           "step's newSignal elements (syzsig_set_restore_keys) when that moves fewer bytes; "
                           "checked equal to M0 after the timed steps",
        }
    if rank == 0:
        traffic, src, note = pmc_traffic(["syz::" + k for k in (K3_KERNELS if not distributed else K3_DIST_KERNELS)
                                          .split("+")], out["config"], expect_ms=k3_ms)
        out["roofline"]["traffic"] = traffic
        out["roofline"]["traffic_source"] = src
        out["roofline"]["traffic_note"] = note
        # K1+K2 (executor write_coverage_signal on device) as its own line
        e_ms = float(np.median(edge_dev_ms))
        e_ach = EDGE_BYTES_PER_PC * npc / (e_ms * 1e-3) / 1e9
        e_traffic, e_src, e_note = pmc_traffic(["syz::k_edge_dedup"], out["config"], expect_ms=e_ms)
        out["lines"] = {"edge": {
            "metric": "KCOV PCs -> edge signals/sec (write_coverage_signal K1 + dedup K2)", "value": npc / (e_ms * 1e-3),
            "unit": "PCs/s", "higher_is_better": True, "ms": e_ms, "dtype": "u64->u32",
            "config": {"workload": f"BASELINE config 2 batch: {P} programs x {C} calls x {L} PCs", "pcs": npc,
                       "signals": nrec},
            "roofline": {"bound": "hbm", "kernel": "k_edge_dedup", "achieved": e_ach, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": e_ach / HBM_PEAK_GBS, "traffic": e_traffic, "traffic_source": e_src,
                         "traffic_note": e_note,
                         "bytes_per_unit": EDGE_BYTES_PER_PC, "units_per_launch": npc, "avg_launch_ms": e_ms}}}
    if rank == 0 and world == 1 and not a.no_min:
        out["lines"]["minimize"] = minimize_line(dev, a.min_contexts, cpu_s=0 if a.no_cpu else a.cpu_seconds / 3)
    if rank == 0 and world == 1 and not a.no_c5:
        out["lines"]["c5"] = c5_line(dev, pairs, cpu_s=0 if a.no_cpu else a.cpu_seconds / 3,
                                     cpu_threads=a.cpu_threads)
        # rounds 1-4's C5 input (power-skewed region walks), kept comparable
        out["lines"]["c5_region_power"] = c5_line(dev, pairs, walk="region")
    if rank == 0 and world == 1 and not a.no_pipe:
        out["lines"]["pipeline"] = pipeline_line(dev, pairs, P, C, L, a.walk)
    if rank == 0 and world == 1 and not a.no_gw:
        other = "region" if a.walk == "global" else "global"
        out["lines"][f"c2_{other}_walk"] = c2_walk_line(dev, pairs, P, C, L, other)
    if rank == 0 and world == 1 and not a.no_c1:
        out["lines"]["c1"] = c1_line(dev)
    if rank == 0 and world == 1 and not a.no_poll:
        out["lines"]["poll"] = poll_line(dev, cpu_s=0 if a.no_cpu else a.cpu_seconds / 3)
    if rank == 0 and world == 1 and not a.no_c4:
        out["lines"]["c4_rank"] = c4_rank_line(dev, sigs, cs, cnt, prio, P, C, L, a.walk)
    if rank == 0 and world == 1 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(dev, sigs, cs, cnt, prio, m0e, m0p, C, a.cpu_seconds, a.cpu_threads)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0 and distributed:
        out["parity"] = parity
    if rank == 0:
        out["achievable_bw"] = ach
        with_achievable(out["roofline"], ach)
        for ln in out["lines"].values():
            with_achievable(ln.get("roofline"), ach)
        print(json.dumps(out), flush=True)
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
