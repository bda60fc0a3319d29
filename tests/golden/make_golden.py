"""Generate the executor golden vectors from the REFERENCE executor itself.

Run in the build container (needs /root/reference and `make -C oracle ref`):
    python tests/golden/make_golden.py [fixture names]
Inputs are synthetic KCOV traces (the engine's deterministic generator plus
hand-crafted corner cases); expected outputs are the per-call signal records
written by the reference's own handle_completion -> write_coverage_signal
(executor/executor.h:492-608), compiled from its sources by oracle/Makefile.
Each fixture is an .npz of plain arrays (load with allow_pickle=False):
  pcs u64[], call_start u64[], call_len u32[], call_failed u8[], prog_call u32[]
  exp_sigs u32[] (call c's signals at call_start[c]..+exp_cnt[c]; 0 elsewhere),
  exp_cnt u32[], exp_completed u32[], exp_errno u32[] (per call; 0 if unpublished)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from syzkaller_amd import synth  # noqa: E402

KERNEL_LO, KERNEL_HI = 0x80000000, 0xFF000000  # low 32 bits allowed by cover_check


def exec_hash(a):
    a &= 0xFFFFFFFF
    a = (a ^ 61) ^ (a >> 16)
    a = (a + (a << 3)) & 0xFFFFFFFF
    a ^= a >> 4
    a = (a * 0x27D4EB2D) & 0xFFFFFFFF
    a ^= a >> 15
    return a


def craft_call(targets, start_low=0x81000000):
    """PCs whose derived signals are exactly `targets` after the first PC
    (sig_0 = pc_0).  Searches pc_0 so that every PC passes cover_check."""
    for p0 in range(start_low, start_low + 5 * 200000, 5):
        pcs, prev = [p0], p0
        ok = True
        for t in targets:
            lo = t ^ exec_hash(prev)
            if not (KERNEL_LO <= lo < KERNEL_HI):
                ok = False
                break
            pcs.append(lo)
            prev = lo
        if ok:
            return np.array([0xFFFFFFFF00000000 | x for x in pcs], dtype=np.uint64)
    raise RuntimeError("no pc_0 found")


def craft_free(targets, seed, far=(2048, 6144)):
    """Like craft_call, for chains of any length: where the next target's PC
    would fail cover_check, a free PC is put in between whose own signal is a
    fresh value homed in `far` (away from the slots under test; it changes no
    window there).  sig_0 = pc_0 is homed in `far` too."""
    rng = np.random.default_rng(seed)
    valid = lambda lo: KERNEL_LO <= lo < KERNEL_HI  # noqa: E731
    used = set(int(t) for t in targets)

    def free_pc(prev, nxt):
        for _ in range(100000):
            p = int(rng.integers(KERNEL_LO, KERNEL_HI))
            s = p ^ (exec_hash(prev) if prev is not None else 0)
            if far[0] <= s % 8192 < far[1] and s not in used and (nxt is None or valid(nxt ^ exec_hash(p))):
                used.add(s)
                return p
        raise RuntimeError("no free pc")

    pcs = [free_pc(None, None)]
    prev = pcs[0]
    for t in targets:
        lo = int(t) ^ exec_hash(prev)
        if not valid(lo):
            pcs.append(free_pc(prev, int(t)))
            prev = pcs[-1]
            lo = int(t) ^ exec_hash(prev)
        pcs.append(lo)
        prev = lo
    return np.array([0xFFFFFFFF00000000 | x for x in pcs], dtype=np.uint64)


def zero_stress_programs(nprog, seed):
    """Programs for the sig == 0 rule of K2 (csrc/edge.hip header): a fill
    call that sets slots 8184..8 to random values homed there (or leaves them
    empty), then calls dense in sig == 0 and in signals homed at 8184..8, with
    few distinct values, so forced overwrites, zero writes (slot 0 emptied)
    and re-inserts meet inside one 256-signal chunk."""
    rng = np.random.default_rng(seed)
    M = 8192
    homes = list(range(M - 8, M)) + list(range(0, 9))
    progs = []
    for p in range(nprog):
        dens = [0.0, 0.5, 0.9, 1.0][p % 4]
        fill = [int(rng.integers(1, 6)) * M + h for h in homes if rng.random() < dens]
        calls = [(False, craft_free(fill, seed * 1000 + p * 10))] if fill else []
        vals = np.array([0] + [k * M + h for h in homes for k in range(1, 4)], np.uint64)
        pr = np.full(vals.size, 1.0)
        pr[0] = [2.0, 6.0, 20.0][p % 3]
        pr /= pr.sum()
        for c in range(3):
            tg = vals[rng.choice(vals.size, int(rng.integers(40, 200)), p=pr)]
            calls.append((False, craft_free(tg.tolist(), seed * 1000 + p * 10 + c + 1)))
        progs.append(calls)
    return progs


def pack(programs):
    """programs = [[(failed, pcs), ...], ...] -> flat arrays"""
    pcs, cs, cl, cf, pc = [], [], [], [], [0]
    pos = 0
    for prog in programs:
        for failed, p in prog:
            p = np.asarray(p, np.uint64)
            pcs.append(p)
            cs.append(pos)
            cl.append(p.size)
            cf.append(int(failed))
            pos += p.size
        pc.append(pc[-1] + len(prog))
    return dict(pcs=np.concatenate(pcs) if pcs else np.empty(0, np.uint64), call_start=np.array(cs, np.uint64),
                call_len=np.array(cl, np.uint32), call_failed=np.array(cf, np.uint8), prog_call=np.array(pc, np.uint32))


def expected(fx, programs):
    ref = O.run_reference_executor(programs)
    n = fx["call_len"].size
    sigs = np.zeros(fx["pcs"].size, np.uint32)
    cnt = np.zeros(n, np.uint32)
    err = np.zeros(n, np.uint32)
    comp = np.zeros(len(programs), np.uint32)
    for p, (completed, calls) in enumerate(ref):
        comp[p] = completed
        for idx, e, rs in calls:
            c = int(fx["prog_call"][p]) + idx
            s = int(fx["call_start"][c])
            sigs[s: s + rs.size] = rs
            cnt[c] = rs.size
            err[c] = e
    return dict(exp_sigs=sigs, exp_cnt=cnt, exp_completed=comp, exp_errno=err)


def synth_programs(cfg, nprog, cpp, ragged, seed, prog_base=0):
    cl = synth.call_lengths(nprog, cpp, 0, ragged=ragged, seed=seed)
    if nprog * cpp > 1:
        cl[3::7] = 0  # calls without coverage (empty KCOV buffer)
    pcs, cs, prio = synth.traces(cfg, prog_base, nprog, cpp, cl)
    progs = []
    for p in range(nprog):
        progs.append([(((prio[c] >> 1) & 1) == 0, pcs[cs[c]: cs[c] + cl[c]]) for c in range(p * cpp, (p + 1) * cpp)])
    return progs


def main(only=None):
    """Writes every fixture, or only those named on the command line."""
    out = {}
    # 1. the survey's KAT: call 0 gives 4 signals (one dup dropped), the same trace
    #    as call 1 gives none (the dedup table is shared across a program's calls)
    kat = np.array([0xFFFFFFFF81000010, 0xFFFFFFFF81000020, 0xFFFFFFFF81000010, 0xFFFFFFFF81000020,
                    0xFFFFFFFF81000030], np.uint64)
    out["executor_kat"] = [[(False, kat), (True, kat)]]
    # 2. synthetic programs, ragged calls incl. empty ones; default and wide
    #    (heavily lossy dedup) regions
    out["executor_synth"] = synth_programs(synth.synth_default(), 6, 8, (0, 4000), 11)
    out["executor_wide"] = synth_programs(synth.synth_default(region_log2=12), 6, 8, (0, 4000), 12, prog_base=100)
    # 3. programs aborted by an out-of-range PC (cover_check -> doexit(0))
    out["executor_abort"] = synth_programs(synth.synth_default(bad_pc_ppm=300), 8, 8, (0, 3000), 13, prog_base=200)
    # 4. sig == 0: a dup while slots 0..3 are not all taken; EMITTED (and slot 0
    #    cleared) once slots 0..3 hold 8192..8195; then 8192 is re-emitted
    zero_dup = craft_call([0, 5, 0])
    zero_emit = craft_call([8192, 8193, 8194, 8195, 0, 8192, 0, 8196])
    out["executor_zero"] = [[(False, zero_dup)], [(False, zero_emit), (False, zero_emit)]]
    # 4b. sig == 0 inside one round-chunk (the round-4 verdict's case: after
    #    8192, 8193, 16384, 8195 fill slots 0..3, 0 is emitted and empties slot
    #    0, so the next 16384 is a new insert at slot 0), the same with the later
    #    lane homed at 8190 / 8191, an earlier lane blocked across a zero write,
    #    an overwrite of a match that lies after the emptied slot 0, and
    #    randomized zero-heavy programs
    out["executor_zero2"] = [
        [(False, craft_call([8192, 8193, 16384, 8195, 0, 16384]))],
        [(False, craft_free([16382, 16383, 24574, 8193, 8194, 8195, 0, 24574], 1))],
        [(False, craft_free([16383, 24575, 8193, 8194, 8195, 0, 24575], 2))],
        [(False, craft_free([8192, 8193, 8194, 32771, 16383], 3)), (False, craft_free([32766, 16382, 0], 4))],
        [(False, craft_free([40960, 40961, 40963, 8196, 24568, 32761, 16380, 40958], 5)),
         (False, craft_free([32768, 16377, 24580, 16376, 0, 24574, 24570, 24573, 32768, 32770], 6))],
    ] + zero_stress_programs(16, 7)
    # 5. a call at the per-call limit region boundary (kCoverSize - 1 PCs)
    big = synth_programs(synth.synth_default(region_log2=14), 1, 1, (262143, 262143), 14, prog_base=300)
    out["executor_big"] = big
    for name, programs in out.items():
        if only and name not in only:
            continue
        fx = pack(programs)
        fx.update(expected(fx, programs))
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **fx)
        print(f"{name}: {len(programs)} programs, {fx['call_len'].size} calls, {fx['pcs'].size} PCs, "
              f"{int(fx['exp_cnt'].sum())} signals, completed {fx['exp_completed'].tolist()}")


if __name__ == "__main__":
    main(sys.argv[1:] or None)
