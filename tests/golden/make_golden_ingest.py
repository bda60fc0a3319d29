"""Generate the executor-output-region golden vectors (pkg/ipc readOutCoverage input).

Run in the build container (needs /root/reference and `make -C oracle ref`):
    python tests/golden/make_golden_ingest.py
The regions are written by the REFERENCE executor itself (oracle/_ref/ref_harness
drives executor.h:530-608 handle_completion, which frames every completed call's
record exactly as the executor's shmem out file holds it).  Expected parse
results come from the readOutCoverage restatement (oracle.read_out_coverage,
ipc.go:328-468; the Go reference cannot run here, no Go toolchain) and are
cross-checked against the harness's own record walk.  The fixture also holds
hand-corrupted regions, one per ipc.go error branch.
Fixture tests/golden/ingest/exec_regions.npz (plain arrays, allow_pickle=False):
  out u32[], prog_off u64[nprog+1], prog_call u32[nprog+1], call_num u32[], call_any u8[],
  exp_call_start u64[], exp_call_len u32[], exp_call_prio u8[], exp_call_errno i32[], exp_status i32[]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle import oracle as O  # noqa: E402
from syzkaller_amd import synth  # noqa: E402
from make_golden import synth_programs  # noqa: E402


def corrupt(region, rng):
    """One hand-corrupted copy of a well-formed region per ipc.go error branch: (region, ncalls, call_num)."""
    r = [int(x) for x in region]
    nc = 8
    cases = []
    cases.append(([], nc))                                    # no ncmd (ipc.go:356-359)
    cases.append((r[:1 + 3], nc))                             # short header (:378-383)
    bad = list(r); bad[1] = nc + 5; cases.append((bad, nc))   # callIndex >= len(p.Calls) (:384-388)
    bad = list(r); bad[2] = 999; cases.append((bad, nc))      # callNum mismatch (:389-395)
    first_len = 7 + r[5] + r[6]
    bad = list(r); bad[0] += 1
    bad += r[1:1 + first_len]                                  # the first record again: double coverage (:396-400)
    cases.append((bad, nc))
    bad = list(r[:1 + first_len]); bad[0] = 1; bad[5] = len(bad) + 10; cases.append((bad, nc))  # signal past end
    bad = list(r[:1 + first_len]); bad[0] = 1; bad[6] = 3; cases.append((bad, nc))               # cover past end
    # comparisons: a valid 8-byte and 4-byte comp, then variants with a bad type / short operands
    rec = [0, 0, 0, 0, 2, 1, 2, 0x81000000, 0x81000005, 0xAB, 6, 1, 2, 3, 4, 1, 7, 8]
    cases.append(([1] + rec, nc))                              # well-formed with comps
    bad = list(rec); bad[10] = 8; cases.append(([1] + bad, nc))   # comp type > 7 (:429-433)
    cases.append(([1] + rec[:-1], nc))                         # short comp operand (:436-445)
    cases.append(([1] + rec[:10], nc))                         # missing comp record (:420-425)
    # empty signal record counts as present: a second record for it is a double
    cases.append(([2, 3, 3, 0, 0, 0, 0, 0, 3, 3, 0, 0, 0, 0, 0], nc))
    cases.append(([2, 3, 3, 0, 0, 0, 0, 0, 4, 4, 5, 0, 0, 0, 0], nc))  # ok: errno 5, two empty calls
    cases.append(([0], nc))                                    # nothing executed
    cases.append(([0], 0))                                     # program with no calls
    return cases


def main():
    rng = np.random.default_rng(20181015)
    progs = synth_programs(synth.synth_default(), 10, 8, (0, 3000), 21, prog_base=500)
    progs += synth_programs(synth.synth_default(bad_pc_ppm=400), 6, 8, (0, 3000), 22, prog_base=700)
    regions = O.run_reference_executor(progs, raw=True)
    parsed = O.run_reference_executor(progs)
    ncalls = [len(p) for p in progs]
    # cross-check the restatement against the harness's own walk of the records
    for reg, (completed, calls), nc in zip(regions, parsed, ncalls):
        st, info = O.read_out_coverage(reg, nc, list(range(nc)))
        assert st == 0
        assert sum(i is not None for i in info) == completed
        for idx, err, sigs in calls:
            e, so, sl, _, _ = info[idx]
            assert e == err and np.array_equal(np.asarray(reg[so:so + sl], np.uint32), sigs)
    call_num = [list(range(nc)) for nc in ncalls]
    for reg, nc in corrupt(regions[0], rng):
        regions.append(np.asarray(reg, np.uint32))
        ncalls.append(nc)
        call_num.append(list(range(nc)))
    call_num = np.array([x for cn in call_num for x in cn], np.uint32)
    call_any = (rng.random(call_num.size) < 0.1).astype(np.uint8)
    out, po, pc, cs, cl, cp, ce, st = O.ingest_batch(regions, ncalls, call_any, call_num)
    np.savez_compressed(os.path.join(HERE, "ingest", "exec_regions.npz"), out=out, prog_off=po, prog_call=pc,
                        call_num=call_num, call_any=call_any, exp_call_start=cs, exp_call_len=cl,
                        exp_call_prio=cp, exp_call_errno=ce, exp_status=st)
    print(f"exec_regions: {len(regions)} programs, {pc[-1]} calls, {out.size} words, "
          f"{int(cl.sum())} signals, status {st.tolist()}")


if __name__ == "__main__":
    main()
