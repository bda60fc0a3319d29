/*
 * oracle.h -- CPU restatement of the reference's coverage-signal hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this code, and only as the checker
 * (or as the timed CPU baseline).  The product path (syzkaller_amd/ and
 * libsyzsig.so) never links, loads or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the upstream syzkaller tree).  Parity status:
 *   - executor half (orc_exec_program): PINNED against the reference C++
 *     executor itself, compiled from its own sources by oracle/Makefile into
 *     oracle/_ref/ref_harness; goldens in tests/golden/.
 *   - pkg/signal + checkNewSignal half: the Go reference cannot be built here
 *     (no Go toolchain in the image), and the reference holds no tests or
 *     fixtures for pkg/signal.  Pinned only by hand-derived known-answer tests
 *     (tests/kat_cases.py) => "parity partially pinned" (see DESIGN.md).
 */
#ifndef SYZSIG_ORACLE_H
#define SYZSIG_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- executor half: executor/executor.h:492-512, :677-706, executor_linux.cc:196-204 ---- */

uint32_t orc_exec_hash(uint32_t a);           /* executor.h:677-685 */
int orc_cover_check(uint64_t pc);             /* executor_linux.cc:196-204 (x86_64) */

/*
 * One program, as one forked executor child (dedup table zeroed, common_linux.h:1995-2030):
 * for call c in order, write_coverage_signal<uint64> over pcs[call_start[c] .. +call_len[c]).
 * Emitted signals of call c are written to out_sig[call_start[c] + i] (i < out_cnt[c]).
 * *completed = number of calls whose record was published (a cover_check failure
 * aborts the program: executor.h:502-503).  Calls >= *completed get out_cnt = 0.
 */
void orc_exec_program(const uint64_t* pcs, const uint64_t* call_start, const uint32_t* call_len,
                      uint32_t ncalls, uint32_t* out_sig, uint32_t* out_cnt, uint32_t* completed);

/* ---- pkg/signal: Signal map[uint32]int8 (pkg/signal/signal.go:11-21) ---- */

typedef struct orc_sig orc_sig;  /* NULL == Go nil map */

orc_sig* orc_sig_new(uint64_t hint);
void orc_sig_free(orc_sig* s);
uint64_t orc_sig_len(const orc_sig* s);                                   /* signal.go:23 */
int orc_sig_get(const orc_sig* s, uint32_t e, int8_t* p);                 /* map lookup */
orc_sig* orc_from_raw(const uint32_t* raw, uint64_t n, uint8_t prio);    /* signal.go:31 */
uint64_t orc_serialize(const orc_sig* s, uint32_t* elems, int8_t* prios);/* signal.go:42 */
/* returns -1 ("corrupted Serial" panic) on length mismatch; signal.go:59 */
int orc_deserialize(const uint32_t* elems, uint64_t ne, const int8_t* prios, uint64_t np,
                    orc_sig** out);
orc_sig* orc_diff(const orc_sig* s, const orc_sig* s1);                  /* signal.go:73 */
orc_sig* orc_diff_raw(const orc_sig* s, const uint32_t* raw, uint64_t n, uint8_t prio); /* :90 */
orc_sig* orc_intersection(const orc_sig* s, const orc_sig* s1);          /* signal.go:104 */
void orc_merge(orc_sig** s, const orc_sig* s1);                           /* signal.go:117 */

/*
 * signal.go:138-166 Minimize.  Contexts are given as Serial arrays
 * (elems/prios at ctx_off[i]..ctx_off[i+1], distinct elements per context).
 * sort.Slice is unstable in the reference; the restatement fixes the order as
 * (Len desc, input index asc).  Writes winning INPUT indices ascending to out_idx,
 * returns their count.
 */
uint64_t orc_minimize(const uint64_t* ctx_off, const uint32_t* elems, const int8_t* prios,
                      uint64_t nctx, uint64_t* out_idx);

/*
 * Batch restatement of syz-fuzzer/fuzzer.go:494-511 checkNewSignal, applied to
 * every call of a batch in serial order (program-major, call-index minor).
 * For call k: diff = max.DiffRaw(sig_k, prio_k); if non-empty: call_new[k] = 1,
 * max.Merge(diff), newsig.Merge(diff).  new_bits bit r (r = record index into
 * sigs[]) is set iff sigs[r] is in its call's diff.
 */
void orc_triage_batch(orc_sig** max_signal, orc_sig** new_signal, const uint32_t* sigs,
                      const uint64_t* call_start, const uint32_t* call_len, const uint8_t* call_prio,
                      uint64_t ncalls, uint32_t* new_bits, uint8_t* call_new);

/*
 * The multi-core CPU baseline: fuzzer.go:494-511 as `nthreads` Procs run it
 * (fuzzer.go:288-295), program p = calls [p*calls_per_prog, (p+1)*calls_per_prog),
 * DiffRaw under a reader lock, Merge under the writer lock (pthread rwlock =
 * signalMu).  Returns the number of calls that reported new signal.
 */
uint64_t orc_triage_batch_mt(orc_sig** max_signal, orc_sig** new_signal, const uint32_t* sigs,
                             const uint64_t* call_start, const uint32_t* call_len, const uint8_t* call_prio,
                             uint64_t nprog, uint64_t calls_per_prog, uint32_t nthreads);

/* Test helper: the Serial entries whose element is in keys[] (input order kept). */
uint64_t orc_filter_keys(const uint32_t* elems, const int8_t* prios, uint64_t n, const uint32_t* keys,
                         uint64_t nkeys, uint32_t* out_e, int8_t* out_p);

#ifdef __cplusplus
}
#endif
#endif
