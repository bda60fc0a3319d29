/*
 * syzsig.h -- C ABI of libsyzsig, the MI355X coverage-signal triage engine.
 *
 * This is the drop-in boundary for syzkaller's per-execution coverage-signal
 * path.  Each entry point names the reference interface it replaces
 * (paths relative to the upstream syzkaller tree); INTEGRATION.md shows the
 * cgo binding that keeps pkg/signal's Go API and its callers unchanged.
 *
 * Conventions
 *  - Every function returns int status: SYZSIG_OK (0) or a negative errno-style
 *    code; syzsig_last_error() gives a message (thread-local).
 *  - A `syzsig_set*` is a device-resident Signal.  NULL is Go's nil Signal:
 *    Len()==0, usable as a receiver, and syzsig_merge allocates it
 *    (signal.go:121-125).  Results that Go returns as nil come back as NULL.
 *  - Host arrays passed in are copied during the call and never retained (cgo
 *    pointer rules; CallInfo.Signal aliases executor shmem, pkg/ipc/ipc.go:410).
 *  - Threading: every entry point locks its context for the duration of the
 *    call, so concurrent readers -- Diff / DiffRaw / Intersection / Len from
 *    several goroutines under fuzzer.signalMu.RLock (syz-fuzzer/fuzzer.go:
 *    488-498) -- are safe and see consistent results.  Writers (Merge, triage)
 *    still need the caller's write lock for Go-level atomicity of their
 *    read-modify-write sequences, exactly as in the reference (signalMu.Lock,
 *    fuzzer.go:500-505; mgr.mu, syz-manager/manager.go:66).  A set must not be
 *    freed while another thread uses it.
 *  - "_dev" / batch entry points take device pointers and run on the context's
 *    stream (syzsig_ctx_set_stream); they return after the work completes.
 */
#ifndef SYZSIG_H
#define SYZSIG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SYZSIG_OK 0
#define SYZSIG_EIO (-5)        /* HIP runtime / device error */
#define SYZSIG_ENOMEM (-12)
#define SYZSIG_EINVAL (-22)
#define SYZSIG_ERANGE (-34)    /* a size limit of this ABI exceeded */
#define SYZSIG_ECORRUPT (-74)  /* panic("corrupted Serial"), pkg/signal/signal.go:60-62 */

#define SYZSIG_ABI_VERSION 4

typedef struct syzsig_ctx syzsig_ctx;
typedef struct syzsig_set syzsig_set;

int syzsig_abi_version(void);
const char* syzsig_last_error(void);

/* ---- context: one per process and GPU ---- */
int syzsig_ctx_create(int device, syzsig_ctx** out);
void syzsig_ctx_destroy(syzsig_ctx* ctx);
/* Run subsequent work on `stream` (a hipStream_t; NULL = the context's own,
 * which is a blocking stream: ordered against the null stream both ways). */
int syzsig_ctx_set_stream(syzsig_ctx* ctx, void* stream);
void* syzsig_ctx_stream(syzsig_ctx* ctx);
/* Record HIP events around the triage kernels (batch stats probe_ms/decide_ms). */
int syzsig_ctx_set_timing(syzsig_ctx* ctx, int enable);
/* With timing on: device time (ms, HIP events on the context stream) of the
 * kernels of the last syzsig_edge_derive_dev / syzsig_minimize_dev call, or the
 * stream work of the last syzsig_manager_poll_batch call (uploads to its last
 * kernel, including the host round trips between). */
double syzsig_ctx_last_ms(syzsig_ctx* ctx);
/* Measurement: a plain device copy of `bytes` (16-B aligned buffers and size)
 * on the context stream, 16 B per lane per step; *ms = its device time (HIP
 * events).  The achievable-bandwidth companion of the bench's rooflines
 * (SURVEY.md 8(d)); not part of pkg/signal.  Synchronises. */
int syzsig_copy_bw_dev(syzsig_ctx* ctx, void* d_dst, const void* d_src, uint64_t bytes, double* ms);
/* Page-locked host memory (hipHostMalloc): host arrays handed to the library
 * from it are uploaded by DMA without a staging copy (the manager's Poll
 * batch builds its Serials there).  *out = NULL for 0 bytes; free with
 * syzsig_host_free (NULL is a no-op). */
int syzsig_host_alloc(syzsig_ctx* ctx, uint64_t bytes, void** out);
int syzsig_host_free(syzsig_ctx* ctx, void* p);
/* Large-batch triage path selection (tests and tuning; results never depend on it):
 * mode 0 = per-call probe path only, 1 = aggregation path for runs of >= 2^20
 * records (default), 2 = aggregation path always; parts = fixed partition
 * count of the aggregation path (0 = adaptive, else 8..2048). */
int syzsig_ctx_set_agg(syzsig_ctx* ctx, int mode, uint32_t parts);

/* Test knobs that change the code path but never the results:
 * SYZSIG_DEBUG_FIN_DEFER = the batch finalize sends every element whose probe
 * sequence leaves its home bucket to the atomic (deferred) path;
 * SYZSIG_DEBUG_MIN_ATOMIC = Minimize takes its per-entry atomicMax path instead
 * of the aggregation path;
 * SYZSIG_DEBUG_EXACT_CELLS = large triage runs partition records into counted
 * cells (count pass + scan) instead of capped cells;
 * SYZSIG_DEBUG_RECS_GATE = the LDS-partitioned records path (records mode,
 * the owner side of a sharded step) reports every input as over its capacity,
 * so the per-record path and the step's owner fix-up run (tests).
 * SYZSIG_DEBUG_CAP_SPILL = capped cells of 64 records, so that dense runs
 * overflow them and take the redo with counted cells.
 * SYZSIG_DEBUG_EDGE_MARKALL / SYZSIG_DEBUG_EDGE_PASSES = syzsig_edge_derive_dev
 * runs the dedup rounds with one marking pass / with marking passes, instead
 * of choosing from the previous launch's duplicate rate.
 * SYZSIG_DEBUG_AGG_IDX64 = the aggregation reads its records with 64-bit
 * indices, the path of runs whose cells reach past record 2^32 (tests).
 * Fault injection (an error, never a wrong result):
 * SYZSIG_DEBUG_POLL_FAIL = the sequential Poll loop (syzsig_manager_poll_batch's
 * exact fallback) fails with SYZSIG_EIO before its last poll, so tests can
 * check that a failed batch leaves every set as it was. */
#define SYZSIG_DEBUG_FIN_DEFER 32u
#define SYZSIG_DEBUG_MIN_ATOMIC 64u
#define SYZSIG_DEBUG_EXACT_CELLS 128u
#define SYZSIG_DEBUG_CAP_SPILL 256u
#define SYZSIG_DEBUG_RECS_GATE 512u
#define SYZSIG_DEBUG_EDGE_MARKALL 1024u
#define SYZSIG_DEBUG_EDGE_PASSES 2048u
#define SYZSIG_DEBUG_POLL_FAIL 4096u
#define SYZSIG_DEBUG_AGG_IDX64 8192u
int syzsig_ctx_set_debug(syzsig_ctx* ctx, uint32_t flags);

/* ---- pkg/signal/signal.go ---- */

/* make(Signal, hint): an empty, non-nil Signal. */
int syzsig_set_make(syzsig_ctx* ctx, uint64_t hint, syzsig_set** out);
void syzsig_set_free(syzsig_set* s);
/* Deep copy (Go copies alias; this is for callers that need a snapshot). */
int syzsig_set_clone(syzsig_ctx* ctx, const syzsig_set* s, syzsig_set** out);
/* Make s empty keeping its storage (grabNewSignal's `fuzzer.newSignal = nil`,
 * syz-fuzzer/fuzzer.go:478-486, without a free/alloc round trip). */
int syzsig_set_clear(syzsig_ctx* ctx, syzsig_set* s);
/* Copy src's contents over dst (same capacity required); for snapshot/restore. */
int syzsig_set_copy_from(syzsig_ctx* ctx, syzsig_set* dst, const syzsig_set* src);
/* Restore dst to the snapshot src it was copied from, given `keys`: a set
 * holding every element whose slot in dst changed since (the newSignal of the
 * batches triaged since, when it was empty at the snapshot).  Only those slots
 * are copied back, so the cost follows the changes, not the table.  Same
 * capacity required (SYZSIG_EINVAL if dst grew).  Stream-ordered. */
int syzsig_set_restore_keys(syzsig_ctx* ctx, syzsig_set* dst, const syzsig_set* src, const syzsig_set* keys);
/* Grow s (if needed) so that `extra` more elements fit under the default load
 * policy -- what a triage call reserves for its worst case; a caller that
 * keeps a snapshot of a set reserves the snapshot alike to keep capacities
 * equal (syzsig_set_restore_keys). */
int syzsig_set_reserve(syzsig_ctx* ctx, syzsig_set* s, uint64_t extra);
/* *equal = 1 iff a and b have the same capacity, length and slot words. */
int syzsig_set_equal(syzsig_ctx* ctx, const syzsig_set* a, const syzsig_set* b, int* equal);
/* Len / Empty, signal.go:23-29. */
uint64_t syzsig_len(const syzsig_set* s);
int syzsig_empty(const syzsig_set* s);
/* Capacity in slots (diagnostics, bench accounting). */
uint64_t syzsig_capacity(const syzsig_set* s);

/* FromRaw, signal.go:31-40 (NULL when n == 0). */
int syzsig_from_raw(syzsig_ctx* ctx, const uint32_t* raw, uint64_t n, uint8_t prio, syzsig_set** out);
/* Serialize, signal.go:42-57.  Order is unspecified (Go: map order).  Writes
 * min(cap, Len) entries and sets *n_out = Len. */
int syzsig_serialize(syzsig_ctx* ctx, const syzsig_set* s, uint32_t* elems, int8_t* prios,
                     uint64_t cap, uint64_t* n_out);
/* Serialize of many sets at once (the manager serializes every Poll reply,
 * manager.go:1049 r.MaxSignal = f.newMaxSignal.Serialize()): one round of
 * kernels and one copy for all of them.  offs[0..nsets] = the sets' Len
 * prefix sums (a NULL set is empty); set i's entries land in
 * elems/prios[offs[i], offs[i+1]).  cap == 0 fills offs only (sizing); a cap
 * below offs[nsets] is SYZSIG_ERANGE. */
int syzsig_serialize_batch(syzsig_ctx* ctx, const syzsig_set* const* sets, uint64_t nsets, uint32_t* elems,
                           int8_t* prios, uint64_t cap, uint64_t* offs);
/* Deserialize, signal.go:59-71: SYZSIG_ECORRUPT if n_elems != n_prios; NULL
 * when empty; a later duplicate element overwrites an earlier one. */
int syzsig_deserialize(syzsig_ctx* ctx, const uint32_t* elems, uint64_t n_elems, const int8_t* prios,
                       uint64_t n_prios, syzsig_set** out);
/* Same, elems/prios already in device memory. */
int syzsig_deserialize_dev(syzsig_ctx* ctx, const uint32_t* d_elems, const int8_t* d_prios, uint64_t n,
                           syzsig_set** out);
/* Diff, signal.go:73-88 (s may be NULL). */
int syzsig_diff(syzsig_ctx* ctx, const syzsig_set* s, const syzsig_set* s1, syzsig_set** out);
/* DiffRaw, signal.go:90-102 (prio compared as int8). */
int syzsig_diff_raw(syzsig_ctx* ctx, const syzsig_set* s, const uint32_t* raw, uint64_t n, uint8_t prio,
                    syzsig_set** out);
/* Intersection, signal.go:104-115: NULL if s1 empty, else non-nil (maybe empty). */
int syzsig_intersection(syzsig_ctx* ctx, const syzsig_set* s, const syzsig_set* s1, syzsig_set** out);
/* (*Signal).Merge, signal.go:117-131: max prio; allocates *s if NULL. */
int syzsig_merge(syzsig_ctx* ctx, syzsig_set** s, const syzsig_set* s1);

/* Minimize, signal.go:133-166.  Contexts as Serial arrays: context i owns
 * elems/prios[ctx_off[i] .. ctx_off[i+1]) (elements distinct within a context,
 * as Serialize produces).  Sort order is (Len desc, index asc) -- a fixed
 * instance of the reference's unstable sort.Slice.  Writes the indices of the
 * surviving contexts, ascending, to out_idx (capacity nctx); *n_out = count.
 * hint_distinct: expected distinct elements (e.g. corpusSignal.Len()), or 0. */
int syzsig_minimize(syzsig_ctx* ctx, const uint64_t* ctx_off, const uint32_t* elems, const int8_t* prios,
                    uint64_t nctx, uint64_t hint_distinct, uint64_t* out_idx, uint64_t* n_out);
/* Same over device arrays; d_keep[i] = 1 iff context i survives. */
int syzsig_minimize_dev(syzsig_ctx* ctx, const uint64_t* d_ctx_off, const uint32_t* d_elems,
                        const int8_t* d_prios, uint64_t nctx, uint64_t hint_distinct, uint8_t* d_keep,
                        uint64_t* n_out);

/* ---- syz-manager/manager.go:1027-1052 Manager.Poll, over a batch of polls ----
 * Poll i (arrival order) comes from fuzzer poll_fuzzer[i] (< nfuzzers) with the
 * Serial a.MaxSignal = elems/prios[poll_off[i] .. poll_off[i+1]) (Deserialize
 * rules, signal.go:59-71: a later duplicate overwrites).  The result is the
 * reference's sequential loop over the polls:
 *   newMax := maxSignal.Diff(Deserialize(a.MaxSignal)); maxSignal.Merge(newMax);
 *   every other fuzzer's newMaxSignal.Merge(newMax);
 *   reply = the polling fuzzer's newMaxSignal, which becomes nil.
 * new_max[g] = fuzzer g's newMaxSignal (NULL = nil): a polling fuzzer's set is
 * freed (nil) and may be replaced by a new one.  replies[i] = poll i's
 * r.MaxSignal as a set (NULL = empty Serial) for the caller to Serialize and
 * free.  Host arrays (the RPC payloads).
 * Limits of one call (SYZSIG_ERANGE, nothing touched): npolls + nfuzzers <
 * 2^24 - 1, npolls * nfuzzers <= 2^28, total entries * nfuzzers <= 2^31.  A
 * caller splits a larger batch into consecutive calls (the loop is sequential,
 * so that is the same result: signal.py manager_poll does).  A call of more
 * than 2^23 entries, or whose entries crowd one element partition past 2048
 * (a hot element in thousands of polls), runs the reference loop poll by poll
 * over the set ops instead of the batch kernels (same result, slower). */
int syzsig_manager_poll_batch(syzsig_ctx* ctx, syzsig_set** max_signal, syzsig_set** new_max, uint32_t nfuzzers,
                              const uint32_t* poll_fuzzer, const uint64_t* poll_off, const uint32_t* elems,
                              const int8_t* prios, uint32_t npolls, syzsig_set** replies);

/* Minimize sharded by element (one process per GPU): shard `shard` of
 * `nshards` takes only the entries whose element it owns (owner_of, as the
 * sharded maxSignal) over the whole corpus description (same ctx_off order on
 * every shard); d_keep[i] = 1 iff context i wins one of the shard's elements.
 * The OR (max) of d_keep over the shards is syzsig_minimize_dev's d_keep:
 * an element's winner depends on that element's entries only.  *n_out = the
 * shard's count. */
int syzsig_minimize_shard_dev(syzsig_ctx* ctx, const uint64_t* d_ctx_off, const uint32_t* d_elems,
                              const int8_t* d_prios, uint64_t nctx, uint32_t nshards, uint32_t shard,
                              uint64_t hint_distinct, uint8_t* d_keep, uint64_t* n_out);

/* Minimize split by data (one process per GPU): part `part` of
 * `nparts` takes a contiguous range of the contexts in sort order (Len desc,
 * index asc), cut at about total/nparts entries per part, and reads only those
 * contexts' entries.  It aggregates them per element and writes one winner
 * record per distinct element of its range,
 *     e << 32 | (prio ^ 0x80) << 24 | (0xFFFFFF - rank)
 * (rank = the context's position in the global sort order; the max of the low
 * 32 bits over the parts is argmax (prio, -rank), the reference's winner),
 * grouped by owner_of(e, nshards) into d_send (send_cap >= the part's entries
 * suffices); send_counts[g] = records for owner g, packed at their exclusive
 * prefix sum.  nshards <= 64; at most 4 distinct prios per part. */
int syzsig_minimize_split_dev(syzsig_ctx* ctx, const uint64_t* d_ctx_off, const uint32_t* d_elems,
                              const int8_t* d_prios, uint64_t nctx, uint32_t nparts, uint32_t part, uint32_t nshards,
                              uint64_t hint_distinct, uint64_t* d_send, uint64_t send_cap, uint64_t* send_counts);
/* Owner side of the split: the winner records every part sent to this owner
 * (d_recs, any order) -> the max per element -> d_keep[i] = 1 iff context i
 * wins one of them.  The OR (max) of d_keep over the owners is
 * syzsig_minimize_dev's d_keep; *n_out = this owner's count. */
int syzsig_minimize_resolve_dev(syzsig_ctx* ctx, const uint64_t* d_ctx_off, uint64_t nctx, const uint64_t* d_recs,
                                uint64_t nrec, uint8_t* d_keep, uint64_t* n_out);

/* ---- pkg/cover/cover.go:7-30: type Cover map[uint32]struct{} ----
 * A Cover is a syzsig_set whose entries all carry prio 0.  Merge(raw)
 * (cover.go:9-18) allocates a NULL *cov even when n == 0, then inserts every
 * PC (manager corpusCover.Merge, syz-manager/manager.go:998).  Len is
 * syzsig_len; Serialize (cover.go:20-26) is syzsig_serialize's elems. */
int syzsig_cover_merge(syzsig_ctx* ctx, syzsig_set** cov, const uint32_t* raw, uint64_t n);
int syzsig_cover_merge_dev(syzsig_ctx* ctx, syzsig_set** cov, const uint32_t* d_raw, uint64_t n);

/* ---- syz-fuzzer/proc.go:107-140 triageInput signal re-runs, over a batch ----
 * Item i's newSignal (corpusSignalDiff of its input signal, serialized) is
 * elems/prios[item_off[i] .. item_off[i+1]); item_flags[i] = SYZSIG_TRIAGE_*.
 * Item i's re-runs are r = i*runs .. i*runs+runs-1 (runs = signalRuns, <= 8):
 * run r's raw signal is run_sigs[run_off[r] .. run_off[r+1]) with
 * run_prio[r] = signalPrio, run_errno[r] = its Errno, run_exec[r] = 0 when
 * len(info) == 0.  Applies the loop of proc.go:119-139 (skip and count runs
 * that did not execute or failed; newSignal = newSignal.Intersection(run);
 * drop the item when it empties unless minimized, or after more than
 * runs/2+1 skipped runs).  Writes item_keep[i] (1 = the item goes on to
 * minimization and the corpus) and elem_keep[j] (1 = element j is in the
 * item's final newSignal).  All pointers are device pointers. */
#define SYZSIG_TRIAGE_MINIMIZED 1 /* item.flags & ProgMinimized */
#define SYZSIG_TRIAGE_ORIG_OK 2   /* item.info.Errno == 0 */
int syzsig_triage_runs_dev(syzsig_ctx* ctx, const uint64_t* d_item_off, uint64_t nitems, const uint32_t* d_elems,
                           const int8_t* d_prios, const uint8_t* d_item_flags, uint32_t runs,
                           const uint64_t* d_run_off, const uint32_t* d_run_sigs, const uint8_t* d_run_prio,
                           const int32_t* d_run_errno, const uint8_t* d_run_exec, uint8_t* d_item_keep,
                           uint8_t* d_elem_keep);

/* The minimize predicate of triageInput (proc.go:141-160) over a batch:
 * same item/run layout as syzsig_triage_runs_dev, with `attempts` runs per
 * item (minimizeAttempts).  pred[i] = 1 iff, going through the attempts in
 * order and skipping ones that did not execute or have no signal, an attempt
 * keeps all of newSignal (newSignal.Intersection(thisSignal).Len() ==
 * newSignal.Len()) before one fails after a successful original. */
int syzsig_minimize_pred_dev(syzsig_ctx* ctx, const uint64_t* d_item_off, uint64_t nitems, const uint32_t* d_elems,
                             const int8_t* d_prios, const uint8_t* d_item_flags, uint32_t attempts,
                             const uint64_t* d_run_off, const uint32_t* d_run_sigs, const uint8_t* d_run_prio,
                             const int32_t* d_run_errno, const uint8_t* d_run_exec, uint8_t* d_pred);

/* ---- syz-fuzzer/fuzzer.go:494-511 checkNewSignal (+ signalPrio :513-521 by caller) ----
 * One program's CallInfo signals in host memory: call i's raw signal is
 * sigs[call_start[i] .. +call_len[i]) with prio call_prio[i].  Sequential over
 * calls as the reference: call i sees merges of calls < i.  Writes indices of
 * calls with new signal to out_calls (capacity ncalls), *n_out = count;
 * merges into *max_signal and *new_signal (allocating NULL ones).
 * new_bits (optional, ceil(nrec/32) words): bit r set iff sigs[r] is in its
 * call's DiffRaw result. */
int syzsig_check_new_signal(syzsig_ctx* ctx, syzsig_set** max_signal, syzsig_set** new_signal,
                            const uint32_t* sigs, uint64_t nrec, const uint64_t* call_start,
                            const uint32_t* call_len, const uint8_t* call_prio, uint32_t ncalls,
                            uint32_t* out_calls, uint32_t* n_out, uint32_t* new_bits);

/* ---- batch triage (device pointers): checkNewSignal over a whole batch ----
 * Serial order = call index order (program-major, call-minor).  Call ranges
 * [call_start, call_start+call_len) must lie inside [0, nrec) and be disjoint.
 * Outputs:
 *  - call_new[c] = 1 iff call c's DiffRaw is non-empty (checkNewSignal's
 *    `calls`, syz-fuzzer/fuzzer.go:498-503);
 *  - new_pairs (optional): every call's DiffRaw result as (call << 32 | elem),
 *    one entry per distinct (call, elem), in unspecified order; at most
 *    new_pairs_cap are written, stats.new_pairs = the total;
 *  - new_bits (optional, NULL = not computed): bit r = record r's element is in
 *    its call's DiffRaw result (every duplicate occurrence is marked).
 * call_new / new_bits are zeroed by the call. */
typedef struct {
	const uint32_t* sigs;       /* nrec raw signal elements */
	const uint64_t* call_start; /* ncalls */
	const uint32_t* call_len;   /* ncalls */
	const uint8_t* call_prio;   /* ncalls, signalPrio values */
	uint64_t ncalls;
	uint64_t nrec;
	uint32_t* new_bits;         /* out (optional): ceil(nrec/32) words, bit r = record r is new */
	uint8_t* call_new;          /* out: ncalls, 1 = call has new signal */
	uint64_t* new_pairs;        /* out (optional): call << 32 | elem per DiffRaw entry */
	uint64_t new_pairs_cap;     /* capacity of new_pairs in entries */
} syzsig_batch;

typedef struct {
	uint64_t records;        /* records processed */
	uint64_t survivors;      /* per-call path: records past the home-bucket filter; aggregation path: distinct elements */
	uint64_t candidates;     /* per-call path: records past the prio filter; aggregation path: = changed */
	uint64_t changed;        /* elements whose maxSignal prio changed (incl. new) */
	uint64_t inserted;       /* elements new to maxSignal */
	uint64_t new_signal_len; /* Len of *new_signal after the batch */
	uint64_t retries;        /* capacity-overflow restarts */
	uint64_t runs;           /* sub-batches (one per <=4 distinct prios) */
	uint64_t parts;          /* aggregation partitions of the last run (0 = per-call path) */
	uint64_t distinct;       /* distinct elements aggregated (aggregation path) */
	uint64_t overflow_parts; /* partitions redone in the HBM table (LDS table too small) */
	uint64_t new_pairs;      /* DiffRaw entries over all calls (see syzsig_batch.new_pairs) */
	double part_ms;          /* device time of record partitioning (0 unless timing enabled) */
	double probe_ms;         /* device time of the probe kernel(s) (0 unless timing enabled) */
	double decide_ms;        /* device time of the decide kernel(s) (0 unless timing enabled) */
} syzsig_batch_stats;

int syzsig_triage_batch(syzsig_ctx* ctx, syzsig_set* max_signal, syzsig_set** new_signal,
                        const syzsig_batch* b, syzsig_batch_stats* stats);

/* ---- executor/executor.h:492-528 + :677-706 on device (K1 edge + K2 dedup) ----
 * Raw KCOV traces for nprog programs; program p owns calls
 * [prog_call[p], prog_call[p+1]); call c's PCs are pcs[call_start[c] .. +call_len[c])
 * (call_len < 262144, executor_linux.cc:186-187).  Each program runs with a
 * fresh 8192-slot dedup table shared by its calls in order, like one forked
 * executor child.  Call c's emitted signals land at sigs[call_start[c] ..
 * +sig_cnt[c]); completed[p] = calls whose record was published (a PC failing
 * cover_check aborts the rest of the program); later calls get sig_cnt = 0.
 * d_sigs has npc entries (same indexing as d_pcs). */
int syzsig_edge_derive_dev(syzsig_ctx* ctx, const uint64_t* d_pcs, uint64_t npc, const uint64_t* d_call_start,
                           const uint32_t* d_call_len, uint64_t ncalls, const uint32_t* d_prog_call,
                           uint64_t nprog, uint32_t* d_sigs, uint32_t* d_sig_cnt, uint32_t* d_completed);

/* ---- pkg/ipc/ipc.go:328-468 readOutCoverage over a batch of executor output regions ----
 * Program p's output region (executor.h:566-604 records, the executor's shmem
 * out file) is d_out[prog_off[p] .. prog_off[p+1]); it has the calls
 * [prog_call[p], prog_call[p+1]) (len(p.Calls)), call_num[c] = the expected
 * syscall ID (c.Meta.ID; NULL = unchecked) and call_any[c] = CallContainsAny
 * (prog/any.go:177-185).  Writes per call: the Signal range inside d_out
 * (aliasing it, ipc.go:410; call_len = 0 if the call has no record), its Errno
 * (-1 = not executed), and its signalPrio (fuzzer.go:513-521); optionally the
 * Cover range.  The result feeds syzsig_triage_batch with sigs = d_out,
 * nrec = nwords.  prog_status[p] = SYZSIG_INGEST_* (the ipc.go error branch
 * hit); a failed program gets no signal (the fuzzer retries that Exec,
 * proc.go:269-278).  *n_failed (optional) = programs with status != 0.
 * Returns SYZSIG_EINVAL if an offset or call range is out of bounds. */
#define SYZSIG_INGEST_OK 0
#define SYZSIG_INGEST_ENCMD 1      /* no ncmd word (ipc.go:356-359) */
#define SYZSIG_INGEST_EHEADER 2    /* short call header (:378-383) */
#define SYZSIG_INGEST_EINDEX 3     /* callIndex >= len(p.Calls) (:384-388) */
#define SYZSIG_INGEST_ECALLNUM 4   /* callNum != c.Meta.ID (:389-395) */
#define SYZSIG_INGEST_EDOUBLE 5    /* double coverage for a call (:396-400) */
#define SYZSIG_INGEST_ESIGNAL 6    /* signalSize past the region (:403-407) */
#define SYZSIG_INGEST_ECOVER 7     /* coverSize past the region (:411-415) */
#define SYZSIG_INGEST_ECOMPS 8     /* short comparison record (:420-445) */
#define SYZSIG_INGEST_ECOMPTYPE 9  /* comparison type > compConstMask|compSizeMask (:429-433) */
#define SYZSIG_INGEST_EBOUNDS 10   /* prog_off / prog_call out of bounds (ABI check) */
int syzsig_ingest_exec_output_dev(syzsig_ctx* ctx, const uint32_t* d_out, uint64_t nwords,
                                  const uint64_t* d_prog_off, uint64_t nprog, const uint32_t* d_prog_call,
                                  uint64_t ncalls, const uint32_t* d_call_num, const uint8_t* d_call_any,
                                  uint64_t* d_call_start, uint32_t* d_call_len, uint8_t* d_call_prio,
                                  int32_t* d_call_errno, uint64_t* d_cover_start, uint32_t* d_cover_len,
                                  int32_t* d_prog_status, uint64_t* n_failed);

/* ---- hash-sharded maxSignal across GPUs (one process per GPU) ----
 * The batch is split by program range over G GPUs (serial order = GPU-major);
 * each element is owned by the GPU owner = syz::owner_of(elem, G).  Records
 * travel packed as
 *   elem << 32 | level << 24 | serial      (serial < 2^24, level < 4)
 * where serial is its call's position in the batch's global serial order and
 * level the rank of its call's prio in `levels` (ascending int8, <= 4 entries,
 * the union of the prios of all GPUs' calls).  A source sends only each
 * element's staircase -- for every level, the element's first local record at
 * that level if no earlier local record has a higher level, <= 4 records per
 * distinct element: records off the staircase can never be new nor raise
 * maxSignal, so the owner's triage of the staircases is checkNewSignal's exact
 * result.  The exchange is the stream-ordered step below; the owner side is
 * records mode:
 *
 * syzsig_triage_records_dev: triage records against the local shard of
 * maxSignal; d_new_flags[i] = 1 iff record i is new (checkNewSignal's DiffRaw
 * result for its call).  Serial order comes from the records' serial fields;
 * records with one serial are one call's, so they carry one level. */
int syzsig_triage_records_dev(syzsig_ctx* ctx, syzsig_set* shard, syzsig_set** new_signal,
                              const uint64_t* d_recs, uint64_t nrec, const int8_t* levels,
                              uint32_t nlevels, uint8_t* d_new_flags, syzsig_batch_stats* stats);

/* ---- the stream-ordered sharded step (one process per GPU) ----
 * The three calls below only enqueue work on the context's stream and return;
 * syzsig_step_finish is the step's one host synchronisation.  The exchange
 * uses fixed-size buckets, so no split sizes have to reach the host first:
 * each source writes, for every owner g, a bucket of cap + 1 words at
 * d_send[g * (cap + 1)]:
 *   word 0      header: records for g (the true count, even past cap)
 *               | SYZSIG_STEP_HDR_VOID (the source's run is void)
 *               | SYZSIG_STEP_HDR_OVF  (more than cap records for g)
 *   words 1..   the staircase records (elem << 32 | level << 24 | serial).
 * An equal-split all-to-all of the buckets gives each owner every source's
 * bucket for it (d_recv, same layout, bucket s from source s); the owner's
 * flags go back the same way, one byte per word (d_flags / d_back, nshards *
 * (cap + 1) bytes; byte 0 of a bucket is the owner's status).  Every owner sees
 * every header, so all ranks agree without another collective that a step is
 * void (nothing committed anywhere; redo it, with exact = 1 on a void source
 * and a larger cap after an overflow) or which owners skipped their records
 * (their records redone with syzsig_step_own_dev(exact = 1) and one more flags
 * exchange, which syzsig_step_back_dev adds to the first).
 * Reference semantics: syz-fuzzer/fuzzer.go:494-511 over the batch in global
 * serial order; the result is the unsharded checkNewSignal's. */
#define SYZSIG_STEP_HDR_VOID (1ull << 63)
#define SYZSIG_STEP_HDR_OVF (1ull << 62)
#define SYZSIG_STEP_HDR_COUNT ((1ull << 40) - 1)
typedef struct {
	uint64_t src_void;     /* this source's run was void: 1 = a cell spilled, a partition overflowed the LDS
	                          table, a call range is bad or the records exceed b->nrec (redo with exact = 1,
	                          which validates), 2 = a call's prio is not among `levels` */
	uint64_t global_void;  /* some bucket was void or over cap: nothing was committed on any rank */
	uint64_t owners_void;  /* bit g: owner g skipped its records (redo them exactly); 0 when global_void */
	uint64_t records;      /* this source's records */
	uint64_t distinct;     /* this source's distinct elements */
	uint64_t sent;         /* this source's staircase records (all owners) */
	uint64_t max_out;      /* the most records this source had for one owner (the cap it needs) */
	uint64_t received;     /* records this owner received */
	uint64_t max_in;       /* the most records one source had for this owner */
	uint64_t own_distinct; /* distinct elements among them */
	uint64_t inserted;     /* elements new to this owner's shard */
	uint64_t changed;      /* elements whose prio rose in this owner's shard */
	uint64_t new_pairs;    /* this source's DiffRaw entries (call << 32 | elem), see syzsig_batch */
	uint64_t own_parts;    /* LDS partitions of the owner's records (0 = exact path) */
	double src_ms, own_ms, back_ms; /* device time of each side (0 unless timing is on) */
} syzsig_step_status;
/* Source side: aggregate b (zeroing call_new) and write its staircase buckets.
 * cap >= 1; d_send has nshards * (cap + 1) words.  exact = 0: one run on
 * capped cells that voids itself on a spill, an LDS partition overflow or a prio
 * outside `levels` (no host round trip); exact = 1: the counted path with its
 * HBM fallback (host round trips; a prio outside `levels` is SYZSIG_EINVAL). */
int syzsig_step_send_dev(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t serial_base, const int8_t* levels,
                         uint32_t nlevels, uint32_t nshards, uint64_t cap, uint64_t* d_send, int exact);
/* Owner side: the buckets every source sent this owner (d_recv, nshards *
 * (cap + 1) words) triaged against its shard and newSignal shard (both
 * non-NULL); d_flags gets one byte per word.  exact = 0: records partitioned by
 * element hash through LDS (per partition its elements' level firsts, per
 * element one shard probe, per record checkNewSignal's verdict in closed form;
 * no sort); a partition over the LDS capacity makes this owner skip its
 * records (owners_void).
 * exact = 1: the per-record path (host round trips), for that redo.  Until
 * syzsig_step_finish, `shard` and `new_signal` take no other call. */
int syzsig_step_own_dev(syzsig_ctx* ctx, syzsig_set* shard, syzsig_set* new_signal, const uint64_t* d_recv,
                        uint32_t nshards, uint64_t cap, const int8_t* levels, uint32_t nlevels, uint8_t* d_flags,
                        int exact);
/* Source side again: the owners' flags (d_back, from the flags exchange) for
 * this source's buckets -> b->call_new, b->new_pairs (new_pairs_cap entries at
 * most; the total in the status); b->new_bits (if set; costs one host
 * synchronisation).  Adds to what an earlier call of the step set. */
int syzsig_step_back_dev(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t serial_base, const uint64_t* d_send,
                         uint32_t nshards, uint64_t cap, const uint8_t* d_back);
/* The step's one host synchronisation: waits for the context's stream (which
 * the collectives' streams joined), commits the owner's table lengths and
 * returns the status of the calls since the last finish. */
int syzsig_step_finish(syzsig_ctx* ctx, syzsig_step_status* status);

/* ---- synthetic workload (deterministic; host and device give identical data) ---- */
typedef struct {
	uint64_t seed;
	uint32_t nblocks_log2, region_log2, nsys, skew, restart_log2;
	uint32_t errno_permille, any_permille, bad_pc_ppm;
	/* 1: SURVEY 8(d)'s global walk -- each call starts at a uniform block and
	 * walks b <- (4b + 1 + r%4) mod 2^nblocks_log2 with no restarts (region_log2,
	 * nsys, skew and restart_log2 then only pick the call's prio draw); M0's
	 * known elements are that walk's whole edge universe. */
	uint32_t global_walk;
} syzsig_synth_cfg;

void syzsig_synth_default(syzsig_synth_cfg* cfg);
/* Per call c of a batch (prog_base + p for program p): call_prio and the raw trace
 * of call_len[c] PCs at pcs[call_start[c]..]. */
int syzsig_synth_traces_host(const syzsig_synth_cfg* cfg, uint64_t prog_base, uint64_t nprog,
                             uint32_t calls_per_prog, const uint64_t* call_start, const uint32_t* call_len,
                             uint64_t* pcs, uint8_t* call_prio);
int syzsig_synth_traces_dev(syzsig_ctx* ctx, const syzsig_synth_cfg* cfg, uint64_t prog_base,
                            uint64_t nprog, uint32_t calls_per_prog, const uint64_t* d_call_start,
                            const uint32_t* d_call_len, uint64_t* d_pcs, uint8_t* d_call_prio);
int syzsig_synth_m0_host(const syzsig_synth_cfg* cfg, uint64_t known_sys, uint64_t n, uint32_t* elems,
                         int8_t* prios);
int syzsig_synth_m0_dev(syzsig_ctx* ctx, const syzsig_synth_cfg* cfg, uint64_t known_sys, uint64_t n,
                        uint32_t* d_elems, int8_t* d_prios);
/* The elements i < n of that M0 which shard `shard` of `nshards` owns
 * (owner_of), in index order, packed into d_elems/d_prios (capacity `cap`);
 * *n_out = how many.  A rank builds its shard of a 1B-element M0 without
 * materialising the whole. */
int syzsig_synth_m0_shard_dev(syzsig_ctx* ctx, const syzsig_synth_cfg* cfg, uint64_t known_sys, uint64_t n,
                              uint32_t nshards, uint32_t shard, uint32_t* d_elems, int8_t* d_prios, uint64_t cap,
                              uint64_t* n_out);

#ifdef __cplusplus
}
#endif
#endif /* SYZSIG_H */
