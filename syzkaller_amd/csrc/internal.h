// internal.h -- private structures and device primitives of libsyzsig.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/syzsig.h"
#include "common.h"

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
namespace syz {
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_fail(hipError_t e, const char* what, const char* file, int line);
}  // namespace syz

#define SYZ_HIP(expr)                                                              \
	do {                                                                           \
		hipError_t e__ = (expr);                                                   \
		if (e__ != hipSuccess)                                                     \
			return syz::hip_fail(e__, #expr, __FILE__, __LINE__);                  \
	} while (0)

// Serialize this C-ABI call against every other call on the same context
// (NULL-safe: the entry point's own argument check then reports the error).
#define SYZ_LOCK(ctx) syz::CtxLock syz_lock__(ctx)

#define SYZ_TRY(expr)                                                              \
	do {                                                                           \
		int r__ = (expr);                                                          \
		if (r__ != SYZSIG_OK)                                                      \
			return r__;                                                            \
	} while (0)

// ---------------------------------------------------------------------------
// host-side objects
// ---------------------------------------------------------------------------
namespace syz {

// Device counters live in one small array per context (zeroed per operation).
enum Counter : int {
	kCntInserted = 0,   // new keys inserted into the destination table
	kCntOverflow,       // probe limit hit (capacity too small) -> retry bigger
	kCntError,          // malformed input detected on device
	kCntCandidates,     // triage: records that passed the prio filter
	kCntTouched,        // triage: distinct elements with a candidate this run
	kCntChanged,        // triage: slots committed (prio raised or inserted)
	kCntAux,            // misc (serialize cursor, minimize winners...)
	kCntAux2,
	kCntDefer,          // triage finalize: elements deferred to the atomic path
	kCntDeferNs,        // triage finalize: newSignal merges deferred to the atomic path
	kCntDistinct,       // one-sync triage run / records mode: distinct elements
	kCntAggOvf,         // one-sync triage run: partitions that overflowed the LDS table
	kCntSpill,          // one-sync triage run: its void flag (low 32 bits; 1 = a cell spilled, 2 = assumptions)
	kCntRecords,        // one-sync triage run: the batch's records
	kNumCounters = 16,
};
// the sharded step's counter blocks in syzsig_ctx::d_step
constexpr int kStepSrc = 0, kStepOwn = 16, kStepBack = 32, kStepCounters = 48;

struct Workspace {
	void* ptr = nullptr;
	size_t size = 0;
};

// the debug flags that change only the path taken, never a result
constexpr uint32_t kDebugResultPreserving =
    SYZSIG_DEBUG_FIN_DEFER | SYZSIG_DEBUG_MIN_ATOMIC | SYZSIG_DEBUG_EXACT_CELLS | SYZSIG_DEBUG_CAP_SPILL |
    SYZSIG_DEBUG_RECS_GATE | SYZSIG_DEBUG_EDGE_MARKALL | SYZSIG_DEBUG_EDGE_PASSES | SYZSIG_DEBUG_AGG_IDX64;
// ... and those a product build accepts: the above plus fault injection
constexpr uint32_t kDebugAccepted = kDebugResultPreserving | SYZSIG_DEBUG_POLL_FAIL;

// capped cells of the aggregation path (agg.hip): default slack, in standard deviations
constexpr float kCapSdDefault = 6.0f;

// ctx->h_pin layout
constexpr size_t kPinMask = 0, kPinPairs = 64, kPinCounts = 1024, kPinBytes = 64 * 1024;

}  // namespace syz

struct syzsig_ctx {
	// Every C-ABI entry point holds this for its whole duration (SYZ_LOCK): the
	// context's stream, scratch slots, counters and pinned staging are shared by
	// all callers, and the reference runs Diff/DiffRaw concurrently under
	// signalMu.RLock (syz-fuzzer/fuzzer.go:488-498).  Recursive: entry points
	// call each other (e.g. triage allocates newSignal through syzsig_set_make).
	std::recursive_mutex mu;
	int device = 0;
	hipStream_t own_stream = nullptr;
	hipStream_t stream = nullptr;
	unsigned long long* d_cnt = nullptr;  // kNumCounters
	unsigned long long* h_cnt = nullptr;  // pinned mirror
	// pinned staging for the small per-batch copies (a pageable copy is staged
	// and synchronous): syz::kPin* offsets
	char* h_pin = nullptr;
	// grow-only scratch buffers by role (35: the one-sync run's fallback): 0-2 set ops, 3-6 triage candidates and
	// small state, 7-10 host uploads of minimize, 11-14 triage partitions and
	// minimize internals and triage pairs (13-15), 16-23 + 30-31 triage aggregation, 55-63 the sharded step and
	// the LDS records path,
	// 24-29 check_new_signal uploads, 32-33 the finalize's deferred lists, 40-47 manager poll
	syz::Workspace ws[64];
	bool timing = false;                  // HIP events around triage kernels
	// tuning knobs (defaults; SYZSIG_* environment overrides read at ctx creation)
	int part_mode = 1;                    // 0 = never use the aggregation path (agg.hip)
	uint32_t agg_parts = 0;               // fixed partition count of the aggregation path (0 = adaptive)
	double agg_distinct_ratio = 0;        // distinct/records of the last aggregated run (sizes the next)
	float cap_sd = syz::kCapSdDefault;    // capped-cell slack in standard deviations (agg.hip; 0 = counted cells)
	float cap_sd_entry = syz::kCapSdDefault;  // the same for Minimize's runs
	bool agg_counted_once = false;        // the next agg_aggregate takes counted cells (a one-sync run spilled)
	uint32_t edge_waves = 4;              // waves per program of k_edge_dedup (4 or 8; SYZSIG_EDGE_WAVES)
	bool edge_mark_all = true;            // k_edge_dedup's marking mode for the next launch (edge.hip)
	uint32_t agg_dbg = 0;                 // SYZSIG_DEBUG_* path flags; timing-only bits need -DSYZ_EXPERIMENTS
	hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
	double last_ms = 0;                   // device time of the last timed entry point's kernels
	// the stream-ordered sharded step (syzsig_step_*): its counters, read once by
	// syzsig_step_finish -- [0,16) source, [16,32) owner, [32,48) flags back
	unsigned long long* d_step = nullptr;
	unsigned long long* h_step = nullptr;  // pinned mirror
	syzsig_set* step_ms = nullptr;         // the owner's shard and newSignal until finish
	syzsig_set* step_ns = nullptr;
	uint64_t step_parts = 0;
	uint64_t step_src_parts = 1;           // the source run's aggregation partitions
	bool step_own_timed = false, step_src_timed = false, step_back_timed = false;
	hipEvent_t ev_step[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
};

struct syzsig_set {
	syzsig_ctx* ctx = nullptr;
	uint64_t* slots = nullptr;   // nbuckets * 8
	uint64_t nbuckets = 0;       // power of two
	uint64_t len = 0;            // live entries (host mirror of device truth)
	// triage side state, allocated on first batch
	uint32_t* firsts = nullptr;  // 4 per slot: epoch_rev << 24 | serial, per prio level
	uint32_t* touched = nullptr; // 1 bit per slot
	uint32_t epoch = 0;          // current epoch_rev (counts down 254..1)
	bool step_busy = false;      // an owner step is in flight on it (len not final until syzsig_step_finish)
	uint64_t nslots() const { return nbuckets * syz::kBucketSlots; }
};

namespace syz {

struct CtxLock {
	syzsig_ctx* c;
	explicit CtxLock(syzsig_ctx* x) : c(x)
	{
		if (c)
			c->mu.lock();
	}
	~CtxLock()
	{
		if (c)
			c->mu.unlock();
	}
	CtxLock(const CtxLock&) = delete;
	CtxLock& operator=(const CtxLock&) = delete;
};

// scratch buffer `i` of the context, grown to at least `bytes` (contents lost on growth)
int ws_get(syzsig_ctx* ctx, int i, size_t bytes, void** out);
// same, keeping the first `keep` bytes across a growth
int ws_grow_keep(syzsig_ctx* ctx, int i, size_t bytes, size_t keep, void** out);
int counters_reset(syzsig_ctx* ctx);
int counters_fetch(syzsig_ctx* ctx);  // sync + copy to ctx->h_cnt

// table lifecycle (table.hip)
uint64_t buckets_for(uint64_t n_entries);
int set_alloc(syzsig_ctx* ctx, uint64_t nbuckets, syzsig_set** out);
int set_reserve(syzsig_set* s, uint64_t extra);  // ensure room for len+extra
int set_reserve_load(syzsig_set* s, uint64_t extra, double load);  // ... at most `load` full
int set_rehash(syzsig_set* s, uint64_t nbuckets, bool drop_absent);
int set_ensure_triage_state(syzsig_set* s);
int merge_pairs_dev(syzsig_ctx* ctx, syzsig_set* dst, const uint64_t* d_pairs, uint64_t n);

// Prio levels of one triage run: DiffRaw compares prios as int8
// (signal.go:93), so levels follow signed order.
struct LevelMap {
	uint8_t lvl[256];  // prio (as u8) -> level, 0xff = not in this run
	int8_t val[4];     // level -> prio
	uint32_t n;
};
constexpr uint32_t kSerialMask = 0xFFFFFF;  // 24-bit serial index inside a run
int level_map_from_levels(const int8_t* levels, uint32_t nlevels, LevelMap* lm);

// aggregation path (agg.hip)
constexpr uint32_t kAggRegion = 7424;  // distinct-list region per partition (= LDS slots of k_agg)
constexpr uint32_t kAggLimitRecs = kAggRegion * 4 / 5;  // distinct elements an LDS partition holds (agg.hip kAggLimit)
struct AggOut {
	const uint32_t* dist_e;  // distinct elements; region r at [r * kAggRegion, + cnt[r])
	const uint4* dist_f;     // their first serial per level (0xFFFFFFFF = none)
	const uint32_t* cnt;     // per region, device
	uint32_t nregions;
	uint32_t parts;          // partitions P; regions [0, P) are partitions (nregions > P: HBM fallback lists)
	uint64_t D;              // distinct elements in all regions
};
// Per-record extras of an aggregation run, for Minimize (minimize.hip); triage
// passes none.
struct AggSrc {
	const int8_t* elem_prio;  // per-record prio, parallel to sigs (level lm.lvl[prio]); nullptr = the call's
	uint32_t nshards, shard;  // keep only the records whose element this shard owns (owner_of)
	double distinct_hint;     // expected distinct elements (0: the batch-ratio policy)
	unsigned int* bad_level = nullptr;  // if set: |= 1 when a record's prio has no level (lm.lvl[prio] == 0xff)
};
int agg_aggregate(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t c0, uint64_t c1, const LevelMap& lm,
                  uint64_t run_recs, syzsig_batch_stats* st, AggOut* out, const AggSrc* x = nullptr);
// validates a batch's call ranges (SYZSIG_EINVAL) and sums its records (triage.hip)
int batch_total_records(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t* total, uint32_t prio_mask[8]);
int agg_triage_run(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const syzsig_batch* b, uint64_t c0, uint64_t c1,
                   const LevelMap& lm, uint64_t run_recs, syzsig_batch_stats* st, uint64_t** pairs,
                   uint64_t* npairs);
// The whole batch as one aggregation run without a presence pass and its
// host round trip: levels 0..3 (signalPrio's range, fuzzer.go:513-521) and at
// most b->nrec records are assumed, checked on device before the scatter
// (k_fast_prep, k_cell_plan_fast), and the run commits nothing when they do not
// hold.  Zeroes b->call_new.  One host synchronisation; stats.records is set.
// *done = false: take the planned path.
int agg_triage_optimistic(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const syzsig_batch* b,
                          syzsig_batch_stats* st, uint64_t** pairs, uint64_t* npairs, bool* done);
int agg_mark_bits(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t c0, uint64_t c1, const uint64_t* pairs,
                  uint64_t p0, uint64_t p1);
// records mode (triage.hip: the per-record path, and the entry; recs.hip: the LDS path)
int triage_records_impl(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const uint64_t* recs, uint64_t nrec,
                        const int8_t* levels, uint32_t nlevels, uint8_t* new_flags, syzsig_batch_stats* st,
                        bool allow_lds = true);
// *done = false: the LDS path voided itself (nothing committed), take the per-record path
int rp_triage_records(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const uint64_t* recs, uint64_t nrec,
                      const LevelMap& lm, uint8_t* new_flags, syzsig_batch_stats* st, bool* done);
// Entries x[r] = e << 32 | r (r < 2^32) grouped by element through the LDS
// partitions of recs.hip, for Poll (poll.hip): on return (enqueued only)
// keys[base[p] .. base[p + 1]) = h_residual << 32 | r of partition p's entries
// (partition = the top pbits of fmix32(e)), base on device (P + 1 entries);
// ctr zeroed, then ctr[kCntSpill] != 0 when a partition exceeds kRpGroupCap
// entries (nothing after it is valid).
constexpr uint32_t kRpGroupCap = 2048;
int rp_group(syzsig_ctx* ctx, const uint64_t* x, uint64_t n, uint64_t** keys, uint32_t** base, uint32_t* pbits,
             unsigned long long* ctr);
// Stable LSD radix sort of n (u32 key, u32 value) pairs, keys < 2^key_bits
// (sort.hip), ping-pong between the input and tmp buffers; *keys_out /
// *vals_out = the sorted pairs.  Enqueues only; scratch workspace slot ws_slot.
int radix_sort_pairs(syzsig_ctx* ctx, uint32_t* keys, uint32_t* vals, uint32_t* keys_tmp, uint32_t* vals_tmp,
                     uint32_t n, uint32_t key_bits, uint32_t** keys_out, uint32_t** vals_out, int ws_slot);
// a set an owner step holds until syzsig_step_finish takes no other call
inline int set_check_idle(const syzsig_set* s)
{
	return s && s->step_busy ? fail(SYZSIG_EINVAL, "set is held by a sharded step until syzsig_step_finish") : 0;
}
int pairs_from_bits(syzsig_ctx* ctx, const syzsig_batch* b, const uint32_t* bits, uint64_t c0, uint64_t c1,
                    uint64_t bound, uint64_t** pairs, uint64_t* npairs);

// the default load-factor policy: a table is grown when live/slots exceeds this
constexpr double kMaxLoad = 0.75;
constexpr double kTargetLoad = 0.5;
constexpr double kHardLoad = 0.9;  // a reservation for a worst case grows the table only past this
constexpr uint32_t kMaxProbeBuckets = 4096;

inline int grid_for(uint64_t n, int block, int max_blocks = 2048)
{
	uint64_t g = (n + block - 1) / block;
	if (g < 1)
		g = 1;
	if (g > (uint64_t)max_blocks)
		g = max_blocks;
	return (int)g;
}

}  // namespace syz

// ---------------------------------------------------------------------------
// device primitives
// ---------------------------------------------------------------------------
#if defined(__HIPCC__)
namespace syz {

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// number of set bits of `mask` below this lane
__device__ __forceinline__ uint32_t lane_rank(uint64_t mask)
{
	return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
#pragma unroll
	for (int o = 32; o > 0; o >>= 1)
		v += __shfl_xor(v, o, 64);
	return v;
}

// Block-wide sum of v added to *counter by one thread.  Every thread of the
// block must call it (uniform control flow).
__device__ __forceinline__ void block_count(unsigned long long* counter, uint64_t v)
{
	__shared__ unsigned long long part;
	if (threadIdx.x == 0)
		part = 0;
	__syncthreads();
	v = wave_sum_u64(v);
	if (lane_id() == 0 && v)
		atomicAdd(&part, (unsigned long long)v);
	__syncthreads();
	if (threadIdx.x == 0 && part)
		atomicAdd(counter, part);
}

struct Bucket {
	uint64_t s[kBucketSlots];
};

__device__ __forceinline__ Bucket load_bucket(const uint64_t* p)
{
	const ulonglong2* q = reinterpret_cast<const ulonglong2*>(p);
	Bucket B;
#pragma unroll
	for (uint32_t i = 0; i < kBucketSlots / 2; i++) {
		const ulonglong2 v = q[i];
		B.s[2 * i] = v.x;
		B.s[2 * i + 1] = v.y;
	}
	return B;
}

// Home bucket = the top bits of fmix32(key): slices of the table then hold
// contiguous ranges of h, which is what lets the aggregation path (agg.hip,
// partitioned by the same top bits) probe one slice per partition.
__device__ __forceinline__ uint64_t home_bucket(uint32_t key, uint64_t bmask)
{
	return ((uint64_t)fmix32(key) * (bmask + 1)) >> 32;
}

// Lookup.  Returns the slot index, or -1 if absent (first empty slot reached:
// slots only ever go EMPTY -> key, so occupied slots form a prefix of every
// probe sequence).
__device__ __forceinline__ int64_t tbl_lookup(const uint64_t* __restrict__ slots, uint64_t bmask, uint32_t key,
                                              uint64_t& val)
{
	uint64_t b = home_bucket(key, bmask);
	for (uint64_t n = 0; n <= bmask; n++) {
		Bucket B = load_bucket(slots + (b << kBucketShift));
#pragma unroll
		for (int i = 0; i < (int)kBucketSlots; i++) {
			if (B.s[i] == kSlotEmpty)
				return -1;
			if (slot_key(B.s[i]) == key) {
				val = B.s[i];
				return (int64_t)((b << kBucketShift) + i);
			}
		}
		b = (b + 1) & bmask;
	}
	return -1;
}

// tbl_lookup with the home bucket already loaded (B = load_bucket of
// home_bucket(key)), so that a thread can issue several tables' home-bucket
// loads before it waits for any.
__device__ __forceinline__ int64_t tbl_lookup_from(const uint64_t* __restrict__ slots, uint64_t bmask, uint32_t key,
                                                   uint64_t& val, Bucket B)
{
	uint64_t b = home_bucket(key, bmask);
	for (uint64_t n = 0; n <= bmask; n++) {
		if (n)
			B = load_bucket(slots + (b << kBucketShift));
#pragma unroll
		for (int i = 0; i < (int)kBucketSlots; i++) {
			if (B.s[i] == kSlotEmpty)
				return -1;
			if (slot_key(B.s[i]) == key) {
				val = B.s[i];
				return (int64_t)((b << kBucketShift) + i);
			}
		}
		b = (b + 1) & bmask;
	}
	return -1;
}

// Find `key`, inserting `ins` (a slot word for `key`) at the first empty slot
// if absent.  old = previous word (0 when this call inserted).  Returns -1
// when max_probe buckets were scanned without success (overflow).
__device__ __forceinline__ int64_t tbl_find_or_insert(uint64_t* slots, uint64_t bmask, uint32_t key, uint64_t ins,
                                                      uint64_t& old, uint64_t max_probe)
{
	uint64_t b = home_bucket(key, bmask);
	for (uint64_t n = 0; n < max_probe; n++) {
		uint64_t* bp = slots + (b << kBucketShift);
		Bucket B = load_bucket(bp);
#pragma unroll
		for (int i = 0; i < (int)kBucketSlots; i++) {
			uint64_t s = B.s[i];
			if (s == kSlotEmpty) {
				s = atomicCAS(reinterpret_cast<unsigned long long*>(bp + i), 0ull, (unsigned long long)ins);
				if (s == kSlotEmpty) {
					old = 0;
					return (int64_t)((b << kBucketShift) + i);
				}
			}
			if (slot_key(s) == key) {
				old = s;
				return (int64_t)((b << kBucketShift) + i);
			}
		}
		b = (b + 1) & bmask;
	}
	return -1;
}

// tbl_find_or_insert with the home bucket already loaded (B = load_bucket of
// home_bucket(key)): a thread can issue the home-bucket loads of several keys
// before it walks any of them.  A stale B is safe for the same reason a fresh
// one is: slots only go EMPTY -> key, and the CAS sees the current word.
__device__ __forceinline__ int64_t tbl_find_or_insert_from(uint64_t* slots, uint64_t bmask, uint32_t key,
                                                           uint64_t ins, uint64_t& old, uint64_t max_probe, Bucket B)
{
	uint64_t b = home_bucket(key, bmask);
	for (uint64_t n = 0; n < max_probe; n++) {
		uint64_t* bp = slots + (b << kBucketShift);
		if (n)
			B = load_bucket(bp);
#pragma unroll
		for (int i = 0; i < (int)kBucketSlots; i++) {
			uint64_t s = B.s[i];
			if (s == kSlotEmpty) {
				s = atomicCAS(reinterpret_cast<unsigned long long*>(bp + i), 0ull, (unsigned long long)ins);
				if (s == kSlotEmpty) {
					old = 0;
					return (int64_t)((b << kBucketShift) + i);
				}
			}
			if (slot_key(s) == key) {
				old = s;
				return (int64_t)((b << kBucketShift) + i);
			}
		}
		b = (b + 1) & bmask;
	}
	return -1;
}

__device__ __forceinline__ uint64_t max_probe_for(uint64_t bmask)
{
	uint64_t nb = bmask + 1;
	return nb < kMaxProbeBuckets ? nb : kMaxProbeBuckets;  // (kMaxProbeBuckets * kBucketSlots slots)
}

// Insert-or-max (Merge rule).  Returns 1 if inserted, 0 otherwise; -1 overflow.
__device__ __forceinline__ int tbl_merge(uint64_t* slots, uint64_t bmask, uint32_t key, int8_t prio)
{
	uint64_t v = make_slot(key, prio), old;
	int64_t idx = tbl_find_or_insert(slots, bmask, key, v, old, max_probe_for(bmask));
	if (idx < 0)
		return -1;
	if (old == 0)
		return 1;
	if (old < v)
		atomicMax(reinterpret_cast<unsigned long long*>(slots + idx), (unsigned long long)v);
	return 0;
}

// tbl_merge from a preloaded home bucket (see tbl_find_or_insert_from).
__device__ __forceinline__ int tbl_merge_from(uint64_t* slots, uint64_t bmask, uint32_t key, int8_t prio, Bucket B)
{
	uint64_t v = make_slot(key, prio), old;
	int64_t idx = tbl_find_or_insert_from(slots, bmask, key, v, old, max_probe_for(bmask), B);
	if (idx < 0)
		return -1;
	if (old == 0)
		return 1;
	if (old < v)
		atomicMax(reinterpret_cast<unsigned long long*>(slots + idx), (unsigned long long)v);
	return 0;
}

}  // namespace syz
#endif
