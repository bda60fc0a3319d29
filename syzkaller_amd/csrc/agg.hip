// agg.hip -- K3 for large batches: checkNewSignal over a whole batch by
// aggregating the batch's records per element in LDS.
//
// Reference: syz-fuzzer/fuzzer.go:494-511 checkNewSignal, pkg/signal/signal.go
// :90-102 DiffRaw and :117-131 Merge.  With the batch in serial order
// (program-major, call-minor; call k has raw signal sig_k and prio p_k) and
// M0 = maxSignal before the batch:
//
//   e in new_k  <=>  e in sig_k  and  p_k > M0[e]  and  no j < k has e in sig_j with p_j >= p_k
//   M_final[e]  =  max(M0[e], max_k p_k)
//   newSignal  +=  { e : M_final[e] != M0[e] } with prio M_final[e]
//
// Everything about an element e is a function of
//   first[e][l] = min serial k over the records of e at prio level l   (<= 4 levels per run)
// and M0[e]: walking the levels from the top down, a level l with
// val[l] > M0[e] holds a new record iff first[e][l] < min_{l' > l} first[e][l'],
// and that record is (first[e][l], e) -- the call's DiffRaw result.  So the
// batch needs ONE maxSignal probe per distinct element, not one per record.
//
// Record format.  h = fmix32(e) is a bijection of u32.  A run is cut into
// P = 2^pbits partitions by the top pbits of h, and into chunks of 2^cbits
// consecutive calls (cbits = pbits - 2).  Partition p stores its records chunk
// after chunk (one "cell" per (chunk, p)), so a record only needs
//   h's low 32 - pbits bits | level (2 bits) | serial inside its chunk (cbits bits)
// = exactly 32 bits: the partition and the chunk are implied by where the
// record is stored.
//
// Pipeline (one run of <= 4 prio levels):
//   k_agg_count / k_agg_scan_chunks / k_agg_scan_totals / k_agg_scatter
//       records -> 4-B packed records grouped by partition, cells in chunk order.
//   k_agg       one 1024-thread workgroup per partition: an LDS hash table
//       (residual key + 4 level firsts, 20 B/slot, kAggSlots slots = 145 KiB)
//       absorbs the partition's records -- one ds_read_b128 of the home bucket,
//       a ds_cmpst on first sight, one ds_min per record; then the distinct
//       elements are written out compactly.  A partition with more distinct
//       elements than kAggLimit is flagged and redone by k_agg_global (the same
//       aggregation in an HBM table).
//   k_agg_finalize  one workgroup per partition's distinct list: probe/insert
//       maxSignal, emit the new (call, elem) pairs and call flags, write
//       M_final, merge newSignal.  maxSignal's home bucket is the top bits of
//       the same h (internal.h home_bucket), so one partition's probes stay in
//       one contiguous slice of the table.  Capacity is reserved before it
//       from the exact distinct count, so nothing is ever retried.
//   k_pairs_mark (optional) per-record new bits from the pairs.
#include <algorithm>
#include <type_traits>
#include <vector>

#include "internal.h"

namespace syz {

constexpr uint32_t kAggThreads = 1024;
constexpr uint32_t kAggSlots = 7424;               // LDS slots per workgroup (+ 8 KB of first-sight queues)
// keys per LDS bucket: 4 (one ds_read_b128 per probe) or 2 (ds_read_b64)
#ifndef SYZ_AGG_BW
#define SYZ_AGG_BW 4
#endif
constexpr uint32_t kAggBW = SYZ_AGG_BW;
using KBucket = std::conditional_t<kAggBW == 4, uint4, uint2>;
constexpr uint32_t kAggBuckets = kAggSlots / kAggBW;
constexpr uint32_t kAggNoSlot = 0xFFFFFFFFu;
static_assert(kAggRegion == kAggSlots, "distinct-list region per partition (internal.h)");
constexpr uint32_t kAggLimit = kAggSlots * 4 / 5;  // distinct elements before a partition overflows
static_assert(kAggLimit == kAggLimitRecs, "internal.h mirror");
constexpr double kAggTargetLoad = 0.4;             // partitions are sized for this LDS load
constexpr double kAggTargetLoadEntry = 0.6;        // ... and for Minimize
#ifndef SYZ_MIN_ITEMS
#define SYZ_MIN_ITEMS 2048  // Minimize: at least this many partitioning work items
#endif
constexpr uint32_t kAggEmpty = 0xFFFFFFFFu;        // empty key (LDS keys are residuals < 2^29)
constexpr uint32_t kAggNone = 0xFFFFFFFFu;         // no record at this level
constexpr uint32_t kAggOverflow = 0xFFFFFFFFu;     // partition count marker
constexpr uint32_t kAggMinBits = 3, kAggMaxBits = 11;
constexpr uint32_t kAggMaxParts = 1u << kAggMaxBits;
constexpr uint32_t kAggTile = 18432;  // records per scatter tile (18 per lane; 6 B of LDS each)
#ifndef SYZ_AGG_GROUP
#define SYZ_AGG_GROUP 8
#endif
constexpr uint32_t kAggGroup = SYZ_AGG_GROUP;  // cells per wave work item of k_agg (<= 64)
// k_agg's record pipeline: U records per lane per batch, D batches in flight ahead
#ifndef SYZ_AGG_U
#define SYZ_AGG_U 4
#endif
#ifndef SYZ_AGG_D
#define SYZ_AGG_D 2
#endif
constexpr uint32_t kAggU = SYZ_AGG_U, kAggD = SYZ_AGG_D;
#ifndef SYZ_AGG_OVF_EACH  // k_agg tests its overflow flag after every batch (1) or per group of cells (0)
#define SYZ_AGG_OVF_EACH 0
#endif

// Partition geometry of one run (see the header).
struct AggGeom {
	uint32_t pbits;  // P = 2^pbits partitions
	uint32_t ibits;  // partitioning work items of 2^ibits calls (<= cbits): a chunk is 2^(cbits-ibits) items
	__host__ __device__ uint32_t rbits() const { return 32 - pbits; }
	__host__ __device__ uint32_t cbits() const { return pbits - 2; }
	__host__ __device__ uint32_t items_per_chunk_log2() const { return cbits() - ibits; }
	__host__ __device__ uint32_t part(uint32_t h) const { return h >> (32 - pbits); }
	__host__ __device__ uint32_t meta(uint32_t level, uint64_t serial) const
	{
		return (level << cbits()) | ((uint32_t)serial & ((1u << cbits()) - 1));
	}
	__host__ __device__ uint32_t rec(uint32_t h, uint32_t meta) const { return (h << pbits) | meta; }
	__host__ __device__ uint32_t resid(uint32_t r) const { return r >> pbits; }
	__host__ __device__ uint32_t level(uint32_t r) const { return (r >> cbits()) & 3; }
	__host__ __device__ uint32_t local(uint32_t r) const { return r & ((1u << cbits()) - 1); }
};

// LDS home bucket of a residual: its top bits (h is already mixed)
__device__ __forceinline__ uint32_t agg_home_bucket(uint32_t key, const AggGeom& g)
{
	return __umulhi(key << g.pbits, kAggBuckets);
}

// Workgroup flag in LDS, read and set without `volatile`: a volatile access
// through a generic pointer compiles to a flat access whose vmcnt(0) wait
// drains every global load in flight (the record prefetch).
__device__ __forceinline__ uint32_t lds_flag(uint32_t* f)
{
	return __hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_flag_set(uint32_t* f)
{
	__hip_atomic_store(f, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// position of e in a 4-key bucket, 4 if absent
__device__ __forceinline__ uint32_t bucket_find(uint4 B, uint32_t e)
{
	return B.x == e ? 0 : B.y == e ? 1 : B.z == e ? 2 : B.w == e ? 3 : 4;
}
__device__ __forceinline__ uint32_t bucket_find(uint2 B, uint32_t e)
{
	return B.x == e ? 0 : B.y == e ? 1 : kAggBW;
}

// position of the first empty key in a 4-key bucket, 4 if full
__device__ __forceinline__ uint32_t bucket_first_empty(uint4 B)
{
	return B.x == kAggEmpty ? 0 : B.y == kAggEmpty ? 1 : B.z == kAggEmpty ? 2 : B.w == kAggEmpty ? 3 : 4;
}
__device__ __forceinline__ uint32_t bucket_first_empty(uint2 B)
{
	return B.x == kAggEmpty ? 0 : B.y == kAggEmpty ? 1 : kAggBW;
}

// Find-or-insert e in the LDS key buckets, bucket-linear from its home bucket
// b, whose snapshot B the caller already read.  Keys only go empty -> key, so
// a key is always at or before the first empty slot of its probe sequence:
// an insert is one ds_cmpst at the snapshot's first empty slot, re-reading the
// bucket only when another lane took that slot first.  Returns the slot
// (ins incremented if this call inserted e), or kAggNoSlot if the probe sequence ran
// through the whole table (the partition is then redone in HBM).
__device__ uint32_t agg_find_insert(KBucket* kb, uint32_t e, uint32_t b, KBucket B, uint32_t* s_ovf, uint32_t& ins)
{
	uint32_t* keys = reinterpret_cast<uint32_t*>(kb);
	for (uint32_t step = 0; step < kAggBuckets;) {
		const uint32_t f = bucket_find(B, e);
		if (f < kAggBW)
			return b * kAggBW + f;
		const uint32_t j = bucket_first_empty(B);
		if (j == kAggBW) {
			b = b + 1 == kAggBuckets ? 0 : b + 1;
			B = kb[b];
			step++;
			continue;
		}
		const uint32_t i = b * kAggBW + j;
		const uint32_t key = atomicCAS(&keys[i], kAggEmpty, e);
		if (key == kAggEmpty) {
			ins++;
			return i;
		}
		if (key == e)
			return i;
		B = kb[b];  // another lane filled the slot first
	}
	lds_flag_set(s_ovf);
	return kAggNoSlot;
}

// Cell boundaries of one group of kAggGroup chunks of a partition (uniform
// over the wave: scalar loads), and the serial of a record inside the group.
struct CellGroup {
	uint64_t ch0;
	uint32_t bnd[kAggGroup + 1];
	__device__ void load(const uint32_t* __restrict__ ot, uint64_t nchunks, uint64_t gi)
	{
		ch0 = gi * kAggGroup;
#pragma unroll
		for (uint32_t i = 0; i <= kAggGroup; i++)
			bnd[i] = ot[min<uint64_t>(ch0 + i, nchunks)];
	}
	__device__ uint32_t serial(uint32_t j, uint32_t r, const AggGeom& g) const
	{
		uint32_t chunk = (uint32_t)ch0;
#pragma unroll
		for (uint32_t i = 1; i < kAggGroup; i++)
			chunk += j >= bnd[i];
		return (chunk << g.cbits()) | g.local(r);
	}
};

// ---------------------------------------------------------------- partitioning
// Calls of the run [c0, c1) in work items of 2^ibits; counts[item][p].  kShard:
// only the records whose element shard x.shard of x.nshards owns (owner_of).
template <bool kShard>
__global__ __launch_bounds__(kAggThreads) void k_agg_count(const uint32_t* __restrict__ sigs,
                                                           const uint64_t* __restrict__ call_start,
                                                           const uint32_t* __restrict__ call_len, uint64_t c0,
                                                           uint64_t c1, AggGeom g, AggSrc x, uint32_t* counts)
{
	__shared__ uint32_t h[kAggMaxParts];
	auto add = [&](uint32_t e) {
		if (!kShard || owner_of(e, x.nshards) == x.shard)
			atomicAdd(&h[g.part(fmix32(e))], 1u);
	};
	const uint32_t P = 1u << g.pbits, cb = g.ibits;  // per work item of 2^ibits calls
	const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = lane_id();
	const uint64_t ncalls = c1 - c0, nchunks = (ncalls + (1ull << cb) - 1) >> cb;
	for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
		for (uint32_t i = threadIdx.x; i < P; i += blockDim.x)
			h[i] = 0;
		__syncthreads();
		const uint64_t ce = min<uint64_t>(ncalls, (ch + 1) << cb);
		for (uint64_t s = (ch << cb) + w; s < ce; s += nw) {
			const uint64_t c = c0 + s, start = call_start[c];
			const uint32_t len = call_len[c];
			uint32_t j = lane;
			for (; j + 192 < len; j += 256) {
				const uint32_t a = sigs[start + j], b = sigs[start + j + 64], d = sigs[start + j + 128],
				               f = sigs[start + j + 192];
				add(a);
				add(b);
				add(d);
				add(f);
			}
			for (; j < len; j += 64)
				add(sigs[start + j]);
		}
		__syncthreads();
		for (uint32_t i = threadIdx.x; i < P; i += blockDim.x)
			counts[ch * P + i] = h[i];
		__syncthreads();
	}
}

// exclusive scan over a 1024-thread block; returns the total
__device__ __forceinline__ uint32_t block_excl_scan_1k(uint32_t v, uint32_t* out)
{
	__shared__ uint32_t wsum[16];
	const uint32_t lane = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
	uint32_t x = v;
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint32_t y = __shfl_up(x, o, 64);
		if (lane >= (uint32_t)o)
			x += y;
	}
	if (lane == 63)
		wsum[w] = x;
	__syncthreads();
	uint32_t pre = 0, tot = 0;
	for (uint32_t i = 0; i < nw; i++) {
		pre += i < w ? wsum[i] : 0;
		tot += wsum[i];
	}
	__syncthreads();
	*out = pre + x - v;
	return tot;
}

// block p: exclusive scan over work items of counts[.][p] -> offs[.][p]
// (item-major, for the scatter) and, at every chunk's first item, offsT[p][.]
// (partition-major by chunk, the partition's total at [nchunks], for k_agg);
// totals[p].  An item is 2^ilog items of a chunk (ilog = 0: items are chunks).
__global__ __launch_bounds__(1024) void k_agg_scan_chunks(const uint32_t* counts, uint64_t nitems, uint32_t ilog,
                                                          uint32_t P, uint32_t* offs, uint32_t* offsT, uint64_t* totals)
{
	const uint32_t p = blockIdx.x;
	const uint64_t nchunks = (nitems + (1ull << ilog) - 1) >> ilog;
	uint32_t* ot = offsT + (uint64_t)p * (nchunks + 1);
	uint64_t run = 0;
	for (uint64_t b0 = 0; b0 < nitems; b0 += blockDim.x) {
		const uint64_t b = b0 + threadIdx.x;
		const uint32_t v = b < nitems ? counts[b * P + p] : 0;
		uint32_t ex;
		const uint32_t tot = block_excl_scan_1k(v, &ex);
		if (b < nitems) {
			offs[b * P + p] = (uint32_t)(run + ex);
			if ((b & ((1ull << ilog) - 1)) == 0)
				ot[b >> ilog] = (uint32_t)(run + ex);
		}
		run += tot;
	}
	if (threadIdx.x == 0) {
		totals[p] = run;
		ot[nchunks] = (uint32_t)run;
	}
}

// totals -> rec_base[P + 1] (one block of 1024 threads, P <= 2048: two
// partitions per thread, a wave scan, then the 16 wave sums)
__global__ __launch_bounds__(1024) void k_agg_scan_totals(const uint64_t* totals, uint32_t P, uint64_t* rec_base)
{
	__shared__ uint64_t wsum[16];
	const uint32_t lane = lane_id(), w = threadIdx.x >> 6, i0 = threadIdx.x * 2;
	const uint64_t a = i0 < P ? totals[i0] : 0, b = i0 + 1 < P ? totals[i0 + 1] : 0;
	uint64_t x = a + b;  // inclusive wave scan of the pair sums
#pragma unroll
	for (int o = 1; o < 64; o <<= 1) {
		const uint64_t y = __shfl_up(x, o, 64);
		if (lane >= (uint32_t)o)
			x += y;
	}
	if (lane == 63)
		wsum[w] = x;
	__syncthreads();
	uint64_t pre = 0, tot = 0;
	for (uint32_t k = 0; k < 16; k++) {
		pre += k < w ? wsum[k] : 0;
		tot += wsum[k];
	}
	const uint64_t ex = pre + x - (a + b);
	if (i0 < P)
		rec_base[i0] = ex;
	if (i0 + 1 < P)
		rec_base[i0 + 1] = ex + a;
	if (threadIdx.x == 0)
		rec_base[P] = tot;
}

// Records of each chunk -> their cells (fixed by the scan, so no global
// atomics).  A tile of kAggTile records lives in registers (kPer per lane),
// is counting-sorted by partition into LDS and written out as one run per
// partition; the runs of one chunk's consecutive tiles continue each other.
// The next tile's loads are issued before the write-out of the current one,
// so HBM reads overlap the stores instead of following them.
// kEntry (Minimize): the level comes from each record's own prio
// (x.elem_prio, parallel to sigs) instead of its call's, and only the records
// whose element shard x.shard owns are kept.
constexpr uint32_t kScatChunkMax = 1u << (kAggMaxBits - 2);  // calls per chunk (cbits <= 9)

// Capped cells (the count-free layout of a triage run):
// chunk c's cells are consecutive regions of cap[c] records (a multiple of 64)
// from base[c], partition after partition; the scatter writes cnt[p][c] and
// raises *ovf when a cell receives more than its capacity (the run is then
// redone with counted cells).
struct CapCells {
	const uint64_t* base;  // [nchunks] first record of chunk c's cells
	const uint32_t* cap;   // [nchunks] records per cell of chunk c
	uint32_t* cnt;         // [P][nchunks] records in cell (c, p)
	uint32_t* ovf;         // set to 1 by a cell overflow
	uint64_t nchunks;
	uint32_t* dummy;       // one 64-B line per block: the target of stores that are not made
	// Two triage scatters over one run (round 6): with split set, k_scat3 takes
	// the work items its one-call tiles would fill (scat3_takes: sizes[] =
	// records, tiles[] = k_scat3 tiles per item) and k_agg_scatter_blk the
	// rest, each skipping the other's items
	const uint64_t* sizes = nullptr;
	const uint32_t* tiles = nullptr;
	bool split = false;
	uint32_t tile = 1024;  // records per k_scat3 tile the tiles[] were counted in (set with tiles)
};

#ifndef SYZ_SCAT3  // triage runs: 0 = k_agg_scatter_blk only, 1 = k_scat3 for the items it fills
#define SYZ_SCAT3 1
#endif
#ifndef SYZ_SCAT3_K  // records per lane per tile
#define SYZ_SCAT3_K 16
#endif
#ifndef SYZ_SCAT3_ENTRY  // Minimize's work items (one shard) through k_scat3 too, split as for triage
#define SYZ_SCAT3_ENTRY 1
#endif
#ifndef SYZ_SCAT3_FILL  // % of its tiles' lanes an item must fill for k_scat3 to take it
#define SYZ_SCAT3_FILL 85
#endif
#ifndef SYZ_SCAT3_V  // k_scat3's flush: dwords per lane (1, or 4: 16-B lanes)
#define SYZ_SCAT3_V 4
#endif
#ifndef SYZ_SCAT_V  // the same for k_agg_scatter_blk
#define SYZ_SCAT_V 4
#endif
typedef uint32_t scat_v4u __attribute__((ext_vector_type(4)));
#ifndef SYZ_SCAT3_T  // threads per workgroup (1024: 4 waves per SIMD, 128 registers; 768: 3, 168; 512: 2, 256)
#define SYZ_SCAT3_T 1024
#endif

// k_scat3's tiles of one work item (every call in ceil(len / tile) tiles), and
// the split between the two triage scatters: k_scat3 takes an item whose tiles
// would be at least SYZ_SCAT3_FILL % full, k_agg_scatter_blk the others.
#ifndef SYZ_SCAT3_KE  // records per lane per tile with per-record levels (Minimize: the prios take registers)
#define SYZ_SCAT3_KE 10
#endif
constexpr uint32_t kScat3Tile = SYZ_SCAT3_K * 64, kScat3TileEntry = SYZ_SCAT3_KE * 64;
__host__ __device__ inline uint64_t scat3_tiles(uint32_t len, uint32_t tile)
{
	return (len + tile - 1) / tile;
}
__device__ inline bool scat3_takes(uint64_t recs, uint32_t tiles, uint32_t tile)
{
	return recs * 100 >= (uint64_t)tiles * tile * SYZ_SCAT3_FILL;
}

template <bool kEntry>
__global__ __launch_bounds__(kAggThreads) void k_agg_scatter(const uint32_t* __restrict__ sigs,
                                                             const uint64_t* __restrict__ call_start,
                                                             const uint32_t* __restrict__ call_len,
                                                             const uint8_t* __restrict__ call_prio, LevelMap lm,
                                                             uint64_t c0, uint64_t c1, AggGeom g, AggSrc x,
                                                             const uint32_t* __restrict__ offs,
                                                             const uint64_t* __restrict__ rec_base, uint32_t* recs)
{
	constexpr uint32_t kWaves = kAggThreads / 64, kQuota = kAggTile / kWaves, kPer = kQuota / 64;
	static_assert(kQuota % 64 == 0, "tile quota per wave");
	__shared__ uint32_t t_rec[kAggTile];   // sorted by partition: packed records
	__shared__ uint16_t t_part[kAggTile];  // ... and their partitions
	__shared__ uint64_t cur[kAggMaxParts];
	__shared__ uint32_t hist[kAggMaxParts], pos[kAggMaxParts];
	__shared__ uint64_t c_start[kScatChunkMax];  // the chunk's calls
	__shared__ uint32_t c_len[kScatChunkMax];
	__shared__ uint16_t c_meta[kScatChunkMax];
	__shared__ uint8_t s_lvl[kEntry ? 256 : 1];
	const uint32_t P = 1u << g.pbits, cb = g.cbits(), ib = g.ibits;
	if (kEntry) {
		for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x)
			s_lvl[i] = lm.lvl[i];
	}
	const uint32_t w = threadIdx.x >> 6, lane = lane_id();
	const uint64_t ncalls = c1 - c0, nitems = (ncalls + (1ull << ib) - 1) >> ib;
	const uint32_t per_t = (P + blockDim.x - 1) / blockDim.x;
	bool badlv = false;
	for (uint64_t ch = blockIdx.x; ch < nitems; ch += gridDim.x) {  // ch: work item (of 2^ibits calls)
		const uint64_t cbeg = ch << ib;
		const uint32_t nc = (uint32_t)min<uint64_t>(ncalls - cbeg, 1ull << ib);
		for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
			cur[i] = rec_base[i] + offs[ch * P + i];
			hist[i] = 0;
		}
		for (uint32_t i = threadIdx.x; i < nc; i += blockDim.x) {
			const uint64_t c = c0 + cbeg + i;
			c_start[i] = call_start[c];
			c_len[i] = call_len[c];
			c_meta[i] = (uint16_t)g.meta(kEntry ? 0 : lm.lvl[call_prio[c]], cbeg + i);
		}
		__syncthreads();
		// this wave's walk: local call wc (then +kWaves), offset wo inside it
		uint32_t wc = w, wo = 0;
		// Per record slot: loc = (wave call number j << 24) | offset in the call
		// (calls hold < 2^24 records, batch validation); the wave's j-th call
		// is local call w + j * kWaves (j < 2^cbits / kWaves <= 32).
		uint32_t ev[kPer], loc[kPer];
		int8_t pv[kEntry ? kPer : 1];
		// issue the loads of this wave's next quota; returns how many records it has
		auto fetch = [&]() -> uint32_t {
			uint32_t q = 0;
			while (q < kQuota && wc < nc) {
				const uint32_t len = c_len[wc], m = min(kQuota - q, len - wo);
				const uint32_t tag = ((wc - w) / kWaves) << 24;
				if (q == 0) {
#pragma unroll
					for (uint32_t u = 0; u < kPer; u++)
						loc[u] = tag | wo;  // clamped default: a valid address
				}
#pragma unroll
				for (uint32_t u = 0; u < kPer; u++) {
					const uint32_t i = u * 64 + lane;
					loc[u] = i >= q && i < q + m ? tag | (wo + i - q) : loc[u];
				}
				q += m;
				wo += m;
				if (wo == len) {
					wc += kWaves;
					wo = 0;
				}
			}
			if (q) {
#pragma unroll
				for (uint32_t u = 0; u < kPer; u++) {
					const uint64_t a = c_start[w + (loc[u] >> 24) * kWaves] + (loc[u] & 0xFFFFFFu);
					ev[u] = __builtin_nontemporal_load(&sigs[a]);
					if (kEntry)
						pv[kEntry ? u : 0] = __builtin_nontemporal_load(&x.elem_prio[a]);
				}
			}
			return q;
		};
		uint32_t n = fetch();
		for (;;) {
			// stage: partition and rank of every record of the tile (loc = ~0: not kept)
#pragma unroll
			for (uint32_t u = 0; u < kPer; u++) {
				const uint32_t i = u * 64 + lane;
				const bool keep = i < n && (!kEntry || x.nshards == 1 || owner_of(ev[u], x.nshards) == x.shard);
				if (keep) {
					const uint32_t h = fmix32(ev[u]), p = g.part(h);
					const uint32_t r = atomicAdd(&hist[p], 1u);
					uint32_t meta = c_meta[w + (loc[u] >> 24) * kWaves];
					if (kEntry) {
						const uint32_t lv = s_lvl[(uint8_t)pv[kEntry ? u : 0]];
						badlv |= lv == 0xff;
						meta |= (lv & 3) << cb;
					}
					ev[u] = g.rec(h, meta);
					loc[u] = p | (r << 16);
				} else {
					loc[u] = ~0u;
				}
			}
			__syncthreads();
			// exclusive scan of hist; pos[p] = the partition's first sorted position
			uint32_t hsum = 0;
			for (uint32_t q = 0; q < per_t; q++) {
				const uint32_t i = threadIdx.x * per_t + q;
				hsum += i < P ? hist[i] : 0;
			}
			uint32_t ex;
			const uint32_t nt = block_excl_scan_1k(hsum, &ex);  // records kept in the tile
			for (uint32_t q = 0; q < per_t; q++) {
				const uint32_t i = threadIdx.x * per_t + q;
				if (i < P) {
					pos[i] = ex;
					cur[i] -= ex;  // cur[p] + d = output index of sorted position d (u64 wrap intended)
					ex += hist[i];
				}
			}
			__syncthreads();
#pragma unroll
			for (uint32_t u = 0; u < kPer; u++) {
				if (loc[u] != ~0u) {
					const uint32_t p = loc[u] & 0xFFFFu, d = pos[p] + (loc[u] >> 16);
					t_rec[d] = ev[u];
					t_part[d] = (uint16_t)p;
				}
			}
			// next tile's loads fly during the write-out
			n = fetch();
			__syncthreads();
			// consecutive threads write consecutive records of one partition's run
			for (uint32_t d = threadIdx.x; d < nt; d += blockDim.x)
				recs[cur[t_part[d]] + d] = t_rec[d];
			__syncthreads();
			for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
				cur[i] += pos[i] + hist[i];  // advance by the run
				hist[i] = 0;
			}
			if (!__syncthreads_or(n != 0))
				break;
		}
	}
	if (kEntry && x.bad_level && __ballot(badlv) && lane == 0)
		atomicOr(x.bad_level, 1u);
}

// Capped cells written in whole 64-B blocks (the triage runs' scatter).
// A store costs one memory request per 64-B segment it touches, whatever the
// bytes: a ~9-record piece of a cell at an arbitrary offset touches ~1.6
// segments, a whole aligned block one (scripts/mb_scatter.hip: 2.0-2.3 vs
// 3.4-3.8 TB/s read+write).  So every partition has a write-combining buffer
// of one block in LDS (2048 x 64 B): records go from registers straight into
// their partition's buffer (one ds_add_rtn for a slot, one ds_write), and a
// buffer that fills is written out whole, 16 lanes per block; a record that
// finds its buffer full waits for the flush (next sub-round).  No tile sort,
// no scan.  A cell's last partial block is written when its chunk ends.
constexpr uint32_t kBlk = 16;            // records per written block (64 B)
constexpr uint32_t kDummyLines = 2048;  // CapCells::dummy lines
// records per lane per tile
#ifndef SYZ_SCAT_PER
#define SYZ_SCAT_PER 12
#endif
#ifndef SYZ_SCAT_PER_ENTRY  // (Minimize: the prios take registers too)
#define SYZ_SCAT_PER_ENTRY 10
#endif

// Work items of 2^ibits calls own their cells (items = chunks for a triage
// batch).  kEntry (Minimize): the level comes from each record's own prio
// (x.elem_prio), and only the records whose element shard x.shard owns are kept.
// kMaxP: the partitions the LDS is sized for; kWpe: waves per SIMD the
// registers are sized for (4: one workgroup per CU, 8: two, each with half
// the LDS: 1024 partitions of 64-B blocks).
template <bool kEntry, uint32_t kB, uint32_t kMaxP = kAggMaxParts, uint32_t kWpe = 4, uint32_t kT = kAggThreads>
__global__ __launch_bounds__(kT, kWpe) void k_agg_scatter_blk(const uint32_t* __restrict__ sigs,
                                                                 const uint64_t* __restrict__ call_start,
                                                                 const uint32_t* __restrict__ call_len,
                                                                 const uint8_t* __restrict__ call_prio, LevelMap lm,
                                                                 uint64_t c0, uint64_t c1, AggGeom g, AggSrc x,
                                                                 CapCells cc, uint32_t* recs, uint32_t dbg)
{
	constexpr uint32_t kWaves = kT / 64, kPer = kEntry ? SYZ_SCAT_PER_ENTRY : SYZ_SCAT_PER, kQuota = kPer * 64;
	constexpr uint32_t kG = 64 / kB;  // blocks a wave writes per store (kB lanes each)
	static_assert(kB == 16 || kB == 32, "block of 64 or 128 B");
	constexpr uint32_t kChunkMax = kMaxP / 4;        // calls per chunk (cbits = pbits - 2)
	__shared__ __align__(16) uint32_t buf[kMaxP * (kMaxP == kAggMaxParts ? kBlk : kB)];  // per partition: the block being filled
	__shared__ uint32_t fillc[kMaxP + 1];   // slots handed out in it (may overshoot kB)
	__shared__ uint32_t written[kMaxP + 1]; // records of the cell written so far (+ a spare)
	// full blocks found after the sub-round's barrier by a scan of the counts,
	// every wave over its own share of the partitions (as in k_scat3)
	constexpr uint32_t kShare = (kMaxP + kT - 1) / kT;  // partitions per lane in the scan
	__shared__ uint16_t flist[kShare * kT]; // per wave: partitions whose block filled this sub-round
	__shared__ uint64_t c_start[kChunkMax]; // the chunk's calls
	__shared__ uint32_t c_len[kChunkMax];
	__shared__ uint16_t c_meta[kChunkMax];
	__shared__ uint8_t s_lvl[kEntry ? 256 : 1];
	__shared__ uint32_t s_or[2][kWaves];
	const uint32_t P = 1u << g.pbits, cb = g.cbits(), ib = g.ibits;
	// the flush: kV dwords per lane (16-B lanes as in k_scat3)
	constexpr uint32_t kV = SYZ_SCAT_V, kLB = kB / kV, kGF = 64 / kLB;
	using FV = std::conditional_t<kV == 4, scat_v4u, uint32_t>;
	const uint32_t w = threadIdx.x >> 6, lane = lane_id(), grp = lane / kB, slot = lane & (kB - 1), fgrp = lane / kLB,
	               fq = lane % kLB;
	// Workgroup OR in one barrier (__syncthreads_or takes three): every wave
	// writes its flag to a row, all read the row; two rows alternate, so a row
	// is rewritten only after every wave passed the barrier of the call between.
	uint32_t seq = 0;
	auto wg_or = [&](bool pred) -> bool {
		uint32_t* r = s_or[seq++ & 1];
		const bool any = __ballot(pred) != 0;
		if (lane == 0)
			r[w] = any;
		__syncthreads();
		return __ballot(r[lane & (kWaves - 1)] != 0) != 0;  // lane i reads wave i's flag
	};
	const uint64_t ncalls = c1 - c0, nchunks = (ncalls + (1ull << ib) - 1) >> ib;  // work items
	if (*cc.ovf)
		return;  // the run is already void (an optimistic run's assumptions failed, or a cell spilled)
	bool spilled = false, badlv = false;
	if (kEntry) {
		for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x)
			s_lvl[kEntry ? i : 0] = lm.lvl[i];
	}
	for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
		const uint64_t cbeg = ch << ib;
		const uint32_t nc = (uint32_t)min<uint64_t>(ncalls - cbeg, 1ull << ib);
		if (cc.split && scat3_takes(cc.sizes[ch], cc.tiles[ch], cc.tile))
			continue;  // long calls: k_scat3's item
		const uint32_t cap = cc.cap[ch];
		const uint64_t cbase = cc.base[ch];
		for (uint32_t i = threadIdx.x; i < P; i += blockDim.x) {
			fillc[i] = 0;
			written[i] = 0;
		}
		for (uint32_t i = threadIdx.x; i < nc; i += blockDim.x) {
			const uint64_t c = c0 + cbeg + i;
			c_start[i] = call_start[c];
			c_len[i] = call_len[c];
			c_meta[i] = (uint16_t)g.meta(kEntry ? 0 : lm.lvl[call_prio[c]], cbeg + i);
		}
		__syncthreads();
		uint32_t wc = w, wo = 0;  // this wave's walk: local call wc (then +kWaves), offset wo inside it
		uint32_t pv[kEntry ? kPer : 1];  // kEntry: the records' prios (of the last fetch)
		// issue the loads of this wave's next quota; returns how many records it has
		auto fetch = [&](uint32_t (&ev)[kPer], uint32_t (&loc)[kPer]) -> uint32_t {
			uint32_t q = 0;
			while (q < kQuota && wc < nc) {
				const uint32_t len = c_len[wc], m = min(kQuota - q, len - wo);
				const uint32_t tag = ((wc - w) / kWaves) << 24;
				if (q == 0) {
#pragma unroll
					for (uint32_t u = 0; u < kPer; u++)
						loc[u] = tag | wo;  // clamped default: a valid address
				}
#pragma unroll
				for (uint32_t u = 0; u < kPer; u++) {
					const uint32_t i = u * 64 + lane;
					loc[u] = i >= q && i < q + m ? tag | (wo + i - q) : loc[u];
				}
				q += m;
				wo += m;
				if (wo == len) {
					wc += kWaves;
					wo = 0;
				}
			}
			if (q) {
#pragma unroll
				for (uint32_t u = 0; u < kPer; u++) {
					const uint64_t at = c_start[w + (loc[u] >> 24) * kWaves] + (loc[u] & 0xFFFFFFu);
					ev[u] = __builtin_nontemporal_load(&sigs[at]);
					if (kEntry)
						pv[kEntry ? u : 0] = (uint8_t)__builtin_nontemporal_load(&x.elem_prio[at]);
				}
			}
			return q;
		};
		// write out the blocks of this wave's share that filled in this
		// sub-round: kLB lanes per block
		auto flush = [&]() {
			uint16_t* wl = flist + w * kShare * 64;  // this wave's list
			uint32_t nw = 0;
#pragma unroll
			for (uint32_t i = 0; i < kShare; i++) {
				const uint32_t p = i * kT + w * 64 + lane;
				const bool f = p < P && fillc[p] >= kB;
				const uint64_t m = __ballot(f);
				if (f)
					wl[nw + lane_rank(m)] = (uint16_t)p;
				nw += (uint32_t)__popcll(m);
			}
			// (the wave's LDS operations run in order: the list is read below as written)
			for (uint32_t jb = 0; jb < nw; jb += kGF) {
				const bool ok = jb + fgrp < nw;
				const uint32_t pp = wl[min(jb + fgrp, nw - 1)];
				const uint32_t wr = written[pp];
				const FV v = *reinterpret_cast<const FV*>(&buf[pp * kB + fq * kV]);
				const bool fits = wr + kB <= cap;
				spilled |= ok && !fits;  // the cell is full: the run is redone with counted cells
				uint32_t* d = ok && fits ? recs + cbase + (uint64_t)pp * cap + wr
				                         : cc.dummy + (blockIdx.x % (kDummyLines * kBlk / kB)) * kB;
				*reinterpret_cast<FV*>(d + fq * kV) = v;
				__builtin_amdgcn_wave_barrier();
				if (fq == 0 && ok) {
					written[pp] = wr + kB;
					fillc[pp] = 0;
				}
			}
		};
		// a tile's records: packed record and partition, and the mask of those to place
		auto pack = [&](const uint32_t (&ev)[kPer], const uint32_t (&loc)[kPer], uint32_t n, uint32_t (&rec)[kPer],
		                uint32_t (&pt)[kPer]) -> uint32_t {
			uint32_t pend = 0;
#pragma unroll
			for (uint32_t u = 0; u < kPer; u++) {
				const uint32_t h = fmix32(ev[u]);
				pt[u] = g.part(h);
				uint32_t meta = c_meta[w + (loc[u] >> 24) * kWaves];
				const bool keep = !kEntry || x.nshards == 1 || owner_of(ev[u], x.nshards) == x.shard;
				if (kEntry) {
					const uint32_t lv = s_lvl[pv[kEntry ? u : 0]];
					badlv |= u * 64 + lane < n && keep && lv == 0xff;
					meta |= (lv & 3) << cb;
				}
				rec[u] = g.rec(h, meta);
				pend |= (uint32_t)(u * 64 + lane < n && keep) << u;
			}
#ifdef SYZ_EXPERIMENTS
			return dbg & 2 ? 0u : pend;  // dbg & 2: timing only, records loaded and dropped
#else
			// (the bit is SYZSIG_DEBUG_EDGE_PASSES >> 10 in product builds: ignored here)
			return pend;
#endif
		};
		// one placement pass: a slot in each record's partition block (all slot
		// requests in flight together), or it waits for the block's flush.
		// Returns what is left.
		auto place = [&](const uint32_t (&rec)[kPer], const uint32_t (&pt)[kPer], uint32_t pend) -> uint32_t {
			uint32_t sl[kPer];
#pragma unroll
			for (uint32_t u = 0; u < kPer; u++)
				sl[u] = (pend >> u) & 1 ? atomicAdd(&fillc[pt[u]], 1u) : kB;
#pragma unroll
			for (uint32_t u = 0; u < kPer; u++) {
				if (sl[u] < kB) {
					buf[pt[u] * kB + sl[u]] = rec[u];
					pend &= ~(1u << u);
				}
			}
			return pend;
		};
		uint32_t ev[kPer], loc[kPer];
		uint32_t n = fetch(ev, loc);
		for (;;) {
			uint32_t rec[kPer], pt[kPer];
			uint32_t pend = pack(ev, loc, n, rec, pt);
			n = fetch(ev, loc);  // the next tile's loads fly while this one is placed
			for (;;) {
				pend = place(rec, pt, pend);
				const bool more = wg_or(pend != 0);
				flush();
				if (!more)
					break;
				__syncthreads();
			}
			if (!wg_or(n != 0))  // (its barrier also ends the last flush)
				break;
		}
		// the chunk's last partial block of every cell, and the cell counts
		for (uint32_t p = w * kG + grp; p < P; p += kWaves * kG) {
			const uint32_t c = fillc[p], wr = written[p];
			if (wr + c > cap)
				spilled = true;
			else if (slot < c)
				recs[cbase + (uint64_t)p * cap + wr + slot] = buf[p * kB + slot];
			if (slot == 0)
				cc.cnt[(uint64_t)p * cc.nchunks + ch] = min(wr + c, cap);
		}
		__syncthreads();  // fillc/written/buf are reset by the next chunk
	}
	if (spilled)
		*cc.ovf = 1u;
	if (kEntry && x.bad_level && __ballot(badlv) && lane == 0)
		atomicOr(x.bad_level, 1u);
}

// The lean scatter of triage runs (round 6): the same capped cells and 64-B
// write-combining blocks, with the per-record bookkeeping of the loads taken
// out.  A wave walks whole calls (calls w, w + kWaves, .. of its chunk) in
// tiles of up to kK * 64 records of ONE call: the tile's start, level and
// serial are wave-uniform scalars (s_load of the call, no LDS call table),
// so a record costs its load, fmix32, one ds_add_rtn and one ds_write.
// The kernel was bound by VALU issue (about 1,200 vector instructions per
// wave and tile of 16 records per lane), so: the flush moves 16 B per lane
// (ds_read_b128, global_store_dwordx4: a quarter of its instructions of 4-B
// lanes), the pending mask comes from the record count, and no flush list is
// built while placing (no per-record "block full" test, no list append):
// after the sub-round's barrier each wave scans the counts of its own share
// of the partitions and flushes the blocks of its share that filled.
// Variants measured slower and removed: two
// workgroups per CU each placing one half of the partitions, records that
// met a full block carried in registers to the next tile, and one slot claim
// per record with the claims past a full block written into its next fill
// (half the barriers, no second claim, but more instructions per tile).
template <uint32_t kT, uint32_t kK, uint32_t kWpe, bool kEntry = false, uint32_t kB = kBlk>
__global__ __launch_bounds__(kT, kWpe) void k_scat3(const uint32_t* __restrict__ sigs,
                                                    const uint64_t* __restrict__ call_start,
                                                    const uint32_t* __restrict__ call_len,
                                                    const uint8_t* __restrict__ call_prio, LevelMap lm, uint64_t c0,
                                                    uint64_t c1, AggGeom g, CapCells cc, uint32_t* recs, AggSrc x)
{
	// kEntry (Minimize, one shard): every record's level comes from its own
	// prio (x.elem_prio, parallel to sigs); kB = 32: 128-B blocks for <= 1024
	// partitions (the same 128 KB of LDS)
	constexpr uint32_t kWaves = kT / 64, kG = 64 / kB, kTile = kK * 64;
	constexpr uint32_t kMaxP = kAggMaxParts * kBlk / kB;
	static_assert(kB == 16 || kB == 32, "block of 64 or 128 B");
	// a flush lane moves kV dwords (4: 16-B LDS reads and block stores, kB / 4
	// lanes per block -- a quarter of the flush's instructions of 4-B lanes)
	constexpr uint32_t kV = SYZ_SCAT3_V, kLB = kB / kV, kGF = 64 / kLB;
	using FV = std::conditional_t<kV == 4, scat_v4u, uint32_t>;
	static_assert(kV == 1 || kV == 4, "flush lanes of 4 or 16 B");
	static_assert(kK <= 31, "pending masks are 32-bit");
	__shared__ __align__(16) uint32_t buf[kMaxP * kB];  // per partition: the block being filled
	__shared__ uint32_t fillc[kMaxP + 1];     // slots handed out in it (may overshoot kB)
	__shared__ uint32_t written[kMaxP + 1];   // records of the cell written so far (+ a spare)
	// No flush list is built while placing: after the sub-round's barrier
	// every wave scans its own share of the partitions' counts (partition
	// i * kT + w * 64 + lane) and flushes the blocks of its share that filled,
	// listed in its own slice of flist
	constexpr uint32_t kShare = (kMaxP + kT - 1) / kT;  // partitions per lane in the scan
	__shared__ uint16_t flist[kShare * kT];   // per wave: partitions whose block filled this sub-round
	__shared__ uint32_t s_or[2][kWaves];
	__shared__ uint8_t s_lvl[256];            // prio -> level (an LDS read: lgkmcnt, not vmcnt)
	const uint32_t Pl = 1u << g.pbits;
	// (w through readfirstlane: the compiler then knows the call walk is
	// wave-uniform and reads the calls with scalar loads, which wait on
	// lgkmcnt -- a vector load there would need vmcnt(0), draining the
	// prefetch and the block stores)
	const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id(), grp = lane / kB,
	               slot = lane & (kB - 1), fgrp = lane / kLB, fq = lane % kLB;
	uint32_t seq = 0;
	auto wg_or = [&](bool pred) -> bool {  // workgroup OR in one barrier (k_agg_scatter_blk)
		uint32_t* r = s_or[seq++ & 1];
		const bool any = __ballot(pred) != 0;
		if (lane == 0)
			r[w] = any;
		__syncthreads();
		return __ballot(lane < kWaves && r[lane < kWaves ? lane : 0] != 0) != 0;
	};
	const uint64_t ncalls = c1 - c0, nchunks = (ncalls + (1ull << g.ibits) - 1) >> g.ibits;
	if (*cc.ovf)
		return;  // the run is already void
	bool spilled = false, badlv = false;
	for (uint32_t i = threadIdx.x; i < 256; i += kT)
		s_lvl[i] = lm.lvl[i];
	for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {  // work items
		const uint64_t cbeg = ch << g.ibits;
		const uint32_t nc = (uint32_t)min<uint64_t>(ncalls - cbeg, 1ull << g.ibits);
		if (cc.split && !scat3_takes(cc.sizes[ch], cc.tiles[ch], cc.tile))
			continue;  // short calls: k_agg_scatter_blk's item
		const uint32_t cap = cc.cap[ch];
		const uint64_t cbase = cc.base[ch];
		for (uint32_t i = threadIdx.x; i < Pl; i += kT) {
			fillc[i] = 0;
			written[i] = 0;
		}
		__syncthreads();
		// this wave's call walk (wave-uniform): call j of the chunk, offset wo
		uint32_t j = w, wo = 0, clen = 0, cmeta = 0;
		uint64_t cstart = 0;
		auto open_call = [&]() {
			while (j < nc) {
				const uint64_t c = c0 + cbeg + j;
				clen = call_len[c];
				if (clen) {
					cstart = call_start[c];
					// the prio byte through a scalar dword load of its aligned word
					// (a byte load would be a vector load, waited for with vmcnt(0))
					const uintptr_t pa = (uintptr_t)(call_prio + c);
					const uint32_t word =
					    *(const __attribute__((address_space(4))) uint32_t*)(pa & ~(uintptr_t)3);  // (constant: s_load)
					cmeta = g.meta(kEntry ? 0 : s_lvl[(word >> (8 * (pa & 3))) & 0xFF], cbeg + j);
					return;
				}
				j += kWaves;
			}
		};
		open_call();
		// the next tile's loads: v[] and its scalars (records n, meta); n = 0: none
		auto fetch = [&](uint32_t (&v)[kK], uint32_t (&pv)[kEntry ? kK : 1], uint32_t& n, uint32_t& meta) {
			n = j < nc ? min(kTile, clen - wo) : 0u;
			meta = cmeta;
			const uint32_t* src = sigs + cstart + wo;
			const uint32_t last = n ? n - 1 : 0;
#pragma unroll
			for (uint32_t u = 0; u < kK; u++)
				v[u] = __builtin_nontemporal_load(&src[min(u * 64 + lane, last)]);
			if constexpr (kEntry) {
				const int8_t* psrc = x.elem_prio + cstart + wo;
#pragma unroll
				for (uint32_t u = 0; u < kK; u++)
					pv[u] = (uint8_t)__builtin_nontemporal_load(&psrc[min(u * 64 + lane, last)]);
			}
			if (n) {
				wo += n;
				if (wo == clen) {
					wo = 0;
					j += kWaves;
					open_call();
				}
			}
		};
		auto flush = [&]() {
			uint16_t* wl = flist + w * kShare * 64;  // this wave's list
			uint32_t nw = 0;
#pragma unroll
			for (uint32_t i = 0; i < kShare; i++) {
				const uint32_t p = i * kT + w * 64 + lane;
				const bool f = p < Pl && fillc[p] >= kB;
				const uint64_t m = __ballot(f);
				if (f)
					wl[nw + lane_rank(m)] = (uint16_t)p;
				nw += (uint32_t)__popcll(m);
			}
			// (the wave's LDS operations run in order: the list is read below as written)
			for (uint32_t jb = 0; jb < nw; jb += kGF) {
				const bool ok = jb + fgrp < nw;
				const uint32_t pp = wl[min(jb + fgrp, nw - 1)];
				const uint32_t wr = written[pp];
				const FV vv = *reinterpret_cast<const FV*>(&buf[pp * kB + fq * kV]);
				const bool fits = wr + kB <= cap;
				spilled |= ok && !fits;
				uint32_t* d = ok && fits ? recs + cbase + (uint64_t)pp * cap + wr
				                         : cc.dummy + (blockIdx.x % (kDummyLines * kBlk / kB)) * kB;
				*reinterpret_cast<FV*>(d + fq * kV) = vv;
				__builtin_amdgcn_wave_barrier();
				if (fq == 0 && ok) {
					written[pp] = wr + kB;
					fillc[pp] = 0;
				}
			}
		};
		auto pack = [&](const uint32_t (&v)[kK], const uint32_t (&pv)[kEntry ? kK : 1], uint32_t n, uint32_t meta,
		                uint32_t (&rec)[kK], uint32_t (&pt)[kK]) -> uint32_t {
			uint32_t pend = 0;
#pragma unroll
			for (uint32_t u = 0; u < kK; u++) {
				const uint32_t h = fmix32(v[u]), p = g.part(h);
				pt[u] = p;
				uint32_t m = meta;
				if constexpr (kEntry) {
					const uint32_t lv = s_lvl[pv[kEntry ? u : 0]];
					badlv |= u * 64 + lane < n && lv == 0xff;
					m |= (lv & 3) << g.cbits();
				}
				rec[u] = g.rec(h, m);
			}
			{  // records u * 64 + lane < n: the lane's first nu (a mask, not a compare per record)
				const uint32_t nu = n > lane ? (n - lane + 63) >> 6 : 0u;  // (<= kK <= 31)
				pend = (1u << nu) - 1;
			}
#if defined(SYZ_EXPERIMENTS) && defined(SYZ_SCAT3_DBG)  // timing only (results wrong): 1 = nothing placed
			if (SYZ_SCAT3_DBG == 1)
				pend = 0;
#endif
			return pend;
		};
		auto place = [&](const auto& rec, const auto& pt, uint32_t pend) -> uint32_t {
			constexpr uint32_t M = sizeof(rec) / sizeof(rec[0]);
			uint32_t sl[M];
#pragma unroll
			for (uint32_t u = 0; u < M; u++)
				sl[u] = (pend >> u) & 1 ? atomicAdd(&fillc[pt[u]], 1u) : kB;
#pragma unroll
			for (uint32_t u = 0; u < M; u++) {
				if (sl[u] < kB) {
					buf[pt[u] * kB + sl[u]] = rec[u];
					pend &= ~(1u << u);
				}
			}
			return pend;
		};
		// one tile: place in sub-rounds until every record is in a block
		auto tile = [&](const uint32_t (&v)[kK], const uint32_t (&pv)[kEntry ? kK : 1], uint32_t n, uint32_t meta) {
			uint32_t rec[kK], pt[kK];
			uint32_t pend = pack(v, pv, n, meta, rec, pt);
			for (;;) {
				pend = place(rec, pt, pend);
				const bool more = wg_or(pend != 0);
				flush();
				if (!more)
					break;
				__syncthreads();
			}
		};
		// two register buffers in turn (static indices: the prefetch lands
		// where it is consumed, no moves that would wait for it)
		uint32_t va[kK], vb[kK], pa[kEntry ? kK : 1], pb[kEntry ? kK : 1], na, nb, ma, mb;
		fetch(va, pa, na, ma);
		for (;;) {
			fetch(vb, pb, nb, mb);
			tile(va, pa, na, ma);
			if (!wg_or(nb != 0))  // (its barrier also ends the last flush)
				break;
			fetch(va, pa, na, ma);
			tile(vb, pb, nb, mb);
			if (!wg_or(na != 0))
				break;
		}
		// the chunk's last partial block of every cell, and the cell counts
		for (uint32_t p = w * kG + grp; p < Pl; p += kWaves * kG) {
			const uint32_t c = fillc[p], wr = written[p];
			const uint32_t pg = p;
			if (wr + c > cap)
				spilled = true;
			else if (slot < c)
				recs[cbase + (uint64_t)pg * cap + wr + slot] = buf[p * kB + slot];
			if (slot == 0)
				cc.cnt[(uint64_t)pg * cc.nchunks + ch] = min(wr + c, cap);
		}
		__syncthreads();  // fillc/written/buf are reset by the next work item
	}
	if (spilled)
		*cc.ovf = 1u;
	if (kEntry && x.bad_level && __ballot(badlv) && lane == 0)
		atomicOr(x.bad_level, 1u);
}


// The scatter's write-combining blocks fill the same 128 KB of LDS: 64 B per
// partition at 2048 partitions, whole 128-B lines at <= 1024.
#ifndef SYZ_SCAT_WIDE
#define SYZ_SCAT_WIDE 1
#endif
// The triage runs' scatter (kEntry = false): k_scat3 when built with
// SYZ_SCAT3 (at most kAggMaxParts partitions), else k_agg_scatter_blk.
static void scatter_triage(uint64_t nchunks, hipStream_t s, uint32_t pbits, const uint32_t* sigs,
                           const uint64_t* call_start, const uint32_t* call_len, const uint8_t* call_prio, LevelMap lm,
                           uint64_t c0, uint64_t c1, AggGeom g, AggSrc x, CapCells cc, uint32_t* recs, uint32_t dbg);
static uint64_t nchunks_of(uint64_t ncalls, uint32_t ibits)
{
	return (ncalls + (1ull << ibits) - 1) >> ibits;
}

template <bool kEntry, typename... A>
static void scatter_blk(uint32_t grid, hipStream_t s, uint32_t pbits, A... a)
{
	if (SYZ_SCAT_WIDE && pbits < kAggMaxBits)
		k_agg_scatter_blk<kEntry, 32><<<grid, kAggThreads, 0, s>>>(a...);
	else
		k_agg_scatter_blk<kEntry, 16><<<grid, kAggThreads, 0, s>>>(a...);
}

static void scatter_triage(uint64_t nchunks, hipStream_t s, uint32_t pbits, const uint32_t* sigs,
                           const uint64_t* call_start, const uint32_t* call_len, const uint8_t* call_prio, LevelMap lm,
                           uint64_t c0, uint64_t c1, AggGeom g, AggSrc x, CapCells cc, uint32_t* recs, uint32_t dbg)
{
	if (SYZ_SCAT3 == 1) {
		// k_scat3's tiles hold one call's records: calls a little longer than a
		// tile leave lanes idle there, so items whose tiles would be less than
		// SYZ_SCAT3_FILL % full go to k_agg_scatter_blk, decided per item on the
		// device (both kernels are launched; each skips the other's items)
		CapCells c2 = cc;
		c2.split = cc.sizes && cc.tiles;
		constexpr uint32_t kT = SYZ_SCAT3_T, kWpe = kT / 256;  // one workgroup per CU
		k_scat3<kT, SYZ_SCAT3_K, kWpe><<<(uint32_t)std::min<uint64_t>(nchunks, 2048), kT, 0, s>>>(
		    sigs, call_start, call_len, call_prio, lm, c0, c1, g, c2, recs, x);
		if (c2.split)
			scatter_blk<false>((uint32_t)std::min<uint64_t>(nchunks, 2048), s, pbits, sigs, call_start, call_len,
			                   call_prio, lm, c0, c1, g, x, c2, recs, dbg);
	} else {
		scatter_blk<false>((uint32_t)std::min<uint64_t>(nchunks, 2048), s, pbits, sigs, call_start, call_len,
		                   call_prio, lm, c0, c1, g, x, cc, recs, dbg);
	}
}

// Capped cells of a run: records per chunk -> cell capacity and chunk base.
// cap = m + sd * sqrt(m) + 64 rounded up to 64, m = the chunk's records / P
// (the cells of a uniformly hashed chunk hold m +- sqrt(m)); the host reserves
// 1.25 * records + nchunks * P * (sd^2 + 128), an upper bound of the sum
// (sd * sqrt(m) <= m / 4 + sd^2).
__global__ __launch_bounds__(256) void k_chunk_sizes(const uint32_t* __restrict__ call_len, uint64_t c0, uint64_t c1,
                                                     uint32_t cbits, uint64_t* sizes, uint32_t* tiles, uint32_t tile)
{
	const uint64_t ch = blockIdx.x, cbeg = c0 + (ch << cbits), cend = min<uint64_t>(c1, cbeg + (1ull << cbits));
	uint64_t s = 0, t = 0;
	for (uint64_t c = cbeg + threadIdx.x; c < cend; c += blockDim.x) {
		s += call_len[c];
		t += scat3_tiles(call_len[c], tile);
	}
	s = wave_sum_u64(s);
	t = wave_sum_u64(t);
	__shared__ uint64_t ws[4][2];
	if (lane_id() == 0) {
		ws[threadIdx.x >> 6][0] = s;
		ws[threadIdx.x >> 6][1] = t;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		sizes[ch] = ws[0][0] + ws[1][0] + ws[2][0] + ws[3][0];
		if (tiles)
			tiles[ch] = (uint32_t)min<uint64_t>(ws[0][1] + ws[1][1] + ws[2][1] + ws[3][1], 0xFFFFFFFFu);
	}
}

__device__ __forceinline__ void cell_plan(const uint64_t* __restrict__ sizes, uint64_t nchunks, uint32_t P, float sd,
                                          uint64_t* base, uint32_t* cap)
{
	__shared__ uint64_t wsum[16];
	uint64_t run = 0;
	for (uint64_t b0 = 0; b0 < nchunks; b0 += blockDim.x) {
		const uint64_t c = b0 + threadIdx.x;
		uint64_t v = 0;
		if (c < nchunks) {
			const float m = (float)sizes[c] / (float)P;
			const uint32_t k = sd < 0 ? 64u : ((uint32_t)(m + sd * sqrtf(m)) + 64 + 63) & ~63u;  // sd < 0: tests
			cap[c] = k;
			v = (uint64_t)k * P;
		}
		// exclusive block scan of v
		uint64_t xs = v;
		const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
		for (int o = 1; o < 64; o <<= 1) {
			const uint64_t y = __shfl_up(xs, o, 64);
			if (lane >= (uint32_t)o)
				xs += y;
		}
		if (lane == 63)
			wsum[w] = xs;
		__syncthreads();
		uint64_t pre = 0, tot = 0;
		for (uint32_t i = 0; i < 16; i++) {
			pre += i < w ? wsum[i] : 0;
			tot += wsum[i];
		}
		if (c < nchunks)
			base[c] = run + pre + xs - v;
		run += tot;
		__syncthreads();
	}
}

__global__ __launch_bounds__(1024) void k_cell_plan(const uint64_t* __restrict__ sizes, uint64_t nchunks, uint32_t P,
                                                    float sd, uint64_t* base, uint32_t* cap)
{
	cell_plan(sizes, nchunks, P, sd, base, cap);
}

// The one-sync triage run's first pass, one block per chunk of calls: the
// chunk's records (for k_cell_plan_fast), call ranges checked, whether a
// prio outside the run's levels (0..3 for a triage run) occurs, and call_new
// zeroed.  part[2 ch] = records,
// part[2 ch + 1] = bad ranges | other prio << 63.
__global__ __launch_bounds__(256) void k_fast_prep(const uint64_t* __restrict__ call_start,
                                                   const uint32_t* __restrict__ call_len,
                                                   const uint8_t* __restrict__ call_prio, uint64_t c0, uint64_t c1,
                                                   uint32_t ibits, uint64_t nrec_space, uint64_t* sizes,
                                                   uint64_t* part, uint8_t* call_new, LevelMap lm, uint32_t* tiles)
{
	const uint64_t ch = blockIdx.x, cbeg = c0 + (ch << ibits), cend = min<uint64_t>(c1, cbeg + (1ull << ibits));
	uint64_t tot = 0, bad = 0, other = 0, nt = 0;
	for (uint64_t c = cbeg + threadIdx.x; c < cend; c += blockDim.x) {
		const uint64_t st = call_start[c];
		const uint32_t ln = call_len[c];
		tot += ln;
		nt += scat3_tiles(ln, kScat3Tile);
		bad += st > nrec_space || ln > nrec_space - st || ln > kSerialMask;
		other |= lm.lvl[call_prio[c]] == 0xff;
		call_new[c] = 0;
	}
	tot = wave_sum_u64(tot);
	bad = wave_sum_u64(bad);
	other = wave_sum_u64(other);
	nt = wave_sum_u64(nt);
	__shared__ uint64_t ws[4][4];
	if (lane_id() == 0) {
		ws[threadIdx.x >> 6][0] = tot;
		ws[threadIdx.x >> 6][1] = bad;
		ws[threadIdx.x >> 6][2] = other;
		ws[threadIdx.x >> 6][3] = nt;
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		uint64_t t = 0, b = 0, o = 0, tl = 0;
		for (int w = 0; w < 4; w++) {
			t += ws[w][0];
			b += ws[w][1];
			o += ws[w][2];
			tl += ws[w][3];
		}
		sizes[ch] = t;
		if (tiles)
			tiles[ch] = (uint32_t)min<uint64_t>(tl, 0xFFFFFFFFu);
		part[2 * ch] = t;
		part[2 * ch + 1] = b | (o ? 1ull << 63 : 0);
	}
}

// k_cell_plan for the one-sync run: the counters are zeroed here (npairs
// preset), the assumptions checked from k_fast_prep's partials -- prios in
// 0..3 (else flag 2), valid ranges and at most `guess` records (else flag 4)
// -- and the run's void flag (ctr[kCntSpill]) set before anything reads it.
__global__ __launch_bounds__(1024) void k_cell_plan_fast(const uint64_t* __restrict__ sizes, uint64_t nchunks,
                                                         uint32_t P, float sd, uint64_t* base, uint32_t* cap,
                                                         const uint64_t* __restrict__ part, uint64_t guess,
                                                         uint64_t npairs0, unsigned long long* ctr)
{
	__shared__ unsigned long long s_tot, s_flag;
	if (threadIdx.x == 0) {
		s_tot = 0;
		s_flag = 0;
	}
	if (threadIdx.x < kNumCounters)
		ctr[threadIdx.x] = threadIdx.x == kCntAux2 ? npairs0 : 0;
	__syncthreads();
	uint64_t t = 0, f = 0;
	for (uint64_t c = threadIdx.x; c < nchunks; c += blockDim.x) {
		t += part[2 * c];
		f |= part[2 * c + 1];
	}
	t = wave_sum_u64(t);
	for (int o = 32; o > 0; o >>= 1)
		f |= __shfl_xor(f, o, 64);
	if (lane_id() == 0) {
		atomicAdd(&s_tot, (unsigned long long)t);
		atomicOr(&s_flag, (unsigned long long)f);
	}
	__syncthreads();
	if (threadIdx.x == 0) {
		ctr[kCntRecords] = s_tot;
		// 2: a prio outside the levels; 4: a bad call range or more records than
		// `guess` (the caller's exact path validates and sizes those)
		ctr[kCntSpill] = (s_flag >> 63 ? 2u : 0u) | ((s_flag & ~(1ull << 63)) || s_tot > guess ? 4u : 0u);
	}
	cell_plan(sizes, nchunks, P, sd, base, cap);
}

// ---------------------------------------------------------------- aggregation
// One workgroup per aggregation partition.  Waves take groups of gsz
// cells (chunks) from an LDS counter and walk each group as one virtual run.
// Cell (c, p): counted layout, the partition's records from rec_base[p] with
// cell offsets offsT[p][.]; capped layout (kCap), cap[c] records from
// base[c] + p * cap[c] of which cnt[p][c] are written.  Output: the
// partition's distinct elements and their level firsts at
// dist_*[p * kAggRegion ...], cnt[p] = how many, or kAggOverflow when they do
// not fit the LDS table.
// U records per lane per batch, D batches in flight ahead of the one absorbed.
// The LDS of one aggregation workgroup: keys (residuals) in 4-slot buckets,
// the level firsts, and per wave the records whose element was not in its
// home bucket (first sight, or a probe chain), gathered across batches and
// resolved 64 at a time with every lane busy: (residual, level << 24 | serial).
struct AggLds {
	KBucket kb[kAggBuckets];
	uint32_t fl[4][kAggSlots];
	uint2 q[kAggThreads / 64][64];
	uint32_t s_n, s_ovf, s_out, s_next;
};

// Where the records of one partition are (see k_agg).
struct AggCells {
	const uint32_t* recs;
	const uint64_t* rec_base;  // counted layout
	const uint32_t* offsT;
	const uint64_t* cap_base;  // capped layout
	const uint32_t* cap_len;
	const uint32_t* cap_cnt;
	uint64_t nchunks;
	uint32_t ilog, gsz;
	const uint32_t* spill;  // nonzero: a cell spilled, the run is redone (nothing aggregated); may be null
	unsigned long long* ctr;  // if set: distinct elements (kCntDistinct) and overflowed partitions (kCntAggOvf)
};

// Aggregate partition p into the LDS table (every thread of the workgroup;
// ends with a barrier).  Returns false when its distinct elements overflow
// the table (s_ovf).
template <uint32_t U, uint32_t D, bool kCap, bool kIdx32>
__device__ __forceinline__ bool agg_partition(AggLds& L, uint32_t p, const AggCells& x, const AggGeom& g)
{
	KBucket* kb = L.kb;
	auto& fl = L.fl;
	const uint32_t* __restrict__ recs = x.recs;
	const uint64_t* __restrict__ rec_base = x.rec_base;
	const uint32_t* __restrict__ offsT = x.offsT;
	const uint64_t* __restrict__ cap_base = x.cap_base;
	const uint32_t* __restrict__ cap_len = x.cap_len;
	const uint32_t* __restrict__ cap_cnt = x.cap_cnt;
	const uint64_t nchunks = x.nchunks;
	const uint32_t ilog = x.ilog, gsz = x.gsz;
	const uint32_t lane = lane_id();
	uint2* wq = L.q[threadIdx.x >> 6];
	uint32_t qn = 0;  // entries in this wave's queue (uniform)
	// resolve the queue: find-or-insert each element, then its level first
	auto flush_queue = [&]() {
		uint32_t ins = 0;
		if (!SYZ_AGG_OVF_EACH && lds_flag(&L.s_ovf)) {  // overflowed: the partition is redone, skip the probes
			qn = 0;
			return;
		}
		if (lane < qn) {
			const uint2 e = wq[lane];
			const uint32_t hb = __umulhi(e.x << g.pbits, kAggBuckets);
			const uint32_t slot = agg_find_insert(kb, e.x, hb, kb[hb], &L.s_ovf, ins);
			if (slot != kAggNoSlot)
				atomicMin(&fl[e.y >> 24][slot], e.y & 0xFFFFFFu);
		}
		// inserts counted per flush (overflow = more than kAggLimit distinct)
		const uint32_t n_ins = (uint32_t)wave_sum_u64(ins);
		if (n_ins && lane == 0 && atomicAdd(&L.s_n, n_ins) + n_ins > kAggLimit)
			lds_flag_set(&L.s_ovf);
		qn = 0;
		__builtin_amdgcn_wave_barrier();
	};
	const uint64_t ngroups = (nchunks + gsz - 1) / gsz;
	for (uint32_t i = threadIdx.x; i < kAggSlots; i += blockDim.x) {
		if (i < kAggSlots)
			reinterpret_cast<uint32_t*>(kb)[i] = kAggEmpty;
		fl[0][i] = fl[1][i] = fl[2][i] = fl[3][i] = kAggNone;
	}
	if (threadIdx.x == 0) {
		L.s_n = 0;
		L.s_ovf = 0;
		L.s_out = 0;
		L.s_next = 0;
	}
	__syncthreads();
	const uint32_t* ot = offsT + (uint64_t)p * (nchunks + 1);
	// no barrier inside: a wave leaves early once overflow is flagged
	for (;;) {
		uint32_t gi = 0;
		if (lane == 0)
			gi = atomicAdd(&L.s_next, 1u);
		gi = __builtin_amdgcn_readfirstlane(__shfl(gi, 0, 64));
		if (gi >= ngroups || lds_flag(&L.s_ovf))
			break;
		// the group's cells, one per lane 0..gsz-1: first record and
		// records.  The group is walked as one virtual run, cell after cell:
		// virtual offset v of cell i is record recs[v + delta_i].
		const uint64_t ch0 = (uint64_t)gi * gsz;
		uint64_t lbase = 0;
		uint32_t llen = 0;
		{
			const uint64_t c = ch0 + lane;
			if (lane < gsz && c < nchunks) {
				if (kCap) {
					lbase = cap_base[c] + (uint64_t)p * cap_len[c];
					llen = cap_cnt[(uint64_t)p * nchunks + c];
				} else {
					lbase = rec_base[p] + ot[c];
					llen = ot[c + 1] - ot[c];
				}
			}
		}
		uint32_t lvs = llen;  // inclusive scan over lanes 0..gsz-1, then exclusive
#pragma unroll
		for (uint32_t o = 1; o < 64; o <<= 1) {
			if (o < gsz) {
				const uint32_t y = __shfl_up(lvs, o, 64);
				if (lane >= o)
					lvs += y;
			}
		}
		const uint32_t n = __builtin_amdgcn_readlane(lvs, gsz - 1);
		if (n == 0)
			continue;
		lvs -= llen;
		const uint64_t ldelta = lbase - lvs;
		const uint32_t nl = n - 1;
		// Per batch [o0, o0 + U * 64): the cell of o0 (the last cell starting
		// at or before it: a non-empty one, as an empty cell shares its
		// successor's start) and the cells starting inside the batch.
		auto cells = [&](uint32_t o0, uint32_t& c0, uint64_t& inside) {
			c0 = (uint32_t)__popcll(__ballot(lane < gsz && lvs <= o0)) - 1;
			inside = __ballot(lane < gsz && lvs > o0 && lvs < o0 + U * 64);
		};
		auto delta_of = [&](uint32_t i) -> uint64_t {
			const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)ldelta, i);
			const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(ldelta >> 32), i);
			return (uint64_t)hi << 32 | lo;
		};
		// Records stream through registers one batch ahead of the LDS work,
		// ping-ponging between register buffers.  Loads are unconditional:
		// lanes past the group re-read its last record -- a second copy of a
		// record changes nothing (min is idempotent), so no lane needs a
		// validity test.
		auto fetch = [&](uint32_t (&buf)[U], uint32_t o0) {
			uint32_t c0;
			uint64_t inside;
			cells(min(o0, nl), c0, inside);  // a prefetch past the group reads its last record
			if constexpr (kIdx32) {
				// every cell lies below record 2^32 (host-checked): 32-bit record
				// indices, the cell deltas taken mod 2^32 (v + delta is the index)
				const uint32_t d0 = __builtin_amdgcn_readlane((uint32_t)ldelta, c0);
				uint32_t v[U], d[U];
#pragma unroll
				for (uint32_t u = 0; u < U; u++) {
					v[u] = min(o0 + u * 64 + lane, nl);
					d[u] = d0;
				}
				for (uint64_t m = inside; m; m &= m - 1) {
					const uint32_t j = __builtin_ctzll(m), vs = __builtin_amdgcn_readlane(lvs, j);
					const uint32_t dj = __builtin_amdgcn_readlane((uint32_t)ldelta, j);
#pragma unroll
					for (uint32_t u = 0; u < U; u++)
						d[u] = v[u] >= vs ? dj : d[u];
				}
#pragma unroll
				for (uint32_t u = 0; u < U; u++)
					buf[u] = __builtin_nontemporal_load(&recs[v[u] + d[u]]);
				return;
			}
			const uint64_t d0 = delta_of(c0);
			uint32_t v[U];
			uint64_t d[U];
#pragma unroll
			for (uint32_t u = 0; u < U; u++) {
				v[u] = min(o0 + u * 64 + lane, nl);
				d[u] = d0;
			}
			for (uint64_t m = inside; m; m &= m - 1) {
				const uint32_t j = __builtin_ctzll(m), vs = __builtin_amdgcn_readlane(lvs, j);
				const uint64_t dj = delta_of(j);
#pragma unroll
				for (uint32_t u = 0; u < U; u++)
					d[u] = v[u] >= vs ? dj : d[u];
			}
#pragma unroll
			for (uint32_t u = 0; u < U; u++)
				buf[u] = __builtin_nontemporal_load(&recs[v[u] + d[u]]);
		};
		auto absorb = [&](const uint32_t (&buf)[U], uint32_t o0) {
			uint32_t c0;
			uint64_t inside;
			cells(o0, c0, inside);
			uint32_t key[U], lv[U], k[U], hb[U], slot[U], c[U];
#pragma unroll
			for (uint32_t u = 0; u < U; u++)
				c[u] = (uint32_t)ch0 + c0;
			// a uniform loop over the (0-2 typically) cells starting inside the batch
			for (uint64_t m = inside; m; m &= m - 1) {
				const uint32_t vs = __builtin_amdgcn_readlane(lvs, __builtin_ctzll(m));
#pragma unroll
				for (uint32_t u = 0; u < U; u++)
					c[u] += min(o0 + u * 64 + lane, nl) >= vs;
			}
#pragma unroll
			for (uint32_t u = 0; u < U; u++) {
				const uint32_t r = buf[u];
				k[u] = ((c[u] >> ilog) << g.cbits()) | g.local(r);
				key[u] = g.resid(r);
				lv[u] = g.level(r);
				hb[u] = __umulhi(r & ~((1u << g.pbits) - 1), kAggBuckets);
			}
			// home buckets of all U records in flight together (ds_read_b128 / b64 each)
			KBucket B[U];
#pragma unroll
			for (uint32_t u = 0; u < U; u++)
				B[u] = kb[hb[u]];
			bool any_need = false;
#pragma unroll
			for (uint32_t u = 0; u < U; u++) {
				const uint32_t f = bucket_find(B[u], key[u]);
				slot[u] = f < kAggBW ? hb[u] * kAggBW + f : kAggNoSlot;
				any_need |= f >= kAggBW;
			}
			// first sight of an element, or a chain past its home bucket: to the
			// wave's queue (the record's own level first is taken there)
			if (__builtin_amdgcn_readfirstlane((uint32_t)(__ballot(any_need) != 0))) {
#pragma unroll
				for (uint32_t u = 0; u < U; u++) {
					const bool nd = slot[u] == kAggNoSlot;
					const uint64_t m = __ballot(nd);
					if (!m)
						continue;
					const uint32_t c = (uint32_t)__popcll(m);
					if (qn + c > 64)
						flush_queue();
					if (nd)
						wq[qn + lane_rank(m)] = make_uint2(key[u], (lv[u] << 24) | k[u]);
					qn += c;
				}
				__builtin_amdgcn_wave_barrier();
			}
#pragma unroll
			for (uint32_t u = 0; u < U; u++)
				if (slot[u] != kAggNoSlot)
					atomicMin(&fl[lv[u]][slot[u]], k[u]);
		};
		// a ring of D + 1 register buffers, rotated by full unrolling (static
		// indices: no register moves that would wait for the prefetch)
		uint32_t buf[D + 1][U];
#pragma unroll
		for (uint32_t d = 0; d < D; d++)
			fetch(buf[d], d * U * 64);
		bool more = true;
		for (uint32_t o0 = 0; more;) {
#pragma unroll
			for (uint32_t t = 0; t <= D; t++) {
				if (more) {
					fetch(buf[(t + D) % (D + 1)], o0 + D * U * 64);
					absorb(buf[t], o0);
					o0 += U * 64;
					// (the overflow flag is an LDS read, and its wait would also wait
					// for this batch's ds_min: checked once per group of cells
					// unless SYZ_AGG_OVF_EACH -- a full table ends every probe
					// chain at once anyway, agg_find_insert)
					more = o0 < n && (!SYZ_AGG_OVF_EACH || !lds_flag(&L.s_ovf));
				}
			}
		}
	}
	flush_queue();  // every record is absorbed before the barrier
	__syncthreads();
	return !L.s_ovf;
}

// ---------------------------------------------------------------- aggregation
// One workgroup per aggregation partition.  Waves take groups of gsz
// cells (chunks) from an LDS counter and walk each group as one virtual run.
// Cell (c, p): counted layout, the partition's records from rec_base[p] with
// cell offsets offsT[p][.]; capped layout (kCap), cap[c] records from
// base[c] + p * cap[c] of which cnt[p][c] are written.  Output: the
// partition's distinct elements and their level firsts at
// dist_*[p * kAggRegion ...], cnt[p] = how many, or kAggOverflow when they do
// not fit the LDS table.
// U records per lane per batch, D batches in flight ahead of the one absorbed.
template <uint32_t U, uint32_t D, bool kCap, bool kIdx32 = false>
__global__ __launch_bounds__(kAggThreads) void k_agg(AggCells x, AggGeom g, uint32_t* dist_e, uint4* dist_f,
                                                     uint32_t* cnt)
{
	__shared__ AggLds L;
	const uint32_t* keys = reinterpret_cast<const uint32_t*>(L.kb);
	const uint32_t P = 1u << g.pbits, lane = lane_id();
	if (x.spill && *x.spill)
		return;  // a cell spilled: the records are incomplete and the run is redone
	for (uint32_t p = blockIdx.x; p < P; p += gridDim.x) {
		if (!agg_partition<U, D, kCap, kIdx32>(L, p, x, g)) {
			if (threadIdx.x == 0) {
				cnt[p] = kAggOverflow;
				if (x.ctr)
					atomicAdd(&x.ctr[kCntAggOvf], 1ull);
			}
			__syncthreads();
			continue;
		}
		// compact the occupied slots, elements restored from (p, residual)
		const uint32_t hp = p << g.rbits();
		for (uint32_t i0 = 0; i0 < kAggSlots; i0 += kAggThreads) {
			const uint32_t i = i0 + threadIdx.x;
			const uint32_t key = i < kAggSlots ? keys[i] : kAggEmpty;
			const bool occ = key != kAggEmpty;
			const uint64_t m = __ballot(occ);
			uint32_t wb = 0;
			if (lane == 0 && m)
				wb = atomicAdd(&L.s_out, (uint32_t)__popcll(m));
			wb = __shfl(wb, 0, 64);
			if (occ) {
				const uint64_t o = (uint64_t)p * kAggRegion + wb + lane_rank(m);
				dist_e[o] = fmix32_inv(hp | key);
				dist_f[o] = make_uint4(L.fl[0][i], L.fl[1][i], L.fl[2][i], L.fl[3][i]);
			}
		}
		__syncthreads();
		if (threadIdx.x == 0) {
			cnt[p] = L.s_out;
			if (x.ctr && L.s_out)
				atomicAdd(&x.ctr[kCntDistinct], (unsigned long long)L.s_out);
		}
		__syncthreads();
	}
}

// k_agg over records [0, extent): 32-bit record indices when they fit (fewer
// vector instructions per record: 1.45 -> 1.40 ms at C2; the
// 64-bit kernel for larger runs, and under SYZSIG_DEBUG_AGG_IDX64 for tests)
template <bool kCap>
static void launch_agg(const syzsig_ctx* ctx, uint64_t extent, uint32_t P, hipStream_t s, const AggCells& xc,
                       const AggGeom& g, void* de, void* df, void* dc)
{
	if (extent <= (1ull << 32) && !(ctx->agg_dbg & SYZSIG_DEBUG_AGG_IDX64))
		k_agg<kAggU, kAggD, kCap, true><<<P, kAggThreads, 0, s>>>(xc, g, (uint32_t*)de, (uint4*)df, (uint32_t*)dc);
	else
		k_agg<kAggU, kAggD, kCap, false><<<P, kAggThreads, 0, s>>>(xc, g, (uint32_t*)de, (uint4*)df, (uint32_t*)dc);
}

// ---- fallback: partitions whose distinct elements overflow the LDS table are
// aggregated in one HBM hash table keyed by h (gkeys[C] + gfl[4][C + 1], C a
// power of two; slot C is h = 0xFFFFFFFF).  Partitions hold disjoint
// elements, so one table serves all of them.  One wave per (partition, group).
__global__ __launch_bounds__(256) void k_agg_global(const uint32_t* __restrict__ recs,
                                                    const uint64_t* __restrict__ rec_base,
                                                    const uint32_t* __restrict__ offsT, uint64_t nchunks, AggGeom g,
                                                    const uint32_t* __restrict__ ovl, uint32_t novl, uint32_t* gkeys,
                                                    uint32_t* gfl, uint64_t C, unsigned long long* err)
{
	const uint32_t lane = lane_id();
	const uint64_t ngroups = (nchunks + kAggGroup - 1) / kAggGroup, items = (uint64_t)novl * ngroups;
	const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	uint64_t bad = 0;
	for (uint64_t it = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); it < items; it += nwaves) {
		const uint32_t p = ovl[it / ngroups];
		const uint32_t* ot = offsT + (uint64_t)p * (nchunks + 1);
		const uint32_t* pr = recs + rec_base[p];
		CellGroup cg;
		cg.load(ot, nchunks, it % ngroups);
		for (uint32_t j = cg.bnd[0] + lane; j < cg.bnd[kAggGroup]; j += 64) {
			const uint32_t r = pr[j];
			const uint32_t k = cg.serial(j, r, g), l = g.level(r);
			const uint32_t h = (p << g.rbits()) | g.resid(r);
			uint64_t i = C;
			if (h != kAggEmpty) {
				i = fmix32(h ^ 0x632BE5ABu) & (C - 1);
				for (uint64_t step = 0;; step++) {
					uint32_t key = gkeys[i];
					if (key == kAggEmpty) {
						key = atomicCAS(&gkeys[i], kAggEmpty, h);
						if (key == kAggEmpty)
							break;
					}
					if (key == h)
						break;
					i = (i + 1) & (C - 1);
					if (step >= C) {
						bad++;
						i = ~0ull;
						break;
					}
				}
			}
			if (i != ~0ull)
				atomicMin(&gfl[(uint64_t)l * (C + 1) + i], k);
		}
	}
	block_count(err, bad);
}

__global__ __launch_bounds__(256) void k_agg_global_compact(const uint32_t* __restrict__ gkeys,
                                                            const uint32_t* __restrict__ gfl, uint64_t C,
                                                            uint32_t* dist_e, uint4* dist_f,
                                                            unsigned long long* out_cnt)
{
	const uint32_t lane = lane_id();
	for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 <= C; i0 += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t i = i0 + threadIdx.x;
		bool occ = false;
		uint32_t h = kAggEmpty;
		uint4 f = make_uint4(kAggNone, kAggNone, kAggNone, kAggNone);
		if (i <= C) {
			f = make_uint4(gfl[i], gfl[(C + 1) + i], gfl[2 * (C + 1) + i], gfl[3 * (C + 1) + i]);
			if (i < C) {
				h = gkeys[i];
				occ = h != kAggEmpty;
			} else {
				occ = (f.x & f.y & f.z & f.w) != kAggNone;
			}
		}
		const uint64_t m = __ballot(occ);
		unsigned long long wb = 0;
		if (lane == 0 && m)
			wb = atomicAdd(out_cnt, (unsigned long long)__popcll(m));
		wb = __shfl(wb, 0, 64);
		if (occ) {
			dist_e[wb + lane_rank(m)] = fmix32_inv(h);
			dist_f[wb + lane_rank(m)] = f;
		}
	}
}

// ---------------------------------------------------------------- finalize
// One workgroup per region r = dist_*[r * kAggRegion, + cnt[r]): a partition's
// distinct elements, whose maxSignal/newSignal home buckets share one slice of
// each table (the same top bits of h), so a block's probes stay in one slice.
// A block gathers its pairs in LDS and appends them with one global atomic
// per flush (a pair that finds the buffer full is appended directly).
// Each thread takes kFinIlp elements per pass and issues the loads of all their
// home buckets (maxSignal and newSignal) before walking any of them: the
// kernel is bound by the latency of these dependent random reads, not by
// bandwidth, so more of them in flight per wave is what makes it faster.
constexpr uint32_t kFinThreads = 256, kFinBuf = 4 * kFinThreads * 2, kFinIlp = 2;

__global__ __launch_bounds__(kFinThreads) void k_agg_finalize(const uint32_t* __restrict__ dist_e,
                                                              const uint4* __restrict__ dist_f,
                                                              const uint32_t* __restrict__ cnt, uint32_t nregions,
                                                              LevelMap lm, uint64_t c0, uint64_t* slots,
                                                              uint64_t bmask, uint64_t* ns_slots, uint64_t ns_bmask,
                                                              uint8_t* call_new, uint64_t* pairs,
                                                              unsigned long long* npairs, unsigned long long* ctr,
                                                              uint32_t dbg)
{
	__shared__ uint64_t buf[kFinBuf];
	__shared__ uint32_t s_n;
	__shared__ unsigned long long s_base;
	const uint64_t max_probe = max_probe_for(bmask);
	uint64_t inserted = 0, changed = 0, ns_ins = 0, ovf = 0;
	if (threadIdx.x == 0)
		s_n = 0;
	__syncthreads();
	auto flush = [&](uint32_t nb) {  // every thread; nb = s_n read after a barrier
		nb = min(nb, kFinBuf);
		if (threadIdx.x == 0)
			s_base = atomicAdd(npairs, (unsigned long long)nb);
		__syncthreads();
		for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x)
			pairs[s_base + t] = buf[t];
		__syncthreads();
		if (threadIdx.x == 0)
			s_n = 0;
		__syncthreads();
	};
	auto emit = [&](uint64_t v) {
		const uint32_t k = atomicAdd(&s_n, 1u);
		if (k < kFinBuf)
			buf[k] = v;
		else
			pairs[atomicAdd(npairs, 1ull)] = v;
	};
	for (uint32_t r = blockIdx.x; r < nregions; r += gridDim.x) {
		const uint32_t n = cnt[r] == kAggOverflow ? 0 : cnt[r];
		for (uint32_t i0 = 0; i0 < n; i0 += kFinIlp * kFinThreads) {
			uint32_t e[kFinIlp];
			uint4 f4[kFinIlp];
			int top[kFinIlp];
#pragma unroll
			for (uint32_t k = 0; k < kFinIlp; k++) {
				const uint32_t i = i0 + k * kFinThreads + threadIdx.x;
				const uint64_t o = (uint64_t)r * kAggRegion + min(i, n - 1);
				e[k] = dist_e[o];
				f4[k] = dist_f[o];
				top[k] = -1;
				const uint32_t f[4] = {f4[k].x, f4[k].y, f4[k].z, f4[k].w};
#pragma unroll
				for (int l = 0; l < 4; l++)
					if (i < n && l < (int)lm.n && f[l] != kAggNone)
						top[k] = l;
			}
			Bucket bm[kFinIlp], bn[kFinIlp];
#pragma unroll
			for (uint32_t k = 0; k < kFinIlp; k++) {
				if (top[k] >= 0) {
					bm[k] = load_bucket(slots + (home_bucket(e[k], bmask) << kBucketShift));
					if (ns_slots)
						bn[k] = load_bucket(ns_slots + (home_bucket(e[k], ns_bmask) << kBucketShift));
				}
			}
#pragma unroll
			for (uint32_t k = 0; k < kFinIlp; k++) {
				if (top[k] < 0)
					continue;
				const uint32_t f[4] = {f4[k].x, f4[k].y, f4[k].z, f4[k].w};
				// one probe sequence: insert M_final if absent, else read M0
				const int8_t P = lm.val[top[k]];
				const uint64_t word = make_slot(e[k], P);
				uint64_t old = 0;
				const int64_t idx = tbl_find_or_insert_from(slots, bmask, e[k], word, old, max_probe, bm[k]);
				if (idx < 0) {
					ovf++;
					continue;
				}
				const bool present = slot_live(old);  // (old == 0: inserted just now)
				const int p0 = present ? (int)slot_prio(old) : -1000;
				if ((int)P <= p0)
					continue;
				if (old != 0)
					slots[idx] = word;  // one entry per element: no other writer
				inserted += !present;   // fresh, or an "absent" marker going live
				changed++;
				const int rr = (dbg & 8) ? 0 : tbl_merge_from(ns_slots, ns_bmask, e[k], P, bn[k]);  // dbg: timing only
				ns_ins += rr == 1;
				ovf += rr < 0;
				// the staircase: first records of strictly rising level above M0[e]
				uint32_t mk = kAggNone;
#pragma unroll
				for (int l = 3; l >= 0; l--) {
					if (l > top[k] || f[l] == kAggNone)
						continue;
					if ((int)lm.val[l] <= p0)
						break;
					if (f[l] < mk) {
						mk = f[l];
						const uint64_t c = c0 + f[l];
						call_new[c] = 1;
						emit((c << 32) | e[k]);
					}
				}
			}
			__syncthreads();
			const uint32_t nb = s_n;
			if (nb > kFinBuf / 2)
				flush(nb);
		}
	}
	__syncthreads();
	const uint32_t nb = s_n;
	if (nb)
		flush(nb);
	block_count(&ctr[kCntInserted], inserted);
	block_count(&ctr[kCntChanged], changed);
	block_count(&ctr[kCntAux], ns_ins);
	block_count(&ctr[kCntOverflow], ovf);
}

// ---- the finalize without device-scope atomics (the fast path) ----
// Region r < P is partition r, and the home buckets of its elements form one
// contiguous slice of maxSignal (and of newSignal) whenever the table has at
// least P buckets: slice = buckets [r << shift, (r + 1) << shift).  Inside a
// slice the block is the only writer during this launch, so a found element is
// updated with a plain store, and an absent one takes the first empty slot of
// its probe sequence that no other element of the block claimed first -- the
// claims are LDS compare-and-swaps on the slot's index, not global atomics
// (measured: device-scope CAS runs at ~20 G/s chip-wide and bounded the
// atomic finalize).  Probe sequences stop at the slice end: such an element
// (or one whose claim table is full) is deferred, and so is a newSignal merge
// that leaves its slice: k_fin_deferred takes both lists after this launch,
// with the global-atomic code.
// Correct slot choice: slots only go empty -> key, so an element present at
// launch start sits before the first slot that was empty then; a slot seen
// occupied, or claimed by another element, is occupied at launch end, so the
// occupied-prefix invariant of every probe sequence still holds.
#ifndef SYZ_FX_BUF
#define SYZ_FX_BUF 2048
#endif
constexpr uint32_t kFxThreads = 512, kFxSet = 8192, kFxBuf = SYZ_FX_BUF, kFxProbe = 64;
enum : int { kFxTaken = 0, kFxClaimed = 1, kFxFull = 2 };

__device__ __forceinline__ int fx_claim(uint32_t* set, uint32_t tag, uint64_t rel)
{
	const uint32_t key = (tag << 31) | (uint32_t)(rel + 1);
	uint32_t h = fmix32(key) & (kFxSet - 1);
	for (uint32_t step = 0; step < kFxProbe; step++) {
		uint32_t v = set[h];
		if (v == 0) {
			v = atomicCAS(&set[h], 0u, key);
			if (v == 0)
				return kFxClaimed;
		}
		if (v == key)
			return kFxTaken;
		h = (h + 1) & (kFxSet - 1);
	}
	return kFxFull;
}

// Walk the probe sequence of e inside [b, bend) (B = the home bucket, loaded).
// Returns the slot index with old = its word (found), or with old = 0 (claimed
// for e); -1 = defer (slice end, or the claim table is full).
__device__ __forceinline__ int64_t fx_walk(const uint64_t* tab, uint64_t b, uint64_t bend, uint64_t slice0,
                                           uint32_t e, Bucket B, uint32_t* set, uint32_t tag, uint64_t& old)
{
	for (uint64_t b0 = b; b < bend; b++) {
		if (b != b0)
			B = load_bucket(tab + (b << kBucketShift));
#pragma unroll
		for (uint32_t i = 0; i < kBucketSlots; i++) {
			const uint64_t sw = B.s[i], idx = (b << kBucketShift) + i;
			if (sw != kSlotEmpty) {
				if (slot_key(sw) == e) {
					old = sw;
					return (int64_t)idx;
				}
				continue;
			}
			const int c = fx_claim(set, tag, idx - slice0);
			if (c == kFxClaimed) {
				old = 0;
				return (int64_t)idx;
			}
			if (c == kFxFull)
				return -1;
		}
	}
	return -1;
}

template <uint32_t kFxIlp>
__global__ __launch_bounds__(kFxThreads) void k_agg_finalize_x(
    const uint32_t* __restrict__ dist_e, const uint4* __restrict__ dist_f, const uint32_t* __restrict__ cnt,
    uint32_t nregions, LevelMap lm, uint64_t c0, uint64_t* slots, uint64_t bmask, uint32_t ms_shift,
    uint64_t* ns_slots, uint64_t ns_bmask, uint32_t ns_shift, uint8_t* call_new, uint64_t* pairs,
    unsigned long long* npairs, unsigned long long* ctr, uint32_t* def_e, uint4* def_f,
    unsigned long long* def_cnt, uint64_t* def_ns, unsigned long long* def_ns_cnt, uint32_t dbg,
    const uint32_t* spill, const unsigned long long* ovf_gate, uint32_t gate_max)
{
	__shared__ uint32_t claim[kFxSet];
	__shared__ uint64_t buf[kFxBuf];
	__shared__ uint32_t s_n;
	__shared__ unsigned long long s_base;
	if (spill && *spill)
		return;  // a cell spilled: nothing is committed, the run is redone
	if (ovf_gate && *ovf_gate > gate_max)
		return;  // the partitions were too few for the run's distinct elements: redone with more
	uint64_t inserted = 0, changed = 0, ns_ins = 0;
	auto flush = [&](uint32_t nb) {  // every thread; nb = s_n read after a barrier
		nb = min(nb, kFxBuf);
		if (threadIdx.x == 0)
			s_base = atomicAdd(npairs, (unsigned long long)nb);
		__syncthreads();
		for (uint32_t t = threadIdx.x; t < nb; t += blockDim.x)
			pairs[s_base + t] = buf[t];
		__syncthreads();
		if (threadIdx.x == 0)
			s_n = 0;
		__syncthreads();
	};
	auto emit = [&](uint64_t v) {
		const uint32_t k = atomicAdd(&s_n, 1u);
		if (k < kFxBuf)
			buf[k] = v;
		else
			pairs[atomicAdd(npairs, 1ull)] = v;
	};
	for (uint32_t r = blockIdx.x; r < nregions; r += gridDim.x) {
		for (uint32_t i = threadIdx.x; i < kFxSet; i += blockDim.x)
			claim[i] = 0;
		if (threadIdx.x == 0)
			s_n = 0;
		__syncthreads();
		const uint64_t ms0 = (uint64_t)r << ms_shift, ms1 = (uint64_t)(r + 1) << ms_shift;
		const uint64_t ns0 = (uint64_t)r << ns_shift, ns1 = (uint64_t)(r + 1) << ns_shift;
		const uint32_t n = cnt[r];
		if (n == kAggOverflow)
			continue;  // past the LDS table: aggregated in HBM and committed after this launch
		for (uint32_t i0 = 0; i0 < n; i0 += kFxIlp * kFxThreads) {
			uint32_t e[kFxIlp];
			uint4 f4[kFxIlp];
			int top[kFxIlp];
#pragma unroll
			for (uint32_t k = 0; k < kFxIlp; k++) {
				const uint32_t i = i0 + k * kFxThreads + threadIdx.x;
				const uint64_t o = (uint64_t)r * kAggRegion + min(i, n - 1);
				e[k] = dist_e[o];
				f4[k] = dist_f[o];
				top[k] = -1;
				const uint32_t f[4] = {f4[k].x, f4[k].y, f4[k].z, f4[k].w};
#pragma unroll
				for (int l = 0; l < 4; l++)
					if (i < n && l < (int)lm.n && f[l] != kAggNone)
						top[k] = l;
			}
			Bucket bm[kFxIlp], bn[kFxIlp];
#pragma unroll
			for (uint32_t k = 0; k < kFxIlp; k++) {
				if (top[k] >= 0) {
					bm[k] = load_bucket(slots + (home_bucket(e[k], bmask) << kBucketShift));
					bn[k] = load_bucket(ns_slots + (home_bucket(e[k], ns_bmask) << kBucketShift));
				}
			}
#pragma unroll
			for (uint32_t k = 0; k < kFxIlp; k++) {
				if (top[k] < 0)
					continue;
				const uint32_t f[4] = {f4[k].x, f4[k].y, f4[k].z, f4[k].w};
				const int8_t P = lm.val[top[k]];
				const uint64_t word = make_slot(e[k], P);
				uint64_t old = 0;
				// (dbg & 32, tests: defer every walk that leaves the home bucket)
				const uint64_t hm = home_bucket(e[k], bmask), hn = home_bucket(e[k], ns_bmask);
				const int64_t idx = fx_walk(slots, hm, dbg & 32 ? hm + 1 : ms1, ms0 << kBucketShift, e[k], bm[k],
				                            claim, 0, old);
				if (idx < 0) {  // the atomic path takes the whole element
					const uint64_t d = atomicAdd(def_cnt, 1ull);
					def_e[d] = e[k];
					def_f[d] = f4[k];
					continue;
				}
				const bool present = slot_live(old);
				const int p0 = present ? (int)slot_prio(old) : -1000;
				if ((int)P <= p0)
					continue;  // (a claimed slot always has P > p0)
				slots[idx] = word;    // the block's own slice: no other writer
				inserted += !present; // fresh, or an "absent" marker going live
				changed++;
				uint64_t nold = 0;
				const int64_t nidx = fx_walk(ns_slots, hn, dbg & 32 ? hn + 1 : ns1, ns0 << kBucketShift, e[k], bn[k],
				                             claim, 1, nold);
				if (nidx < 0) {
					def_ns[atomicAdd(def_ns_cnt, 1ull)] = ((uint64_t)e[k] << 32) | prio_biased(P);
				} else if (nold == 0 || nold < word) {
					ns_slots[nidx] = word;
					ns_ins += nold == 0;
				}
				// the staircase: first records of strictly rising level above M0[e]
				uint32_t mk = kAggNone;
#pragma unroll
				for (int l = 3; l >= 0; l--) {
					if (l > top[k] || f[l] == kAggNone)
						continue;
					if ((int)lm.val[l] <= p0)
						break;
					if (f[l] < mk) {
						mk = f[l];
						const uint64_t c = c0 + f[l];
						call_new[c] = 1;
						emit((c << 32) | e[k]);
					}
				}
			}
			__syncthreads();
			const uint32_t nb = s_n;
			if (nb > kFxBuf / 2)
				flush(nb);
		}
		__syncthreads();
		const uint32_t nb = s_n;
		if (nb)
			flush(nb);
	}
	block_count(&ctr[kCntInserted], inserted);
	block_count(&ctr[kCntChanged], changed);
	block_count(&ctr[kCntAux], ns_ins);
}

// Deferred elements of k_agg_finalize_x, with the global-atomic table code
// (launched after it: the slices are free for everyone again).
__device__ void fin_deferred(const uint32_t* __restrict__ def_e, const uint4* __restrict__ def_f,
                                                      const unsigned long long* __restrict__ def_cnt, LevelMap lm,
                                                      uint64_t c0, uint64_t* slots, uint64_t bmask, uint64_t* ns_slots,
                                                      uint64_t ns_bmask, uint8_t* call_new, uint64_t* pairs,
                                                      unsigned long long* npairs, unsigned long long* ctr,
                                                      uint32_t nblocks, uint32_t block)
{
	const uint64_t n = *def_cnt, max_probe = max_probe_for(bmask);
	uint64_t inserted = 0, changed = 0, ns_ins = 0, ovf = 0;
	for (uint64_t i = block * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)nblocks * blockDim.x) {
		const uint32_t e = def_e[i];
		const uint4 f4 = def_f[i];
		const uint32_t f[4] = {f4.x, f4.y, f4.z, f4.w};
		int top = -1;
#pragma unroll
		for (int l = 0; l < 4; l++)
			if (l < (int)lm.n && f[l] != kAggNone)
				top = l;
		if (top < 0)
			continue;
		const int8_t P = lm.val[top];
		const uint64_t word = make_slot(e, P);
		uint64_t old = 0;
		const int64_t idx = tbl_find_or_insert(slots, bmask, e, word, old, max_probe);
		if (idx < 0) {
			ovf++;
			continue;
		}
		const bool present = slot_live(old);
		const int p0 = present ? (int)slot_prio(old) : -1000;
		if ((int)P <= p0)
			continue;
		if (old != 0)
			slots[idx] = word;
		inserted += !present;
		changed++;
		const int rr = tbl_merge(ns_slots, ns_bmask, e, P);
		ns_ins += rr == 1;
		ovf += rr < 0;
		uint32_t mk = kAggNone;
#pragma unroll
		for (int l = 3; l >= 0; l--) {
			if (l > top || f[l] == kAggNone)
				continue;
			if ((int)lm.val[l] <= p0)
				break;
			if (f[l] < mk) {
				mk = f[l];
				const uint64_t c = c0 + f[l];
				call_new[c] = 1;
				pairs[atomicAdd(npairs, 1ull)] = (c << 32) | e;
			}
		}
	}
	block_count(&ctr[kCntInserted], inserted);
	block_count(&ctr[kCntChanged], changed);
	block_count(&ctr[kCntAux], ns_ins);
	block_count(&ctr[kCntOverflow], ovf);
}

// Deferred newSignal merges of k_agg_finalize_x: (elem << 32 | prio ^ 0x80).
__device__ void ns_deferred(const uint64_t* __restrict__ def_ns, const unsigned long long* __restrict__ def_ns_cnt,
                            uint64_t* ns_slots, uint64_t ns_bmask, unsigned long long* ctr, uint32_t nblocks,
                            uint32_t block)
{
	const uint64_t n = *def_ns_cnt;
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = block * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)nblocks * blockDim.x) {
		const uint64_t v = def_ns[i];
		const int r = tbl_merge(ns_slots, ns_bmask, (uint32_t)(v >> 32), (int8_t)((uint8_t)v ^ 0x80u));
		ins += r == 1;
		ovf += r < 0;
	}
	block_count(&ctr[kCntAux], ins);
	block_count(&ctr[kCntOverflow], ovf);
}

// Both deferred lists in one launch: the first kDeferBlocks blocks take the
// elements, the rest the newSignal merges (both sides only ever max-merge
// newSignal with atomics, so they commute).
constexpr uint32_t kDeferBlocks = 64;
__global__ __launch_bounds__(256) void k_fin_deferred(const uint32_t* __restrict__ def_e, const uint4* __restrict__ def_f,
                                                      const unsigned long long* __restrict__ def_cnt, LevelMap lm,
                                                      uint64_t c0, uint64_t* slots, uint64_t bmask, uint64_t* ns_slots,
                                                      uint64_t ns_bmask, uint8_t* call_new, uint64_t* pairs,
                                                      unsigned long long* npairs, unsigned long long* ctr,
                                                      const uint64_t* __restrict__ def_ns,
                                                      const unsigned long long* __restrict__ def_ns_cnt)
{
	if (blockIdx.x < kDeferBlocks)
		fin_deferred(def_e, def_f, def_cnt, lm, c0, slots, bmask, ns_slots, ns_bmask, call_new, pairs, npairs, ctr,
		             kDeferBlocks, blockIdx.x);
	else
		ns_deferred(def_ns, def_ns_cnt, ns_slots, ns_bmask, ctr, gridDim.x - kDeferBlocks, blockIdx.x - kDeferBlocks);
}

// ---------------------------------------------------------------- one-sync run
// The arguments of the finalize of a one-sync triage run (agg_triage_fused).
// (Round 3 measured aggregation and finalize in one launch -- the distinct
// elements kept in registers, the freed LDS as claim set -- at 1.18 ms against
// 0.64 + 0.27 for the two launches at C2, and removed it: one 1024-thread
// workgroup per CU held the LDS through its random probes.)
struct FinArgs {
	LevelMap lm;
	uint64_t c0;
	uint64_t* slots;
	uint64_t bmask;
	uint32_t ms_shift;
	uint64_t* ns_slots;
	uint64_t ns_bmask;
	uint32_t ns_shift;
	uint8_t* call_new;
	uint64_t* pairs;
	unsigned long long* npairs;
	unsigned long long* ctr;
	uint32_t* def_e;
	uint4* def_f;
	unsigned long long* def_cnt;
	uint64_t* def_ns;
	unsigned long long* def_ns_cnt;
	const uint32_t* spill;
	uint32_t dbg;
};

// Fallback of the one-sync run: the records of the partitions that overflowed
// the LDS table, aggregated in one HBM table keyed by h (as k_agg_global) from
// their capped cells.  One wave per (partition, chunk).
__global__ __launch_bounds__(256) void k_agg_global_cap(const uint32_t* __restrict__ recs,
                                                        const uint64_t* __restrict__ cap_base,
                                                        const uint32_t* __restrict__ cap_len,
                                                        const uint32_t* __restrict__ cap_cnt, uint64_t nchunks,
                                                        AggGeom g, const uint32_t* __restrict__ ovl, uint32_t novl,
                                                        uint32_t* gkeys, uint32_t* gfl, uint64_t C,
                                                        unsigned long long* err)
{
	const uint32_t lane = lane_id();
	const uint64_t items = (uint64_t)novl * nchunks, nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	uint64_t bad = 0;
	for (uint64_t it = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); it < items; it += nwaves) {
		const uint32_t p = ovl[it / nchunks];
		const uint64_t c = it % nchunks;
		const uint32_t* pr = recs + cap_base[c] + (uint64_t)p * cap_len[c];
		const uint32_t n = cap_cnt[(uint64_t)p * nchunks + c];
		for (uint32_t j = lane; j < n; j += 64) {
			const uint32_t r = pr[j];
			const uint32_t k = ((uint32_t)c << g.cbits()) | g.local(r), l = g.level(r);
			const uint32_t h = (p << g.rbits()) | g.resid(r);
			uint64_t i = C;
			if (h != kAggEmpty) {
				i = fmix32(h ^ 0x632BE5ABu) & (C - 1);
				for (uint64_t step = 0;; step++) {
					uint32_t key = gkeys[i];
					if (key == kAggEmpty) {
						key = atomicCAS(&gkeys[i], kAggEmpty, h);
						if (key == kAggEmpty)
							break;
					}
					if (key == h)
						break;
					i = (i + 1) & (C - 1);
					if (step >= C) {
						bad++;
						i = ~0ull;
						break;
					}
				}
			}
			if (i != ~0ull)
				atomicMin(&gfl[(uint64_t)l * (C + 1) + i], k);
		}
	}
	block_count(err, bad);
}

// ---------------------------------------------------------------- new bits
__device__ __forceinline__ uint64_t pair_hash(uint64_t k)
{
	k ^= k >> 33;
	k *= 0xff51afd7ed558ccdull;
	k ^= k >> 33;
	k *= 0xc4ceb9fe1a85ec53ull;
	k ^= k >> 33;
	return k;
}

// Insert pairs into a set of capacity C (power of two, empty = ~0).
// Duplicates are dropped; `uniq` counts distinct ones.
__global__ __launch_bounds__(256) void k_pairs_set(const uint64_t* __restrict__ pairs, uint64_t n, uint64_t* set,
                                                   uint64_t C, unsigned long long* uniq)
{
	uint64_t u = 0;
	for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t v = pairs[t];
		uint64_t i = pair_hash(v) & (C - 1);
		for (uint64_t step = 0; step < C; step++) {
			uint64_t k = set[i];
			if (k == ~0ull) {
				k = atomicCAS((unsigned long long*)&set[i], ~0ull, (unsigned long long)v);
				if (k == ~0ull) {
					u++;
					break;
				}
			}
			if (k == v)
				break;
			i = (i + 1) & (C - 1);
		}
	}
	block_count(uniq, u);
}

__device__ __forceinline__ bool pairs_has(const uint64_t* set, uint64_t C, uint64_t v)
{
	uint64_t i = pair_hash(v) & (C - 1);
	for (uint64_t step = 0; step < C; step++) {
		const uint64_t k = set[i];
		if (k == v)
			return true;
		if (k == ~0ull)
			return false;
		i = (i + 1) & (C - 1);
	}
	return false;
}

// one wave per call: bit r = (call, sigs[r]) is a new pair
__global__ __launch_bounds__(256) void k_pairs_mark(const uint32_t* __restrict__ sigs,
                                                    const uint64_t* __restrict__ call_start,
                                                    const uint32_t* __restrict__ call_len, uint64_t c0, uint64_t c1,
                                                    const uint8_t* __restrict__ call_new, const uint64_t* set,
                                                    uint64_t C, uint32_t* new_bits)
{
	const uint32_t lane = lane_id();
	const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	for (uint64_t c = c0 + blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); c < c1; c += nwaves) {
		if (!call_new[c])
			continue;
		const uint64_t st = call_start[c];
		const uint32_t len = call_len[c];
		for (uint32_t j = lane; j < len; j += 64)
			if (pairs_has(set, C, (c << 32) | sigs[st + j]))
				atomicOr(&new_bits[(st + j) >> 5], 1u << ((st + j) & 31));
	}
}

// dedupped pairs from the set (compaction)
__global__ __launch_bounds__(256) void k_pairs_compact(const uint64_t* __restrict__ set, uint64_t C, uint64_t* out,
                                                       unsigned long long* n)
{
	const uint32_t lane = lane_id();
	for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < C; i0 += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t i = i0 + threadIdx.x;
		const uint64_t v = i < C ? set[i] : ~0ull;
		const bool occ = v != ~0ull;
		const uint64_t m = __ballot(occ);
		unsigned long long wb = 0;
		if (lane == 0 && m)
			wb = atomicAdd(n, (unsigned long long)__popcll(m));
		wb = __shfl(wb, 0, 64);
		if (occ)
			out[wb + lane_rank(m)] = v;
	}
}

// pairs from per-record bits of calls [c0, c1) (per-call path); may repeat a pair
__global__ __launch_bounds__(256) void k_bits_to_pairs(const uint32_t* __restrict__ sigs,
                                                       const uint64_t* __restrict__ call_start,
                                                       const uint32_t* __restrict__ call_len, uint64_t c0, uint64_t c1,
                                                       const uint8_t* __restrict__ call_new,
                                                       const uint32_t* __restrict__ bits, uint64_t* pairs,
                                                       unsigned long long* n)
{
	const uint32_t lane = lane_id();
	const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	for (uint64_t c = c0 + blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); c < c1; c += nwaves) {
		if (!call_new[c])
			continue;
		const uint64_t st = call_start[c];
		const uint32_t len = call_len[c];
		for (uint32_t j0 = 0; j0 < len; j0 += 64) {
			const uint32_t j = j0 + lane;
			const bool on = j < len && ((bits[(st + j) >> 5] >> ((st + j) & 31)) & 1);
			const uint64_t m = __ballot(on);
			unsigned long long wb = 0;
			if (lane == 0 && m)
				wb = atomicAdd(n, (unsigned long long)__popcll(m));
			wb = __shfl(wb, 0, 64);
			if (on)
				pairs[wb + lane_rank(m)] = (c << 32) | sigs[st + j];
		}
	}
}

// ---------------------------------------------------------------- host
static uint64_t pow2_at_least(uint64_t x)
{
	uint64_t p = 1;
	while (p < x)
		p <<= 1;
	return p;
}

static AggGeom agg_geom_for(syzsig_ctx* ctx, uint64_t nrec, double distinct_hint, double load = kAggTargetLoad)
{
	AggGeom g;
	if (ctx->agg_parts) {
		g.pbits = 31 - __builtin_clz(ctx->agg_parts);  // validated power of two in [8, 2048]
		return g;
	}
	// expected distinct elements: the caller's hint, else the ratio seen on the
	// previous large batch (1/32 before the first); big runs keep >= 256
	// partitions (one per CU)
	const double ratio = ctx->agg_distinct_ratio > 0 ? ctx->agg_distinct_ratio : 1.0 / 32;
	const double d = distinct_hint > 0 ? distinct_hint : ratio * (double)nrec;
	uint32_t pb = nrec >= (1ull << 24) ? 8 : kAggMinBits;
	while (pb < kAggMaxBits && d > load * kAggSlots * (double)(1u << pb))
		pb++;
	g.pbits = pb;
	return g;
}

// k_agg's cells per wave work item: ~64 items per partition (4 per wave),
// at least kAggGroup and at most one cell per lane
static uint32_t agg_group_size(uint64_t ncells)
{
	uint32_t gz = kAggGroup;
	while (gz < 64 && ncells / gz > 64)
		gz <<= 1;
	return gz;
}

// The count-free attempt: scatter into capped cells (no count pass, no scan),
// then aggregate.  Cells belong to work items of 2^g.ibits calls (chunks for a
// triage run, smaller items for Minimize: xp != nullptr).  *done = false when
// the run must be redone with counted cells: a cell overflowed (the slack is
// doubled for the next run of the kind, and capped cells are given up past
// kCapSdMax), or a partition overflowed the LDS table (its HBM fallback reads
// counted cells).
constexpr float kCapSdMax = 24.0f;
static int agg_capped(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t c0, uint64_t c1, const LevelMap& lm,
                      uint64_t run_recs, const AggGeom& g, const AggSrc* xp, syzsig_batch_stats* st, AggOut* out,
                      bool* done)
{
	*done = false;
	const AggGeom gs = g;
	const uint32_t S = 1u << gs.pbits, P = S;
	const uint64_t nchunks = (c1 - c0 + (1ull << gs.ibits) - 1) >> gs.ibits;  // work items
	const bool tight = ctx->agg_dbg & SYZSIG_DEBUG_CAP_SPILL;
	float& slack = xp ? ctx->cap_sd_entry : ctx->cap_sd;
	const float sd = tight ? 0.0f : slack;
	// upper bound of sum_c S * cap[c] (k_cell_plan): 1.25 records + per cell sd^2 + 128
	const uint64_t bound = (run_recs + run_recs / 4 + nchunks * S * (uint64_t)(sd * sd + 128.0f) + 127) & ~63ull;  // (the dummy lines after it: 16-B stores)
	void *recs, *cm, *de, *df, *dc;
	SYZ_TRY(ws_get(ctx, 16, (bound + kDummyLines * kBlk) * 4, &recs));
	SYZ_TRY(ws_get(ctx, 17, nchunks * 24 + (uint64_t)S * nchunks * 4 + 256, &cm));
	uint64_t* sizes = (uint64_t*)cm;
	uint64_t* cbase = sizes + nchunks;
	uint32_t* ccap = (uint32_t*)(cbase + nchunks);
	uint32_t* ccnt = ccap + nchunks;
	uint32_t* ovf = ccnt + (uint64_t)S * nchunks;
	uint32_t* tiles = ovf + 1;
	SYZ_TRY(ws_get(ctx, 19, (uint64_t)P * kAggRegion * 4 + 64, &de));
	SYZ_TRY(ws_get(ctx, 20, (uint64_t)P * kAggRegion * 16 + 64, &df));
	SYZ_TRY(ws_get(ctx, 21, (uint64_t)(P + 1) * 4 + 64, &dc));
	const hipStream_t s = ctx->stream;
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[0], s));
	SYZ_HIP(hipMemsetAsync(ovf, 0, 4, s));
	const uint32_t tile = xp ? kScat3TileEntry : kScat3Tile;
	k_chunk_sizes<<<(uint32_t)nchunks, 256, 0, s>>>(b->call_len, c0, c1, gs.ibits, sizes, tiles, tile);
	k_cell_plan<<<1, 1024, 0, s>>>(sizes, nchunks, S, tight ? -1.0f : sd, cbase, ccap);
	const CapCells cc{cbase, ccap, ccnt, ovf, nchunks, (uint32_t*)recs + bound, sizes, tiles, false, tile};
	const int pg = (int)std::min<uint64_t>(nchunks, 2048);
	if (xp && SYZ_SCAT3_ENTRY && xp->nshards == 1) {
		// Minimize: the contexts in rank order (Len desc), so the heavy first
		// work items fill k_scat3's one-call tiles; the split as for triage
		CapCells c2 = cc;
		c2.split = true;
		if (gs.pbits < kAggMaxBits)
			k_scat3<kAggThreads, SYZ_SCAT3_KE, 4, true, 32><<<pg, kAggThreads, 0, s>>>(
			    b->sigs, b->call_start, b->call_len, b->call_prio, lm, c0, c1, gs, c2, (uint32_t*)recs, *xp);
		else
			k_scat3<kAggThreads, SYZ_SCAT3_KE, 4, true, 16><<<pg, kAggThreads, 0, s>>>(
			    b->sigs, b->call_start, b->call_len, b->call_prio, lm, c0, c1, gs, c2, (uint32_t*)recs, *xp);
		scatter_blk<true>(pg, s, gs.pbits, b->sigs, b->call_start, b->call_len, b->call_prio, lm, c0, c1, gs, *xp, c2,
		                  (uint32_t*)recs, ctx->agg_dbg >> 10);
	} else if (xp)
		scatter_blk<true>(pg, s, gs.pbits, b->sigs, b->call_start, b->call_len, b->call_prio, lm, c0,
		                                                   c1, gs, *xp, cc, (uint32_t*)recs, ctx->agg_dbg >> 10);
	else
		scatter_triage(nchunks_of(c1 - c0, gs.ibits), s, gs.pbits, b->sigs, b->call_start, b->call_len, b->call_prio,
		               lm, c0, c1, gs, AggSrc{nullptr, 1, 0, 0}, cc, (uint32_t*)recs, ctx->agg_dbg >> 10);
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[1], s));
	const AggCells xc{(const uint32_t*)recs, nullptr, nullptr, cbase, ccap, ccnt, nchunks, gs.items_per_chunk_log2(),
	                  agg_group_size(nchunks)};
	launch_agg<true>(ctx, bound, P, s, xc, gs, de, df, dc);
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[2], s));
	uint32_t* hov = (uint32_t*)(ctx->h_pin + kPinCounts);
	uint32_t* hcp = hov + 16;
	SYZ_HIP(hipMemcpyAsync(hcp, dc, P * 4, hipMemcpyDeviceToHost, s));
	SYZ_HIP(hipMemcpyAsync(hov, ovf, 4, hipMemcpyDeviceToHost, s));
	SYZ_HIP(hipStreamSynchronize(s));
	if (ctx->timing) {
		float t0 = 0, t1 = 0;
		SYZ_HIP(hipEventElapsedTime(&t0, ctx->ev[0], ctx->ev[1]));
		SYZ_HIP(hipEventElapsedTime(&t1, ctx->ev[1], ctx->ev[2]));
		st->part_ms += t0;
		st->probe_ms += t1;
	}
	if (*hov) {
		st->retries++;
		if (!tight)
			slack = slack * 2 > kCapSdMax ? 0.0f : slack * 2;
		return SYZSIG_OK;
	}
	uint64_t D = 0;
	for (uint32_t p = 0; p < P; p++) {
		if (hcp[p] == kAggOverflow) {
			st->retries++;
			return SYZSIG_OK;
		}
		D += hcp[p];
	}
	st->distinct += D;
	st->parts = P;
	st->survivors += D;
	if (!xp)
		ctx->agg_distinct_ratio = run_recs ? (double)D / (double)run_recs : 0;
	out->dist_e = (const uint32_t*)de;
	out->dist_f = (const uint4*)df;
	out->cnt = (const uint32_t*)dc;
	out->nregions = P;
	out->parts = P;
	out->D = D;
	*done = true;
	return SYZSIG_OK;
}

// Count, scatter and aggregate (plus the HBM fallback) one run of calls
// [c0, c1) with level map lm: every distinct element of the run with its level
// firsts (run serials), in regions of kAggRegion entries.  A triage run tries
// capped cells first (agg_capped), counted cells are the exact path.
int agg_aggregate(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t c0, uint64_t c1, const LevelMap& lm,
                  uint64_t run_recs, syzsig_batch_stats* st, AggOut* out, const AggSrc* xp)
{
	const AggSrc x = xp ? *xp : AggSrc{nullptr, 1, 0, 0};
	const bool entry = xp != nullptr;
	// Minimize: fuller LDS tables, so half the partitions and whole 128-B
	// scatter blocks (C3: 2.70-2.78 -> 2.65 ms; a triage run's finalize and
	// k_agg lose more than its scatter gains)
	AggGeom g = agg_geom_for(ctx, run_recs, x.distinct_hint, entry ? kAggTargetLoadEntry : kAggTargetLoad);
	const uint32_t P = 1u << g.pbits;
	const uint64_t nchunks = (c1 - c0 + (1ull << g.cbits()) - 1) >> g.cbits();
	// Work items of the count/scatter: whole chunks for a batch (its calls are
	// alike), smaller ones for Minimize, whose calls (contexts in Len-desc
	// order) make the first chunks far heavier than the last: >= ~2048 items.
	g.ibits = g.cbits();
	if (entry)
		while (g.ibits > 0 && ((c1 - c0) >> g.ibits) < SYZ_MIN_ITEMS)
			g.ibits--;
	const bool counted_once = ctx->agg_counted_once;
	ctx->agg_counted_once = false;
	if (((entry ? ctx->cap_sd_entry : ctx->cap_sd) > 0 || (ctx->agg_dbg & SYZSIG_DEBUG_CAP_SPILL)) &&
	    !(ctx->agg_dbg & SYZSIG_DEBUG_EXACT_CELLS) && !counted_once) {
		bool done = false;
		SYZ_TRY(agg_capped(ctx, b, c0, c1, lm, run_recs, g, xp, st, out, &done));
		if (done)
			return SYZSIG_OK;
	}
	const uint32_t ilog = g.items_per_chunk_log2();
	const uint64_t nitems = (c1 - c0 + (1ull << g.ibits) - 1) >> g.ibits;
	void *recs, *cm, *pm, *de, *df, *dc;
	SYZ_TRY(ws_get(ctx, 16, run_recs * 4 + 64, &recs));
	SYZ_TRY(ws_get(ctx, 17, (2 * nitems * P + (uint64_t)P * (nchunks + 1)) * 4 + 64, &cm));
	SYZ_TRY(ws_get(ctx, 18, (kAggMaxParts + 1) * 8 * 2, &pm));
	uint32_t* counts = (uint32_t*)cm;
	uint32_t* offs = counts + nitems * P;
	uint32_t* offsT = offs + nitems * P;
	uint64_t* totals = (uint64_t*)pm;
	uint64_t* rec_base = totals + kAggMaxParts + 1;
	const hipStream_t s = ctx->stream;
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[0], s));
	const int pg = (int)std::min<uint64_t>(nitems, 2048);
	if (x.nshards > 1)
		k_agg_count<true><<<pg, kAggThreads, 0, s>>>(b->sigs, b->call_start, b->call_len, c0, c1, g, x, counts);
	else
		k_agg_count<false><<<pg, kAggThreads, 0, s>>>(b->sigs, b->call_start, b->call_len, c0, c1, g, x, counts);
	k_agg_scan_chunks<<<P, 1024, 0, s>>>(counts, nitems, ilog, P, offs, offsT, totals);
	k_agg_scan_totals<<<1, 1024, 0, s>>>(totals, P, rec_base);
	if (entry)
		k_agg_scatter<true><<<pg, kAggThreads, 0, s>>>(b->sigs, b->call_start, b->call_len, b->call_prio, lm, c0, c1,
		                                               g, x, offs, rec_base, (uint32_t*)recs);
	else
		k_agg_scatter<false><<<pg, kAggThreads, 0, s>>>(b->sigs, b->call_start, b->call_len, b->call_prio, lm, c0, c1,
		                                                g, x, offs, rec_base, (uint32_t*)recs);
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[1], s));
	// aggregation
	SYZ_TRY(ws_get(ctx, 19, (uint64_t)P * kAggRegion * 4 + 64, &de));
	SYZ_TRY(ws_get(ctx, 20, (uint64_t)P * kAggRegion * 16 + 64, &df));
	SYZ_TRY(ws_get(ctx, 21, (uint64_t)(P + 1) * 4 + 64, &dc));
	const AggCells xc{(const uint32_t*)recs, rec_base, offsT, nullptr, nullptr, nullptr, nchunks, 0,
	                  agg_group_size(nchunks)};
	launch_agg<false>(ctx, run_recs, P, s, xc, g, de, df, dc);
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[2], s));
	static_assert(kPinCounts + kAggMaxParts * 4 + (kAggMaxParts + 1) * 8 <= kPinBytes, "pinned staging");
	uint64_t* hbp = (uint64_t*)(ctx->h_pin + kPinCounts);
	uint32_t* hcp = (uint32_t*)(hbp + kAggMaxParts + 1);
	SYZ_HIP(hipMemcpyAsync(hcp, dc, P * 4, hipMemcpyDeviceToHost, s));
	SYZ_HIP(hipMemcpyAsync(hbp, rec_base, (P + 1) * 8, hipMemcpyDeviceToHost, s));
	SYZ_HIP(hipStreamSynchronize(s));
	const std::vector<uint32_t> hc(hcp, hcp + P);
	const std::vector<uint64_t> hb(hbp, hbp + P + 1);
	if (ctx->timing) {
		float t0 = 0, t1 = 0;
		SYZ_HIP(hipEventElapsedTime(&t0, ctx->ev[0], ctx->ev[1]));
		SYZ_HIP(hipEventElapsedTime(&t1, ctx->ev[1], ctx->ev[2]));
		st->part_ms += t0;
		st->probe_ms += t1;
	}
	uint64_t D = 0, ovrec = 0;
	std::vector<uint32_t> ovl;
	for (uint32_t p = 0; p < P; p++) {
		if (hc[p] == kAggOverflow) {
			ovl.push_back(p);
			ovrec += hb[p + 1] - hb[p];
		} else {
			D += hc[p];
		}
	}
	uint32_t nregions = P;
	void* dist_e = de;
	void* dist_f = df;
	if (!ovl.empty()) {
		// fallback: HBM aggregation table for the overflowed partitions; their
		// distinct list is appended as extra regions after the P LDS regions
		const uint64_t C = pow2_at_least(std::max<uint64_t>(2 * ovrec, 1024));
		const uint64_t extra_regions = (ovrec + kAggRegion - 1) / kAggRegion + 1;
		void *gk, *gf, *ol;
		SYZ_TRY(ws_get(ctx, 23, C * 4 + (C + 1) * 16 + 64, &gk));
		gf = (char*)gk + C * 4;
		SYZ_TRY(ws_get(ctx, 22, ovl.size() * 4 + 64, &ol));
		// distinct lists must be contiguous with the regions: grow 19/20 keeping the LDS part
		const uint64_t tot_e = ((uint64_t)P + extra_regions) * kAggRegion;
		void *de2, *df2;
		SYZ_TRY(ws_get(ctx, 30, tot_e * 4 + 64, &de2));
		SYZ_TRY(ws_get(ctx, 31, tot_e * 16 + 64, &df2));
		SYZ_HIP(hipMemcpyAsync(de2, de, (uint64_t)P * kAggRegion * 4, hipMemcpyDeviceToDevice, s));
		SYZ_HIP(hipMemcpyAsync(df2, df, (uint64_t)P * kAggRegion * 16, hipMemcpyDeviceToDevice, s));
		SYZ_HIP(hipMemsetAsync(gk, 0xff, C * 4 + (C + 1) * 16, s));
		SYZ_HIP(hipMemcpyAsync(ol, ovl.data(), ovl.size() * 4, hipMemcpyHostToDevice, s));
		SYZ_TRY(counters_reset(ctx));
		const uint64_t items = ovl.size() * ((nchunks + kAggGroup - 1) / kAggGroup);
		k_agg_global<<<grid_for(items * 64, 256, 8192), 256, 0, s>>>((const uint32_t*)recs, rec_base,
		                                                              (const uint32_t*)offsT, nchunks, g,
		                                                              (const uint32_t*)ol, (uint32_t)ovl.size(),
		                                                              (uint32_t*)gk, (uint32_t*)gf, C,
		                                                              &ctx->d_cnt[kCntError]);
		k_agg_global_compact<<<grid_for(C + 1, 256, 8192), 256, 0, s>>>(
		    (const uint32_t*)gk, (const uint32_t*)gf, C, (uint32_t*)de2 + (uint64_t)P * kAggRegion,
		    (uint4*)df2 + (uint64_t)P * kAggRegion, &ctx->d_cnt[kCntAux2]);
		SYZ_HIP(hipGetLastError());
		SYZ_TRY(counters_fetch(ctx));
		if (ctx->h_cnt[kCntError])
			return fail(SYZSIG_EIO, "triage: aggregation table overflow (internal error)");
		const uint64_t gcnt = ctx->h_cnt[kCntAux2];
		D += gcnt;
		// region counts: LDS partitions (overflowed = 0), then the fallback list in kAggRegion pieces
		std::vector<uint32_t> rc(hc);
		for (uint32_t p : ovl)
			rc[p] = 0;
		for (uint64_t left = gcnt; left; left -= std::min<uint64_t>(left, kAggRegion))
			rc.push_back((uint32_t)std::min<uint64_t>(left, kAggRegion));
		nregions = (uint32_t)rc.size();
		void* dc2;
		SYZ_TRY(ws_get(ctx, 21, rc.size() * 4 + 64, &dc2));
		SYZ_HIP(hipMemcpyAsync(dc2, rc.data(), rc.size() * 4, hipMemcpyHostToDevice, s));
		SYZ_HIP(hipStreamSynchronize(s));  // rc is a host temporary
		dc = dc2;
		dist_e = de2;
		dist_f = df2;
		st->overflow_parts += ovl.size();
	}
	st->distinct += D;
	st->parts = P;
	st->survivors += D;
	if (!entry)
		ctx->agg_distinct_ratio = run_recs ? (double)D / (double)run_recs : 0;
	out->dist_e = (const uint32_t*)dist_e;
	out->dist_f = (const uint4*)dist_f;
	out->cnt = (const uint32_t*)dc;
	out->nregions = nregions;
	out->parts = P;
	out->D = D;
	return SYZSIG_OK;
}

// Distinct elements per partition (top pbits of fmix32) over regions [r0, r1).
__global__ __launch_bounds__(256) void k_part_hist(const uint32_t* __restrict__ dist_e,
                                                   const uint32_t* __restrict__ cnt, uint32_t r0, uint32_t r1,
                                                   uint32_t pbits, uint32_t* hist)
{
	for (uint32_t r = r0 + blockIdx.x; r < r1; r += gridDim.x) {
		const uint32_t n = cnt[r] == kAggOverflow ? 0 : cnt[r];
		for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
			atomicAdd(&hist[fmix32(dist_e[(uint64_t)r * kAggRegion + i]) >> (32 - pbits)], 1u);
	}
}

// The finalize probes a partition's elements from its own slice of a table
// (home buckets = the top bits of the same h).  The HBM fallback's partitions
// hold more than kAggLimit distinct elements, possibly many more when the
// elements are not spread by the hash: their slice must take them at most 3/4
// full, or their probe sequences pile up past the probe limit.  Grows s so
// that every such partition's slice does.  Synchronises.
static int reserve_slices(syzsig_ctx* ctx, syzsig_set* s, const uint32_t* dist_e, const uint32_t* d_cnt, uint32_t r0,
                          uint32_t r1, uint32_t pbits)
{
	if (!s || r1 <= r0)
		return SYZSIG_OK;
	const uint32_t P = 1u << pbits;
	void* wh;
	SYZ_TRY(ws_get(ctx, 53, (uint64_t)P * 4 + 64, &wh));
	const hipStream_t st = ctx->stream;
	SYZ_HIP(hipMemsetAsync(wh, 0, (uint64_t)P * 4, st));
	k_part_hist<<<std::min<uint32_t>(r1 - r0, 2048), 256, 0, st>>>(dist_e, d_cnt, r0, r1, pbits, (uint32_t*)wh);
	SYZ_HIP(hipGetLastError());
	std::vector<uint32_t> h(P);
	SYZ_HIP(hipMemcpyAsync(h.data(), wh, (uint64_t)P * 4, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipStreamSynchronize(st));
	const uint64_t mx = *std::max_element(h.begin(), h.end());
	const uint64_t need = pow2_at_least((uint64_t)((double)P * (double)mx / (kBucketSlots * kMaxLoad)) + 1);
	if (need > s->nbuckets)
		SYZ_TRY(set_rehash(s, need, false));
	return SYZSIG_OK;
}

// One triage run with one host synchronisation at the end ("the
// one-sync triage run"): scatter into capped cells, k_agg, the slice-exclusive
// finalize and the deferred lists.  maxSignal and newSignal are reserved for
// the run's largest possible distinct count D_max = min(records, P * kAggLimit)
// (a growth only when len + D_max would pass 90 % of the table; the usual
// policy loads apply to the expected count), so the kernels never wait for
// the host.  fast: the caller skipped the presence pass (k_fast_prep checks its
// assumptions).  *done = false: nothing was committed (*assumed_bad: the
// assumptions failed; *regeom: too few partitions, redo; else a cell spilled:
// counted cells next, the slack doubled).
static int agg_triage_fused(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const syzsig_batch* b, uint64_t c0,
                            uint64_t c1, const LevelMap& lm, uint64_t run_recs, syzsig_batch_stats* st,
                            uint64_t** pairs_out, uint64_t* npairs_io, bool* done, bool fast = false,
                            bool* assumed_bad = nullptr, bool* regeom = nullptr)
{
	*done = false;
	bool regeom_local = false;
	if (!regeom)
		regeom = &regeom_local;
	*regeom = false;
	if (assumed_bad)
		*assumed_bad = false;
	AggGeom g = agg_geom_for(ctx, run_recs, 0);
	g.ibits = g.cbits();  // work items are whole chunks
	const uint32_t S = 1u << g.pbits, P = S;
	const uint64_t nchunks = (c1 - c0 + (1ull << g.ibits) - 1) >> g.ibits;
	// distinct elements the run can commit: an LDS partition holds at
	// most kAggLimit (one that overflows is committed after the sync)
	const uint64_t d_max = std::min<uint64_t>(run_recs, (uint64_t)P * kAggLimit);
	const double ratio = ctx->agg_distinct_ratio > 0 ? ctx->agg_distinct_ratio : 1.0 / 32;
	const uint64_t d_est = std::min<uint64_t>(d_max, (uint64_t)(ratio * (double)run_recs) + 1);
	// capacity for every possible change, before anything is committed
	SYZ_TRY(set_reserve(ms, d_est));
	SYZ_TRY(set_reserve_load(ms, d_max, kHardLoad));
	// newSignal.Merge allocates a nil receiver (signal.go:121-125) -- but only
	// when some DiffRaw is non-empty: a fresh set is dropped again if nothing changed
	const bool fresh_ns = !*ns;
	if (fresh_ns)
		SYZ_TRY(syzsig_set_make(ctx, d_est, ns));
	syzsig_set* nsp = *ns;
	// at most half full for the expected changes (short probe chains: 0.34 ->
	// 0.28 ms at C2), never past kHardLoad for the largest possible count
	SYZ_TRY(set_reserve_load(nsp, d_est, kTargetLoad));
	SYZ_TRY(set_reserve_load(nsp, d_max, kHardLoad));
	if (ms->nbuckets < P || nsp->nbuckets < P) {  // slices need a bucket per partition
		if (fresh_ns) {
			syzsig_set_free(nsp);
			*ns = nullptr;
		}
		return SYZSIG_OK;
	}
	const float sd = ctx->cap_sd;
	const uint64_t bound = (run_recs + run_recs / 4 + nchunks * S * (uint64_t)(sd * sd + 128.0f) + 127) & ~63ull;  // (the dummy lines after it: 16-B stores)
	void *recs, *cm, *dc, *pr, *dd, *dn;
	SYZ_TRY(ws_get(ctx, 16, (bound + kDummyLines * kBlk) * 4, &recs));
	SYZ_TRY(ws_get(ctx, 17, nchunks * 24 + (uint64_t)S * nchunks * 4 + 256, &cm));
	uint64_t* sizes = (uint64_t*)cm;
	uint64_t* cbase = sizes + nchunks;
	uint32_t* ccap = (uint32_t*)(cbase + nchunks);
	uint32_t* ccnt = ccap + nchunks;
	uint32_t* ovf = ccnt + (uint64_t)S * nchunks;
	uint32_t* tiles = ovf + 1;
	SYZ_TRY(ws_get(ctx, 21, (uint64_t)(P + 1) * 4 + 64, &dc));
	if (fast && *npairs_io == 0 && b->new_pairs && b->new_pairs_cap >= 4 * d_max) {
		pr = b->new_pairs;  // every possible pair fits the caller's buffer: no copy afterwards
	} else {
		SYZ_TRY(ws_grow_keep(ctx, 15, (*npairs_io + 4 * d_max) * 8 + 64, *npairs_io * 8, &pr));
	}
	*pairs_out = (uint64_t*)pr;
	SYZ_TRY(ws_get(ctx, 32, d_max * 20 + 64, &dd));
	SYZ_TRY(ws_get(ctx, 33, d_max * 8 + 64, &dn));
	const hipStream_t s = ctx->stream;
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[0], s));
	if (fast) {
		// two launches before the scatter: per-chunk sizes and checks (call_new
		// zeroed too), then the cell plan, which also zeroes the counters and
		// sets the run's void flag (ovf = the low word of ctr[kCntSpill])
		void* dpart;
		SYZ_TRY(ws_get(ctx, 54, nchunks * 16 + 64, &dpart));
		ovf = (uint32_t*)&ctx->d_cnt[kCntSpill];
		k_fast_prep<<<(uint32_t)nchunks, 256, 0, s>>>(b->call_start, b->call_len, b->call_prio, c0, c1, g.ibits, b->nrec,
		                                              sizes, (uint64_t*)dpart, b->call_new, lm, tiles);
		k_cell_plan_fast<<<1, 1024, 0, s>>>(sizes, nchunks, S, sd, cbase, ccap, (const uint64_t*)dpart, run_recs,
		                                    *npairs_io, ctx->d_cnt);
	} else {
		SYZ_TRY(counters_reset(ctx));
		memcpy(ctx->h_pin + kPinPairs, npairs_io, 8);  // consumed before the counters_fetch below
		SYZ_HIP(hipMemcpyAsync(&ctx->d_cnt[kCntAux2], ctx->h_pin + kPinPairs, 8, hipMemcpyHostToDevice, s));
		SYZ_HIP(hipMemsetAsync(ovf, 0, 4, s));
		k_chunk_sizes<<<(uint32_t)nchunks, 256, 0, s>>>(b->call_len, c0, c1, g.ibits, sizes, tiles, kScat3Tile);
		k_cell_plan<<<1, 1024, 0, s>>>(sizes, nchunks, S, sd, cbase, ccap);
	}
	const CapCells cc{cbase, ccap, ccnt, ovf, nchunks, (uint32_t*)recs + bound, sizes, tiles, false, kScat3Tile};
	scatter_triage(nchunks, s, g.pbits, b->sigs, b->call_start, b->call_len, b->call_prio, lm, c0, c1, g,
	               AggSrc{nullptr, 1, 0, 0}, cc, (uint32_t*)recs, ctx->agg_dbg >> 10);
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[1], s));
	const uint32_t pb = g.pbits;
	FinArgs fa;
	fa.lm = lm;
	fa.c0 = c0;
	fa.slots = ms->slots;
	fa.bmask = ms->nbuckets - 1;
	fa.ms_shift = (63 - __builtin_clzll(ms->nbuckets)) - pb;
	fa.ns_slots = nsp->slots;
	fa.ns_bmask = nsp->nbuckets - 1;
	fa.ns_shift = (63 - __builtin_clzll(nsp->nbuckets)) - pb;
	fa.call_new = b->call_new;
	fa.pairs = (uint64_t*)pr;
	fa.npairs = &ctx->d_cnt[kCntAux2];
	fa.ctr = ctx->d_cnt;
	fa.def_e = (uint32_t*)dd;
	fa.def_f = (uint4*)((char*)dd + ((d_max * 4 + 15) & ~15ull));
	fa.def_cnt = &ctx->d_cnt[kCntDefer];
	fa.def_ns = (uint64_t*)dn;
	fa.def_ns_cnt = &ctx->d_cnt[kCntDeferNs];
	fa.spill = ovf;
	fa.dbg = ctx->agg_dbg;
	const AggCells xc{(const uint32_t*)recs, nullptr, nullptr, cbase, ccap, ccnt, nchunks, 0, agg_group_size(nchunks),
	                  ovf, ctx->d_cnt};
	// more overflowed partitions than this and the split path commits nothing:
	// the run is redone with partitions sized from what k_agg counted
	const uint32_t gate = P / 8;
	{
		// k_agg's distinct lists through HBM (5 M x 20 B at C2), then the
		// slice-exclusive finalize: a workgroup of the finalize is small, so
		// many run per CU and their random probes overlap
		void *de, *df;
		SYZ_TRY(ws_get(ctx, 19, (uint64_t)P * kAggRegion * 4 + 64, &de));
		SYZ_TRY(ws_get(ctx, 20, (uint64_t)P * kAggRegion * 16 + 64, &df));
		launch_agg<true>(ctx, bound, P, s, xc, g, de, df, dc);
		SYZ_HIP(hipGetLastError());
		if (ctx->timing)
			SYZ_HIP(hipEventRecord(ctx->ev[2], s));
		k_agg_finalize_x<2><<<P, kFxThreads, 0, s>>>(
		    (const uint32_t*)de, (const uint4*)df, (const uint32_t*)dc, P, lm, c0, fa.slots, fa.bmask, fa.ms_shift,
		    fa.ns_slots, fa.ns_bmask, fa.ns_shift, fa.call_new, fa.pairs, fa.npairs, ctx->d_cnt, fa.def_e, fa.def_f,
		    fa.def_cnt, fa.def_ns, fa.def_ns_cnt, ctx->agg_dbg, ovf, &ctx->d_cnt[kCntAggOvf], gate);
		SYZ_HIP(hipGetLastError());
	}
	// (the deferred lists in a launch of their own: taken by the finalize's last
	// block instead, they made the finalize 1.03 ms instead of 0.27 at C2)
	k_fin_deferred<<<2 * kDeferBlocks, 256, 0, s>>>(fa.def_e, fa.def_f, fa.def_cnt, lm, c0, ms->slots, ms->nbuckets - 1,
	                                                nsp->slots, nsp->nbuckets - 1, b->call_new, (uint64_t*)pr,
	                                                fa.npairs, ctx->d_cnt, fa.def_ns, fa.def_ns_cnt);
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[3], s));
	uint32_t* hov = (uint32_t*)(ctx->h_pin + kPinCounts);
	if (!fast)
		SYZ_HIP(hipMemcpyAsync(hov, ovf, 4, hipMemcpyDeviceToHost, s));
	SYZ_TRY(counters_fetch(ctx));  // the run's one synchronisation
	if (fast) {
		*hov = (uint32_t)ctx->h_cnt[kCntSpill];
		st->records = ctx->h_cnt[kCntRecords];
	}
	if (ctx->timing) {
		float t0 = 0, t1 = 0, t2 = 0;
		SYZ_HIP(hipEventElapsedTime(&t0, ctx->ev[0], ctx->ev[1]));
		SYZ_HIP(hipEventElapsedTime(&t1, ctx->ev[1], ctx->ev[2]));
		SYZ_HIP(hipEventElapsedTime(&t2, ctx->ev[2], ctx->ev[3]));
		st->part_ms += t0;
		st->probe_ms += t1;
		st->decide_ms += t2;
	}
	if (*hov & 6) {  // an optimistic run's assumptions failed: nothing committed
		*assumed_bad = true;
		if (fresh_ns) {
			syzsig_set_free(nsp);
			*ns = nullptr;
		}
		return SYZSIG_OK;
	}
	if (*hov) {  // a cell spilled: nothing committed, redo with counted cells
		st->retries++;
		ctx->cap_sd = ctx->cap_sd * 2 > kCapSdMax ? 0.0f : ctx->cap_sd * 2;
		if (fresh_ns) {
			syzsig_set_free(nsp);
			*ns = nullptr;
		}
		return SYZSIG_OK;
	}
	if (ctx->h_cnt[kCntOverflow])
		return fail(SYZSIG_EIO, "triage: table overflow after reserve (internal error; one-sync run)");
	uint64_t D = ctx->h_cnt[kCntDistinct];
	uint64_t inserted = ctx->h_cnt[kCntInserted], changed = ctx->h_cnt[kCntChanged], ns_ins = ctx->h_cnt[kCntAux];
	uint64_t inserted_done = 0;  // already added to maxSignal's length
	uint64_t npairs = ctx->h_cnt[kCntAux2];
	const uint64_t novf = ctx->h_cnt[kCntAggOvf];
	if (novf > gate) {
		// too few partitions (the distinct-ratio guess was low): nothing was
		// committed; the next attempt sizes them for at least what was seen
		// (an overflowed partition held more than kAggLimit)
		// (most partitions overflowed: what they held is unknown, so size for the
		// worst case, one distinct element per record)
		const double seen = novf * 2 >= P ? (double)run_recs : (double)D + 2.0 * (double)novf * kAggLimit;
		ctx->agg_distinct_ratio = std::max(ctx->agg_distinct_ratio, seen / (double)std::max<uint64_t>(run_recs, 1));
		st->retries++;
		if (fresh_ns) {
			syzsig_set_free(nsp);
			*ns = nullptr;
		}
		*regeom = true;
		return SYZSIG_OK;
	}
	if (novf) {
		// partitions past the LDS table: aggregated in HBM from their cells,
		// then finalized with the atomic code (their elements are disjoint from
		// every committed partition's).  The committed partitions' inserts count
		// first: the reservations below start from the tables' true lengths.
		ms->len += inserted;
		nsp->len += ns_ins;
		inserted_done += inserted;
		inserted = ns_ins = 0;
		std::vector<uint32_t> hc(P);
		SYZ_HIP(hipMemcpy(hc.data(), dc, P * 4, hipMemcpyDeviceToHost));
		std::vector<uint32_t> ovl;
		uint64_t ovrec = 0;
		std::vector<uint32_t> hcnt((uint64_t)P * nchunks);
		SYZ_HIP(hipMemcpy(hcnt.data(), ccnt, hcnt.size() * 4, hipMemcpyDeviceToHost));
		for (uint32_t q = 0; q < P; q++) {
			if (hc[q] != kAggOverflow)
				continue;
			ovl.push_back(q);
			for (uint64_t c = 0; c < nchunks; c++)
				ovrec += hcnt[(uint64_t)q * nchunks + c];
		}
		const uint64_t C = pow2_at_least(std::max<uint64_t>(2 * ovrec, 1024));
		void *gk, *ol, *de2, *df2, *dc2;
		SYZ_TRY(ws_get(ctx, 23, C * 4 + (C + 1) * 16 + 64, &gk));
		void* gf = (char*)gk + C * 4;
		SYZ_TRY(ws_get(ctx, 22, ovl.size() * 4 + 64, &ol));
		SYZ_TRY(ws_get(ctx, 30, ovrec * 4 + 64, &de2));
		SYZ_TRY(ws_get(ctx, 31, ovrec * 16 + 64, &df2));
		SYZ_HIP(hipMemsetAsync(gk, 0xff, C * 4 + (C + 1) * 16, s));
		SYZ_HIP(hipMemcpyAsync(ol, ovl.data(), ovl.size() * 4, hipMemcpyHostToDevice, s));
		SYZ_TRY(counters_reset(ctx));
		k_agg_global_cap<<<grid_for(ovl.size() * nchunks * 64, 256, 8192), 256, 0, s>>>(
		    (const uint32_t*)recs, cbase, ccap, ccnt, nchunks, g, (const uint32_t*)ol, (uint32_t)ovl.size(),
		    (uint32_t*)gk, (uint32_t*)gf, C, &ctx->d_cnt[kCntError]);
		k_agg_global_compact<<<grid_for(C + 1, 256, 8192), 256, 0, s>>>((const uint32_t*)gk, (const uint32_t*)gf, C,
		                                                                 (uint32_t*)de2, (uint4*)df2,
		                                                                 &ctx->d_cnt[kCntAux2]);
		SYZ_HIP(hipGetLastError());
		SYZ_TRY(counters_fetch(ctx));
		if (ctx->h_cnt[kCntError])
			return fail(SYZSIG_EIO, "triage: aggregation table overflow (internal error)");
		const uint64_t gcnt = ctx->h_cnt[kCntAux2];
		D += gcnt;
		std::vector<uint32_t> rc;
		for (uint64_t left = gcnt; left; left -= std::min<uint64_t>(left, kAggRegion))
			rc.push_back((uint32_t)std::min<uint64_t>(left, kAggRegion));
		if (!rc.empty()) {
			// the reservations above covered the committed partitions (<= kAggLimit
			// distinct each); these elements come on top
			SYZ_TRY(set_reserve(ms, gcnt));
			SYZ_TRY(set_reserve_load(nsp, gcnt, kHardLoad));
			SYZ_TRY(ws_get(ctx, 35, rc.size() * 4 + 64, &dc2));
			SYZ_HIP(hipMemcpyAsync(dc2, rc.data(), rc.size() * 4, hipMemcpyHostToDevice, s));
			SYZ_TRY(reserve_slices(ctx, ms, (const uint32_t*)de2, (const uint32_t*)dc2, 0, (uint32_t)rc.size(), pb));
			SYZ_TRY(reserve_slices(ctx, nsp, (const uint32_t*)de2, (const uint32_t*)dc2, 0, (uint32_t)rc.size(), pb));
			if (pr == b->new_pairs) {
				// the run wrote its pairs straight into the caller's buffer: keep
				// appending there while it has room, else move them to workspace
				// 15 first (ws_grow_keep keeps only what that workspace held)
				if (b->new_pairs_cap < npairs + 4 * gcnt) {
					void* w;
					SYZ_TRY(ws_get(ctx, 15, (npairs + 4 * gcnt) * 8 + 64, &w));
					if (npairs)
						SYZ_HIP(hipMemcpyAsync(w, pr, npairs * 8, hipMemcpyDeviceToDevice, s));
					pr = w;
				}
			} else {
				SYZ_TRY(ws_grow_keep(ctx, 15, (npairs + 4 * gcnt) * 8 + 64, npairs * 8, &pr));
			}
			*pairs_out = (uint64_t*)pr;
			SYZ_TRY(counters_reset(ctx));
			memcpy(ctx->h_pin + kPinPairs, &npairs, 8);
			SYZ_HIP(hipMemcpyAsync(&ctx->d_cnt[kCntAux2], ctx->h_pin + kPinPairs, 8, hipMemcpyHostToDevice, s));
			k_agg_finalize<<<(uint32_t)rc.size(), kFinThreads, 0, s>>>(
			    (const uint32_t*)de2, (const uint4*)df2, (const uint32_t*)dc2, (uint32_t)rc.size(), lm, c0, ms->slots,
			    ms->nbuckets - 1, nsp->slots, nsp->nbuckets - 1, b->call_new, (uint64_t*)pr, &ctx->d_cnt[kCntAux2],
			    ctx->d_cnt, ctx->agg_dbg);
			SYZ_HIP(hipGetLastError());
			SYZ_TRY(counters_fetch(ctx));  // (synchronizes: rc is consumed)
			if (ctx->h_cnt[kCntOverflow])
				return fail(SYZSIG_EIO, "triage: table overflow after reserve (internal error; one-sync run, HBM partitions)");
			inserted += ctx->h_cnt[kCntInserted];
			changed += ctx->h_cnt[kCntChanged];
			ns_ins += ctx->h_cnt[kCntAux];
			npairs = ctx->h_cnt[kCntAux2];
		}
		st->overflow_parts += novf;
	}
	if (fresh_ns && changed == 0) {
		syzsig_set_free(nsp);
		*ns = nullptr;
		nsp = nullptr;
	}
	ms->len += inserted;
	if (nsp)
		nsp->len += ns_ins;
	inserted += inserted_done;
	st->distinct += D;
	st->parts = P;
	st->survivors += D;
	st->inserted += inserted;
	st->changed += changed;
	st->candidates += changed;
	st->runs++;
	ctx->agg_distinct_ratio = run_recs ? (double)D / (double)run_recs : 0;
	*npairs_io = npairs;
	*done = true;
	return SYZSIG_OK;
}

// One run of calls [c0, c1) with level map lm.  Pairs are appended at
// pairs[*npairs_io ...] (internal buffer, grown as needed).
int agg_triage_run(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const syzsig_batch* b, uint64_t c0, uint64_t c1,
                   const LevelMap& lm, uint64_t run_recs, syzsig_batch_stats* st, uint64_t** pairs_out,
                   uint64_t* npairs_io)
{
	if (ctx->cap_sd > 0 && !(ctx->agg_dbg & (SYZSIG_DEBUG_EXACT_CELLS | SYZSIG_DEBUG_CAP_SPILL | 16)) &&
	    !ctx->agg_counted_once) {
		bool done = false, regeom = false;
		uint64_t retries0 = st->retries;
		SYZ_TRY(agg_triage_fused(ctx, ms, ns, b, c0, c1, lm, run_recs, st, pairs_out, npairs_io, &done, false,
		                         nullptr, &regeom));
		if (regeom) {  // once more with partitions for what the first attempt counted
			retries0 = st->retries;
			SYZ_TRY(agg_triage_fused(ctx, ms, ns, b, c0, c1, lm, run_recs, st, pairs_out, npairs_io, &done));
		}
		if (done)
			return SYZSIG_OK;
		// a spilled cell: this run is redone with counted cells, not capped ones again
		ctx->agg_counted_once = st->retries != retries0;
	}
	AggOut a;
	SYZ_TRY(agg_aggregate(ctx, b, c0, c1, lm, run_recs, st, &a));
	const uint64_t D = a.D;
	const hipStream_t s = ctx->stream;
	void* pr;
	// capacity for every possible change, then finalize (never retried)
	SYZ_TRY(set_reserve(ms, D));
	// newSignal.Merge allocates a nil receiver (signal.go:121-125) -- but only
	// when some DiffRaw is non-empty: a fresh set is dropped again if nothing changed
	const bool fresh_ns = D && !*ns;
	if (fresh_ns)
		SYZ_TRY(syzsig_set_make(ctx, D, ns));
	// newSignal takes up to D changes per batch: kept at most half full, so its
	// probe chains stay short in the finalize (0.34 -> 0.28 ms at C2)
	if (D)
		SYZ_TRY(set_reserve_load(*ns, D, kTargetLoad));
	if (a.nregions > a.parts) {  // the HBM fallback's partitions: room in their slices
		const uint32_t pb = 31 - __builtin_clz(a.parts);
		SYZ_TRY(reserve_slices(ctx, ms, a.dist_e, a.cnt, a.parts, a.nregions, pb));
		SYZ_TRY(reserve_slices(ctx, *ns, a.dist_e, a.cnt, a.parts, a.nregions, pb));
	}
	const uint64_t need_pairs = *npairs_io + 4 * D;
	SYZ_TRY(ws_grow_keep(ctx, 15, need_pairs * 8 + 64, *npairs_io * 8, &pr));
	*pairs_out = (uint64_t*)pr;
	SYZ_TRY(counters_reset(ctx));
	memcpy(ctx->h_pin + kPinPairs, npairs_io, 8);  // consumed before the counters_fetch below
	SYZ_HIP(hipMemcpyAsync(&ctx->d_cnt[kCntAux2], ctx->h_pin + kPinPairs, 8, hipMemcpyHostToDevice, s));
	syzsig_set* nsp = *ns;
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[2], s));
	// the slice-exclusive finalize when every region is a partition and both
	// tables have at least one bucket per partition; else the atomic one
	const bool fx = D && nsp && a.nregions == a.parts && ms->nbuckets >= a.parts && nsp->nbuckets >= a.parts &&
	                !(ctx->agg_dbg & 16);
	if (fx) {
		const uint32_t pb = 31 - __builtin_clz(a.parts);
		const uint32_t ms_shift = (63 - __builtin_clzll(ms->nbuckets)) - pb;
		const uint32_t ns_shift = (63 - __builtin_clzll(nsp->nbuckets)) - pb;
		void *dd, *dn;
		SYZ_TRY(ws_get(ctx, 32, D * 20 + 64, &dd));
		SYZ_TRY(ws_get(ctx, 33, D * 8 + 64, &dn));
		uint32_t* def_e = (uint32_t*)dd;
		uint4* def_f = (uint4*)((char*)dd + ((D * 4 + 15) & ~15ull));
		k_agg_finalize_x<2><<<a.nregions, kFxThreads, 0, s>>>(
		    a.dist_e, a.dist_f, a.cnt, a.nregions, lm, c0, ms->slots, ms->nbuckets - 1, ms_shift, nsp->slots,
		    nsp->nbuckets - 1, ns_shift, b->call_new, (uint64_t*)pr, &ctx->d_cnt[kCntAux2], ctx->d_cnt, def_e, def_f,
		    &ctx->d_cnt[kCntDefer], (uint64_t*)dn, &ctx->d_cnt[kCntDeferNs], ctx->agg_dbg, nullptr, nullptr, 0);
		k_fin_deferred<<<2 * kDeferBlocks, 256, 0, s>>>(def_e, def_f, &ctx->d_cnt[kCntDefer], lm, c0, ms->slots,
		                                                ms->nbuckets - 1, nsp->slots, nsp->nbuckets - 1, b->call_new,
		                                                (uint64_t*)pr, &ctx->d_cnt[kCntAux2], ctx->d_cnt,
		                                                (const uint64_t*)dn, &ctx->d_cnt[kCntDeferNs]);
	} else if (D) {
		k_agg_finalize<<<a.nregions, kFinThreads, 0, s>>>(
		    a.dist_e, a.dist_f, a.cnt, a.nregions, lm, c0, ms->slots,
		    ms->nbuckets - 1, nsp ? nsp->slots : nullptr, nsp ? nsp->nbuckets - 1 : 0, b->call_new, (uint64_t*)pr,
		    &ctx->d_cnt[kCntAux2], ctx->d_cnt, ctx->agg_dbg);
	}
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[3], s));
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->timing) {
		float t = 0;
		SYZ_HIP(hipEventElapsedTime(&t, ctx->ev[2], ctx->ev[3]));
		st->decide_ms += t;
	}
	if (ctx->h_cnt[kCntOverflow])
		return fail(SYZSIG_EIO, "triage: table overflow after reserve (internal error; planned run)");
	if (fresh_ns && ctx->h_cnt[kCntChanged] == 0) {
		syzsig_set_free(*ns);
		*ns = nullptr;
		nsp = nullptr;
	}
	ms->len += ctx->h_cnt[kCntInserted];
	st->inserted += ctx->h_cnt[kCntInserted];
	st->changed += ctx->h_cnt[kCntChanged];
	st->candidates += ctx->h_cnt[kCntChanged];
	if (nsp)
		nsp->len += ctx->h_cnt[kCntAux];
	*npairs_io = ctx->h_cnt[kCntAux2];
	st->runs++;
	return SYZSIG_OK;
}

int agg_triage_optimistic(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const syzsig_batch* b,
                          syzsig_batch_stats* st, uint64_t** pairs, uint64_t* npairs, bool* done)
{
	*done = false;
	if (ctx->cap_sd <= 0 || ctx->agg_counted_once ||
	    (ctx->agg_dbg & (SYZSIG_DEBUG_EXACT_CELLS | SYZSIG_DEBUG_CAP_SPILL | 16)))
		return SYZSIG_OK;
	LevelMap lm;
	const int8_t lv[4] = {0, 1, 2, 3};
	SYZ_TRY(level_map_from_levels(lv, 4, &lm));
	bool bad = false, regeom = false;
	uint64_t retries0 = st->retries;
	SYZ_TRY(agg_triage_fused(ctx, ms, ns, b, 0, b->ncalls, lm, b->nrec, st, pairs, npairs, done, true, &bad,
	                         &regeom));
	if (regeom) {  // once more with partitions for what the first attempt counted
		retries0 = st->retries;
		SYZ_TRY(agg_triage_fused(ctx, ms, ns, b, 0, b->ncalls, lm, b->nrec, st, pairs, npairs, done, true, &bad));
	}
	// a spilled cell: the planned path redoes the batch with counted cells
	ctx->agg_counted_once = !*done && st->retries != retries0;
	return SYZSIG_OK;
}

// Per-record bits of calls [c0, c1) from the run's pairs [p0, p1).
int agg_mark_bits(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t c0, uint64_t c1, const uint64_t* pairs,
                  uint64_t p0, uint64_t p1)
{
	if (p1 == p0 || !b->new_bits)
		return SYZSIG_OK;
	const uint64_t n = p1 - p0, C = pow2_at_least(2 * n + 16);
	void* set;
	SYZ_TRY(ws_get(ctx, 14, C * 8, &set));
	const hipStream_t s = ctx->stream;
	SYZ_HIP(hipMemsetAsync(set, 0xff, C * 8, s));
	SYZ_TRY(counters_reset(ctx));
	k_pairs_set<<<grid_for(n, 256, 8192), 256, 0, s>>>(pairs + p0, n, (uint64_t*)set, C, &ctx->d_cnt[kCntAux]);
	k_pairs_mark<<<grid_for((c1 - c0) * 64, 256, 8192), 256, 0, s>>>(b->sigs, b->call_start, b->call_len, c0, c1,
	                                                                  b->call_new, (const uint64_t*)set, C, b->new_bits);
	SYZ_HIP(hipGetLastError());
	return SYZSIG_OK;
}

// Pairs of the per-call path from its bits: collect, then dedup through a set.
int pairs_from_bits(syzsig_ctx* ctx, const syzsig_batch* b, const uint32_t* bits, uint64_t c0, uint64_t c1,
                    uint64_t bound, uint64_t** pairs_io, uint64_t* npairs_io)
{
	const hipStream_t s = ctx->stream;
	void *raw, *set, *out;
	SYZ_TRY(ws_get(ctx, 13, bound * 8 + 64, &raw));
	SYZ_TRY(counters_reset(ctx));
	k_bits_to_pairs<<<grid_for((c1 - c0) * 64, 256, 8192), 256, 0, s>>>(b->sigs, b->call_start, b->call_len, c0, c1,
	                                                                     b->call_new, bits, (uint64_t*)raw,
	                                                                     &ctx->d_cnt[kCntAux]);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	const uint64_t n = ctx->h_cnt[kCntAux];
	if (n == 0)
		return SYZSIG_OK;
	const uint64_t C = pow2_at_least(2 * n + 16);
	SYZ_TRY(ws_get(ctx, 14, C * 8, &set));
	SYZ_HIP(hipMemsetAsync(set, 0xff, C * 8, s));
	SYZ_TRY(ws_grow_keep(ctx, 15, (*npairs_io + n) * 8 + 64, *npairs_io * 8, &out));
	*pairs_io = (uint64_t*)out;
	SYZ_TRY(counters_reset(ctx));
	memcpy(ctx->h_pin + kPinPairs, npairs_io, 8);  // consumed before the counters_fetch below
	SYZ_HIP(hipMemcpyAsync(&ctx->d_cnt[kCntAux2], ctx->h_pin + kPinPairs, 8, hipMemcpyHostToDevice, s));
	k_pairs_set<<<grid_for(n, 256, 8192), 256, 0, s>>>((const uint64_t*)raw, n, (uint64_t*)set, C,
	                                                   &ctx->d_cnt[kCntAux]);
	k_pairs_compact<<<grid_for(C, 256, 8192), 256, 0, s>>>((const uint64_t*)set, C, (uint64_t*)out,
	                                                       &ctx->d_cnt[kCntAux2]);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	*npairs_io = ctx->h_cnt[kCntAux2];
	return SYZSIG_OK;
}

// ---------------------------------------------------------------- sharded batches
// A GPU's batch is aggregated locally and only each distinct element's
// staircase is routed to the element's owner: level l with first serial f[l]
// is on it iff f[l] < f[l'] for every higher level l'.  Any other record of e
// has an earlier local record of at least its level, so it is never new and
// never raises M_final -- and whatever dominates a staircase record in the
// whole batch, some staircase record (of any GPU) dominates it too.  So the
// owner's records-mode triage of the staircases gives checkNewSignal's exact
// result, at <= 4 records per distinct element instead of every record
// (SURVEY.md 8(e) "local filter").
constexpr uint32_t kMaxShardsAgg = 64;

__device__ __forceinline__ uint32_t stair_levels(uint4 f4, uint32_t nlev)
{
	const uint32_t f[4] = {f4.x, f4.y, f4.z, f4.w};
	uint32_t m = 0, mk = kAggNone;
#pragma unroll
	for (int l = 3; l >= 0; l--)
		if (l < (int)nlev && f[l] < mk) {
			mk = f[l];
			m |= 1u << l;
		}
	return m;
}




// ---- the stream-ordered step's source side (syzsig_step_send_dev / _back_dev)
// Staircase records into fixed buckets: owner g's at send[g * (cap + 1) + 1 ...],
// cursor[g] = its true count (records past cap are counted, not written).
// Nothing is written when the run is void (gate: its spill flag or an LDS
// partition overflow).
__global__ __launch_bounds__(256) void k_stair_bucket(const uint32_t* __restrict__ dist_e,
                                                      const uint4* __restrict__ dist_f,
                                                      const uint32_t* __restrict__ cnt, uint32_t nregions,
                                                      uint32_t nlev, uint32_t nshards, uint64_t serial_base,
                                                      uint64_t cap, unsigned long long* cursor, uint64_t* send,
                                                      const unsigned long long* gate)
{
	__shared__ uint32_t h[kMaxShardsAgg];
	__shared__ unsigned long long base[kMaxShardsAgg];
	if (gate[kCntSpill] || gate[kCntAggOvf])
		return;
	for (uint32_t r = blockIdx.x; r < nregions; r += gridDim.x) {
		if (threadIdx.x < kMaxShardsAgg)
			h[threadIdx.x] = 0;
		__syncthreads();
		const uint32_t n = cnt[r] == kAggOverflow ? 0 : cnt[r];
		for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
			const uint64_t o = (uint64_t)r * kAggRegion + i;
			const uint32_t m = stair_levels(dist_f[o], nlev);
			if (m)
				atomicAdd(&h[owner_of(dist_e[o], nshards)], (uint32_t)__popc(m));
		}
		__syncthreads();
		if (threadIdx.x < nshards) {
			base[threadIdx.x] = h[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)h[threadIdx.x]) : 0;
			h[threadIdx.x] = 0;
		}
		__syncthreads();
		for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
			const uint64_t o = (uint64_t)r * kAggRegion + i;
			const uint4 f4 = dist_f[o];
			const uint32_t m = stair_levels(f4, nlev);
			if (!m)
				continue;
			const uint32_t e = dist_e[o], g = owner_of(e, nshards);
			const uint32_t f[4] = {f4.x, f4.y, f4.z, f4.w};
			uint64_t pos = base[g] + atomicAdd(&h[g], (uint32_t)__popc(m));
			uint64_t* bk = send + (uint64_t)g * (cap + 1) + 1;
#pragma unroll
			for (uint32_t l = 0; l < 4; l++)
				if ((m >> l) & 1) {
					if (pos < cap)
						bk[pos] = ((uint64_t)e << 32) | ((uint64_t)l << 24) | ((serial_base + f[l]) & kSerialMask);
					pos++;
				}
		}
		__syncthreads();
	}
}

// bucket headers; the source's sent records and its largest bucket
__global__ void k_stair_heads(const unsigned long long* __restrict__ cursor, uint32_t nshards, uint64_t cap,
                              uint64_t* send, unsigned long long* sc)
{
	if (threadIdx.x != 0)
		return;
	const bool vd = sc[kCntSpill] != 0 || sc[kCntAggOvf] != 0;
	uint64_t tot = 0, mx = 0;
	for (uint32_t g = 0; g < nshards; g++) {
		const uint64_t c = vd ? 0 : cursor[g];
		tot += c;
		mx = max(mx, c);
	}
	// an overflow toward any owner is flagged to every owner, so that all of
	// them skip the step alike
	for (uint32_t g = 0; g < nshards; g++) {
		const uint64_t c = vd ? 0 : cursor[g];
		send[(uint64_t)g * (cap + 1)] = (c & SYZSIG_STEP_HDR_COUNT) | (vd ? SYZSIG_STEP_HDR_VOID : 0) |
		                                (mx > cap ? SYZSIG_STEP_HDR_OVF : 0);
	}
	sc[kCntCandidates] = tot;
	sc[kCntTouched] = mx;
}

// The owners' flags back at the source (blockIdx.y = owner g): the owner's
// status byte (1: the step is void, 2: the owner skipped) and, when 0, every
// flagged record of bucket g as the pair (call = serial - serial_base, e).
__global__ __launch_bounds__(256) void k_step_back(const uint64_t* __restrict__ send, const uint8_t* __restrict__ back,
                                                   uint64_t cap, uint64_t serial_base, uint8_t* call_new,
                                                   uint64_t* pairs, uint64_t pairs_cap, unsigned long long* bc)
{
	const uint32_t g = blockIdx.y, lane = lane_id();
	const uint64_t s0 = (uint64_t)g * (cap + 1);
	const uint8_t st = back[s0];
	if (st) {
		if (blockIdx.x == 0 && threadIdx.x == 0) {
			if (st == 1)
				atomicOr(&bc[kCntError], 1ull);
			else
				atomicOr(&bc[kCntAux], 1ull << g);
		}
		return;
	}
	// one device atomic per block and pass (a per-wave atomic on the one
	// counter serialised the kernel: 176 us at C4)
	__shared__ uint32_t wcnt[4];
	__shared__ unsigned long long s_base;
	const uint32_t w = threadIdx.x >> 6;
	const uint64_t n = min<uint64_t>(send[s0] & SYZSIG_STEP_HDR_COUNT, cap);
	for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < n; i0 += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t i = i0 + threadIdx.x;
		const bool on = i < n && back[s0 + 1 + i];
		uint64_t v = 0;
		if (on) {
			const uint64_t r = send[s0 + 1 + i];
			const uint64_t c = (r & kSerialMask) - serial_base;
			call_new[c] = 1;
			v = (c << 32) | (r >> 32);
		}
		const uint64_t m = __ballot(on);
		if (lane == 0)
			wcnt[w] = (uint32_t)__popcll(m);
		__syncthreads();
		uint32_t before = 0, tot = 0;
		for (uint32_t k = 0; k < 4; k++) {
			before += k < w ? wcnt[k] : 0;
			tot += wcnt[k];
		}
		if (threadIdx.x == 0)
			s_base = tot ? atomicAdd(&bc[kCntAux2], (unsigned long long)tot) : 0;
		__syncthreads();
		const uint64_t o = s_base + before + lane_rank(m);
		if (on && pairs && o < pairs_cap)
			pairs[o] = v;
		__syncthreads();  // wcnt / s_base are rewritten by the next pass
	}
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzsig_step_send_dev(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t serial_base, const int8_t* levels,
                         uint32_t nlevels, uint32_t nshards, uint64_t cap, uint64_t* d_send, int exact)
{
	SYZ_LOCK(ctx);
	if (!ctx || !b || !d_send || (b->nrec && !b->sigs) ||
	    (b->ncalls && (!b->call_start || !b->call_len || !b->call_prio || !b->call_new)))
		return fail(SYZSIG_EINVAL, "step_send: NULL argument");
	if (nshards == 0 || nshards > kMaxShardsAgg || cap == 0 || cap > SYZSIG_STEP_HDR_COUNT)
		return fail(SYZSIG_EINVAL, "step_send: need 1 <= nshards <= 64 and 1 <= cap < 2^40");
	if (b->nrec >= (1ull << 32))
		return fail(SYZSIG_ERANGE, "step_send: >= 2^32 records per GPU");
	if (serial_base + b->ncalls > kSerialMask + 1ull)
		return fail(SYZSIG_ERANGE, "step_send: batch serial order exceeds 2^24 calls");
	LevelMap lm;
	SYZ_TRY(level_map_from_levels(levels, nlevels, &lm));
	const hipStream_t s = ctx->stream;
	unsigned long long* sc = ctx->d_step + kStepSrc;
	void* wcur;
	SYZ_TRY(ws_get(ctx, 63, kMaxShardsAgg * 8 + 64, &wcur));
	unsigned long long* cursor = (unsigned long long*)wcur;
	ctx->step_src_timed = ctx->timing;
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev_step[0], s));
	// the flags-back counters start the step; the source counters are zeroed
	// below (or by k_cell_plan_fast)
	SYZ_HIP(hipMemsetAsync(ctx->d_step + kStepBack, 0, kNumCounters * 8, s));
	SYZ_HIP(hipMemsetAsync(cursor, 0, kMaxShardsAgg * 8, s));
	if (b->new_bits)
		SYZ_HIP(hipMemsetAsync(b->new_bits, 0, ((b->nrec + 31) / 32) * 4, s));
	const bool fast = !exact && ctx->cap_sd > 0 && !ctx->agg_counted_once && b->ncalls && b->nrec &&
	                  !(ctx->agg_dbg & (SYZSIG_DEBUG_EXACT_CELLS | SYZSIG_DEBUG_CAP_SPILL));
	if (fast) {
		// one capped-cell run with its assumptions checked on device (as the
		// one-sync triage run): prios among `levels`, valid ranges, <= nrec records
		AggGeom g = agg_geom_for(ctx, b->nrec, 0);
		g.ibits = g.cbits();
		const uint32_t S = 1u << g.pbits, P = S;
		const uint64_t nchunks = (b->ncalls + (1ull << g.ibits) - 1) >> g.ibits;
		const float sd = ctx->cap_sd;
		ctx->step_src_parts = P;
		const uint64_t bound = b->nrec + b->nrec / 4 + nchunks * S * (uint64_t)(sd * sd + 128.0f) + 64;
		void *recs, *cm, *dc, *de, *df, *dpart;
		SYZ_TRY(ws_get(ctx, 16, (bound + kDummyLines * kBlk) * 4, &recs));
		SYZ_TRY(ws_get(ctx, 17, nchunks * 24 + (uint64_t)S * nchunks * 4 + 256, &cm));
		SYZ_TRY(ws_get(ctx, 21, (uint64_t)(P + 1) * 4 + 64, &dc));
		SYZ_TRY(ws_get(ctx, 19, (uint64_t)P * kAggRegion * 4 + 64, &de));
		SYZ_TRY(ws_get(ctx, 20, (uint64_t)P * kAggRegion * 16 + 64, &df));
		SYZ_TRY(ws_get(ctx, 54, nchunks * 16 + 64, &dpart));
		uint64_t* sizes = (uint64_t*)cm;
		uint64_t* cbase = sizes + nchunks;
		uint32_t* ccap = (uint32_t*)(cbase + nchunks);
		uint32_t* ccnt = ccap + nchunks;
		uint32_t* tiles = ccnt + (uint64_t)S * nchunks;
		uint32_t* ovf = (uint32_t*)&sc[kCntSpill];
		k_fast_prep<<<(uint32_t)nchunks, 256, 0, s>>>(b->call_start, b->call_len, b->call_prio, 0, b->ncalls, g.ibits,
		                                              b->nrec, sizes, (uint64_t*)dpart, b->call_new, lm, tiles);
		k_cell_plan_fast<<<1, 1024, 0, s>>>(sizes, nchunks, S, sd, cbase, ccap, (const uint64_t*)dpart, b->nrec, 0, sc);
		const CapCells cc{cbase, ccap, ccnt, ovf, nchunks, (uint32_t*)recs + bound, sizes, tiles, false, kScat3Tile};
		scatter_triage(nchunks, s, g.pbits, b->sigs, b->call_start, b->call_len, b->call_prio, lm, 0, b->ncalls, g,
		               AggSrc{nullptr, 1, 0, 0}, cc, (uint32_t*)recs, ctx->agg_dbg >> 10);
		const AggCells xc{(const uint32_t*)recs, nullptr, nullptr, cbase, ccap, ccnt, nchunks, 0, agg_group_size(nchunks),
		                  ovf, sc};
		launch_agg<true>(ctx, bound, P, s, xc, g, de, df, dc);
		k_stair_bucket<<<(int)std::min<uint32_t>(P, 2048), 256, 0, s>>>(
		    (const uint32_t*)de, (const uint4*)df, (const uint32_t*)dc, P, lm.n, nshards, serial_base, cap, cursor,
		    d_send, sc);
		SYZ_HIP(hipGetLastError());
	} else {
		// the exact path: validated, counted cells, the HBM fallback (host round trips)
		unsigned long long* hs = ctx->h_step + kStepSrc;
		memset(hs, 0, kNumCounters * 8);
		if (b->ncalls)
			SYZ_HIP(hipMemsetAsync(b->call_new, 0, b->ncalls, s));
		if (b->ncalls && b->nrec) {
			uint64_t total = 0;
			uint32_t mask[8];
			SYZ_TRY(batch_total_records(ctx, b, &total, mask));
			for (int p = 0; p < 256; p++)
				if (((mask[p >> 5] >> (p & 31)) & 1) && lm.lvl[p] == 0xff)
					return fail(SYZSIG_EINVAL, "step_send: a call's prio is not among `levels`");
			hs[kCntRecords] = total;
			if (total) {
				syzsig_batch_stats st;
				memset(&st, 0, sizeof(st));
				AggOut a;
				SYZ_TRY(agg_aggregate(ctx, b, 0, b->ncalls, lm, total, &st, &a));
				hs[kCntDistinct] = a.D;
				SYZ_HIP(hipMemcpyAsync(sc, hs, kNumCounters * 8, hipMemcpyHostToDevice, s));
				k_stair_bucket<<<(int)std::min<uint32_t>(a.nregions, 2048), 256, 0, s>>>(
				    a.dist_e, a.dist_f, a.cnt, a.nregions, lm.n, nshards, serial_base, cap, cursor, d_send, sc);
				SYZ_HIP(hipGetLastError());
			}
		}
		SYZ_HIP(hipMemcpyAsync(sc, hs, kNumCounters * 8, hipMemcpyHostToDevice, s));
		SYZ_HIP(hipStreamSynchronize(s));  // hs is consumed
	}
	k_stair_heads<<<1, 64, 0, s>>>(cursor, nshards, cap, d_send, sc);
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev_step[1], s));
	return SYZSIG_OK;
}

int syzsig_step_back_dev(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t serial_base, const uint64_t* d_send,
                         uint32_t nshards, uint64_t cap, const uint8_t* d_back)
{
	SYZ_LOCK(ctx);
	if (!ctx || !b || !d_send || !d_back || (b->ncalls && !b->call_new) || (b->new_pairs_cap && !b->new_pairs))
		return fail(SYZSIG_EINVAL, "step_back: NULL argument");
	if (nshards == 0 || nshards > kMaxShardsAgg || cap == 0 || cap > SYZSIG_STEP_HDR_COUNT)
		return fail(SYZSIG_EINVAL, "step_back: need 1 <= nshards <= 64 and 1 <= cap < 2^40");
	const hipStream_t s = ctx->stream;
	unsigned long long* bc = ctx->d_step + kStepBack;
	ctx->step_back_timed = ctx->timing;
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev_step[4], s));
	const dim3 grid(grid_for(cap, 256, std::max(1, 2048 / (int)nshards)), nshards);
	if (!b->new_bits) {
		k_step_back<<<grid, 256, 0, s>>>(d_send, d_back, cap, serial_base, b->call_new, b->new_pairs,
		                                 b->new_pairs ? b->new_pairs_cap : 0, bc);
		SYZ_HIP(hipGetLastError());
	} else {
		// per-record bits need the pairs' count on the host: this call synchronises
		unsigned long long* hb = ctx->h_step + kStepBack;
		SYZ_HIP(hipMemcpyAsync(hb, bc, kNumCounters * 8, hipMemcpyDeviceToHost, s));
		SYZ_HIP(hipStreamSynchronize(s));
		const uint64_t np0 = hb[kCntAux2], bound = np0 + (uint64_t)nshards * cap;
		void* wp;
		SYZ_TRY(ws_grow_keep(ctx, 55, bound * 8 + 64, np0 * 8, &wp));
		k_step_back<<<grid, 256, 0, s>>>(d_send, d_back, cap, serial_base, b->call_new, (uint64_t*)wp, bound, bc);
		SYZ_HIP(hipGetLastError());
		SYZ_HIP(hipMemcpyAsync(hb, bc, kNumCounters * 8, hipMemcpyDeviceToHost, s));
		SYZ_HIP(hipStreamSynchronize(s));
		const uint64_t np1 = hb[kCntAux2];
		SYZ_TRY(agg_mark_bits(ctx, b, 0, b->ncalls, (const uint64_t*)wp, np0, np1));
		if (b->new_pairs && np1 > np0 && np0 < b->new_pairs_cap)
			SYZ_HIP(hipMemcpyAsync(b->new_pairs + np0, (const uint64_t*)wp + np0,
			                       (std::min(np1, b->new_pairs_cap) - np0) * 8, hipMemcpyDeviceToDevice, s));
	}
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev_step[5], s));
	return SYZSIG_OK;
}

}  // extern "C"
