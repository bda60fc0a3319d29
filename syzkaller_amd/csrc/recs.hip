// recs.hip -- records-mode triage through LDS: the owner side of a sharded
// step (syzsig_step_own_dev) and syzsig_triage_records_dev on large inputs.
//
// A record is e << 32 | level << 24 | serial (serial = the call's position in
// the batch's global serial order).  checkNewSignal over the records
// (syz-fuzzer/fuzzer.go:494-511, DiffRaw + Merge per call in serial order) is,
// per element e independently: walk e's records in serial order from
// m = M0[e]; a record is new iff its prio exceeds m (then m rises), or it
// repeats the last new record's serial (DiffRaw collapses duplicates inside a
// call, signal.go:90-102); the final m, if it rose, is merged into the shard
// and newSignal (signal.go:117-131).
//
// So the records only need grouping by element (not even ordering: see
// k_rp_agg).  Instead of a device-wide sort:
//   k_rp_count    tiles of the record buffer: per partition counts, where the
//                 partition is the top pbits of h = fmix32(e) -- the shard's
//                 home-bucket bits, so one partition probes one slice of it
//   k_rp_colsum / k_rp_scan / k_rp_coloffs
//                 each (tile, partition) cell's place: partitions contiguous,
//                 tiles in order inside one; a partition over kRpCap records
//                 voids the run (the gate) before anything is committed
//   k_rp_scatter  key = h_residual << 39 | serial << 15 | level << 13 | local
//                 position, and the record's buffer index beside it
//   k_rp_agg / k_rp_elems / k_rp_flags
//                 per partition an LDS hash of its elements with their level
//                 firsts; per element one shard probe and the merges; per
//                 record its flag in closed form (no ordering: see k_rp_agg).
// No device-scope atomics per record (those run at ~20 G/s chip-wide).
#include <algorithm>
#include <vector>

#include "internal.h"

namespace syz {

constexpr uint32_t kRpCap = 2048;       // records of one partition in LDS (local positions < 2^13)
constexpr uint32_t kRpTarget = 1024;    // partitions are sized for this mean
constexpr uint32_t kRpMinBits = 7;      // h residuals of <= 25 bits fit the key
constexpr uint32_t kRpMaxBits = 13;     // <= 32 KB of LDS counters per tile
constexpr uint32_t kRpTileMin = 16384;  // slots per counting / scatter tile (more for big inputs: <= ~1024 tiles)
constexpr uint32_t kRpTileThreads = 512;
constexpr uint32_t kRpGroups = 16;      // tile groups of the column scans
constexpr uint32_t kRpThreads = 256;    // k_rp_agg: 8 records per thread
constexpr uint64_t kRpPosMask = 8191;    // the key's 13 position bits

// Where the records are: segment g's cnt[g] records at recs[g * stride + hdr ...].
struct RpSrc {
	const uint64_t* recs;
	uint64_t stride;
	uint32_t hdr, nseg;
	const uint64_t* cnt;  // device, nseg entries
	uint32_t tiles_per_seg;
	uint32_t tile;        // slots per tile
};

// gate bits (ctr[kCntSpill]): 1 = a source bucket was void or over cap,
// 2 = a partition over kRpCap, 4 = a record's level out of range
__device__ __forceinline__ bool rp_gated(const unsigned long long* ctr) { return ctr[kCntSpill] != 0; }

__device__ __forceinline__ uint32_t rp_part(uint64_t r, uint32_t pbits) { return fmix32((uint32_t)(r >> 32)) >> (32 - pbits); }

// tile t of the source: slots [off, off + kRpTile) of segment g, valid while < cnt
__device__ __forceinline__ void rp_tile(const RpSrc& s, uint32_t t, uint32_t& g, uint64_t& j0, uint64_t& n)
{
	g = t / s.tiles_per_seg;
	j0 = (uint64_t)(t % s.tiles_per_seg) * s.tile;
	const uint64_t c = s.cnt[g];
	n = j0 < c ? min<uint64_t>(s.tile, c - j0) : 0;
}

__global__ __launch_bounds__(kRpTileThreads) void k_rp_count(RpSrc s, uint32_t pbits, uint32_t nlev, uint32_t* cnt,
                                                             unsigned long long* ctr)
{
	extern __shared__ uint32_t h[];  // P counters
	if (rp_gated(ctr))
		return;
	const uint32_t P = 1u << pbits;
	for (uint32_t p = threadIdx.x; p < P; p += blockDim.x)
		h[p] = 0;
	__syncthreads();
	uint32_t g;
	uint64_t j0, n;
	rp_tile(s, blockIdx.x, g, j0, n);
	const uint64_t* r = s.recs + g * s.stride + s.hdr + j0;
	uint32_t bad = 0;
	for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
		const uint64_t x = r[k];
		bad |= ((x >> 24) & 0xff) >= nlev;
		atomicAdd(&h[rp_part(x, pbits)], 1u);
	}
	__syncthreads();
	uint32_t* row = cnt + (uint64_t)blockIdx.x * P;
	for (uint32_t p = threadIdx.x; p < P; p += blockDim.x)
		row[p] = h[p];
	if (__ballot(bad) && lane_id() == 0)
		atomicOr(&ctr[kCntSpill], 4ull);
}

// per partition: its records over all tiles.  Block = 64 partitions x
// kRpGroups groups of consecutive tiles (loads coalesced across partitions);
// gsum[grp][p] keeps each group's part for k_rp_coloffs.
__global__ __launch_bounds__(1024) void k_rp_colsum(const uint32_t* __restrict__ cnt, uint32_t ntiles, uint32_t P,
                                                    uint32_t* gsum, uint32_t* tot, const unsigned long long* ctr)
{
	__shared__ uint32_t part[kRpGroups][64];
	if (rp_gated(ctr))
		return;
	const uint32_t pl = threadIdx.x & 63, grp = threadIdx.x >> 6, p = blockIdx.x * 64 + pl;
	const uint32_t per = (ntiles + kRpGroups - 1) / kRpGroups, t0 = grp * per, t1 = min(ntiles, t0 + per);
	uint32_t sum = 0;
	if (p < P) {
#pragma unroll 8
		for (uint32_t t = t0; t < t1; t++)
			sum += cnt[(uint64_t)t * P + p];
		gsum[(uint64_t)grp * P + p] = sum;
	}
	part[grp][pl] = sum;
	__syncthreads();
	if (grp == 0 && p < P) {
		uint32_t t = 0;
		for (uint32_t k = 0; k < kRpGroups; k++)
			t += part[k][pl];
		tot[p] = t;
	}
}

// partition bases (exclusive scan of tot into base[0..P]); the gate when a
// partition has more than kRpCap records; records and the largest partition
__global__ __launch_bounds__(1024) void k_rp_scan(const uint32_t* __restrict__ tot, uint32_t P, uint32_t* base,
                                                  unsigned long long* ctr, uint32_t force_gate)
{
	__shared__ uint32_t part[1024];
	__shared__ uint32_t mx[1024];
	if (rp_gated(ctr))
		return;
	const uint32_t per = (P + 1023) / 1024, a = threadIdx.x * per, z = min(P, a + per);
	uint32_t s = 0, m = 0;
	for (uint32_t p = a; p < z; p++) {
		s += tot[p];
		m = max(m, tot[p]);
	}
	part[threadIdx.x] = s;
	mx[threadIdx.x] = m;
	__syncthreads();
	if (threadIdx.x == 0) {
		uint32_t run = 0, mm = 0;
		for (int k = 0; k < 1024; k++) {
			const uint32_t v = part[k];
			part[k] = run;
			run += v;
			mm = max(mm, mx[k]);
		}
		base[P] = run;
		ctr[kCntRecords] = run;
		ctr[kCntAux2] = mm;
		if (mm > kRpCap || force_gate)  // (force_gate: SYZSIG_DEBUG_RECS_GATE, tests)
			ctr[kCntSpill] |= 2ull;
	}
	__syncthreads();
	uint32_t run = part[threadIdx.x];
	for (uint32_t p = a; p < z; p++) {
		base[p] = run;
		run += tot[p];
	}
}

// cell offsets: off[t][p] = base[p] + records of p in tiles < t (in place)
__global__ __launch_bounds__(1024) void k_rp_coloffs(uint32_t* cnt, uint32_t ntiles, uint32_t P,
                                                     const uint32_t* __restrict__ gsum,
                                                     const uint32_t* __restrict__ base, const unsigned long long* ctr)
{
	if (rp_gated(ctr))
		return;
	const uint32_t pl = threadIdx.x & 63, grp = threadIdx.x >> 6, p = blockIdx.x * 64 + pl;
	if (p >= P)
		return;
	const uint32_t per = (ntiles + kRpGroups - 1) / kRpGroups, t0 = grp * per, t1 = min(ntiles, t0 + per);
	uint32_t run = base[p];
	for (uint32_t k = 0; k < grp; k++)
		run += gsum[(uint64_t)k * P + p];
	for (uint32_t t = t0; t < t1; t++) {
		const uint64_t o = (uint64_t)t * P + p;
		const uint32_t v = cnt[o];
		cnt[o] = run;
		run += v;
	}
}

__global__ __launch_bounds__(kRpTileThreads) void k_rp_scatter(RpSrc s, uint32_t pbits,
                                                               const uint32_t* __restrict__ off,
                                                               const uint32_t* __restrict__ base, uint64_t* keys,
                                                               uint32_t* idx, const unsigned long long* ctr)
{
	extern __shared__ uint32_t cur[];  // P cursors
	if (rp_gated(ctr))
		return;
	const uint32_t P = 1u << pbits;
	const uint32_t* row = off + (uint64_t)blockIdx.x * P;
	for (uint32_t p = threadIdx.x; p < P; p += blockDim.x)
		cur[p] = row[p];
	__syncthreads();
	uint32_t g;
	uint64_t j0, n;
	rp_tile(s, blockIdx.x, g, j0, n);
	const uint64_t slot0 = g * s.stride + s.hdr + j0;
	const uint64_t* r = s.recs + slot0;
	const uint32_t rmask = pbits >= 32 ? 0u : (uint32_t)((1ull << (32 - pbits)) - 1);
	for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
		const uint64_t x = r[k];
		const uint32_t h = fmix32((uint32_t)(x >> 32)), p = h >> (32 - pbits);
		const uint32_t pos = atomicAdd(&cur[p], 1u);
		const uint64_t local = (pos - base[p]) & kRpPosMask;  // < kRpCap: the gate holds
		keys[pos] = ((uint64_t)(h & rmask) << 39) | ((x & kSerialMask) << 15) | (((x >> 24) & 3) << 13) | local;
		idx[pos] = (uint32_t)(slot0 + k);
	}
}

struct RpTables {
	uint64_t *ms, ms_bmask, *ns, ns_bmask;
};

// Element e's records need no ordering.  With first[l] = the smallest serial
// among e's records at level l, replaying checkNewSignal over them in serial
// order from m = M0[e] flags record (s, l) exactly when
//     prio(l) > M0[e]  and  first[l] == s  and  first[l'] > s for every l' > l
// (m before serial s is the max of M0 and the prios of the serials before s,
// and a serial is one call, so one level; duplicates of an element in one call
// share (s, l) and are flagged together, as DiffRaw collapses them), and the
// final prio is max(M0[e], the top level present).  So the owner side is the
// K3 aggregation again, without its scatter pass (the records arrive grouped
// by partition from k_rp_scatter), in three kernels:
//   k_rp_agg    one workgroup per partition: an LDS hash of its elements (the h
//               residual) with the level firsts (ds_min), its distinct
//               elements written out at the partition's own offset (no
//               allocation atomics: a partition has at most as many elements
//               as records), and every record's element index;
//   k_rp_elems  one thread per element, thousands in flight (the dependent
//               shard probe and merges are latency chains that a
//               partition-resident workgroup could only overlap ~80 at a time):
//               M0[e], the merges, M0 kept for the flags;
//   k_rp_flags  one thread per record: the closed form above.
constexpr uint32_t kRpEmpty = 0xFFFFFFFFu;
constexpr int16_t kRpAbsent = -32768;  // elem_m0 of an element absent from the shard

struct RpElems {
	uint32_t* e;      // element
	uint4* f;         // level firsts (kSerialMask + 1 = none)
	int16_t* m0;      // M0[e] (kRpAbsent: absent)
	uint32_t* rec_el; // per partitioned record: its element's index
	uint32_t* ecnt;   // per partition: elements
};

struct RpAggLds {
	uint32_t key[kRpCap];
	uint32_t fl[4][kRpCap];
	uint16_t rank[kRpCap];
	uint32_t wsum[kRpThreads / 64];
};
static_assert(sizeof(RpAggLds) <= 160 * 1024 / 3 - 64, "three workgroups per CU");

__global__ __launch_bounds__(kRpThreads) void k_rp_agg(const uint64_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ base, uint32_t pbits, RpElems el,
                                                       const unsigned long long* ctr)
{
	__shared__ RpAggLds L;
	if (rp_gated(ctr))
		return;
	constexpr uint32_t kPer = kRpCap / kRpThreads;
	const uint32_t p = blockIdx.x, tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
	const uint32_t b0 = base[p], n = base[p + 1] - b0;
	for (uint32_t i = tid; i < kRpCap; i += kRpThreads) {
		L.key[i] = kRpEmpty;
		L.fl[0][i] = L.fl[1][i] = L.fl[2][i] = L.fl[3][i] = kSerialMask + 1;
	}
	__syncthreads();
	uint32_t sl[kPer];
#pragma unroll
	for (uint32_t k = 0; k < kPer; k++) {
		const uint32_t i = k * kRpThreads + tid;
		sl[k] = 0;
		if (i < n) {
			const uint64_t x = keys[b0 + i];
			const uint32_t hr = (uint32_t)(x >> 39);
			// linear probing (h is already mixed; the residual's width depends
			// on pbits, so its low bits); never full: n <= kRpCap
			uint32_t s0 = hr & (kRpCap - 1);
			for (;;) {
				const uint32_t cur = L.key[s0];
				if (cur == hr)
					break;
				if (cur == kRpEmpty) {
					const uint32_t old = atomicCAS(&L.key[s0], kRpEmpty, hr);
					if (old == kRpEmpty || old == hr)
						break;
				}
				s0 = (s0 + 1) & (kRpCap - 1);
			}
			atomicMin(&L.fl[(x >> 13) & 3][s0], (uint32_t)(x >> 15) & kSerialMask);
			sl[k] = s0;
		}
	}
	__syncthreads();
	// the occupied slots' ranks: thread t owns slots [t * kPer, t * kPer + kPer)
	uint32_t occ = 0;
#pragma unroll
	for (uint32_t k = 0; k < kPer; k++)
		occ |= (uint32_t)(L.key[tid * kPer + k] != kRpEmpty) << k;
	const uint32_t c = (uint32_t)__popc(occ);
	uint32_t inc = c;
#pragma unroll
	for (uint32_t d = 1; d < 64; d <<= 1) {
		const uint32_t t = __shfl_up(inc, d, 64);
		inc += lane >= d ? t : 0;
	}
	if (lane == 63)
		L.wsum[w] = inc;
	__syncthreads();
	uint32_t r = inc - c, tot = 0;
	for (uint32_t k = 0; k < kRpThreads / 64; k++) {
		r += k < w ? L.wsum[k] : 0;
		tot += L.wsum[k];
	}
	const uint32_t hp = p << (32 - pbits);
#pragma unroll
	for (uint32_t k = 0; k < kPer; k++) {
		if ((occ >> k) & 1) {
			const uint32_t s0 = tid * kPer + k;
			L.rank[s0] = (uint16_t)r;
			el.e[b0 + r] = fmix32_inv(hp | L.key[s0]);
			el.f[b0 + r] = make_uint4(L.fl[0][s0], L.fl[1][s0], L.fl[2][s0], L.fl[3][s0]);
			r++;
		}
	}
	if (tid == 0)
		el.ecnt[p] = tot;
	__syncthreads();
#pragma unroll
	for (uint32_t k = 0; k < kPer; k++) {
		const uint32_t i = k * kRpThreads + tid;
		if (i < n)
			el.rec_el[b0 + i] = b0 + L.rank[sl[k]];
	}
}

// the per-partition counts of k_rp_elems (written by each workgroup, summed
// by k_rp_reduce: a device atomic per workgroup and counter on five shared
// addresses serialises thousands of workgroups)
constexpr uint32_t kRpNumCnt = 5;
constexpr int kRpCntIdx[kRpNumCnt] = {kCntInserted, kCntChanged, kCntAux, kCntOverflow, kCntDistinct};
constexpr uint32_t kRpElemThreads = 128;

__global__ __launch_bounds__(kRpElemThreads) void k_rp_elems(const uint32_t* __restrict__ base, LevelMap lm,
                                                             RpTables tb, RpElems el, const unsigned long long* ctr,
                                                             uint32_t* sums)
{
	__shared__ uint32_t part[kRpNumCnt][kRpElemThreads / 64];
	if (rp_gated(ctr))
		return;
	const uint32_t p = blockIdx.x, b0 = base[p], ne = el.ecnt[p];
	uint32_t inserted = 0, changed = 0, ns_ins = 0, ovf = 0;
	for (uint32_t j = threadIdx.x; j < ne; j += kRpElemThreads) {
		const uint32_t i = b0 + j, e = el.e[i];
		const Bucket bm = load_bucket(tb.ms + (home_bucket(e, tb.ms_bmask) << kBucketShift));
		const Bucket bn = load_bucket(tb.ns + (home_bucket(e, tb.ns_bmask) << kBucketShift));
		const uint4 f4 = el.f[i];
		const int top = f4.w <= kSerialMask ? 3 : f4.z <= kSerialMask ? 2 : f4.y <= kSerialMask ? 1 : 0;
		uint64_t v = 0;
		const int64_t at = tbl_lookup_from(tb.ms, tb.ms_bmask, e, v, bm);
		const bool present = at >= 0 && slot_live(v);
		const int m0 = present ? (int)slot_prio(v) : -1000;  // absent: below every prio (signal.go:93-95)
		el.m0[i] = present ? (int16_t)m0 : kRpAbsent;
		const int m = max(m0, (int)lm.val[top]);
		if (m > m0) {  // maxSignal.Merge / newSignal.Merge of the element's final prio
			changed++;
			inserted += !present;
			if (at >= 0)
				tb.ms[at] = make_slot(e, (int8_t)m);  // e's only writer this launch
			else
				ovf += tbl_merge(tb.ms, tb.ms_bmask, e, (int8_t)m) < 0;
			const int r = tbl_merge_from(tb.ns, tb.ns_bmask, e, (int8_t)m, bn);
			ns_ins += r == 1;
			ovf += r < 0;
		}
	}
	const uint32_t v[kRpNumCnt] = {inserted, changed, ns_ins, ovf, 0};
	const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
	for (uint32_t k = 0; k < kRpNumCnt; k++) {
		const uint32_t s = (uint32_t)wave_sum_u64(v[k]);
		if (lane == 0)
			part[k][w] = s;
	}
	__syncthreads();
	if (threadIdx.x < kRpNumCnt) {
		uint32_t t = 0;
		for (uint32_t q = 0; q < kRpElemThreads / 64; q++)
			t += part[threadIdx.x][q];
		sums[(uint64_t)p * kRpNumCnt + threadIdx.x] = threadIdx.x == 4 ? ne : t;
	}
}

__global__ __launch_bounds__(1024) void k_rp_reduce(const uint32_t* __restrict__ sums, uint32_t P,
                                                    unsigned long long* ctr)
{
	if (rp_gated(ctr))
		return;
	__shared__ unsigned long long acc[kRpNumCnt];
	if (threadIdx.x < kRpNumCnt)
		acc[threadIdx.x] = 0;
	__syncthreads();
	uint64_t v[kRpNumCnt] = {0, 0, 0, 0, 0};
	for (uint32_t p = threadIdx.x; p < P; p += blockDim.x)
#pragma unroll
		for (uint32_t k = 0; k < kRpNumCnt; k++)
			v[k] += sums[(uint64_t)p * kRpNumCnt + k];
#pragma unroll
	for (uint32_t k = 0; k < kRpNumCnt; k++) {
		const uint64_t s = wave_sum_u64(v[k]);
		if (lane_id() == 0 && s)
			atomicAdd(&acc[k], (unsigned long long)s);
	}
	__syncthreads();
	if (threadIdx.x < kRpNumCnt)
		ctr[kRpCntIdx[threadIdx.x]] += acc[threadIdx.x];
}

// one thread per partitioned record: the flag in closed form
__global__ __launch_bounds__(256) void k_rp_flags(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ idx,
                                                  const uint32_t* __restrict__ base, uint32_t P, LevelMap lm,
                                                  RpElems el, uint8_t* flags, const unsigned long long* ctr)
{
	if (rp_gated(ctr))
		return;
	const uint32_t n = base[P];
	for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
		const uint64_t x = keys[i];
		const uint32_t k = el.rec_el[i];
		const int16_t m0 = el.m0[k];
		const uint32_t lv = (uint32_t)(x >> 13) & 3, ser = (uint32_t)(x >> 15) & kSerialMask;
		if ((int)lm.val[lv] <= (m0 == kRpAbsent ? -1000 : (int)m0))
			continue;
		const uint4 f4 = el.f[k];
		const uint32_t f[4] = {f4.x, f4.y, f4.z, f4.w};
		bool nw = f[lv] == ser;
#pragma unroll
		for (uint32_t l = 0; l < 4; l++)
			nw = nw && !(l > lv && f[l] <= ser);
		if (nw)
			flags[idx[i]] = 1;
	}
}

// ---- the step's owner glue ----
// Headers of the received buckets -> per-segment record counts (capped),
// the gate when a source bucket is void or over cap, records and the largest
// bucket.  The run's counters are zeroed here.
__global__ void k_step_heads(const uint64_t* __restrict__ recv, uint32_t nshards, uint64_t cap, uint64_t* seg_cnt,
                             unsigned long long* ctr)
{
	if (threadIdx.x < kNumCounters)
		ctr[threadIdx.x] = 0;
	__syncthreads();
	if (threadIdx.x == 0) {
		uint64_t tot = 0, mx = 0, gate = 0;
		for (uint32_t g = 0; g < nshards; g++) {
			const uint64_t hd = recv[(uint64_t)g * (cap + 1)];
			const uint64_t c = hd & SYZSIG_STEP_HDR_COUNT;
			gate |= (hd & (SYZSIG_STEP_HDR_VOID | SYZSIG_STEP_HDR_OVF)) != 0 || c > cap;
			seg_cnt[g] = min(c, cap);
			tot += min(c, cap);
			mx = max(mx, c);
		}
		ctr[kCntSpill] = gate;
		ctr[kCntCandidates] = tot;
		ctr[kCntTouched] = mx;
	}
}

// the owner's status into byte 0 of every flags bucket: 0 = triaged,
// 1 = skipped (a void bucket somewhere: the whole step is void), 2 = skipped
// (this owner's own overflow)
__global__ void k_step_status(uint8_t* flags, uint32_t nshards, uint64_t cap, const unsigned long long* ctr)
{
	const uint64_t gt = ctr[kCntSpill];
	const uint8_t st = gt == 0 ? 0 : (gt & 1) ? 1 : 2;
	for (uint32_t g = threadIdx.x; g < nshards; g += blockDim.x)
		flags[(uint64_t)g * (cap + 1)] = st;
}

// valid records of the buckets, compacted (exact path), with their slots
__global__ void k_step_compact(const uint64_t* __restrict__ recv, uint32_t nshards, uint64_t cap,
                               const uint64_t* __restrict__ seg_cnt, const uint64_t* __restrict__ seg_off,
                               uint64_t* out, uint64_t* slot)
{
	const uint32_t g = blockIdx.y;
	const uint64_t c = seg_cnt[g], o = seg_off[g], s0 = (uint64_t)g * (cap + 1) + 1;
	for (uint64_t j = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; j < c; j += (uint64_t)gridDim.x * blockDim.x) {
		out[o + j] = recv[s0 + j];
		slot[o + j] = s0 + j;
	}
}

__global__ void k_step_uncompact(const uint8_t* __restrict__ f, const uint64_t* __restrict__ slot, uint64_t n,
                                 uint8_t* flags)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
		flags[slot[i]] = f[i];
}

// Partition bits for at most `bound` records: mean <= kRpTarget.
static uint32_t rp_pbits(uint64_t bound)
{
	uint32_t pb = kRpMinBits;
	while (pb < kRpMaxBits && (bound >> pb) > kRpTarget)
		pb++;
	return pb;
}

// One LDS-partitioned records run over src (at most `bound` records), gated
// and counted through ctr (the caller zeroed it or k_step_heads did).  Enqueues
// only; the caller reads ctr after its synchronisation.  The shard and
// newSignal must have room for `bound` more elements.
int rp_run(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set* nsp, const RpSrc& src0, uint64_t bound, const LevelMap& lm,
           uint8_t* flags, unsigned long long* ctr, uint32_t* pbits_out)
{
	RpSrc src = src0;
	const uint64_t seg_slots = src.stride - src.hdr;
	const uint64_t slots = seg_slots * src.nseg;
	// about <= 1024 tiles: the tile x partition count matrix stays small
	const uint64_t tile = std::max<uint64_t>(kRpTileMin, (slots / 1024 + 4095) & ~4095ull);
	if (tile >= (1ull << 31) || bound >= (1ull << 32))
		return fail(SYZSIG_ERANGE, "records: too many records for the LDS path");
	src.tile = (uint32_t)tile;
	src.tiles_per_seg = (uint32_t)std::max<uint64_t>(1, (seg_slots + tile - 1) / tile);
	const uint64_t ntiles = (uint64_t)src.tiles_per_seg * src.nseg;
	const uint32_t pbits = rp_pbits(bound), P = 1u << pbits;
	*pbits_out = pbits;
	void *wk, *wc, *wb;
	// per bound record: key 8 + index 4 + its element's index 4 + (as elements)
	// element 4 + firsts 16 + M0 2
	const uint64_t nb = (bound + 3) & ~3ull;  // array strides: the firsts stay 16-B aligned
	SYZ_TRY(ws_get(ctx, 56, nb * 38 + 1024, &wk));
	SYZ_TRY(ws_get(ctx, 57, ntiles * P * 4 + 256, &wc));
	SYZ_TRY(ws_get(ctx, 58, (uint64_t)(kRpGroups + 3 + kRpNumCnt) * P * 4 + 256, &wb));
	uint64_t* keys = (uint64_t*)wk;
	uint4* ef = (uint4*)(keys + nb);
	uint32_t* idx = (uint32_t*)(ef + nb);
	RpElems el;
	el.f = ef;
	el.rec_el = idx + nb;
	el.e = el.rec_el + nb;
	el.m0 = (int16_t*)(el.e + nb);
	uint32_t* cnt = (uint32_t*)wc;
	uint32_t* tot = (uint32_t*)wb;
	uint32_t* base = tot + P;               // P + 1 entries
	uint32_t* gsum = base + P + 2;          // kRpGroups x P
	uint32_t* sums = gsum + (uint64_t)kRpGroups * P;  // kRpNumCnt per partition
	el.ecnt = sums + (uint64_t)kRpNumCnt * P;
	const hipStream_t s = ctx->stream;
	const uint32_t cg = (P + 63) / 64;
	k_rp_count<<<(uint32_t)ntiles, kRpTileThreads, P * 4, s>>>(src, pbits, lm.n, cnt, ctr);
	k_rp_colsum<<<cg, 1024, 0, s>>>(cnt, (uint32_t)ntiles, P, gsum, tot, ctr);
	k_rp_scan<<<1, 1024, 0, s>>>(tot, P, base, ctr, ctx->agg_dbg & SYZSIG_DEBUG_RECS_GATE);
	k_rp_coloffs<<<cg, 1024, 0, s>>>(cnt, (uint32_t)ntiles, P, gsum, base, ctr);
	k_rp_scatter<<<(uint32_t)ntiles, kRpTileThreads, P * 4, s>>>(src, pbits, cnt, base, keys, idx, ctr);
	const RpTables tb{ms->slots, ms->nbuckets - 1, nsp->slots, nsp->nbuckets - 1};
	k_rp_agg<<<P, kRpThreads, 0, s>>>(keys, base, pbits, el, ctr);
	k_rp_elems<<<P, kRpElemThreads, 0, s>>>(base, lm, tb, el, ctr, sums);
	k_rp_reduce<<<1, 1024, 0, s>>>(sums, P, ctr);
	k_rp_flags<<<grid_for(bound, 256, 8192), 256, 0, s>>>(keys, idx, base, P, lm, el, flags, ctr);
	SYZ_HIP(hipGetLastError());
	return SYZSIG_OK;
}

}  // namespace syz

namespace syz {

// Poll's grouping (rp_group): key = h_residual << 32 | the entry's index
__global__ __launch_bounds__(kRpTileThreads) void k_rp_scatter_idx(RpSrc s, uint32_t pbits,
                                                                   const uint32_t* __restrict__ off,
                                                                   uint64_t* keys, const unsigned long long* ctr)
{
	extern __shared__ uint32_t cur[];  // P cursors
	if (rp_gated(ctr))
		return;
	const uint32_t P = 1u << pbits;
	const uint32_t* row = off + (uint64_t)blockIdx.x * P;
	for (uint32_t p = threadIdx.x; p < P; p += blockDim.x)
		cur[p] = row[p];
	__syncthreads();
	uint32_t g;
	uint64_t j0, n;
	rp_tile(s, blockIdx.x, g, j0, n);
	const uint64_t* r = s.recs + g * s.stride + s.hdr + j0;
	const uint32_t rmask = (uint32_t)((1ull << (32 - pbits)) - 1);
	for (uint32_t k = threadIdx.x; k < n; k += blockDim.x) {
		const uint64_t x = r[k];
		const uint32_t h = fmix32((uint32_t)(x >> 32)), p = h >> (32 - pbits);
		keys[atomicAdd(&cur[p], 1u)] = ((uint64_t)(h & rmask) << 32) | (uint32_t)x;
	}
}

__global__ void k_rp_one_seg(uint64_t* seg, uint64_t n, unsigned long long* ctr)
{
	if (threadIdx.x < kNumCounters)
		ctr[threadIdx.x] = 0;
	if (threadIdx.x == 0)
		seg[0] = n;
}

static_assert(kRpGroupCap == kRpCap, "internal.h mirror");

int rp_group(syzsig_ctx* ctx, const uint64_t* x, uint64_t n, uint64_t** keys_out, uint32_t** base_out,
             uint32_t* pbits_out, unsigned long long* ctr)
{
	if (n >= (1ull << 32))
		return fail(SYZSIG_ERANGE, "group: 2^32 entries or more");
	void *wseg, *wk, *wc, *wb;
	SYZ_TRY(ws_get(ctx, 48, 64, &wseg));
	RpSrc src{x, n, 0, 1, (const uint64_t*)wseg, 0, 0};
	const uint64_t tile = std::max<uint64_t>(kRpTileMin, (n / 1024 + 4095) & ~4095ull);
	src.tile = (uint32_t)tile;
	src.tiles_per_seg = (uint32_t)std::max<uint64_t>(1, (n + tile - 1) / tile);
	const uint64_t ntiles = src.tiles_per_seg;
	const uint32_t pbits = rp_pbits(n), P = 1u << pbits;
	SYZ_TRY(ws_get(ctx, 49, n * 8 + 64, &wk));
	SYZ_TRY(ws_get(ctx, 50, ntiles * P * 4 + 256, &wc));
	SYZ_TRY(ws_get(ctx, 51, (uint64_t)(kRpGroups + 3) * P * 4 + 256, &wb));
	uint32_t* cnt = (uint32_t*)wc;
	uint32_t* tot = (uint32_t*)wb;
	uint32_t* base = tot + P;       // P + 1 entries
	uint32_t* gsum = base + P + 2;  // kRpGroups x P
	const hipStream_t s = ctx->stream;
	const uint32_t cg = (P + 63) / 64;
	k_rp_one_seg<<<1, 64, 0, s>>>((uint64_t*)wseg, n, ctr);
	k_rp_count<<<(uint32_t)ntiles, kRpTileThreads, P * 4, s>>>(src, pbits, 256, cnt, ctr);
	k_rp_colsum<<<cg, 1024, 0, s>>>(cnt, (uint32_t)ntiles, P, gsum, tot, ctr);
	k_rp_scan<<<1, 1024, 0, s>>>(tot, P, base, ctr, ctx->agg_dbg & SYZSIG_DEBUG_RECS_GATE);
	k_rp_coloffs<<<cg, 1024, 0, s>>>(cnt, (uint32_t)ntiles, P, gsum, base, ctr);
	k_rp_scatter_idx<<<(uint32_t)ntiles, kRpTileThreads, P * 4, s>>>(src, pbits, cnt, (uint64_t*)wk, ctr);
	SYZ_HIP(hipGetLastError());
	*keys_out = (uint64_t*)wk;
	*base_out = base;
	*pbits_out = pbits;
	return SYZSIG_OK;
}

int rp_triage_records(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const uint64_t* recs, uint64_t nrec,
                      const LevelMap& lm, uint8_t* new_flags, syzsig_batch_stats* st, bool* done)
{
	*done = false;
	// room for every record's element changing, before anything is committed
	SYZ_TRY(set_reserve(ms, nrec));
	const bool fresh_ns = !*ns;
	if (fresh_ns)
		SYZ_TRY(syzsig_set_make(ctx, nrec, ns));  // newSignal.Merge allocates a nil receiver (signal.go:121-125)
	syzsig_set* nsp = *ns;
	SYZ_TRY(set_reserve_load(nsp, nrec, kHardLoad));
	void* ws;
	SYZ_TRY(ws_get(ctx, 59, 64, &ws));
	const hipStream_t s = ctx->stream;
	k_rp_one_seg<<<1, 64, 0, s>>>((uint64_t*)ws, nrec, ctx->d_cnt);
	const RpSrc src{recs, nrec, 0, 1, (const uint64_t*)ws, 0, 0};
	uint32_t pbits = 0;
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[2], s));
	SYZ_TRY(rp_run(ctx, ms, nsp, src, nrec, lm, new_flags, ctx->d_cnt, &pbits));
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[3], s));
	SYZ_TRY(counters_fetch(ctx));
	const uint64_t gate = ctx->h_cnt[kCntSpill];
	if (gate & 4)
		return fail(SYZSIG_EINVAL, "triage_records: a record's prio level is out of range");
	if (gate) {  // a partition past the LDS capacity: nothing was committed
		if (fresh_ns) {
			syzsig_set_free(nsp);
			*ns = nullptr;
		}
		return SYZSIG_OK;
	}
	if (ctx->h_cnt[kCntOverflow])
		return fail(SYZSIG_EIO, "triage_records: table overflow after reserve (internal error)");
	if (ctx->timing) {
		float t = 0;
		SYZ_HIP(hipEventElapsedTime(&t, ctx->ev[2], ctx->ev[3]));
		st->decide_ms += t;
	}
	const uint64_t changed = ctx->h_cnt[kCntChanged];
	ms->len += ctx->h_cnt[kCntInserted];
	nsp->len += ctx->h_cnt[kCntAux];
	if (fresh_ns && changed == 0) {
		syzsig_set_free(nsp);
		*ns = nullptr;
	}
	st->inserted += ctx->h_cnt[kCntInserted];
	st->changed += changed;
	st->candidates += changed;
	st->distinct += ctx->h_cnt[kCntDistinct];
	st->survivors += ctx->h_cnt[kCntDistinct];
	st->parts = 1ull << pbits;
	st->runs++;
	*done = true;
	return SYZSIG_OK;
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzsig_step_own_dev(syzsig_ctx* ctx, syzsig_set* shard, syzsig_set* new_signal, const uint64_t* d_recv,
                        uint32_t nshards, uint64_t cap, const int8_t* levels, uint32_t nlevels, uint8_t* d_flags,
                        int exact)
{
	SYZ_LOCK(ctx);
	if (!ctx || !shard || !new_signal || !d_recv || !d_flags)
		return fail(SYZSIG_EINVAL, "step_own: NULL argument");
	if (shard == new_signal)
		return fail(SYZSIG_EINVAL, "step_own: new_signal aliases the shard");
	if (nshards == 0 || nshards > 64 || cap == 0 || cap > SYZSIG_STEP_HDR_COUNT)
		return fail(SYZSIG_EINVAL, "step_own: need 1 <= nshards <= 64 and 1 <= cap < 2^40");
	if ((ctx->step_ms && ctx->step_ms != shard) || (ctx->step_ns && ctx->step_ns != new_signal))
		return fail(SYZSIG_EINVAL, "step_own: another owner step is in flight (syzsig_step_finish first)");
	LevelMap lm;
	SYZ_TRY(level_map_from_levels(levels, nlevels, &lm));
	const uint64_t stride = cap + 1, bound = (uint64_t)nshards * cap;
	if ((uint64_t)nshards * stride >= (1ull << 32))
		return fail(SYZSIG_ERANGE, "step_own: buckets of 2^32 words or more");
	// room for every received record's element changing (a growth syncs; the
	// step's caps change rarely, so this is rare)
	SYZ_TRY(set_reserve(shard, bound));
	SYZ_TRY(set_reserve_load(new_signal, bound, kHardLoad));
	const hipStream_t s = ctx->stream;
	unsigned long long* oc = ctx->d_step + kStepOwn;
	void* wsg;
	SYZ_TRY(ws_get(ctx, 60, (uint64_t)nshards * 16 + 64, &wsg));
	uint64_t* seg_cnt = (uint64_t*)wsg;
	uint64_t* seg_off = seg_cnt + nshards;
	ctx->step_own_timed = ctx->timing;
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev_step[2], s));
	SYZ_HIP(hipMemsetAsync(d_flags, 0, (uint64_t)nshards * stride, s));
	k_step_heads<<<1, 64, 0, s>>>(d_recv, nshards, cap, seg_cnt, oc);
	SYZ_HIP(hipGetLastError());
	shard->step_busy = new_signal->step_busy = true;
	ctx->step_ms = shard;
	ctx->step_ns = new_signal;
	// on an error past this point the sets are released again (no finish will
	// come for this step)
	const int rc = [&]() -> int {
		if (!exact) {
			const RpSrc src{d_recv, stride, 1, nshards, seg_cnt, 0, 0};
			uint32_t pbits = 0;
			SYZ_TRY(rp_run(ctx, shard, new_signal, src, bound, lm, d_flags, oc, &pbits));
			ctx->step_parts = 1ull << pbits;
		} else {
			// the per-record path over this owner's records, compacted (host round trips)
			ctx->step_parts = 0;
			unsigned long long* hc = ctx->h_step + kStepOwn;
			SYZ_HIP(hipMemcpyAsync(hc, oc, kNumCounters * 8, hipMemcpyDeviceToHost, s));
			std::vector<uint64_t> cnt(nshards);
			SYZ_HIP(hipMemcpyAsync(cnt.data(), seg_cnt, nshards * 8, hipMemcpyDeviceToHost, s));
			SYZ_HIP(hipStreamSynchronize(s));
			const uint64_t gate = hc[kCntSpill];
			if (!gate) {
				std::vector<uint64_t> off(nshards);
				uint64_t n = 0;
				for (uint32_t g = 0; g < nshards; g++) {
					off[g] = n;
					n += cnt[g];
				}
				syzsig_batch_stats st;
				memset(&st, 0, sizeof(st));
				if (n) {
					void *wr, *wf;
					SYZ_TRY(ws_get(ctx, 61, n * 16 + 64, &wr));
					SYZ_TRY(ws_get(ctx, 62, n + 64, &wf));
					uint64_t* comp = (uint64_t*)wr;
					uint64_t* slot = comp + n;
					SYZ_HIP(hipMemcpyAsync(seg_off, off.data(), nshards * 8, hipMemcpyHostToDevice, s));
					k_step_compact<<<dim3(grid_for(n, 256, 1024), nshards), 256, 0, s>>>(d_recv, nshards, cap, seg_cnt,
					                                                                     seg_off, comp, slot);
					SYZ_HIP(hipGetLastError());
					syzsig_set* nsp = new_signal;
					SYZ_TRY(triage_records_impl(ctx, shard, &nsp, comp, n, levels, nlevels, (uint8_t*)wf, &st, false));
					k_step_uncompact<<<grid_for(n, 256, 8192), 256, 0, s>>>((const uint8_t*)wf, slot, n, d_flags);
					SYZ_HIP(hipGetLastError());
				}
				// the owner counters as the LDS path leaves them; the lengths are
				// already committed by the per-record path
				hc[kCntInserted] = 0;
				hc[kCntAux] = 0;
				hc[kCntChanged] = st.changed;
				hc[kCntDistinct] = st.distinct;
				hc[kCntRecords] = n;
				hc[kCntOverflow] = 0;
				SYZ_HIP(hipMemcpyAsync(oc, hc, kNumCounters * 8, hipMemcpyHostToDevice, s));
				SYZ_HIP(hipStreamSynchronize(s));
			}
		}
		k_step_status<<<1, 64, 0, s>>>(d_flags, nshards, cap, oc);
		SYZ_HIP(hipGetLastError());
		if (ctx->timing)
			SYZ_HIP(hipEventRecord(ctx->ev_step[3], s));
		return SYZSIG_OK;
	}();
	if (rc != SYZSIG_OK) {
		shard->step_busy = new_signal->step_busy = false;
		ctx->step_ms = ctx->step_ns = nullptr;
	}
	return rc;
}

int syzsig_step_finish(syzsig_ctx* ctx, syzsig_step_status* out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out)
		return fail(SYZSIG_EINVAL, "step_finish: NULL argument");
	const hipStream_t s = ctx->stream;
	SYZ_HIP(hipMemcpyAsync(ctx->h_step, ctx->d_step, kStepCounters * 8, hipMemcpyDeviceToHost, s));
	SYZ_HIP(hipStreamSynchronize(s));
	const unsigned long long* h = ctx->h_step;
	const unsigned long long *src = h + kStepSrc, *own = h + kStepOwn, *bk = h + kStepBack;
	memset(out, 0, sizeof(*out));
	// 2 only for a prio outside the levels (an error); a spill (1), a bad call
	// range or more records than assumed (4, k_cell_plan_fast) and LDS
	// overflows send the source to its exact path, which validates and sizes
	out->src_void = src[kCntSpill] & 2 ? 2 : src[kCntSpill] || src[kCntAggOvf] ? 1 : 0;
	if (src[kCntSpill] & 1)  // a capped cell spilled: more slack for the next runs (as agg_capped does)
		ctx->cap_sd = ctx->cap_sd * 2 > 24.0f ? 0.0f : ctx->cap_sd * 2;
	if (!(src[kCntSpill] & 6) && src[kCntAggOvf] && src[kCntRecords]) {
		// LDS partitions overflowed: the distinct-ratio guess was low; size the
		// next runs for at least what was seen (as the one-sync triage run does)
		const double P = (double)ctx->step_src_parts, novf = (double)src[kCntAggOvf];
		const double seen = novf * 2 >= P ? (double)src[kCntRecords]
		                                  : (double)src[kCntDistinct] + 2.0 * novf * kAggLimitRecs;
		ctx->agg_distinct_ratio = std::max(ctx->agg_distinct_ratio, seen / (double)src[kCntRecords]);
	}
	out->global_void = bk[kCntError] != 0;
	out->owners_void = out->global_void ? 0 : bk[kCntAux];
	out->records = src[kCntRecords];
	out->distinct = src[kCntDistinct];
	out->sent = src[kCntCandidates];
	out->max_out = src[kCntTouched];
	out->new_pairs = bk[kCntAux2];
	int rc = SYZSIG_OK;
	if (ctx->step_ms) {
		out->received = own[kCntCandidates];
		out->max_in = own[kCntTouched];
		out->own_parts = ctx->step_parts;
		if (!own[kCntSpill]) {
			out->own_distinct = own[kCntDistinct];
			out->inserted = own[kCntInserted];
			out->changed = own[kCntChanged];
			ctx->step_ms->len += own[kCntInserted];
			ctx->step_ns->len += own[kCntAux];
			if (own[kCntOverflow])
				rc = fail(SYZSIG_EIO, "step: table overflow after reserve (internal error)");
		}
		if ((double)ctx->step_ms->len > kMaxLoad * (double)ctx->step_ms->nslots() && rc == SYZSIG_OK)
			rc = set_rehash(ctx->step_ms, buckets_for(ctx->step_ms->len), false);
		ctx->step_ms->step_busy = ctx->step_ns->step_busy = false;
		ctx->step_ms = ctx->step_ns = nullptr;
		// the owner counters are consumed: a second finish must not commit them again
		memset(ctx->h_step + kStepOwn, 0, kNumCounters * 8);
		SYZ_HIP(hipMemcpyAsync(ctx->d_step + kStepOwn, ctx->h_step + kStepOwn, kNumCounters * 8,
		                       hipMemcpyHostToDevice, s));
	}
	// the void reports are consumed (a fix-up round's flags come next); the
	// pairs count keeps running until the next step's send
	SYZ_HIP(hipMemsetAsync(ctx->d_step + kStepBack + kCntAux, 0, 8, s));
	SYZ_HIP(hipMemsetAsync(ctx->d_step + kStepBack + kCntError, 0, 8, s));
	float t = 0;
	if (ctx->step_src_timed && hipEventElapsedTime(&t, ctx->ev_step[0], ctx->ev_step[1]) == hipSuccess)
		out->src_ms = t;
	if (ctx->step_own_timed && hipEventElapsedTime(&t, ctx->ev_step[2], ctx->ev_step[3]) == hipSuccess)
		out->own_ms = t;
	if (ctx->step_back_timed && hipEventElapsedTime(&t, ctx->ev_step[4], ctx->ev_step[5]) == hipSuccess)
		out->back_ms = t;
	ctx->step_src_timed = ctx->step_own_timed = ctx->step_back_timed = false;
	return rc;
}

}  // extern "C"
