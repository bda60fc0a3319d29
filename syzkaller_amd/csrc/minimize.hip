// minimize.hip -- K5: pkg/signal/signal.go:133-166 Minimize on device.
//
// Reference: sort contexts by Len() desc (sort.Slice, unstable), then for each
// element keep covered[e] = (prio, idx), replaced only on a STRICTLY greater
// prio, so the earliest sorted index wins ties; survivors are the contexts
// that win at least one element.  Restatement: with the order fixed as
// (Len desc, index asc) by a stable radix sort, the winner of e is
//   argmax over entries of (prio, -rank)
// which one atomicMax per entry computes on the slot word
//   e << 32 | (prio ^ 0x80) << 24 | (0xFFFFFF - rank)        (rank < 2^24 - 1).
//
// The main path does it without device-scope atomics: the contexts in rank
// order are a "batch" whose call r is context order[r], and its entries go
// through the aggregation pipeline of agg.hip (partition by element, LDS hash
// per partition) with each entry's own prio as its level.  Per element that
// yields first[l] = the smallest rank with an entry at level l, so the winner
// is first[top level present] -- argmax (prio, -rank) again.  The atomic form
// above remains the fallback for more than 4 distinct prios (the records
// carry 2 level bits) or a context of >= 2^24 entries.
#include <algorithm>
#include <vector>

#include "internal.h"

namespace syz {

// the longest context (clamped to 2^32 - 1) into *mx (zeroed by the caller)
__global__ __launch_bounds__(256) void k_min_maxlen(const uint64_t* __restrict__ off, uint64_t n, uint32_t* mx)
{
	uint32_t m = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
		m = max(m, (uint32_t)min<uint64_t>(off[i + 1] - off[i], 0xFFFFFFFFull));
	for (int o = 32; o > 0; o >>= 1)
		m = max(m, (uint32_t)__shfl_xor(m, o, 64));
	if (lane_id() == 0 && m)
		atomicMax(mx, m);
}

// ascending key = Len desc: maxlen - len (< 2^bits(maxlen), the sort's passes)
__global__ void k_min_keys(const uint64_t* __restrict__ off, uint64_t n, uint32_t maxlen, uint32_t* keys,
                           uint32_t* idx)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t len = off[i + 1] - off[i];
		keys[i] = maxlen - (uint32_t)min<uint64_t>(len, maxlen);
		idx[i] = (uint32_t)i;
	}
}

static uint32_t bits_of(uint32_t x)
{
	uint32_t b = 0;
	while (b < 32 && (x >> b))
		b++;
	return b;
}

__global__ void k_min_rank(const uint32_t* __restrict__ order, uint64_t n, uint32_t* rank_of)
{
	for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x)
		rank_of[order[r]] = (uint32_t)r;
}

// one wave per context; with nshards > 1 only the entries whose element this
// shard owns (syz::owner_of) -- the winner of an element depends on that
// element's entries alone, so shards of the element space are independent
// (Minimize sharded by element)
__global__ __launch_bounds__(256) void k_min_cover(uint64_t* slots, uint64_t bmask, const uint64_t* __restrict__ off,
                                                   const uint32_t* __restrict__ elems, const int8_t* __restrict__ prios,
                                                   const uint32_t* __restrict__ rank_of, uint64_t n,
                                                   uint32_t nshards, uint32_t shard, unsigned long long* cnt)
{
	const uint32_t lane = lane_id();
	const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	const uint64_t maxp = max_probe_for(bmask);
	uint64_t ovf = 0;
	for (uint64_t c = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); c < n; c += nwaves) {
		const uint32_t low_rank = 0xFFFFFFu - rank_of[c];
		for (uint64_t j = off[c] + lane; j < off[c + 1]; j += 64) {
			const uint32_t e = elems[j];
			if (nshards > 1 && owner_of(e, nshards) != shard)
				continue;
			const uint64_t v = ((uint64_t)e << 32) | ((uint64_t)prio_biased(prios[j]) << 24) | low_rank;
			uint64_t old;
			const int64_t s = tbl_find_or_insert(slots, bmask, e, v, old, maxp);
			if (s < 0)
				ovf++;
			else if (old != 0 && old < v)
				atomicMax(reinterpret_cast<unsigned long long*>(slots + s), (unsigned long long)v);
		}
	}
	block_count(&cnt[kCntOverflow], ovf);
}

__global__ void k_min_winners(const uint64_t* __restrict__ slots, uint64_t nslots, const uint32_t* __restrict__ order,
                              uint8_t* keep)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t v = slots[i];
		if (v == kSlotEmpty)
			continue;
		keep[order[0xFFFFFFu - (uint32_t)(v & 0xFFFFFF)]] = 1;
	}
}

// the virtual batch: call r = context order[r] (call_len 0 + bad for a
// context too long for the aggregation records)
__global__ void k_min_calls(const uint64_t* __restrict__ off, const uint32_t* __restrict__ order, uint64_t n,
                            uint64_t* cstart, uint32_t* clen, unsigned long long* bad)
{
	uint64_t nb = 0;
	for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
		const uint32_t c = order[r];
		const uint64_t s = off[c], len = off[c + 1] - s;
		cstart[r] = s;
		clen[r] = len < (1ull << 24) ? (uint32_t)len : 0;
		nb += len >= (1ull << 24);
	}
	block_count(bad, nb);
}

// prios present among the entries (256-bit mask, by u8 value): a per-lane
// mask of 0..31 on the fast path, the full 8 words only when a wave sees one
// outside it
__global__ __launch_bounds__(256) void k_min_prio_mask(const uint8_t* __restrict__ prios, uint64_t n, uint32_t* mask)
{
	uint32_t lo = 0, m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	auto add_slow = [&](uint32_t u) {
#pragma unroll
		for (uint32_t k = 0; k < 8; k++)
			m[k] |= (u >> 5) == k ? 1u << (u & 31) : 0u;
	};
	const uint64_t n16 = ((uintptr_t)prios & 15) ? 0 : n / 16;
	const uint4* p16 = reinterpret_cast<const uint4*>(prios);
	// four 16-B loads in flight per thread (one at a time leaves the stream
	// latency-bound); a load past the end re-reads element 0, which is harmless
	// for a set of values
	const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += 4 * stride) {
		uint4 vv[4];
#pragma unroll
		for (uint32_t j = 0; j < 4; j++)
			vv[j] = p16[i + j * stride < n16 ? i + j * stride : 0];
#pragma unroll
		for (uint32_t j = 0; j < 4; j++) {
			const uint4 v = vv[j];
			const uint32_t w[4] = {v.x, v.y, v.z, v.w};
			if (((v.x | v.y | v.z | v.w) & 0xE0E0E0E0u) == 0) {  // every byte < 32
#pragma unroll
				for (uint32_t k = 0; k < 16; k++)
					lo |= 1u << ((w[k >> 2] >> ((k & 3) * 8)) & 31);
			} else {
#pragma unroll
				for (uint32_t k = 0; k < 16; k++)
					add_slow((w[k >> 2] >> ((k & 3) * 8)) & 0xFF);
			}
		}
	}
	for (uint64_t i = n16 * 16 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
	     i += (uint64_t)gridDim.x * blockDim.x)
		add_slow(prios[i]);
	m[0] |= lo;
#pragma unroll
	for (uint32_t k = 0; k < 8; k++) {
		uint32_t r = m[k];
		for (int d = 32; d >= 1; d >>= 1)
			r |= __shfl_xor(r, d, 64);
		if (lane_id() == 0 && r)
			atomicOr(&mask[k], r);
	}
}

// winners: per distinct element, the rank of its first entry at the top level
// present -> keep[that context]
__global__ __launch_bounds__(256) void k_min_from_dist(const uint4* __restrict__ dist_f,
                                                       const uint32_t* __restrict__ cnt, uint32_t nregions,
                                                       const uint32_t* __restrict__ order, uint8_t* keep)
{
	for (uint32_t r = blockIdx.x; r < nregions; r += gridDim.x) {
		const uint32_t n = cnt[r];
		for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
			const uint4 f = dist_f[(uint64_t)r * kAggRegion + i];
			const uint32_t rank = f.w != 0xFFFFFFFFu ? f.w : f.z != 0xFFFFFFFFu ? f.z : f.y != 0xFFFFFFFFu ? f.y : f.x;
			keep[order[rank]] = 1;
		}
	}
}

// prios present among the entries of the virtual batch's calls (one wave per
// call): the data-split parts read only their own contexts' entries
__global__ __launch_bounds__(256) void k_min_prio_mask_calls(const uint64_t* __restrict__ cstart,
                                                             const uint32_t* __restrict__ clen, uint64_t n,
                                                             const uint8_t* __restrict__ prios, uint32_t* mask)
{
	uint32_t m[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	for (uint64_t c = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); c < n; c += nwaves) {
		const uint64_t s0 = cstart[c];
		for (uint32_t j = lane_id(); j < clen[c]; j += 64) {
			const uint32_t u = prios[s0 + j];
#pragma unroll
			for (uint32_t k = 0; k < 8; k++)
				m[k] |= (u >> 5) == k ? 1u << (u & 31) : 0u;
		}
	}
#pragma unroll
	for (uint32_t k = 0; k < 8; k++) {
		uint32_t r = m[k];
		for (int d = 32; d >= 1; d >>= 1)
			r |= __shfl_xor(r, d, 64);
		if (lane_id() == 0 && r)
			atomicOr(&mask[k], r);
	}
}

// A part's winner record of a distinct element (see syzsig_minimize_split_dev):
// e << 32 | (prio ^ 0x80) << 24 | (0xFFFFFF - global rank); the max of the low
// 32 bits over the parts is argmax (prio, -rank), the reference's winner.
__device__ __forceinline__ uint64_t min_winner(uint32_t e, uint4 f4, const LevelMap& lm, uint32_t rank_lo)
{
	const uint32_t f[4] = {f4.x, f4.y, f4.z, f4.w};
	int top = 0;
#pragma unroll
	for (int l = 0; l < 4; l++)
		if (l < (int)lm.n && f[l] != 0xFFFFFFFFu)
			top = l;
	return ((uint64_t)e << 32) | ((uint64_t)prio_biased(lm.val[top]) << 24) | (0xFFFFFFu - (rank_lo + f[top]));
}

constexpr uint32_t kMinMaxShards = 64;

// winner records per owner (block histogram, one atomic per owner per block)
__global__ __launch_bounds__(256) void k_min_split_count(const uint32_t* __restrict__ dist_e,
                                                         const uint32_t* __restrict__ cnt, uint32_t nregions,
                                                         uint32_t nshards, unsigned long long* counts)
{
	__shared__ uint32_t h[kMinMaxShards];
	if (threadIdx.x < kMinMaxShards)
		h[threadIdx.x] = 0;
	__syncthreads();
	for (uint32_t r = blockIdx.x; r < nregions; r += gridDim.x) {
		const uint32_t n = cnt[r];
		for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
			atomicAdd(&h[owner_of(dist_e[(uint64_t)r * kAggRegion + i], nshards)], 1u);
	}
	__syncthreads();
	if (threadIdx.x < nshards && h[threadIdx.x])
		atomicAdd(&counts[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// winner records -> send[], grouped by owner (cursor[g] = next free slot of g)
__global__ __launch_bounds__(256) void k_min_split_scatter(const uint32_t* __restrict__ dist_e,
                                                           const uint4* __restrict__ dist_f,
                                                           const uint32_t* __restrict__ cnt, uint32_t nregions,
                                                           LevelMap lm, uint32_t rank_lo, uint32_t nshards,
                                                           unsigned long long* cursor, uint64_t* send)
{
	__shared__ uint32_t h[kMinMaxShards];
	__shared__ unsigned long long base[kMinMaxShards];
	for (uint32_t r = blockIdx.x; r < nregions; r += gridDim.x) {
		if (threadIdx.x < kMinMaxShards)
			h[threadIdx.x] = 0;
		__syncthreads();
		const uint32_t n = cnt[r];
		for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
			atomicAdd(&h[owner_of(dist_e[(uint64_t)r * kAggRegion + i], nshards)], 1u);
		__syncthreads();
		if (threadIdx.x < nshards) {
			base[threadIdx.x] = h[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)h[threadIdx.x]) : 0;
			h[threadIdx.x] = 0;
		}
		__syncthreads();
		for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
			const uint64_t o = (uint64_t)r * kAggRegion + i;
			const uint32_t e = dist_e[o], g = owner_of(e, nshards);
			send[base[g] + atomicAdd(&h[g], 1u)] = min_winner(e, dist_f[o], lm, rank_lo);
		}
		__syncthreads();
	}
}

// The split's atomic fallback (more than 4 distinct prios in the part, or a
// context of >= 2^24 entries): one wave per rank r of the part, every entry's
// record atomicMax'ed into a table keyed by element -- the slot word is the
// winner record min_winner builds, argmax (prio, -rank)
__global__ __launch_bounds__(256) void k_min_cover_ranks(uint64_t* slots, uint64_t bmask,
                                                         const uint64_t* __restrict__ off,
                                                         const uint32_t* __restrict__ elems,
                                                         const int8_t* __restrict__ prios,
                                                         const uint32_t* __restrict__ order, uint64_t r_lo,
                                                         uint64_t n, unsigned long long* cnt)
{
	const uint32_t lane = lane_id();
	const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	const uint64_t maxp = max_probe_for(bmask);
	uint64_t ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); i < n; i += nwaves) {
		const uint32_t c = order[r_lo + i];
		const uint32_t low_rank = 0xFFFFFFu - (uint32_t)(r_lo + i);
		for (uint64_t j = off[c] + lane; j < off[c + 1]; j += 64) {
			const uint32_t e = elems[j];
			const uint64_t v = ((uint64_t)e << 32) | ((uint64_t)prio_biased(prios[j]) << 24) | low_rank;
			uint64_t old;
			const int64_t s = tbl_find_or_insert(slots, bmask, e, v, old, maxp);
			if (s < 0)
				ovf++;
			else if (old != 0 && old < v)
				atomicMax(reinterpret_cast<unsigned long long*>(slots + s), (unsigned long long)v);
		}
	}
	block_count(&cnt[kCntOverflow], ovf);
}

// the fallback table's records per owner, then -> send[] grouped by owner
__global__ __launch_bounds__(256) void k_min_split_tbl(const uint64_t* __restrict__ slots, uint64_t nslots,
                                                       uint32_t nshards, unsigned long long* counts,
                                                       unsigned long long* cursor, uint64_t* send)
{
	__shared__ uint32_t h[kMinMaxShards];
	__shared__ unsigned long long base[kMinMaxShards];
	const uint64_t per = (nslots + gridDim.x - 1) / gridDim.x;
	const uint64_t s0 = blockIdx.x * per, s1 = min<uint64_t>(nslots, s0 + per);
	if (threadIdx.x < kMinMaxShards)
		h[threadIdx.x] = 0;
	__syncthreads();
	for (uint64_t i = s0 + threadIdx.x; i < s1; i += blockDim.x) {
		const uint64_t v = slots[i];
		if (v != kSlotEmpty)
			atomicAdd(&h[owner_of((uint32_t)(v >> 32), nshards)], 1u);
	}
	__syncthreads();
	if (threadIdx.x < nshards) {
		if (!send) {
			if (h[threadIdx.x])
				atomicAdd(&counts[threadIdx.x], (unsigned long long)h[threadIdx.x]);
		} else {
			base[threadIdx.x] = h[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)h[threadIdx.x]) : 0;
		}
		h[threadIdx.x] = 0;
	}
	__syncthreads();
	if (!send)
		return;
	for (uint64_t i = s0 + threadIdx.x; i < s1; i += blockDim.x) {
		const uint64_t v = slots[i];
		if (v == kSlotEmpty)
			continue;
		const uint32_t g = owner_of((uint32_t)(v >> 32), nshards);
		send[base[g] + atomicAdd(&h[g], 1u)] = v;
	}
}

// owner side: the max winner record per element (the slot word IS the record:
// key e in the top 32 bits, never 0 because rank < 2^24 - 1)
__global__ void k_min_resolve(uint64_t* slots, uint64_t bmask, const uint64_t* __restrict__ recs, uint64_t n,
                              unsigned long long* cnt)
{
	const uint64_t maxp = max_probe_for(bmask);
	uint64_t ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t v = recs[i];
		uint64_t old;
		const int64_t s = tbl_find_or_insert(slots, bmask, (uint32_t)(v >> 32), v, old, maxp);
		if (s < 0)
			ovf++;
		else if (old != 0 && old < v)
			atomicMax(reinterpret_cast<unsigned long long*>(slots + s), (unsigned long long)v);
	}
	block_count(&cnt[kCntOverflow], ovf);
}

__global__ void k_count_u8(const uint8_t* __restrict__ a, uint64_t n, unsigned long long* cnt)
{
	uint64_t c = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
		c += a[i] != 0;
	block_count(&cnt[kCntAux], c);
}

}  // namespace syz

using namespace syz;

// The aggregation path (header).  *used = false: the atomic path must run
// (more than 4 distinct prios, or a context of >= 2^24 entries).
// exact: find the prios present first (one pass over them and a host round
// trip); else assume signalPrio's 0..3 (fuzzer.go:513-521) and let the
// scatter flag a prio outside them (*redo: nothing usable, call again exact).
static int minimize_agg_run(syzsig_ctx* ctx, const uint64_t* d_off, const uint32_t* d_elems, const int8_t* d_prios,
                            uint64_t nctx, uint64_t total, uint32_t nshards, uint32_t shard, uint64_t hint,
                            const uint32_t* order, uint8_t* d_keep, bool exact, bool* used, bool* redo)
{
	*used = false;
	*redo = false;
	hipStream_t st = ctx->stream;
	void* vb;
	SYZ_TRY(ws_get(ctx, 34, nctx * 12 + 128, &vb));
	uint32_t* dmask = (uint32_t*)vb;                               // [0, 32)
	uint32_t* dflag = (uint32_t*)((char*)vb + 48);                 // a prio without a level (optimistic run)
	unsigned long long* dbad = (unsigned long long*)((char*)vb + 56);  // contexts of >= 2^24 entries
	uint64_t* cstart = (uint64_t*)((char*)vb + 64);
	uint32_t* clen = (uint32_t*)(cstart + nctx);
	SYZ_HIP(hipMemsetAsync(vb, 0, 64, st));
	k_min_calls<<<grid_for(nctx, 256), 256, 0, st>>>(d_off, order, nctx, cstart, clen, dbad);
	int8_t levels[4] = {0, 1, 2, 3};
	uint32_t nl = 4;
	if (exact) {
		k_min_prio_mask<<<grid_for(total / 16 + 1, 256, 2048), 256, 0, st>>>((const uint8_t*)d_prios, total, dmask);
		SYZ_HIP(hipGetLastError());
		uint32_t* hmask = (uint32_t*)(ctx->h_pin + kPinMask);
		SYZ_HIP(hipMemcpyAsync(hmask, vb, 64, hipMemcpyDeviceToHost, st));
		SYZ_HIP(hipStreamSynchronize(st));
		uint64_t nbad;
		memcpy(&nbad, (char*)hmask + 56, 8);
		if (nbad)
			return SYZSIG_OK;
		nl = 0;
		for (int v = -128; v <= 127; v++) {
			const uint8_t u = (uint8_t)(int8_t)v;
			if ((hmask[u >> 5] >> (u & 31)) & 1) {
				if (nl == 4)
					return SYZSIG_OK;
				levels[nl++] = (int8_t)v;
			}
		}
	}
	SYZ_HIP(hipGetLastError());
	LevelMap lm;
	SYZ_TRY(level_map_from_levels(levels, nl, &lm));
	syzsig_batch b = {};
	b.sigs = d_elems;
	b.call_start = cstart;
	b.call_len = clen;
	b.ncalls = nctx;
	b.nrec = total;
	AggSrc x{d_prios, nshards, shard, (double)(hint ? hint : total)};  // distinct <= entries
	if (!exact)
		x.bad_level = dflag;
	syzsig_batch_stats bst = {};
	AggOut a;
	SYZ_TRY(agg_aggregate(ctx, &b, 0, nctx, lm, total, &bst, &a, &x));
	if (!exact) {  // (agg_aggregate synchronised: the flags are final)
		uint32_t* hf = (uint32_t*)(ctx->h_pin + kPinMask);
		SYZ_HIP(hipMemcpyAsync(hf, vb, 64, hipMemcpyDeviceToHost, st));
		SYZ_HIP(hipStreamSynchronize(st));
		uint64_t nbad;
		memcpy(&nbad, (char*)hf + 56, 8);
		if (nbad)
			return SYZSIG_OK;  // a context too long for the serial: the atomic path
		if (hf[12]) {
			*redo = true;
			return SYZSIG_OK;
		}
	}
	SYZ_HIP(hipMemsetAsync(d_keep, 0, nctx, st));
	k_min_from_dist<<<std::min<uint32_t>(a.nregions, 8192), 256, 0, st>>>(a.dist_f, a.cnt, a.nregions, order, d_keep);
	SYZ_HIP(hipGetLastError());
	*used = true;
	return SYZSIG_OK;
}

static int minimize_agg(syzsig_ctx* ctx, const uint64_t* d_off, const uint32_t* d_elems, const int8_t* d_prios,
                        uint64_t nctx, uint64_t total, uint32_t nshards, uint32_t shard, uint64_t hint,
                        const uint32_t* order, uint8_t* d_keep, bool* used)
{
	bool redo = false;
	SYZ_TRY(minimize_agg_run(ctx, d_off, d_elems, d_prios, nctx, total, nshards, shard, hint, order, d_keep, false, used,
	                         &redo));
	if (redo)
		SYZ_TRY(minimize_agg_run(ctx, d_off, d_elems, d_prios, nctx, total, nshards, shard, hint, order, d_keep, true,
		                         used, &redo));
	return SYZSIG_OK;
}

// The stable order by (Len desc, index asc) of nctx contexts: order[r] = the
// context at rank r (scratch slots 13-15).
static int minimize_order(syzsig_ctx* ctx, const uint64_t* d_off, uint64_t nctx, const uint32_t** order)
{
	hipStream_t st = ctx->stream;
	void* dk;
	SYZ_TRY(ws_get(ctx, 13, nctx * 16 + 64, &dk));
	uint32_t* dv = (uint32_t*)dk + nctx;
	uint32_t* dk2 = dv + nctx;
	uint32_t* dv2 = dk2 + nctx;
	uint32_t maxlen = 0;
	SYZ_HIP(hipMemsetAsync(dk2, 0, 4, st));
	k_min_maxlen<<<grid_for(nctx, 256, 1024), 256, 0, st>>>(d_off, nctx, dk2);
	SYZ_HIP(hipMemcpyAsync(&maxlen, dk2, 4, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipStreamSynchronize(st));
	k_min_keys<<<grid_for(nctx, 256), 256, 0, st>>>(d_off, nctx, maxlen, (uint32_t*)dk, dv);
	uint32_t *sk, *sv;
	SYZ_TRY(radix_sort_pairs(ctx, (uint32_t*)dk, dv, dk2, dv2, (uint32_t)nctx, bits_of(maxlen), &sk, &sv, 15));
	*order = sv;
	return SYZSIG_OK;
}

extern "C" {

int syzsig_minimize_split_dev(syzsig_ctx* ctx, const uint64_t* d_off, const uint32_t* d_elems, const int8_t* d_prios,
                              uint64_t nctx, uint32_t nparts, uint32_t part, uint32_t nshards, uint64_t hint_distinct,
                              uint64_t* d_send, uint64_t send_cap, uint64_t* send_counts)
{
	SYZ_LOCK(ctx);
	if (!ctx || !send_counts || (nctx && !d_off) || (send_cap && !d_send))
		return fail(SYZSIG_EINVAL, "minimize_split: NULL argument");
	if (nparts == 0 || part >= nparts || nshards == 0 || nshards > kMinMaxShards)
		return fail(SYZSIG_EINVAL, "minimize_split: need part < nparts and 1 <= nshards <= 64");
	for (uint32_t g = 0; g < nshards; g++)
		send_counts[g] = 0;
	if (nctx == 0)
		return SYZSIG_OK;
	if (nctx >= 0xFFFFFFull)
		return fail(SYZSIG_ERANGE, "minimize: more than 2^24-2 contexts");
	hipStream_t st = ctx->stream;
	const uint32_t* order = nullptr;
	SYZ_TRY(minimize_order(ctx, d_off, nctx, &order));
	// this part's range of ranks: cut at about part * total / nparts entries
	std::vector<uint64_t> off(nctx + 1);
	std::vector<uint32_t> ord(nctx);
	SYZ_HIP(hipMemcpyAsync(off.data(), d_off, (nctx + 1) * 8, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipMemcpyAsync(ord.data(), order, nctx * 4, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipStreamSynchronize(st));
	uint64_t total = 0;
	for (uint64_t i = 0; i < nctx; i++) {
		if (off[i + 1] < off[i])
			return fail(SYZSIG_EINVAL, "minimize_split: ctx_off not monotone");
		total += off[i + 1] - off[i];
	}
	if (total && (!d_elems || !d_prios))
		return fail(SYZSIG_EINVAL, "minimize: NULL entry arrays");
	const uint64_t want_lo = total * part / nparts, want_hi = total * (part + 1) / nparts;
	uint64_t cum = 0, r_lo = nctx, r_hi = nctx;
	for (uint64_t r = 0; r < nctx; r++) {
		if (r_lo == nctx && cum >= want_lo && (part > 0 || r == 0))
			r_lo = r;
		if (cum >= want_hi && part + 1 < nparts) {
			r_hi = r;
			break;
		}
		cum += off[ord[r] + 1] - off[ord[r]];
	}
	if (r_lo > r_hi)
		r_lo = r_hi;
	uint64_t local = 0;
	for (uint64_t r = r_lo; r < r_hi; r++)
		local += off[ord[r] + 1] - off[ord[r]];
	if (local == 0)
		return SYZSIG_OK;
	if (local > send_cap)
		return fail(SYZSIG_ERANGE, "minimize_split: send buffer smaller than the part's entries");
	// the part's contexts as a virtual batch in rank order
	const uint64_t n = r_hi - r_lo;
	void* vb;
	SYZ_TRY(ws_get(ctx, 34, n * 12 + 128, &vb));
	uint32_t* dmask = (uint32_t*)vb;
	uint64_t* cstart = (uint64_t*)((char*)vb + 64);
	uint32_t* clen = (uint32_t*)(cstart + n);
	SYZ_TRY(counters_reset(ctx));
	SYZ_HIP(hipMemsetAsync(dmask, 0, 32, st));
	k_min_calls<<<grid_for(n, 256), 256, 0, st>>>(d_off, order + r_lo, n, cstart, clen, &ctx->d_cnt[kCntAux]);
	k_min_prio_mask_calls<<<grid_for(n * 64, 256, 4096), 256, 0, st>>>(cstart, clen, n, (const uint8_t*)d_prios, dmask);
	SYZ_HIP(hipGetLastError());
	uint32_t* hmask = (uint32_t*)(ctx->h_pin + kPinMask);
	SYZ_HIP(hipMemcpyAsync(hmask, dmask, 32, hipMemcpyDeviceToHost, st));
	SYZ_TRY(counters_fetch(ctx));
	int8_t levels[4];
	uint32_t nl = 0;
	bool atomic_path = ctx->h_cnt[kCntAux] != 0 || (ctx->agg_dbg & SYZSIG_DEBUG_MIN_ATOMIC);
	for (int v = -128; v <= 127 && !atomic_path; v++) {
		const uint8_t u = (uint8_t)(int8_t)v;
		if ((hmask[u >> 5] >> (u & 31)) & 1) {
			if (nl == 4)
				atomic_path = true;  // the records carry 2 level bits
			else
				levels[nl++] = (int8_t)v;
		}
	}
	if (atomic_path) {
		// a context of >= 2^24 entries or more than 4 prios: any int8 prio is a
		// valid DiffRaw/Minimize prio (signal.go:138-166), so the part's winners
		// come from the per-entry atomicMax table instead of failing
		syzsig_set* t = nullptr;
		SYZ_TRY(set_alloc(ctx, buckets_for(local), &t));
		void* dcur;
		int rc = ws_get(ctx, 36, 2 * kMinMaxShards * 8, &dcur);
		unsigned long long* counts = (unsigned long long*)dcur;
		unsigned long long* cursor = counts + kMinMaxShards;
		unsigned long long h[kMinMaxShards] = {};
		const int tg = (int)std::min<uint64_t>(std::max<uint64_t>(t->nslots() / 4096, 1), 4096);
		if (rc == SYZSIG_OK)
			rc = counters_reset(ctx);
		if (rc == SYZSIG_OK) {
			(void)hipMemsetAsync(counts, 0, kMinMaxShards * 8, st);
			k_min_cover_ranks<<<grid_for(n * 64, 256, 8192), 256, 0, st>>>(t->slots, t->nbuckets - 1, d_off, d_elems,
			                                                               d_prios, order, r_lo, n, ctx->d_cnt);
			k_min_split_tbl<<<tg, 256, 0, st>>>(t->slots, t->nslots(), nshards, counts, nullptr, nullptr);
			hipError_t e = hipGetLastError();
			if (e == hipSuccess)
				e = hipMemcpyAsync(h, counts, nshards * 8, hipMemcpyDeviceToHost, st);
			rc = e == hipSuccess ? counters_fetch(ctx) : hip_fail(e, "k_min_cover_ranks", __FILE__, __LINE__);
		}
		if (rc == SYZSIG_OK && ctx->h_cnt[kCntOverflow])
			rc = fail(SYZSIG_EIO, "minimize_split: table overflow (internal error)");
		if (rc == SYZSIG_OK) {
			unsigned long long offs[kMinMaxShards], run = 0;
			for (uint32_t g = 0; g < nshards; g++) {
				offs[g] = run;
				run += h[g];
				send_counts[g] = h[g];
			}
			hipError_t e = hipMemcpyAsync(cursor, offs, nshards * 8, hipMemcpyHostToDevice, st);
			if (e == hipSuccess) {
				k_min_split_tbl<<<tg, 256, 0, st>>>(t->slots, t->nslots(), nshards, counts, cursor, d_send);
				e = hipGetLastError();
			}
			if (e == hipSuccess)
				e = hipStreamSynchronize(st);
			if (e != hipSuccess)
				rc = hip_fail(e, "k_min_split_tbl", __FILE__, __LINE__);
		}
		syzsig_set_free(t);
		return rc;
	}
	LevelMap lm;
	SYZ_TRY(level_map_from_levels(levels, nl, &lm));
	syzsig_batch b = {};
	b.sigs = d_elems;
	b.call_start = cstart;
	b.call_len = clen;
	b.ncalls = n;
	b.nrec = total;
	const AggSrc x{d_prios, 1, 0, (double)(hint_distinct ? std::min(hint_distinct, local) : local)};
	syzsig_batch_stats bst = {};
	AggOut a;
	SYZ_TRY(agg_aggregate(ctx, &b, 0, n, lm, local, &bst, &a, &x));
	void* dcur;
	SYZ_TRY(ws_get(ctx, 36, 2 * kMinMaxShards * 8, &dcur));
	unsigned long long* counts = (unsigned long long*)dcur;
	unsigned long long* cursor = counts + kMinMaxShards;
	SYZ_HIP(hipMemsetAsync(counts, 0, kMinMaxShards * 8, st));
	const int grid = (int)std::min<uint32_t>(a.nregions, 2048);
	k_min_split_count<<<grid, 256, 0, st>>>(a.dist_e, a.cnt, a.nregions, nshards, counts);
	SYZ_HIP(hipGetLastError());
	unsigned long long h[kMinMaxShards];
	SYZ_HIP(hipMemcpyAsync(h, counts, nshards * 8, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipStreamSynchronize(st));
	unsigned long long offs[kMinMaxShards], run = 0;
	for (uint32_t g = 0; g < nshards; g++) {
		offs[g] = run;
		run += h[g];
		send_counts[g] = h[g];
	}
	SYZ_HIP(hipMemcpyAsync(cursor, offs, nshards * 8, hipMemcpyHostToDevice, st));
	k_min_split_scatter<<<grid, 256, 0, st>>>(a.dist_e, a.dist_f, a.cnt, a.nregions, lm, (uint32_t)r_lo, nshards, cursor,
	                                          d_send);
	SYZ_HIP(hipGetLastError());
	SYZ_HIP(hipStreamSynchronize(st));
	return SYZSIG_OK;
}

int syzsig_minimize_resolve_dev(syzsig_ctx* ctx, const uint64_t* d_off, uint64_t nctx, const uint64_t* d_recs,
                                uint64_t nrec, uint8_t* d_keep, uint64_t* n_out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !n_out || (nctx && (!d_off || !d_keep)) || (nrec && !d_recs))
		return fail(SYZSIG_EINVAL, "minimize_resolve: NULL argument");
	*n_out = 0;
	if (nctx == 0)
		return SYZSIG_OK;
	if (nctx >= 0xFFFFFFull)
		return fail(SYZSIG_ERANGE, "minimize: more than 2^24-2 contexts");
	hipStream_t st = ctx->stream;
	SYZ_HIP(hipMemsetAsync(d_keep, 0, nctx, st));
	if (nrec) {
		const uint32_t* order = nullptr;
		SYZ_TRY(minimize_order(ctx, d_off, nctx, &order));
		syzsig_set* t = nullptr;
		SYZ_TRY(set_alloc(ctx, buckets_for(nrec), &t));
		SYZ_TRY(counters_reset(ctx));
		k_min_resolve<<<grid_for(nrec, 256, 8192), 256, 0, st>>>(t->slots, t->nbuckets - 1, d_recs, nrec, ctx->d_cnt);
		k_min_winners<<<grid_for(t->nslots(), 256), 256, 0, st>>>(t->slots, t->nslots(), order, d_keep);
		hipError_t e = hipGetLastError();
		int rc = e == hipSuccess ? counters_fetch(ctx) : hip_fail(e, "k_min_resolve", __FILE__, __LINE__);
		syzsig_set_free(t);
		SYZ_TRY(rc);
		if (ctx->h_cnt[kCntOverflow])
			return fail(SYZSIG_EIO, "minimize_resolve: table overflow (internal error)");
	}
	SYZ_TRY(counters_reset(ctx));
	k_count_u8<<<grid_for(nctx, 256), 256, 0, st>>>(d_keep, nctx, ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	*n_out = ctx->h_cnt[kCntAux];
	return SYZSIG_OK;
}

int syzsig_minimize_shard_dev(syzsig_ctx* ctx, const uint64_t* d_off, const uint32_t* d_elems, const int8_t* d_prios,
                              uint64_t nctx, uint32_t nshards, uint32_t shard, uint64_t hint_distinct, uint8_t* d_keep,
                              uint64_t* n_out)
{
	SYZ_LOCK(ctx);
	if (nshards == 0 || shard >= nshards)
		return fail(SYZSIG_EINVAL, "minimize_shard: shard must be < nshards");
	if (!ctx || !n_out || (nctx && (!d_off || !d_keep)))
		return fail(SYZSIG_EINVAL, "minimize: NULL argument");
	*n_out = 0;
	if (nctx == 0)
		return SYZSIG_OK;
	if (nctx >= 0xFFFFFFull)
		return fail(SYZSIG_ERANGE, "minimize: more than 2^24-2 contexts");
	hipStream_t st = ctx->stream;
	void *dk, *dv, *dk2, *dv2, *drank;
	SYZ_TRY(ws_get(ctx, 13, nctx * 16 + 64, &dk));
	dv = (uint32_t*)dk + nctx;
	dk2 = (uint32_t*)dv + nctx;
	dv2 = (uint32_t*)dk2 + nctx;
	SYZ_TRY(ws_get(ctx, 14, nctx * 4 + 64, &drank));
	// the entry count and the longest context (the order's sort passes), one sync
	uint64_t total = 0;
	uint32_t maxlen = 0;
	SYZ_HIP(hipMemsetAsync(dk2, 0, 4, st));
	k_min_maxlen<<<grid_for(nctx, 256, 1024), 256, 0, st>>>(d_off, nctx, (uint32_t*)dk2);
	SYZ_HIP(hipMemcpyAsync(&maxlen, dk2, 4, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipMemcpyAsync(&total, d_off + nctx, 8, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipStreamSynchronize(st));
	if (total && (!d_elems || !d_prios))
		return fail(SYZSIG_EINVAL, "minimize: NULL entry arrays");
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[3], st));
	// 1. stable order by (Len desc, index asc)
	k_min_keys<<<grid_for(nctx, 256), 256, 0, st>>>(d_off, nctx, maxlen, (uint32_t*)dk, (uint32_t*)dv);
	uint32_t *sk, *sv;
	SYZ_TRY(radix_sort_pairs(ctx, (uint32_t*)dk, (uint32_t*)dv, (uint32_t*)dk2, (uint32_t*)dv2, (uint32_t)nctx,
	                         bits_of(maxlen), &sk, &sv, 15));
	const uint32_t* order = sv;
	bool used = false;
	if (total && !(ctx->agg_dbg & SYZSIG_DEBUG_MIN_ATOMIC))
		SYZ_TRY(minimize_agg(ctx, d_off, d_elems, d_prios, nctx, total, nshards, shard, hint_distinct, order, d_keep,
		                     &used));
	if (used) {
		SYZ_TRY(counters_reset(ctx));
		k_count_u8<<<grid_for(nctx, 256), 256, 0, st>>>(d_keep, nctx, ctx->d_cnt);
		SYZ_HIP(hipGetLastError());
		if (ctx->timing)
			SYZ_HIP(hipEventRecord(ctx->ev[0], st));
		SYZ_TRY(counters_fetch(ctx));
		float t = 0;
		if (ctx->timing && hipEventElapsedTime(&t, ctx->ev[3], ctx->ev[0]) == hipSuccess)
			ctx->last_ms = t;
		*n_out = ctx->h_cnt[kCntAux];
		return SYZSIG_OK;
	}
	k_min_rank<<<grid_for(nctx, 256), 256, 0, st>>>(order, nctx, (uint32_t*)drank);
	// 2. per-element argmax of (prio, -rank)
	uint64_t nb = buckets_for(hint_distinct ? hint_distinct : std::max<uint64_t>(total, 1));
	for (;;) {
		syzsig_set* t = nullptr;
		SYZ_TRY(set_alloc(ctx, nb, &t));
		SYZ_TRY(counters_reset(ctx));
		k_min_cover<<<grid_for(nctx * 64, 256, 4096), 256, 0, st>>>(t->slots, nb - 1, d_off, d_elems, d_prios,
		                                                             (const uint32_t*)drank, nctx, nshards, shard,
		                                                             ctx->d_cnt);
		hipError_t e = hipGetLastError();
		int rc = e == hipSuccess ? counters_fetch(ctx) : hip_fail(e, "k_min_cover", __FILE__, __LINE__);
		if (rc == SYZSIG_OK && ctx->h_cnt[kCntOverflow]) {
			syzsig_set_free(t);
			nb *= 8;
			continue;
		}
		if (rc == SYZSIG_OK) {
			// 3. survivors
			if (hipMemsetAsync(d_keep, 0, nctx, st) != hipSuccess)
				rc = fail(SYZSIG_EIO, "memset keep");
			k_min_winners<<<grid_for(t->nslots(), 256), 256, 0, st>>>(t->slots, t->nslots(), order, d_keep);
			k_count_u8<<<grid_for(nctx, 256), 256, 0, st>>>(d_keep, nctx, ctx->d_cnt);
			if (ctx->timing && hipEventRecord(ctx->ev[1], st) != hipSuccess)
				rc = fail(SYZSIG_EIO, "event record");
			if (rc == SYZSIG_OK)
				rc = counters_fetch(ctx);
			float t = 0;
			if (rc == SYZSIG_OK && ctx->timing && hipEventElapsedTime(&t, ctx->ev[3], ctx->ev[1]) == hipSuccess)
				ctx->last_ms = t;
		}
		syzsig_set_free(t);
		SYZ_TRY(rc);
		*n_out = ctx->h_cnt[kCntAux];
		return SYZSIG_OK;
	}
}

int syzsig_minimize_dev(syzsig_ctx* ctx, const uint64_t* d_off, const uint32_t* d_elems, const int8_t* d_prios,
                        uint64_t nctx, uint64_t hint_distinct, uint8_t* d_keep, uint64_t* n_out)
{
	return syzsig_minimize_shard_dev(ctx, d_off, d_elems, d_prios, nctx, 1, 0, hint_distinct, d_keep, n_out);
}

int syzsig_minimize(syzsig_ctx* ctx, const uint64_t* ctx_off, const uint32_t* elems, const int8_t* prios,
                    uint64_t nctx, uint64_t hint_distinct, uint64_t* out_idx, uint64_t* n_out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !n_out || (nctx && (!ctx_off || !out_idx)))
		return fail(SYZSIG_EINVAL, "minimize: NULL argument");
	*n_out = 0;
	if (nctx == 0)
		return SYZSIG_OK;
	for (uint64_t i = 0; i < nctx; i++)
		if (ctx_off[i + 1] < ctx_off[i])
			return fail(SYZSIG_EINVAL, "minimize: ctx_off not monotone");
	const uint64_t total = ctx_off[nctx] - ctx_off[0];
	if (ctx_off[0] != 0)
		return fail(SYZSIG_EINVAL, "minimize: ctx_off[0] must be 0");
	void *doff, *de, *dp, *dkeep;
	SYZ_TRY(ws_get(ctx, 7, (nctx + 1) * 8, &doff));
	SYZ_TRY(ws_get(ctx, 8, total * 4 + 4, &de));
	SYZ_TRY(ws_get(ctx, 9, total + 1, &dp));
	SYZ_TRY(ws_get(ctx, 10, nctx + 1, &dkeep));
	SYZ_HIP(hipMemcpyAsync(doff, ctx_off, (nctx + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
	if (total) {
		SYZ_HIP(hipMemcpyAsync(de, elems, total * 4, hipMemcpyHostToDevice, ctx->stream));
		SYZ_HIP(hipMemcpyAsync(dp, prios, total, hipMemcpyHostToDevice, ctx->stream));
	}
	uint64_t n = 0;
	SYZ_TRY(syzsig_minimize_dev(ctx, (const uint64_t*)doff, (const uint32_t*)de, (const int8_t*)dp, nctx,
	                            hint_distinct, (uint8_t*)dkeep, &n));
	std::vector<uint8_t> keep(nctx);
	SYZ_HIP(hipMemcpyAsync(keep.data(), dkeep, nctx, hipMemcpyDeviceToHost, ctx->stream));
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	uint64_t k = 0;
	for (uint64_t i = 0; i < nctx; i++)
		if (keep[i])
			out_idx[k++] = i;
	*n_out = k;
	return SYZSIG_OK;
}

}  // extern "C"
