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
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <vector>

#include "internal.h"

namespace syz {

__global__ void k_min_keys(const uint64_t* __restrict__ off, uint64_t n, uint32_t* keys, uint32_t* idx)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t len = off[i + 1] - off[i];
		keys[i] = 0xFFFFFFFFu - (uint32_t)min<uint64_t>(len, 0xFFFFFFFFull);  // ascending key = Len desc
		idx[i] = (uint32_t)i;
	}
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

__global__ void k_count_u8(const uint8_t* __restrict__ a, uint64_t n, unsigned long long* cnt)
{
	uint64_t c = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
		c += a[i] != 0;
	block_count(&cnt[kCntAux], c);
}

}  // namespace syz

using namespace syz;

extern "C" {

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
	uint64_t total = 0;
	SYZ_HIP(hipMemcpyAsync(&total, d_off + nctx, 8, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipStreamSynchronize(st));
	if (total && (!d_elems || !d_prios))
		return fail(SYZSIG_EINVAL, "minimize: NULL entry arrays");
	// 1. stable order by (Len desc, index asc)
	void *dk, *dv, *dk2, *dv2, *drank, *dtmp = nullptr;
	SYZ_TRY(ws_get(ctx, 13, nctx * 16 + 64, &dk));
	dv = (uint32_t*)dk + nctx;
	dk2 = (uint32_t*)dv + nctx;
	dv2 = (uint32_t*)dk2 + nctx;
	SYZ_TRY(ws_get(ctx, 14, nctx * 4 + 64, &drank));
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[0], st));
	k_min_keys<<<grid_for(nctx, 256), 256, 0, st>>>(d_off, nctx, (uint32_t*)dk, (uint32_t*)dv);
	size_t tmp_bytes = 0;
	SYZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, (uint32_t*)dk, (uint32_t*)dk2, (uint32_t*)dv,
	                                           (uint32_t*)dv2, (int)nctx, 0, 32, st));
	SYZ_TRY(ws_get(ctx, 15, tmp_bytes + 64, &dtmp));
	SYZ_HIP(hipcub::DeviceRadixSort::SortPairs(dtmp, tmp_bytes, (uint32_t*)dk, (uint32_t*)dk2, (uint32_t*)dv,
	                                           (uint32_t*)dv2, (int)nctx, 0, 32, st));
	const uint32_t* order = (const uint32_t*)dv2;
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
			if (rc == SYZSIG_OK && ctx->timing && hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]) == hipSuccess)
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
