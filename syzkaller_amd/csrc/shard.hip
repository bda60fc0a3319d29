// shard.hip -- routing of a batch's records to the GPU that owns their element
// (maxSignal hash-partitioned over G GPUs), and the return path of new flags.
//
// The exchange itself is an all-to-all over xGMI (RCCL, driven by the host
// through torch.distributed); this file builds the send buffer grouped by
// owner and scatters the returned flags back to records and calls.  The
// triage on the owner is order-independent (it keys on the serial field), so
// the order of records inside an owner group does not matter.
#include <vector>

#include "internal.h"

namespace syz {

constexpr uint32_t kMaxShards = 64;
constexpr uint32_t kCallsPerBlock = 32;

__device__ __forceinline__ bool call_ok(const syzsig_batch& b, uint64_t c, uint64_t& start, uint32_t& len)
{
	start = b.call_start[c];
	len = b.call_len[c];
	return start <= b.nrec && len <= b.nrec - start;
}

// per-owner record counts (block histogram in LDS, one atomic per owner per block)
__global__ __launch_bounds__(256) void k_shard_count(syzsig_batch b, uint32_t nshards, unsigned long long* counts,
                                                     unsigned long long* cnt)
{
	__shared__ uint32_t h[kMaxShards];
	if (threadIdx.x < kMaxShards)
		h[threadIdx.x] = 0;
	__syncthreads();
	const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = lane_id();
	uint64_t err = 0;
	const uint64_t nchunks = (b.ncalls + kCallsPerBlock - 1) / kCallsPerBlock;
	for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
		const uint64_t ce = min<uint64_t>(b.ncalls, (ch + 1) * kCallsPerBlock);
		for (uint64_t c = ch * kCallsPerBlock + w; c < ce; c += nw) {
			uint64_t start;
			uint32_t len;
			if (!call_ok(b, c, start, len)) {
				err += lane == 0;
				continue;
			}
			for (uint32_t j = lane; j < len; j += 64)
				atomicAdd(&h[owner_of(b.sigs[start + j], nshards)], 1u);
		}
	}
	__syncthreads();
	if (threadIdx.x < nshards && h[threadIdx.x])
		atomicAdd(&counts[threadIdx.x], (unsigned long long)h[threadIdx.x]);
	block_count(&cnt[kCntError], err);
}

__global__ __launch_bounds__(256) void k_shard_scatter(syzsig_batch b, uint64_t serial_base, LevelMap lm,
                                                       uint32_t nshards, unsigned long long* cursor, uint64_t* send,
                                                       uint32_t* send_pos)
{
	__shared__ uint32_t h[kMaxShards];
	__shared__ unsigned long long base[kMaxShards];
	const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = lane_id();
	const uint64_t nchunks = (b.ncalls + kCallsPerBlock - 1) / kCallsPerBlock;
	for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
		if (threadIdx.x < kMaxShards)
			h[threadIdx.x] = 0;
		__syncthreads();
		const uint64_t ce = min<uint64_t>(b.ncalls, (ch + 1) * kCallsPerBlock);
		for (uint64_t c = ch * kCallsPerBlock + w; c < ce; c += nw) {
			uint64_t start;
			uint32_t len;
			if (!call_ok(b, c, start, len))
				continue;
			for (uint32_t j = lane; j < len; j += 64)
				atomicAdd(&h[owner_of(b.sigs[start + j], nshards)], 1u);
		}
		__syncthreads();
		if (threadIdx.x < nshards) {
			base[threadIdx.x] = h[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], (unsigned long long)h[threadIdx.x]) : 0;
			h[threadIdx.x] = 0;
		}
		__syncthreads();
		for (uint64_t c = ch * kCallsPerBlock + w; c < ce; c += nw) {
			uint64_t start;
			uint32_t len;
			if (!call_ok(b, c, start, len))
				continue;
			const uint64_t head = ((uint64_t)lm.lvl[b.call_prio[c]] << 24) | ((serial_base + c) & kSerialMask);
			for (uint32_t j = lane; j < len; j += 64) {
				const uint32_t e = b.sigs[start + j];
				const uint32_t o = owner_of(e, nshards);
				const uint64_t pos = base[o] + atomicAdd(&h[o], 1u);
				send[pos] = ((uint64_t)e << 32) | head;
				send_pos[start + j] = (uint32_t)pos;
			}
		}
		__syncthreads();
	}
}

__global__ __launch_bounds__(256) void k_shard_unpart(syzsig_batch b, const uint32_t* __restrict__ send_pos,
                                                      const uint8_t* __restrict__ back)
{
	const uint32_t lane = lane_id();
	const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
	for (uint64_t c = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); c < b.ncalls; c += nwaves) {
		uint64_t start;
		uint32_t len;
		if (!call_ok(b, c, start, len))
			continue;
		bool any = false;
		for (uint32_t j = lane; j < len; j += 64) {
			if (back[send_pos[start + j]]) {
				const uint64_t r = start + j;
				atomicOr(&b.new_bits[r >> 5], 1u << (r & 31));
				any = true;
			}
		}
		if (__ballot(any) && lane == 0)
			b.call_new[c] = 1;
	}
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzsig_shard_partition_dev(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t serial_base, const int8_t* levels,
                               uint32_t nlevels, uint32_t nshards, uint64_t* d_send, uint32_t* d_send_pos,
                               uint64_t* send_counts)
{
	SYZ_LOCK(ctx);
	if (!ctx || !b || !send_counts || (b->nrec && (!d_send || !d_send_pos || !b->sigs)) ||
	    (b->ncalls && (!b->call_start || !b->call_len || !b->call_prio)))
		return fail(SYZSIG_EINVAL, "shard_partition: NULL argument");
	if (nshards == 0 || nshards > kMaxShards)
		return fail(SYZSIG_EINVAL, "shard_partition: nshards must be 1..64");
	if (b->nrec >= (1ull << 32))
		return fail(SYZSIG_ERANGE, "shard_partition: >= 2^32 records per GPU");
	if (serial_base + b->ncalls > kSerialMask + 1ull)
		return fail(SYZSIG_ERANGE, "shard_partition: batch serial order exceeds 2^24 calls");
	LevelMap lm;
	SYZ_TRY(level_map_from_levels(levels, nlevels, &lm));
	for (uint32_t i = 0; i < nshards; i++)
		send_counts[i] = 0;
	if (b->ncalls == 0)
		return SYZSIG_OK;
	void* dcur;
	SYZ_TRY(ws_get(ctx, 6, 2 * kMaxShards * 8, &dcur));
	unsigned long long* counts = (unsigned long long*)dcur;
	unsigned long long* cursor = counts + kMaxShards;
	SYZ_HIP(hipMemsetAsync(counts, 0, kMaxShards * 8, ctx->stream));
	SYZ_TRY(counters_reset(ctx));
	const uint64_t nchunks = (b->ncalls + kCallsPerBlock - 1) / kCallsPerBlock;
	const int grid = (int)std::min<uint64_t>(nchunks, 2048);
	k_shard_count<<<grid, 256, 0, ctx->stream>>>(*b, nshards, counts, ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	unsigned long long h[kMaxShards];
	SYZ_HIP(hipMemcpyAsync(h, counts, kMaxShards * 8, hipMemcpyDeviceToHost, ctx->stream));
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->h_cnt[kCntError])
		return fail(SYZSIG_EINVAL, "shard_partition: a call range lies outside [0, nrec)");
	unsigned long long off[kMaxShards];
	unsigned long long run = 0;
	for (uint32_t i = 0; i < nshards; i++) {
		off[i] = run;
		run += h[i];
		send_counts[i] = h[i];
	}
	SYZ_HIP(hipMemcpyAsync(cursor, off, nshards * 8, hipMemcpyHostToDevice, ctx->stream));
	k_shard_scatter<<<grid, 256, 0, ctx->stream>>>(*b, serial_base, lm, nshards, cursor, d_send, d_send_pos);
	SYZ_HIP(hipGetLastError());
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	return SYZSIG_OK;
}

int syzsig_shard_unpartition_dev(syzsig_ctx* ctx, const syzsig_batch* b, const uint32_t* d_send_pos,
                                 const uint8_t* d_back_flags)
{
	SYZ_LOCK(ctx);
	if (!ctx || !b || (b->nrec && (!d_send_pos || !d_back_flags || !b->new_bits)) || (b->ncalls && !b->call_new))
		return fail(SYZSIG_EINVAL, "shard_unpartition: NULL argument");
	SYZ_HIP(hipMemsetAsync(b->new_bits, 0, ((b->nrec + 31) / 32) * 4, ctx->stream));
	if (b->ncalls) {
		SYZ_HIP(hipMemsetAsync(b->call_new, 0, b->ncalls, ctx->stream));
		k_shard_unpart<<<grid_for(b->ncalls * 64, 256, 4096), 256, 0, ctx->stream>>>(*b, d_send_pos, d_back_flags);
		SYZ_HIP(hipGetLastError());
	}
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	return SYZSIG_OK;
}

}  // extern "C"
