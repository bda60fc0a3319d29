// sort.hip -- a stable LSD radix sort of (u32 key, u32 value) pairs, for the
// small sorts of the path: Minimize's context order by (Len desc, index asc)
// (minimize.hip; pkg/signal/signal.go:138-166 sorts the inputs by Len before
// the greedy pass).  200k contexts at C3: microseconds, so it is written for
// simplicity, not speed -- no library sort.
//
// One pass per 8-bit digit of the keys' significant bits.  Per pass: k_rs_hist counts each tile's digits
// (tiles of kRsTile keys, one wave each), k_rs_scan turns the digit-major
// counts into every (digit, tile) run's place, and k_rs_scatter writes the
// tile's keys in order: one wave walks its tile 64 keys at a time, a key's rank
// among the earlier keys of its digit in that step from eight ballots (the
// lanes whose digit equals its own), the digit's running position in LDS.  A
// single wave per tile keeps every LDS update in program order, so the pass
// is stable without a barrier.
#include <algorithm>

#include "internal.h"

namespace syz {

constexpr uint32_t kRsTile = 1024;  // keys per tile (one wave)

__global__ __launch_bounds__(64) void k_rs_hist(const uint32_t* __restrict__ keys, uint32_t n, uint32_t shift,
                                                uint32_t ntiles, uint32_t* hist)
{
	__shared__ uint32_t h[256];
	const uint32_t lane = threadIdx.x, t = blockIdx.x, i0 = t * kRsTile;
	for (uint32_t d = lane; d < 256; d += 64)
		h[d] = 0;
	__builtin_amdgcn_wave_barrier();
	for (uint32_t i = i0 + lane; i < min(n, i0 + kRsTile); i += 64)
		atomicAdd(&h[(keys[i] >> shift) & 255], 1u);
	__builtin_amdgcn_wave_barrier();
	for (uint32_t d = lane; d < 256; d += 64)
		hist[(uint64_t)d * ntiles + t] = h[d];
}

// exclusive scan of m counts in place (one workgroup): 1024 counts per step,
// coalesced, a block scan each, the running total carried
__global__ __launch_bounds__(1024) void k_rs_scan(uint32_t* v, uint32_t m)
{
	__shared__ uint32_t wsum[16];
	__shared__ uint32_t s_carry;
	const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
	if (tid == 0)
		s_carry = 0;
	for (uint32_t b = 0; b < m; b += 1024) {
		const uint32_t i = b + tid;
		const uint32_t x = i < m ? v[i] : 0;
		uint32_t inc = x;
#pragma unroll
		for (uint32_t d = 1; d < 64; d <<= 1) {
			const uint32_t y = __shfl_up(inc, d, 64);
			inc += lane >= d ? y : 0;
		}
		if (lane == 63)
			wsum[w] = inc;
		__syncthreads();
		uint32_t pre = s_carry, tot = 0;
		for (uint32_t k = 0; k < 16; k++) {
			pre += k < w ? wsum[k] : 0;
			tot += wsum[k];
		}
		if (i < m)
			v[i] = pre + inc - x;
		__syncthreads();  // wsum and s_carry are rewritten by the next step
		if (tid == 0)
			s_carry += tot;
	}
}

__global__ __launch_bounds__(64) void k_rs_scatter(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                   uint32_t n, uint32_t shift, uint32_t ntiles,
                                                   const uint32_t* __restrict__ off, uint32_t* kout, uint32_t* vout)
{
	__shared__ uint32_t run[256];
	const uint32_t lane = threadIdx.x, t = blockIdx.x, i0 = t * kRsTile;
	for (uint32_t d = lane; d < 256; d += 64)
		run[d] = off[(uint64_t)d * ntiles + t];
	__builtin_amdgcn_wave_barrier();
	const uint64_t below = (1ull << lane) - 1;
	for (uint32_t s = i0; s < min(n, i0 + kRsTile); s += 64) {
		const uint32_t i = s + lane;
		const bool valid = i < n;
		const uint32_t k = valid ? kin[i] : 0, d = (k >> shift) & 255;
		uint64_t peers = __ballot(valid);
#pragma unroll
		for (uint32_t b = 0; b < 8; b++) {
			const uint64_t m = __ballot((d >> b) & 1);
			peers &= (d >> b) & 1 ? m : ~m;
		}
		const uint32_t pos = run[d] + (uint32_t)__popcll(peers & below);
		if (valid) {
			kout[pos] = k;
			vout[pos] = vin[i];
		}
		__builtin_amdgcn_wave_barrier();
		if (valid && (peers & below) == 0)  // the digit's first lane moves its run on
			run[d] += (uint32_t)__popcll(peers);
		__builtin_amdgcn_wave_barrier();
	}
}

int radix_sort_pairs(syzsig_ctx* ctx, uint32_t* keys, uint32_t* vals, uint32_t* keys_tmp, uint32_t* vals_tmp,
                     uint32_t n, uint32_t key_bits, uint32_t** keys_out, uint32_t** vals_out, int ws_slot)
{
	*keys_out = keys;
	*vals_out = vals;
	if (n == 0)
		return SYZSIG_OK;
	const uint32_t ntiles = (n + kRsTile - 1) / kRsTile;
	void* wh;
	SYZ_TRY(ws_get(ctx, ws_slot, (uint64_t)256 * ntiles * 4 + 64, &wh));
	uint32_t* hist = (uint32_t*)wh;
	const hipStream_t s = ctx->stream;
	uint32_t *ki = keys, *vi = vals, *ko = keys_tmp, *vo = vals_tmp;
	for (uint32_t shift = 0; shift < std::min(key_bits, 32u); shift += 8) {  // (keys < 2^key_bits)
		k_rs_hist<<<ntiles, 64, 0, s>>>(ki, n, shift, ntiles, hist);
		k_rs_scan<<<1, 1024, 0, s>>>(hist, 256 * ntiles);
		k_rs_scatter<<<ntiles, 64, 0, s>>>(ki, vi, n, shift, ntiles, hist, ko, vo);
		std::swap(ki, ko);
		std::swap(vi, vo);
	}
	SYZ_HIP(hipGetLastError());
	*keys_out = ki;
	*vals_out = vi;
	return SYZSIG_OK;
}

}  // namespace syz
