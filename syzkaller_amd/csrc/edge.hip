// edge.hip -- K1 (trace -> edge signal) + K2 (the executor's lossy dedup),
// bit-exact with executor/executor.h:492-512 write_coverage_signal<uint64>,
// :677-685 hash and :687-706 dedup, and executor_linux.cc:196-204 cover_check.
//
// One 64-lane workgroup per program (= one forked executor child): the 32 KB
// dedup table lives in LDS for the program's lifetime, calls run in order.
// K1 is data-parallel: sig_i = (u32)pc_i ^ hash((u32)pc_{i-1}) with the
// previous PC's hash taken from the neighbour lane.  K2 is a sequential state
// machine, parallelised exactly: signal i touches only its 4-slot window
// {h, h+1, h+2, h+3} (h = sig % 8192, forced overwrite at h), so operations
// with disjoint windows commute.  Per 64-signal chunk, lanes run in rounds; a
// lane runs once no EARLIER pending lane shares an 8-slot bin with its window
// (conflict stamps in LDS: atomicMax of round<<8 | (63-lane) per bin).  Every
// conflicting pair therefore keeps its trace order, which is all the
// sequential semantics depend on.
#include "internal.h"

namespace syz {

constexpr uint32_t kBinShift = 3;  // 8-slot bins
constexpr uint32_t kBins = kDedupSize >> kBinShift;
constexpr uint32_t kEpochMax = 0xFFFFFF;

__global__ __launch_bounds__(64) void k_edge_dedup(const uint64_t* __restrict__ pcs, uint64_t npc,
                                                   const uint64_t* __restrict__ call_start,
                                                   const uint32_t* __restrict__ call_len, uint64_t ncalls,
                                                   const uint32_t* __restrict__ prog_call, uint64_t nprog,
                                                   uint32_t* sigs, uint32_t* sig_cnt, uint32_t* completed,
                                                   unsigned long long* cnt)
{
	__shared__ uint32_t table[kDedupSize];
	__shared__ uint32_t stamp[kBins];
	const uint32_t lane = threadIdx.x;
	uint64_t err = 0;
	for (uint64_t p = blockIdx.x; p < nprog; p += gridDim.x) {
		const uint64_t cb = prog_call[p], ce = prog_call[p + 1];
		if (cb > ce || ce > ncalls) {
			err += lane == 0;
			continue;
		}
		// fresh table per program (common_linux.h:1995-2030: fork zeroes it)
		for (uint32_t i = lane; i < kDedupSize / 4; i += 64)
			reinterpret_cast<uint4*>(table)[i] = make_uint4(0, 0, 0, 0);
		for (uint32_t i = lane; i < kBins; i += 64)
			stamp[i] = 0;
		__syncthreads();
		uint32_t epoch = 0;
		uint64_t done = ce - cb;
		bool aborted = false;
		for (uint64_t c = cb; c < ce && !aborted; c++) {
			const uint64_t start = call_start[c];
			const uint32_t len = call_len[c];
			if (len >= kCoverSize || start > npc || len > npc - start) {
				// executor_linux.cc:186-187 fail("too much cover") / malformed input
				err += lane == 0;
				aborted = true;
				done = c - cb;
				break;
			}
			uint32_t nsig = 0, carry = 0;
			uint64_t next = lane < len ? pcs[start + lane] : 0;
			for (uint32_t base = 0; base < len; base += 64) {
				const uint32_t j = base + lane;
				const bool valid = j < len;
				const uint64_t pc = next;
				next = (j + 64 < len) ? pcs[start + j + 64] : 0;  // prefetch the next chunk
				if (__ballot(valid && !cover_check(pc))) {
					aborted = true;  // doexit(0): this call and the rest publish nothing
					done = c - cb;
					break;
				}
				const uint32_t h = exec_hash((uint32_t)pc);
				const uint32_t up = __shfl_up(h, 1, 64);
				const uint32_t sig = (uint32_t)pc ^ (lane == 0 ? carry : up);
				carry = __shfl(h, 63, 64);
				const uint32_t home = sig & (kDedupSize - 1);
				const uint32_t b0 = home >> kBinShift, b1 = ((home + 3) & (kDedupSize - 1)) >> kBinShift;
				bool pending = valid, emit = false;
				while (__ballot(pending)) {
					if (epoch == kEpochMax) {
						for (uint32_t i = lane; i < kBins; i += 64)
							stamp[i] = 0;
						epoch = 0;
						__syncthreads();
					}
					epoch++;
					const uint32_t v = (epoch << 8) | (63 - lane);
					if (pending) {
						atomicMax(&stamp[b0], v);
						if (b1 != b0)
							atomicMax(&stamp[b1], v);
					}
					__syncthreads();
					bool conflict = false;
					if (pending) {
						const uint32_t s0 = stamp[b0], s1 = stamp[b1];
						conflict = ((s0 >> 8) == epoch && 63 - (s0 & 255) < lane) ||
						           ((s1 >> 8) == epoch && 63 - (s1 & 255) < lane);
					}
					if (pending && !conflict) {
						// executor.h:692-706, literally
						bool dup = false, placed = false;
#pragma unroll
						for (uint32_t i = 0; i < 4; i++) {
							const uint32_t pos = (sig + i) & (kDedupSize - 1);
							const uint32_t t = table[pos];
							if (t == sig) {
								dup = true;
								break;
							}
							if (t == 0) {
								table[pos] = sig;
								placed = true;
								break;
							}
						}
						if (!dup && !placed)
							table[home] = sig;
						emit = !dup;
						pending = false;
					}
					__syncthreads();
				}
				const uint64_t m = __ballot(emit);
				if (emit)
					sigs[start + nsig + lane_rank(m)] = sig;  // write_output order == trace order
				nsig += (uint32_t)__popcll(m);
			}
			if (!aborted && lane == 0)
				sig_cnt[c] = nsig;
		}
		// calls not published (aborted and later) report no signal (ipc.go:362-365)
		for (uint64_t c = cb + done + lane; c < ce; c += 64)
			sig_cnt[c] = 0;
		if (lane == 0)
			completed[p] = (uint32_t)done;
		__syncthreads();
	}
	block_count(&cnt[kCntError], err);
}

}  // namespace syz

using namespace syz;

extern "C" int syzsig_edge_derive_dev(syzsig_ctx* ctx, const uint64_t* d_pcs, uint64_t npc,
                                      const uint64_t* d_call_start, const uint32_t* d_call_len, uint64_t ncalls,
                                      const uint32_t* d_prog_call, uint64_t nprog, uint32_t* d_sigs,
                                      uint32_t* d_sig_cnt, uint32_t* d_completed)
{
	if (!ctx || (nprog && (!d_prog_call || !d_completed)) || (ncalls && (!d_call_start || !d_call_len || !d_sig_cnt)) ||
	    (npc && (!d_pcs || !d_sigs)))
		return fail(SYZSIG_EINVAL, "edge_derive: NULL argument");
	if (nprog == 0)
		return SYZSIG_OK;
	SYZ_TRY(counters_reset(ctx));
	const int grid = (int)std::min<uint64_t>(nprog, 256 * 4);
	k_edge_dedup<<<grid, 64, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls, d_prog_call, nprog,
	                                           d_sigs, d_sig_cnt, d_completed, ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->h_cnt[kCntError])
		return fail(SYZSIG_EINVAL, "edge_derive: malformed program/call ranges or a call with >= 262144 PCs");
	return SYZSIG_OK;
}
