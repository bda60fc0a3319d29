// edge.hip -- K1 (trace -> edge signal) + K2 (the executor's lossy dedup),
// bit-exact with executor/executor.h:492-512 write_coverage_signal<uint64>,
// :677-685 hash and :687-706 dedup, and executor_linux.cc:196-204 cover_check.
//
// One 64-lane workgroup per program (= one forked executor child): the 32 KB
// dedup table lives in LDS for the program's lifetime, calls run in order.
// K1 is data-parallel: sig_i = (u32)pc_i ^ hash((u32)pc_{i-1}) with the
// previous PC's hash taken from the neighbour lane.  K2 is a sequential state
// machine, parallelised exactly.  Signal i reads only its 4-slot window
// {h, h+1, h+2, h+3} (h = sig % 8192) and writes at most one slot of it (insert
// at the first empty slot, or the forced overwrite at h); a duplicate writes
// nothing.  Per 64-signal chunk, lanes run in rounds:
//   1. every pending lane evaluates dedup() against the table as it stands
//      (read only): duplicate, or a write at some slot of its window;
//   2. writers mark the 8-slot bins their window touches (LDS stamps keep the
//      earliest marking lane per bin); a pending lane with an EARLIER marker in
//      its bins is blocked -- and marks its own bins too, since its re-run may
//      turn into a write (repeated until no new marks);
//   3. unblocked lanes are final: writers store, everyone leaves the round.
// A final lane has only final duplicates before it inside its window, and
// duplicates change nothing, so it saw exactly the sequential table state;
// a lane after it that writes into its window does so after it read.  Mostly
// duplicates (repeated edges) therefore finish in one round.
// Latency: the trace is read kEdgeDepth chunks ahead of the chunk being
// deduplicated (registers), so the HBM round trip overlaps LDS work.
#include "internal.h"

namespace syz {

constexpr uint32_t kBinShift = 3;  // 8-slot bins
constexpr uint32_t kBins = kDedupSize >> kBinShift;
constexpr uint32_t kEpochMax = 0xFFFFFF;
constexpr uint32_t kEdgeDepth = 8;  // chunks of 64 PCs in flight per wave

// The workgroup is ONE wave, so LDS traffic between its lanes needs no s_barrier
// -- and __syncthreads() would also drain every outstanding global load (the
// workgroup-scope release waits for vmcnt(0)), defeating the trace prefetch.
// A wave's DS instructions execute in order; wait for them (lgkmcnt(0) only)
// and keep the compiler from moving LDS accesses across.
__device__ __forceinline__ void wave_lds_sync()
{
	__builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
	__builtin_amdgcn_s_waitcnt(0xC07F);  // vmcnt/expcnt untouched, lgkmcnt(0)
	__builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ bool stamp_earlier(uint32_t s, uint32_t epoch, uint32_t lane)
{
	return (s >> 8) == epoch && 63 - (s & 255) < lane;
}

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
			const uint32_t nch = (len + 63) / 64;
			if (len == 0) {  // nothing to load (pcs may even be empty)
				if (lane == 0)
					sig_cnt[c] = 0;
				continue;
			}
			// Loads are unconditional (index clamped into the call, value masked
			// later): a load under a branch makes the compiler drain vmcnt(0)
			// before the first use, i.e. wait for the whole prefetch.
			const uint64_t last = start + (len ? len - 1 : 0);
			uint64_t buf[kEdgeDepth];
#pragma unroll
			for (uint32_t u = 0; u < kEdgeDepth; u++)
				buf[u] = pcs[min<uint64_t>(start + u * 64 + lane, last)];
			for (uint32_t g = 0; g < nch && !aborted; g += kEdgeDepth) {
				uint64_t cur[kEdgeDepth];
#pragma unroll
				for (uint32_t u = 0; u < kEdgeDepth; u++) {
					cur[u] = buf[u];
					buf[u] = pcs[min<uint64_t>(start + (g + kEdgeDepth + u) * 64 + lane, last)];
				}
#pragma unroll
				for (uint32_t u = 0; u < kEdgeDepth; u++) {
					if (g + u >= nch)
						break;
					const uint32_t j = (g + u) * 64 + lane;
					const bool valid = j < len;
					const uint64_t pc = valid ? cur[u] : 0;
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
						// 1. evaluate dedup() (executor.h:692-706, literally) on the current table
						bool writer = false;
						uint32_t wpos = home;
						if (pending) {
							uint32_t t[4];
#pragma unroll
							for (uint32_t i = 0; i < 4; i++)
								t[i] = table[(sig + i) & (kDedupSize - 1)];
							bool decided = false;
#pragma unroll
							for (uint32_t i = 0; i < 4; i++) {
								if (!decided && t[i] == sig) {
									decided = true;  // duplicate
								} else if (!decided && t[i] == 0) {
									decided = true;
									writer = true;
									wpos = (sig + i) & (kDedupSize - 1);
								}
							}
							writer = writer || !decided;  // all 4 taken: forced overwrite at home
						}
						// 2. mark / block until stable
						if (epoch == kEpochMax) {
							for (uint32_t i = lane; i < kBins; i += 64)
								stamp[i] = 0;
							epoch = 0;
							wave_lds_sync();
						}
						epoch++;
						const uint32_t v = (epoch << 8) | (63 - lane);
						bool marker = pending && writer, blocked = false;
						bool mark_now = marker;
						for (;;) {
							if (mark_now) {
								atomicMax(&stamp[b0], v);
								if (b1 != b0)
									atomicMax(&stamp[b1], v);
							}
							wave_lds_sync();
							blocked = pending && (stamp_earlier(stamp[b0], epoch, lane) ||
							                      stamp_earlier(stamp[b1], epoch, lane));
							mark_now = blocked && !marker;
							marker = marker || mark_now;
							if (!__ballot(mark_now))
								break;
						}
						// 3. final lanes commit
						if (pending && !blocked) {
							if (writer)
								table[wpos] = sig;
							emit = writer;
							pending = false;
						}
						wave_lds_sync();
					}
					const uint64_t m = __ballot(emit);
					if (emit)
						sigs[start + nsig + lane_rank(m)] = sig;  // write_output order == trace order
					nsig += (uint32_t)__popcll(m);
				}
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
