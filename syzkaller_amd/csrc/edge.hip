// edge.hip -- K1 (trace -> edge signal) + K2 (the executor's lossy dedup),
// bit-exact with executor/executor.h:492-512 write_coverage_signal<uint64>,
// :677-685 hash and :687-706 dedup, and executor_linux.cc:196-204 cover_check.
//
// One workgroup of kEdgeWaves waves per program (= one forked executor
// child): the 32 KB dedup table lives in LDS for the program's lifetime, calls
// run in order, and the trace goes through in chunks of kEdgeChunk = 256
// signals (4 per CU: the table bounds residency, so the waves of a program
// are what fills the SIMDs).  K1 is data-parallel: sig_i = (u32)pc_i ^
// hash((u32)pc_{i-1}), the previous PC's hash taken from the lane below
// (across waves through LDS, across chunks from a carry).  K2 is a sequential
// state machine, parallelised exactly.  Signal i reads only its 4-slot window
// {h, h+1, h+2, h+3} (h = sig % 8192) and writes at most one slot of it
// (insert at the first empty slot, or the forced overwrite at h); a duplicate
// writes nothing.  Per chunk, lanes run in rounds:
//   1. every pending lane evaluates dedup() against the table as it stands
//      (read only): duplicate, or a write at some slot of its window;
//   2. writers mark the 8-slot bins their window touches (LDS stamps keep the
//      earliest marking position per bin); a pending lane with an EARLIER
//      marker in its bins is blocked -- and marks its own bins too, since its
//      re-run may turn into a write (repeated until no new marks);
//   3. unblocked lanes are final: writers store, everyone leaves the round.
// A final lane has only final duplicates before it inside its window, and
// duplicates change nothing, so it saw exactly the sequential table state;
// a lane after it that writes into its window does so after it read.  Mostly
// duplicates (repeated edges) therefore finish in few rounds (3.1 per 256-signal
// chunk at C2, against 1.8 per 64-signal chunk: 2.3x fewer rounds per signal).
// Rounds need workgroup barriers; they are LDS-only (lds_barrier), so the
// trace loads in flight are never drained.  The trace is read kEdgeDepth
// chunks ahead of the chunk being deduplicated, ping-ponging between two
// register buffers.
#include "internal.h"

namespace syz {

constexpr uint32_t kBinShift = 3;  // 8-slot bins
constexpr uint32_t kBins = kDedupSize >> kBinShift;
constexpr uint32_t kEdgeDepth = 4;  // chunks in flight per buffer

// Geometry of one variant: W waves per program, chunks of 64 * W signals; a
// conflict stamp is epoch << kPosBits | (chunk - 1 - position).
template <uint32_t W>
struct EdgeGeom {
	static constexpr uint32_t kChunk = 64 * W;
	static constexpr uint32_t kPosBits = W <= 4 ? 8 : 9;
	static constexpr uint32_t kPosMask = (1u << kPosBits) - 1;
	static constexpr uint32_t kEpochMax = (1u << (32 - kPosBits)) - 1;
	static_assert(kChunk <= (1u << kPosBits), "stamp position field");
};

// Workgroup barrier that orders LDS only: a plain __syncthreads() is also a
// release of global memory, i.e. it waits for every global load in flight.
__device__ __forceinline__ void lds_barrier()
{
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
	__builtin_amdgcn_s_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// A bin's stamp is the max of epoch << kPosBits | (kPosMask - position) over
// this epoch's markers (older epochs compare lower): it was set by a position
// before mine this epoch  <=>  stamp > my own v = epoch << kPosBits | (kPosMask - pos).

template <uint32_t W>
__global__ __launch_bounds__(64 * W) void k_edge_dedup(const uint64_t* __restrict__ pcs, uint64_t npc,
                                                           const uint64_t* __restrict__ call_start,
                                                           const uint32_t* __restrict__ call_len, uint64_t ncalls,
                                                           const uint32_t* __restrict__ prog_call, uint64_t nprog,
                                                           uint32_t* sigs, uint32_t* sig_cnt, uint32_t* completed,
                                                           unsigned long long* cnt)
{
	using G = EdgeGeom<W>;
	constexpr uint32_t kEdgeWaves = W, kEdgeChunk = G::kChunk, kEpochMax = G::kEpochMax;
	__shared__ uint32_t table[kDedupSize];
	__shared__ uint32_t stamp[kBins];
	__shared__ __align__(16) uint32_t s_any[2][kEdgeWaves];
	__shared__ uint32_t s_carry[2][kEdgeWaves];
	const uint32_t lane = lane_id(), w = threadIdx.x >> 6, pos = threadIdx.x;  // pos: place in a chunk
	uint32_t seq = 0;
	// Workgroup OR of a predicate (one barrier): every wave writes its own
	// flag, ds_read_b128s read them all.  Two rows alternate: a row is
	// rewritten two calls later, after every wave passed the barrier between.
	// A wave may publish a payload with its flag (row[w] = payload << 1 | flag,
	// readable in `row` until the next call but one).
	const uint32_t* row = s_any[0];
	auto wg_any = [&](bool pred, uint32_t payload) -> bool {
		uint32_t* r = s_any[seq & 1];
		const uint32_t any = __ballot(pred) != 0;
		if (lane == 0)
			r[w] = payload << 1 | any;
		lds_barrier();
		uint32_t o = 0;
		if constexpr (W >= 4) {
#pragma unroll
			for (uint32_t i = 0; i < W / 4; i++) {
				const uint4 a = reinterpret_cast<const uint4*>(r)[i];
				o |= a.x | a.y | a.z | a.w;
			}
		} else {
#pragma unroll
			for (uint32_t i = 0; i < W; i++)
				o |= r[i];
		}
		seq++;
		row = r;
		return (o & 1) != 0;
	};
	uint64_t err = 0;
	uint32_t epoch = 0;
	for (uint64_t p = blockIdx.x; p < nprog; p += gridDim.x) {
		const uint64_t cb = prog_call[p], ce = prog_call[p + 1];
		if (cb > ce || ce > ncalls) {
			err += threadIdx.x == 0;
			continue;
		}
		// fresh table per program (common_linux.h:1995-2030: fork zeroes it)
		for (uint32_t i = threadIdx.x; i < kDedupSize / 4; i += kEdgeChunk)
			reinterpret_cast<uint4*>(table)[i] = make_uint4(0, 0, 0, 0);
		for (uint32_t i = threadIdx.x; i < kBins; i += kEdgeChunk)
			stamp[i] = 0;
		epoch = 0;
		lds_barrier();
		uint64_t done = ce - cb;
		bool aborted = false;
		for (uint64_t c = cb; c < ce && !aborted; c++) {
			const uint64_t start = call_start[c];
			const uint32_t len = call_len[c];
			if (len >= kCoverSize || start > npc || len > npc - start) {
				// executor_linux.cc:186-187 fail("too much cover") / malformed input
				err += threadIdx.x == 0;
				aborted = true;
				done = c - cb;
				break;
			}
			if (len == 0) {  // nothing to load (pcs may even be empty)
				if (threadIdx.x == 0)
					sig_cnt[c] = 0;
				continue;
			}
			uint32_t nsig = 0, carry = 0;  // carry: hash of the previous chunk's last PC
			const uint32_t nch = (len + kEdgeChunk - 1) / kEdgeChunk;
			const uint64_t last = start + len - 1;
			// Loads are unconditional (index clamped into the call, value masked
			// later): a load under a branch makes the compiler drain vmcnt(0)
			// before the first use, i.e. wait for the whole prefetch.
			auto fetch = [&](uint64_t (&buf)[kEdgeDepth], uint32_t g) {
#pragma unroll
				for (uint32_t u = 0; u < kEdgeDepth; u++)
					buf[u] = pcs[min<uint64_t>(start + (uint64_t)(g + u) * kEdgeChunk + pos, last)];
			};
			// chunk q of the call; false once the program aborts
			auto chunk = [&](uint64_t pcv, uint32_t q) -> bool {
				const uint32_t j = q * kEdgeChunk + pos;
				const bool valid = j < len;
				const uint64_t pc = valid ? pcv : 0;
				const uint32_t h = exec_hash((uint32_t)pc);
				uint32_t up = __shfl_up(h, 1, 64);
				if (lane == 63)
					s_carry[q & 1][w] = h;
				// cover_check (executor_linux.cc:196-204): doexit(0), this call and
				// the rest of the program publish nothing
				if (wg_any(valid && !cover_check(pc), 0))
					return false;
				if (lane == 0)
					up = w == 0 ? carry : s_carry[q & 1][w - 1];
				carry = s_carry[q & 1][kEdgeWaves - 1];
				const uint32_t sig = (uint32_t)pc ^ up;
				const uint32_t home = sig & (kDedupSize - 1);
				const uint32_t b0 = home >> kBinShift, b1 = ((home + 3) & (kDedupSize - 1)) >> kBinShift;
				bool pending = valid, emit = false;
				// rounds until no lane is pending (a chunk always has a valid lane, so
				// the first round needs no test); the test after the last round also
				// publishes every wave's emit count for the output below
				for (;;) {
					// 1. evaluate dedup() (executor.h:692-706) on the current table,
					// branch-free: the first probe i with T[h+i] == sig (duplicate)
					// or T[h+i] == 0 (insert there), else the forced overwrite at h
					uint32_t eqm = 0, zm = 0;
#pragma unroll
					for (uint32_t i = 0; i < 4; i++) {
						const uint32_t t = table[(sig + i) & (kDedupSize - 1)];
						eqm |= (uint32_t)(t == sig) << i;
						zm |= (uint32_t)(t == 0) << i;
					}
					const uint32_t first = __builtin_ctz(eqm | zm | 16u);
					const bool writer = !((eqm >> first) & 1);
					const uint32_t wpos = (sig + (first & 3)) & (kDedupSize - 1);
					// 2. mark / block until stable
					if (epoch == kEpochMax) {
						for (uint32_t i = threadIdx.x; i < kBins; i += kEdgeChunk)
							stamp[i] = 0;
						epoch = 0;
						lds_barrier();
					}
					epoch++;
					const uint32_t v = (epoch << G::kPosBits) | (G::kPosMask - pos);
					bool marker = pending && writer, blocked = false;
					bool mark_now = marker;
					for (;;) {
						if (mark_now) {
							atomicMax(&stamp[b0], v);
							if (b1 != b0)
								atomicMax(&stamp[b1], v);
						}
						lds_barrier();
						const uint32_t s0 = stamp[b0], s1 = stamp[b1];
						blocked = pending && (s0 > v || s1 > v);
						mark_now = blocked && !marker;
						marker = marker || mark_now;
						if (!wg_any(mark_now, 0))
							break;
					}
					// 3. final lanes commit (visible after the next round's barrier)
					const bool fin_w = pending && !blocked && writer;
					if (fin_w)
						table[wpos] = sig;
					emit = emit || fin_w;
					pending = pending && blocked;
					if (!wg_any(pending, (uint32_t)__popcll(__ballot(emit))))
						break;
				}
				// write_output order == trace order: waves in order, lanes in order
				const uint64_t m = __ballot(emit);
				uint32_t base = nsig, tot = 0;
#pragma unroll
				for (uint32_t i = 0; i < kEdgeWaves; i++) {
					const uint32_t x = row[i] >> 1;
					base += i < w ? x : 0;
					tot += x;
				}
				if (emit)
					sigs[start + base + lane_rank(m)] = sig;
				nsig += tot;
				return true;
			};
			auto run = [&](const uint64_t (&buf)[kEdgeDepth], uint32_t g) -> bool {
#pragma unroll
				for (uint32_t u = 0; u < kEdgeDepth; u++)
					if (g + u < nch && !chunk(buf[u], g + u))
						return false;
				return true;
			};
			uint64_t ba[kEdgeDepth], bb[kEdgeDepth];
			fetch(ba, 0);
			for (uint32_t g = 0;;) {
				fetch(bb, g + kEdgeDepth);
				if (!run(ba, g)) {
					aborted = true;
					break;
				}
				g += kEdgeDepth;
				if (g >= nch)
					break;
				fetch(ba, g + kEdgeDepth);
				if (!run(bb, g)) {
					aborted = true;
					break;
				}
				g += kEdgeDepth;
				if (g >= nch)
					break;
			}
			if (aborted) {
				done = c - cb;
				break;
			}
			if (threadIdx.x == 0)
				sig_cnt[c] = nsig;
		}
		// calls not published (aborted and later) report no signal (ipc.go:362-365)
		for (uint64_t c = cb + done + threadIdx.x; c < ce; c += kEdgeChunk)
			sig_cnt[c] = 0;
		if (threadIdx.x == 0)
			completed[p] = (uint32_t)done;
		lds_barrier();  // the table is re-zeroed for the next program
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
	SYZ_LOCK(ctx);
	if (!ctx || (nprog && (!d_prog_call || !d_completed)) || (ncalls && (!d_call_start || !d_call_len || !d_sig_cnt)) ||
	    (npc && (!d_pcs || !d_sigs)))
		return fail(SYZSIG_EINVAL, "edge_derive: NULL argument");
	if (nprog == 0)
		return SYZSIG_OK;
	SYZ_TRY(counters_reset(ctx));
	// 4 programs per CU (the 32 KB dedup tables bound residency); W waves each
	const int grid = (int)std::min<uint64_t>(nprog, 256 * 4);
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[0], ctx->stream));
#ifdef SYZ_EXPERIMENTS
	// measured slower: 8 waves 25 ms, 2 waves 16.1, 1 wave 21.3 vs 4 waves 14.9 at C2
	if (ctx->edge_waves == 8)
		k_edge_dedup<8><<<grid, 512, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls, d_prog_call,
		                                               nprog, d_sigs, d_sig_cnt, d_completed, ctx->d_cnt);
	else if (ctx->edge_waves == 2)
		k_edge_dedup<2><<<grid, 128, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls, d_prog_call,
		                                               nprog, d_sigs, d_sig_cnt, d_completed, ctx->d_cnt);
	else if (ctx->edge_waves == 1)
		k_edge_dedup<1><<<grid, 64, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls, d_prog_call,
		                                              nprog, d_sigs, d_sig_cnt, d_completed, ctx->d_cnt);
	else
#endif
		k_edge_dedup<4><<<grid, 256, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls, d_prog_call,
		                                               nprog, d_sigs, d_sig_cnt, d_completed, ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[1], ctx->stream));
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->timing) {
		float t = 0;
		SYZ_HIP(hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]));
		ctx->last_ms = t;
	}
	if (ctx->h_cnt[kCntError])
		return fail(SYZSIG_EINVAL, "edge_derive: malformed program/call ranges or a call with >= 262144 PCs");
	return SYZSIG_OK;
}
