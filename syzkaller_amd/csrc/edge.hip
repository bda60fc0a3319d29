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
// (across waves through LDS, across chunks from a carry; for all the chunks of
// a prefetch group under one barrier).  K2 is a sequential
// state machine, parallelised exactly.  Signal i reads only its 4-slot window
// {h, h+1, h+2, h+3} (h = sig % 8192) and writes at most one slot of it
// (insert at the first empty slot, or the forced overwrite at h); a duplicate
// writes nothing.  Per chunk, lanes run in rounds:
//   1. every pending lane evaluates dedup() against the table as it stands
//      (read only): its DECISION slot d (the first match or zero of its
//      window, or h for the forced overwrite), and whether it writes there;
//   2. lanes mark slots (8-slot bin stamps keep the earliest marking position
//      per bin; per-slot bits count markers up to two).  A pending lane is
//      blocked iff an earlier lane marked d's bin and another lane marked d
//      itself (conservative about which lane: the earliest pending lane is
//      never blocked, so every round finalises at least one); a blocked lane
//      marks too, and marking repeats until no new marks.  Writers mark in the
//      first pass (in the mark-all mode every pending lane does, which is the
//      passes' fixed point at once).  What a lane marks: every slot it can
//      write, now or after a re-run -- h and its window's slots that are empty
//      now -- and, when blocked, d (a later lane must not write what it will
//      read again);
//   3. unblocked lanes are final: writers store, everyone leaves the round.
// Why that is exact: a lane's outcome depends on d only, as long as no slot
// of its window becomes empty again.  An earlier write of a nonzero value !=
// sig before d changes none of the predicates it evaluated (and an earlier
// lane with the same sig has the same d), a write at d is marked, and a later
// final lane writes only slots no pending earlier lane can still read.  The
// one write that empties a slot is the forced overwrite of sig == 0, which
// stores 0 at slot 0 (executor.h:704).  Inside a window holding slot 0 (h in
// 8189..8191, 0) a slot can therefore hold sig while slot 0 before it is
// empty, so the lane's decision can move past today's d once slot 0 fills
// again, and a later zero write changes a slot it read.  Hence two more marks
// (tests/test_edge_rounds_cpu.py restates them and stresses them against
// sequential dedup on zero-heavy chunks; golden executor_zero2 pins them):
//   - a lane whose window holds slot 0 marks its whole window;
//   - a sig == 0 lane marks 8189..8191 and 0..3: every decision slot of a
//     window holding slot 0, so such a later lane waits for the zero write.
// A final lane has no earlier pending writer that could touch what it read,
// and duplicates change nothing, so its outcome is the sequential one.
// The same invariant says that after any round the pending lanes, run in
// trace order on the table as it stands, give the sequential outcome: once a
// round leaves at most kEdgeSeqMax lanes pending (7 per 256-signal chunk on
// average on the global walk), one wave runs them through plain dedup, one
// signal per step, instead of further rounds and their barriers.
// After the first round 7 of 256 lanes are pending on average on the global
// walk (19.5 on the region walk; host simulation).
// Rounds need workgroup barriers; they are LDS-only (lds_barrier), so the
// trace loads in flight are never drained.  The trace is read kEdgeDepth
// chunks ahead of the chunk being deduplicated, ping-ponging between two
// register buffers.
#include "internal.h"

namespace syz {

constexpr uint32_t kBinShift = 3;  // 8-slot bins
constexpr uint32_t kBins = kDedupSize >> kBinShift;
#ifndef SYZ_EDGE_DEPTH
#define SYZ_EDGE_DEPTH 4
#endif
// trace signals in flight per lane per buffer; every chunk of a buffer is a
// copy of the chunk code (the instruction cache bounds how many fit)
constexpr uint32_t kEdgeDepthSignals = SYZ_EDGE_DEPTH;
#ifndef SYZ_EDGE_KS
#define SYZ_EDGE_KS 1
#endif
constexpr uint32_t kEdgeKS = SYZ_EDGE_KS;  // signals per lane per chunk
#ifndef SYZ_EDGE_SEQ
#define SYZ_EDGE_SEQ 32
#endif
#ifndef SYZ_EDGE_GROUP_K1
#define SYZ_EDGE_GROUP_K1 1
#endif
// a round that leaves at most this many lanes pending hands them to one wave,
// which runs them through plain dedup in trace order (0: rounds only)
constexpr uint32_t kEdgeSeqMax = SYZ_EDGE_SEQ;
static_assert(kEdgeSeqMax <= 32, "the tail's masks are 32 bits");
// Two marking modes, one kernel instantiation each (both exact; one code
// path per kernel keeps it small and straight):
//   passes   -- writers mark, blocked lanes mark in further passes until no
//               new marks (one workgroup OR per pass);
//   mark-all -- every pending lane marks in the one pass (its write slots and
//               d: the passes' fixed point at once, extra marks only block
//               more), no second workgroup OR per round.  On a thrashing table
//               almost every lane is a writer and marks anyway, so it costs no
//               blocking there; on mostly-duplicate traces it blocks more.
// The host picks per launch from the previous launch's duplicate rate.
constexpr uint32_t kEdgeMarkAllMaxDupPct = 5;  // mark-all below 5 % first-round duplicates

// Geometry of one variant: W waves per program, KS signals per lane, chunks of
// 64 * W * KS signals (lane l of wave w holds positions k * 64 W + 64 w + l,
// k < KS); a conflict stamp is epoch << kPosBits | (kPosMask - position).
template <uint32_t W, uint32_t KS>
struct EdgeGeom {
	static constexpr uint32_t kLanes = 64 * W;
	static constexpr uint32_t kChunk = kLanes * KS;
	static constexpr uint32_t kPosBits = kChunk <= 256 ? 8 : kChunk <= 512 ? 9 : 10;
	static constexpr uint32_t kPosMask = (1u << kPosBits) - 1;
	static constexpr uint32_t kEpochMax = (1u << (32 - kPosBits)) - 1;
	static constexpr uint32_t kDepth = kEdgeDepthSignals / KS;  // chunks in flight per buffer
	static_assert(kChunk <= (1u << kPosBits), "stamp position field");
	static_assert(KS >= 1 && KS <= 3 && kDepth >= 1, "emit counts: 8 bits per signal slot in a 31-bit payload");
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

template <uint32_t W, uint32_t KS, bool kMarkAll>
__global__ __launch_bounds__(64 * W) void k_edge_dedup(const uint64_t* __restrict__ pcs, uint64_t npc,
                                                           const uint64_t* __restrict__ call_start,
                                                           const uint32_t* __restrict__ call_len, uint64_t ncalls,
                                                           const uint32_t* __restrict__ prog_call, uint64_t nprog,
                                                           uint32_t* sigs, uint32_t* sig_cnt, uint32_t* completed,
                                                           unsigned long long* cnt)
{
	using G = EdgeGeom<W, KS>;
	constexpr uint32_t kEdgeWaves = W, kLanes = G::kLanes, kEdgeChunk = G::kChunk, kEpochMax = G::kEpochMax;
	constexpr uint32_t kDepth = G::kDepth;
	// (+ a mirror of slots 0..2 past the end: a window reads h..h+3 without
	// wrapping, two ds_read2 instead of four reads; every store goes through
	// tstore)
	__shared__ __align__(16) uint32_t table[kDedupSize + 4];
	auto tstore = [&](uint32_t slot, uint32_t val) {
		table[slot] = val;
		if (slot < 3)
			table[kDedupSize + slot] = val;
	};
	__shared__ uint32_t stamp[kBins];
	// per-slot marks of the current round: fm1 = marked at least once, fm2 =
	// marked at least twice (2 KB: four programs still fit a CU's LDS)
	__shared__ uint32_t fm1[kDedupSize / 32], fm2[kDedupSize / 32];
	__shared__ __align__(16) uint32_t s_any[2][kEdgeWaves];
	// K1 for a whole prefetch group of kDepth chunks at once (KS == 1): one
	// barrier exchanges the waves' boundary hashes and cover_check verdicts of
	// all of them, instead of one per chunk
	constexpr bool kGroupK1 = KS == 1 && SYZ_EDGE_GROUP_K1;
	__shared__ uint32_t s_carry[kGroupK1 ? kDepth : 2][KS][kEdgeWaves];
	// the tail (KS == 1): each wave's pending signals packed, and per wave the
	// tail's emitted ones by rank
	constexpr bool kSeq = KS == 1 && W == 4 && kEdgeSeqMax > 0;  // (the tail assumes 256 lanes)
	__shared__ __align__(16) uint32_t s_sig[kSeq ? kLanes : 1];
	__shared__ uint32_t s_th[kSeq ? 32 : 1];  // the tail's window homes
	__shared__ uint64_t s_pm[kEdgeWaves];
	const uint32_t lane = lane_id(), w = threadIdx.x >> 6, pos = threadIdx.x;  // pos: place in a sub-chunk
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
	uint64_t dups = 0;  // first-round duplicates of every chunk (uniform; the host's mode choice)
	for (uint64_t p = blockIdx.x; p < nprog; p += gridDim.x) {
		const uint64_t cb = prog_call[p], ce = prog_call[p + 1];
		if (cb > ce || ce > ncalls) {
			err += threadIdx.x == 0;
			continue;
		}
		// fresh table per program (common_linux.h:1995-2030: fork zeroes it)
		for (uint32_t i = threadIdx.x; i < kDedupSize / 4 + 1; i += kLanes)
			reinterpret_cast<uint4*>(table)[i] = make_uint4(0, 0, 0, 0);
		for (uint32_t i = threadIdx.x; i < kBins; i += kLanes)
			stamp[i] = 0;
		for (uint32_t i = threadIdx.x; i < kDedupSize / 32; i += kLanes)
			fm1[i] = fm2[i] = 0;
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
			auto fetch = [&](uint64_t (&buf)[kDepth][KS], uint32_t g) {
#pragma unroll
				for (uint32_t u = 0; u < kDepth; u++)
#pragma unroll
					for (uint32_t k = 0; k < KS; k++)
						buf[u][k] = pcs[min<uint64_t>(start + (uint64_t)(g + u) * kEdgeChunk + k * kLanes + pos, last)];
			};
			// chunk q of the call; false once the program aborts
			auto chunk = [&](const uint64_t (&pcv)[KS], uint32_t sgv, uint32_t q) -> bool {
				uint32_t sig[KS], b0[KS], b1[KS], v[KS], wpos[KS];
				bool pending[KS], emit[KS], writer[KS], blocked[KS];
				bool bad = false;
				if constexpr (kGroupK1) {  // (its K1 ran for the whole group: `run`)
					pending[0] = q * kEdgeChunk + pos < len;
					sig[0] = sgv;
				}
#pragma unroll
				for (uint32_t k = 0; k < (kGroupK1 ? 0 : KS); k++) {
					const uint32_t j = q * kEdgeChunk + k * kLanes + pos;
					pending[k] = j < len;
					const uint64_t pc = pending[k] ? pcv[k] : 0;
					// cover_check (executor_linux.cc:196-204): doexit(0), this call and
					// the rest of the program publish nothing
					bad |= pending[k] && !cover_check(pc);
					const uint32_t h = exec_hash((uint32_t)pc);
					sig[k] = __shfl_up(h, 1, 64);
					if (lane == 63)
						s_carry[q & 1][k][w] = h;
					b0[k] = (uint32_t)pc;  // (the PC's low half, until the previous hash is known)
				}
				if (!kGroupK1 && wg_any(bad, 0))
					return false;
#pragma unroll
				for (uint32_t k = 0; k < KS; k++) {
					if constexpr (!kGroupK1) {
						uint32_t up = sig[k];
						if (lane == 0)
							up = w > 0 ? s_carry[q & 1][k][w - 1] : k > 0 ? s_carry[q & 1][k - 1][kEdgeWaves - 1] : carry;
						sig[k] = b0[k] ^ up;
					}
					const uint32_t home = sig[k] & (kDedupSize - 1);
					b0[k] = home >> kBinShift;
					b1[k] = ((home + 3) & (kDedupSize - 1)) >> kBinShift;
					emit[k] = false;
				}
				if constexpr (!kGroupK1)
					carry = s_carry[q & 1][KS - 1][kEdgeWaves - 1];
				// rounds until no lane is pending (a chunk always has a valid lane, so
				// the first round needs no test); the test after the last round also
				// publishes every wave's emit counts for the output below
				bool wb1[KS];  // the window's second bin takes a mark
				uint32_t pset[KS];  // window offsets the lane can write: 0 (h) and the empty slots
				bool first_round = true;
				// one round; 0: no lane pending, 1: the tail finished the chunk (output
				// written), 2: another round.  Instantiated per marking mode, so that
				// each is straight code.
				auto round = [&](auto ma_c) -> int {
					constexpr bool ma = decltype(ma_c)::value;
					bool dup[KS];
					// 1. evaluate dedup() (executor.h:692-706) on the current table,
					// branch-free: the first probe i with T[h+i] == sig (duplicate)
					// or T[h+i] == 0 (insert there), else the forced overwrite at h
#pragma unroll
					for (uint32_t k = 0; k < KS; k++) {
						uint32_t eqm = 0, zm = 0;
#pragma unroll
						for (uint32_t i = 0; i < 4; i++) {
							const uint32_t t = table[(sig[k] & (kDedupSize - 1)) + i];
							eqm |= (uint32_t)(t == sig[k]) << i;
							zm |= (uint32_t)(t == 0) << i;
						}
						const uint32_t first = __builtin_ctz(eqm | zm | 16u);
						writer[k] = !((eqm >> first) & 1);
						dup[k] = pending[k] && !writer[k];
						wpos[k] = (sig[k] + (first & 3)) & (kDedupSize - 1);
						// whatever it writes, now or after a re-run, goes to h or to a slot
						// that is empty now (only slot 0 ever becomes empty again); a window
						// holding slot 0 is marked whole (header); the second bin of the
						// window is marked only if a marked slot lies in it
						const uint32_t hs = sig[k] & (kDedupSize - 1);
						pset[k] = hs >= kDedupSize - 3 || hs == 0 ? 15u : 1u | zm;
						wb1[k] = b1[k] != b0[k] && (pset[k] >> (8u - (sig[k] & 7u))) != 0;
					}
					// 2. mark / block until stable
					if (epoch == kEpochMax) {
						for (uint32_t i = threadIdx.x; i < kBins; i += kLanes)
							stamp[i] = 0;
						epoch = 0;
						lds_barrier();
					}
					epoch++;
					// (the conflict rule: header of this file)
					uint32_t dbin[KS];
					bool mark_win[KS], win_marked[KS];
#pragma unroll
					for (uint32_t k = 0; k < KS; k++) {
						v[k] = (epoch << G::kPosBits) | (G::kPosMask - (k * kLanes + pos));
						dbin[k] = wpos[k] >> kBinShift;
						mark_win[k] = win_marked[k] = pending[k] && (ma || writer[k]);
						blocked[k] = false;
					}
					for (;;) {
#pragma unroll
						for (uint32_t k = 0; k < KS; k++) {
							if (mark_win[k]) {
								atomicMax(&stamp[b0[k]], v[k]);
								if (wb1[k])  // (rare on a full table: a branch, not a second atomic)
									atomicMax(&stamp[b1[k]], v[k]);
								// the slots themselves, counted up to two (a blocked lane also its
								// decision slot: a later lane must not write what it will read again)
								const uint32_t hs = sig[k] & (kDedupSize - 1), off = hs & 31;
								const uint64_t m = (uint64_t)(pset[k] | 1u << ((wpos[k] - sig[k]) & 3)) << off;
								const uint32_t wa = hs >> 5, wbw = (wa + 1) & (kDedupSize / 32 - 1);
								const uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
								const uint32_t oa = atomicOr(&fm1[wa], lo);
								atomicOr(&fm2[wa], oa & lo);  // (0: nothing; no branch)
								if (hi) {
									const uint32_t ob = atomicOr(&fm1[wbw], hi);
									if (ob & hi)
										atomicOr(&fm2[wbw], ob & hi);
								}
								if (sig[k] == 0) {
									// the zero write empties slot 0: it also marks 8189..8191 (with
									// 0..3, every decision slot of a window that holds slot 0)
									constexpr uint32_t zw = kDedupSize / 32 - 1, zb = 7u << 29;
									atomicMax(&stamp[kBins - 1], v[k]);
									const uint32_t oz = atomicOr(&fm1[zw], zb);
									if (oz & zb)
										atomicOr(&fm2[zw], oz & zb);
								}
							}
						}
						lds_barrier();
						bool any_new = false;
#pragma unroll
						for (uint32_t k = 0; k < KS; k++) {
							// an earlier mark in the decision slot's bin, and a mark on the slot
							// itself by some other lane (conservative: that lane may be a later
							// one; the earliest pending lane is never blocked)
							const uint32_t fb = 1u << (wpos[k] & 31);
							const bool mine = win_marked[k];  // (its marks include its decision slot)
							// (mark-all: every pending lane marked its decision slot)
							const uint32_t fw = ma || mine ? fm2[wpos[k] >> 5] : fm1[wpos[k] >> 5];
							blocked[k] = pending[k] && stamp[dbin[k]] > v[k] && (fw & fb);
							mark_win[k] = blocked[k] && !win_marked[k];
							win_marked[k] = win_marked[k] || mark_win[k];
							any_new |= mark_win[k];
						}
						if (ma || !wg_any(any_new, 0))
							break;
					}
					// this round's slot marks are read: cleared for the next round (the
					// commit's barrier orders this before the next round's marks; with
					// one marking pass no barrier follows the tests, so the clear waits
					// for the commit's barrier and needs one of its own before a next round)
					auto clear_marks = [&]() {
						for (uint32_t i = threadIdx.x; i < kDedupSize / 32; i += kLanes)
							fm1[i] = fm2[i] = 0;
					};
					if (!ma)
						clear_marks();
					// 3. final lanes commit (visible after the next round's barrier)
					bool any_pending = false;
					uint32_t counts = 0;
#pragma unroll
					for (uint32_t k = 0; k < KS; k++) {
						const bool fin_w = pending[k] && !blocked[k] && writer[k];
						if (fin_w)
							tstore(wpos[k], sig[k]);
						emit[k] = emit[k] || fin_w;
						pending[k] = pending[k] && blocked[k];
						any_pending |= pending[k];
						counts |= (uint32_t)__popcll(__ballot(emit[k])) << (8 * k);
					}
					if constexpr (kSeq) {
						const uint64_t pm = __ballot(pending[0]);
						if (pending[0])  // this wave's pending signals, packed in trace order
							s_sig[64 * w + lane_rank(pm)] = sig[0];
						const uint32_t ndup = first_round ? __popcll(__ballot(dup[0])) : 0;
						const bool more = wg_any(any_pending, counts | (uint32_t)__popcll(pm) << 8 | ndup << 16);
						if (first_round) {
#pragma unroll
							for (uint32_t i = 0; i < kEdgeWaves; i++)
								dups += row[i] >> 17;
						}
						first_round = false;
						if (ma)
							clear_marks();
						if (!more) {
							// The clear must land before any wave marks again.  The next
							// chunk of the same prefetch group starts marking without a
							// barrier of its own (K1 ran for the whole group), so a fast
							// wave could otherwise OR its marks into words a slow wave is
							// still zeroing.  (Rare on the global walk: a chunk leaves no
							// lane pending after its first round.)
							if (ma)
								lds_barrier();
							return 0;
						}
						uint32_t npend = 0;
#pragma unroll
						for (uint32_t i = 0; i < kEdgeWaves; i++)
							npend += (row[i] >> 9) & 0xFF;
						if (npend <= kEdgeSeqMax) {
							// The tail in one wave, no barriers: lane j holds the j-th pending
							// signal in trace order.  It waits only for earlier pending signals
							// whose windows overlap its own -- every write lies in the writer's
							// window, so a signal no earlier pending window overlaps reads
							// nothing they can write, and writes nothing they read: its
							// dedup() (executor.h:692-706) on the table as it stands is the
							// sequential one.  Passes until none is left; the wave's LDS
							// operations run in order, so a pass sees the previous one's stores.
#if defined(SYZ_EXPERIMENTS) && defined(SYZ_EDGE_TAIL_DROP)  // timing only (results wrong): the tail skipped
							if (w == 0 && lane < kEdgeWaves)
								s_pm[lane] = 0;
							if (false) {
#else
							if (w == 0) {
#endif
								uint32_t seg = 0, segbase = 0, acc = 0;
#pragma unroll
								for (uint32_t i = 0; i < kEdgeWaves; i++) {
									const uint32_t c = (row[i] >> 9) & 0xFF;
									if (lane >= acc) {
										seg = i;
										segbase = acc;
									}
									acc += c;
								}
								const bool item = lane < npend;
								const uint32_t sg = item ? s_sig[64 * seg + lane - segbase] : 0;
								const uint32_t h = sg & (kDedupSize - 1);
								// earlier pending signals with an overlapping window (distance <= 3):
								// candidates from 32-slot buckets (s_sig is free once gathered: the
								// wave's LDS operations run in order), then the exact distance
								static_assert(kSeq ? kLanes == 256 && kEdgeSeqMax <= 32 : true, "tail buckets");
								reinterpret_cast<uint4*>(s_sig)[lane] = make_uint4(0, 0, 0, 0);
								const uint32_t bk = h >> 5;
								if (item) {
									atomicOr(&s_sig[bk], 1u << lane);
									s_th[lane] = h;
								}
								uint32_t cand = s_sig[(bk + 255) & 255] | s_sig[bk] | s_sig[(bk + 1) & 255];
								cand = item ? cand & ((1u << lane) - 1) : 0u;
								uint32_t ovm = 0;
								while (cand) {  // (rare: most tails have no two windows within 32 slots)
									const uint32_t k = __builtin_ctz(cand);
									cand &= cand - 1;
									ovm |= ((h - s_th[k] + 3) & (kDedupSize - 1)) <= 6 ? 1u << k : 0u;
								}
								uint32_t act = (uint32_t)__ballot(item), em = 0;
								while (act) {
									const bool go = item && ((act >> (lane & 31)) & 1) && !(ovm & act);
									bool wr = false;
									if (go) {
										uint32_t first = 4, tf = 0;
#pragma unroll
										for (int q = 3; q >= 0; q--) {
											const uint32_t t = table[h + q];
											if (t == sg || t == 0) {
												first = q;
												tf = t;
											}
										}
										wr = first == 4 || tf != sg;
										if (wr)
											tstore((h + (first & 3)) & (kDedupSize - 1), sg);
									}
									em |= (uint32_t)__ballot(wr);
									act &= ~(uint32_t)__ballot(go);
								}
								// the emitted ones, per source wave, by rank among its pending lanes
								if (lane < kEdgeWaves) {
									uint32_t c = 0, b = 0;
#pragma unroll
									for (uint32_t i = 0; i < kEdgeWaves; i++) {
										const uint32_t x = (row[i] >> 9) & 0xFF;
										b += i < lane ? x : 0;
										c = i == lane ? x : c;
									}
									s_pm[lane] = c ? (em >> b) & (~0u >> (32 - c)) : 0;
								}
							}
							lds_barrier();
							const uint64_t tail = s_pm[w];
							const bool mine = emit[0] || (pending[0] && ((tail >> lane_rank(pm)) & 1));
							const uint64_t me = __ballot(mine);
							uint32_t base = nsig, tot = 0;
#pragma unroll
							for (uint32_t i = 0; i < kEdgeWaves; i++) {
								const uint32_t x = ((row[i] >> 1) & 0xFF) + __popcll(s_pm[i]);
								base += i < w ? x : 0;
								tot += x;
							}
							if (mine)
								sigs[start + base + lane_rank(me)] = sig[0];
							nsig += tot;
							return 1;
						}
						if (ma)
							lds_barrier();  // the clear before the next round's marks
					} else {
						if (!wg_any(any_pending, counts))
							return 0;
					}
					return 2;
				};
				int st;
				do
					st = round(std::integral_constant<bool, kSeq && kMarkAll>{});
				while (st == 2);
				if (st == 1)
					return true;
				// write_output order == trace order: sub-chunks in order, then waves,
				// then lanes
#pragma unroll
				for (uint32_t k = 0; k < KS; k++) {
					const uint64_t m = __ballot(emit[k]);
					uint32_t base = nsig, tot = 0;
#pragma unroll
					for (uint32_t i = 0; i < kEdgeWaves; i++) {
						const uint32_t x = (row[i] >> (1 + 8 * k)) & 0xFF;
						base += i < w ? x : 0;
						tot += x;
					}
					if (emit[k])
						sigs[start + base + lane_rank(m)] = sig[k];
					nsig += tot;
				}
				return true;
			};
			// K1 of a prefetch group (kGroupK1): sig_i = (u32)pc_i ^ hash((u32)pc_{i-1})
			// for its chunks; a cover_check failure anywhere in them aborts the call
			// before any of them runs (the call publishes nothing either way)
			auto k1 = [&](const uint64_t (&buf)[kDepth][KS], uint32_t g, uint32_t (&sgv)[kDepth]) -> bool {
				uint32_t lo[kDepth], badm = 0;
#pragma unroll
				for (uint32_t u = 0; u < kDepth; u++) {
					const bool pend = (g + u) * kEdgeChunk + pos < len;
					const uint64_t pc = pend ? buf[u][0] : 0;
					badm |= __ballot(pend && !cover_check(pc)) ? 1u << u : 0u;
					const uint32_t h = exec_hash((uint32_t)pc);
					sgv[u] = __shfl_up(h, 1, 64);
					if (lane == 63)
						s_carry[u][0][w] = h;
					lo[u] = (uint32_t)pc;
				}
				if (wg_any(badm != 0, 0))
					return false;
#pragma unroll
				for (uint32_t u = 0; u < kDepth; u++) {
					if (lane == 0)
						sgv[u] = w > 0 ? s_carry[u][0][w - 1] : u > 0 ? s_carry[u - 1][0][kEdgeWaves - 1] : carry;
					sgv[u] ^= lo[u];
				}
				carry = s_carry[kDepth - 1][0][kEdgeWaves - 1];
				return true;
			};
			{
				auto run = [&](const uint64_t (&buf)[kDepth][KS], uint32_t g) -> bool {
					uint32_t sgv[kDepth] = {};
					if constexpr (kGroupK1) {
						if (!k1(buf, g, sgv))
							return false;
					}
#pragma unroll
					for (uint32_t u = 0; u < kDepth; u++)
						if (g + u < nch && !chunk(buf[u], sgv[u], g + u))
							return false;
					return true;
				};
				uint64_t ba[kDepth][KS], bb[kDepth][KS];
				fetch(ba, 0);
				for (uint32_t g = 0;;) {
					fetch(bb, g + kDepth);
					if (!run(ba, g)) {
						aborted = true;
						break;
					}
					g += kDepth;
					if (g >= nch)
						break;
					fetch(ba, g + kDepth);
					if (!run(bb, g)) {
						aborted = true;
						break;
					}
					g += kDepth;
					if (g >= nch)
						break;
				}
			}
			if (aborted) {
				done = c - cb;
				break;
			}
			if (threadIdx.x == 0)
				sig_cnt[c] = nsig;
		}
		// calls not published (aborted and later) report no signal (ipc.go:362-365)
		for (uint64_t c = cb + done + threadIdx.x; c < ce; c += kLanes)
			sig_cnt[c] = 0;
		if (threadIdx.x == 0)
			completed[p] = (uint32_t)done;
		lds_barrier();  // the table is re-zeroed for the next program
	}
	block_count(&cnt[kCntError], err);
	block_count(&cnt[kCntAux], threadIdx.x == 0 ? dups : 0);
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
	// the marking mode: forced by a debug flag, else mark-all while the last
	// launch's first rounds saw few duplicates (they mark in one pass too)
	const bool mark_all = ctx->agg_dbg & SYZSIG_DEBUG_EDGE_MARKALL   ? true
	                      : ctx->agg_dbg & SYZSIG_DEBUG_EDGE_PASSES ? false
	                                                                : ctx->edge_mark_all;
#ifdef SYZ_EXPERIMENTS
	// measured slower: 8 waves 25 ms, 2 waves 16.1, 1 wave 21.3 vs 4 waves 14.9 at C2
	if (ctx->edge_waves == 8)
		k_edge_dedup<8, kEdgeKS, false><<<grid, 512, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls,
		                                                          d_prog_call, nprog, d_sigs, d_sig_cnt, d_completed,
		                                                          ctx->d_cnt);
	else if (ctx->edge_waves == 2)
		k_edge_dedup<2, kEdgeKS, false><<<grid, 128, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls,
		                                                          d_prog_call, nprog, d_sigs, d_sig_cnt, d_completed,
		                                                          ctx->d_cnt);
	else if (ctx->edge_waves == 1)
		k_edge_dedup<1, kEdgeKS, false><<<grid, 64, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls,
		                                                         d_prog_call, nprog, d_sigs, d_sig_cnt, d_completed,
		                                                         ctx->d_cnt);
	else
#endif
	if (mark_all)
		k_edge_dedup<4, kEdgeKS, true><<<grid, 256, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls,
		                                                         d_prog_call, nprog, d_sigs, d_sig_cnt, d_completed,
		                                                         ctx->d_cnt);
	else
		k_edge_dedup<4, kEdgeKS, false><<<grid, 256, 0, ctx->stream>>>(d_pcs, npc, d_call_start, d_call_len, ncalls,
		                                                          d_prog_call, nprog, d_sigs, d_sig_cnt, d_completed,
		                                                          ctx->d_cnt);
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
	if (npc)
		ctx->edge_mark_all = ctx->h_cnt[kCntAux] * 100 < (unsigned long long)kEdgeMarkAllMaxDupPct * npc;
	return SYZSIG_OK;
}
