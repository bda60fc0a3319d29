// triage.hip -- K3: batched checkNewSignal (DiffRaw + Merge) against a
// device-resident maxSignal, bit-exact with the reference's sequential order.
//
// Reference: syz-fuzzer/fuzzer.go:494-511 checkNewSignal, pkg/signal/signal.go
// :90-102 DiffRaw and :117-131 Merge.  Over a batch in serial order
// (program-major, call-minor; call k has raw signal sig_k and prio p_k), with
// M0 = maxSignal before the batch:
//
//   e in new_k  <=>  e in sig_k  and  p_k > M0[e]  and  no j < k has e in sig_j with p_j >= p_k
//   M_final[e]  =  max(M0[e], max_k p_k)               (absent < every prio)
//   newSignal   +=  { e : M_final[e] != M0[e] } with prio M_final[e]
//
// Parallel restatement (per run of calls with <= 4 distinct prios, each prio
// mapped to a level by signed order): for every slot and level keep
//   first[slot][l] = min serial k over records of level l  (epoch-tagged u32)
// Phase 1 (probe): each record finds/inserts its element, drops itself if
//   p_k <= M0[e] or if an already-recorded first at a level >= l is < k
//   (firsts only decrease, so a stale read never drops a record wrongly),
//   else atomicMin's its level and is kept as a candidate.  The thread that
//   first marks a slot "touched" becomes its committer.
// Phase 2 (decide): a candidate is new iff min_{l' >= l} first[l'] == k; the
//   committer writes M_final (top set level) and merges it into newSignal.
// One wave per call; candidates are compacted in place inside the call's own
// record range, so the phases need no global atomics besides the per-block
// counters.
#include <algorithm>
#include <vector>

#include "internal.h"

namespace syz {


__device__ __forceinline__ uint32_t min_from_level(uint4 f, uint32_t l)
{
	uint32_t m = f.w;
	if (l <= 2)
		m = min(m, f.z);
	if (l <= 1)
		m = min(m, f.y);
	if (l == 0)
		m = min(m, f.x);
	return m;
}

__device__ __forceinline__ uint32_t first_at(uint4 f, uint32_t l)
{
	return l == 0 ? f.x : l == 1 ? f.y : l == 2 ? f.z : f.w;
}

// ---------------------------------------------------------------- inputs
// A run is processed as segments of records, one wave per segment; candidates
// are compacted in place inside the segment's own record range.
//  - CallsIn: segment = one call (prio and serial uniform per segment).
//  - RecsIn:  segment = 4096 packed records (owner side of a sharded batch).
//  - PartIn:  the run's records radix-partitioned by table region (2 MB
//             slices of maxSignal); partition p is processed by the blocks of
//             XCD p % 8 (blockIdx % 8, round-robin dispatch), partition after
//             partition, so the slice being probed stays in that XCD's L2.
//             Placement only affects speed: any block may process any segment.
struct Seg {
	uint64_t start;  // first record
	uint32_t len;    // records
	uint32_t level;  // CallsIn: the call's level
	uint32_t serial; // CallsIn: the call's serial index in the run
	bool ok;
};

__device__ __forceinline__ void set_bit(uint32_t* bits, uint64_t r) { atomicOr(&bits[r >> 5], 1u << (r & 31)); }

struct CallsIn {
	const uint32_t* sigs;
	const uint64_t* call_start;
	const uint32_t* call_len;
	const uint8_t* call_prio;
	uint64_t c0, c1, nrec;
	uint32_t* new_bits;
	uint8_t* call_new;

	template <typename F>
	__device__ void for_each_segment(const LevelMap& lm, F f) const
	{
		const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
		for (uint64_t s = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); s < c1 - c0; s += nwaves) {
			Seg g;
			const uint64_t c = c0 + s;
			g.start = call_start[c];
			g.len = call_len[c];
			g.ok = g.start <= nrec && g.len <= nrec - g.start && g.len <= kSerialMask;
			g.level = lm.lvl[call_prio[c]];
			g.ok = g.ok && g.level < lm.n;
			g.serial = (uint32_t)s;
			f(s, g);
		}
	}
	__device__ void rec(const Seg& g, uint32_t j, uint32_t& e, uint32_t& l, uint32_t& k) const
	{
		e = __builtin_nontemporal_load(&sigs[g.start + j]);  // streamed once: keep caches for the table
		l = g.level;
		k = g.serial;
	}
	__device__ void mark_new(const Seg& g, uint32_t j, uint32_t) const { set_bit(new_bits, g.start + j); }
	__device__ void seg_has_new(uint64_t s) const { call_new[c0 + s] = 1; }
};

constexpr uint32_t kSegRecs = 4096;

struct RecsIn {
	const uint64_t* recs;
	uint64_t nrec;
	uint8_t* new_flags;

	template <typename F>
	__device__ void for_each_segment(const LevelMap&, F f) const
	{
		const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
		const uint64_t nseg = (nrec + kSegRecs - 1) / kSegRecs;
		for (uint64_t s = blockIdx.x * (uint64_t)(blockDim.x >> 6) + (threadIdx.x >> 6); s < nseg; s += nwaves) {
			Seg g;
			g.start = s * kSegRecs;
			g.len = (uint32_t)min<uint64_t>(kSegRecs, nrec - g.start);
			g.ok = true;
			g.level = 0;
			g.serial = 0;
			f(s, g);
		}
	}
	__device__ void rec(const Seg& g, uint32_t j, uint32_t& e, uint32_t& l, uint32_t& k) const
	{
		const uint64_t r = recs[g.start + j];
		e = (uint32_t)(r >> 32);
		l = (uint32_t)(r >> 24) & 0xff;
		k = (uint32_t)r & kSerialMask;
	}
	__device__ void mark_new(const Seg& g, uint32_t j, uint32_t) const { new_flags[g.start + j] = 1; }
	__device__ void seg_has_new(uint64_t) const {}
};

constexpr uint32_t kPartSeg = 1024;  // records per segment in partitioned mode

struct PartIn {
	const uint64_t* recs;      // packed elem << 32 | level << 24 | serial, grouped by partition
	const uint32_t* orig;      // record index in the caller's sigs[] (for the new bit)
	const uint64_t* rec_base;  // nparts + 1
	const uint64_t* seg_base;  // nparts + 1
	uint32_t nparts;           // multiple of 8
	uint64_t c0;
	uint32_t* new_bits;
	uint8_t* call_new;

	template <typename F>
	__device__ void for_each_segment(const LevelMap&, F f) const
	{
		const uint32_t x = blockIdx.x & 7, i = blockIdx.x >> 3, nbx = gridDim.x >> 3;
		const uint32_t w = threadIdx.x >> 6, wpb = blockDim.x >> 6;
		for (uint32_t p = x; p < nparts; p += 8) {
			const uint64_t base = rec_base[p], n = rec_base[p + 1] - base;
			const uint64_t nseg = (n + kPartSeg - 1) / kPartSeg, sb = seg_base[p];
			for (uint64_t s = (uint64_t)i * wpb + w; s < nseg; s += (uint64_t)nbx * wpb) {
				Seg g;
				g.start = base + s * kPartSeg;
				g.len = (uint32_t)min<uint64_t>(kPartSeg, n - s * kPartSeg);
				g.ok = true;
				g.level = 0;
				g.serial = 0;
				f(sb + s, g);
			}
		}
	}
	__device__ void rec(const Seg& g, uint32_t j, uint32_t& e, uint32_t& l, uint32_t& k) const
	{
		const uint64_t r = __builtin_nontemporal_load(&recs[g.start + j]);
		e = (uint32_t)(r >> 32);
		l = (uint32_t)(r >> 24) & 0xff;
		k = (uint32_t)r & kSerialMask;
	}
	__device__ void mark_new(const Seg& g, uint32_t j, uint32_t k) const
	{
		set_bit(new_bits, orig[g.start + j]);
		call_new[c0 + k] = 1;
	}
	__device__ void seg_has_new(uint64_t) const {}
};

// ---------------------------------------------------------------- phase 1
// Run hint stored in a slot's bits 10..28 by a candidate (l, k): H = (l+1) << 16 |
// (0xFFFF - (k >> 8)), larger = better.  It records a fact of this run -- a
// record with level l and serial <= ((k >> 8) << 8) | 0xFF carries the element
// -- so any record (l', k') with l' <= l and (k' >> 8) > (k >> 8) cannot be new
// and cannot raise M_final.  Written with a plain store: a reader that misses it
// only loses the shortcut.  Every hinted slot has a candidate, hence a
// committer, which rewrites the word without hint bits.
__device__ __forceinline__ uint32_t make_hint(uint32_t l, uint32_t k) { return ((l + 1) << 16) | (0xFFFF - (k >> 8)); }
__device__ __forceinline__ bool hint_settles(uint32_t H, uint32_t l, uint32_t k)
{
	return H != 0 && (H >> 16) - 1 >= l && (0xFFFF - (H & 0xFFFF)) < (k >> 8);
}

constexpr uint32_t kKnown = 0x80000000u;  // queue hint: slot index known from the home bucket

// Phase 1 -- probe.  Filter: kProbeU records per lane in flight; a record
// whose element sits in its (16-B) home bucket with a live prio >= p_k, or
// whose run hint settles it, is done (not new, changes nothing).  Survivors go
// to this wave's LDS queue (with the slot index and word when the home bucket
// already told them) and are drained kDrain at a time, kDrain/64 per lane in
// flight: find/insert if needed, prio filter against M0, firsts filter,
// atomicMin of the record's level, and a run hint for later records of the
// element.  The slow path thus runs dense and survivors never leave the chip;
// the drain runs inside the segment loop so hints reach later segments.
template <typename In, uint32_t kProbeU, uint32_t kDrain>
__global__ __launch_bounds__(256) void k_probe(uint64_t* slots, uint64_t bmask, uint32_t* firsts, uint32_t* touched,
                                               In in, LevelMap lm, uint32_t epoch, uint32_t* cand_slot,
                                               uint32_t* cand_meta, uint32_t* cand_cnt, unsigned long long* cnt,
                                               int dbg)
{
	constexpr uint32_t QCAP = kDrain + 64 * kProbeU;
	__shared__ uint64_t q_rec[4][QCAP];  // per-wave survivor queue: e << 32 | level << 24 | serial
	__shared__ uint32_t q_j[4][QCAP];    // offset in the segment
	__shared__ uint32_t q_s[4][QCAP];    // kKnown | slot index, or 0
	__shared__ uint32_t q_v[4][QCAP];    // low word of the slot seen by the filter (when known)
	const uint32_t lane = lane_id();
	const uint64_t max_probe = max_probe_for(bmask);
	uint64_t ncand = 0, ntouch = 0, ovf = 0, err = 0, nsurv = 0;
	uint64_t* qr = q_rec[threadIdx.x >> 6];
	uint32_t* qj = q_j[threadIdx.x >> 6];
	uint32_t* qs = q_s[threadIdx.x >> 6];
	uint32_t* qv = q_v[threadIdx.x >> 6];
	in.for_each_segment(lm, [&](uint64_t s, const Seg& g) {
		if (!g.ok) {
			err += lane == 0;
			if (lane == 0)
				cand_cnt[s] = 0;
			return;
		}
		uint32_t nc = 0, qn = 0;
		auto drain = [&](uint32_t n) {  // queue entries [0, n), n <= kDrain
			constexpr uint32_t D = kDrain / 64;
			uint32_t sidx[D], l[D], k[D], j[D], lw[D], e[D];
			bool live[D];
			uint4 f[D];
#pragma unroll
			for (uint32_t u = 0; u < D; u++) {
				const uint32_t q = u * 64 + lane;
				live[u] = q < n && !(dbg & 1);
				if (live[u]) {
					const uint64_t r = qr[q];
					const uint32_t hint = qs[q];
					e[u] = (uint32_t)(r >> 32);
					j[u] = qj[q];
					k[u] = (uint32_t)r & kSerialMask;
					l[u] = (uint32_t)(r >> 24) & 0xff;
					if (hint & kKnown) {
						sidx[u] = hint & ~kKnown;
						lw[u] = qv[q];
					} else {
						const uint32_t want = (uint32_t)make_slot(0, lm.val[l[u]]);
						uint64_t old;
						const int64_t idx = tbl_find_or_insert(slots, bmask, e[u], make_absent(e[u]), old, max_probe);
						if (idx < 0) {
							ovf++;
							live[u] = false;
						} else if (slot_live(old) && slot_state(old) >= want) {
							live[u] = false;  // settled after all (element beyond its home bucket)
						}
						sidx[u] = (uint32_t)idx;
						lw[u] = old ? (uint32_t)old : (uint32_t)make_absent(e[u]);
					}
				}
			}
#pragma unroll
			for (uint32_t u = 0; u < D; u++)
				if (live[u])
					f[u] = reinterpret_cast<const uint4*>(firsts)[sidx[u]];
#pragma unroll
			for (uint32_t u = 0; u < D; u++) {
				bool cand = false, toucher = false;
				if (live[u]) {
					const uint32_t tag = (epoch << 24) | k[u];
					if (min_from_level(f[u], l[u]) >= tag) {
						const uint32_t prev = atomicMin(&firsts[4 * (uint64_t)sidx[u] + l[u]], tag);
						if (prev > ((epoch << 24) | kSerialMask)) {
							const uint32_t bit = 1u << (sidx[u] & 31);
							toucher = !(atomicOr(&touched[sidx[u] >> 5], bit) & bit);
						}
						cand = true;
						const uint32_t Hn = make_hint(l[u], k[u]);
						if (!(dbg & 2) && Hn > ((lw[u] & (uint32_t)kHintMask) >> 10))
							slots[sidx[u]] = ((uint64_t)e[u] << 32) | (lw[u] & ~(uint32_t)kHintMask) | ((uint64_t)Hn << 10);
					}
				}
				const uint64_t m = __ballot(cand);
				if (cand) {
					const uint64_t pos = g.start + nc + lane_rank(m);
					cand_slot[pos] = sidx[u];
					cand_meta[pos] = ((uint32_t)toucher << 31) | (l[u] << 24) | j[u];
				}
				nc += (uint32_t)__popcll(m);
				ntouch += toucher;
			}
		};
		for (uint32_t base = 0; base < g.len; base += 64 * kProbeU) {
			uint32_t e[kProbeU], l[kProbeU], k[kProbeU];
			ulonglong2 h0[kProbeU];
#pragma unroll
			for (uint32_t u = 0; u < kProbeU; u++) {
				const uint32_t j = base + u * 64 + lane;
				l[u] = 0xff;
				if (j < g.len)
					in.rec(g, j, e[u], l[u], k[u]);
			}
#pragma unroll
			for (uint32_t u = 0; u < kProbeU; u++)
				if (l[u] < lm.n)
					h0[u] = *reinterpret_cast<const ulonglong2*>(slots + (home_bucket(e[u], bmask) << kBucketShift));
#pragma unroll
			for (uint32_t u = 0; u < kProbeU; u++) {
				bool surv = false;
				uint32_t hint = 0, lwv = 0;
				if (l[u] != 0xff) {
					if (l[u] >= lm.n) {
						err++;
					} else {
						const uint32_t want = (uint32_t)make_slot(0, lm.val[l[u]]);
						const uint64_t a0 = h0[u].x, a1 = h0[u].y;
						const uint64_t hb = home_bucket(e[u], bmask) << kBucketShift;
						// position of e in its home bucket: 0, 1, or unknown (2)
						const uint32_t at = (a0 != kSlotEmpty && slot_key(a0) == e[u]) ? 0
						                    : (a0 != kSlotEmpty && a1 != kSlotEmpty && slot_key(a1) == e[u]) ? 1 : 2;
						const uint64_t sv = at == 0 ? a0 : a1;
						const uint32_t H = (uint32_t)((sv & kHintMask) >> 10);
						const bool settled = at < 2 && ((slot_live(sv) && slot_state(sv) >= want) ||
						                                hint_settles(H, l[u], k[u]));
						surv = !settled;
						if (surv && at < 2 && hb + at < kKnown) {
							hint = kKnown | (uint32_t)(hb + at);
							lwv = (uint32_t)sv;
						}
					}
				}
				const uint64_t m = __ballot(surv);
				if (surv) {
					const uint32_t qp = qn + lane_rank(m);
					qr[qp] = ((uint64_t)e[u] << 32) | ((uint64_t)l[u] << 24) | k[u];
					qj[qp] = base + u * 64 + lane;
					qs[qp] = hint;
					qv[qp] = lwv;
				}
				qn += (uint32_t)__popcll(m);
				nsurv += lane == 0 ? __popcll(m) : 0;
			}
			if (qn >= kDrain) {
				__builtin_amdgcn_wave_barrier();
				drain(kDrain);
				qn -= kDrain;
				// move the tail (< 64 * kProbeU entries) to the queue head
				for (uint32_t t = 0; t < qn; t += 64) {
					uint64_t tr = 0;
					uint32_t tj = 0, ts = 0, tv = 0;
					if (t + lane < qn) {
						tr = qr[kDrain + t + lane];
						tj = qj[kDrain + t + lane];
						ts = qs[kDrain + t + lane];
						tv = qv[kDrain + t + lane];
					}
					__builtin_amdgcn_wave_barrier();
					if (t + lane < qn) {
						qr[t + lane] = tr;
						qj[t + lane] = tj;
						qs[t + lane] = ts;
						qv[t + lane] = tv;
					}
				}
				__builtin_amdgcn_wave_barrier();
			}
		}
		if (qn) {
			__builtin_amdgcn_wave_barrier();
			drain(qn);
			__builtin_amdgcn_wave_barrier();
		}
		if (lane == 0) {
			cand_cnt[s] = nc;
			ncand += nc;
		}
	});
	block_count(&cnt[kCntCandidates], ncand);
	block_count(&cnt[kCntTouched], ntouch);
	block_count(&cnt[kCntOverflow], ovf);
	block_count(&cnt[kCntError], err);
	block_count(&cnt[kCntAux2], nsurv);
}

// ---------------------------------------------------------------- phase 2
template <typename In>
__global__ __launch_bounds__(256) void k_decide(uint64_t* slots, const uint32_t* __restrict__ firsts,
                                                uint64_t* ns_slots, uint64_t ns_bmask, In in, LevelMap lm,
                                                uint32_t epoch, const uint32_t* __restrict__ cand_slot,
                                                const uint32_t* __restrict__ cand_meta,
                                                const uint32_t* __restrict__ cand_cnt, unsigned long long* cnt)
{
	const uint32_t lane = lane_id();
	const uint32_t cur_hi = (epoch << 24) | kSerialMask;
	uint64_t inserted = 0, changed = 0, ns_ins = 0, ovf = 0;
	in.for_each_segment(lm, [&](uint64_t s, const Seg& g) {
		const uint32_t nc = cand_cnt[s];
		if (nc == 0)
			return;
		bool any_new = false;
		for (uint32_t base = 0; base < nc; base += 64) {
			const uint32_t i = base + lane;
			if (i >= nc)
				continue;
			const uint32_t sidx = cand_slot[g.start + i];
			const uint32_t meta = cand_meta[g.start + i];
			const uint32_t l = (meta >> 24) & 3, j = meta & kSerialMask;
			uint32_t e, l2, k;
			in.rec(g, j, e, l2, k);
			const uint4 f = reinterpret_cast<const uint4*>(firsts)[sidx];
			if (min_from_level(f, l) == ((epoch << 24) | k)) {
				in.mark_new(g, j, k);
				any_new = true;
			}
			if (meta >> 31) {
				// committer: M_final = prio of the highest level recorded this epoch
				uint32_t top = 0;
#pragma unroll
				for (uint32_t t = 0; t < 4; t++)
					if (t < lm.n && first_at(f, t) <= cur_hi)
						top = t;
				const int8_t P = lm.val[top];
				const uint64_t old = slots[sidx];
				slots[sidx] = make_slot(e, P);
				inserted += !slot_live(old);
				changed++;
				const int r = tbl_merge(ns_slots, ns_bmask, e, P);
				ns_ins += r == 1;
				ovf += r < 0;
			}
		}
		if (__ballot(any_new) && lane == 0)
			in.seg_has_new(s);
	});
	block_count(&cnt[kCntInserted], inserted);
	block_count(&cnt[kCntChanged], changed);
	block_count(&cnt[kCntAux], ns_ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// ---------------------------------------------------------------- partitioning
// Records of calls [c0, c1) -> packed records grouped by table region
// (partition = home bucket >> shift).  Block b owns the chunk of calls
// [b*kPartCPB, (b+1)*kPartCPB); its slice of every partition is fixed by a
// scan of the per-(chunk, partition) counts, so the scatter needs no global
// atomics.  The scatter stages kTile records in LDS, sorts them by partition
// (counting sort) and writes each partition's run contiguously.
constexpr uint32_t kPartCPB = 128;
constexpr uint32_t kMaxParts = 1024;
constexpr uint32_t kTile = 2048;

__device__ __forceinline__ uint32_t part_of(uint32_t e, uint64_t bmask, uint32_t shift)
{
	return (uint32_t)((fmix32(e) & bmask) >> shift);
}

__global__ __launch_bounds__(256) void k_part_count(CallsIn in, uint64_t bmask, uint32_t shift, uint32_t nparts,
                                                    uint32_t* counts)
{
	__shared__ uint32_t h[kMaxParts];
	const uint32_t w = threadIdx.x >> 6, nw = blockDim.x >> 6, lane = lane_id();
	const uint64_t ncalls = in.c1 - in.c0, nchunks = (ncalls + kPartCPB - 1) / kPartCPB;
	for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
		for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x)
			h[i] = 0;
		__syncthreads();
		const uint64_t ce = min<uint64_t>(ncalls, (ch + 1) * kPartCPB);
		for (uint64_t s = ch * kPartCPB + w; s < ce; s += nw) {
			const uint64_t c = in.c0 + s, start = in.call_start[c];
			const uint32_t len = in.call_len[c];
			for (uint32_t j = lane; j < len; j += 64)
				atomicAdd(&h[part_of(in.sigs[start + j], bmask, shift)], 1u);
		}
		__syncthreads();
		for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x)
			counts[ch * nparts + i] = h[i];
		__syncthreads();
	}
}

// exclusive scan of v over the block (256 threads); returns the block total
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* out)
{
	__shared__ uint32_t wsum[4];
	const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
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
	for (uint32_t i = 0; i < 4; i++) {
		pre += i < w ? wsum[i] : 0;
		tot += wsum[i];
	}
	__syncthreads();
	*out = pre + x - v;
	return tot;
}

// block p: exclusive scan over chunks of counts[.][p] -> offs[.][p]; totals[p]
__global__ __launch_bounds__(256) void k_part_scan_chunks(const uint32_t* counts, uint64_t nchunks, uint32_t nparts,
                                                          uint32_t* offs, uint64_t* totals)
{
	const uint32_t p = blockIdx.x;
	uint64_t run = 0;
	for (uint64_t b0 = 0; b0 < nchunks; b0 += blockDim.x) {
		const uint64_t b = b0 + threadIdx.x;
		const uint32_t v = b < nchunks ? counts[b * nparts + p] : 0;
		uint32_t ex;
		const uint32_t tot = block_excl_scan(v, &ex);
		if (b < nchunks)
			offs[b * nparts + p] = (uint32_t)(run + ex);
		run += tot;
	}
	if (threadIdx.x == 0)
		totals[p] = run;
}

// totals -> rec_base / seg_base
__global__ void k_part_scan(const uint64_t* totals, uint32_t nparts, uint64_t* rec_base, uint64_t* seg_base)
{
	if (threadIdx.x != 0 || blockIdx.x != 0)
		return;
	uint64_t r = 0, sg = 0;
	for (uint32_t p = 0; p < nparts; p++) {
		rec_base[p] = r;
		seg_base[p] = sg;
		r += totals[p];
		sg += (totals[p] + kPartSeg - 1) / kPartSeg;
	}
	rec_base[nparts] = r;
	seg_base[nparts] = sg;
}

__global__ __launch_bounds__(256) void k_part_scatter(CallsIn in, LevelMap lm, uint64_t bmask, uint32_t shift,
                                                      uint32_t nparts, const uint32_t* __restrict__ offs,
                                                      const uint64_t* __restrict__ rec_base, uint64_t* recs,
                                                      uint32_t* orig)
{
	__shared__ uint64_t t_rec[kTile], s_rec[kTile];
	__shared__ uint32_t t_orig[kTile], s_orig[kTile];
	__shared__ uint16_t t_part[kTile], s_part[kTile];
	__shared__ uint32_t cur[kMaxParts], hist[kMaxParts], bin[kMaxParts], pos[kMaxParts];
	__shared__ uint32_t tile_n, more;
	const uint32_t w = threadIdx.x >> 6, lane = lane_id();
	const uint64_t ncalls = in.c1 - in.c0, nchunks = (ncalls + kPartCPB - 1) / kPartCPB;
	const uint32_t per_t = (nparts + blockDim.x - 1) / blockDim.x;  // bins per thread in the scan
	for (uint64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
		const uint64_t cb = ch * kPartCPB, ce = min<uint64_t>(ncalls, cb + kPartCPB);
		for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x)
			cur[i] = offs[ch * nparts + i];
		// per-wave cursor: call cb + w, +4, ...; offset inside the call
		uint64_t wc = cb + w;
		uint32_t wo = 0;
		for (;;) {
			for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x)
				hist[i] = 0;
			if (threadIdx.x == 0) {
				tile_n = 0;
				more = 0;
			}
			__syncthreads();
			// fill: each wave contributes up to kTile/4 records
			uint32_t quota = kTile / 4;
			while (quota && wc < ce) {
				const uint64_t c = in.c0 + wc, start = in.call_start[c];
				const uint32_t len = in.call_len[c];
				const uint32_t m = min(quota, len - wo);
				uint32_t tb = 0;
				if (lane == 0 && m)
					tb = atomicAdd(&tile_n, m);
				tb = __shfl(tb, 0, 64);
				const uint64_t head = ((uint64_t)lm.lvl[in.call_prio[c]] << 24) | (wc & kSerialMask);
				// all loads of this piece first (independent, in flight together)
				uint32_t ev[kTile / 4 / 64];
#pragma unroll
				for (uint32_t u = 0; u < kTile / 4 / 64; u++) {
					const uint32_t i = u * 64 + lane;
					ev[u] = i < m ? in.sigs[start + wo + i] : 0;
				}
#pragma unroll
				for (uint32_t u = 0; u < kTile / 4 / 64; u++) {
					const uint32_t i = u * 64 + lane;
					if (i < m) {
						const uint32_t p = part_of(ev[u], bmask, shift);
						t_rec[tb + i] = ((uint64_t)ev[u] << 32) | head;
						t_orig[tb + i] = (uint32_t)(start + wo + i);
						t_part[tb + i] = (uint16_t)p;
						atomicAdd(&hist[p], 1u);
					}
				}
				quota -= m;
				wo += m;
				if (wo == len) {
					wc += 4;
					wo = 0;
				}
			}
			if (lane == 0 && wc < ce)
				atomicOr(&more, 1u);
			__syncthreads();
			const uint32_t n = tile_n;
			// exclusive scan of hist -> bin (per_t consecutive bins per thread)
			uint32_t loc = 0;
			for (uint32_t q = 0; q < per_t; q++) {
				const uint32_t i = threadIdx.x * per_t + q;
				loc += i < nparts ? hist[i] : 0;
			}
			uint32_t ex;
			block_excl_scan(loc, &ex);
			for (uint32_t q = 0; q < per_t; q++) {
				const uint32_t i = threadIdx.x * per_t + q;
				if (i < nparts) {
					bin[i] = ex;
					pos[i] = ex;
					ex += hist[i];
				}
			}
			__syncthreads();
			for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
				const uint32_t p = t_part[i];
				const uint32_t d = atomicAdd(&pos[p], 1u);
				s_rec[d] = t_rec[i];
				s_orig[d] = t_orig[i];
				s_part[d] = (uint16_t)p;
			}
			__syncthreads();
			// consecutive threads write consecutive records of one partition run
			for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
				const uint32_t p = s_part[i];
				const uint64_t g = rec_base[p] + cur[p] + (i - bin[p]);
				recs[g] = s_rec[i];
				orig[g] = s_orig[i];
			}
			__syncthreads();
			for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x)
				cur[i] += hist[i];
			const bool again = more != 0;
			__syncthreads();
			if (!again)
				break;
		}
	}
}

// prio presence over calls -> 256-bit mask (block-local, one atomic per word
// per block), plus the number of records (sum of call_len)
__global__ void k_prio_presence(const uint8_t* __restrict__ prio, const uint32_t* __restrict__ len,
                                const uint64_t* __restrict__ start, uint64_t n, uint64_t nrec_space, uint32_t* mask,
                                unsigned long long* nrec, unsigned long long* bad)
{
	__shared__ uint32_t m[8];
	if (threadIdx.x < 8)
		m[threadIdx.x] = 0;
	__syncthreads();
	uint64_t tot = 0, nbad = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		uint8_t p = prio[i];
		atomicOr(&m[p >> 5], 1u << (p & 31));
		const uint64_t st = start[i];
		const uint32_t ln = len[i];
		tot += ln;
		nbad += st > nrec_space || ln > nrec_space - st || ln > kSerialMask;
	}
	__syncthreads();
	if (threadIdx.x < 8 && m[threadIdx.x])
		atomicOr(&mask[threadIdx.x], m[threadIdx.x]);
	block_count(nrec, tot);
	block_count(bad, nbad);
}

// ---------------------------------------------------------------- host

struct Run {
	uint64_t c0, c1;
	LevelMap lm;
};

static void level_map_from(const bool present[256], LevelMap* lm)
{
	memset(lm, 0xff, sizeof(*lm));
	// levels in signed int8 order of the prio (DiffRaw compares prioType(prio))
	uint32_t n = 0;
	for (int v = -128; v <= 127; v++) {
		uint8_t u = (uint8_t)(int8_t)v;
		if (present[u]) {
			lm->lvl[u] = (uint8_t)n;
			lm->val[n] = (int8_t)v;
			n++;
		}
	}
	lm->n = n;
}

static int plan_runs(syzsig_ctx* ctx, const syzsig_batch* b, std::vector<Run>* runs, uint64_t* total_recs)
{
	void* dmask;
	SYZ_TRY(ws_get(ctx, 6, 64, &dmask));
	SYZ_HIP(hipMemsetAsync(dmask, 0, 48, ctx->stream));
	k_prio_presence<<<grid_for(b->ncalls, 256, 256), 256, 0, ctx->stream>>>(
	    b->call_prio, b->call_len, b->call_start, b->ncalls, b->nrec, (uint32_t*)dmask,
	    (unsigned long long*)((char*)dmask + 32), (unsigned long long*)((char*)dmask + 40));
	SYZ_HIP(hipGetLastError());
	uint32_t hmask[12];
	SYZ_HIP(hipMemcpyAsync(hmask, dmask, 48, hipMemcpyDeviceToHost, ctx->stream));
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	memcpy(total_recs, &hmask[8], 8);
	uint64_t nbad;
	memcpy(&nbad, &hmask[10], 8);
	if (nbad)
		return fail(SYZSIG_EINVAL, "triage_batch: a call range lies outside [0, nrec) or has >= 2^24 records");
	bool present[256];
	int np = 0;
	for (int i = 0; i < 256; i++) {
		present[i] = (hmask[i >> 5] >> (i & 31)) & 1;
		np += present[i];
	}
	if (np <= 4) {
		LevelMap lm;
		level_map_from(present, &lm);
		for (uint64_t c0 = 0; c0 < b->ncalls; c0 += kSerialMask)
			runs->push_back({c0, std::min<uint64_t>(b->ncalls, c0 + kSerialMask), lm});
		return SYZSIG_OK;
	}
	// More than 4 distinct prios: split the serial order into maximal runs with
	// <= 4 distinct prios each; runs execute one after another, so each sees
	// the merges of all earlier calls exactly as the sequential loop does.
	std::vector<uint8_t> hp(b->ncalls);
	SYZ_HIP(hipMemcpy(hp.data(), b->call_prio, b->ncalls, hipMemcpyDeviceToHost));
	uint64_t c0 = 0;
	while (c0 < b->ncalls) {
		bool pres[256] = {false};
		int cnt = 0;
		uint64_t c = c0;
		for (; c < b->ncalls && c - c0 < kSerialMask; c++) {
			if (!pres[hp[c]]) {
				if (cnt == 4)
					break;
				pres[hp[c]] = true;
				cnt++;
			}
		}
		LevelMap lm;
		level_map_from(pres, &lm);
		runs->push_back({c0, c, lm});
		c0 = c;
	}
	return SYZSIG_OK;
}

// One run (<= 4 prio levels): probe, then decide+commit.  On capacity
// overflow the run's only table side effects -- absent markers -- are dropped
// by a rehash into a bigger table and the run restarts.
// probe variants: records per lane in flight (probe_u) x survivors drained per batch
template <typename In>
static void launch_probe(syzsig_ctx* ctx, int grid, syzsig_set* ms, const In& in, const LevelMap& lm,
                         uint32_t* cand_slot, uint32_t* cand_meta, uint32_t* cand_cnt)
{
#define SYZ_PROBE(U, D)                                                                                     \
	k_probe<In, U, D><<<grid, 256, 0, ctx->stream>>>(ms->slots, ms->nbuckets - 1, ms->firsts, ms->touched, in, lm, \
	                                                 ms->epoch, cand_slot, cand_meta, cand_cnt, ctx->d_cnt,         \
	                                                 ctx->debug_skip_b)
	const bool u2 = ctx->probe_u == 2, d2 = ctx->probe_drain == 128;
	if (u2 && d2)
		SYZ_PROBE(2, 128);
	else if (u2)
		SYZ_PROBE(2, 256);
	else if (d2)
		SYZ_PROBE(1, 128);
	else
		SYZ_PROBE(1, 256);
#undef SYZ_PROBE
}

// `prep(&in, &grid)` builds the kernels' input for the table's current
// geometry (it runs again after a restart on a bigger table).
template <typename In, typename Prep>
static int triage_run(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, Prep prep, const LevelMap& lm,
                      uint32_t* cand_slot, uint32_t* cand_meta, uint32_t* cand_cnt, syzsig_batch_stats* st)
{
	for (;;) {
		if (--ms->epoch == 0) {
			SYZ_HIP(hipMemsetAsync(ms->firsts, 0xff, ms->nslots() * 16, ctx->stream));
			ms->epoch = 254;
		}
		SYZ_HIP(hipMemsetAsync(ms->touched, 0, (ms->nslots() / 32 + 1) * 4, ctx->stream));
		In in;
		int grid = 0;
		SYZ_TRY(prep(&in, &grid, st));
		SYZ_TRY(counters_reset(ctx));
		if (ctx->timing)
			SYZ_HIP(hipEventRecord(ctx->ev[0], ctx->stream));
		launch_probe<In>(ctx, grid, ms, in, lm, cand_slot, cand_meta, cand_cnt);
		SYZ_HIP(hipGetLastError());
		if (ctx->timing)
			SYZ_HIP(hipEventRecord(ctx->ev[1], ctx->stream));
		SYZ_TRY(counters_fetch(ctx));
		if (ctx->timing) {
			float ms = 0;
			SYZ_HIP(hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]));
			st->probe_ms += ms;
		}
		if (ctx->h_cnt[kCntError])
			return fail(SYZSIG_EINVAL, "triage: a call range lies outside [0, nrec), a call has >= 2^24 "
			                           "records, or a record's prio level is out of range");
		if (ctx->h_cnt[kCntOverflow]) {
			SYZ_TRY(set_rehash(ms, ms->nbuckets * 8, true));
			st->retries++;
			continue;
		}
		const uint64_t touched = ctx->h_cnt[kCntTouched];
		st->candidates += ctx->h_cnt[kCntCandidates];
		st->survivors += ctx->h_cnt[kCntAux2];
		if (touched && !*ns)
			SYZ_TRY(syzsig_set_make(ctx, touched, ns));  // newSignal.Merge allocates (signal.go:121-125)
		if (touched)
			SYZ_TRY(set_reserve(*ns, touched));
		SYZ_TRY(counters_reset(ctx));
		syzsig_set* nsp = *ns;
		if (ctx->timing)
			SYZ_HIP(hipEventRecord(ctx->ev[2], ctx->stream));
		k_decide<In><<<grid, 256, 0, ctx->stream>>>(ms->slots, ms->firsts, nsp ? nsp->slots : nullptr,
		                                            nsp ? nsp->nbuckets - 1 : 0, in, lm, ms->epoch, cand_slot,
		                                            cand_meta, cand_cnt, ctx->d_cnt);
		SYZ_HIP(hipGetLastError());
		if (ctx->timing)
			SYZ_HIP(hipEventRecord(ctx->ev[3], ctx->stream));
		SYZ_TRY(counters_fetch(ctx));
		if (ctx->timing) {
			float ms = 0;
			SYZ_HIP(hipEventElapsedTime(&ms, ctx->ev[2], ctx->ev[3]));
			st->decide_ms += ms;
		}
		if (ctx->h_cnt[kCntOverflow])
			return fail(SYZSIG_EIO, "newSignal overflow (internal error)");
		ms->len += ctx->h_cnt[kCntInserted];
		st->inserted += ctx->h_cnt[kCntInserted];
		st->changed += ctx->h_cnt[kCntChanged];
		if (nsp)
			nsp->len += ctx->h_cnt[kCntAux];
		st->runs++;
		return SYZSIG_OK;
	}
}

// Partitioned mode pays off once maxSignal no longer fits the L2s and the
// run is large; it needs record indices < 2^32.
static uint32_t parts_for(const syzsig_set* ms, uint64_t nrecs, uint64_t nrec_space)
{
	const syzsig_ctx* ctx = ms->ctx;
	const uint64_t bytes = ms->nslots() * 8;
	if (!ctx->part_mode || bytes < (32ull << 20) || nrecs < (1ull << 20) || nrec_space >= (1ull << 32))
		return 0;
	uint32_t parts = 8;
	while (parts < kMaxParts && bytes / parts > ctx->part_slice && parts < ms->nbuckets)
		parts <<= 1;
	return parts;
}

static uint32_t log2u(uint64_t x)
{
	uint32_t r = 0;
	while ((1ull << r) < x)
		r++;
	return r;
}

int triage_batch_impl(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const syzsig_batch* b,
                      syzsig_batch_stats* st)
{
	SYZ_HIP(hipMemsetAsync(b->new_bits, 0, ((b->nrec + 31) / 32) * 4, ctx->stream));
	if (b->ncalls)
		SYZ_HIP(hipMemsetAsync(b->call_new, 0, b->ncalls, ctx->stream));
	if (b->ncalls == 0 || b->nrec == 0) {
		SYZ_HIP(hipStreamSynchronize(ctx->stream));
		return SYZSIG_OK;
	}
	SYZ_TRY(set_ensure_triage_state(ms));
	std::vector<Run> runs;
	uint64_t total = 0;
	SYZ_TRY(plan_runs(ctx, b, &runs, &total));
	st->records = total;
	uint64_t maxrun = 0;
	for (auto& r : runs)
		maxrun = std::max(maxrun, r.c1 - r.c0);
	for (auto& r : runs) {
		CallsIn in;
		in.sigs = b->sigs;
		in.call_start = b->call_start;
		in.call_len = b->call_len;
		in.call_prio = b->call_prio;
		in.c0 = r.c0;
		in.c1 = r.c1;
		in.nrec = b->nrec;
		in.new_bits = b->new_bits;
		in.call_new = b->call_new;
		const uint64_t run_recs = runs.size() == 1 ? total : b->nrec;  // bound
		if (parts_for(ms, run_recs, b->nrec)) {
			// ---- partitioned: records regrouped by table region, one XCD per region
			void *cs, *cm, *cc, *pr, *po, *pm, *pc;
			const uint64_t nseg_max = run_recs / kPartSeg + kMaxParts + 1;
			const uint64_t nchunks = (r.c1 - r.c0 + kPartCPB - 1) / kPartCPB;
			SYZ_TRY(ws_get(ctx, 3, run_recs * 4 + 64, &cs));
			SYZ_TRY(ws_get(ctx, 4, run_recs * 4 + 64, &cm));
			SYZ_TRY(ws_get(ctx, 5, nseg_max * 4, &cc));
			SYZ_TRY(ws_get(ctx, 11, run_recs * 8 + 64, &pr));
			SYZ_TRY(ws_get(ctx, 12, run_recs * 4 + 64, &po));
			SYZ_TRY(ws_get(ctx, 13, (kMaxParts + 1) * 8 * 3, &pm));
			SYZ_TRY(ws_get(ctx, 14, nchunks * kMaxParts * 4 * 2 + 64, &pc));
			uint64_t* totals = (uint64_t*)pm;
			uint64_t* rec_base = totals + kMaxParts + 1;
			uint64_t* seg_base = rec_base + kMaxParts + 1;
			auto prep = [&](PartIn* pin, int* grid, syzsig_batch_stats* stp) -> int {
				const uint32_t parts = parts_for(ms, run_recs, b->nrec);
				if (!parts)
					return fail(SYZSIG_EIO, "partitioned triage lost its geometry (internal error)");
				const uint32_t shift = log2u(ms->nbuckets) - log2u(parts);
				uint32_t* counts = (uint32_t*)pc;
				uint32_t* offs = counts + nchunks * parts;
				if (ctx->timing)
					SYZ_HIP(hipEventRecord(ctx->ev[0], ctx->stream));
				const int pg = (int)std::min<uint64_t>(nchunks, 4096);
				k_part_count<<<pg, 256, 0, ctx->stream>>>(in, ms->nbuckets - 1, shift, parts, counts);
				k_part_scan_chunks<<<parts, 256, 0, ctx->stream>>>(counts, nchunks, parts, offs, totals);
				k_part_scan<<<1, 64, 0, ctx->stream>>>(totals, parts, rec_base, seg_base);
				k_part_scatter<<<pg, 256, 0, ctx->stream>>>(in, r.lm, ms->nbuckets - 1, shift, parts, offs, rec_base,
				                                            (uint64_t*)pr, (uint32_t*)po);
				SYZ_HIP(hipGetLastError());
				if (ctx->timing) {
					float t = 0;
					SYZ_HIP(hipEventRecord(ctx->ev[1], ctx->stream));
					SYZ_HIP(hipEventSynchronize(ctx->ev[1]));
					SYZ_HIP(hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]));
					stp->part_ms += t;
				}
				pin->recs = (const uint64_t*)pr;
				pin->orig = (const uint32_t*)po;
				pin->rec_base = rec_base;
				pin->seg_base = seg_base;
				pin->nparts = parts;
				stp->parts = parts;
				pin->c0 = r.c0;
				pin->new_bits = b->new_bits;
				pin->call_new = b->call_new;
				*grid = ctx->part_grid;  // multiple of 8: block b works on XCD b % 8's partitions
				return SYZSIG_OK;
			};
			SYZ_TRY(triage_run<PartIn>(ctx, ms, ns, prep, r.lm, (uint32_t*)cs, (uint32_t*)cm, (uint32_t*)cc, st));
		} else {
			void *cs, *cm, *cc;
			SYZ_TRY(ws_get(ctx, 3, b->nrec * 4, &cs));
			SYZ_TRY(ws_get(ctx, 4, b->nrec * 4, &cm));
			SYZ_TRY(ws_get(ctx, 5, maxrun * 4, &cc));
			auto prep = [&](CallsIn* cin, int* grid, syzsig_batch_stats*) -> int {
				*cin = in;
				*grid = grid_for((r.c1 - r.c0) * 64, 256, 4096);
				return SYZSIG_OK;
			};
			SYZ_TRY(triage_run<CallsIn>(ctx, ms, ns, prep, r.lm, (uint32_t*)cs, (uint32_t*)cm, (uint32_t*)cc, st));
		}
	}
	if ((double)ms->len > kMaxLoad * (double)ms->nslots())
		SYZ_TRY(set_rehash(ms, buckets_for(ms->len), false));
	st->new_signal_len = syzsig_len(*ns);
	return SYZSIG_OK;
}

// levels[] (ascending int8, <= 4) -> LevelMap
int level_map_from_levels(const int8_t* levels, uint32_t nlevels, LevelMap* lm)
{
	if (!levels || nlevels == 0 || nlevels > 4)
		return fail(SYZSIG_EINVAL, "levels: need 1..4 prio levels");
	bool present[256] = {false};
	for (uint32_t i = 0; i < nlevels; i++) {
		if (i && levels[i] <= levels[i - 1])
			return fail(SYZSIG_EINVAL, "levels: must be strictly ascending");
		present[(uint8_t)levels[i]] = true;
	}
	level_map_from(present, lm);
	return SYZSIG_OK;
}

int triage_records_impl(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const uint64_t* recs, uint64_t nrec,
                        const int8_t* levels, uint32_t nlevels, uint8_t* new_flags, syzsig_batch_stats* st)
{
	LevelMap lm;
	SYZ_TRY(level_map_from_levels(levels, nlevels, &lm));
	st->records = nrec;
	if (nrec == 0)
		return SYZSIG_OK;
	SYZ_HIP(hipMemsetAsync(new_flags, 0, nrec, ctx->stream));
	SYZ_TRY(set_ensure_triage_state(ms));
	const uint64_t nseg = (nrec + kSegRecs - 1) / kSegRecs;
	void *cs, *cm, *cc;
	SYZ_TRY(ws_get(ctx, 3, nrec * 4, &cs));
	SYZ_TRY(ws_get(ctx, 4, nrec * 4, &cm));
	SYZ_TRY(ws_get(ctx, 5, nseg * 4, &cc));
	auto prep = [&](RecsIn* in, int* grid, syzsig_batch_stats*) -> int {
		in->recs = recs;
		in->nrec = nrec;
		in->new_flags = new_flags;
		*grid = grid_for(nseg * 64, 256, 4096);
		return SYZSIG_OK;
	};
	SYZ_TRY(triage_run<RecsIn>(ctx, ms, ns, prep, lm, (uint32_t*)cs, (uint32_t*)cm, (uint32_t*)cc, st));
	if ((double)ms->len > kMaxLoad * (double)ms->nslots())
		SYZ_TRY(set_rehash(ms, buckets_for(ms->len), false));
	st->new_signal_len = syzsig_len(*ns);
	return SYZSIG_OK;
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzsig_triage_batch(syzsig_ctx* ctx, syzsig_set* max_signal, syzsig_set** new_signal, const syzsig_batch* b,
                        syzsig_batch_stats* stats)
{
	if (!ctx || !max_signal || !new_signal || !b)
		return fail(SYZSIG_EINVAL, "triage_batch: NULL argument");
	if (*new_signal == max_signal)
		return fail(SYZSIG_EINVAL, "triage_batch: new_signal aliases max_signal");
	if (b->nrec && (!b->sigs || !b->new_bits))
		return fail(SYZSIG_EINVAL, "triage_batch: NULL record arrays");
	if (b->ncalls && (!b->call_start || !b->call_len || !b->call_prio || !b->call_new))
		return fail(SYZSIG_EINVAL, "triage_batch: NULL call arrays");
	syzsig_batch_stats st;
	memset(&st, 0, sizeof(st));
	int rc = triage_batch_impl(ctx, max_signal, new_signal, b, &st);
	if (stats)
		*stats = st;
	return rc;
}

int syzsig_check_new_signal(syzsig_ctx* ctx, syzsig_set** max_signal, syzsig_set** new_signal, const uint32_t* sigs,
                            uint64_t nrec, const uint64_t* call_start, const uint32_t* call_len,
                            const uint8_t* call_prio, uint32_t ncalls, uint32_t* out_calls, uint32_t* n_out,
                            uint32_t* new_bits)
{
	if (!ctx || !max_signal || !new_signal || !n_out || (ncalls && (!call_start || !call_len || !call_prio)) ||
	    (nrec && !sigs) || (ncalls && !out_calls))
		return fail(SYZSIG_EINVAL, "check_new_signal: NULL argument");
	*n_out = 0;
	for (uint32_t i = 0; i < ncalls; i++)
		if (call_start[i] > nrec || call_len[i] > nrec - call_start[i])
			return fail(SYZSIG_EINVAL, "check_new_signal: call range outside sigs");
	if (!*max_signal)
		SYZ_TRY(syzsig_set_make(ctx, 0, max_signal));
	const uint64_t nwords = (nrec + 31) / 32;
	void *ds, *dcs, *dcl, *dcp, *dbits, *dnew;
	SYZ_TRY(ws_get(ctx, 24, nrec * 4 + 4, &ds));
	SYZ_TRY(ws_get(ctx, 25, ncalls * 8 + 8, &dcs));
	SYZ_TRY(ws_get(ctx, 26, ncalls * 4 + 4, &dcl));
	SYZ_TRY(ws_get(ctx, 27, ncalls + 1, &dcp));
	SYZ_TRY(ws_get(ctx, 28, nwords * 4 + 4, &dbits));
	SYZ_TRY(ws_get(ctx, 29, ncalls + 1, &dnew));
	if (nrec)
		SYZ_HIP(hipMemcpyAsync(ds, sigs, nrec * 4, hipMemcpyHostToDevice, ctx->stream));
	if (ncalls) {
		SYZ_HIP(hipMemcpyAsync(dcs, call_start, ncalls * 8, hipMemcpyHostToDevice, ctx->stream));
		SYZ_HIP(hipMemcpyAsync(dcl, call_len, ncalls * 4, hipMemcpyHostToDevice, ctx->stream));
		SYZ_HIP(hipMemcpyAsync(dcp, call_prio, ncalls, hipMemcpyHostToDevice, ctx->stream));
	}
	syzsig_batch b;
	b.sigs = (const uint32_t*)ds;
	b.call_start = (const uint64_t*)dcs;
	b.call_len = (const uint32_t*)dcl;
	b.call_prio = (const uint8_t*)dcp;
	b.ncalls = ncalls;
	b.nrec = nrec;
	b.new_bits = (uint32_t*)dbits;
	b.call_new = (uint8_t*)dnew;
	syzsig_batch_stats st;
	memset(&st, 0, sizeof(st));
	SYZ_TRY(triage_batch_impl(ctx, *max_signal, new_signal, &b, &st));
	std::vector<uint8_t> cn(ncalls);
	if (ncalls)
		SYZ_HIP(hipMemcpyAsync(cn.data(), dnew, ncalls, hipMemcpyDeviceToHost, ctx->stream));
	if (new_bits && nwords)
		SYZ_HIP(hipMemcpyAsync(new_bits, dbits, nwords * 4, hipMemcpyDeviceToHost, ctx->stream));
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	uint32_t n = 0;
	for (uint32_t i = 0; i < ncalls; i++)
		if (cn[i])
			out_calls[n++] = i;
	*n_out = n;
	return SYZSIG_OK;
}

int syzsig_triage_records_dev(syzsig_ctx* ctx, syzsig_set* shard, syzsig_set** new_signal, const uint64_t* d_recs,
                              uint64_t nrec, const int8_t* levels, uint32_t nlevels, uint8_t* d_new_flags,
                              syzsig_batch_stats* stats)
{
	if (!ctx || !shard || !new_signal || (nrec && (!d_recs || !d_new_flags)))
		return fail(SYZSIG_EINVAL, "triage_records: NULL argument");
	if (*new_signal == shard)
		return fail(SYZSIG_EINVAL, "triage_records: new_signal aliases the shard");
	syzsig_batch_stats st;
	memset(&st, 0, sizeof(st));
	int rc = triage_records_impl(ctx, shard, new_signal, d_recs, nrec, levels, nlevels, d_new_flags, &st);
	if (stats)
		*stats = st;
	return rc;
}

}  // extern "C"
