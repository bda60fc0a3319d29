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
// (Large runs take the aggregation path of agg.hip instead.)
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

int batch_total_records(syzsig_ctx* ctx, const syzsig_batch* b, uint64_t* total, uint32_t prio_mask[8])
{
	void* dmask;
	SYZ_TRY(ws_get(ctx, 6, 64, &dmask));
	SYZ_HIP(hipMemsetAsync(dmask, 0, 48, ctx->stream));
	k_prio_presence<<<grid_for(b->ncalls, 256, 256), 256, 0, ctx->stream>>>(
	    b->call_prio, b->call_len, b->call_start, b->ncalls, b->nrec, (uint32_t*)dmask,
	    (unsigned long long*)((char*)dmask + 32), (unsigned long long*)((char*)dmask + 40));
	SYZ_HIP(hipGetLastError());
	uint32_t* hmask = (uint32_t*)(ctx->h_pin + kPinMask);
	SYZ_HIP(hipMemcpyAsync(hmask, dmask, 48, hipMemcpyDeviceToHost, ctx->stream));
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	memcpy(total, &hmask[8], 8);
	uint64_t nbad;
	memcpy(&nbad, &hmask[10], 8);
	if (nbad)
		return fail(SYZSIG_EINVAL, "triage_batch: a call range lies outside [0, nrec) or has >= 2^24 records");
	if (prio_mask)
		memcpy(prio_mask, hmask, 32);
	return SYZSIG_OK;
}

static int plan_runs(syzsig_ctx* ctx, const syzsig_batch* b, std::vector<Run>* runs, uint64_t* total_recs)
{
	uint32_t hmask[8];
	SYZ_TRY(batch_total_records(ctx, b, total_recs, hmask));
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
template <typename In>
static void launch_probe(syzsig_ctx* ctx, int grid, syzsig_set* ms, const In& in, const LevelMap& lm,
                         uint32_t* cand_slot, uint32_t* cand_meta, uint32_t* cand_cnt)
{
	k_probe<In, 1, 128><<<grid, 256, 0, ctx->stream>>>(ms->slots, ms->nbuckets - 1, ms->firsts, ms->touched, in, lm,
	                                                   ms->epoch, cand_slot, cand_meta, cand_cnt, ctx->d_cnt, 0);
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
		if (ctx->h_cnt[kCntError]) {
			// The valid records of this launch already left absent markers and run
			// hints in maxSignal; a same-size rehash that drops absent slots and
			// masks hints restores exactly M0 before the error is reported.
			SYZ_TRY(set_rehash(ms, ms->nbuckets, true));
			return fail(SYZSIG_EINVAL, "triage: a call range lies outside [0, nrec), a call has >= 2^24 "
			                           "records, or a record's prio level is out of range");
		}
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

// The aggregation path (agg.hip) pays off once a run is large: one maxSignal
// probe per distinct element instead of one per record.
static bool use_agg(const syzsig_ctx* ctx, uint64_t run_recs, uint64_t nrec_space)
{
	return nrec_space < (1ull << 32) && (ctx->part_mode == 2 || (ctx->part_mode == 1 && run_recs >= (1ull << 20)));
}

int triage_batch_impl(syzsig_ctx* ctx, syzsig_set* ms, syzsig_set** ns, const syzsig_batch* b,
                      syzsig_batch_stats* st)
{
	std::vector<Run> runs;
	uint64_t total = 0;
	uint64_t* pairs = nullptr;
	uint64_t npairs = 0;
	if (b->ncalls && b->nrec && b->ncalls <= kSerialMask && use_agg(ctx, b->nrec, b->nrec) && !b->new_bits) {
		// a large batch: one aggregation run without the presence pass's round
		// trip (levels 0..3 assumed and checked on device)
		bool done = false;
		SYZ_TRY(agg_triage_optimistic(ctx, ms, ns, b, st, &pairs, &npairs, &done));
		if (done)
			goto finish;
	}
	if (b->new_bits)
		SYZ_HIP(hipMemsetAsync(b->new_bits, 0, ((b->nrec + 31) / 32) * 4, ctx->stream));
	if (b->ncalls)
		SYZ_HIP(hipMemsetAsync(b->call_new, 0, b->ncalls, ctx->stream));
	if (b->ncalls == 0 || b->nrec == 0) {
		SYZ_HIP(hipStreamSynchronize(ctx->stream));
		return SYZSIG_OK;
	}
	SYZ_TRY(plan_runs(ctx, b, &runs, &total));
	st->records = total;
	{
	uint64_t maxrun = 0;
	for (auto& r : runs)
		maxrun = std::max(maxrun, r.c1 - r.c0);
	for (auto& r : runs) {
		const uint64_t run_recs = runs.size() == 1 ? total : b->nrec;  // bound
		if (use_agg(ctx, run_recs, b->nrec)) {
			const uint64_t p0 = npairs;
			SYZ_TRY(agg_triage_run(ctx, ms, ns, b, r.c0, r.c1, r.lm, run_recs, st, &pairs, &npairs));
			SYZ_TRY(agg_mark_bits(ctx, b, r.c0, r.c1, pairs, p0, npairs));
			continue;
		}
		// per-call path: probe + decide against maxSignal, per-record bits
		SYZ_TRY(set_ensure_triage_state(ms));
		uint32_t* bits = b->new_bits;
		if (!bits) {
			void* ib;
			SYZ_TRY(ws_get(ctx, 12, ((b->nrec + 31) / 32) * 4 + 64, &ib));
			bits = (uint32_t*)ib;
			SYZ_HIP(hipMemsetAsync(bits, 0, ((b->nrec + 31) / 32) * 4, ctx->stream));
		}
		CallsIn in;
		in.sigs = b->sigs;
		in.call_start = b->call_start;
		in.call_len = b->call_len;
		in.call_prio = b->call_prio;
		in.c0 = r.c0;
		in.c1 = r.c1;
		in.nrec = b->nrec;
		in.new_bits = bits;
		in.call_new = b->call_new;
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
		SYZ_TRY(pairs_from_bits(ctx, b, bits, r.c0, r.c1, run_recs, &pairs, &npairs));
	}
	}
finish:
	if ((double)ms->len > kMaxLoad * (double)ms->nslots())
		SYZ_TRY(set_rehash(ms, buckets_for(ms->len), false));
	st->new_signal_len = syzsig_len(*ns);
	st->new_pairs = npairs;
	if (b->new_pairs && npairs && pairs != b->new_pairs) {
		SYZ_HIP(hipMemcpyAsync(b->new_pairs, pairs, std::min(npairs, b->new_pairs_cap) * 8, hipMemcpyDeviceToDevice,
		                       ctx->stream));
	}
	SYZ_HIP(hipStreamSynchronize(ctx->stream));  // (idle unless a copy or a rehash is queued)
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
                        const int8_t* levels, uint32_t nlevels, uint8_t* new_flags, syzsig_batch_stats* st,
                        bool allow_lds)
{
	LevelMap lm;
	SYZ_TRY(level_map_from_levels(levels, nlevels, &lm));
	st->records = nrec;
	if (nrec == 0)
		return SYZSIG_OK;
	SYZ_HIP(hipMemsetAsync(new_flags, 0, nrec, ctx->stream));
	if (nrec >= (1ull << 20) && nrec < (1ull << 31) && ctx->part_mode != 0 && allow_lds) {
		// partitioned by element through LDS (recs.hip); a partition past the LDS
		// capacity (a hot element's records in a generic input) voids that run
		// before anything is committed and the per-record path below runs instead
		bool done = false;
		SYZ_TRY(rp_triage_records(ctx, ms, ns, recs, nrec, lm, new_flags, st, &done));
		if (done) {
			if ((double)ms->len > kMaxLoad * (double)ms->nslots())
				SYZ_TRY(set_rehash(ms, buckets_for(ms->len), false));
			st->new_signal_len = syzsig_len(*ns);
			return SYZSIG_OK;
		}
	}
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
	SYZ_LOCK(ctx);
	if (!ctx || !max_signal || !new_signal || !b)
		return fail(SYZSIG_EINVAL, "triage_batch: NULL argument");
	if (*new_signal == max_signal)
		return fail(SYZSIG_EINVAL, "triage_batch: new_signal aliases max_signal");
	if (b->nrec && !b->sigs)
		return fail(SYZSIG_EINVAL, "triage_batch: NULL record arrays");
	if (b->new_pairs_cap && !b->new_pairs)
		return fail(SYZSIG_EINVAL, "triage_batch: new_pairs_cap without new_pairs");
	if (b->ncalls && (!b->call_start || !b->call_len || !b->call_prio || !b->call_new))
		return fail(SYZSIG_EINVAL, "triage_batch: NULL call arrays");
	SYZ_TRY(set_check_idle(max_signal));
	SYZ_TRY(set_check_idle(*new_signal));
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
	SYZ_LOCK(ctx);
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
	b.new_pairs = nullptr;
	b.new_pairs_cap = 0;
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
	SYZ_LOCK(ctx);
	if (!ctx || !shard || !new_signal || (nrec && (!d_recs || !d_new_flags)))
		return fail(SYZSIG_EINVAL, "triage_records: NULL argument");
	if (*new_signal == shard)
		return fail(SYZSIG_EINVAL, "triage_records: new_signal aliases the shard");
	SYZ_TRY(set_check_idle(shard));
	SYZ_TRY(set_check_idle(*new_signal));
	syzsig_batch_stats st;
	memset(&st, 0, sizeof(st));
	int rc = triage_records_impl(ctx, shard, new_signal, d_recs, nrec, levels, nlevels, d_new_flags, &st, true);
	if (stats)
		*stats = st;
	return rc;
}

}  // extern "C"
