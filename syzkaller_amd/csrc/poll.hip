// poll.hip -- syz-manager/manager.go:1027-1052 Manager.Poll over a batch of
// polls, on device.
//
// Reference, per poll (in arrival order) of fuzzer f with a.MaxSignal s:
//   newMax := mgr.maxSignal.Diff(s.Deserialize())
//   if !newMax.Empty(): mgr.maxSignal.Merge(newMax); for every f1 != f: f1.newMaxSignal.Merge(newMax)
//   if !f.newMaxSignal.Empty(): reply = f.newMaxSignal.Serialize(); f.newMaxSignal = nil
//
// Batch restatement.  For element e let p_i = Deserialize(s_i)[e] (the last
// entry of e in s_i).  e is in newMax_i  <=>  p_i > max(M0[e], p_j for every
// earlier poll j carrying e) -- the same strictly-greater running maximum as
// checkNewSignal -- so newMax over the batch is a list of "events" (e, i, p)
// whose prios rise with i for each e.  Fan-out: an event of poll i reaches
// fuzzer g != f_i in g's next poll after i (its reply), or g's newMaxSignal
// after the batch if g does not poll again; g's newMaxSignal from before the
// batch goes into the reply of g's first poll.  Merge is max-prio, so every
// target (a reply, or a fuzzer's final newMaxSignal) is the max-merge of the
// (e, p) routed to it:
//   k_poll_x / rp_group        the entries grouped by element through the LDS
//                              partitions of recs.hip (no device-wide sort)
//   k_poll_part_walk           one workgroup per partition: its entries sorted
//                              by (element, entry index) in LDS (bitonic), then
//                              one thread per element: the events (read-only)
//   k_poll_commit              maxSignal.Merge of the events, once every target exists
//   k_poll_fanout              (target, e, p) of every event for every other
//                              fuzzer into one max-table keyed by (target, e)
//   k_poll_pre                 pre-batch newMaxSignal of polling fuzzers
//   k_poll_count / k_poll_scatter   the table into the target sets
#include <algorithm>
#include <vector>

#include <chrono>

#include "internal.h"

namespace syz {

constexpr uint64_t kPollEmpty = ~0ull;
constexpr uint32_t kPollMaxTargets = (1u << 24) - 2;  // targets < 2^24 - 1 keep a word != kPollEmpty
constexpr uint64_t kPollMaxNext = 1ull << 28;     // polls x fuzzers per batch (the dense next-target table)
constexpr uint64_t kPollMaxFanout = 1ull << 31;   // polled entries x fuzzers per batch (bounds the fan-out table)
constexpr uint64_t kPollMaxEntries = 1ull << 23;  // polled entries per batch (the element partitions' capacity)

// target-table word: target << 40 | elem << 8 | prio ^ 0x80 (key = the top 56 bits)
__device__ __forceinline__ uint64_t poll_word(uint32_t t, uint32_t e, uint32_t pb)
{
	return ((uint64_t)t << 40) | ((uint64_t)e << 8) | pb;
}

__device__ __forceinline__ uint64_t poll_hash(uint64_t k)
{
	k ^= k >> 33;
	k *= 0xff51afd7ed558ccdull;
	k ^= k >> 33;
	k *= 0xc4ceb9fe1a85ec53ull;
	k ^= k >> 33;
	return k;
}

// max-insert into the target table (C a power of two, sized >= 2 * entries)
__device__ __forceinline__ void poll_put(uint64_t* T, uint64_t C, uint64_t w)
{
	const uint64_t key = w >> 8;
	uint64_t h = poll_hash(key) & (C - 1);
	for (uint64_t step = 0; step < C; step++) {
		uint64_t s = T[h];
		if (s == kPollEmpty) {
			s = atomicCAS((unsigned long long*)&T[h], kPollEmpty, (unsigned long long)w);
			if (s == kPollEmpty)
				return;
		}
		if ((s >> 8) == key) {
			if (s < w)
				atomicMax((unsigned long long*)&T[h], (unsigned long long)w);
			return;
		}
		h = (h + 1) & (C - 1);
	}
}

// every entry's poll (poll_off as the caller gave it: entries from off[0] on)
__global__ __launch_bounds__(256) void k_poll_recpoll(const uint64_t* __restrict__ off, uint32_t K, uint32_t* rec_poll)
{
	const uint64_t o0 = off[0];
	for (uint32_t i = blockIdx.x; i < K; i += gridDim.x)
		for (uint64_t r = off[i] + threadIdx.x; r < off[i + 1]; r += blockDim.x)
			rec_poll[r - o0] = i;
}

// the entries for rp_group: e << 32 | entry index
__global__ void k_poll_x(const uint32_t* __restrict__ elems, uint64_t n, uint64_t* x)
{
	for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x)
		x[r] = ((uint64_t)elems[r] << 32) | r;
}

// One workgroup per element partition (<= kRpGroupCap entries, keys
// h_residual << 32 | entry index from rp_group).  The keys are sorted in LDS
// (bitonic, padded to a power of two), so each element's entries are one run
// in entry order -- poll order, and inside a poll the Serial's order -- and
// one thread per run walks it: M0[e], then each poll's last entry of e
// (Deserialize: a later duplicate wins), an event wherever the prio exceeds
// the running maximum.  Read-only on maxSignal: the events are committed by
// k_poll_commit once every target set exists, so a failed allocation leaves
// the manager untouched.  The block's events are gathered in LDS and written
// with one device atomic.
constexpr uint32_t kPollWalkThreads = 256;
__global__ __launch_bounds__(kPollWalkThreads) void k_poll_part_walk(const uint64_t* __restrict__ keys,
                                                                     const uint32_t* __restrict__ base, uint32_t pbits,
                                                                     const uint32_t* __restrict__ rec_poll,
                                                                     const int8_t* __restrict__ prios, const uint64_t* ms,
                                                                     uint64_t ms_bmask, uint64_t* ev,
                                                                     unsigned long long* nev,
                                                                     const unsigned long long* ctr)
{
	__shared__ uint64_t k[kRpGroupCap];
	__shared__ uint64_t out[kRpGroupCap];
	__shared__ uint32_t s_n;
	__shared__ unsigned long long s_base;
	if (ctr[kCntSpill])
		return;  // a partition past kRpGroupCap: the batch takes the sequential path
	const uint32_t p = blockIdx.x, tid = threadIdx.x, b0 = base[p], n = base[p + 1] - b0;
	if (n == 0)
		return;
	uint32_t N = 2;
	while (N < n)
		N <<= 1;
	for (uint32_t i = tid; i < N; i += kPollWalkThreads)
		k[i] = i < n ? keys[b0 + i] : ~0ull;
	if (tid == 0)
		s_n = 0;
	for (uint32_t size = 2; size <= N; size <<= 1) {
		for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
			__syncthreads();
			for (uint32_t t = tid; t < N / 2; t += kPollWalkThreads) {
				const uint32_t i = 2 * t - (t & (stride - 1)), j = i + stride;
				const uint64_t a = k[i], b = k[j];
				if ((a > b) == ((i & size) == 0)) {
					k[i] = b;
					k[j] = a;
				}
			}
		}
	}
	__syncthreads();
	const uint32_t hp = p << (32 - pbits);
	for (uint32_t i = tid; i < n; i += kPollWalkThreads) {
		const uint32_t hr = (uint32_t)(k[i] >> 32);
		if (i > 0 && (uint32_t)(k[i - 1] >> 32) == hr)
			continue;  // not the head of e's run
		const uint32_t e = fmix32_inv(hp | hr);
		uint64_t v = 0;
		int m = -1000;  // absent: below every prio (signal.go:79-81)
		if (tbl_lookup(ms, ms_bmask, e, v) >= 0 && slot_live(v))
			m = slot_prio(v);
		uint32_t poll_next = 0;
		for (uint32_t q = i; q < n && (uint32_t)(k[q] >> 32) == hr; q++) {
			const uint32_t r = (uint32_t)k[q], poll = q == i ? rec_poll[r] : poll_next;
			const bool more = q + 1 < n && (uint32_t)(k[q + 1] >> 32) == hr;
			poll_next = more ? rec_poll[(uint32_t)k[q + 1]] : 0;
			if (more && poll_next == poll)
				continue;  // an earlier duplicate inside one Serial
			const int pr = prios[r];
			if (pr > m) {
				out[atomicAdd(&s_n, 1u)] = ((uint64_t)e << 32) | ((uint64_t)(poll & 0xFFFFFFu) << 8) | prio_biased((int8_t)pr);
				m = pr;
			}
		}
	}
	__syncthreads();
	const uint32_t ne = s_n;
	if (tid == 0)
		s_base = ne ? atomicAdd(nev, (unsigned long long)ne) : 0;
	__syncthreads();
	for (uint32_t i = tid; i < ne; i += kPollWalkThreads)
		ev[s_base + i] = out[i];
}

// maxSignal.Merge(newMax_i) for every poll: the events, max-merged (an
// element's last event carries its final max, the earlier ones are below it).
__global__ void k_poll_commit(const uint64_t* __restrict__ ev, uint64_t n, uint64_t* ms, uint64_t ms_bmask,
                              unsigned long long* ctr)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < n; x += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t w = ev[x];
		const int rr = tbl_merge(ms, ms_bmask, (uint32_t)(w >> 32), (int8_t)((uint8_t)w ^ 0x80u));
		ins += rr == 1;
		ovf += rr < 0;
	}
	block_count(&ctr[kCntInserted], ins);
	block_count(&ctr[kCntOverflow], ovf);
}

// every event of poll i, for every fuzzer g != f_i: target next_target[i * F + g]
__global__ void k_poll_fanout(const uint64_t* __restrict__ ev, const unsigned long long* __restrict__ nev,
                              const uint32_t* __restrict__ poll_fuzzer, const uint32_t* __restrict__ next_target,
                              uint32_t F, uint64_t* T, uint64_t C)
{
	const uint64_t n = *nev * F;
	for (uint64_t x = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; x < n; x += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t w = ev[x / F];
		const uint32_t g = (uint32_t)(x % F), i = (uint32_t)(w >> 8) & 0xFFFFFF;
		if (poll_fuzzer[i] == g)
			continue;
		poll_put(T, C, poll_word(next_target[(uint64_t)i * F + g], (uint32_t)(w >> 32), (uint32_t)w & 0xFF));
	}
}

// a polling fuzzer's newMaxSignal from before the batch -> its first reply
__global__ void k_poll_pre(const uint64_t* __restrict__ slots, uint64_t nslots, uint32_t target, uint64_t* T,
                           uint64_t C)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t s = slots[i];
		if (slot_live(s))
			poll_put(T, C, poll_word(target, slot_key(s), (uint32_t)s & 0xFF));
	}
}

// Per-target counts (k_poll_count) and inserts (k_poll_scatter) are summed
// in LDS per workgroup when the targets fit (a batch has K + F of them, and
// thousands of workgroups adding into a few hundred global counters serialise
// on them), else with global atomics.
constexpr uint32_t kPollLdsTargets = 8192;

__global__ __launch_bounds__(256) void k_poll_count(const uint64_t* __restrict__ T, uint64_t C, unsigned int* tcount,
                                                    uint32_t ntargets)
{
	__shared__ unsigned int lc[kPollLdsTargets];
	const bool lds = ntargets <= kPollLdsTargets;
	if (lds) {
		for (uint32_t t = threadIdx.x; t < ntargets; t += blockDim.x)
			lc[t] = 0;
		__syncthreads();
	}
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < C; i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t w = T[i];
		if (w != kPollEmpty)
			atomicAdd(lds ? &lc[w >> 40] : &tcount[w >> 40], 1u);
	}
	if (lds) {
		__syncthreads();
		for (uint32_t t = threadIdx.x; t < ntargets; t += blockDim.x)
			if (lc[t])
				atomicAdd(&tcount[t], lc[t]);
	}
}

struct PollTarget {
	uint64_t* slots;
	uint64_t bmask;
};

__global__ __launch_bounds__(256) void k_poll_scatter(const uint64_t* __restrict__ T, uint64_t C,
                                                      const PollTarget* __restrict__ tg, unsigned int* tins,
                                                      uint32_t ntargets, unsigned long long* ctr)
{
	__shared__ unsigned int lc[kPollLdsTargets];
	const bool lds = ntargets <= kPollLdsTargets;
	if (lds) {
		for (uint32_t t = threadIdx.x; t < ntargets; t += blockDim.x)
			lc[t] = 0;
		__syncthreads();
	}
	uint64_t ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < C; i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t w = T[i];
		if (w == kPollEmpty)
			continue;
		const uint32_t t = (uint32_t)(w >> 40);
		const int r = tbl_merge(tg[t].slots, tg[t].bmask, (uint32_t)(w >> 8), (int8_t)((uint8_t)w ^ 0x80u));
		if (r == 1)
			atomicAdd(lds ? &lc[t] : &tins[t], 1u);
		ovf += r < 0;
	}
	if (lds) {
		__syncthreads();
		for (uint32_t t = threadIdx.x; t < ntargets; t += blockDim.x)
			if (lc[t])
				atomicAdd(&tins[t], lc[t]);
	}
	block_count(&ctr[kCntOverflow], ovf);
}

static uint64_t pow2_ge(uint64_t x)
{
	uint64_t p = 1;
	while (p < x)
		p <<= 1;
	return p;
}

}  // namespace syz

using namespace syz;

// Sets this call made, freed again if it fails before the commit.
struct PollFresh {
	std::vector<syzsig_set*> sets;
	~PollFresh()
	{
		for (syzsig_set* x : sets)
			syzsig_set_free(x);
	}
};

// The reference loop itself (manager.go:1027-1052), one poll after the other
// over the set ops: the exact path for a batch whose entries crowd one element
// partition past kRpGroupCap (a hot element polled thousands of times).
// All or nothing, like the batched path: the loop runs on clones of
// maxSignal and of every fuzzer's newMaxSignal, and only a loop that ran to
// the end swaps them in and hands out the replies; on any error the clones
// and the replies made so far are freed and the caller's sets are untouched.
static int poll_sequential(syzsig_ctx* ctx, syzsig_set** max_signal, syzsig_set** new_max, const uint32_t* poll_fuzzer,
                           const uint64_t* poll_off, const uint32_t* elems, const int8_t* prios, uint32_t npolls,
                           uint32_t nfuzzers, syzsig_set** replies)
{
	// (the set ops below record the context's own events: this path's
	// last_ms is host wall time over the loop, the stream drained at its end)
	const auto t0 = std::chrono::steady_clock::now();
	PollFresh work;  // clones and replies, freed unless the loop completes
	syzsig_set* ms = nullptr;
	SYZ_TRY(syzsig_set_clone(ctx, *max_signal, &ms));
	if (ms)
		work.sets.push_back(ms);
	std::vector<syzsig_set*> nm(nfuzzers, nullptr), rep(npolls, nullptr);
	for (uint32_t g = 0; g < nfuzzers; g++) {
		SYZ_TRY(syzsig_set_clone(ctx, new_max[g], &nm[g]));
		if (nm[g])
			work.sets.push_back(nm[g]);
	}
	for (uint32_t i = 0; i < npolls; i++) {
		if ((ctx->agg_dbg & SYZSIG_DEBUG_POLL_FAIL) && i + 1 == npolls && i > 0)
			return fail(SYZSIG_EIO, "manager_poll_batch: injected failure (SYZSIG_DEBUG_POLL_FAIL)");
		const uint32_t f = poll_fuzzer[i];
		const uint64_t a = poll_off[i], z = poll_off[i + 1];
		syzsig_set* d = nullptr;
		SYZ_TRY(syzsig_deserialize(ctx, elems + a, z - a, prios + a, z - a, &d));
		PollFresh nw;  // newMax of this poll, freed at the end of the iteration
		nw.sets.push_back(nullptr);
		const int rc = syzsig_diff(ctx, ms, d, &nw.sets[0]);
		syzsig_set_free(d);
		SYZ_TRY(rc);
		if (!syzsig_empty(nw.sets[0])) {
			syzsig_set* const ms0 = ms;
			SYZ_TRY(syzsig_merge(ctx, &ms, nw.sets[0]));
			if (!ms0)
				work.sets.push_back(ms);  // Merge allocated a nil maxSignal
			for (uint32_t g = 0; g < nfuzzers; g++) {
				if (g == f)
					continue;
				syzsig_set* const n0 = nm[g];
				SYZ_TRY(syzsig_merge(ctx, &nm[g], nw.sets[0]));
				if (!n0)
					work.sets.push_back(nm[g]);
			}
		}
		if (!syzsig_empty(nm[f])) {  // the reply takes the fuzzer's set (the clone is in work.sets)
			rep[i] = nm[f];
			nm[f] = nullptr;
		}
	}
	// commit: nothing below fails.  maxSignal keeps its handle (callers hold
	// it: the batched path merges in place too), so the clone's contents move
	// into it; the fuzzers' newMaxSignal handles are replaced, as the batched
	// path replaces a polled fuzzer's.
	work.sets.clear();
	if (*max_signal) {
		std::swap(**max_signal, *ms);
		syzsig_set_free(ms);  // (the old storage)
	} else {
		*max_signal = ms;  // nil, or allocated by a Merge
	}
	for (uint32_t g = 0; g < nfuzzers; g++) {
		syzsig_set_free(new_max[g]);
		new_max[g] = nm[g];
	}
	for (uint32_t i = 0; i < npolls; i++)
		replies[i] = rep[i];
	if (ctx->timing) {
		SYZ_HIP(hipStreamSynchronize(ctx->stream));
		ctx->last_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
	}
	return SYZSIG_OK;
}

extern "C" int syzsig_manager_poll_batch(syzsig_ctx* ctx, syzsig_set** max_signal, syzsig_set** new_max,
                                         uint32_t nfuzzers, const uint32_t* poll_fuzzer, const uint64_t* poll_off,
                                         const uint32_t* elems, const int8_t* prios, uint32_t npolls,
                                         syzsig_set** replies)
{
	SYZ_LOCK(ctx);
	if (!ctx || !max_signal || (nfuzzers && !new_max) || (npolls && (!poll_fuzzer || !poll_off || !replies)))
		return fail(SYZSIG_EINVAL, "manager_poll_batch: NULL argument");
	if ((uint64_t)npolls + nfuzzers > kPollMaxTargets)
		return fail(SYZSIG_ERANGE, "manager_poll_batch: too many polls + fuzzers");
	for (uint32_t i = 0; i < npolls; i++) {
		replies[i] = nullptr;
		if (poll_fuzzer[i] >= nfuzzers || poll_off[i + 1] < poll_off[i])
			return fail(SYZSIG_EINVAL, "manager_poll_batch: bad poll_fuzzer or poll_off");
	}
	if (npolls == 0)
		return SYZSIG_OK;
	const uint64_t n = poll_off[npolls] - poll_off[0];
	if (n && (!elems || !prios))
		return fail(SYZSIG_EINVAL, "manager_poll_batch: NULL Serial arrays");
	if (n > kPollMaxEntries)  // (one poll past it: signal.manager_poll cuts batches at it otherwise)
		return poll_sequential(ctx, max_signal, new_max, poll_fuzzer, poll_off, elems, prios, npolls, nfuzzers,
		                       replies);
	const uint32_t F = nfuzzers, K = npolls;
	// the dense next-target table (K * F) and the fan-out table (<= n * (F - 1)
	// events) are bounded before any state is touched
	if ((uint64_t)K * F > kPollMaxNext || n * (uint64_t)F > kPollMaxFanout)
		return fail(SYZSIG_ERANGE, "manager_poll_batch: polls x fuzzers or entries x fuzzers too large for one batch");
	const hipStream_t s = ctx->stream;
	// next target of (poll i, fuzzer g): g's next poll after i, else K + g (its final newMaxSignal)
	std::vector<uint32_t> next((uint64_t)K * F), last(F);
	for (uint32_t g = 0; g < F; g++)
		last[g] = K + g;
	for (uint32_t i = K; i-- > 0;) {
		std::copy(last.begin(), last.end(), next.begin() + (uint64_t)i * F);
		last[poll_fuzzer[i]] = i;
	}
	// Nothing the caller can see changes until every set is made and sized:
	// sets made here are freed again on an early return (PollFresh), and
	// maxSignal, the fuzzers' sets and the replies are written only by the
	// commit at the end, whose only failure is an internal overflow.
	PollFresh fresh;
	syzsig_set* ms = *max_signal;
	const bool fresh_ms = !ms;  // Merge allocates a nil maxSignal only for a non-empty newMax
	if (fresh_ms) {
		SYZ_TRY(syzsig_set_make(ctx, n, &ms));
		fresh.sets.push_back(ms);
	}
	SYZ_TRY(set_reserve(ms, n));  // (a growth keeps the contents)
	// uploads and scratch: entries, their grouping input, events, the target table
	void *de, *dp, *drp, *dx, *dev, *dnext;
	SYZ_TRY(ws_get(ctx, 40, n * 4 + 64, &de));
	SYZ_TRY(ws_get(ctx, 41, n + 64, &dp));
	SYZ_TRY(ws_get(ctx, 42, n * 4 + ((uint64_t)K + 1) * 8 + 64, &drp));
	uint64_t* doff = (uint64_t*)((uint32_t*)drp + ((n + 1) & ~1ull));
	SYZ_TRY(ws_get(ctx, 43, n * 8 + 64, &dx));
	SYZ_TRY(ws_get(ctx, 44, n * 8 + ((uint64_t)K * F + K) * 4 + 64, &dev));
	dnext = (uint64_t*)dev + n;
	uint32_t* dpf = (uint32_t*)dnext + (uint64_t)K * F;
	if (ctx->timing)  // (the call's stream work from its uploads to its last kernel: ctx last_ms)
		SYZ_HIP(hipEventRecord(ctx->ev[0], s));
	if (n) {
		SYZ_HIP(hipMemcpyAsync(de, elems + poll_off[0], n * 4, hipMemcpyHostToDevice, s));
		SYZ_HIP(hipMemcpyAsync(dp, prios + poll_off[0], n, hipMemcpyHostToDevice, s));
		SYZ_HIP(hipMemcpyAsync(doff, poll_off, ((uint64_t)K + 1) * 8, hipMemcpyHostToDevice, s));
		k_poll_recpoll<<<std::min<uint32_t>(K, 65536), 256, 0, s>>>(doff, K, (uint32_t*)drp);
	}
	if ((uint64_t)K * F)
		SYZ_HIP(hipMemcpyAsync(dnext, next.data(), (uint64_t)K * F * 4, hipMemcpyHostToDevice, s));
	SYZ_HIP(hipMemcpyAsync(dpf, poll_fuzzer, (uint64_t)K * 4, hipMemcpyHostToDevice, s));
	SYZ_TRY(counters_reset(ctx));
	unsigned long long* nev = &ctx->d_cnt[kCntAux];
	if (n) {
		k_poll_x<<<grid_for(n, 256), 256, 0, s>>>((const uint32_t*)de, n, (uint64_t*)dx);
		uint64_t* keys;
		uint32_t* base;
		uint32_t pbits;
		SYZ_TRY(rp_group(ctx, (const uint64_t*)dx, n, &keys, &base, &pbits, ctx->d_cnt));  // (zeroes the counters)
		k_poll_part_walk<<<1u << pbits, kPollWalkThreads, 0, s>>>(keys, base, pbits, (const uint32_t*)drp,
		                                                          (const int8_t*)dp, ms->slots, ms->nbuckets - 1,
		                                                          (uint64_t*)dev, nev, ctx->d_cnt);
		SYZ_HIP(hipGetLastError());
	}
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->h_cnt[kCntSpill]) {
		// an element partition past the LDS capacity: nothing was touched; the
		// reference loop instead (a fresh maxSignal made above is dropped again)
		fresh.sets.clear();
		if (fresh_ms)
			syzsig_set_free(ms);
		return poll_sequential(ctx, max_signal, new_max, poll_fuzzer, poll_off, elems, prios, npolls, nfuzzers,
		                       replies);
	}
	const uint64_t E = ctx->h_cnt[kCntAux];
	// the target table: every event for every other fuzzer + pre-batch sets of polling fuzzers
	uint64_t entries = E * (F ? F - 1 : 0);
	for (uint32_t g = 0; g < F; g++)
		if (last[g] < K)
			entries += syzsig_len(new_max[g]);
	const uint64_t C = pow2_ge(std::max<uint64_t>(2 * entries, 1024));
	void *dT, *dtc;
	SYZ_TRY(ws_get(ctx, 46, C * 8 + 64, &dT));
	SYZ_TRY(ws_get(ctx, 47, ((uint64_t)K + F) * 8 + 64, &dtc));
	unsigned int* tcount = (unsigned int*)dtc;
	unsigned int* tins = tcount + K + F;
	SYZ_HIP(hipMemsetAsync(dT, 0xff, C * 8, s));
	SYZ_HIP(hipMemsetAsync(dtc, 0, ((uint64_t)K + F) * 8, s));
	if (E && F > 1)
		k_poll_fanout<<<grid_for(E * F, 256, 8192), 256, 0, s>>>((const uint64_t*)dev, nev, dpf,
		                                                         (const uint32_t*)dnext, F, (uint64_t*)dT, C);
	for (uint32_t g = 0; g < F; g++)
		if (last[g] < K && syzsig_len(new_max[g]))
			k_poll_pre<<<grid_for(new_max[g]->nslots(), 256), 256, 0, s>>>(new_max[g]->slots, new_max[g]->nslots(),
			                                                               last[g], (uint64_t*)dT, C);
	k_poll_count<<<grid_for(C, 256, 2048), 256, 0, s>>>((const uint64_t*)dT, C, tcount, K + F);
	SYZ_HIP(hipGetLastError());
	std::vector<unsigned int> hc((uint64_t)K + F);
	SYZ_HIP(hipMemcpyAsync(hc.data(), tcount, ((uint64_t)K + F) * 4, hipMemcpyDeviceToHost, s));
	SYZ_HIP(hipStreamSynchronize(s));
	// target sets: the replies, then every fuzzer's newMaxSignal after the batch.
	// A polling fuzzer's own set goes into its first reply and is nil after its
	// poll (manager.go:1049-1052), so its final set is a new one.
	std::vector<syzsig_set*> tset((uint64_t)K + F, nullptr);
	std::vector<PollTarget> tg((uint64_t)K + F, PollTarget{nullptr, 0});
	for (uint64_t t = 0; t < (uint64_t)K + F; t++) {
		if (!hc[t])
			continue;
		const bool keep = t >= K && last[t - K] >= K && new_max[t - K];  // a non-polling fuzzer's existing set
		if (keep) {
			tset[t] = new_max[t - K];
			SYZ_TRY(set_reserve(tset[t], hc[t]));
		} else {
			SYZ_TRY(syzsig_set_make(ctx, hc[t], &tset[t]));
			fresh.sets.push_back(tset[t]);
		}
		tg[t] = PollTarget{tset[t]->slots, tset[t]->nbuckets - 1};
	}
	void* dtg;
	SYZ_TRY(ws_get(ctx, 39, ((uint64_t)K + F) * sizeof(PollTarget) + 64, &dtg));
	SYZ_HIP(hipMemcpyAsync(dtg, tg.data(), ((uint64_t)K + F) * sizeof(PollTarget), hipMemcpyHostToDevice, s));
	// ---- commit: maxSignal.Merge of the events, the targets filled ----
	// (the event count is passed by value: the counter reset clears *nev)
	SYZ_TRY(counters_reset(ctx));
	if (E)
		k_poll_commit<<<grid_for(E, 256, 8192), 256, 0, s>>>((const uint64_t*)dev, E, ms->slots, ms->nbuckets - 1,
		                                                     ctx->d_cnt);
	k_poll_scatter<<<grid_for(C, 256, 2048), 256, 0, s>>>((const uint64_t*)dT, C, (const PollTarget*)dtg, tins, K + F,
	                                                      ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	std::vector<unsigned int> hi((uint64_t)K + F);
	SYZ_HIP(hipMemcpyAsync(hi.data(), tins, ((uint64_t)K + F) * 4, hipMemcpyDeviceToHost, s));
	if (ctx->timing)
		SYZ_HIP(hipEventRecord(ctx->ev[1], s));
	SYZ_TRY(counters_fetch(ctx));  // (synchronizes: hi and tg are consumed)
	if (ctx->timing) {
		float t = 0;
		SYZ_HIP(hipEventElapsedTime(&t, ctx->ev[0], ctx->ev[1]));
		ctx->last_ms = t;
	}
	if (ctx->h_cnt[kCntOverflow])
		return fail(SYZSIG_EIO, "manager_poll_batch: table overflow after reserve (internal error)");
	fresh.sets.clear();  // everything made here is handed out now
	ms->len += ctx->h_cnt[kCntInserted];
	if (fresh_ms && !E)
		syzsig_set_free(ms);  // nothing merged: maxSignal stays nil
	else
		*max_signal = ms;
	for (uint32_t g = 0; g < F; g++) {
		if (last[g] < K) {  // polled: the old set went into a reply; the final one is new (or nil)
			syzsig_set_free(new_max[g]);
			new_max[g] = tset[K + g];
		} else if (!new_max[g]) {
			new_max[g] = tset[K + g];
		}
	}
	for (uint64_t t = 0; t < (uint64_t)K + F; t++)
		if (tset[t])
			tset[t]->len += hi[t];
	for (uint32_t i = 0; i < K; i++)
		replies[i] = tset[i];
	return SYZSIG_OK;
}
