// table.hip -- device-resident Signal (pkg/signal/signal.go) and its algebra.
//
// A Signal is an open-addressed table of u64 slots (encoding: common.h) in
// 64-B buckets of 8 slots, probed bucket-linearly from fmix32(elem).  Every
// operation is one or two grid-stride kernels on the context stream; results
// are sized from the operation's bound (len(s1), len(raw), ...) so inserts
// never overflow, and the live count comes back through a block-aggregated
// device counter.
#include <algorithm>

#include "internal.h"

#include <vector>

namespace syz {

// ---------------------------------------------------------------- kernels

// helper: exclusive rank of `pred` within the block + block total (all threads call)
__device__ __forceinline__ uint32_t block_rank(bool pred, uint32_t* total)
{
	__shared__ uint32_t wcount[16];
	uint64_t m = __ballot(pred);
	uint32_t w = threadIdx.x >> 6;
	if (lane_id() == 0)
		wcount[w] = (uint32_t)__popcll(m);
	__syncthreads();
	uint32_t base = 0, tot = 0;
	for (uint32_t i = 0; i < (blockDim.x >> 6); i++) {
		if (i < w)
			base += wcount[i];
		tot += wcount[i];
	}
	__syncthreads();
	*total = tot;
	return base + lane_rank(m);
}

__global__ void k_rehash(const uint64_t* __restrict__ old, uint64_t nslots, uint64_t* nw, uint64_t bmask,
                         int drop_absent, unsigned long long* cnt)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t s = old[i] & ~kHintMask;  // a restarted triage run leaves hints behind
		if (s == kSlotEmpty || (drop_absent && !slot_live(s)))
			continue;
		uint64_t prev;
		if (tbl_find_or_insert(nw, bmask, slot_key(s), s, prev, max_probe_for(bmask)) < 0)
			ovf++;
		else
			ins += prev == 0;
	}
	block_count(&cnt[kCntInserted], ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// FromRaw (signal.go:31-40): s[e] = prio for every raw element.
__global__ void k_from_raw(uint64_t* slots, uint64_t bmask, const uint32_t* __restrict__ raw, uint64_t n,
                           int8_t prio, unsigned long long* cnt)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		int r = tbl_merge(slots, bmask, raw[i], prio);
		ins += r == 1;
		ovf += r < 0;
	}
	block_count(&cnt[kCntInserted], ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// Deserialize (signal.go:59-71), pass 1: the LAST index of each element wins
// (a later `s[e] = p` overwrites).  The slot temporarily holds 0x80000000|index.
__global__ void k_deser_index(uint64_t* slots, uint64_t bmask, const uint32_t* __restrict__ elems, uint64_t n,
                              unsigned long long* cnt)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		uint32_t e = elems[i];
		uint64_t v = ((uint64_t)e << 32) | 0x80000000ull | i, old;
		int64_t idx = tbl_find_or_insert(slots, bmask, e, v, old, max_probe_for(bmask));
		if (idx < 0) {
			ovf++;
			continue;
		}
		if (old == 0)
			ins++;
		else if (old < v)
			atomicMax(reinterpret_cast<unsigned long long*>(slots + idx), (unsigned long long)v);
	}
	block_count(&cnt[kCntInserted], ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// Deserialize pass 2: index -> prio.
__global__ void k_deser_prio(uint64_t* slots, uint64_t nslots, const int8_t* __restrict__ prios)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t s = slots[i];
		if (s == kSlotEmpty)
			continue;
		slots[i] = make_slot(slot_key(s), prios[s & 0x7fffffffull]);
	}
}

// Diff (signal.go:73-88): res[e] = p1 for (e,p1) in s1 unless s[e] >= p1.
__global__ void k_diff(const uint64_t* __restrict__ s, uint64_t s_bmask, int have_s, const uint64_t* __restrict__ s1,
                       uint64_t s1_nslots, uint64_t* res, uint64_t r_bmask, unsigned long long* cnt)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < s1_nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t v1 = s1[i];
		if (!slot_live(v1))
			continue;
		uint64_t v;
		if (have_s && tbl_lookup(s, s_bmask, slot_key(v1), v) >= 0 && slot_prio(v) >= slot_prio(v1))
			continue;
		int r = tbl_merge(res, r_bmask, slot_key(v1), slot_prio(v1));
		ins += r == 1;
		ovf += r < 0;
	}
	block_count(&cnt[kCntInserted], ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// DiffRaw (signal.go:90-102): res[e] = prio for raw e unless s[e] >= prio (int8).
__global__ void k_diff_raw(const uint64_t* __restrict__ s, uint64_t s_bmask, int have_s,
                           const uint32_t* __restrict__ raw, uint64_t n, int8_t prio, uint64_t* res,
                           uint64_t r_bmask, unsigned long long* cnt)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		uint32_t e = raw[i];
		uint64_t v;
		if (have_s && tbl_lookup(s, s_bmask, e, v) >= 0 && slot_prio(v) >= prio)
			continue;
		int r = tbl_merge(res, r_bmask, e, prio);
		ins += r == 1;
		ovf += r < 0;
	}
	block_count(&cnt[kCntInserted], ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// Intersection (signal.go:104-115): res[e] = p for (e,p) in s if s1[e] >= p.
__global__ void k_intersection(const uint64_t* __restrict__ s, uint64_t s_nslots, const uint64_t* __restrict__ s1,
                               uint64_t s1_bmask, uint64_t* res, uint64_t r_bmask, unsigned long long* cnt)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < s_nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t v = s[i];
		if (!slot_live(v))
			continue;
		uint64_t v1;
		if (tbl_lookup(s1, s1_bmask, slot_key(v), v1) < 0 || slot_prio(v1) < slot_prio(v))
			continue;
		int r = tbl_merge(res, r_bmask, slot_key(v), slot_prio(v));
		ins += r == 1;
		ovf += r < 0;
	}
	block_count(&cnt[kCntInserted], ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// Merge (signal.go:117-131): s[e] = p1 if absent or s[e] < p1.
__global__ void k_merge(uint64_t* dst, uint64_t d_bmask, const uint64_t* __restrict__ s1, uint64_t s1_nslots,
                        unsigned long long* cnt)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < s1_nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t v1 = s1[i];
		if (!slot_live(v1))
			continue;
		int r = tbl_merge(dst, d_bmask, slot_key(v1), slot_prio(v1));
		ins += r == 1;
		ovf += r < 0;
	}
	block_count(&cnt[kCntInserted], ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// Merge of packed (elem << 32 | prio_biased) pairs, e.g. a triage delta list.
__global__ void k_merge_pairs(uint64_t* dst, uint64_t d_bmask, const uint64_t* __restrict__ pairs, uint64_t n,
                              unsigned long long* cnt)
{
	uint64_t ins = 0, ovf = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
		uint64_t p = pairs[i];
		int r = tbl_merge(dst, d_bmask, (uint32_t)(p >> 32), (int8_t)((uint8_t)p ^ 0x80u));
		ins += r == 1;
		ovf += r < 0;
	}
	block_count(&cnt[kCntInserted], ins);
	block_count(&cnt[kCntOverflow], ovf);
}

// Serialize (signal.go:42-57) in three passes: per-chunk live counts, an
// exclusive scan of the (<= 2048) chunk counts, ordered per-chunk writes.
// Snapshot restore by keys (syzsig_set_restore_keys): the slot of every key of
// `keys` in dst, found before anything is written (a restored slot may go
// empty and would cut the probe sequences of later lookups), then src's word
// copied into each.
__global__ void k_restore_find(const uint64_t* __restrict__ dst, uint64_t d_bmask, const uint64_t* __restrict__ keys,
                               uint64_t k_nslots, int64_t* idx)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < k_nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t w = keys[i];
		uint64_t v = 0;
		idx[i] = slot_live(w) ? tbl_lookup(dst, d_bmask, slot_key(w), v) : -1;
	}
}

__global__ void k_restore_apply(uint64_t* dst, const uint64_t* __restrict__ src, const int64_t* __restrict__ idx,
                                uint64_t k_nslots)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < k_nslots;
	     i += (uint64_t)gridDim.x * blockDim.x) {
		const int64_t j = idx[i];
		if (j >= 0)
			dst[j] = src[j];
	}
}

__global__ void k_slots_differ(const uint64_t* __restrict__ a, const uint64_t* __restrict__ b, uint64_t n,
                               unsigned long long* ndiff)
{
	uint64_t d = 0;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
		d += a[i] != b[i];
	block_count(ndiff, d);
}

__global__ void k_count_live(const uint64_t* __restrict__ slots, uint64_t nslots, uint64_t chunk,
                             unsigned long long* counts)
{
	uint64_t lo = blockIdx.x * chunk, hi = min(nslots, lo + chunk), c = 0;
	for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
		c += slot_live(slots[i]);
	__shared__ unsigned long long part;
	if (threadIdx.x == 0)
		part = 0;
	__syncthreads();
	c = wave_sum_u64(c);
	if (lane_id() == 0)
		atomicAdd(&part, (unsigned long long)c);
	__syncthreads();
	if (threadIdx.x == 0)
		counts[blockIdx.x] = part;
}

// exclusive scan of the per-block counts in place, *total = their sum: one
// workgroup, 1024 counts per step (a serial loop over them was a chain of
// dependent global loads, ~17 us per Serialize of a small set)
__global__ __launch_bounds__(1024) void k_scan_counts(unsigned long long* counts, uint32_t n,
                                                      unsigned long long* total)
{
	__shared__ unsigned long long wsum[16];
	__shared__ unsigned long long s_carry;
	const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
	if (tid == 0)
		s_carry = 0;
	for (uint32_t b = 0; b < n; b += 1024) {
		const uint32_t i = b + tid;
		const unsigned long long x = i < n ? counts[i] : 0;
		unsigned long long inc = x;
#pragma unroll
		for (uint32_t d = 1; d < 64; d <<= 1) {
			const unsigned long long y = __shfl_up(inc, d, 64);
			inc += lane >= d ? y : 0;
		}
		if (lane == 63)
			wsum[w] = inc;
		__syncthreads();
		unsigned long long pre = s_carry, tot = 0;
		for (uint32_t k = 0; k < 16; k++) {
			pre += k < w ? wsum[k] : 0;
			tot += wsum[k];
		}
		if (i < n)
			counts[i] = pre + inc - x;
		__syncthreads();  // wsum and s_carry are rewritten by the next step
		if (tid == 0)
			s_carry += tot;
	}
	__syncthreads();
	if (tid == 0)
		*total = s_carry;
}

__global__ void k_write_live(const uint64_t* __restrict__ slots, uint64_t nslots, uint64_t chunk,
                             const unsigned long long* __restrict__ offs, uint32_t* elems, int8_t* prios,
                             uint64_t cap)
{
	uint64_t lo = blockIdx.x * chunk, hi = min(nslots, lo + chunk);
	uint64_t pos = offs[blockIdx.x];
	for (uint64_t base = lo; base < hi; base += blockDim.x) {
		uint64_t i = base + threadIdx.x;
		uint64_t s = i < hi ? slots[i] : 0;
		bool live = slot_live(s);
		uint32_t tot;
		uint32_t r = block_rank(live, &tot);
		if (live && pos + r < cap) {
			elems[pos + r] = slot_key(s);
			prios[pos + r] = slot_prio(s);
		}
		pos += tot;
	}
}

// the batch Serialize: block b of the launch covers chunk (b - blk0) of the
// set blk_set[b]; one scan over every block's count places each set's
// entries right after the previous set's (their live counts are their Lens)
struct SerDesc {
	const uint64_t* slots;
	uint64_t nslots, chunk;
	uint32_t blk0, pad;
};

__global__ void k_count_live_multi(const SerDesc* __restrict__ d, const uint32_t* __restrict__ blk_set,
                                   unsigned long long* counts)
{
	const SerDesc sd = d[blk_set[blockIdx.x]];
	const uint64_t lo = (blockIdx.x - sd.blk0) * sd.chunk, hi = min(sd.nslots, lo + sd.chunk);
	uint64_t c = 0;
	for (uint64_t i = lo + threadIdx.x; i < hi; i += blockDim.x)
		c += slot_live(sd.slots[i]);
	__shared__ unsigned long long part;
	if (threadIdx.x == 0)
		part = 0;
	__syncthreads();
	c = wave_sum_u64(c);
	if (lane_id() == 0)
		atomicAdd(&part, (unsigned long long)c);
	__syncthreads();
	if (threadIdx.x == 0)
		counts[blockIdx.x] = part;
}

__global__ void k_write_live_multi(const SerDesc* __restrict__ d, const uint32_t* __restrict__ blk_set,
                                   const unsigned long long* __restrict__ offs, uint32_t* elems, int8_t* prios)
{
	const SerDesc sd = d[blk_set[blockIdx.x]];
	const uint64_t lo = (blockIdx.x - sd.blk0) * sd.chunk, hi = min(sd.nslots, lo + sd.chunk);
	uint64_t pos = offs[blockIdx.x];
	for (uint64_t base = lo; base < hi; base += blockDim.x) {
		const uint64_t i = base + threadIdx.x;
		const uint64_t sl = i < hi ? sd.slots[i] : 0;
		const bool live = slot_live(sl);
		uint32_t tot;
		const uint32_t r = block_rank(live, &tot);
		if (live) {
			elems[pos + r] = slot_key(sl);
			prios[pos + r] = slot_prio(sl);
		}
		pos += tot;
	}
}

// ---------------------------------------------------------------- host side

uint64_t buckets_for(uint64_t n)
{
	uint64_t want = (uint64_t)((double)n / (kBucketSlots * kTargetLoad)) + 1;
	uint64_t b = 2;
	while (b < want)
		b <<= 1;
	return b;
}

int set_alloc(syzsig_ctx* ctx, uint64_t nbuckets, syzsig_set** out)
{
	if (nbuckets * kBucketSlots > (1ull << 32))
		return fail(SYZSIG_ERANGE, "signal table above 2^32 slots");
	syzsig_set* s = new syzsig_set();
	s->ctx = ctx;
	s->nbuckets = nbuckets;
	hipError_t e = hipMallocAsync((void**)&s->slots, nbuckets * kBucketSlots * sizeof(uint64_t), ctx->stream);
	if (e == hipSuccess)
		e = hipMemsetAsync(s->slots, 0, nbuckets * kBucketSlots * sizeof(uint64_t), ctx->stream);
	if (e != hipSuccess) {
		delete s;
		return hip_fail(e, "set_alloc", __FILE__, __LINE__);
	}
	*out = s;
	return SYZSIG_OK;
}

static void set_release_storage(syzsig_set* s)
{
	hipStream_t st = s->ctx->stream;
	if (s->slots)
		(void)hipFreeAsync(s->slots, st);
	if (s->firsts)
		(void)hipFreeAsync(s->firsts, st);
	if (s->touched)
		(void)hipFreeAsync(s->touched, st);
	s->slots = nullptr;
	s->firsts = nullptr;
	s->touched = nullptr;
}

int set_rehash(syzsig_set* s, uint64_t nbuckets, bool drop_absent)
{
	syzsig_ctx* ctx = s->ctx;
	syzsig_set* n = nullptr;
	SYZ_TRY(set_alloc(ctx, nbuckets, &n));
	SYZ_TRY(counters_reset(ctx));
	k_rehash<<<grid_for(s->nslots(), 256), 256, 0, ctx->stream>>>(s->slots, s->nslots(), n->slots,
	                                                               nbuckets - 1, drop_absent, ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->h_cnt[kCntOverflow])
		return fail(SYZSIG_EIO, "rehash overflow (internal error)");
	bool had_triage = s->firsts != nullptr;
	set_release_storage(s);
	s->slots = n->slots;
	s->nbuckets = nbuckets;
	s->len = ctx->h_cnt[kCntInserted];
	n->slots = nullptr;
	delete n;
	if (had_triage)
		SYZ_TRY(set_ensure_triage_state(s));
	return SYZSIG_OK;
}

int set_reserve(syzsig_set* s, uint64_t extra)
{
	return set_reserve_load(s, extra, kMaxLoad);
}

int set_reserve_load(syzsig_set* s, uint64_t extra, double load)
{
	uint64_t need = s->len + extra;
	if ((double)need <= load * (double)s->nslots())
		return SYZSIG_OK;
	return set_rehash(s, buckets_for(need), false);
}

int set_ensure_triage_state(syzsig_set* s)
{
	if (s->firsts)
		return SYZSIG_OK;
	hipStream_t st = s->ctx->stream;
	SYZ_HIP(hipMallocAsync((void**)&s->firsts, s->nslots() * 4 * sizeof(uint32_t), st));
	SYZ_HIP(hipMemsetAsync(s->firsts, 0xff, s->nslots() * 4 * sizeof(uint32_t), st));
	SYZ_HIP(hipMallocAsync((void**)&s->touched, (s->nslots() / 32 + 1) * sizeof(uint32_t), st));
	s->epoch = 254;
	return SYZSIG_OK;
}

int merge_pairs_dev(syzsig_ctx* ctx, syzsig_set* dst, const uint64_t* d_pairs, uint64_t n)
{
	if (n == 0)
		return SYZSIG_OK;
	SYZ_TRY(set_reserve(dst, n));
	SYZ_TRY(counters_reset(ctx));
	k_merge_pairs<<<grid_for(n, 256), 256, 0, ctx->stream>>>(dst->slots, dst->nbuckets - 1, d_pairs, n, ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->h_cnt[kCntOverflow])
		return fail(SYZSIG_EIO, "merge overflow (internal error)");
	dst->len += ctx->h_cnt[kCntInserted];
	return SYZSIG_OK;
}

// Result-producing op helper: allocate a result sized for `bound` entries,
// run `launch`, and return NULL instead of an empty result when nil_if_empty.
template <typename F>
static int make_result(syzsig_ctx* ctx, uint64_t bound, bool nil_if_empty, syzsig_set** out, F launch)
{
	*out = nullptr;
	syzsig_set* r = nullptr;
	SYZ_TRY(set_alloc(ctx, buckets_for(bound), &r));
	int rc = counters_reset(ctx);
	if (rc == SYZSIG_OK) {
		launch(r);
		hipError_t e = hipGetLastError();
		rc = e == hipSuccess ? counters_fetch(ctx) : hip_fail(e, "kernel launch", __FILE__, __LINE__);
	}
	if (rc == SYZSIG_OK && ctx->h_cnt[kCntOverflow])
		rc = fail(SYZSIG_EIO, "result table overflow (internal error)");
	if (rc != SYZSIG_OK) {
		syzsig_set_free(r);
		return rc;
	}
	r->len = ctx->h_cnt[kCntInserted];
	if (nil_if_empty && r->len == 0) {
		syzsig_set_free(r);
		return SYZSIG_OK;
	}
	*out = r;
	return SYZSIG_OK;
}

static int upload(syzsig_ctx* ctx, int ws, const void* host, size_t bytes, void** dev)
{
	SYZ_TRY(ws_get(ctx, ws, bytes, dev));
	if (bytes)
		SYZ_HIP(hipMemcpyAsync(*dev, host, bytes, hipMemcpyHostToDevice, ctx->stream));
	return SYZSIG_OK;
}

}  // namespace syz

using namespace syz;

extern "C" {

int syzsig_set_make(syzsig_ctx* ctx, uint64_t hint, syzsig_set** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out)
		return fail(SYZSIG_EINVAL, "set_make: NULL argument");
	return set_alloc(ctx, buckets_for(hint), out);
}

void syzsig_set_free(syzsig_set* s)
{
	SYZ_LOCK(s ? s->ctx : nullptr);
	if (!s)
		return;
	if (s->step_busy && s->ctx) {  // freed under an owner step: the step forgets its sets
		syzsig_ctx* c = s->ctx;
		if (c->step_ms)
			c->step_ms->step_busy = false;
		if (c->step_ns)
			c->step_ns->step_busy = false;
		c->step_ms = c->step_ns = nullptr;
	}
	set_release_storage(s);
	delete s;
}

int syzsig_set_clone(syzsig_ctx* ctx, const syzsig_set* s, syzsig_set** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out)
		return fail(SYZSIG_EINVAL, "set_clone: NULL argument");
	SYZ_TRY(set_check_idle(s));
	*out = nullptr;
	if (!s)
		return SYZSIG_OK;
	syzsig_set* n = nullptr;
	SYZ_TRY(set_alloc(ctx, s->nbuckets, &n));
	SYZ_HIP(hipMemcpyAsync(n->slots, s->slots, s->nslots() * sizeof(uint64_t), hipMemcpyDeviceToDevice, ctx->stream));
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	n->len = s->len;
	*out = n;
	return SYZSIG_OK;
}

// Whole-table copy (the benchmark's maxSignal reset to M0, 268 MB at C2): one
// 16-B element per lane over a grid that covers the table, nontemporal -- the
// form of runtime.hip's k_copy16 that measured 6.2-6.6 TB/s on 1 GiB
// (DESIGN.md 7), against ~4.4 TB/s for the runtime's device copy.
#ifndef SYZ_TBL_COPY_KERNEL
#define SYZ_TBL_COPY_KERNEL 1
#endif
typedef uint32_t tbl_v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_tbl_copy16(const tbl_v4u* __restrict__ src, tbl_v4u* __restrict__ dst,
                                                    uint64_t n)
{
	const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride)
		__builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}

// Whole-table clear as 16-B stores, four per thread (the runtime's fill kernel
// reaches ~2 TB/s on a 64 MB table, this one ~2.7).
// Tables are a whole number of 16-B buckets and hipMalloc'd (256-B aligned).
__global__ __launch_bounds__(256) void k_tbl_fill0(uint4* __restrict__ d, uint64_t n)
{
	const uint64_t T = (uint64_t)gridDim.x * blockDim.x;
	const uint4 z = make_uint4(0, 0, 0, 0);
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += 4 * T) {
#pragma unroll
		for (uint32_t k = 0; k < 4; k++)
			if (i + k * T < n)
				d[i + k * T] = z;
	}
}

static uint32_t stream_grid(uint64_t n16)
{
	return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n16 + 1023) / 1024, 8192));
}

int syzsig_set_clear(syzsig_ctx* ctx, syzsig_set* s)
{
	SYZ_LOCK(ctx);
	if (!ctx || !s)
		return fail(SYZSIG_EINVAL, "set_clear: NULL argument");
	SYZ_TRY(set_check_idle(s));
	const uint64_t n16 = s->nslots() / 2;
	k_tbl_fill0<<<stream_grid(n16), 256, 0, ctx->stream>>>((uint4*)s->slots, n16);
	SYZ_HIP(hipGetLastError());
	s->len = 0;
	return SYZSIG_OK;
}

int syzsig_set_copy_from(syzsig_ctx* ctx, syzsig_set* dst, const syzsig_set* src)
{
	SYZ_LOCK(ctx);
	if (!ctx || !dst || !src)
		return fail(SYZSIG_EINVAL, "set_copy_from: NULL argument");
	SYZ_TRY(set_check_idle(dst));
	SYZ_TRY(set_check_idle(src));
	if (dst->nbuckets != src->nbuckets)
		return fail(SYZSIG_EINVAL, "set_copy_from: capacity mismatch");
	const uint64_t n16 = src->nslots() * sizeof(uint64_t) / 16;  // (tables are whole 16-B buckets)
	if (SYZ_TBL_COPY_KERNEL && n16) {
		const uint32_t grid = (uint32_t)std::min<uint64_t>((n16 + 255) / 256, 1u << 22);
		k_tbl_copy16<<<grid, 256, 0, ctx->stream>>>((const tbl_v4u*)src->slots, (tbl_v4u*)dst->slots, n16);
		SYZ_HIP(hipGetLastError());
	} else {
		SYZ_HIP(hipMemcpyAsync(dst->slots, src->slots, src->nslots() * sizeof(uint64_t), hipMemcpyDeviceToDevice,
		                       ctx->stream));  // (the runtime's copy: ~4.4 TB/s; a 4 x 16-B-per-thread kernel ran 3.8)
	}
	dst->len = src->len;
	return SYZSIG_OK;
}

int syzsig_set_restore_keys(syzsig_ctx* ctx, syzsig_set* dst, const syzsig_set* src, const syzsig_set* keys)
{
	SYZ_LOCK(ctx);
	if (!ctx || !dst || !src)
		return fail(SYZSIG_EINVAL, "set_restore_keys: NULL argument");
	SYZ_TRY(set_check_idle(dst));
	SYZ_TRY(set_check_idle(src));
	SYZ_TRY(set_check_idle(keys));
	if (dst->nbuckets != src->nbuckets)
		return fail(SYZSIG_EINVAL, "set_restore_keys: capacity mismatch (dst grew since the snapshot)");
	if (keys && keys->len) {
		void* ib;
		SYZ_TRY(ws_get(ctx, 11, keys->nslots() * 8 + 64, &ib));
		const int g = grid_for(keys->nslots(), 256, 8192);
		k_restore_find<<<g, 256, 0, ctx->stream>>>(dst->slots, dst->nbuckets - 1, keys->slots, keys->nslots(),
		                                           (int64_t*)ib);
		k_restore_apply<<<g, 256, 0, ctx->stream>>>(dst->slots, src->slots, (const int64_t*)ib, keys->nslots());
		SYZ_HIP(hipGetLastError());
	}
	dst->len = src->len;
	return SYZSIG_OK;
}

int syzsig_set_reserve(syzsig_ctx* ctx, syzsig_set* s, uint64_t extra)
{
	SYZ_LOCK(ctx);
	if (!ctx || !s)
		return fail(SYZSIG_EINVAL, "set_reserve: NULL argument");
	SYZ_TRY(set_check_idle(s));
	return set_reserve(s, extra);
}

int syzsig_set_equal(syzsig_ctx* ctx, const syzsig_set* a, const syzsig_set* b, int* equal)
{
	SYZ_LOCK(ctx);
	if (!ctx || !a || !b || !equal)
		return fail(SYZSIG_EINVAL, "set_equal: NULL argument");
	SYZ_TRY(set_check_idle(a));
	SYZ_TRY(set_check_idle(b));
	*equal = 0;
	if (a->nbuckets != b->nbuckets || a->len != b->len)
		return SYZSIG_OK;
	SYZ_TRY(counters_reset(ctx));
	k_slots_differ<<<grid_for(a->nslots(), 256, 8192), 256, 0, ctx->stream>>>(a->slots, b->slots, a->nslots(),
	                                                                        &ctx->d_cnt[kCntAux]);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	*equal = ctx->h_cnt[kCntAux] == 0;
	return SYZSIG_OK;
}

uint64_t syzsig_len(const syzsig_set* s)
{
	SYZ_LOCK(s ? s->ctx : nullptr);
	return s ? s->len : 0;
}

int syzsig_empty(const syzsig_set* s) { return syzsig_len(s) == 0; }

uint64_t syzsig_capacity(const syzsig_set* s)
{
	SYZ_LOCK(s ? s->ctx : nullptr);
	return s ? s->nslots() : 0;
}

int syzsig_from_raw(syzsig_ctx* ctx, const uint32_t* raw, uint64_t n, uint8_t prio, syzsig_set** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out || (n && !raw))
		return fail(SYZSIG_EINVAL, "from_raw: NULL argument");
	*out = nullptr;
	if (n == 0)
		return SYZSIG_OK;  // signal.go:32-34
	void* d = nullptr;
	SYZ_TRY(upload(ctx, 0, raw, n * 4, &d));
	return make_result(ctx, n, false, out, [&](syzsig_set* r) {
		k_from_raw<<<grid_for(n, 256), 256, 0, ctx->stream>>>(r->slots, r->nbuckets - 1, (const uint32_t*)d, n,
		                                                       (int8_t)prio, ctx->d_cnt);
	});
}

int syzsig_serialize(syzsig_ctx* ctx, const syzsig_set* s, uint32_t* elems, int8_t* prios, uint64_t cap,
                     uint64_t* n_out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !n_out || (cap && (!elems || !prios)))
		return fail(SYZSIG_EINVAL, "serialize: NULL argument");
	SYZ_TRY(set_check_idle(s));
	*n_out = 0;
	if (!s || s->len == 0)
		return SYZSIG_OK;  // signal.go:43-45
	uint64_t nslots = s->nslots();
	int nblk = grid_for(nslots, 256);
	uint64_t chunk = (nslots + nblk - 1) / nblk;
	uint64_t m = std::min<uint64_t>(cap, s->len);
	void *d_counts, *d_out;
	SYZ_TRY(ws_get(ctx, 1, (nblk + 1) * sizeof(unsigned long long), &d_counts));
	SYZ_TRY(ws_get(ctx, 2, m * 5 + 16, &d_out));
	unsigned long long* counts = (unsigned long long*)d_counts;
	k_count_live<<<nblk, 256, 0, ctx->stream>>>(s->slots, nslots, chunk, counts);
	k_scan_counts<<<1, 1024, 0, ctx->stream>>>(counts, nblk, counts + nblk);
	uint32_t* de = (uint32_t*)d_out;
	int8_t* dp = (int8_t*)(de + m);
	k_write_live<<<nblk, 256, 0, ctx->stream>>>(s->slots, nslots, chunk, counts, de, dp, m);
	SYZ_HIP(hipGetLastError());
	if (m) {
		SYZ_HIP(hipMemcpyAsync(elems, de, m * 4, hipMemcpyDeviceToHost, ctx->stream));
		SYZ_HIP(hipMemcpyAsync(prios, dp, m, hipMemcpyDeviceToHost, ctx->stream));
	}
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	*n_out = s->len;
	return SYZSIG_OK;
}

int syzsig_serialize_batch(syzsig_ctx* ctx, const syzsig_set* const* sets, uint64_t nsets, uint32_t* elems,
                           int8_t* prios, uint64_t cap, uint64_t* offs)
{
	SYZ_LOCK(ctx);
	if (!ctx || !offs || (nsets && !sets))
		return fail(SYZSIG_EINVAL, "serialize_batch: NULL argument");
	offs[0] = 0;
	for (uint64_t i = 0; i < nsets; i++) {
		SYZ_TRY(set_check_idle(sets[i]));
		offs[i + 1] = offs[i] + (sets[i] ? sets[i]->len : 0);
	}
	const uint64_t total = offs[nsets];
	if (cap == 0 || total == 0)
		return SYZSIG_OK;  // the offsets only (sizing), or nothing to write
	if (!elems || !prios)
		return fail(SYZSIG_EINVAL, "serialize_batch: NULL output");
	if (cap < total)
		return fail(SYZSIG_ERANGE, "serialize_batch: cap below the sets' total Len (offs holds it)");
	std::vector<SerDesc> desc;
	std::vector<uint32_t> blk_set;
	for (uint64_t i = 0; i < nsets; i++) {
		const syzsig_set* st = sets[i];
		if (!st || st->len == 0)
			continue;
		const uint64_t nslots = st->nslots();
		const uint32_t nblk = (uint32_t)grid_for(nslots, 256);
		desc.push_back(SerDesc{st->slots, nslots, (nslots + nblk - 1) / nblk, (uint32_t)blk_set.size(), 0});
		blk_set.insert(blk_set.end(), nblk, (uint32_t)(desc.size() - 1));
	}
	const uint64_t nb = blk_set.size();
	if (nb >= (1u << 31))
		return fail(SYZSIG_ERANGE, "serialize_batch: too many sets");
	void *d_desc, *d_blk, *d_counts, *d_out;
	SYZ_TRY(ws_get(ctx, 0, desc.size() * sizeof(SerDesc), &d_desc));
	SYZ_TRY(ws_get(ctx, 1, (nb + 1) * sizeof(unsigned long long), &d_counts));
	SYZ_TRY(ws_get(ctx, 2, total * 5 + 16, &d_out));
	SYZ_TRY(ws_get(ctx, 3, nb * sizeof(uint32_t), &d_blk));
	SYZ_HIP(hipMemcpyAsync(d_desc, desc.data(), desc.size() * sizeof(SerDesc), hipMemcpyHostToDevice, ctx->stream));
	SYZ_HIP(hipMemcpyAsync(d_blk, blk_set.data(), nb * sizeof(uint32_t), hipMemcpyHostToDevice, ctx->stream));
	unsigned long long* counts = (unsigned long long*)d_counts;
	k_count_live_multi<<<(uint32_t)nb, 256, 0, ctx->stream>>>((const SerDesc*)d_desc, (const uint32_t*)d_blk, counts);
	k_scan_counts<<<1, 1024, 0, ctx->stream>>>(counts, (uint32_t)nb, counts + nb);
	uint32_t* de = (uint32_t*)d_out;
	int8_t* dp = (int8_t*)(de + total);
	k_write_live_multi<<<(uint32_t)nb, 256, 0, ctx->stream>>>((const SerDesc*)d_desc, (const uint32_t*)d_blk, counts,
	                                                        de, dp);
	SYZ_HIP(hipGetLastError());
	SYZ_HIP(hipMemcpyAsync(elems, de, total * 4, hipMemcpyDeviceToHost, ctx->stream));
	SYZ_HIP(hipMemcpyAsync(prios, dp, total, hipMemcpyDeviceToHost, ctx->stream));
	SYZ_HIP(hipStreamSynchronize(ctx->stream));  // (the host vectors above outlive the copies)
	return SYZSIG_OK;
}

int syzsig_deserialize_dev(syzsig_ctx* ctx, const uint32_t* d_elems, const int8_t* d_prios, uint64_t n,
                           syzsig_set** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out || (n && (!d_elems || !d_prios)))
		return fail(SYZSIG_EINVAL, "deserialize: NULL argument");
	*out = nullptr;
	if (n == 0)
		return SYZSIG_OK;  // signal.go:63-65
	if (n >= 0x80000000ull)
		return fail(SYZSIG_ERANGE, "deserialize: more than 2^31 elements");
	return make_result(ctx, n, false, out, [&](syzsig_set* r) {
		k_deser_index<<<grid_for(n, 256), 256, 0, ctx->stream>>>(r->slots, r->nbuckets - 1, d_elems, n, ctx->d_cnt);
		k_deser_prio<<<grid_for(r->nslots(), 256), 256, 0, ctx->stream>>>(r->slots, r->nslots(), d_prios);
	});
}

int syzsig_deserialize(syzsig_ctx* ctx, const uint32_t* elems, uint64_t n_elems, const int8_t* prios,
                       uint64_t n_prios, syzsig_set** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out)
		return fail(SYZSIG_EINVAL, "deserialize: NULL argument");
	*out = nullptr;
	if (n_elems != n_prios)
		return fail(SYZSIG_ECORRUPT, "corrupted Serial");  // signal.go:60-62
	if (n_elems == 0)
		return SYZSIG_OK;
	if (!elems || !prios)
		return fail(SYZSIG_EINVAL, "deserialize: NULL argument");
	void *de, *dp;
	SYZ_TRY(upload(ctx, 0, elems, n_elems * 4, &de));
	SYZ_TRY(upload(ctx, 1, prios, n_elems, &dp));
	return syzsig_deserialize_dev(ctx, (const uint32_t*)de, (const int8_t*)dp, n_elems, out);
}

int syzsig_diff(syzsig_ctx* ctx, const syzsig_set* s, const syzsig_set* s1, syzsig_set** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out)
		return fail(SYZSIG_EINVAL, "diff: NULL argument");
	SYZ_TRY(set_check_idle(s));
	SYZ_TRY(set_check_idle(s1));
	*out = nullptr;
	if (syzsig_empty(s1))
		return SYZSIG_OK;  // signal.go:74-76
	bool have = s && s->len;
	return make_result(ctx, s1->len, true, out, [&](syzsig_set* r) {
		k_diff<<<grid_for(s1->nslots(), 256), 256, 0, ctx->stream>>>(
		    have ? s->slots : nullptr, have ? s->nbuckets - 1 : 0, have, s1->slots, s1->nslots(), r->slots,
		    r->nbuckets - 1, ctx->d_cnt);
	});
}

int syzsig_diff_raw(syzsig_ctx* ctx, const syzsig_set* s, const uint32_t* raw, uint64_t n, uint8_t prio,
                    syzsig_set** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out || (n && !raw))
		return fail(SYZSIG_EINVAL, "diff_raw: NULL argument");
	SYZ_TRY(set_check_idle(s));
	*out = nullptr;
	if (n == 0)
		return SYZSIG_OK;
	void* d = nullptr;
	SYZ_TRY(upload(ctx, 0, raw, n * 4, &d));
	bool have = s && s->len;
	return make_result(ctx, n, true, out, [&](syzsig_set* r) {
		k_diff_raw<<<grid_for(n, 256), 256, 0, ctx->stream>>>(have ? s->slots : nullptr, have ? s->nbuckets - 1 : 0,
		                                                       have, (const uint32_t*)d, n, (int8_t)prio, r->slots,
		                                                       r->nbuckets - 1, ctx->d_cnt);
	});
}

int syzsig_intersection(syzsig_ctx* ctx, const syzsig_set* s, const syzsig_set* s1, syzsig_set** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out)
		return fail(SYZSIG_EINVAL, "intersection: NULL argument");
	SYZ_TRY(set_check_idle(s));
	SYZ_TRY(set_check_idle(s1));
	*out = nullptr;
	if (syzsig_empty(s1))
		return SYZSIG_OK;  // signal.go:105-107
	uint64_t bound = syzsig_len(s);
	return make_result(ctx, bound, false, out, [&](syzsig_set* r) {
		if (bound)
			k_intersection<<<grid_for(s->nslots(), 256), 256, 0, ctx->stream>>>(
			    s->slots, s->nslots(), s1->slots, s1->nbuckets - 1, r->slots, r->nbuckets - 1, ctx->d_cnt);
	});
}

// pkg/cover/cover.go:9-18 Cover.Merge(raw): the receiver is allocated when nil
// (even for an empty raw), then every PC is inserted; a Cover's entries all
// carry prio 0 (map[uint32]struct{}: the value is unused).
static int cover_merge_dev(syzsig_ctx* ctx, syzsig_set** cov, const uint32_t* d_raw, uint64_t n)
{
	if (!*cov)
		SYZ_TRY(syzsig_set_make(ctx, n, cov));
	if (n == 0)
		return SYZSIG_OK;
	syzsig_set* s = *cov;
	SYZ_TRY(set_reserve(s, n));
	SYZ_TRY(counters_reset(ctx));
	k_from_raw<<<grid_for(n, 256), 256, 0, ctx->stream>>>(s->slots, s->nbuckets - 1, d_raw, n, 0, ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->h_cnt[kCntOverflow])
		return fail(SYZSIG_EIO, "cover merge overflow (internal error)");
	s->len += ctx->h_cnt[kCntInserted];
	return SYZSIG_OK;
}

int syzsig_cover_merge(syzsig_ctx* ctx, syzsig_set** cov, const uint32_t* raw, uint64_t n)
{
	SYZ_LOCK(ctx);
	if (!ctx || !cov || (n && !raw))
		return fail(SYZSIG_EINVAL, "cover_merge: NULL argument");
	void* d = nullptr;
	SYZ_TRY(upload(ctx, 0, raw, n * 4, &d));
	return cover_merge_dev(ctx, cov, (const uint32_t*)d, n);
}

int syzsig_cover_merge_dev(syzsig_ctx* ctx, syzsig_set** cov, const uint32_t* d_raw, uint64_t n)
{
	SYZ_LOCK(ctx);
	if (!ctx || !cov || (n && !d_raw))
		return fail(SYZSIG_EINVAL, "cover_merge_dev: NULL argument");
	return cover_merge_dev(ctx, cov, d_raw, n);
}

int syzsig_merge(syzsig_ctx* ctx, syzsig_set** sp, const syzsig_set* s1)
{
	SYZ_LOCK(ctx);
	if (!ctx || !sp)
		return fail(SYZSIG_EINVAL, "merge: NULL argument");
	SYZ_TRY(set_check_idle(*sp));
	SYZ_TRY(set_check_idle(s1));
	if (syzsig_empty(s1))
		return SYZSIG_OK;  // signal.go:118-120
	if (!*sp)
		SYZ_TRY(syzsig_set_make(ctx, s1->len, sp));  // signal.go:121-125
	syzsig_set* s = *sp;
	SYZ_TRY(set_reserve(s, s1->len));
	SYZ_TRY(counters_reset(ctx));
	k_merge<<<grid_for(s1->nslots(), 256), 256, 0, ctx->stream>>>(s->slots, s->nbuckets - 1, s1->slots, s1->nslots(),
	                                                               ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->h_cnt[kCntOverflow])
		return fail(SYZSIG_EIO, "merge overflow (internal error)");
	s->len += ctx->h_cnt[kCntInserted];
	return SYZSIG_OK;
}

}  // extern "C"
