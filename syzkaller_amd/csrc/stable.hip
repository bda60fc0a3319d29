// stable.hip -- triageInput's signal re-runs over a batch of triage items.
//
// Reference: syz-fuzzer/proc.go:107-140 triageInput.  For one item (a call
// whose execution had new signal), newSignal = corpusSignalDiff(inputSignal)
// is re-checked against signalRuns re-executions:
//
//   notexecuted = 0
//   for each run r (in order):
//     if the call was not executed, has no signal, or failed although the
//        original succeeded (proc.go:122-128):  notexecuted++;
//        if notexecuted > signalRuns/2 + 1: give up (item dropped); continue
//     newSignal = newSignal.Intersection(FromRaw(run signal, run prio))
//     if newSignal.Empty() && !minimized: item dropped             (:133-137)
//
// Intersection (pkg/signal/signal.go:104-115) keeps e of newSignal iff the run
// has e with prio_r >= prio_e (int8), so an element's fate is a bitmask over
// the runs, and the control flow of an item only needs, after each run, how
// many of its elements are still alive.  Kernels:
//   k_runs_insert     every (run, elem) of the re-runs into one hash set
//   k_stable_elems    one thread per newSignal element: present-bits per run,
//                     alive-after-run counts per item (atomics)
//   k_stable_items    one thread per item: the sequential control above
//   k_stable_final    each element's membership in the item's final newSignal
// The same set answers the minimize predicate (proc.go:141-160):
// newSignal.Intersection(thisSignal).Len() == newSignal.Len().
#include <algorithm>

#include "internal.h"

namespace syz {

constexpr uint32_t kStableMaxRuns = 8;
constexpr uint64_t kRunKeyEmpty = ~0ull;

__device__ __forceinline__ uint64_t run_key_hash(uint64_t k)
{
	k ^= k >> 33;
	k *= 0xff51afd7ed558ccdull;
	k ^= k >> 33;
	k *= 0xc4ceb9fe1a85ec53ull;
	k ^= k >> 33;
	return k;
}

// run r of the batch owns sigs[run_off[r] .. run_off[r+1]); key = r << 32 | elem
__global__ void k_runs_insert(const uint64_t* __restrict__ run_off, uint64_t nruns, const uint32_t* __restrict__ sigs,
                              uint64_t* set, uint64_t C)
{
	for (uint64_t r = blockIdx.x; r < nruns; r += gridDim.x) {
		const uint64_t a = run_off[r], b = run_off[r + 1];
		for (uint64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
			const uint64_t key = (r << 32) | sigs[i];
			uint64_t h = run_key_hash(key) & (C - 1);
			for (;;) {  // C >= 2 * keys: an empty slot always exists
				uint64_t k = set[h];
				if (k == kRunKeyEmpty) {
					k = atomicCAS((unsigned long long*)&set[h], kRunKeyEmpty, (unsigned long long)key);
					if (k == kRunKeyEmpty || k == key)
						break;
				} else if (k == key) {
					break;
				}
				h = (h + 1) & (C - 1);
			}
		}
	}
}

__device__ __forceinline__ bool runs_has(const uint64_t* __restrict__ set, uint64_t C, uint64_t key)
{
	uint64_t h = run_key_hash(key) & (C - 1);
	for (;;) {
		const uint64_t k = set[h];
		if (k == key)
			return true;
		if (k == kRunKeyEmpty)
			return false;
		h = (h + 1) & (C - 1);
	}
}

// run r is usable (proc.go:122-128): executed, non-empty signal, and not
// failed when the original call succeeded
__device__ __forceinline__ bool run_ok(const uint64_t* run_off, const uint8_t* run_exec, const int32_t* run_errno,
                                       uint8_t item_flags, uint64_t r)
{
	const bool orig_ok = item_flags & SYZSIG_TRIAGE_ORIG_OK;
	return run_exec[r] && run_off[r + 1] > run_off[r] && !(orig_ok && run_errno[r] != 0);
}

__global__ void k_stable_elems(const uint64_t* __restrict__ item_off, uint64_t nitems,
                               const uint32_t* __restrict__ elems, const int8_t* __restrict__ prios, uint32_t R,
                               const uint64_t* __restrict__ run_off, const uint8_t* __restrict__ run_exec,
                               const int32_t* __restrict__ run_errno, const uint8_t* __restrict__ run_prio,
                               const uint8_t* __restrict__ item_flags, const uint64_t* __restrict__ set, uint64_t C,
                               uint8_t* __restrict__ alive, unsigned long long* __restrict__ alive_cnt, bool chain)
{
	for (uint64_t it = blockIdx.x; it < nitems; it += gridDim.x) {
		const uint64_t a = item_off[it], b = item_off[it + 1];
		for (uint64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
			const uint32_t e = elems[i];
			const int pe = prios[i];
			uint32_t m = 0, live = 1;
			for (uint32_t r = 0; r < R; r++) {
				const uint64_t rr = it * R + r;
				if (!run_ok(run_off, run_exec, run_errno, item_flags[it], rr)) {
					m |= live << r;  // a skipped run changes nothing
					continue;
				}
				const uint32_t here = (int)(int8_t)run_prio[rr] >= pe && runs_has(set, C, (rr << 32) | e);
				live = chain ? live & here : here;  // chained Intersections, or each run on its own
				m |= live << r;
				if (live)
					atomicAdd(&alive_cnt[rr], 1ull);
			}
			alive[i] = (uint8_t)m;
		}
	}
}

__global__ void k_stable_items(const uint64_t* __restrict__ item_off, uint64_t nitems, uint32_t R,
                               const uint64_t* __restrict__ run_off, const uint8_t* __restrict__ run_exec,
                               const int32_t* __restrict__ run_errno, const uint8_t* __restrict__ item_flags,
                               const unsigned long long* __restrict__ alive_cnt, uint8_t* __restrict__ item_keep,
                               int8_t* __restrict__ item_stop)
{
	const uint64_t it = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (it >= nitems)
		return;
	const bool minimized = item_flags[it] & SYZSIG_TRIAGE_MINIMIZED;
	uint32_t notexec = 0;
	int stop = -1;
	bool keep = item_off[it + 1] > item_off[it];  // proc.go:109-111: nothing new, nothing to triage
	for (uint32_t r = 0; r < R && keep; r++) {
		const uint64_t rr = it * R + r;
		if (!run_ok(run_off, run_exec, run_errno, item_flags[it], rr)) {
			if (++notexec > R / 2 + 1)
				keep = false;  // proc.go:125-127
			continue;
		}
		stop = (int)r;
		if (alive_cnt[rr] == 0 && !minimized)
			keep = false;  // proc.go:133-137
	}
	item_keep[it] = keep;
	item_stop[it] = (int8_t)stop;
}

__global__ void k_stable_final(const uint64_t* __restrict__ item_off, uint64_t nitems,
                               const uint8_t* __restrict__ item_keep, const int8_t* __restrict__ item_stop,
                               const uint8_t* __restrict__ alive, uint8_t* __restrict__ keep_elem)
{
	for (uint64_t it = blockIdx.x; it < nitems; it += gridDim.x) {
		const uint64_t a = item_off[it], b = item_off[it + 1];
		const int stop = item_stop[it];
		const bool k = item_keep[it];
		for (uint64_t i = a + threadIdx.x; i < b; i += blockDim.x)
			keep_elem[i] = k && (stop < 0 || ((alive[i] >> stop) & 1));
	}
}

// The minimize predicate (proc.go:141-160) per item: attempts in order; one
// that did not execute or has no signal is skipped; a failure after a
// successful original is a "no"; a run whose Intersection with newSignal keeps
// all of it is a "yes"; running out of attempts is a "no".
__global__ void k_pred_items(const uint64_t* __restrict__ item_off, uint64_t nitems, uint32_t R,
                             const uint64_t* __restrict__ run_off, const uint8_t* __restrict__ run_exec,
                             const int32_t* __restrict__ run_errno, const uint8_t* __restrict__ item_flags,
                             const unsigned long long* __restrict__ alive_cnt, uint8_t* __restrict__ pred)
{
	const uint64_t it = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (it >= nitems)
		return;
	const bool orig_ok = item_flags[it] & SYZSIG_TRIAGE_ORIG_OK;
	const uint64_t len = item_off[it + 1] - item_off[it];
	uint8_t res = 0;
	for (uint32_t r = 0; r < R; r++) {
		const uint64_t rr = it * R + r;
		if (!run_exec[rr] || run_off[rr + 1] == run_off[rr])
			continue;  // proc.go:146-148
		if (orig_ok && run_errno[rr] != 0)
			break;  // proc.go:150-154
		if (alive_cnt[rr] == len) {
			res = 1;  // proc.go:157-159
			break;
		}
	}
	pred[it] = res;
}

static uint64_t pow2_ge(uint64_t v)
{
	uint64_t c = 1;
	while (c < v)
		c <<= 1;
	return c;
}

}  // namespace syz

using namespace syz;

extern "C" int syzsig_triage_runs_dev(syzsig_ctx* ctx, const uint64_t* d_item_off, uint64_t nitems,
                                      const uint32_t* d_elems, const int8_t* d_prios, const uint8_t* d_item_flags,
                                      uint32_t runs, const uint64_t* d_run_off, const uint32_t* d_run_sigs,
                                      const uint8_t* d_run_prio, const int32_t* d_run_errno,
                                      const uint8_t* d_run_exec, uint8_t* d_item_keep, uint8_t* d_elem_keep)
{
	SYZ_LOCK(ctx);
	if (!ctx || (nitems && (!d_item_off || !d_item_flags || !d_item_keep)) ||
	    (nitems && runs && (!d_run_off || !d_run_prio || !d_run_errno || !d_run_exec)))
		return fail(SYZSIG_EINVAL, "triage_runs: NULL argument");
	if (runs > kStableMaxRuns)
		return fail(SYZSIG_ERANGE, "triage_runs: at most 8 runs per item");
	if (nitems == 0)
		return SYZSIG_OK;
	const hipStream_t s = ctx->stream;
	const uint64_t nruns = nitems * runs;
	uint64_t h_off[2] = {0, 0}, h_roff = 0;
	SYZ_HIP(hipMemcpyAsync(&h_off[1], d_item_off + nitems, 8, hipMemcpyDeviceToHost, s));
	if (nruns)
		SYZ_HIP(hipMemcpyAsync(&h_roff, d_run_off + nruns, 8, hipMemcpyDeviceToHost, s));
	SYZ_HIP(hipStreamSynchronize(s));
	const uint64_t nelem = h_off[1], nsig = h_roff;
	if ((nelem && (!d_elems || !d_prios || !d_elem_keep)) || (nsig && !d_run_sigs))
		return fail(SYZSIG_EINVAL, "triage_runs: NULL argument");
	if (nruns >= (1ull << 32))
		return fail(SYZSIG_ERANGE, "triage_runs: too many runs");
	const uint64_t C = pow2_ge(std::max<uint64_t>(2 * nsig + 16, 64));
	void *set, *alive, *cnt, *stop;
	SYZ_TRY(ws_get(ctx, 0, C * 8, &set));
	SYZ_TRY(ws_get(ctx, 1, nelem + 64, &alive));
	SYZ_TRY(ws_get(ctx, 2, nruns * 8 + 64, &cnt));
	SYZ_TRY(ws_get(ctx, 3, nitems + 64, &stop));
	SYZ_HIP(hipMemsetAsync(set, 0xff, C * 8, s));
	SYZ_HIP(hipMemsetAsync(cnt, 0, nruns * 8 + 8, s));
	if (nsig)
		k_runs_insert<<<(int)std::min<uint64_t>(nruns, 8192), 256, 0, s>>>(d_run_off, nruns, d_run_sigs, (uint64_t*)set, C);
	k_stable_elems<<<(int)std::min<uint64_t>(nitems, 8192), 256, 0, s>>>(
		d_item_off, nitems, d_elems, d_prios, runs, d_run_off, d_run_exec, d_run_errno, d_run_prio, d_item_flags,
		(const uint64_t*)set, C, (uint8_t*)alive, (unsigned long long*)cnt, true);
	k_stable_items<<<(int)((nitems + 255) / 256), 256, 0, s>>>(
		d_item_off, nitems, runs, d_run_off, d_run_exec, d_run_errno, d_item_flags,
		(const unsigned long long*)cnt, d_item_keep, (int8_t*)stop);
	if (nelem)
		k_stable_final<<<(int)std::min<uint64_t>(nitems, 8192), 256, 0, s>>>(d_item_off, nitems, d_item_keep,
		                                                           (const int8_t*)stop, (const uint8_t*)alive,
		                                                           d_elem_keep);
	SYZ_HIP(hipGetLastError());
	SYZ_HIP(hipStreamSynchronize(s));
	return SYZSIG_OK;
}

extern "C" int syzsig_minimize_pred_dev(syzsig_ctx* ctx, const uint64_t* d_item_off, uint64_t nitems,
                                        const uint32_t* d_elems, const int8_t* d_prios, const uint8_t* d_item_flags,
                                        uint32_t attempts, const uint64_t* d_run_off, const uint32_t* d_run_sigs,
                                        const uint8_t* d_run_prio, const int32_t* d_run_errno,
                                        const uint8_t* d_run_exec, uint8_t* d_pred)
{
	SYZ_LOCK(ctx);
	if (!ctx || (nitems && (!d_item_off || !d_item_flags || !d_pred)) ||
	    (nitems && attempts && (!d_run_off || !d_run_prio || !d_run_errno || !d_run_exec)))
		return fail(SYZSIG_EINVAL, "minimize_pred: NULL argument");
	if (attempts > kStableMaxRuns)
		return fail(SYZSIG_ERANGE, "minimize_pred: at most 8 attempts per item");
	if (nitems == 0)
		return SYZSIG_OK;
	const hipStream_t s = ctx->stream;
	const uint64_t nruns = nitems * attempts;
	uint64_t h_off[2] = {0, 0}, h_roff = 0;
	SYZ_HIP(hipMemcpyAsync(&h_off[1], d_item_off + nitems, 8, hipMemcpyDeviceToHost, s));
	if (nruns)
		SYZ_HIP(hipMemcpyAsync(&h_roff, d_run_off + nruns, 8, hipMemcpyDeviceToHost, s));
	SYZ_HIP(hipStreamSynchronize(s));
	const uint64_t nelem = h_off[1], nsig = h_roff;
	if ((nelem && (!d_elems || !d_prios)) || (nsig && !d_run_sigs))
		return fail(SYZSIG_EINVAL, "minimize_pred: NULL argument");
	if (nruns >= (1ull << 32))
		return fail(SYZSIG_ERANGE, "minimize_pred: too many runs");
	const uint64_t C = pow2_ge(std::max<uint64_t>(2 * nsig + 16, 64));
	void *set, *alive, *cnt;
	SYZ_TRY(ws_get(ctx, 0, C * 8, &set));
	SYZ_TRY(ws_get(ctx, 1, nelem + 64, &alive));
	SYZ_TRY(ws_get(ctx, 2, nruns * 8 + 64, &cnt));
	SYZ_HIP(hipMemsetAsync(set, 0xff, C * 8, s));
	SYZ_HIP(hipMemsetAsync(cnt, 0, nruns * 8 + 8, s));
	if (nsig)
		k_runs_insert<<<(int)std::min<uint64_t>(nruns, 8192), 256, 0, s>>>(d_run_off, nruns, d_run_sigs,
		                                                                    (uint64_t*)set, C);
	// every attempt is checked on its own: an attempt the predicate skips
	// (run_ok false for other reasons) is never consulted by k_pred_items
	k_stable_elems<<<(int)std::min<uint64_t>(nitems, 8192), 256, 0, s>>>(
		d_item_off, nitems, d_elems, d_prios, attempts, d_run_off, d_run_exec, d_run_errno, d_run_prio,
		d_item_flags, (const uint64_t*)set, C, (uint8_t*)alive, (unsigned long long*)cnt, false);
	k_pred_items<<<(int)((nitems + 255) / 256), 256, 0, s>>>(d_item_off, nitems, attempts, d_run_off, d_run_exec,
	                                                          d_run_errno, d_item_flags,
	                                                          (const unsigned long long*)cnt, d_pred);
	SYZ_HIP(hipGetLastError());
	SYZ_HIP(hipStreamSynchronize(s));
	return SYZSIG_OK;
}
