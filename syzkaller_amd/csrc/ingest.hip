// ingest.hip -- executor output regions -> a triage batch, on device.
//
// Reference: pkg/ipc/ipc.go:328-468 readOutCoverage, which parses one
// executor's shmem output region (written by executor/executor.h:566-604
// handle_completion and executor_linux.cc:206-219 write_output/write_completed):
//
//   word 0                 ncmd = completed calls
//   per completed call     callIndex, callNum, errno, faultInjected,
//                          signalSize, coverSize, compsSize,
//                          sig[signalSize], cover[coverSize],
//                          compsSize x { typ, op1, op2 }   (op = 2 words if
//                          typ & compSizeMask == compSize8, else 1)
//
// into CallInfo{Signal, Cover, Errno} for each of the program's len(p.Calls)
// calls.  Like the reference, Signal aliases the region (ipc.go:410): a call's
// signal is d_out[call_start .. +call_len), so the batch feeds
// syzsig_triage_batch with sigs = d_out and no copy.  Calls without a record
// keep Errno = -1 and no signal (ipc.go:362-365).  Every error branch of the
// reference (short region, callIndex out of range, callNum mismatch, double
// record, short signal/cover, bad or short comparison) makes the whole program
// fail: the fuzzer retries such an Exec and never uses its info
// (syz-fuzzer/proc.go:269-278), so a failed program contributes no signal and
// its status says which branch fired.  The comparison operands themselves
// (prog.CompMap, used by hint mutation) are validated and skipped, not kept.
//
// One thread per program: the records of a region form a dependent chain (each
// record's length places the next), so a program is a sequential walk of <=
// len(p.Calls) headers; programs are independent.  Nothing else in the kernel
// waits on memory: which calls have a record is kept in LDS, and each call's
// outputs are written exactly once.  prio = signalPrio
// (syz-fuzzer/fuzzer.go:513-521) from errno and the caller's per-call
// CallContainsAny bit (prog/any.go:177-185, a property of the program).
#include "internal.h"

namespace syz {

constexpr uint32_t kNilLen = 0xFFFFFFFFu;  // "Signal == nil" while a program is parsed
constexpr uint32_t kCompSizeMask = 6, kCompSize8 = 6, kCompConstMask = 1;  // ipc.go:185-190

constexpr uint32_t kIngestThreads = 256;
constexpr uint32_t kSeenCalls = 256;  // calls per program tracked in LDS (beyond: a global sentinel)

__global__ __launch_bounds__(kIngestThreads) void k_ingest_exec_output(
	const uint32_t* __restrict__ out, uint64_t nwords, const uint64_t* __restrict__ prog_off, uint64_t nprog,
	const uint32_t* __restrict__ prog_call, uint64_t ncalls, const uint32_t* __restrict__ call_num,
	const uint8_t* __restrict__ call_any, uint64_t* __restrict__ call_start, uint32_t* __restrict__ call_len,
	uint8_t* __restrict__ call_prio, int32_t* __restrict__ call_errno, uint64_t* __restrict__ cover_start,
	uint32_t* __restrict__ cover_len, int32_t* __restrict__ prog_status, unsigned long long* __restrict__ cnt)
{
	// "Signal != nil" of the program's first kSeenCalls calls, one bitmap per
	// thread: the record walk is the only dependent chain, the call arrays are
	// written once and never read back.
	__shared__ uint32_t seen_w[kIngestThreads][kSeenCalls / 32 + 1];  // +1: no bank aliasing between threads
	uint32_t* seen = seen_w[threadIdx.x];
	const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
	if (p >= nprog)
		return;
	const uint64_t lo = prog_off[p], hi = prog_off[p + 1];
	const uint64_t c0 = prog_call[p], c1 = prog_call[p + 1];
	if (hi < lo || hi > nwords || c1 < c0 || c1 > ncalls) {
		prog_status[p] = SYZSIG_INGEST_EBOUNDS;
		atomicAdd(&cnt[kCntError], 1ull);
		return;
	}
	const uint64_t nc = c1 - c0;
#pragma unroll
	for (uint32_t w = 0; w < kSeenCalls / 32; w++)
		seen[w] = 0;
	for (uint64_t c = c0 + kSeenCalls; c < c1; c++)  // long programs only
		call_len[c] = kNilLen;
	auto is_seen = [&](uint64_t i) -> bool {
		return i < kSeenCalls ? (seen[i >> 5] >> (i & 31)) & 1 : call_len[c0 + i] != kNilLen;
	};
	int32_t status = SYZSIG_INGEST_OK;
	uint64_t pos = lo;
	if (pos >= hi) {
		status = SYZSIG_INGEST_ENCMD;  // ipc.go:356-359
	} else {
		const uint32_t ncmd = out[pos++];
		for (uint32_t i = 0; i < ncmd && status == SYZSIG_INGEST_OK; i++) {
			if (hi - pos < 7) {  // ipc.go:378-383
				status = SYZSIG_INGEST_EHEADER;
				break;
			}
			const uint32_t idx = out[pos], num = out[pos + 1], err = out[pos + 2];
			const uint32_t nsig = out[pos + 4], ncover = out[pos + 5], ncomps = out[pos + 6];
			pos += 7;
			if (idx >= nc) {  // ipc.go:384-388
				status = SYZSIG_INGEST_EINDEX;
				break;
			}
			const uint64_t c = c0 + idx;
			if (call_num && call_num[c] != num) {  // ipc.go:389-395
				status = SYZSIG_INGEST_ECALLNUM;
				break;
			}
			if (is_seen(idx)) {  // ipc.go:396-400 (an empty Signal is non-nil too)
				status = SYZSIG_INGEST_EDOUBLE;
				break;
			}
			if (nsig > hi - pos) {  // ipc.go:403-407
				status = SYZSIG_INGEST_ESIGNAL;
				break;
			}
			const uint64_t sig_pos = pos;
			pos += nsig;
			if (ncover > hi - pos) {  // ipc.go:411-415
				status = SYZSIG_INGEST_ECOVER;
				break;
			}
			if (idx < kSeenCalls)
				seen[idx >> 5] |= 1u << (idx & 31);
			call_start[c] = sig_pos;
			call_len[c] = nsig;
			call_errno[c] = (int32_t)err;
			call_prio[c] = signal_prio(err != 0, call_any[c]);
			if (cover_start) {
				cover_start[c] = pos;
				cover_len[c] = ncover;
			}
			pos += ncover;
			for (uint32_t j = 0; j < ncomps; j++) {  // ipc.go:420-458
				if (pos >= hi) {
					status = SYZSIG_INGEST_ECOMPS;
					break;
				}
				const uint32_t typ = out[pos++];
				if (typ > (kCompConstMask | kCompSizeMask)) {
					status = SYZSIG_INGEST_ECOMPTYPE;
					break;
				}
				const uint32_t w = (typ & kCompSizeMask) == kCompSize8 ? 4 : 2;
				if (hi - pos < w) {
					status = SYZSIG_INGEST_ECOMPS;
					break;
				}
				pos += w;
			}
		}
	}
	// calls without a record: Errno = -1, Signal = nil (ipc.go:362-365); a failed
	// Exec is retried, so none of its calls reaches checkNewSignal
	const bool bad = status != SYZSIG_INGEST_OK;
	for (uint64_t i = 0; i < nc; i++) {
		if (!bad && is_seen(i))
			continue;
		const uint64_t c = c0 + i;
		call_start[c] = lo;
		call_len[c] = 0;
		call_errno[c] = -1;
		call_prio[c] = signal_prio(1, call_any[c]);
		if (cover_start) {
			cover_start[c] = lo;
			cover_len[c] = 0;
		}
	}
	prog_status[p] = status;
	if (bad)
		atomicAdd(&cnt[kCntAux], 1ull);
}

}  // namespace syz

using namespace syz;

extern "C" int syzsig_ingest_exec_output_dev(syzsig_ctx* ctx, const uint32_t* d_out, uint64_t nwords,
                                             const uint64_t* d_prog_off, uint64_t nprog, const uint32_t* d_prog_call,
                                             uint64_t ncalls, const uint32_t* d_call_num, const uint8_t* d_call_any,
                                             uint64_t* d_call_start, uint32_t* d_call_len, uint8_t* d_call_prio,
                                             int32_t* d_call_errno, uint64_t* d_cover_start, uint32_t* d_cover_len,
                                             int32_t* d_prog_status, uint64_t* n_failed)
{
	SYZ_LOCK(ctx);
	if (!ctx || (nwords && !d_out) || (nprog && (!d_prog_off || !d_prog_call || !d_prog_status)) ||
	    (ncalls && (!d_call_any || !d_call_start || !d_call_len || !d_call_prio || !d_call_errno)) ||
	    (!d_cover_start != !d_cover_len))
		return fail(SYZSIG_EINVAL, "ingest_exec_output: NULL argument");
	if (n_failed)
		*n_failed = 0;
	if (nprog == 0)
		return SYZSIG_OK;
	SYZ_TRY(counters_reset(ctx));
	const uint64_t blocks = (nprog + kIngestThreads - 1) / kIngestThreads;
	k_ingest_exec_output<<<(unsigned)blocks, kIngestThreads, 0, ctx->stream>>>(
		d_out, nwords, d_prog_off, nprog, d_prog_call, ncalls, d_call_num, d_call_any, d_call_start, d_call_len,
		d_call_prio, d_call_errno, d_cover_start, d_cover_len, d_prog_status, ctx->d_cnt);
	SYZ_HIP(hipGetLastError());
	SYZ_TRY(counters_fetch(ctx));
	if (ctx->h_cnt[kCntError])
		return fail(SYZSIG_EINVAL, "ingest_exec_output: program offsets or call ranges out of bounds");
	if (n_failed)
		*n_failed = ctx->h_cnt[kCntAux];
	return SYZSIG_OK;
}
