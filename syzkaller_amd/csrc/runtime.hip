// runtime.hip -- context, stream, scratch and error plumbing of libsyzsig.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "internal.h"

namespace syz {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg)
{
	set_error(msg);
	return code;
}

int hip_fail(hipError_t e, const char* what, const char* file, int line)
{
	char buf[512];
	snprintf(buf, sizeof(buf), "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
	set_error(buf);
	return e == hipErrorOutOfMemory ? SYZSIG_ENOMEM : SYZSIG_EIO;
}

int ws_get(syzsig_ctx* ctx, int i, size_t bytes, void** out)
{
	Workspace& w = ctx->ws[i];
	if (w.size < bytes) {
		if (w.ptr) {
			SYZ_HIP(hipStreamSynchronize(ctx->stream));
			SYZ_HIP(hipFree(w.ptr));
			w.ptr = nullptr;
			w.size = 0;
		}
		size_t want = bytes + bytes / 4 + 4096;
		SYZ_HIP(hipMalloc(&w.ptr, want));
		w.size = want;
	}
	*out = w.ptr;
	return SYZSIG_OK;
}

int ws_grow_keep(syzsig_ctx* ctx, int i, size_t bytes, size_t keep, void** out)
{
	Workspace& w = ctx->ws[i];
	if (w.size >= bytes) {
		*out = w.ptr;
		return SYZSIG_OK;
	}
	void* n = nullptr;
	const size_t want = bytes + bytes / 4 + 4096;
	SYZ_HIP(hipMalloc(&n, want));
	if (w.ptr) {
		if (keep)
			SYZ_HIP(hipMemcpyAsync(n, w.ptr, std::min(keep, w.size), hipMemcpyDeviceToDevice, ctx->stream));
		SYZ_HIP(hipStreamSynchronize(ctx->stream));
		SYZ_HIP(hipFree(w.ptr));
	}
	w.ptr = n;
	w.size = want;
	*out = n;
	return SYZSIG_OK;
}

int counters_reset(syzsig_ctx* ctx)
{
	SYZ_HIP(hipMemsetAsync(ctx->d_cnt, 0, sizeof(unsigned long long) * kNumCounters, ctx->stream));
	return SYZSIG_OK;
}

int counters_fetch(syzsig_ctx* ctx)
{
	SYZ_HIP(hipMemcpyAsync(ctx->h_cnt, ctx->d_cnt, sizeof(unsigned long long) * kNumCounters,
	                       hipMemcpyDeviceToHost, ctx->stream));
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	return SYZSIG_OK;
}

}  // namespace syz

namespace syz {
// A plain device copy (the achievable-bandwidth companion of the rooflines:
// SURVEY 8(d) "also measure achievable BW with a device copy kernel"): one
// 16-B element per lane, nontemporal, one wave-pass over the buffer -- of the
// forms measured (scripts/mb_copy.hip: 1-8 elements per lane, grid-stride or
// not, plain or nontemporal) the fastest, 6.2-6.6 TB/s on 1 GiB.
typedef uint32_t v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_copy16(const v4u* __restrict__ src, v4u* __restrict__ dst, uint64_t n)
{
	const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride)
		__builtin_nontemporal_store(__builtin_nontemporal_load(&src[i]), &dst[i]);
}
}  // namespace syz

extern "C" {

int syzsig_abi_version(void) { return SYZSIG_ABI_VERSION; }

const char* syzsig_last_error(void) { return syz::g_last_error.c_str(); }

int syzsig_ctx_create(int device, syzsig_ctx** out)
{
	if (!out)
		return syz::fail(SYZSIG_EINVAL, "ctx_create: out is NULL");
	*out = nullptr;
	int ndev = 0;
	SYZ_HIP(hipGetDeviceCount(&ndev));
	if (device < 0 || device >= ndev)
		return syz::fail(SYZSIG_EINVAL, "ctx_create: no such HIP device");
	SYZ_HIP(hipSetDevice(device));
	syzsig_ctx* c = new syzsig_ctx();
	c->device = device;
	// A BLOCKING stream: it is ordered after work already queued on the null
	// stream and the null stream after it (legacy default-stream semantics).
	// torch's default stream is the null stream, so tensors produced there --
	// and RCCL results a synchronous collective made it wait for -- are ready
	// when a library kernel on this stream reads them, without a host sync.
	hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamDefault);
	if (e == hipSuccess)
		e = hipMalloc(&c->d_cnt, sizeof(unsigned long long) * syz::kNumCounters);
	if (e == hipSuccess)
		e = hipHostMalloc(&c->h_cnt, sizeof(unsigned long long) * syz::kNumCounters, hipHostMallocDefault);
	if (e == hipSuccess)
		e = hipHostMalloc(&c->h_pin, syz::kPinBytes, hipHostMallocDefault);
	if (e == hipSuccess)
		e = hipMalloc(&c->d_step, sizeof(unsigned long long) * syz::kStepCounters);
	if (e == hipSuccess)
		e = hipMemset(c->d_step, 0, sizeof(unsigned long long) * syz::kStepCounters);
	if (e == hipSuccess)
		e = hipHostMalloc(&c->h_step, sizeof(unsigned long long) * syz::kStepCounters, hipHostMallocDefault);
	if (e != hipSuccess) {
		syzsig_ctx_destroy(c);
		return syz::hip_fail(e, "ctx_create", __FILE__, __LINE__);
	}
	c->stream = c->own_stream;
	if (const char* v = getenv("SYZSIG_PART_MODE"))
		c->part_mode = atoi(v);
	if (const char* v = getenv("SYZSIG_AGG_DBG")) {
		c->agg_dbg = (uint32_t)atoi(v);
#ifndef SYZ_EXPERIMENTS
		// timing-only bits (skipped merges, dropped records) exist only in an
		// experiment build (make exp EXPFLAGS=-DSYZ_EXPERIMENTS): a stray variable
		// can select the result-preserving debug paths and nothing else
		c->agg_dbg &= syz::kDebugAccepted;
#endif
	}
#ifdef SYZ_EXPERIMENTS
	if (const char* v = getenv("SYZSIG_EDGE_WAVES"))
		c->edge_waves = atoi(v) == 8 ? 8 : atoi(v) == 2 ? 2 : atoi(v) == 1 ? 1 : 4;
#endif
	if (const char* v = getenv("SYZSIG_AGG_PARTS")) {
		const uint32_t n = (uint32_t)atoi(v);
		if (n >= 8 && n <= 2048 && !(n & (n - 1)))
			c->agg_parts = n;
	}
	*out = c;
	return SYZSIG_OK;
}

void syzsig_ctx_destroy(syzsig_ctx* c)
{
	if (!c)
		return;
	(void)hipSetDevice(c->device);
	if (c->stream)
		(void)hipStreamSynchronize(c->stream);
	for (auto& w : c->ws)
		if (w.ptr)
			(void)hipFree(w.ptr);
	if (c->d_cnt)
		(void)hipFree(c->d_cnt);
	if (c->h_cnt)
		(void)hipHostFree(c->h_cnt);
	if (c->h_pin)
		(void)hipHostFree(c->h_pin);
	if (c->d_step)
		(void)hipFree(c->d_step);
	if (c->h_step)
		(void)hipHostFree(c->h_step);
	for (auto& e : c->ev)
		if (e)
			(void)hipEventDestroy(e);
	for (auto& e : c->ev_step)
		if (e)
			(void)hipEventDestroy(e);
	if (c->own_stream)
		(void)hipStreamDestroy(c->own_stream);
	delete c;
}

int syzsig_ctx_set_stream(syzsig_ctx* ctx, void* stream)
{
	SYZ_LOCK(ctx);
	if (!ctx)
		return syz::fail(SYZSIG_EINVAL, "ctx_set_stream: ctx is NULL");
	ctx->stream = stream ? (hipStream_t)stream : ctx->own_stream;
	return SYZSIG_OK;
}

void* syzsig_ctx_stream(syzsig_ctx* ctx)
{
	SYZ_LOCK(ctx);
	return ctx ? (void*)ctx->stream : nullptr;
}

int syzsig_ctx_set_agg(syzsig_ctx* ctx, int mode, uint32_t parts)
{
	SYZ_LOCK(ctx);
	if (!ctx)
		return syz::fail(SYZSIG_EINVAL, "ctx_set_agg: ctx is NULL");
	if (mode < 0 || mode > 2 || (parts && (parts < 8 || parts > 2048 || (parts & (parts - 1)))))
		return syz::fail(SYZSIG_EINVAL, "ctx_set_agg: mode must be 0..2 and parts 0 or a power of two in 8..2048");
	ctx->part_mode = mode;
	ctx->agg_parts = parts;
	ctx->cap_sd = ctx->cap_sd_entry = syz::kCapSdDefault;  // capped cells again, with the default slack
	return SYZSIG_OK;
}

int syzsig_ctx_set_debug(syzsig_ctx* ctx, uint32_t flags)
{
	SYZ_LOCK(ctx);
	if (!ctx)
		return syz::fail(SYZSIG_EINVAL, "ctx_set_debug: ctx is NULL");
	ctx->agg_dbg = flags & syz::kDebugAccepted;
	return SYZSIG_OK;
}

double syzsig_ctx_last_ms(syzsig_ctx* ctx)
{
	SYZ_LOCK(ctx);
	return ctx ? ctx->last_ms : 0;
}

int syzsig_copy_bw_dev(syzsig_ctx* ctx, void* d_dst, const void* d_src, uint64_t bytes, double* ms)
{
	SYZ_LOCK(ctx);
	if (!ctx || !ms || (bytes && (!d_dst || !d_src)))
		return syz::fail(SYZSIG_EINVAL, "copy_bw: NULL argument");
	if ((bytes & 15) || ((uintptr_t)d_dst & 15) || ((uintptr_t)d_src & 15))
		return syz::fail(SYZSIG_EINVAL, "copy_bw: 16-B aligned buffers and size");
	hipEvent_t ev[2];
	SYZ_HIP(hipEventCreate(&ev[0]));
	SYZ_HIP(hipEventCreate(&ev[1]));
	const uint64_t n = bytes / 16;
	// one 16-B element per lane, one pass (grid-stride only past 2^30 threads)
	const uint32_t grid = (uint32_t)std::min<uint64_t>(std::max<uint64_t>((n + 255) / 256, 1), 1u << 22);
	int rc = SYZSIG_OK;
	if (hipEventRecord(ev[0], ctx->stream) != hipSuccess)
		rc = syz::fail(SYZSIG_EIO, "copy_bw: event record");
	if (rc == SYZSIG_OK && n)
		syz::k_copy16<<<grid, 256, 0, ctx->stream>>>((const syz::v4u*)d_src, (syz::v4u*)d_dst, n);
	if (rc == SYZSIG_OK && (hipGetLastError() != hipSuccess || hipEventRecord(ev[1], ctx->stream) != hipSuccess ||
	                        hipEventSynchronize(ev[1]) != hipSuccess))
		rc = syz::fail(SYZSIG_EIO, "copy_bw: kernel");
	float t = 0;
	if (rc == SYZSIG_OK && hipEventElapsedTime(&t, ev[0], ev[1]) != hipSuccess)
		rc = syz::fail(SYZSIG_EIO, "copy_bw: elapsed time");
	*ms = t;
	(void)hipEventDestroy(ev[0]);
	(void)hipEventDestroy(ev[1]);
	return rc;
}

int syzsig_host_alloc(syzsig_ctx* ctx, uint64_t bytes, void** out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !out)
		return syz::fail(SYZSIG_EINVAL, "host_alloc: NULL argument");
	*out = nullptr;
	if (bytes == 0)
		return SYZSIG_OK;
	if (hipHostMalloc(out, bytes, hipHostMallocDefault) != hipSuccess) {
		*out = nullptr;
		return syz::fail(SYZSIG_ENOMEM, "host_alloc: hipHostMalloc failed");
	}
	return SYZSIG_OK;
}

int syzsig_host_free(syzsig_ctx* ctx, void* p)
{
	SYZ_LOCK(ctx);
	if (p && hipHostFree(p) != hipSuccess)
		return syz::fail(SYZSIG_EIO, "host_free: hipHostFree failed");
	return SYZSIG_OK;
}

int syzsig_ctx_set_timing(syzsig_ctx* ctx, int enable)
{
	SYZ_LOCK(ctx);
	if (!ctx)
		return syz::fail(SYZSIG_EINVAL, "ctx_set_timing: ctx is NULL");
	if (enable && !ctx->ev[0]) {
		for (auto& e : ctx->ev)
			SYZ_HIP(hipEventCreate(&e));
		for (auto& e : ctx->ev_step)
			SYZ_HIP(hipEventCreate(&e));
	}
	ctx->timing = enable != 0;
	return SYZSIG_OK;
}

}  // extern "C"
