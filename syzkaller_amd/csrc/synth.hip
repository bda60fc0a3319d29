// synth.hip -- the deterministic synthetic workload (common.h), on host and
// device.  Test and bench input generation only; not part of the triage path.
#include "internal.h"

namespace syz {

static SynthCfg to_cfg(const syzsig_synth_cfg* c)
{
	SynthCfg s;
	s.seed = c->seed;
	s.nblocks_log2 = c->nblocks_log2;
	s.region_log2 = c->region_log2;
	s.nsys = c->nsys;
	s.skew = c->skew;
	s.restart_log2 = c->restart_log2;
	s.errno_permille = c->errno_permille;
	s.any_permille = c->any_permille;
	s.bad_pc_ppm = c->bad_pc_ppm;
	s.global_walk = c->global_walk;
	return s;
}

static bool cfg_ok(const syzsig_synth_cfg* c)
{
	return c && c->nblocks_log2 >= 1 && c->nblocks_log2 <= 24 && c->region_log2 >= 1 &&
	       c->region_log2 <= c->nblocks_log2 && c->nsys >= 1 && c->restart_log2 >= 1 && c->restart_log2 <= 30;
}

__global__ void k_synth_traces(SynthCfg cfg, uint64_t prog_base, uint64_t ncalls, uint32_t cpp,
                               const uint64_t* __restrict__ call_start, const uint32_t* __restrict__ call_len,
                               uint64_t* pcs, uint8_t* call_prio)
{
	for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < ncalls;
	     c += (uint64_t)gridDim.x * blockDim.x) {
		const uint64_t prog = prog_base + c / cpp;
		const uint32_t call = (uint32_t)(c % cpp);
		SynthCall sc = synth_call(cfg, prog, call);
		call_prio[c] = signal_prio(sc.failed, sc.any);
		synth_trace(cfg, prog, call, pcs + call_start[c], call_len[c]);
	}
}

__global__ void k_synth_m0(SynthCfg cfg, uint64_t n_known, uint64_t n, uint32_t* elems, int8_t* prios)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
		synth_m0_elem(cfg, i, n_known, &elems[i], &prios[i]);
}

// One rank's shard of M0 (syzsig_synth_m0_shard_dev), in index order: per tile
// of kM0Tile indices the owned count, a scan over the tiles, then each tile
// writes its owned elements at its offset, ordered by index (wave ballots and
// a running offset in LDS).
constexpr uint32_t kM0Tile = 4096, kM0Threads = 256;

__global__ __launch_bounds__(kM0Threads) void k_m0_shard_count(SynthCfg cfg, uint64_t n_known, uint64_t n,
                                                               uint32_t nshards, uint32_t shard, uint64_t* tcnt)
{
	const uint64_t t0 = (uint64_t)blockIdx.x * kM0Tile;
	uint64_t c = 0;
	for (uint32_t u = threadIdx.x; u < kM0Tile; u += kM0Threads) {
		const uint64_t i = t0 + u;
		if (i < n) {
			uint32_t e;
			int8_t p;
			synth_m0_elem(cfg, i, n_known, &e, &p);
			c += owner_of(e, nshards) == shard;
		}
	}
	__shared__ unsigned long long s;
	if (threadIdx.x == 0)
		s = 0;
	__syncthreads();
	c = wave_sum_u64(c);
	if (lane_id() == 0)
		atomicAdd(&s, (unsigned long long)c);
	__syncthreads();
	if (threadIdx.x == 0)
		tcnt[blockIdx.x] = s;
}

// exclusive scan of ntiles counts (one block), total -> *total
__global__ __launch_bounds__(1024) void k_m0_shard_scan(uint64_t* tcnt, uint64_t ntiles, uint64_t* total)
{
	__shared__ uint64_t part[1024];
	const uint64_t per = (ntiles + 1023) / 1024, a = threadIdx.x * per, z = min<uint64_t>(ntiles, a + per);
	uint64_t s = 0;
	for (uint64_t i = a; i < z; i++)
		s += tcnt[i];
	part[threadIdx.x] = s;
	__syncthreads();
	if (threadIdx.x == 0) {
		uint64_t run = 0;
		for (int k = 0; k < 1024; k++) {
			const uint64_t v = part[k];
			part[k] = run;
			run += v;
		}
		*total = run;
	}
	__syncthreads();
	uint64_t run = part[threadIdx.x];
	for (uint64_t i = a; i < z; i++) {
		const uint64_t v = tcnt[i];
		tcnt[i] = run;
		run += v;
	}
}

__global__ __launch_bounds__(kM0Threads) void k_m0_shard_write(SynthCfg cfg, uint64_t n_known, uint64_t n,
                                                               uint32_t nshards, uint32_t shard,
                                                               const uint64_t* __restrict__ toff, uint32_t* elems,
                                                               int8_t* prios, uint64_t cap)
{
	__shared__ uint32_t wc[kM0Threads / 64];
	const uint32_t w = threadIdx.x >> 6, lane = lane_id();
	const uint64_t t0 = (uint64_t)blockIdx.x * kM0Tile;
	uint64_t run = toff[blockIdx.x];
	for (uint32_t u = 0; u < kM0Tile; u += kM0Threads) {
		const uint64_t i = t0 + u + threadIdx.x;
		uint32_t e = 0;
		int8_t p = 0;
		bool own = false;
		if (i < n) {
			synth_m0_elem(cfg, i, n_known, &e, &p);
			own = owner_of(e, nshards) == shard;
		}
		const uint64_t m = __ballot(own);
		if (lane == 0)
			wc[w] = (uint32_t)__popcll(m);
		__syncthreads();
		uint32_t before = 0, tot = 0;
		for (uint32_t k = 0; k < kM0Threads / 64; k++) {
			before += k < w ? wc[k] : 0;
			tot += wc[k];
		}
		const uint64_t o = run + before + lane_rank(m);
		if (own && o < cap) {
			elems[o] = e;
			prios[o] = p;
		}
		run += tot;
		__syncthreads();  // wc is rewritten by the next step
	}
}

}  // namespace syz

using namespace syz;

extern "C" {

void syzsig_synth_default(syzsig_synth_cfg* c)
{
	c->seed = 20181015;
	c->nblocks_log2 = 20;
	c->region_log2 = 8;
	c->nsys = 4096;
	c->skew = 0;
	c->restart_log2 = 5;
	c->errno_permille = 300;
	c->any_permille = 100;
	c->bad_pc_ppm = 0;
	c->global_walk = 0;
}

int syzsig_synth_traces_host(const syzsig_synth_cfg* cfg, uint64_t prog_base, uint64_t nprog, uint32_t cpp,
                             const uint64_t* call_start, const uint32_t* call_len, uint64_t* pcs, uint8_t* call_prio)
{
	if (!cfg_ok(cfg) || cpp == 0 || (nprog && (!call_start || !call_len || !pcs || !call_prio)))
		return fail(SYZSIG_EINVAL, "synth_traces: bad argument");
	SynthCfg s = to_cfg(cfg);
	for (uint64_t c = 0; c < nprog * cpp; c++) {
		const uint64_t prog = prog_base + c / cpp;
		const uint32_t call = (uint32_t)(c % cpp);
		SynthCall sc = synth_call(s, prog, call);
		call_prio[c] = signal_prio(sc.failed, sc.any);
		synth_trace(s, prog, call, pcs + call_start[c], call_len[c]);
	}
	return SYZSIG_OK;
}

int syzsig_synth_traces_dev(syzsig_ctx* ctx, const syzsig_synth_cfg* cfg, uint64_t prog_base, uint64_t nprog,
                            uint32_t cpp, const uint64_t* d_call_start, const uint32_t* d_call_len, uint64_t* d_pcs,
                            uint8_t* d_call_prio)
{
	SYZ_LOCK(ctx);
	if (!ctx || !cfg_ok(cfg) || cpp == 0)
		return fail(SYZSIG_EINVAL, "synth_traces: bad argument");
	const uint64_t ncalls = nprog * cpp;
	if (!ncalls)
		return SYZSIG_OK;
	k_synth_traces<<<grid_for(ncalls, 256, 8192), 256, 0, ctx->stream>>>(to_cfg(cfg), prog_base, ncalls, cpp,
	                                                                     d_call_start, d_call_len, d_pcs, d_call_prio);
	SYZ_HIP(hipGetLastError());
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	return SYZSIG_OK;
}

int syzsig_synth_m0_host(const syzsig_synth_cfg* cfg, uint64_t known_sys, uint64_t n, uint32_t* elems, int8_t* prios)
{
	if (!cfg_ok(cfg) || (n && (!elems || !prios)))
		return fail(SYZSIG_EINVAL, "synth_m0: bad argument");
	SynthCfg s = to_cfg(cfg);
	uint64_t n_known = synth_n_known(s, known_sys);
	for (uint64_t i = 0; i < n; i++)
		synth_m0_elem(s, i, n_known, &elems[i], &prios[i]);
	return SYZSIG_OK;
}

int syzsig_synth_m0_dev(syzsig_ctx* ctx, const syzsig_synth_cfg* cfg, uint64_t known_sys, uint64_t n,
                        uint32_t* d_elems, int8_t* d_prios)
{
	SYZ_LOCK(ctx);
	if (!ctx || !cfg_ok(cfg))
		return fail(SYZSIG_EINVAL, "synth_m0: bad argument");
	if (!n)
		return SYZSIG_OK;
	SynthCfg s = to_cfg(cfg);
	k_synth_m0<<<grid_for(n, 256, 8192), 256, 0, ctx->stream>>>(s, synth_n_known(s, known_sys), n, d_elems,
	                                                             d_prios);
	SYZ_HIP(hipGetLastError());
	SYZ_HIP(hipStreamSynchronize(ctx->stream));
	return SYZSIG_OK;
}

int syzsig_synth_m0_shard_dev(syzsig_ctx* ctx, const syzsig_synth_cfg* cfg, uint64_t known_sys, uint64_t n,
                              uint32_t nshards, uint32_t shard, uint32_t* d_elems, int8_t* d_prios, uint64_t cap,
                              uint64_t* n_out)
{
	SYZ_LOCK(ctx);
	if (!ctx || !cfg_ok(cfg) || !n_out || nshards == 0 || shard >= nshards || (cap && (!d_elems || !d_prios)))
		return fail(SYZSIG_EINVAL, "synth_m0_shard: bad argument");
	*n_out = 0;
	if (!n)
		return SYZSIG_OK;
	SynthCfg s = to_cfg(cfg);
	const uint64_t nk = synth_n_known(s, known_sys), ntiles = (n + kM0Tile - 1) / kM0Tile;
	if (ntiles > 0x7FFFFFFFull)
		return fail(SYZSIG_ERANGE, "synth_m0_shard: n too large");
	void* w;
	SYZ_TRY(ws_get(ctx, 9, (ntiles + 1) * 8 + 64, &w));
	uint64_t* tcnt = (uint64_t*)w;
	uint64_t* tot = tcnt + ntiles;
	const hipStream_t st = ctx->stream;
	k_m0_shard_count<<<(uint32_t)ntiles, kM0Threads, 0, st>>>(s, nk, n, nshards, shard, tcnt);
	k_m0_shard_scan<<<1, 1024, 0, st>>>(tcnt, ntiles, tot);
	k_m0_shard_write<<<(uint32_t)ntiles, kM0Threads, 0, st>>>(s, nk, n, nshards, shard, tcnt, d_elems, d_prios, cap);
	SYZ_HIP(hipGetLastError());
	uint64_t* h = (uint64_t*)(ctx->h_pin + kPinPairs);
	SYZ_HIP(hipMemcpyAsync(h, tot, 8, hipMemcpyDeviceToHost, st));
	SYZ_HIP(hipStreamSynchronize(st));
	*n_out = *h;
	if (*h > cap)
		return fail(SYZSIG_ERANGE, "synth_m0_shard: cap smaller than the shard");
	return SYZSIG_OK;
}

}  // extern "C"
