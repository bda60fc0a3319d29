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

}  // extern "C"
