// Microbenchmark: cost of the K3 scatter's write pattern as a function of the
// piece size.  Every workgroup (one per CU, 1024 threads) owns a region of
// ncell cells and appends `piece` consecutive u32 to every cell per round, as
// k_agg_scatter does per tile; the source is streamed once (read of the same
// bytes).  Prints GB/s of (read + write) per piece size.
//   hipcc --offload-arch=gfx950 -O3 -o build/mb_scatter scripts/mb_scatter.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
	do {                                                                           \
		hipError_t e_ = (x);                                                       \
		if (e_ != hipSuccess) {                                                    \
			fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
			exit(1);                                                               \
		}                                                                          \
	} while (0)

// per block: records [blk * per_blk, +per_blk) of src; cells of cap records at
// dst + blk * per_blk + c * cap; a round writes `piece` records into every cell
__global__ __launch_bounds__(1024) void k_scat(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                               uint32_t per_blk, uint32_t ncell, uint32_t piece, uint32_t nt)
{
	const uint64_t base = (uint64_t)blockIdx.x * per_blk;
	const uint32_t tile = ncell * piece, cap = per_blk / ncell;
	for (uint32_t r = 0; r * tile < per_blk; r++) {
		for (uint32_t d = threadIdx.x; d < tile; d += blockDim.x) {
			const uint32_t c = d / piece, k = d - c * piece;
			const uint64_t i = (uint64_t)r * tile + d;
			if (i < per_blk) {
				const uint32_t v = nt ? __builtin_nontemporal_load(&src[base + i]) : src[base + i];
				dst[base + (uint64_t)c * cap + r * piece + k] = v;
			}
		}
		__syncthreads();
	}
}

// plain streaming copy for reference
__global__ __launch_bounds__(1024) void k_copy(const uint4* __restrict__ s, uint4* __restrict__ d, uint64_t n)
{
	for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
		d[i] = s[i];
}

int main(int argc, char** argv)
{
	const uint32_t nblk = 256 * (argc > 1 ? atoi(argv[1]) : 2);
	const uint64_t per_blk = 2048 * 640;  // ~5.2 MB per block
	const uint64_t n = (uint64_t)nblk * per_blk;
	uint32_t *src, *dst;
	CK(hipMalloc(&src, n * 4));
	CK(hipMalloc(&dst, n * 4));
	CK(hipMemset(src, 1, n * 4));
	CK(hipMemset(dst, 0, n * 4));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	float ms;
	for (int it = 0; it < 2; it++) {
		CK(hipEventRecord(a));
		k_copy<<<4096, 1024>>>((const uint4*)src, (uint4*)dst, n / 4);
		CK(hipEventRecord(b));
		CK(hipEventSynchronize(b));
		CK(hipEventElapsedTime(&ms, a, b));
	}
	printf("copy  %.3f ms  %.0f GB/s (r+w)\n", ms, 2.0 * n * 4 / ms / 1e6);
	// open cells per block x piece size (records): the L2 working set is
	// 32 blocks per XCD x ncell lines
	const uint32_t ncells[] = {2048, 1024, 512, 256};
	const uint32_t pieces[] = {9, 18, 36, 16, 32};
	for (uint32_t ncell : ncells)
		for (uint32_t piece : pieces) {
			for (int it = 0; it < 2; it++) {
				CK(hipEventRecord(a));
				k_scat<<<nblk, 1024>>>(src, dst, (uint32_t)per_blk, ncell, piece, 1);
				CK(hipEventRecord(b));
				CK(hipEventSynchronize(b));
				CK(hipEventElapsedTime(&ms, a, b));
			}
			printf("scatter ncell %4u piece %3u  %.3f ms  %.0f GB/s (r+w)\n", ncell, piece, ms, 2.0 * n * 4 / ms / 1e6);
		}
	return 0;
}
