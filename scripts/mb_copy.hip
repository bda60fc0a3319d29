// mb_copy.hip -- variants of a plain device copy (1 GiB, HBM to HBM), to pick
// the achievable-bandwidth kernel bench.py reports (csrc/runtime.hip k_copy16).
// Build: hipcc --offload-arch=gfx950 -O3 -o mb_copy scripts/mb_copy.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, uint64_t n)
{
	const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
	uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
	for (; i + (U - 1) * stride < n; i += U * stride) {
		v4u a[U];
#pragma unroll
		for (int u = 0; u < U; u++)
			a[u] = NT ? __builtin_nontemporal_load(&src[i + u * stride]) : src[i + u * stride];
#pragma unroll
		for (int u = 0; u < U; u++) {
			if (NT)
				__builtin_nontemporal_store(a[u], &dst[i + u * stride]);
			else
				dst[i + u * stride] = a[u];
		}
	}
	for (; i < n; i += stride)
		dst[i] = src[i];
}

template <int U, bool NT>
static void run(const char* name, v4u* s, v4u* d, uint64_t n, int grid)
{
	hipEvent_t a, b;
	hipEventCreate(&a);
	hipEventCreate(&b);
	float best = 1e9;
	for (int r = 0; r < 6; r++) {
		hipEventRecord(a);
		k_copy<U, NT><<<grid, 256>>>(s, d, n);
		hipEventRecord(b);
		hipEventSynchronize(b);
		float t;
		hipEventElapsedTime(&t, a, b);
		if (r && t < best)
			best = t;
	}
	printf("%-28s grid %6d  %.3f ms  %.0f GB/s\n", name, grid, best, 2.0 * n * 16 / (best * 1e-3) / 1e9);
}

int main()
{
	const uint64_t bytes = 1ull << 30, n = bytes / 16;
	v4u *s, *d;
	if (hipMalloc(&s, bytes) != hipSuccess || hipMalloc(&d, bytes) != hipSuccess)
		return 1;
	hipMemset(s, 1, bytes);
	for (int grid : {16384, 32768, 65536, 131072, 262144}) {
		run<2, true>("U2 nt", s, d, n, grid);
		run<1, true>("U1 nt", s, d, n, grid);
		run<4, true>("U4 nt", s, d, n, grid);
	}
	return 0;
}
