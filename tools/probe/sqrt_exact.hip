// Exhaustive check (all 2^32 float bit patterns) of gfx950's single-instruction v_sqrt_f32 /
// v_rcp_f32 against the compiler's IEEE-correct sqrtf / 1.0f/x expansions. Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void check(unsigned long long* bad, uint32_t* first, uint32_t base)
{
    const uint32_t n = blockDim.x * gridDim.x;
    unsigned long long badS = 0, badR = 0, badSN = 0, badRN = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += n) {
        const uint32_t u = (uint32_t)i;
        const float x = __uint_as_float(u);
        const float a = sqrtf(x), b = __builtin_amdgcn_sqrtf(x);
        const bool nanA = a != a, nanB = b != b;
        const bool diffS = nanA != nanB || (!nanA && __float_as_uint(a) != __float_as_uint(b));
        const float c = 1.0f / x, d = __builtin_amdgcn_rcpf(x);
        const bool nanC = c != c, nanD = d != d;
        const bool diffR = nanC != nanD || (!nanC && __float_as_uint(c) != __float_as_uint(d));
        const uint32_t e = (u >> 23) & 0xFFu;
        const bool normal = e != 0u && e != 0xFFu;
        if (diffS) { ++badS; if (normal) ++badSN; if (atomicAdd(&first[0], 1u) < 8u) first[2 + (first[0] & 7)] = u; }
        if (diffR) { ++badR; if (normal) ++badRN; if (atomicAdd(&first[1], 1u) < 8u) first[10 + (first[1] & 7)] = u; }
    }
    atomicAdd(&bad[0], badS); atomicAdd(&bad[1], badSN); atomicAdd(&bad[2], badR); atomicAdd(&bad[3], badRN);
}

int main()
{
    unsigned long long* bad; uint32_t* first;
    hipMalloc(&bad, 4 * sizeof(unsigned long long)); hipMalloc(&first, 32 * sizeof(uint32_t));
    hipMemset(bad, 0, 4 * sizeof(unsigned long long)); hipMemset(first, 0, 32 * sizeof(uint32_t));
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, bad, first, 0u);
    unsigned long long h[4]; uint32_t f[32];
    hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost); hipMemcpy(f, first, sizeof(f), hipMemcpyDeviceToHost);
    printf("sqrt: %llu differ (%llu normal inputs); rcp: %llu differ (%llu normal inputs)\n", h[0], h[1], h[2], h[3]);
    printf("sqrt samples:"); for (int i = 0; i < 8; ++i) printf(" %08x", f[2 + i]); printf("\n");
    printf("rcp samples:"); for (int i = 0; i < 8; ++i) printf(" %08x", f[10 + i]); printf("\n");
    return 0;
}
