// Exhaustive check (every float bit pattern in the tested range) of reciprocal sequences
// built on v_rcp_f32 + FMA corrections against the compiler's IEEE-correct 1.0f / x.
// Diagnostic only: tells whether a shorter sequence is bit-identical over a range.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ float rcp_a(float x)   // one Newton step
{
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__device__ __forceinline__ float rcp_b(float x)   // Newton step + Markstein correction
{
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    const float r1 = __builtin_fmaf(e, r, r);
    const float e2 = __builtin_fmaf(-x, r1, 1.0f);
    return __builtin_fmaf(e2, r1, r1);
}

__global__ void check(unsigned long long* bad, uint32_t* sample)
{
    const uint32_t n = blockDim.x * gridDim.x;
    unsigned long long ba = 0, bb = 0, tested = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += n) {
        const uint32_t u = (uint32_t)i;
        const uint32_t e = (u >> 23) & 0xFFu;
        if (e < 1u || e > 252u) continue;   // normal x whose reciprocal is normal
        ++tested;
        const float x = __uint_as_float(u);
        const float ref = 1.0f / x;
        if (__float_as_uint(rcp_a(x)) != __float_as_uint(ref)) ++ba;
        if (__float_as_uint(rcp_b(x)) != __float_as_uint(ref)) { ++bb; sample[0] = u; }
    }
    atomicAdd(&bad[0], ba); atomicAdd(&bad[1], bb); atomicAdd(&bad[2], tested);
}

int main()
{
    unsigned long long* bad; uint32_t* sample;
    (void)hipMalloc(&bad, 3 * sizeof(unsigned long long)); (void)hipMalloc(&sample, 4);
    (void)hipMemset(bad, 0, 3 * sizeof(unsigned long long)); (void)hipMemset(sample, 0, 4);
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, bad, sample);
    unsigned long long h[3]; uint32_t s;
    (void)hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost); (void)hipMemcpy(&s, sample, 4, hipMemcpyDeviceToHost);
    printf("tested %llu: one Newton step differs on %llu, with the correction on %llu (e.g. %08x)\n", h[2], h[0], h[1], s);
    return 0;
}
