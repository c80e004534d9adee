// Exhaustive check of sqrt_ieee's fast path (csrc/device/dmath.h: v_sqrt_f32 and the residuals
// of its two neighbours) against the compiler's IEEE-correct sqrtf, for every x it takes: sign 0,
// biased exponent 31..254. Diagnostic only.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe/sqrt_fast tools/probe/sqrt_fast.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

__device__ __forceinline__ float sqrt_fast(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float lo = __uint_as_float(__float_as_uint(s) - 1u), hi = __uint_as_float(__float_as_uint(s) + 1u);
    const float rlo = __builtin_fmaf(-lo, s, x), rhi = __builtin_fmaf(-hi, s, x);
    const float r = rlo <= 0.0f ? lo : s;
    return rhi > 0.0f ? hi : r;
}

__global__ void check(unsigned long long* out, uint32_t* sample)
{
    const uint64_t first = 31ull << 23, last = 255ull << 23;   // [2^-96, 2^128)
    unsigned long long bad = 0, tested = 0;
    for (uint64_t i = first + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < last; i += (uint64_t)gridDim.x * blockDim.x) {
        const float x = __uint_as_float((uint32_t)i);
        ++tested;
        if (__float_as_uint(sqrt_fast(x)) != __float_as_uint(sqrtf(x))) { ++bad; sample[0] = (uint32_t)i; }
    }
    atomicAdd(&out[0], bad);
    atomicAdd(&out[1], tested);
}

int main()
{
    unsigned long long* d; uint32_t* s;
    (void)hipMalloc(&d, 2 * sizeof(unsigned long long)); (void)hipMalloc(&s, 4);
    (void)hipMemset(d, 0, 2 * sizeof(unsigned long long)); (void)hipMemset(s, 0, 4);
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, d, s);
    unsigned long long h[2]; uint32_t e;
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost); (void)hipMemcpy(&e, s, 4, hipMemcpyDeviceToHost);
    std::printf("tested %llu: the fast path differs on %llu (e.g. %08x)\n", h[1], h[0], e);
    return h[0] != 0;
}
