// fetch_calib.hip -- calibrates rocprofv3's FETCH_SIZE / TCC_EA0_RDREQ against known byte counts
// for the access patterns of the cast kernel (diagnostic tool, not part of the product).
//
// Over a 2 GiB buffer (8x the 256 MiB Infinity Cache, so most lines come from HBM):
//   stream16        every lane reads consecutive float4s (coalesced streaming, 16 B/lane);
//   chase{16,32,64,128}  every lane follows a dependent chain of random records of R bytes
//                   (R/16 float4 loads of one R-aligned record; the next record's index is the
//                   record's first word) -- the node / triangle fetches of the traversal.
// Each kernel is launched once per pass; the program prints the bytes it requested per kernel,
// which tools/fetch_calib.py divides into the profiled FETCH_SIZE / TCC_EA0_RDREQ.
//   hipcc --offload-arch=gfx950 -O3 -o fetch_calib tools/probe/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
            std::exit(1);                                                                 \
        }                                                                                 \
    } while (0)

constexpr size_t kBytes = size_t(2) << 30;          // 2 GiB
constexpr uint32_t kLanes = 256 * 256 * 4;           // 4 workgroups of 256 per CU
constexpr uint32_t kHops = 64;

__global__ void stream16(const float4* __restrict__ buf, size_t n, float* out)
{
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    float s = 0.0f;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 v = buf[i];
        s += v.x + v.y + v.z + v.w;
    }
    out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int R>
__global__ void chase(const float4* __restrict__ buf, uint32_t records, const uint32_t* __restrict__ start, uint32_t hops,
                      float* out)
{
    const uint32_t lane = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t rec = start[lane] % records;
    float s = 0.0f;
    for (uint32_t h = 0; h < hops; ++h) {
        const float4* p = buf + (size_t)rec * (R / 16);
        float4 v[R / 16];
#pragma unroll
        for (int k = 0; k < R / 16; ++k) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < R / 16; ++k) s += v[k].y + v[k].z + v[k].w;
        rec = __float_as_uint(v[0].x) % records;
    }
    out[lane] = s;
}

// every float4's x: a random record index (a 32-bit LCG per element)
__global__ void fill(float4* buf, size_t n)
{
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        uint32_t x = (uint32_t)(i * 2654435761ull) ^ 0x9E3779B9u;
        x = x * 1664525u + 1013904223u;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        buf[i] = make_float4(__uint_as_float(x), 1.0f, 2.0f, 3.0f);
    }
}

template <int R>
void run_chase(const float4* buf, const uint32_t* start, float* out)
{
    const uint32_t records = (uint32_t)(kBytes / R);
    hipLaunchKernelGGL(chase<R>, dim3(kLanes / 256), dim3(256), 0, 0, buf, records, start, kHops, out);
    CHECK(hipDeviceSynchronize());
    std::printf("chase%d requested_bytes %llu accesses %llu\n", R, (unsigned long long)kLanes * kHops * R,
                (unsigned long long)kLanes * kHops);
}

int main()
{
    float4* buf = nullptr;
    uint32_t* start = nullptr;
    float* out = nullptr;
    const size_t n = kBytes / 16;
    CHECK(hipMalloc(&buf, kBytes));
    CHECK(hipMalloc(&start, kLanes * 4));
    CHECK(hipMalloc(&out, (size_t)kLanes * 4 * 4));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, buf, n);
    std::vector<uint32_t> s(kLanes);
    uint64_t x = 88172645463325252ull;
    for (auto& v : s) {
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        v = (uint32_t)(x >> 16);
    }
    CHECK(hipMemcpy(start, s.data(), kLanes * 4, hipMemcpyHostToDevice));
    CHECK(hipDeviceSynchronize());
    // streaming: 1 GiB of the buffer, coalesced float4 per lane
    hipLaunchKernelGGL(stream16, dim3(kLanes / 256), dim3(256), 0, 0, (const float4*)buf, n / 2, out);
    CHECK(hipDeviceSynchronize());
    std::printf("stream16 requested_bytes %llu accesses %llu\n", (unsigned long long)(n / 2) * 16, (unsigned long long)(n / 2));
    run_chase<16>(buf, start, out);
    run_chase<32>(buf, start, out);
    run_chase<64>(buf, start, out);
    run_chase<128>(buf, start, out);
    CHECK(hipFree(buf));
    CHECK(hipFree(start));
    CHECK(hipFree(out));
    return 0;
}
