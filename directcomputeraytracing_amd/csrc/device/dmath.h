// dmath.h -- device math for the MI355X wavefront path tracer.
//
// Floating point follows the reference HLSL operation by operation (compiled
// with -ffp-contract=off, IEEE division/sqrt), and the transcendentals use one
// fixed float-only definition (range reduction + minimax polynomial) so a
// pixel's value is the same bits on every device and on the CPU restatement.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define DEV __device__ __forceinline__

namespace dcrt {
namespace dev {

constexpr float kPi = 3.14159265359f;          // Math.inc.hlsl:4
constexpr float kPiMul2 = 6.283185307f;        // Math.inc.hlsl:5
constexpr float kInvPi = 1.0f / 3.14159265359f;
constexpr float kShadowEpsilon = 1e-3f;        // RayTracingCommon.inc.hlsl:3
constexpr float kAlphaThreshold = 0.00052441f; // BSDFs.inc.hlsl:12

DEV float asf(uint32_t u) { return __uint_as_float(u); }
DEV uint32_t asu(float f) { return __float_as_uint(f); }
DEV float inf() { return __uint_as_float(0x7f800000u); }

// ---- deterministic transcendentals ----------------------------------------
DEV float reduce_pio2(float x, int* q)
{
    const float k = rintf(x * 0.636619772f);
    *q = ((int)k) & 3;
    float r = x - k * 1.5703125f;
    r = r - k * 4.837512969970703125e-4f;
    r = r - k * 7.54978995489188216e-8f;
    return r;
}
DEV float sin_poly(float r)
{
    const float z = r * r;
    float y = -1.9515295891e-4f * z;
    y = y + 8.3321608736e-3f;
    y = y * z;
    y = y - 1.6666654611e-1f;
    y = y * z;
    y = y * r;
    return y + r;
}
DEV float cos_poly(float r)
{
    const float z = r * r;
    float y = 2.443315711809948e-5f * z;
    y = y - 1.388731625493765e-3f;
    y = y * z;
    y = y + 4.166664568298827e-2f;
    y = y * z;
    y = y * z;
    y = y - 0.5f * z;
    return y + 1.0f;
}
DEV void det_sincos(float x, float* s, float* c)
{
    if (!(fabsf(x) <= 1.0e30f)) { *s = x - x; *c = x - x; return; }
    int q;
    const float r = reduce_pio2(x, &q);
    const float sp = sin_poly(r), cp = cos_poly(r);
    switch (q) {
    case 0: *s = sp; *c = cp; break;
    case 1: *s = cp; *c = -sp; break;
    case 2: *s = -sp; *c = -cp; break;
    default: *s = -cp; *c = sp; break;
    }
}
DEV float det_sin(float x) { float s, c; det_sincos(x, &s, &c); return s; }
DEV float det_cos(float x) { float s, c; det_sincos(x, &s, &c); return c; }
DEV float det_exp(float x)
{
    if (x != x) return x;
    if (x > 88.72283905f) return inf();
    if (x < -103.972084f) return 0.0f;
    const float z = floorf(x * 1.44269504088896341f + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    const int n = (int)z;
    const float zz = x * x;
    float y = 1.9875691500e-4f * x;
    y = y + 1.3981999507e-3f; y = y * x;
    y = y + 8.3334519073e-3f; y = y * x;
    y = y + 4.1665795894e-2f; y = y * x;
    y = y + 1.6666665459e-1f; y = y * x;
    y = y + 5.0000001201e-1f;
    y = y * zz;
    y = y + x;
    y = y + 1.0f;
    const int n1 = n / 2, n2 = n - n1;
    y = y * asf((uint32_t)(n1 + 127) << 23);
    y = y * asf((uint32_t)(n2 + 127) << 23);
    return y;
}
// Cephes logf restated; the same code in the oracle (post-processing luminance).
DEV float det_log(float x)
{
    if (x != x) return x;
    if (x < 0.0f) return asf(0x7FC00000u);
    if (x == 0.0f) return -inf();
    if (x == inf()) return x;
    int e = 0;
    if (x < 1.17549435e-38f) { x = x * 8388608.0f; e = -23; }          // denormal: scale by 2^23
    const uint32_t bits = asu(x);
    e += (int)((bits >> 23) & 0xFFu) - 126;
    float m = asf((bits & 0x007FFFFFu) | 0x3F000000u);                   // [0.5, 1)
    if (m < 0.707106781186547524f) { e -= 1; m = m + m - 1.0f; } else { m = m - 1.0f; }
    const float z = m * m;
    float y = 7.0376836292e-2f * m;
    y = y - 1.1514610310e-1f; y = y * m;
    y = y + 1.1676998740e-1f; y = y * m;
    y = y - 1.2420140846e-1f; y = y * m;
    y = y + 1.4249322787e-1f; y = y * m;
    y = y - 1.6668057665e-1f; y = y * m;
    y = y + 2.0000714765e-1f; y = y * m;
    y = y - 2.4999993993e-1f; y = y * m;
    y = y + 3.3333331174e-1f; y = y * m;
    y = y * z;
    const float fe = (float)e;
    y = y + -2.12194440e-4f * fe;
    y = y + -0.5f * z;
    float r = m + y;
    r = r + 0.693359375f * fe;
    return r;
}
DEV float det_atan(float x)
{
    if (x != x) return x;
    float sign = 1.0f;
    if (x < 0.0f) { sign = -1.0f; x = -x; }
    float y;
    if (x > 2.414213562373095f) { y = 1.5707963267948966f; x = -1.0f / x; }
    else if (x > 0.4142135623730950f) { y = 0.7853981633974483f; x = (x - 1.0f) / (x + 1.0f); }
    else { y = 0.0f; }
    const float z = x * x;
    float p = 8.05374449538e-2f * z;
    p = p - 1.38776856032e-1f; p = p * z;
    p = p + 1.99777106478e-1f; p = p * z;
    p = p - 3.33329491539e-1f; p = p * z;
    p = p * x;
    p = p + x;
    y = y + p;
    return sign * y;
}

// ---- float3 with HLSL semantics ----------------------------------------------
struct V3 {
    float x, y, z;
};
DEV V3 mk(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
DEV V3 operator+(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
DEV V3 operator-(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
DEV V3 operator-(V3 a) { return mk(-a.x, -a.y, -a.z); }
DEV V3 operator*(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
DEV V3 operator*(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
DEV V3 operator/(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
DEV float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
DEV V3 cross(V3 a, V3 b) { return mk(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
DEV float length(V3 a) { return sqrtf(dot(a, a)); }
// 1.0f / x, bit for bit, in fewer instructions: v_rcp_f32 and one FMA Newton step give the
// correctly rounded reciprocal of every normal x whose reciprocal is normal (biased exponent
// 1..252; checked over all 2^32 bit patterns on gfx950, tools/probe/rcp_exact.hip) -- 3 VALU
// instead of the 11 of the compiler's IEEE division. Zero, denormal, huge, infinite and NaN x
// take that division.
DEV float rcp_ieee(float x)
{
    if (__builtin_expect(((asu(x) >> 23) & 0xFFu) - 1u < 252u, 1)) {
        const float r = __builtin_amdgcn_rcpf(x);
        return __builtin_fmaf(__builtin_fmaf(-x, r, 1.0f), r, r);
    }
    return 1.0f / x;
}
DEV V3 normalize(V3 a) { const float s = rcp_ieee(sqrtf(dot(a, a))); return a * s; }
DEV bool all_zero(V3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
DEV bool any_pos(V3 a) { return a.x > 0.0f || a.y > 0.0f || a.z > 0.0f; }
DEV float comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
DEV V3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
DEV float saturate(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }
DEV float lerp(float a, float b, float t) { return a + t * (b - a); }
DEV float fsign(float x) { return (float)((x > 0.0f) - (x < 0.0f)); }
DEV uint32_t f2u_sat(float f) { if (!(f > 0.0f)) return 0u; if (f >= 4294967296.0f) return 0xFFFFFFFFu; return (uint32_t)f; }

// mul(float4(v, w), float4x3 M), M stored as 3 columns of 4 floats (Scene.cpp:431-444)
DEV V3 mul43(V3 v, float w, const float4* M)
{
    const float4 c0 = M[0], c1 = M[1], c2 = M[2];
    V3 r;
    r.x = v.x * c0.x + v.y * c0.y + v.z * c0.z + w * c0.w;
    r.y = v.x * c1.x + v.y * c1.y + v.z * c1.z + w * c1.w;
    r.z = v.x * c2.x + v.y * c2.y + v.z * c2.z + w * c2.w;
    return r;
}
// mul(float4(v, w), row_major float4x4 M).xyz
DEV V3 mul44(V3 v, float w, const float* M)
{
    V3 r;
    r.x = v.x * M[0] + v.y * M[4] + v.z * M[8] + w * M[12];
    r.y = v.x * M[1] + v.y * M[5] + v.z * M[9] + w * M[13];
    r.z = v.x * M[2] + v.y * M[6] + v.z * M[10] + w * M[14];
    return r;
}

DEV V3 reflect(V3 i, V3 n) { const float d2 = 2.0f * dot(i, n); return mk(i.x - d2 * n.x, i.y - d2 * n.y, i.z - d2 * n.z); }
DEV V3 refract(V3 i, V3 n, float eta)
{
    const float d = dot(i, n);
    const float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return mk(0.0f, 0.0f, 0.0f);
    const float s = eta * d + sqrtf(k);
    return mk(eta * i.x - s * n.x, eta * i.y - s * n.y, eta * i.z - s * n.z);
}

// ---- RNG: xoshiro128** 1.0 seeded by SplitMix64 (Xoshiro.inc.hlsl, Samples.inc.hlsl)
struct Rng {
    uint32_t s0, s1, s2, s3;
};
DEV uint32_t rotl(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }
DEV uint32_t next_u32(Rng& r)
{
    const uint32_t result = rotl(r.s0 * 5u, 7) * 9u;
    const uint32_t t = r.s1 << 9;
    r.s2 ^= r.s0;
    r.s3 ^= r.s1;
    r.s1 ^= r.s2;
    r.s0 ^= r.s3;
    r.s2 ^= t;
    r.s3 = rotl(r.s3, 11);
    return result;
}
DEV float next1(Rng& r) { return (float)(next_u32(r) >> 8) / 16777216.0f; }
DEV uint32_t morton(uint32_t px, uint32_t py)
{
    uint32_t x = px & 0xFFFFu, y = py & 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu; x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u; x = (x | (x << 1)) & 0x55555555u;
    y = (y | (y << 8)) & 0x00FF00FFu; y = (y | (y << 4)) & 0x0F0F0F0Fu;
    y = (y | (y << 2)) & 0x33333333u; y = (y | (y << 1)) & 0x55555555u;
    return x | (y << 1);
}
// SplitMix64 on a native 64-bit register: the reference's 32-bit-pair
// emulation (UInt64.inc.hlsl) is an exact restatement of this arithmetic.
DEV uint64_t splitmix64(uint64_t& state)
{
    uint64_t z = (state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
DEV Rng rng_init(uint32_t px, uint32_t py, uint32_t seed)
{
    uint64_t st = ((uint64_t)seed << 32) | morton(px, py);
    const uint64_t a = splitmix64(st), b = splitmix64(st);
    Rng r;
    r.s0 = (uint32_t)a; r.s1 = (uint32_t)(a >> 32); r.s2 = (uint32_t)b; r.s3 = (uint32_t)(b >> 32);
    return r;
}

// ---- Monte Carlo (MonteCarlo.inc.hlsl) ---------------------------------------
DEV void concentric_disk(float sx, float sy, float* ox, float* oy)
{
    float r, theta;
    const float x = 2.0f * sx - 1.0f, y = 2.0f * sy - 1.0f;
    if (x == 0.0f && y == 0.0f) { *ox = 0.0f; *oy = 0.0f; return; }
    if (x >= -y) {
        if (x > y) { r = x; theta = y > 0.0f ? y / r : 8.0f + y / r; }
        else { r = y; theta = 2.0f - x / r; }
    } else {
        if (x <= y) { r = -x; theta = 4.0f - y / r; }
        else { r = -y; theta = 6.0f + x / r; }
    }
    theta = theta * (kPi / 4.0f);
    float s, c;
    det_sincos(theta, &s, &c);
    *ox = r * c;
    *oy = r * s;
}
DEV V3 cosine_hemisphere(float sx, float sy)
{
    float dx, dy;
    concentric_disk(sx, sy, &dx, &dy);
    return mk(dx, dy, sqrtf(fmaxf(0.0f, 1.0f - (dx * dx + dy * dy))));
}
DEV V3 uniform_sphere(float sx, float sy)
{
    const float z = 1.0f - 2.0f * sx;
    const float r = sqrtf(fmaxf(0.0f, 1.0f - z * z));
    const float phi = 2.0f * kPi * sy;
    float s, c;
    det_sincos(phi, &s, &c);
    return mk(r * c, r * s, z);
}
DEV float uniform_sphere_pdf() { return 1.0f / (4.0f * kPi); }
DEV float power_heuristic(float f, float g) { return (f * f) / (f * f + g * g); }

// ---- OffsetRayOrigin (RayTracingCommon.inc.hlsl:23-36) -----------------------
DEV float offset_axis(float p, float n)
{
    const int32_t of = (int32_t)(256.0f * n);
    const uint32_t moved = asu(p) + (uint32_t)(p < 0.0f ? -of : of);
    return fabsf(p) < (1.0f / 32.0f) ? p + (1.0f / 65536.0f) * n : asf(moved);
}
DEV V3 offset_ray_origin(V3 p, V3 n, V3 d)
{
    n = n * fsign(dot(n, d));
    return mk(offset_axis(p.x, n.x), offset_axis(p.y, n.y), offset_axis(p.z, n.z));
}

}  // namespace dev
}  // namespace dcrt
