/*
 * dcrt_oracle.c -- TEST INFRASTRUCTURE ONLY (see dcrt_oracle.h).
 *
 * Scalar C restatement of the reference's wavefront path tracer shaders.
 * Every function cites the HLSL it follows (paths relative to the reference
 * root, Shaders/ unless stated). Floating point follows the shader source
 * operation by operation, left to right, with no contraction (compile with
 * -ffp-contract=off -fno-fast-math). HLSL intrinsics with implementation-
 * defined precision are given one fixed definition, documented in DESIGN.md:
 *   normalize(v) = v * (1 / sqrt(dot(v, v)));  lerp(a, b, t) = a + t * (b - a);
 *   sin/cos/exp/atan = the Cephes-style float polynomials below;
 *   hardware bilinear filtering = float weights (1 - f, f).
 *
 * Not a product path: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline load this file's shared object.
 */
#include "dcrt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

/* ------------------------------------------------------------------ */
/* constants: Math.inc.hlsl:4-6, RayTracingCommon.inc.hlsl:2-3        */
/* ------------------------------------------------------------------ */
#define O_PI        3.14159265359f
#define O_PI_MUL_2  6.283185307f
#define O_INV_PI    (1.0f / 3.14159265359f)
#define O_SHADOW_EPSILON 1e-3f
#define O_ALPHA_THRESHOLD 0.00052441f       /* BSDFs.inc.hlsl:12 */

static float o_inf(void) { union { uint32_t u; float f; } c; c.u = 0x7f800000u; return c.f; }
static inline uint32_t asuint(float f) { union { uint32_t u; float f; } c; c.f = f; return c.u; }
static inline float asfloat(uint32_t u) { union { uint32_t u; float f; } c; c.u = u; return c.f; }

/* ------------------------------------------------------------------ */
/* Deterministic transcendentals (definition shared with the HIP path) */
/* ------------------------------------------------------------------ */
static float det_reduce_pio2(float x, int* quadrant)
{
    float k = rintf(x * 0.636619772f);
    *quadrant = ((int)k) & 3;
    float r = x - k * 1.5703125f;
    r = r - k * 4.837512969970703125e-4f;
    r = r - k * 7.54978995489188216e-8f;
    return r;
}
static float det_sin_poly(float r)
{
    float z = r * r;
    float y = -1.9515295891e-4f * z;
    y = y + 8.3321608736e-3f;
    y = y * z;
    y = y - 1.6666654611e-1f;
    y = y * z;
    y = y * r;
    return y + r;
}
static float det_cos_poly(float r)
{
    float z = r * r;
    float y = 2.443315711809948e-5f * z;
    y = y - 1.388731625493765e-3f;
    y = y * z;
    y = y + 4.166664568298827e-2f;
    y = y * z;
    y = y * z;
    y = y - 0.5f * z;
    return y + 1.0f;
}
static float det_sinf(float x)
{
    if (!(fabsf(x) <= 1.0e30f)) return x - x;
    int q; float r = det_reduce_pio2(x, &q);
    switch (q) {
    case 0: return det_sin_poly(r);
    case 1: return det_cos_poly(r);
    case 2: return -det_sin_poly(r);
    default: return -det_cos_poly(r);
    }
}
static float det_cosf(float x)
{
    if (!(fabsf(x) <= 1.0e30f)) return x - x;
    int q; float r = det_reduce_pio2(x, &q);
    switch (q) {
    case 0: return det_cos_poly(r);
    case 1: return -det_sin_poly(r);
    case 2: return -det_cos_poly(r);
    default: return det_sin_poly(r);
    }
}
static float det_expf(float x)
{
    if (x != x) return x;
    if (x > 88.72283905f) return o_inf();
    if (x < -103.972084f) return 0.0f;
    float z = floorf(x * 1.44269504088896341f + 0.5f);
    x = x - z * 0.693359375f;
    x = x - z * -2.12194440e-4f;
    int n = (int)z;
    float zz = x * x;
    float y = 1.9875691500e-4f * x;
    y = y + 1.3981999507e-3f; y = y * x;
    y = y + 8.3334519073e-3f; y = y * x;
    y = y + 4.1665795894e-2f; y = y * x;
    y = y + 1.6666665459e-1f; y = y * x;
    y = y + 5.0000001201e-1f;
    y = y * zz;
    y = y + x;
    y = y + 1.0f;
    /* y * 2^n in two exact steps (n in [-150, 128]) */
    int n1 = n / 2;
    int n2 = n - n1;
    y = y * asfloat((uint32_t)(n1 + 127) << 23);
    y = y * asfloat((uint32_t)(n2 + 127) << 23);
    return y;
}
/* Cephes logf restated (same code as det_log in csrc/device/dmath.h) */
static float det_logf(float x)
{
    if (x != x) return x;
    if (x < 0.0f) return asfloat(0x7FC00000u);
    if (x == 0.0f) return -o_inf();
    if (x == o_inf()) return x;
    int e = 0;
    if (x < 1.17549435e-38f) { x = x * 8388608.0f; e = -23; }
    const uint32_t bits = asuint(x);
    e += (int)((bits >> 23) & 0xFFu) - 126;
    float m = asfloat((bits & 0x007FFFFFu) | 0x3F000000u);
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
static float det_atanf(float x)
{
    if (x != x) return x;
    float sign = 1.0f;
    if (x < 0.0f) { sign = -1.0f; x = -x; }
    float y;
    if (x > 2.414213562373095f) { y = 1.5707963267948966f; x = -1.0f / x; }
    else if (x > 0.4142135623730950f) { y = 0.7853981633974483f; x = (x - 1.0f) / (x + 1.0f); }
    else { y = 0.0f; }
    float z = x * x;
    float p = 8.05374449538e-2f * z;
    p = p - 1.38776856032e-1f; p = p * z;
    p = p + 1.99777106478e-1f; p = p * z;
    p = p - 3.33329491539e-1f; p = p * z;
    p = p * x;
    p = p + x;
    y = y + p;
    return sign * y;
}

void oracle_math_eval(int function, const float* x, uint32_t count, float* y)
{
    for (uint32_t i = 0; i < count; ++i) {
        switch (function) {
        case 0: y[i] = det_sinf(x[i]); break;
        case 1: y[i] = det_cosf(x[i]); break;
        case 2: y[i] = det_expf(x[i]); break;
        case 4: y[i] = det_logf(x[i]); break;
        default: y[i] = det_atanf(x[i]); break;
        }
    }
}

/* ------------------------------------------------------------------ */
/* float3 helpers (HLSL vector semantics)                              */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y; } f2;
static inline v3 V3(float x, float y, float z) { v3 r = { x, y, z }; return r; }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vscale(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 vdivs(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 vcross(v3 a, v3 b) { return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
static inline float vlength(v3 a) { return sqrtf(vdot(a, a)); }
static inline v3 vnormalize(v3 a) { float s = 1.0f / sqrtf(vdot(a, a)); return vscale(a, s); }
static inline int vall_zero(v3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
static inline int vany_pos(v3 a) { return a.x > 0.0f || a.y > 0.0f || a.z > 0.0f; }
static inline float vget(v3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
static inline v3 vload(const float* p) { return V3(p[0], p[1], p[2]); }
static inline float saturatef(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }
static inline float lerpf(float a, float b, float t) { return a + t * (b - a); }
static inline float fracf(float x) { return x - floorf(x); }
/* D3D float->uint conversion saturates (NaN -> 0) */
static inline uint32_t f2u_sat(float f) { if (!(f > 0.0f)) return 0u; if (f >= 4294967296.0f) return 0xFFFFFFFFu; return (uint32_t)f; }

/* mul(float4(v, w), float4x3 M) with M column-major (Scene.cpp:431-444) */
static inline v3 mul43(v3 v, float w, const dcrt_float4x3* M)
{
    const float* m = M->m;
    v3 r;
    r.x = v.x * m[0] + v.y * m[1] + v.z * m[2] + w * m[3];
    r.y = v.x * m[4] + v.y * m[5] + v.z * m[6] + w * m[7];
    r.z = v.x * m[8] + v.y * m[9] + v.z * m[10] + w * m[11];
    return r;
}
/* mul(float4(v, w), row_major float4x4 M).xyz */
static inline v3 mul44(v3 v, float w, const float* M)
{
    v3 r;
    r.x = v.x * M[0] + v.y * M[4] + v.z * M[8] + w * M[12];
    r.y = v.x * M[1] + v.y * M[5] + v.z * M[9] + w * M[13];
    r.z = v.x * M[2] + v.y * M[6] + v.z * M[10] + w * M[14];
    return r;
}

/* ------------------------------------------------------------------ */
/* RNG: Xoshiro.inc.hlsl:16-30 (xoshiro128** 1.0), UInt64.inc.hlsl,    */
/*      Samples.inc.hlsl:4-70                                          */
/* ------------------------------------------------------------------ */
static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

uint32_t oracle_rng_next(uint32_t s[4])
{
    const uint32_t result = rotl32(s[0] * 5u, 7) * 9u;
    const uint32_t t = s[1] << 9;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl32(s[3], 11);
    return result;
}

/* Xoshiro.inc.hlsl:35-63 */
void oracle_xoshiro_jump(uint32_t s[4])
{
    static const uint32_t JUMP[4] = { 0x8764000bu, 0xf542d2d3u, 0x6fa035c3u, 0x77f2db5bu };
    uint32_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
    for (int i = 0; i < 4; i++) {
        for (int b = 0; b < 32; b++) {
            if (JUMP[i] & (1u << b)) { s0 ^= s[0]; s1 ^= s[1]; s2 ^= s[2]; s3 ^= s[3]; }
            oracle_rng_next(s);
        }
    }
    s[0] = s0; s[1] = s1; s[2] = s2; s[3] = s3;
}

/* UInt64.inc.hlsl:4-46: 64-bit arithmetic on (lo, hi) pairs */
static void u64_add(const uint32_t a[2], const uint32_t b[2], uint32_t r[2])
{
    uint32_t sumLo = a[0] + b[0];
    uint32_t sumHi = a[1] + b[1];
    uint32_t x = a[0] ^ b[0];
    uint32_t carry = ((x & (~sumLo)) | (a[0] & b[0])) >> 31;
    r[0] = sumLo; r[1] = sumHi + carry;
}
static void u64_shr(const uint32_t v[2], uint32_t n, uint32_t r[2])
{
    uint32_t hi = v[1] >> n;
    uint32_t lo = (v[0] >> n) | (v[1] << (32 - n));
    r[0] = lo; r[1] = hi;
}
static void u32_mul_wide(uint32_t a, uint32_t b, uint32_t r[2])
{
    uint32_t a0 = a & 0xFFFFu, a1 = a >> 16;
    uint32_t b0 = b & 0xFFFFu, b1 = b >> 16;
    uint32_t p11 = a1 * b1, p01 = a0 * b1;
    uint32_t p10 = a1 * b0, p00 = a0 * b0;
    uint32_t middle = p10 + (p00 >> 16) + (p01 & 0xFFFFu);
    r[1] = p11 + (middle >> 16) + (p01 >> 16);
    r[0] = (middle << 16) | (p00 & 0xFFFFu);
}
static void u64_mul(const uint32_t a[2], const uint32_t b[2], uint32_t r[2])
{
    uint32_t m[2];
    u32_mul_wide(a[0], b[0], m);
    m[1] += a[1] * b[0] + a[0] * b[1];
    r[0] = m[0]; r[1] = m[1];
}
/* Samples.inc.hlsl:50-57 */
static void splitmix64_next(uint32_t state[2], uint32_t out[2])
{
    static const uint32_t gamma[2] = { 0x7F4A7C15u, 0x9E3779B9u };
    static const uint32_t m1[2] = { 0x1CE4E5B9u, 0xBF58476Du };
    static const uint32_t m2[2] = { 0x133111EBu, 0x94D049BBu };
    uint32_t z[2], t[2], x[2];
    u64_add(state, gamma, z);
    state[0] = z[0]; state[1] = z[1];
    u64_shr(z, 30, t); x[0] = z[0] ^ t[0]; x[1] = z[1] ^ t[1]; u64_mul(x, m1, z);
    u64_shr(z, 27, t); x[0] = z[0] ^ t[0]; x[1] = z[1] ^ t[1]; u64_mul(x, m2, z);
    u64_shr(z, 31, t); out[0] = z[0] ^ t[0]; out[1] = z[1] ^ t[1];
}
void oracle_splitmix64_pair(uint32_t lo, uint32_t hi, uint32_t out[6])
{
    uint32_t st[2] = { lo, hi }, a[2], b[2];
    splitmix64_next(st, a);
    splitmix64_next(st, b);
    out[0] = a[0]; out[1] = a[1]; out[2] = b[0]; out[3] = b[1]; out[4] = st[0]; out[5] = st[1];
}
/* Samples.inc.hlsl:30-46 */
uint32_t oracle_morton(uint32_t px, uint32_t py)
{
    uint32_t x = px & 0x0000FFFFu, y = py & 0x0000FFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu; x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u; x = (x | (x << 1)) & 0x55555555u;
    y = (y | (y << 8)) & 0x00FF00FFu; y = (y | (y << 4)) & 0x0F0F0F0Fu;
    y = (y | (y << 2)) & 0x33333333u; y = (y | (y << 1)) & 0x55555555u;
    return x | (y << 1);
}
/* Samples.inc.hlsl:59-70 */
void oracle_rng_init(uint32_t px, uint32_t py, uint32_t frame_seed, uint32_t s[4])
{
    uint32_t st[2] = { oracle_morton(px, py), frame_seed }, a[2], b[2];
    splitmix64_next(st, a);
    splitmix64_next(st, b);
    s[0] = a[0]; s[1] = a[1]; s[2] = b[0]; s[3] = b[1];
}
/* Samples.inc.hlsl:4-28 */
static inline float next1d(uint32_t s[4]) { uint32_t bits = oracle_rng_next(s); return (float)(bits >> 8) / (float)(1 << 24); }
static inline f2 next2d(uint32_t s[4]) { f2 r; r.x = next1d(s); r.y = next1d(s); return r; }
static inline v3 next3d(uint32_t s[4]) { v3 r; r.x = next1d(s); r.y = next1d(s); r.z = next1d(s); return r; }

/* ------------------------------------------------------------------ */
/* MonteCarlo.inc.hlsl                                                 */
/* ------------------------------------------------------------------ */
static f2 concentric_sample_disk(f2 sample)   /* :6-46 */
{
    float r, theta;
    f2 s; s.x = 2.0f * sample.x - 1.0f; s.y = 2.0f * sample.y - 1.0f;
    if (s.x == 0.0f && s.y == 0.0f) { f2 z = { 0.0f, 0.0f }; return z; }
    if (s.x >= -s.y) {
        if (s.x > s.y) { r = s.x; if (s.y > 0.0f) theta = s.y / r; else theta = 8.0f + s.y / r; }
        else { r = s.y; theta = 2.0f - s.x / r; }
    } else {
        if (s.x <= s.y) { r = -s.x; theta = 4.0f - s.y / r; }
        else { r = -s.y; theta = 6.0f + s.x / r; }
    }
    theta = theta * (O_PI / 4.0f);
    f2 o; o.x = r * det_cosf(theta); o.y = r * det_sinf(theta);
    return o;
}
static v3 cosine_sample_hemisphere(f2 sample)  /* :48-52 */
{
    f2 s = concentric_sample_disk(sample);
    return V3(s.x, s.y, sqrtf(fmaxf(0.0f, 1.0f - (s.x * s.x + s.y * s.y))));
}
static f2 sample_triangle(f2 sample)            /* :55-59 */
{
    float s = sqrtf(sample.x);
    f2 r; r.x = 1.0f - s; r.y = sample.y * s; return r;
}
static v3 sample_sphere(f2 sample)              /* :61-67 */
{
    float z = 1.0f - 2.0f * sample.x;
    float r = sqrtf(fmaxf(0.0f, 1.0f - z * z));
    float phi = 2.0f * O_PI * sample.y;
    return V3(r * det_cosf(phi), r * det_sinf(phi), z);
}
static inline float uniform_sphere_pdf(void) { return 1.0f / (4.0f * O_PI); }
static inline float power_heuristic(float fPdf, float gPdf)   /* :74-79, nf = ng = 1 */
{
    float f = 1.0f * fPdf, g = 1.0f * gPdf;
    return (f * f) / (f * f + g * g);
}

/* ------------------------------------------------------------------ */
/* RayTracingCommon.inc.hlsl:23-36  OffsetRayOrigin                   */
/* ------------------------------------------------------------------ */
static float offset_component(float p, float n)
{
    int32_t of_i = (int32_t)(256.0f * n);
    int32_t pi = (int32_t)asuint(p);
    uint32_t moved = (uint32_t)pi + (uint32_t)(p < 0.0f ? -of_i : of_i);
    float p_i = asfloat(moved);
    return fabsf(p) < (1.0f / 32.0f) ? p + (1.0f / 65536.0f) * n : p_i;
}
static v3 offset_ray_origin(v3 p, v3 n, v3 d)
{
    float dn = vdot(n, d);
    float sgn = (float)((dn > 0.0f) - (dn < 0.0f));
    n = vscale(n, sgn);
    return V3(offset_component(p.x, n.x), offset_component(p.y, n.y), offset_component(p.z, n.z));
}
void oracle_offset_ray_origin(const float p[3], const float n[3], const float d[3], float out[3])
{
    v3 r = offset_ray_origin(vload(p), vload(n), vload(d));
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}

/* ------------------------------------------------------------------ */
/* Camera: RayTracingCommon.inc.hlsl:38-86                             */
/* ------------------------------------------------------------------ */
static f2 sample_aperture(v3 samples, float apertureRadius, uint32_t bladeCount, f2 vertexPos, float bladeAngle, float baseAngle)
{
    if (bladeCount <= 2) {
        f2 d = concentric_sample_disk((f2){ samples.x, samples.y });
        d.x = d.x * apertureRadius; d.y = d.y * apertureRadius;
        return d;
    }
    f2 uv = sample_triangle((f2){ samples.x, samples.y });
    f2 p; p.x = vertexPos.x * (uv.x + uv.y); p.y = vertexPos.y * uv.x - vertexPos.y * uv.y;
    float n = floorf(samples.z * (float)bladeCount);
    float theta = n * bladeAngle + baseAngle;
    float c = det_cosf(theta), s = det_sinf(theta);
    f2 r; r.x = p.x * c - p.y * s; r.y = p.y * c + p.x * s;
    return r;
}
static void generate_ray(f2 filmSample, v3 apertureSample, const dcrt_frame_params* f, v3* origin, v3* direction)
{
    v3 filmPos = V3(-filmSample.x + 0.5f, filmSample.y - 0.5f, -f->film_distance);
    filmPos.x = filmPos.x * f->film_size[0];
    filmPos.y = filmPos.y * f->film_size[1];
    v3 o = V3(0.0f, 0.0f, 0.0f);
    v3 d = vnormalize(vneg(filmPos));
    if (f->aperture_radius > 0.0f) {
        f2 vp = { f->blade_vertex_pos[0], f->blade_vertex_pos[1] };
        f2 ap = sample_aperture(apertureSample, f->aperture_radius, f->blade_count, vp,
                                O_PI_MUL_2 / (float)f->blade_count, f->aperture_base_angle);
        v3 aperturePos = V3(ap.x, ap.y, 0.0f);
        v3 focusPoint = vscale(d, f->focal_distance / d.z);
        o = aperturePos;
        d = vnormalize(vsub(focusPoint, o));
    }
    *origin = mul44(o, 1.0f, f->camera_transform);
    *direction = mul44(d, 0.0f, f->camera_transform);
}

/* ------------------------------------------------------------------ */
/* RayPrimitiveIntersect.inc.hlsl                                     */
/* ------------------------------------------------------------------ */
static int max_component_index(v3 v)              /* Intrinsics.inc.hlsl:9-14 */
{
    int index = v.x >= v.y ? 0 : 1;
    index = vget(v, index) >= v.z ? index : 2;
    return index;
}
static void ray_permute_shear(v3 dir, int perm[3], v3* shear)   /* BVHAccel.inc.hlsl:72-83 */
{
    perm[2] = max_component_index(V3(fabsf(dir.x), fabsf(dir.y), fabsf(dir.z)));
    perm[0] = perm[2] + 1; perm[0] = perm[0] == 3 ? 0 : perm[0];
    perm[1] = perm[0] + 1; perm[1] = perm[1] == 3 ? 0 : perm[1];
    v3 d = V3(vget(dir, perm[0]), vget(dir, perm[1]), vget(dir, perm[2]));
    float invZ = 1.0f / d.z;
    shear->x = -d.x * invZ;
    shear->y = -d.y * invZ;
    shear->z = invZ;
}
static int tri_watertight(v3 origin, v3 shear, const int perm[3], float tMin, float tMax, v3 v0, v3 v1, v3 v2,
                          float* t, float* u, float* v, int* backface)   /* :8-70 */
{
    *t = 0.0f; *u = 0.0f; *v = 0.0f; *backface = 0;
    v3 v0v1 = vsub(v1, v0), v0v2 = vsub(v2, v0);
    v3 cp = vcross(v0v1, v0v2);
    if (vdot(cp, cp) == 0.0f) return 0;
    v3 a = vsub(v0, origin), b = vsub(v1, origin), c = vsub(v2, origin);
    v3 p0t = V3(vget(a, perm[0]), vget(a, perm[1]), vget(a, perm[2]));
    v3 p1t = V3(vget(b, perm[0]), vget(b, perm[1]), vget(b, perm[2]));
    v3 p2t = V3(vget(c, perm[0]), vget(c, perm[1]), vget(c, perm[2]));
    p0t.x = p0t.x + shear.x * p0t.z; p0t.y = p0t.y + shear.y * p0t.z;
    p1t.x = p1t.x + shear.x * p1t.z; p1t.y = p1t.y + shear.y * p1t.z;
    p2t.x = p2t.x + shear.x * p2t.z; p2t.y = p2t.y + shear.y * p2t.z;
    float e0 = p1t.x * p2t.y - p2t.x * p1t.y;
    float e1 = p2t.x * p0t.y - p0t.x * p2t.y;
    float e2 = p0t.x * p1t.y - p1t.x * p0t.y;
    if ((e0 < 0.0f || e1 < 0.0f || e2 < 0.0f) && (e0 > 0.0f || e1 > 0.0f || e2 > 0.0f)) return 0;
    float det = e0 + e1 + e2;
    p0t.z = p0t.z * shear.z; p1t.z = p1t.z * shear.z; p2t.z = p2t.z * shear.z;
    float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    float invDet = 1.0f / det;
    *t = tScaled * invDet;
    *u = e1 * invDet;
    *v = e2 * invDet;
    float sgn = (float)((shear.z > 0.0f) - (shear.z < 0.0f));
    *backface = (sgn * det) < 0.0f;
    return det != 0.0f && *t >= tMin && *t < tMax;
}
static int tri_moller(v3 origin, v3 direction, float tMin, float tMax, v3 v0, v3 v1, v3 v2,
                      float* t, float* u, float* v, int* backface)   /* :72-103 */
{
    v3 v0v1 = vsub(v1, v0), v0v2 = vsub(v2, v0);
    v3 pvec = vcross(direction, v0v2);
    float det = vdot(v0v1, pvec);
    float invDet = 1.0f / det;
    v3 tvec = vsub(origin, v0);
    *u = vdot(tvec, pvec) * invDet;
    v3 qvec = vcross(tvec, v0v1);
    *v = vdot(direction, qvec) * invDet;
    *t = vdot(v0v2, qvec) * invDet;
    *backface = det > -1e-10f;
    return fabsf(det) >= 1e-10f && *u >= 0.0f && *u <= 1.0f && *v >= 0.0f && *u + *v <= 1.0f && *t >= tMin && *t < tMax;
}
static int ray_aabb(v3 o, v3 invDir, float tMin, float tMax, const float* bmin, const float* bmax)  /* :106-133 */
{
    float tx0 = (bmin[0] - o.x) * invDir.x;
    float tx1 = (bmax[0] - o.x) * invDir.x;
    float t0 = fminf(tx0, tx1);
    float t1 = fmaxf(tx0, tx1);
    float ty0 = (bmin[1] - o.y) * invDir.y;
    float ty1 = (bmax[1] - o.y) * invDir.y;
    t0 = fmaxf(t0, fminf(ty0, ty1));
    t1 = fminf(t1, fmaxf(ty0, ty1));
    float tz0 = (bmin[2] - o.z) * invDir.z;
    float tz1 = (bmax[2] - o.z) * invDir.z;
    t0 = fmaxf(t0, fminf(tz0, tz1));
    t1 = fminf(t1, fmaxf(tz0, tz1));
    return t1 >= t0 && (t0 < tMax && t1 >= tMin);
}

/* ------------------------------------------------------------------ */
/* BVHAccel.inc.hlsl:85-369 two-level traversal                        */
/* ------------------------------------------------------------------ */
typedef struct hit_info { float t, u, v; uint32_t triangleId, instanceIndex; int backface; } hit_info;

#define O_MAX_STACK 256

static int any_hit_shader(const dcrt_flat_scene* sc, uint32_t tri, uint32_t materialOverride, float u, float v,
                          float opacitySample);

/* `opacitySample` is used only with DCRT_FEATURE_ALLOW_ANYHIT (BVHAccel.inc.hlsl:95-101, 182-190). */
static int bvh_intersect(const dcrt_flat_scene* sc, v3 origin, v3 direction, float tMin, float tMaxIn,
                         int anyHit, uint32_t features, float opacitySample, hit_info* hit, uint64_t* nodeVisits,
                         uint64_t* triTests, uint64_t* blasEntries)
{
    uint32_t stack[O_MAX_STACK];
    int count = 0;
    float tMax = tMaxIn;
    const int watertight = (features & DCRT_FEATURE_WATERTIGHT) != 0;
    const int f2b = (features & DCRT_FEATURE_NO_FRONT_TO_BACK) == 0;
    const int allowAnyHit = (features & DCRT_FEATURE_ALLOW_ANYHIT) != 0;
    uint32_t nodeIndex = 0, instanceIndex = 0;
    uint32_t materialOverride = DCRT_INSTANCE_MATERIAL_OVERRIDE_NONE;
    int isBLAS = 0, isOpaque = 0;
    v3 lo = origin, ld = direction;
    const uint32_t instanceCount = sc->instance_count;
    for (;;) {
        if (nodeVisits) ++*nodeVisits;
        int popNode = 0;
        const dcrt_bvh_node* node = &sc->bvh_nodes[nodeIndex];
        v3 invDir = V3(1.0f / ld.x, 1.0f / ld.y, 1.0f / ld.z);
        if (ray_aabb(lo, invDir, tMin, tMax, node->bbox_min, node->bbox_max)) {
            int hasBLAS = (node->misc & 0x4u) != 0;
            uint32_t primCountOrInstance = (node->misc >> 3) & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT;
            if (hasBLAS) {
                const dcrt_float4x3* inv = &sc->instance_transforms[instanceCount + primCountOrInstance];
                lo = mul43(origin, 1.0f, inv);
                ld = mul43(direction, 0.0f, inv);
                isBLAS = 1;
                instanceIndex = primCountOrInstance;
                nodeIndex = node->right_child_or_prim_index;
                isOpaque = (sc->instance_flags[primCountOrInstance] & DCRT_INSTANCE_FLAG_OPAQUE) != 0;   /* :136-139 */
                materialOverride = sc->instance_material_overrides[primCountOrInstance];
                if (blasEntries) ++*blasEntries;
            } else if (primCountOrInstance == 0) {
                uint32_t axis = node->misc & 0x3u;
                int neg = 0;
                if (f2b) neg = axis == 0 ? ld.x < 0.0f : (axis == 1 ? ld.y < 0.0f : ld.z < 0.0f);
                uint32_t push = neg ? nodeIndex + 1 : node->right_child_or_prim_index;
                nodeIndex = neg ? node->right_child_or_prim_index : nodeIndex + 1;
                if (count < O_MAX_STACK) stack[count++] = (push & 0x7FFFFFFFu) | (isBLAS ? 0x80000000u : 0u);
            } else {
                int perm[3]; v3 shear;
                if (watertight) ray_permute_shear(ld, perm, &shear);
                uint32_t primBegin = node->right_child_or_prim_index;
                uint32_t primEnd = primBegin + primCountOrInstance;
                for (uint32_t p = primBegin; p < primEnd; ++p) {
                    if (triTests) ++*triTests;
                    v3 v0 = vload(sc->vertices[sc->triangles[p * 3]].position);
                    v3 v1 = vload(sc->vertices[sc->triangles[p * 3 + 1]].position);
                    v3 v2 = vload(sc->vertices[sc->triangles[p * 3 + 2]].position);
                    float t, u, v; int bf;
                    int h = watertight ? tri_watertight(lo, shear, perm, tMin, tMax, v0, v1, v2, &t, &u, &v, &bf)
                                       : tri_moller(lo, ld, tMin, tMax, v0, v1, v2, &t, &u, &v, &bf);
                    if (h && allowAnyHit && !isOpaque)
                        h = any_hit_shader(sc, p, materialOverride, u, v, opacitySample);
                    if (h) {
                        if (anyHit) return 1;
                        tMax = t;
                        hit->t = t; hit->u = u; hit->v = v; hit->backface = bf;
                        hit->triangleId = p; hit->instanceIndex = instanceIndex;
                    }
                }
                popNode = 1;
            }
        } else {
            popNode = 1;
        }
        if (popNode) {
            int lastIsBLAS = isBLAS;
            if (count == 0) break;
            uint32_t packed = stack[--count];
            nodeIndex = packed & 0x7FFFFFFFu;
            isBLAS = (packed & 0x80000000u) != 0;
            if (lastIsBLAS != isBLAS) { lo = origin; ld = direction; }
        }
    }
    if (anyHit) return 0;
    return !isinf(tMax);
}

/* ------------------------------------------------------------------ */
/* Texture emulation (D3D12 SampleLevel, LOD 0, linear filter)         */
/* ------------------------------------------------------------------ */
static float lut_texel(const uint16_t* t, int x, int y, int w) { return (float)t[y * w + x] / 65535.0f; }
static float bilinear_u16_clamp(const uint16_t* tex, int w, int h, float u, float v)
{
    float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float fx = x - fx0, fy = y - fy0;
    int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
    x0 = x0 < 0 ? 0 : (x0 > w - 1 ? w - 1 : x0); x1 = x1 < 0 ? 0 : (x1 > w - 1 ? w - 1 : x1);
    y0 = y0 < 0 ? 0 : (y0 > h - 1 ? h - 1 : y0); y1 = y1 < 0 ? 0 : (y1 > h - 1 ? h - 1 : y1);
    float a = lut_texel(tex, x0, y0, w) * (1.0f - fx) + lut_texel(tex, x1, y0, w) * fx;
    float b = lut_texel(tex, x0, y1, w) * (1.0f - fx) + lut_texel(tex, x1, y1, w) * fx;
    return a * (1.0f - fy) + b * fy;
}
static int array_slice(float fslice, int slices)
{
    float r = floorf(fslice + 0.5f);
    if (!(r > 0.0f)) return 0;
    if (r > (float)(slices - 1)) return slices - 1;
    return (int)r;
}
/* BxDFTextures.inc.hlsl:7-21 */
static inline float texcoord_remap(uint32_t dim, float u) { return u * ((float)(dim - 1) / (float)dim) + 0.5f / (float)dim; }
/* BxDFTextures.inc.hlsl:33-40 */
static float sample_array_linear(const uint16_t* tex, uint32_t w, uint32_t h, uint32_t slices, v3 uvw, uint32_t dz, uint32_t sliceOffset)
{
    float slicePos = uvw.z * ((float)dz - 1.0f);
    float fraction = fracf(slicePos);
    float u = texcoord_remap(w, uvw.x), v = texcoord_remap(h, uvw.y);
    uint32_t s0 = (uint32_t)(int32_t)slicePos + sliceOffset;
    uint32_t s1 = (uint32_t)(int32_t)slicePos + 1u + sliceOffset;
    int i0 = array_slice((float)s0, (int)slices), i1 = array_slice((float)s1, (int)slices);
    float v0 = bilinear_u16_clamp(tex + (size_t)i0 * w * h, (int)w, (int)h, u, v);
    float v1 = bilinear_u16_clamp(tex + (size_t)i1 * w * h, (int)w, (int)h, u, v);
    return lerpf(v0, v1, fraction);
}
static const dcrt_bxdf_luts* g_luts;   /* set per render call (single scene at a time) */

static float sample_brdf_texture(float cosThetaO, float alpha)               /* :47-51 */
{
    return bilinear_u16_clamp(g_luts->brdf, 32, 32, texcoord_remap(32, cosThetaO), texcoord_remap(32, alpha));
}
static float sample_brdf_average_texture(float alpha)                        /* :53-56 */
{
    float u = texcoord_remap(32, alpha);
    return bilinear_u16_clamp(g_luts->brdf_avg, 32, 1, u, u);
}
static float sample_brdf_dielectric_texture(float cosThetaO, float alpha, float eta, int isEntering)  /* :58-64 */
{
    uint32_t sliceOffset = isEntering ? 16u : 0u;
    float w = (eta - 1.0f) / 2.0f;
    return sample_array_linear(g_luts->brdf_dielectric, 32, 16, 32, V3(cosThetaO, alpha, w), 16, sliceOffset);
}
static float sample_brdf_dielectric_average_texture(float alpha, float eta, int isEntering)  /* :66-72 */
{
    uint32_t sliceOffset = isEntering ? 1u : 0u;
    float v = (eta - 1.0f) / 2.0f;
    return sample_array_linear(g_luts->brdf_dielectric_avg, 16, 16, 2, V3(alpha, v, 0.0f), 1, sliceOffset);
}
static float sample_bsdf_texture(float cosThetaO, float alpha, float eta, int isEntering)    /* :74-80 */
{
    uint32_t sliceOffset = isEntering ? 16u : 0u;
    float w = (eta - 1.0f) / 2.0f;
    return sample_array_linear(g_luts->bsdf, 32, 16, 32, V3(cosThetaO, alpha, w), 16, sliceOffset);
}
static float sample_bsdf_average_texture(float alpha, float eta, int isEntering)            /* :82-88 */
{
    uint32_t sliceOffset = isEntering ? 1u : 0u;
    float v = (eta - 1.0f) / 2.0f;
    return sample_array_linear(g_luts->bsdf_avg, 16, 16, 2, V3(alpha, v, 0.0f), 1, sliceOffset);
}

/* sRGB texture sampling (HitShader.inc.hlsl:64-68): decode per texel, then filter */
static float g_srgb_table[256];
static int g_srgb_ready;
static void init_srgb(void)
{
    if (g_srgb_ready) return;
    for (int i = 0; i < 256; ++i) {
        double c = i / 255.0;
        g_srgb_table[i] = (float)(c <= 0.04045 ? c / 12.92 : pow((c + 0.055) / 1.055, 2.4));
    }
    g_srgb_ready = 1;
}
static int wrap_index(int i, int n) { int r = i % n; return r < 0 ? r + n : r; }
static void texel_rgba(const dcrt_texture* t, int x, int y, float out[4])
{
    if (t->format == DCRT_TEXTURE_FORMAT_R8_UNORM) {
        float v = (float)t->pixels[(size_t)y * t->width + x] / 255.0f;
        out[0] = v; out[1] = 0.0f; out[2] = 0.0f; out[3] = 1.0f;
    } else {
        const uint8_t* p = t->pixels + ((size_t)y * t->width + x) * 4;
        out[0] = g_srgb_table[p[0]]; out[1] = g_srgb_table[p[1]]; out[2] = g_srgb_table[p[2]];
        out[3] = (float)p[3] / 255.0f;
    }
}
static void sample_texture_wrap(const dcrt_texture* t, float u, float v, float out[4])
{
    int w = (int)t->width, h = (int)t->height;
    float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float fx = x - fx0, fy = y - fy0;
    int x0 = wrap_index((int)fx0, w), x1 = wrap_index((int)fx0 + 1, w);
    int y0 = wrap_index((int)fy0, h), y1 = wrap_index((int)fy0 + 1, h);
    float a[4], b[4], c[4], d[4];
    texel_rgba(t, x0, y0, a); texel_rgba(t, x1, y0, b); texel_rgba(t, x0, y1, c); texel_rgba(t, x1, y1, d);
    for (int i = 0; i < 4; ++i) {
        float top = a[i] * (1.0f - fx) + b[i] * fx;
        float bot = c[i] * (1.0f - fx) + d[i] * fx;
        out[i] = top * (1.0f - fy) + bot * fy;
    }
}
/* AnyHitShader (HitShader.inc.hlsl:86-113): accept when opacitySample < opacity. */
static f2 bary2(const float* p0, const float* p1, const float* p2, float u, float v);
static int any_hit_shader(const dcrt_flat_scene* sc, uint32_t tri, uint32_t materialOverride, float u, float v,
                          float opacitySample)
{
    const uint32_t mid = materialOverride != DCRT_INSTANCE_MATERIAL_OVERRIDE_NONE ? materialOverride : sc->material_ids[tri];
    const dcrt_material* m = &sc->materials[mid];
    float opacity = m->opacity;
    if (m->opacity_texture_index != -1) {
        f2 tc = bary2(sc->vertices[sc->triangles[tri * 3]].texcoord, sc->vertices[sc->triangles[tri * 3 + 1]].texcoord,
                      sc->vertices[sc->triangles[tri * 3 + 2]].texcoord, u, v);
        tc.x = tc.x * m->tex_tiling[0];
        tc.y = tc.y * m->tex_tiling[1];
        float rgba[4];
        sample_texture_wrap(&sc->textures[m->opacity_texture_index], tc.x, tc.y, rgba);
        opacity = opacity * rgba[0];
    }
    return opacitySample < opacity;
}

/* TextureCube<float3>.SampleLevel(clamp, dir, 0): D3D face selection, bilinear within the face */
static v3 sample_env_cube(const dcrt_flat_scene* sc, v3 d)
{
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int face; float sc_, tc, ma;
    if (ax >= ay && ax >= az) { ma = ax; if (d.x >= 0.0f) { face = 0; sc_ = -d.z; tc = -d.y; } else { face = 1; sc_ = d.z; tc = -d.y; } }
    else if (ay >= az) { ma = ay; if (d.y >= 0.0f) { face = 2; sc_ = d.x; tc = d.z; } else { face = 3; sc_ = d.x; tc = -d.z; } }
    else { ma = az; if (d.z >= 0.0f) { face = 4; sc_ = d.x; tc = -d.y; } else { face = 5; sc_ = -d.x; tc = -d.y; } }
    float u = (sc_ / ma + 1.0f) * 0.5f, v = (tc / ma + 1.0f) * 0.5f;
    int n = (int)sc->env_cube_size;
    float x = u * (float)n - 0.5f, y = v * (float)n - 0.5f;
    float fx0 = floorf(x), fy0 = floorf(y);
    float fx = x - fx0, fy = y - fy0;
    int x0 = (int)fx0, y0 = (int)fy0, x1 = x0 + 1, y1 = y0 + 1;
    x0 = x0 < 0 ? 0 : (x0 > n - 1 ? n - 1 : x0); x1 = x1 < 0 ? 0 : (x1 > n - 1 ? n - 1 : x1);
    y0 = y0 < 0 ? 0 : (y0 > n - 1 ? n - 1 : y0); y1 = y1 < 0 ? 0 : (y1 > n - 1 ? n - 1 : y1);
    const float* base = sc->env_cube_rgb + (size_t)face * n * n * 3;
    float out[3];
    for (int i = 0; i < 3; ++i) {
        float a = base[((size_t)y0 * n + x0) * 3 + i], b = base[((size_t)y0 * n + x1) * 3 + i];
        float c = base[((size_t)y1 * n + x0) * 3 + i], e = base[((size_t)y1 * n + x1) * 3 + i];
        float top = a * (1.0f - fx) + b * fx;
        float bot = c * (1.0f - fx) + e * fx;
        out[i] = top * (1.0f - fy) + bot * fy;
    }
    return V3(out[0], out[1], out[2]);
}

/* ------------------------------------------------------------------ */
/* Intersection + HitShader: HitShader.inc.hlsl:14-84,                 */
/* RayTracingCommon.inc.hlsl:88-116                                    */
/* ------------------------------------------------------------------ */
typedef struct isect {
    v3 albedo; float alpha; v3 position, normal, tangent, geometryNormal, ior;
    int isTwoSided, backface, multiscattering;
    uint32_t internalScatteringMode, materialType, lightIndex, triangleIndex;
} isect;

static v3 bary3(v3 p0, v3 p1, v3 p2, float u, float v)   /* Math.inc.hlsl:35-43 */
{
    v3 r1 = vsub(p1, p0), r2 = vsub(p2, p0);
    r1 = vscale(r1, u); r2 = vscale(r2, v);
    r1 = vadd(r1, p0); r1 = vadd(r1, r2);
    return r1;
}
static f2 bary2(const float* p0, const float* p1, const float* p2, float u, float v)  /* Math.inc.hlsl:23-33 */
{
    f2 r1 = { p1[0] - p0[0], p1[1] - p0[1] }, r2 = { p2[0] - p0[0], p2[1] - p0[1] };
    r1.x = r1.x * u; r1.y = r1.y * u; r2.x = r2.x * v; r2.y = r2.y * v;
    r1.x = r1.x + p0[0]; r1.y = r1.y + p0[1];
    r1.x = r1.x + r2.x; r1.y = r1.y + r2.y;
    return r1;
}

static void hit_to_intersection(const dcrt_flat_scene* sc, const hit_info* h, isect* it)
{
    const uint32_t inst = h->instanceIndex, tri = h->triangleId;
    it->lightIndex = sc->instance_light_indices[inst];
    it->triangleIndex = tri;
    const uint32_t materialOverride = sc->instance_material_overrides[inst];
    const dcrt_vertex* V0 = &sc->vertices[sc->triangles[tri * 3]];
    const dcrt_vertex* V1 = &sc->vertices[sc->triangles[tri * 3 + 1]];
    const dcrt_vertex* V2 = &sc->vertices[sc->triangles[tri * 3 + 2]];
    const float u = h->u, v = h->v;
    /* HitShader */
    it->position = bary3(vload(V0->position), vload(V1->position), vload(V2->position), u, v);
    it->normal = vnormalize(bary3(vload(V0->normal), vload(V1->normal), vload(V2->normal), u, v));
    v3 tangent = bary3(vload(V0->tangent), vload(V1->tangent), vload(V2->tangent), u, v);
    float tangentLength = vlength(tangent);
    if (tangentLength >= 0.000001f) {
        tangent = vsub(tangent, vscale(it->normal, vdot(tangent, it->normal)));
        tangentLength = vlength(tangent);
    }
    if (tangentLength < 0.000001f) {
        tangent = vcross(it->normal, V3(0.0f, 1.0f, 0.0f));
        tangentLength = vlength(tangent);
        tangent = tangentLength >= 0.000001f ? tangent : V3(1.0f, 0.0f, 0.0f);
    }
    it->tangent = vdivs(tangent, tangentLength);
    v3 v0v1 = vsub(vload(V1->position), vload(V0->position));
    v3 v0v2 = vsub(vload(V2->position), vload(V0->position));
    it->geometryNormal = vnormalize(vcross(v0v2, v0v1));
    const uint32_t materialId = materialOverride != DCRT_INSTANCE_MATERIAL_OVERRIDE_NONE ? materialOverride : sc->material_ids[tri];
    const dcrt_material* m = &sc->materials[materialId];
    f2 tc = bary2(V0->texcoord, V1->texcoord, V2->texcoord, u, v);
    tc.x = tc.x * m->tex_tiling[0]; tc.y = tc.y * m->tex_tiling[1];
    v3 albedo = vload(m->albedo);
    if (m->albedo_texture_index != -1) {
        float rgba[4];
        sample_texture_wrap(&sc->textures[m->albedo_texture_index], tc.x, tc.y, rgba);
        albedo = vmul(albedo, V3(rgba[0], rgba[1], rgba[2]));
    }
    float checker = ((f2u_sat(tc.x * 2.0f) + f2u_sat(tc.y * 2.0f)) & 0x1u) != 0 ? 1.0f : 0.0f;
    float roughness = m->roughness;
    roughness = roughness * ((m->flags & DCRT_MATERIAL_FLAG_ROUGHNESS_TEXTURE) != 0 ? checker : 1.0f);
    it->albedo = albedo;
    it->alpha = roughness * roughness;
    it->ior = vload(m->ior);
    it->materialType = m->flags & DCRT_MATERIAL_FLAG_TYPE_MASK;
    it->isTwoSided = (m->flags & DCRT_MATERIAL_FLAG_IS_TWOSIDED) != 0;
    it->multiscattering = (m->flags & DCRT_MATERIAL_FLAG_MULTISCATTERING) != 0;
    it->internalScatteringMode = (m->flags & DCRT_MATERIAL_FLAG_INTERNAL_SCATTERING_MASK) >> DCRT_MATERIAL_FLAG_INTERNAL_SCATTERING_SHIFT;
    it->backface = h->backface;
    /* back to RayTracingCommon.inc.hlsl:112-115 */
    const dcrt_float4x3* M = &sc->instance_transforms[inst];
    it->position = mul43(it->position, 1.0f, M);
    it->normal = vnormalize(mul43(it->normal, 0.0f, M));
    it->geometryNormal = vnormalize(mul43(it->geometryNormal, 0.0f, M));
    it->tangent = vnormalize(mul43(it->tangent, 0.0f, M));
}

/* ------------------------------------------------------------------ */
/* Lights: Light.inc.hlsl, RayTracingCommon.inc.hlsl:124-225           */
/* ------------------------------------------------------------------ */
static inline uint32_t light_tri_offset(const dcrt_light* l) { return asuint(l->position_or_triangle_range[0]); }
static inline uint32_t light_tri_count(const dcrt_light* l) { return asuint(l->position_or_triangle_range[1]); }
static inline uint32_t light_instance(const dcrt_light* l) { return asuint(l->position_or_triangle_range[2]); }

typedef struct light_sample { v3 radiance, wi; float pdf, distance; int isDeltaLight; } light_sample;

static v3 tri_pos(const dcrt_flat_scene* sc, uint32_t tri, int k) { return vload(sc->vertices[sc->triangles[tri * 3 + k]].position); }

static light_sample sample_light_direct(const dcrt_flat_scene* sc, v3 p, uint32_t lightCount, uint32_t s[4])
{
    light_sample r;
    memset(&r, 0, sizeof(r));
    float lightSelectionSample = next1d(s);
    uint32_t lightIndex = (uint32_t)floorf(lightSelectionSample * (float)lightCount);
    const dcrt_light* light = &sc->lights[lightIndex];
    r.isDeltaLight = 0;
    if (light->flags & DCRT_LIGHT_FLAGS_POINT_LIGHT) {                    /* Light.inc.hlsl:4-12 */
        v3 lp = vload(light->position_or_triangle_range);
        r.wi = vsub(lp, p);
        r.distance = vlength(r.wi);
        r.wi = vdivs(r.wi, r.distance);
        r.radiance = vdivs(vload(light->radiance), r.distance * r.distance);
        r.pdf = 1.0f;
        r.isDeltaLight = 1;
    } else if (light->flags & DCRT_LIGHT_FLAGS_DIRECTIONAL_LIGHT) {       /* :14-20 */
        r.wi = vneg(vload(light->position_or_triangle_range));
        r.distance = o_inf();
        r.radiance = vload(light->radiance);
        r.pdf = 1.0f;
        r.isDeltaLight = 1;
    } else if (light->flags & DCRT_LIGHT_FLAGS_MESH_LIGHT) {
        float triangleSelectionSample = next1d(s);
        f2 triangleSample = next2d(s);
        float ftri = (float)light_tri_offset(light) + floorf(triangleSelectionSample * (float)light_tri_count(light));
        uint32_t triangleIndex = (uint32_t)ftri;
        v3 v0 = tri_pos(sc, triangleIndex, 0), v1 = tri_pos(sc, triangleIndex, 1), v2 = tri_pos(sc, triangleIndex, 2);
        const dcrt_float4x3* M = &sc->instance_transforms[light_instance(light)];
        /* TriangleLight_Sample, Light.inc.hlsl:45-73 */
        v3 vws0 = mul43(v0, 1.0f, M), vws1 = mul43(v1, 1.0f, M), vws2 = mul43(v2, 1.0f, M);
        float surfaceArea = vlength(vcross(vsub(vws2, vws0), vsub(vws1, vws0))) * 0.5f;
        f2 b = sample_triangle(triangleSample);
        v3 samplePos = bary3(v0, v1, v2, b.x, b.y);
        v3 v0v1 = vsub(v1, v0), v0v2 = vsub(v2, v0);
        v3 normal = vnormalize(vcross(v0v2, v0v1));
        float pdf = surfaceArea >= 1e-6f ? 1.0f / (surfaceArea * 0.5f) : 0.0f;
        samplePos = mul43(samplePos, 1.0f, M);
        normal = vnormalize(mul43(normal, 0.0f, M));
        r.wi = vsub(samplePos, p);
        r.distance = vlength(r.wi);
        r.wi = vdivs(r.wi, r.distance);
        float WIdotN = -vdot(r.wi, normal);
        pdf = pdf * (r.distance * r.distance / WIdotN);
        r.radiance = (WIdotN > 0.0f && pdf > 0.0f) ? vload(light->radiance) : V3(0.0f, 0.0f, 0.0f);
        r.pdf = WIdotN > 0.0f ? pdf : 0.0f;
        r.pdf = r.pdf / (float)light_tri_count(light);
    } else if (light->flags & DCRT_LIGHT_FLAGS_ENVIRONMENT_LIGHT) {       /* :94-104 */
        f2 samples = next2d(s);
        r.wi = sample_sphere(samples);
        r.pdf = uniform_sphere_pdf();
        r.radiance = sc->env_cube_rgb ? vmul(sample_env_cube(sc, r.wi), vload(light->radiance)) : vload(light->radiance);
        r.distance = o_inf();
    }
    r.pdf = r.pdf / (float)lightCount;
    if (r.distance != o_inf()) r.distance = r.distance * (1.0f - O_SHADOW_EPSILON);
    return r;
}

static void evaluate_light_direct(const dcrt_flat_scene* sc, uint32_t lightIndex, uint32_t triangleIndex, v3 normal, v3 wi,
                                  float distance, uint32_t lightCount, v3* radiance, float* pdf)
{
    *radiance = V3(0.0f, 0.0f, 0.0f);
    *pdf = 0.0f;
    const dcrt_light* light = &sc->lights[lightIndex];
    if (light->flags & DCRT_LIGHT_FLAGS_MESH_LIGHT) {
        v3 v0 = tri_pos(sc, triangleIndex, 0), v1 = tri_pos(sc, triangleIndex, 1), v2 = tri_pos(sc, triangleIndex, 2);
        const dcrt_float4x3* M = &sc->instance_transforms[light_instance(light)];
        /* TriangleLight_EvaluateWithPDF, Light.inc.hlsl:27-43 */
        v0 = mul43(v0, 1.0f, M); v1 = mul43(v1, 1.0f, M); v2 = mul43(v2, 1.0f, M);
        v3 v0v1 = vsub(v1, v0), v0v2 = vsub(v2, v0);
        float surfaceArea = vlength(vcross(v0v2, v0v1));
        float p = surfaceArea >= 1e-6f ? 1.0f / (surfaceArea * 0.5f) : 0.0f;
        float WIdotN = -vdot(wi, normal);
        *radiance = WIdotN > 0.0f ? vload(light->radiance) : V3(0.0f, 0.0f, 0.0f);
        p = p * (WIdotN > 0.0f ? distance * distance / vdot(vneg(wi), normal) : 0.0f);
        *pdf = p / (float)light_tri_count(light);
    } else if (light->flags & DCRT_LIGHT_FLAGS_ENVIRONMENT_LIGHT) {
        *radiance = sc->env_cube_rgb ? vmul(sample_env_cube(sc, wi), vload(light->radiance)) : vload(light->radiance);
        *pdf = uniform_sphere_pdf();
    }
    *pdf = *pdf / (float)lightCount;
}

/* ------------------------------------------------------------------ */
/* BxDFs                                                               */
/* ------------------------------------------------------------------ */
typedef struct lctx { v3 H; float WOdotH; int isInverted; } lctx;   /* LightingContext.inc.hlsl */

static void lctx_calc_h(v3 wo, v3 wi, lctx* c)
{
    c->H = vadd(wi, wo);
    c->H = vall_zero(c->H) ? V3(0.0f, 0.0f, 0.0f) : vnormalize(c->H);
    c->WOdotH = vdot(c->H, wo);
}
static void lctx_assign_h(v3 wo, v3 h, lctx* c) { c->H = h; c->WOdotH = vdot(h, wo); }

static v3 reflect3(v3 i, v3 n) { float d = vdot(i, n); float d2 = 2.0f * d; return V3(i.x - d2 * n.x, i.y - d2 * n.y, i.z - d2 * n.z); }
static v3 refract3(v3 i, v3 n, float eta)
{
    float d = vdot(i, n);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return V3(0.0f, 0.0f, 0.0f);
    float s = eta * d + sqrtf(k);
    return V3(eta * i.x - s * n.x, eta * i.y - s * n.y, eta * i.z - s * n.z);
}

/* Fresnel.inc.hlsl:4-63 */
static float fresnel_dielectric(float cosThetaI, float etaO, float etaI)
{
    cosThetaI = fminf(fmaxf(cosThetaI, -1.0f), 1.0f);
    if (cosThetaI < 0.0f) { float t = etaO; etaO = etaI; etaI = t; cosThetaI = -cosThetaI; }
    float sinThetaI = sqrtf(1.0f - cosThetaI * cosThetaI);
    float sinThetaT = etaO / etaI * sinThetaI;
    if (sinThetaT >= 1.0f) return 1.0f;
    float cosThetaT = sqrtf(1.0f - sinThetaT * sinThetaT);
    float Rparl = ((etaI * cosThetaI) - (etaO * cosThetaT)) / ((etaI * cosThetaI) + (etaO * cosThetaT));
    float Rperp = ((etaO * cosThetaI) - (etaI * cosThetaT)) / ((etaO * cosThetaI) + (etaI * cosThetaT));
    return (Rparl * Rparl + Rperp * Rperp) * 0.5f;
}
static float fresnel_conductor1(float cosThetaI, float etaO, float etaI, float k)
{
    cosThetaI = fminf(fmaxf(cosThetaI, -1.0f), 1.0f);
    float eta = etaI / etaO;
    float etak = k / etaO;
    float cosThetaI2 = cosThetaI * cosThetaI;
    float sinThetaI2 = 1.0f - cosThetaI2;
    float eta2 = eta * eta;
    float etak2 = etak * etak;
    float t0 = eta2 - etak2 - sinThetaI2;
    float a2plusb2 = sqrtf(fmaxf(0.0f, t0 * t0 + 4.0f * eta2 * etak2));
    float t1 = a2plusb2 + cosThetaI2;
    float a = sqrtf(fmaxf(0.0f, 0.5f * (a2plusb2 + t0)));
    float t2 = 2.0f * cosThetaI * a;
    float Rs = (t1 - t2) / (t1 + t2);
    float t3 = cosThetaI2 * a2plusb2 + sinThetaI2 * sinThetaI2;
    float t4 = t2 * sinThetaI2;
    float Rp = Rs * (t3 - t4) / (t3 + t4);
    return 0.5f * (Rp + Rs);
}
static v3 fresnel_conductor(float cosThetaI, v3 etaI, v3 k)    /* etaO = 1 */
{
    return V3(fresnel_conductor1(cosThetaI, 1.0f, etaI.x, k.x), fresnel_conductor1(cosThetaI, 1.0f, etaI.y, k.y),
              fresnel_conductor1(cosThetaI, 1.0f, etaI.z, k.z));
}

/* CookTorranceBSDF.inc.hlsl */
static float ggx_g1(float alpha2, v3 m, v3 w)                             /* :13-23 */
{
    if (vdot(w, m) * w.z <= 0.0f) return 0.0f;
    float NdotW = fabsf(w.z);
    float denominator = sqrtf(alpha2 + (1.0f - alpha2) * NdotW * NdotW) + NdotW;
    return 2.0f * NdotW / denominator;
}
static float ggx_g(v3 wi, v3 wo, v3 m, float alpha)                      /* :25-29 */
{
    float alpha2 = alpha * alpha;
    return ggx_g1(alpha2, m, wi) * ggx_g1(alpha2, m, wo);
}
static v3 sample_ggx_ndf(f2 sample, float alpha)                          /* :35-42 */
{
    float theta = det_atanf(alpha * sqrtf(sample.x / (1.0f - sample.x)));
    float phi = 2.0f * O_PI * sample.y;
    float s = det_sinf(theta);
    return V3(det_cosf(phi) * s, det_sinf(phi) * s, det_cosf(theta));
}
static v3 sample_ggx_vndf(v3 wo, f2 sample, float alpha)                  /* :45-67 */
{
    float U1 = sample.x, U2 = sample.y;
    v3 Vh = vnormalize(V3(alpha * wo.x, alpha * wo.y, wo.z));
    float lensq = Vh.x * Vh.x + Vh.y * Vh.y;
    v3 T1;
    if (lensq > 0.0f) { float sl = sqrtf(lensq); T1 = V3(-Vh.y / sl, Vh.x / sl, 0.0f / sl); }
    else T1 = V3(1.0f, 0.0f, 0.0f);
    v3 T2 = vcross(Vh, T1);
    float r = sqrtf(U1);
    float phi = 2.0f * O_PI * U2;
    float t1 = r * det_cosf(phi);
    float t2 = r * det_sinf(phi);
    float s = 0.5f * (1.0f + Vh.z);
    t2 = (1.0f - s) * sqrtf(1.0f - t1 * t1) + s * t2;
    v3 Nh = vadd(vadd(vscale(T1, t1), vscale(T2, t2)), vscale(Vh, sqrtf(fmaxf(0.0f, 1.0f - t1 * t1 - t2 * t2))));
    return vnormalize(V3(alpha * Nh.x, alpha * Nh.y, fmaxf(0.0f, Nh.z)));
}
static float ggx_d(v3 m, float alpha)                                     /* :69-77 */
{
    float alpha2 = alpha * alpha;
    float NdotM = m.z;
    float NdotM2 = NdotM * NdotM;
    float factor = NdotM2 * (alpha2 - 1.0f) + 1.0f;
    float denominator = factor * factor * O_PI;
    return alpha2 / denominator;
}
static int g_vndf = 1;   /* GGX_SAMPLE_VNDF variant of the current call */
static float ggx_d_pdf(v3 wo, v3 m, float alpha)                          /* :79-86 */
{
    if (g_vndf) return ggx_d(m, alpha) * ggx_g1(alpha * alpha, m, wo) * fmaxf(0.0f, vdot(wo, m)) / wo.z;
    return ggx_d(m, alpha) * fabsf(m.z);
}
static v3 sample_ggx(v3 wo, f2 sample, float alpha)                       /* :98-105 */
{
    return g_vndf ? sample_ggx_vndf(wo, sample, alpha) : sample_ggx_ndf(sample, alpha);
}
static float ct_brdf(v3 wi, v3 wo, float alpha, const lctx* c)            /* :111-124 */
{
    if (wi.z <= 0.0f || wo.z <= 0.0f || c->WOdotH <= 0.0f) return 0.0f;
    v3 m = c->H;
    if (vall_zero(m)) return 0.0f;
    return ggx_d(m, alpha) * ggx_g(wi, wo, m, alpha) / (4.0f * wi.z * wo.z);
}
static float ct_brdf_pdf(v3 wi, v3 wo, float alpha, const lctx* c)        /* :126-137 */
{
    if (wi.z <= 0.0f || wo.z <= 0.0f || c->WOdotH <= 0.0f) return 0.0f;
    float pdf = ggx_d_pdf(wo, c->H, alpha);
    return pdf / (4.0f * c->WOdotH);
}
static void ct_brdf_sample(v3 wo, f2 sample, float alpha, v3* wi, lctx* c) /* :139-146 */
{
    v3 m = sample_ggx(wo, sample, alpha);
    *wi = vneg(reflect3(wo, m));
    lctx_assign_h(wo, m, c);
}
static _Thread_local int g_refraction_no_scale;   /* REFRACTION_NO_SCALE_FACTOR (LUT builder only; per thread) */
static float ct_bsdf(v3 wi, v3 wo, float alpha, float etaO, float etaI)   /* :152-189 */
{
    int active = wo.z != 0.0f && wi.z != 0.0f;
    int refl = wi.z * wo.z > 0.0f;
    v3 m = vnormalize(vadd(vscale(wo, refl ? 1.0f : etaO), vscale(wi, refl ? 1.0f : etaI)));
    m = m.z < 0.0f ? vneg(m) : m;
    float WIdotM = vdot(wi, m), WOdotM = vdot(wo, m);
    float D = ggx_d(m, alpha);
    float F = fresnel_dielectric(WOdotM, etaO, etaI);
    float G = ggx_g(wi, wo, m, alpha);
    float WIdotN = wi.z, WOdotN = wo.z;
    if (refl) return active ? F * D * G / (4.0f * fabsf(WIdotN) * fabsf(WOdotN)) : 0.0f;
    float sqrtDenom = etaO * WOdotM + etaI * WIdotM;
    float scale = g_refraction_no_scale ? etaI : etaO;
    float value = (1.0f - F) * fabsf(D * G * fabsf(WIdotM) * fabsf(WOdotM) * scale * scale
                                     / (WOdotN * WIdotN * sqrtDenom * sqrtDenom));
    return active ? value : 0.0f;
}
static float ct_bsdf_pdf(v3 wi, v3 wo, float alpha, float etaO, float etaI)  /* :191-216 */
{
    int active = wo.z != 0.0f && wi.z != 0.0f;
    int refl = wi.z * wo.z > 0.0f;
    v3 m = vnormalize(vadd(vscale(wo, refl ? 1.0f : etaO), vscale(wi, refl ? 1.0f : etaI)));
    m = m.z < 0.0f ? vneg(m) : m;
    float WIdotM = vdot(wi, m), WOdotM = vdot(wo, m);
    active = active && (WIdotM * wi.z > 0.0f && WOdotM * wo.z > 0.0f);
    float sqrtDenom = etaO * WOdotM + etaI * WIdotM;
    float dwh_dwi = refl ? 1.0f / (4.0f * WIdotM) : fabsf((etaI * etaI * WIdotM) / (sqrtDenom * sqrtDenom));
    float pdf = ggx_d_pdf(wo, m, alpha);
    float F = fresnel_dielectric(WOdotM, etaO, etaI);
    return active ? pdf * (refl ? F : 1.0f - F) * dwh_dwi : 0.0f;
}
static void ct_bsdf_sample(v3 wo, float sel, f2 sample, float alpha, float etaO, float etaI, v3* wi, lctx* c)  /* :218-256 */
{
    *wi = V3(0.0f, 0.0f, 0.0f);
    if (wo.z == 0.0f) return;
    if (etaO == etaI) { *wi = vneg(wo); return; }
    v3 m = sample_ggx(wo, sample, alpha);
    float WOdotM = vdot(wo, m);
    c->H = m; c->WOdotH = WOdotM;
    if (WOdotM <= 0.0f) return;
    float F = fresnel_dielectric(WOdotM, etaO, etaI);
    if (sel < F) *wi = vneg(reflect3(wo, m));
    else *wi = refract3(vneg(wo), m, etaO / etaI);
}

/* KullaConty.inc.hlsl */
static float ms_favg_dielectric(float eta)                                /* :13-19 */
{
    float eta2 = eta * eta;
    return eta >= 1.0f ? (eta - 1.0f) / (4.08567f + 1.00071f * eta)
                       : 0.997118f + 0.1014f * eta - 0.965241f * eta2 - 0.130607f * eta2 * eta;
}
static float ms_favg_conductor1(float eta, float k)                       /* :52-55 */
{
    float numerator = eta * (133.736f - 98.9833f * eta) + k * (eta * (59.5617f - 3.98288f * eta) - 182.37f)
                    + ((0.30818f * eta - 13.1093f) * eta - 62.5919f) * k * k - 8.21474f;
    float denominator = k * (eta * (94.6517f - 15.8558f * eta) - 187.166f) + (-78.476f * eta - 395.268f) * eta
                      + (eta * (eta - 15.4387f) - 62.0752f) * k * k;
    return saturatef(numerator / denominator);
}
static float ms_fresnel(float Eavg, float Favg) { return Favg * Favg * Eavg / (1.0f - Favg * (1.0f - Eavg)); }  /* :58-61 */
static float ms_bxdf(float Ei, float Eo, float Eavg)                     /* :68-73 */
{
    return Eavg < 1.0f ? (1.0f - Ei) * (1.0f - Eo) / (O_PI * (1.0f - Eavg)) : 0.0f;
}
static float ct_ms_bsdf(v3 wi, float alpha, float ratio, float eta, float Eo, float Eavg, float Eavg_inv, int isEntering)  /* :79-89 */
{
    float cosThetaI = fabsf(wi.z);
    if (cosThetaI == 0.0f) return 0.0f;
    int evalRefl = wi.z > 0.0f;
    float Ei = sample_bsdf_texture(cosThetaI, alpha, eta, evalRefl ? isEntering : !isEntering);
    float factor = evalRefl ? (1.0f - ratio) : ratio;
    return ms_bxdf(Ei, Eo, evalRefl ? Eavg : Eavg_inv) * factor;
}
static float ct_ms_bsdf_pdf(v3 wi, float ratio)                            /* :91-101 */
{
    float cosThetaI = fabsf(wi.z);
    if (cosThetaI == 0.0f) return 0.0f;
    int refl = wi.z > 0.0f;
    float pdf = fabsf(wi.z) * O_INV_PI;
    pdf = pdf * (refl ? 1.0f - ratio : ratio);
    return pdf;
}
static void ct_ms_bsdf_sample(v3 wo, float sel, f2 sample, float ratio, v3* wi)  /* :103-118 (context by value) */
{
    *wi = V3(0.0f, 0.0f, 0.0f);
    if (wo.z == 0.0f) return;
    int sampleRefl = sel >= ratio;
    *wi = cosine_sample_hemisphere(sample);
    if (!sampleRefl) wi->z = -wi->z;
}
static float reciprocal_factor(float Fl, float Fe, float El, float Ee, float eta)  /* :120-127 */
{
    float inv_eta = 1.0f / eta;
    float factor = (1.0f - Fl) * (1.0f - El);
    float factor1 = (1.0f - Fe) * (1.0f - Ee) * inv_eta * inv_eta;
    return factor1 / fmaxf(0.00001f, factor + factor1);
}
static v3 ct_ms_brdf(v3 wi, v3 wo, float alpha, float Eo, float Eavg, v3 factor)  /* :133-142 */
{
    if (wo.z <= 0.0f || wi.z <= 0.0f) return V3(0.0f, 0.0f, 0.0f);
    float Ei = sample_brdf_texture(wi.z, alpha);
    return vscale(factor, ms_bxdf(Ei, Eo, Eavg));
}
static float ct_ms_brdf_pdf(v3 wi, v3 wo)                                 /* :144-152 */
{
    if (wo.z <= 0.0f || wi.z <= 0.0f) return 0.0f;
    return wi.z * O_INV_PI;
}

/* LambertBRDF.inc.hlsl, SpecularBxDF.inc.hlsl */
static inline float lambert(v3 wi, v3 wo) { return wi.z > 0.0f && wo.z > 0.0f ? O_INV_PI : 0.0f; }
static inline float lambert_pdf(v3 wi, v3 wo) { return wi.z > 0.0f && wo.z > 0.0f ? wi.z * O_INV_PI : 0.0f; }
static void specular_brdf_sample(v3 wo, v3* wi, float* value, float* pdf, lctx* c)   /* :17-29 */
{
    *wi = V3(-wo.x, -wo.y, wo.z);
    c->H = V3(0.0f, 0.0f, 1.0f); c->WOdotH = wo.z;
    if (wo.z <= 0.0f) return;
    *value = 1.0f / wi->z;
    *pdf = 1.0f;
}
static void specular_bsdf_sample(v3 wo, float sample, float etaO, float etaI, int isThin, v3* wi, float* value, float* pdf, lctx* c)  /* :41-98 */
{
    *wi = V3(0.0f, 0.0f, 0.0f);
    c->H = V3(0.0f, 0.0f, 1.0f); c->WOdotH = wo.z;
    if (etaO == etaI) { *value = 1.0f / wo.z; *pdf = 1.0f; *wi = vneg(wo); return; }
    if (wo.z == 0.0f) return;
    float F = fresnel_dielectric(wo.z, etaO, etaI);
    float T = 1.0f - F;
    if (isThin && F < 1.0f) { F = F + T * T * F / (1.0f - F * F); T = 1.0f - F; }
    if (sample < F) {
        *wi = wo; wi->x = -wi->x; wi->y = -wi->y;
        *value = F / wi->z;
        *pdf = F;
    } else {
        if (!isThin) *wi = refract3(vneg(wo), V3(0.0f, 0.0f, 1.0f), etaO / etaI);
        else *wi = vneg(wo);
        if (wi->z == 0.0f) return;
        float scale = g_refraction_no_scale ? 1.0f : (!isThin ? (etaO * etaO) / (etaI * etaI) : 1.0f);
        *value = g_refraction_no_scale ? T / (-wi->z) : T * scale / (-wi->z);
        *pdf = T;
    }
}

/* BSDFs.inc.hlsl */
static inline float specular_weight(float cosThetaO, float alpha, float ior) { return sample_brdf_dielectric_texture(cosThetaO, alpha, ior, 0); }
static v3 internal_scattering_factor(float alpha, v3 albedo, float ior, uint32_t mode)   /* :19-36 */
{
    if (mode == DCRT_INTERNAL_SCATTERING_IGNORE) return V3(1.0f, 1.0f, 1.0f);
    float avg = sample_brdf_dielectric_average_texture(alpha, ior, 1);
    v3 factor = V3(1.0f - avg, 1.0f - avg, 1.0f - avg);
    if (mode == DCRT_INTERNAL_SCATTERING_MULTIPLE)
        factor = V3(factor.x / (1.0f - albedo.x * avg), factor.y / (1.0f - albedo.y * avg), factor.z / (1.0f - albedo.z * avg));
    return factor;
}
static inline v3 to_tbn(v3 w, const isect* it, v3 b) { return V3(vdot(w, it->tangent), vdot(w, b), vdot(w, it->normal)); }
static inline v3 from_tbn(v3 w, const isect* it, v3 b)
{
    v3 t = it->tangent, n = it->normal;
    return V3(w.x * t.x + w.y * b.x + w.z * n.x, w.x * t.y + w.y * b.y + w.z * n.y, w.x * t.z + w.y * b.z + w.z * n.z);
}

static v3 evaluate_bsdf(v3 wi, v3 wo, const isect* it)                    /* :42-163 */
{
    v3 b = vcross(it->normal, it->tangent);
    wo = to_tbn(wo, it, b);
    wi = to_tbn(wi, it, b);
    int isInverted = wo.z < 0.0f;
    if (isInverted) { wo.z = -wo.z; wi.z = -wi.z; }
    float cosThetaO = wo.z;
    lctx c = { { 0, 0, 0 }, 0.0f, isInverted };
    lctx_calc_h(wo, wi, &c);
    int perfectSmooth = it->alpha < O_ALPHA_THRESHOLD;
    v3 value = V3(0.0f, 0.0f, 0.0f);
    const uint32_t type = it->materialType;
    if (type != DCRT_MATERIAL_TYPE_DIELECTRIC && type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC) {
        int hasLambert = 0, hasCT = 0, hasCTms = 0, dielectricFresnel = 0;
        float ratio_lambert = 0.0f, E = 0.0f, E_avg = 0.0f;
        v3 F_ms = V3(0.0f, 0.0f, 0.0f), isf = V3(1.0f, 1.0f, 1.0f);
        int hasAnyBrdf = !isInverted || it->isTwoSided;
        if (it->multiscattering && (type == DCRT_MATERIAL_TYPE_PLASTIC || type == DCRT_MATERIAL_TYPE_CONDUCTOR) && hasAnyBrdf && !perfectSmooth) {
            E = sample_brdf_texture(cosThetaO, it->alpha);
            E_avg = sample_brdf_average_texture(it->alpha);
        }
        if (type == DCRT_MATERIAL_TYPE_DIFFUSE && hasAnyBrdf) {
            hasLambert = 1; ratio_lambert = 1.0f;
        } else if (type == DCRT_MATERIAL_TYPE_PLASTIC && hasAnyBrdf) {
            hasLambert = 1; hasCT = !perfectSmooth; hasCTms = it->multiscattering && !perfectSmooth; dielectricFresnel = 1;
            ratio_lambert = 1.0f - specular_weight(cosThetaO, it->alpha, it->ior.x);
            if (hasCTms) {
                float F_avg = ms_favg_dielectric(it->ior.x);
                float fms = ms_fresnel(E_avg, F_avg);
                F_ms = V3(fms, fms, fms);
                ratio_lambert = fmaxf(ratio_lambert - F_ms.x * (1.0f - E), 0.0f);
            }
            isf = internal_scattering_factor(it->alpha, it->albedo, it->ior.x, it->internalScatteringMode);
        } else if (type == DCRT_MATERIAL_TYPE_CONDUCTOR && hasAnyBrdf && !perfectSmooth) {
            hasCT = 1; hasCTms = it->multiscattering; dielectricFresnel = 0;
            if (hasCTms) {
                v3 k = it->albedo;
                v3 F_avg = V3(ms_favg_conductor1(it->ior.x, k.x), ms_favg_conductor1(it->ior.y, k.y), ms_favg_conductor1(it->ior.z, k.z));
                F_ms = V3(ms_fresnel(E_avg, F_avg.x), ms_fresnel(E_avg, F_avg.y), ms_fresnel(E_avg, F_avg.z));
            }
        }
        if (hasLambert) value = vadd(value, vmul(vscale(it->albedo, lambert(wi, wo) * ratio_lambert), isf));
        if (hasCT) {
            float bv = ct_brdf(wi, wo, it->alpha, &c);
            v3 F = dielectricFresnel ? V3(fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x), fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x), fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x))
                                     : fresnel_conductor(c.WOdotH, it->ior, it->albedo);
            value = vadd(value, vscale(F, bv));
        }
        if (hasCTms) value = vadd(value, ct_ms_brdf(wi, wo, it->alpha, E, E_avg, F_ms));
    } else if (type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC && !perfectSmooth) {
        float etaO = isInverted ? it->ior.x : 1.0f;
        float etaI = isInverted ? 1.0f : it->ior.x;
        float bv = ct_bsdf(wi, wo, it->alpha, etaO, etaI);
        value = vadd(value, V3(bv, bv, bv));
        if (it->multiscattering) {
            float ior = it->ior.x;
            float E_avg_enter = sample_bsdf_average_texture(it->alpha, ior, 1);
            float F_avg_enter = ms_favg_dielectric(1.0f / ior);
            float E_avg_leave = sample_bsdf_average_texture(it->alpha, ior, 0);
            float F_avg_leave = ms_favg_dielectric(ior);
            float rf = reciprocal_factor(F_avg_leave, F_avg_enter, E_avg_leave, E_avg_enter, ior);
            float E = sample_bsdf_texture(cosThetaO, it->alpha, ior, isInverted);
            float F_avg = isInverted ? F_avg_enter : F_avg_leave;
            float E_avg = isInverted ? E_avg_enter : E_avg_leave;
            float E_inv_avg = isInverted ? E_avg_leave : E_avg_enter;
            float ratio = (isInverted ? 1.0f - rf : rf) * (1.0f - F_avg);
            float mv = ct_ms_bsdf(wi, it->alpha, ratio, ior, E, E_avg, E_inv_avg, isInverted);
            value = vadd(value, V3(mv, mv, mv));
        }
    }
    return value;
}

static float evaluate_bsdf_pdf(v3 wi, v3 wo, const isect* it)             /* :165-287 */
{
    v3 b = vcross(it->normal, it->tangent);
    wo = to_tbn(wo, it, b);
    wi = to_tbn(wi, it, b);
    int isInverted = wo.z < 0.0f;
    if (isInverted) { wo.z = -wo.z; wi.z = -wi.z; }
    float cosThetaO = wo.z;
    lctx c = { { 0, 0, 0 }, 0.0f, isInverted };
    lctx_calc_h(wo, wi, &c);
    int perfectSmooth = it->alpha < O_ALPHA_THRESHOLD;
    float pdf = 0.0f;
    const uint32_t type = it->materialType;
    if (type != DCRT_MATERIAL_TYPE_DIELECTRIC && type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC) {
        int hasLambert = 0, hasCT = 0, hasCTms = 0;
        float wl = 0.0f, wct = 0.0f, wms = 0.0f;
        int hasAnyBrdf = !isInverted || it->isTwoSided;
        if (type == DCRT_MATERIAL_TYPE_DIFFUSE && hasAnyBrdf) {
            hasLambert = 1; wl = 1.0f;
        } else if (type == DCRT_MATERIAL_TYPE_PLASTIC && hasAnyBrdf) {
            hasLambert = 1; hasCT = !perfectSmooth; hasCTms = it->multiscattering && !perfectSmooth;
            wct = specular_weight(cosThetaO, it->alpha, it->ior.x);
            wl = 1.0f - wct;
            if (hasCTms) {
                float E = sample_brdf_texture(cosThetaO, it->alpha);
                float E_avg = sample_brdf_average_texture(it->alpha);
                float F_avg = ms_favg_dielectric(it->ior.x);
                float F_ms = ms_fresnel(E_avg, F_avg);
                wms = F_ms * (1.0f - E);
                wl = fmaxf(wl - wms, 0.0f);
            }
        } else if (type == DCRT_MATERIAL_TYPE_CONDUCTOR && hasAnyBrdf && !perfectSmooth) {
            hasCT = 1; hasCTms = it->multiscattering;
            wct = 1.0f;
            if (hasCTms) { wct = 0.5f; wms = 0.5f; }
        }
        if (hasLambert) pdf = pdf + lambert_pdf(wi, wo) * wl;
        if (hasCT) pdf = pdf + ct_brdf_pdf(wi, wo, it->alpha, &c) * wct;
        if (hasCTms) pdf = pdf + ct_ms_brdf_pdf(wi, wo) * wms;
    } else if (type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC && !perfectSmooth) {
        int hasMs = it->multiscattering;
        float wb = 1.0f, wms = 0.0f, ratio = 0.0f;
        float etaO = isInverted ? it->ior.x : 1.0f;
        float etaI = isInverted ? 1.0f : it->ior.x;
        if (hasMs) {
            float ior = it->ior.x;
            float E_avg_enter = sample_bsdf_average_texture(it->alpha, ior, 1);
            float F_avg_enter = ms_favg_dielectric(1.0f / ior);
            float E_avg_leave = sample_bsdf_average_texture(it->alpha, ior, 0);
            float F_avg_leave = ms_favg_dielectric(ior);
            float rf = reciprocal_factor(F_avg_leave, F_avg_enter, E_avg_leave, E_avg_enter, ior);
            float E = sample_bsdf_texture(cosThetaO, it->alpha, ior, isInverted);
            float F_avg = isInverted ? F_avg_enter : F_avg_leave;
            ratio = (isInverted ? 1.0f - rf : rf) * (1.0f - F_avg);
            wb = E; wms = 1.0f - E;
        }
        pdf = pdf + ct_bsdf_pdf(wi, wo, it->alpha, etaO, etaI) * wb;
        if (hasMs) pdf = pdf + ct_ms_bsdf_pdf(wi, ratio) * wms;
    }
    return pdf;
}

static void sample_bsdf(v3 wo, f2 sample, float sel, const isect* it, v3* wiOut, v3* valueOut, float* pdfOut, int* isDelta)  /* :289-505 */
{
    v3 wi = V3(0.0f, 0.0f, 0.0f);
    v3 value = V3(0.0f, 0.0f, 0.0f);
    float pdf = 0.0f;
    *isDelta = 0;
    v3 b = vcross(it->normal, it->tangent);
    wo = to_tbn(wo, it, b);
    int isInverted = wo.z < 0.0f;
    if (isInverted) wo.z = -wo.z;
    float cosThetaO = wo.z;
    lctx c = { { 0, 0, 0 }, 0.0f, isInverted };
    int perfectSmooth = it->alpha < O_ALPHA_THRESHOLD;
    const uint32_t type = it->materialType;
    if (type != DCRT_MATERIAL_TYPE_DIELECTRIC && type != DCRT_MATERIAL_TYPE_THIN_DIELECTRIC) {
        int hasLambert = 0, hasCT = 0, hasCTms = 0, dielectricFresnel = 0;
        float wl = 0.0f, wct = 0.0f, wms = 0.0f, E = 0.0f, E_avg = 0.0f;
        v3 F_ms = V3(0.0f, 0.0f, 0.0f), isf = V3(1.0f, 1.0f, 1.0f);
        int hasAnyBrdf = !isInverted || it->isTwoSided;
        if (it->multiscattering && (type == DCRT_MATERIAL_TYPE_PLASTIC || type == DCRT_MATERIAL_TYPE_CONDUCTOR) && hasAnyBrdf) {
            E = sample_brdf_texture(cosThetaO, it->alpha);
            E_avg = sample_brdf_average_texture(it->alpha);
        }
        if (type == DCRT_MATERIAL_TYPE_DIFFUSE && hasAnyBrdf) {
            hasLambert = 1; wl = 1.0f;
        } else if (type == DCRT_MATERIAL_TYPE_PLASTIC && hasAnyBrdf) {
            hasLambert = 1; hasCT = 1; hasCTms = it->multiscattering && !perfectSmooth; dielectricFresnel = 1;
            wct = specular_weight(cosThetaO, it->alpha, it->ior.x);
            wl = 1.0f - wct;
            if (hasCTms) {
                float F_avg = ms_favg_dielectric(it->ior.x);
                float fms = ms_fresnel(E_avg, F_avg);
                F_ms = V3(fms, fms, fms);
                wms = F_ms.x * (1.0f - E);
                wl = fmaxf(wl - wms, 0.0f);
            }
            isf = internal_scattering_factor(it->alpha, it->albedo, it->ior.x, it->internalScatteringMode);
        } else if (type == DCRT_MATERIAL_TYPE_CONDUCTOR && hasAnyBrdf) {
            hasCT = 1; hasCTms = it->multiscattering && !perfectSmooth; dielectricFresnel = 0;
            wct = 1.0f;
            if (hasCTms) {
                v3 k = it->albedo;
                v3 F_avg = V3(ms_favg_conductor1(it->ior.x, k.x), ms_favg_conductor1(it->ior.y, k.y), ms_favg_conductor1(it->ior.z, k.z));
                F_ms = V3(ms_fresnel(E_avg, F_avg.x), ms_fresnel(E_avg, F_avg.y), ms_fresnel(E_avg, F_avg.z));
                wct = 0.5f; wms = 0.5f;
            }
        }
        if (sel < wl) {
            wi = cosine_sample_hemisphere(sample);
            lctx_calc_h(wo, wi, &c);
        } else if (sel < wl + wct) {
            if (!perfectSmooth) {
                ct_brdf_sample(wo, sample, it->alpha, &wi, &c);
            } else {
                float vr = value.x;
                specular_brdf_sample(wo, &wi, &vr, &pdf, &c);
                v3 F = dielectricFresnel ? V3(fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x), fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x), fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x))
                                         : fresnel_conductor(c.WOdotH, it->ior, it->albedo);
                value = vscale(F, vr);
                pdf = pdf * wct;
                *isDelta = 1;
                hasLambert = 0; hasCT = 0; hasCTms = 0;
            }
        } else {
            wi = cosine_sample_hemisphere(sample);
            lctx_calc_h(wo, wi, &c);
        }
        if (hasLambert) {
            value = vadd(value, vmul(vscale(it->albedo, lambert(wi, wo) * wl), isf));
            pdf = pdf + lambert_pdf(wi, wo) * wl;
        }
        if (hasCT && !perfectSmooth) {
            float mv = ct_brdf(wi, wo, it->alpha, &c);
            v3 F = dielectricFresnel ? V3(fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x), fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x), fresnel_dielectric(c.WOdotH, 1.0f, it->ior.x))
                                     : fresnel_conductor(c.WOdotH, it->ior, it->albedo);
            value = vadd(value, vscale(F, mv));
            pdf = pdf + ct_brdf_pdf(wi, wo, it->alpha, &c) * wct;
        }
        if (hasCTms) {
            value = vadd(value, ct_ms_brdf(wi, wo, it->alpha, E, E_avg, F_ms));
            pdf = pdf + ct_ms_brdf_pdf(wi, wo) * wms;
        }
    } else if (type == DCRT_MATERIAL_TYPE_THIN_DIELECTRIC || perfectSmooth) {
        int isThin = type == DCRT_MATERIAL_TYPE_THIN_DIELECTRIC;
        int isEntering = isThin ? 0 : isInverted;
        float etaO = isEntering ? it->ior.x : 1.0f;
        float etaI = isEntering ? 1.0f : it->ior.x;
        float vr = value.x;
        specular_bsdf_sample(wo, sel, etaO, etaI, isThin, &wi, &vr, &pdf, &c);
        value = V3(vr, vr, vr);
        *isDelta = 1;
    } else {
        int hasMs = it->multiscattering;
        float wb = 1.0f, wms = 0.0f, E = 0.0f, E_avg = 0.0f, E_inv_avg = 0.0f, ratio = 0.0f;
        float etaO = isInverted ? it->ior.x : 1.0f;
        float etaI = isInverted ? 1.0f : it->ior.x;
        if (hasMs) {
            float ior = it->ior.x;
            float E_avg_enter = sample_bsdf_average_texture(it->alpha, ior, 1);
            float F_avg_enter = ms_favg_dielectric(1.0f / ior);
            float E_avg_leave = sample_bsdf_average_texture(it->alpha, ior, 0);
            float F_avg_leave = ms_favg_dielectric(ior);
            float rf = reciprocal_factor(F_avg_leave, F_avg_enter, E_avg_leave, E_avg_enter, ior);
            E = sample_bsdf_texture(cosThetaO, it->alpha, ior, isInverted);
            float F_avg = isInverted ? F_avg_enter : F_avg_leave;
            E_avg = isInverted ? E_avg_enter : E_avg_leave;
            E_inv_avg = isInverted ? E_avg_leave : E_avg_enter;
            ratio = (isInverted ? 1.0f - rf : rf) * (1.0f - F_avg);
            wb = E; wms = 1.0f - E;
        }
        if (sel < wb) ct_bsdf_sample(wo, sel, sample, it->alpha, etaO, etaI, &wi, &c);
        else ct_ms_bsdf_sample(wo, sel, sample, ratio, &wi);
        float bv = ct_bsdf(wi, wo, it->alpha, etaO, etaI);
        value = vadd(value, V3(bv, bv, bv));
        pdf = pdf + ct_bsdf_pdf(wi, wo, it->alpha, etaO, etaI) * wb;
        if (hasMs) {
            float mv = ct_ms_bsdf(wi, it->alpha, ratio, it->ior.x, E, E_avg, E_inv_avg, isInverted);
            value = vadd(value, V3(mv, mv, mv));
            pdf = pdf + ct_ms_bsdf_pdf(wi, ratio) * wms;
        }
    }
    if (isInverted) wi.z = -wi.z;
    *wiOut = from_tbn(wi, it, b);
    *valueOut = value;
    *pdfOut = pdf;
}

/* ------------------------------------------------------------------ */
/* One path, wavefront semantics (WavefrontPathTracing.hlsl:176-607)   */
/* or megakernel semantics (MegakernelPathTracing.hlsl:110-208).       */
/* ------------------------------------------------------------------ */
/* Debug aid: DCRT_ORACLE_TRACE="x,y" prints each bounce of that pixel's path to stderr. */
static int trace_enabled(uint32_t px, uint32_t py)
{
    static int parsed = 0, tx = -1, ty = -1;
    if (!parsed) {
        const char* e = getenv("DCRT_ORACLE_TRACE");
        if (e) sscanf(e, "%d,%d", &tx, &ty);
        parsed = 1;
    }
    return (int)px == tx && (int)py == ty;
}

static void trace_path(const dcrt_flat_scene* sc, const dcrt_frame_params* f, int mode, uint32_t px, uint32_t py,
                       float outPos[2], float outVal[3], uint32_t outRng[4], oracle_counters* cnt)
{
    const int dbg = trace_enabled(px, py);
    uint32_t s[4];
    oracle_rng_init(px, py, f->frame_seed, s);
    /* NEW_PATH :214-237 */
    f2 pixelSample = next2d(s);
    f2 filmSample;
    filmSample.x = (pixelSample.x + (float)px) / (float)f->resolution[0];
    filmSample.y = (pixelSample.y + (float)py) / (float)f->resolution[1];
    v3 apertureSample = next3d(s);
    v3 origin, direction;
    generate_ray(filmSample, apertureSample, f, &origin, &direction);
    const uint32_t features = f->features;
    const int lightVisible = (features & DCRT_FEATURE_LIGHT_VISIBLE) != 0;
    /* ALLOW_ANYHIT_SHADER: one opacity sample per cast ray. Wavefront: NEW_PATH :223-226,
     * then MATERIAL :422-430 (extension, then shadow, after the BSDF sample). Megakernel:
     * drawn inside IntersectScene / IsOcculuded (MegakernelPathTracing.hlsl:27-28, 57-58),
     * i.e. the shadow ray's before the BSDF sample. The first ray's is the same in both. */
    const int anyHitOn = (features & DCRT_FEATURE_ALLOW_ANYHIT) != 0;
    float extOpacity = anyHitOn ? next1d(s) : 0.0f, shadowOpacity = 0.0f;
    v3 T = V3(1.0f, 1.0f, 1.0f), Li = V3(0.0f, 0.0f, 0.0f);
    float bsdfPdfPrev = 0.0f;
    int isDeltaPrev = 1;
    uint32_t bounce = 0;
    v3 ro = origin, rd = direction;
    for (;;) {
        /* EXTENSION_RAY_CAST :84-120 */
        hit_info h; memset(&h, 0, sizeof(h));
        if (cnt) cnt->extension_rays++;
        int hasHit = bvh_intersect(sc, ro, rd, 0.0f, o_inf(), 0, features, extOpacity, &h,
                                   cnt ? &cnt->node_visits : NULL, cnt ? &cnt->triangle_tests : NULL, cnt ? &cnt->blas_entries : NULL);
        float hitT = hasHit ? h.t : o_inf();
        /* MATERIAL :302-479 */
        isect it; memset(&it, 0, sizeof(it));
        if (hasHit) hit_to_intersection(sc, &h, &it);
        {
            uint32_t lightIndex = hasHit ? it.lightIndex : f->environment_light_index;
            int doEval = lightVisible ? lightIndex != DCRT_LIGHT_INDEX_INVALID : (bounce > 0 && lightIndex != DCRT_LIGHT_INDEX_INVALID);
            if (doEval) {
                if (mode == ORACLE_MODE_MEGAKERNEL && bounce == 0) {
                    /* MegakernelPathTracing.hlsl:135-140, 200-205 */
                    const dcrt_light* L = &sc->lights[lightIndex];
                    if (hasHit) Li = vdot(vneg(rd), it.geometryNormal) > 0.0f ? vload(L->radiance) : V3(0.0f, 0.0f, 0.0f);
                    else Li = sc->env_cube_rgb ? vmul(sample_env_cube(sc, rd), vload(L->radiance)) : vload(L->radiance);
                } else {
                    v3 radiance; float lightPdf;
                    evaluate_light_direct(sc, lightIndex, it.triangleIndex, it.geometryNormal, rd, hitT, f->light_count, &radiance, &lightPdf);
                    if (lightPdf > 0.0f) {
                        float weight = !isDeltaPrev ? power_heuristic(bsdfPdfPrev, lightPdf) : 1.0f;
                        Li = vadd(Li, vscale(vmul(T, radiance), weight));
                    }
                }
            }
        }
        v3 lsr = V3(0.0f, 0.0f, 0.0f);
        int terminate = 0, hasShadowRay = 0;
        v3 so = V3(0, 0, 0), sd = V3(0, 0, 0);
        float sdist = 0.0f;
        if (bounce > f->max_bounce_count || !hasHit) {
            terminate = 1;
        } else {
            v3 wo = vneg(rd);
            if (f->light_count != 0) {
                light_sample ls = sample_light_direct(sc, it.position, f->light_count, s);
                if (vany_pos(ls.radiance) && ls.pdf > 0.0f) {
                    v3 bsdf = evaluate_bsdf(ls.wi, wo, &it);
                    float NdotWI = fabsf(vdot(it.normal, ls.wi));
                    float bsdfPdf = evaluate_bsdf_pdf(ls.wi, wo, &it);
                    float weight = ls.isDeltaLight ? 1.0f : power_heuristic(ls.pdf, bsdfPdf);
                    v3 tmp = vmul(vmul(T, ls.radiance), bsdf);
                    tmp = vscale(tmp, NdotWI);
                    tmp = vscale(tmp, weight);
                    lsr = vdivs(tmp, ls.pdf);
                    if (dbg)
                        fprintf(stderr, "  nee wi(%g %g %g) Le(%g %g %g) pdf %g dist %g delta %d f(%g %g %g) bsdfPdf %g w %g\n", ls.wi.x, ls.wi.y, ls.wi.z,
                                ls.radiance.x, ls.radiance.y, ls.radiance.z, ls.pdf, ls.distance, ls.isDeltaLight, bsdf.x, bsdf.y, bsdf.z, bsdfPdf, weight);
                    sd = ls.wi;
                    so = offset_ray_origin(it.position, it.geometryNormal, ls.wi);
                    sdist = ls.distance;
                    hasShadowRay = 1;
                    if (anyHitOn && mode == ORACLE_MODE_MEGAKERNEL) shadowOpacity = next1d(s);
                }
            }
            float bsdfPdf = 0.0f; int isDeltaB = 0;
            {
                float sel = next1d(s);
                f2 bs = next2d(s);
                v3 wi, bsdf;
                sample_bsdf(wo, bs, sel, &it, &wi, &bsdf, &bsdfPdf, &isDeltaB);
                if (dbg)
                    fprintf(stderr, "b%u mat%u n(%g %g %g) wo(%g %g %g) sel %g bs(%g %g) -> wi(%g %g %g) f(%g %g %g) pdf %g delta %d T(%g %g %g) lsr(%g %g %g) Li(%g %g %g)\n",
                            bounce, it.materialType, it.normal.x, it.normal.y, it.normal.z, wo.x, wo.y, wo.z, sel, bs.x, bs.y,
                            wi.x, wi.y, wi.z, bsdf.x, bsdf.y, bsdf.z, bsdfPdf, isDeltaB, T.x, T.y, T.z, lsr.x, lsr.y, lsr.z, Li.x, Li.y, Li.z);
                if ((bsdf.x != 0.0f || bsdf.y != 0.0f || bsdf.z != 0.0f) && bsdfPdf != 0.0f) {
                    float NdotWI = fabsf(vdot(it.normal, wi));
                    T = vdivs(vscale(vmul(T, bsdf), NdotWI), bsdfPdf);
                    rd = wi;
                    ro = offset_ray_origin(it.position, it.geometryNormal, wi);
                    bounce += 1;
                } else {
                    terminate = 1;
                }
            }
            bsdfPdfPrev = bsdfPdf;
            isDeltaPrev = isDeltaB;
            if (anyHitOn) {
                if (!terminate) extOpacity = next1d(s);
                if (hasShadowRay && mode != ORACLE_MODE_MEGAKERNEL) shadowOpacity = next1d(s);
            }
        }
        /* SHADOW_RAY_CAST :141-172 */
        int shadowHit = 0;
        if (hasShadowRay) {
            if (cnt) cnt->shadow_rays++;
            shadowHit = bvh_intersect(sc, so, sd, 0.0f, sdist, 1, features, shadowOpacity, &h,
                                      cnt ? &cnt->shadow_node_visits : NULL, cnt ? &cnt->shadow_triangle_tests : NULL,
                                      cnt ? &cnt->shadow_blas_entries : NULL);
        }
        /* CONTROL :519-537 */
        if (!shadowHit) Li = vadd(Li, lsr);
        else Li = vadd(Li, V3(0.0f, 0.0f, 0.0f));
        if (terminate) break;
    }
    outPos[0] = pixelSample.x; outPos[1] = pixelSample.y;
    outVal[0] = Li.x; outVal[1] = Li.y; outVal[2] = Li.z;
    if (outRng) { outRng[0] = s[0]; outRng[1] = s[1]; outRng[2] = s[2]; outRng[3] = s[3]; }
}

/* Test entries: one material's BSDF in the frame n = (0,0,1), t = (1,0,0) (see dcrt_oracle.h) */
static isect bsdf_test_isect(const oracle_bsdf_material* m)
{
    isect it;
    memset(&it, 0, sizeof(it));
    it.albedo = V3(m->albedo[0], m->albedo[1], m->albedo[2]);
    it.alpha = m->alpha;
    it.normal = V3(0.0f, 0.0f, 1.0f);
    it.geometryNormal = V3(0.0f, 0.0f, 1.0f);
    it.tangent = V3(1.0f, 0.0f, 0.0f);
    it.ior = V3(m->ior, 1.0f, 1.0f);
    it.isTwoSided = m->two_sided;
    it.multiscattering = m->multiscattering;
    it.internalScatteringMode = m->internal_scattering;
    it.materialType = m->type;
    it.lightIndex = DCRT_LIGHT_INDEX_INVALID;
    return it;
}
void oracle_bsdf_eval(const dcrt_bxdf_luts* luts, const oracle_bsdf_material* m, const float* wi, const float* wo,
                      uint32_t count, float* f_out, float* pdf_out)
{
    g_luts = luts;
    const isect it = bsdf_test_isect(m);
    for (uint32_t i = 0; i < count; ++i) {
        const v3 a = V3(wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]), b = V3(wo[3 * i], wo[3 * i + 1], wo[3 * i + 2]);
        const v3 f = evaluate_bsdf(a, b, &it);
        f_out[3 * i] = f.x; f_out[3 * i + 1] = f.y; f_out[3 * i + 2] = f.z;
        pdf_out[i] = evaluate_bsdf_pdf(a, b, &it);
    }
}
void oracle_bsdf_sample(const dcrt_bxdf_luts* luts, const oracle_bsdf_material* m, const float* wo, const float* u,
                        uint32_t count, float* wi_out, float* f_out, float* pdf_out, int* delta_out)
{
    g_luts = luts;
    const isect it = bsdf_test_isect(m);
    for (uint32_t i = 0; i < count; ++i) {
        const v3 b = V3(wo[3 * i], wo[3 * i + 1], wo[3 * i + 2]);
        f2 smp; smp.x = u[3 * i]; smp.y = u[3 * i + 1];
        v3 wi, f; float pdf; int delta;
        sample_bsdf(b, smp, u[3 * i + 2], &it, &wi, &f, &pdf, &delta);
        wi_out[3 * i] = wi.x; wi_out[3 * i + 1] = wi.y; wi_out[3 * i + 2] = wi.z;
        f_out[3 * i] = f.x; f_out[3 * i + 1] = f.y; f_out[3 * i + 2] = f.z;
        pdf_out[i] = pdf; delta_out[i] = delta;
    }
}

void oracle_generate_camera_ray(const dcrt_frame_params* f, uint32_t px, uint32_t py, float origin[3], float direction[3], uint32_t rng_out[4])
{
    uint32_t s[4];
    oracle_rng_init(px, py, f->frame_seed, s);
    f2 pixelSample = next2d(s);
    f2 filmSample;
    filmSample.x = (pixelSample.x + (float)px) / (float)f->resolution[0];
    filmSample.y = (pixelSample.y + (float)py) / (float)f->resolution[1];
    v3 apertureSample = next3d(s);
    v3 o, d;
    generate_ray(filmSample, apertureSample, f, &o, &d);
    origin[0] = o.x; origin[1] = o.y; origin[2] = o.z;
    direction[0] = d.x; direction[1] = d.y; direction[2] = d.z;
    if (rng_out) memcpy(rng_out, s, 16);
}

typedef struct render_job {
    const dcrt_flat_scene* sc; const dcrt_frame_params* f; int mode;
    uint32_t x0, y0, w, h;
    float* pos; float* val; uint32_t* rng;
    volatile uint32_t* next_row; pthread_mutex_t* lock;
    oracle_counters cnt;
} render_job;

static void* render_worker(void* arg)
{
    render_job* j = (render_job*)arg;
    const uint32_t W = j->f->resolution[0];
    for (;;) {
        uint32_t row;
        pthread_mutex_lock(j->lock);
        row = (*j->next_row)++;
        pthread_mutex_unlock(j->lock);
        if (row >= j->h) break;
        uint32_t y = j->y0 + row;
        for (uint32_t x = j->x0; x < j->x0 + j->w; ++x) {
            size_t p = (size_t)y * W + x;
            float val[3];
            trace_path(j->sc, j->f, j->mode, x, y, j->pos + p * 2, val, j->rng ? j->rng + p * 4 : NULL, &j->cnt);
            j->val[p * 4 + 0] = val[0]; j->val[p * 4 + 1] = val[1]; j->val[p * 4 + 2] = val[2]; j->val[p * 4 + 3] = 0.0f;
        }
    }
    return NULL;
}

int oracle_render(const dcrt_flat_scene* sc, const dcrt_bxdf_luts* luts, const dcrt_frame_params* f, int mode,
                  uint32_t x0, uint32_t y0, uint32_t w, uint32_t h, float* pos, float* val, uint32_t* rng,
                  oracle_counters* counters, int num_threads)
{
    if (!sc || !luts || !f || !pos || !val) return DCRT_E_INVALID_ARG;
    if ((uint64_t)x0 + w > f->resolution[0] || (uint64_t)y0 + h > f->resolution[1]) return DCRT_E_INVALID_ARG;
    init_srgb();
    g_luts = luts;
    g_vndf = (f->features & DCRT_FEATURE_GGX_SAMPLE_VNDF) != 0;
    if (num_threads < 1) num_threads = 1;
    if (num_threads > 256) num_threads = 256;
    uint32_t next_row = 0;
    pthread_mutex_t lock = PTHREAD_MUTEX_INITIALIZER;
    render_job jobs[256];
    pthread_t th[256];
    for (int i = 0; i < num_threads; ++i) {
        render_job j = { sc, f, mode, x0, y0, w, h, pos, val, rng, &next_row, &lock, { 0 } };
        jobs[i] = j;
    }
    for (int i = 1; i < num_threads; ++i) pthread_create(&th[i], NULL, render_worker, &jobs[i]);
    render_worker(&jobs[0]);
    for (int i = 1; i < num_threads; ++i) pthread_join(th[i], NULL);
    if (counters) {
        memset(counters, 0, sizeof(*counters));
        for (int i = 0; i < num_threads; ++i) {
            counters->extension_rays += jobs[i].cnt.extension_rays;
            counters->shadow_rays += jobs[i].cnt.shadow_rays;
            counters->node_visits += jobs[i].cnt.node_visits;
            counters->triangle_tests += jobs[i].cnt.triangle_tests;
            counters->blas_entries += jobs[i].cnt.blas_entries;
            counters->shadow_node_visits += jobs[i].cnt.shadow_node_visits;
            counters->shadow_triangle_tests += jobs[i].cnt.shadow_triangle_tests;
            counters->shadow_blas_entries += jobs[i].cnt.shadow_blas_entries;
        }
    }
    return DCRT_OK;
}

void oracle_trace_rays(const dcrt_flat_scene* sc, const dcrt_ray* rays, uint32_t count, dcrt_ray_hit* hits, uint32_t features, oracle_counters* cnt)
{
    for (uint32_t i = 0; i < count; ++i) {
        hit_info h; memset(&h, 0, sizeof(h));
        int hasHit = bvh_intersect(sc, vload(rays[i].origin), vload(rays[i].direction), 0.0f, o_inf(), 0, features & ~DCRT_FEATURE_ALLOW_ANYHIT, 0.0f, &h,
                                   cnt ? &cnt->node_visits : NULL, cnt ? &cnt->triangle_tests : NULL, cnt ? &cnt->blas_entries : NULL);
        if (cnt) cnt->extension_rays++;
        /* WavefrontPathTracing.hlsl:113-117; miss fields are defined as zero here (A.5) */
        hits[i].t = hasHit ? h.t : o_inf();
        hits[i].u = hasHit ? h.u : 0.0f;
        hits[i].v = hasHit ? h.v : 0.0f;
        hits[i].triangle_id = hasHit ? ((h.triangleId & 0x7FFFFFFFu) | (h.backface ? 0x80000000u : 0u)) : 0u;
        hits[i].instance_index = hasHit ? h.instanceIndex : 0u;
    }
}

void oracle_occluded(const dcrt_flat_scene* sc, const dcrt_ray* rays, uint32_t count, uint32_t* occ, uint32_t features, oracle_counters* cnt)
{
    for (uint32_t i = 0; i < count; ++i) {
        hit_info h;
        occ[i] = (uint32_t)bvh_intersect(sc, vload(rays[i].origin), vload(rays[i].direction), 0.0f, rays[i].t_max, 1, features & ~DCRT_FEATURE_ALLOW_ANYHIT, 0.0f, &h,
                                         cnt ? &cnt->shadow_node_visits : NULL, cnt ? &cnt->shadow_triangle_tests : NULL,
                                         cnt ? &cnt->shadow_blas_entries : NULL);
        if (cnt) cnt->shadow_rays++;
    }
}

/* ------------------------------------------------------------------ */
/* SampleConvolution.hlsl:24-106                                       */
/* ------------------------------------------------------------------ */
typedef struct filter_consts { float radius, gaussianAlpha, gaussianExp, mf[7]; uint32_t tau, kind; } filter_consts;

static float f_gaussian(const filter_consts* c, float d) { return fmaxf(0.0f, det_expf(-c->gaussianAlpha * d * d) - c->gaussianExp); }
static float f_mitchell1d(const filter_consts* c, float x)
{
    x = fabsf(2.0f * x);
    float r = x < 1.0f ? c->mf[4] * x * x * x + c->mf[5] * x * x + c->mf[6]
                       : (x < 2.0f ? c->mf[0] * x * x * x + c->mf[1] * x * x + c->mf[2] * x + c->mf[3] : 0.0f);
    r = r * (1.0f / 6.0f);
    return r;
}
static float f_sinc(float x) { x = fabsf(x); return x >= 1e-5f ? det_sinf(3.1415926535f * x) / (3.1415926535f * x) : 1.0f; }
static float f_windowed_sinc(const filter_consts* c, float x, float radius)
{
    x = fabsf(x);
    float lanczos = f_sinc(x / (float)c->tau);
    return x > radius ? 0.0f : f_sinc(x) * lanczos;
}
static float evaluate_filter(const filter_consts* c, float r, float px, float py)
{
    switch (c->kind) {
    case DCRT_FILTER_TRIANGLE: return fmaxf(0.0f, r - fabsf(px)) * fmaxf(0.0f, r - fabsf(py));
    case DCRT_FILTER_GAUSSIAN: return f_gaussian(c, px) * f_gaussian(c, py);
    case DCRT_FILTER_MITCHELL: return f_mitchell1d(c, px / c->radius) * f_mitchell1d(c, py / c->radius);
    case DCRT_FILTER_LANCZOS: return f_windowed_sinc(c, px, c->radius) * f_windowed_sinc(c, py, c->radius);
    default: return (fabsf(px) <= r && fabsf(py) <= r) ? 1.0f : 0.0f;
    }
}
/* host constants: SampleConvolution.cpp:100-130 */
static void make_filter_consts(const dcrt_filter_params* p, filter_consts* c)
{
    memset(c, 0, sizeof(*c));
    c->kind = p->filter;
    c->radius = p->radius;
    if (p->filter == DCRT_FILTER_GAUSSIAN) {
        c->gaussianAlpha = p->gaussian_alpha;
        c->gaussianExp = expf(-p->gaussian_alpha * p->radius * p->radius);
    } else if (p->filter == DCRT_FILTER_MITCHELL) {
        const float B = p->mitchell_b, C = p->mitchell_c;
        c->mf[0] = -B - 6 * C; c->mf[1] = 6 * B + 30 * C; c->mf[2] = -12 * B - 48 * C; c->mf[3] = 8 * B + 24 * C;
        c->mf[4] = 12 - 9 * B - 6 * C; c->mf[5] = -18 + 12 * B + 6 * C; c->mf[6] = 6 - 2 * B;
    } else if (p->filter == DCRT_FILTER_LANCZOS) {
        c->tau = p->lanczos_tau;
    }
}
void oracle_sample_convolution(const dcrt_filter_params* fp, uint32_t W, uint32_t H, const float* spos, const float* sval,
                               float* film, uint32_t row_begin, uint32_t row_end)
{
    filter_consts c;
    make_filter_consts(fp, &c);
    const float r = fp->radius;
    for (uint32_t py = row_begin; py < row_end && py < H; ++py) {
        for (uint32_t px = 0; px < W; ++px) {
            float wsum = 0.0f; v3 sum = V3(0.0f, 0.0f, 0.0f);
            float cx = (float)px + 0.5f, cy = (float)py + 0.5f;
            int xs = (int)floorf(cx - r); xs = xs < 0 ? 0 : xs;
            int xe = (int)floorf(cx + r); xe = xe > (int)W - 1 ? (int)W - 1 : xe;
            int ys = (int)floorf(cy - r); ys = ys < 0 ? 0 : ys;
            int ye = (int)floorf(cy + r); ye = ye > (int)H - 1 ? (int)H - 1 : ye;
            for (int y = ys; y <= ye; ++y) {
                for (int x = xs; x <= xe; ++x) {
                    size_t q = (size_t)y * W + x;
                    float spx = spos[q * 2] + (float)x, spy = spos[q * 2 + 1] + (float)y;
                    v3 v = V3(sval[q * 4], sval[q * 4 + 1], sval[q * 4 + 2]);
                    float w = evaluate_filter(&c, r, cx - spx, cy - spy);
                    sum = vadd(sum, vscale(v, w));
                    wsum = wsum + w;
                }
            }
            size_t p = (size_t)py * W + px;
            film[p * 4 + 0] = film[p * 4 + 0] + sum.x;
            film[p * 4 + 1] = film[p * 4 + 1] + sum.y;
            film[p * 4 + 2] = film[p * 4 + 2] + sum.z;
            film[p * 4 + 3] = film[p * 4 + 3] + wsum;
        }
    }
}

/* ------------------------------------------------------------------ */
/* BxDF LUT builder: BxDFTexturesBuilding.hlsl:10-186 with the defines */
/* BxDFTexturesBuilding.cpp:142-458 formats with "%f".                 */
/* ------------------------------------------------------------------ */
typedef struct lut_cfg { float ix, iy, iz, sz; double weight; uint32_t batches, w, h, slices; int type; int fresnel; } lut_cfg;
static void lut_config(int which, lut_cfg* c)
{
    /* "%f"-rounded literal values of the compiled defines */
    c->ix = 0.032258f;
    if (which == 0) { c->iy = 0.032258f; c->iz = 1.0f; c->sz = 0.0f; c->weight = 0.000049; c->batches = 5; c->w = 32; c->h = 32; c->slices = 1; c->type = 0; c->fresnel = 0; }
    else if (which == 1) { c->iy = 0.066667f; c->iz = 0.133333f; c->sz = 1.0f; c->weight = 0.000049; c->batches = 5; c->w = 32; c->h = 16; c->slices = 32; c->type = 0; c->fresnel = 1; }
    else { c->iy = 0.066667f; c->iz = 0.133333f; c->sz = 1.0f; c->weight = 0.000010; c->batches = 24; c->w = 32; c->h = 16; c->slices = 32; c->type = 1; c->fresnel = 1; }
}
static float lut_texel_integrate(const lut_cfg* c, uint32_t tx, uint32_t ty, uint32_t slice)
{
    const uint32_t entering = slice >= 16 ? 1u : 0u;
    const uint32_t tz = slice & 15u;
    const float cosThetaO = fmaxf((float)tx * c->ix, 0.0001f);
    const float alpha = (float)ty * c->iy;
    const float Ior = (float)tz * c->iz + c->sz;
    const int perfectSmooth = alpha < 0.00052441f;
    float acc = 0.0f;
    for (uint32_t batch = 0; batch < c->batches; ++batch) {
        uint32_t s[4];
        oracle_rng_init(0, 0, batch, s);
        double result = batch == 0 ? 0.0 : (double)acc;
        for (uint32_t i = 0; i < 4096; ++i) {
            v3 wo = V3(sqrtf(1.0f - cosThetaO * cosThetaO), 0.0f, cosThetaO);
            v3 wi = V3(0.0f, 0.0f, 0.0f);
            lctx ctx = { { 0, 0, 0 }, 0.0f, 0 };
            float value = 0.0f, pdf = 0.0f;
            if (c->type == 0) {
                if (perfectSmooth) {
                    specular_brdf_sample(wo, &wi, &value, &pdf, &ctx);
                } else {
                    f2 smp = next2d(s);
                    ct_brdf_sample(wo, smp, alpha, &wi, &ctx);
                    value = ct_brdf(wi, wo, alpha, &ctx);
                    pdf = ct_brdf_pdf(wi, wo, alpha, &ctx);
                }
                if (pdf > 0.0f) {
                    if (c->fresnel) {
                        const float etaO = entering ? Ior : 1.0f;
                        const float etaI = entering ? 1.0f : Ior;
                        value = value * fresnel_dielectric(ctx.WOdotH, etaO, etaI);
                    }
                    result += c->weight * (double)value * (double)fabsf(wi.z) / (double)pdf;
                }
            } else {
                const float etaO = entering ? Ior : 1.0f;
                const float etaI = entering ? 1.0f : Ior;
                float sel = next1d(s);
                if (perfectSmooth) {
                    specular_bsdf_sample(wo, sel, etaO, etaI, 0, &wi, &value, &pdf, &ctx);
                } else {
                    f2 smp = next2d(s);
                    ct_bsdf_sample(wo, sel, smp, alpha, etaO, etaI, &wi, &ctx);
                    value = ct_bsdf(wi, wo, alpha, etaO, etaI);
                    pdf = ct_bsdf_pdf(wi, wo, alpha, etaO, etaI);
                }
                if (pdf > 0.0f) result += c->weight * (double)value * (double)fabsf(wi.z) / (double)pdf;
            }
        }
        acc = (float)result;
    }
    return acc;
}
void oracle_lut_integrate(int which, uint32_t texel_begin, uint32_t texel_end, float* out)
{
    lut_cfg c; lut_config(which, &c);
    g_vndf = 1;                                   /* BxDFTexturesBuilding.cpp:38 */
    g_refraction_no_scale = (c.type == 1);        /* :50-53 */
    const uint32_t per_slice = c.w * c.h;
    for (uint32_t t = texel_begin; t < texel_end; ++t) {
        uint32_t slice = t / per_slice, rem = t % per_slice;
        uint32_t ty = rem / c.w, tx = rem % c.w;
        out[t - texel_begin] = lut_texel_integrate(&c, tx, ty, slice);
    }
    g_refraction_no_scale = 0;
}
static uint16_t to_unorm16(float f)
{
    f = saturatef(f);
    return (uint16_t)rintf(f * 65535.0f);
}
/* INTEGRATE_AVERAGE :116-162, n = 31, LUT_INTERVAL_X = 0.032258 */
static float lut_average_row(const float* row)
{
    const uint32_t n = 31;
    double fa = (double)(row[0] * 0.0001f);
    double sum = 0.0;
    for (uint32_t i = 1; i < n; ++i) {
        const double cosTheta = (double)((float)i * 0.032258f);
        sum += (double)saturatef(row[i]) * cosTheta;
    }
    double fb = (double)row[n];
    double result = (sum + (fa + fb) * 0.5) * (double)(1.0f / (float)n);
    return (float)(result * 2.0);
}
void oracle_lut_finalize(const float* brdf, const float* brdfd, const float* bsdf, dcrt_bxdf_luts* L)
{
    for (int i = 0; i < DCRT_LUT_BRDF_COUNT; ++i) L->brdf[i] = to_unorm16(brdf[i]);
    for (int y = 0; y < 32; ++y) L->brdf_avg[y] = to_unorm16(lut_average_row(brdf + y * 32));
    for (int i = 0; i < DCRT_LUT_BRDF_DIELECTRIC_COUNT; ++i) { L->brdf_dielectric[i] = to_unorm16(brdfd[i]); L->bsdf[i] = to_unorm16(bsdf[i]); }
    /* threadId.y = alpha row, threadId.z = slice -> dest (alpha, slice % 16, slice / 16) */
    for (int z = 0; z < 32; ++z) {
        for (int y = 0; y < 16; ++y) {
            int dest = (z / 16) * 256 + (z % 16) * 16 + y;
            L->brdf_dielectric_avg[dest] = to_unorm16(lut_average_row(brdfd + (size_t)z * 512 + y * 32));
            L->bsdf_avg[dest] = to_unorm16(lut_average_row(bsdf + (size_t)z * 512 + y * 32));
        }
    }
}

typedef struct lut_job { int which; uint32_t begin, end; float* out; } lut_job;
static void* lut_worker(void* a) { lut_job* j = (lut_job*)a; oracle_lut_integrate(j->which, j->begin, j->end, j->out + j->begin); return NULL; }

int oracle_build_luts(dcrt_bxdf_luts* L, int num_threads)
{
    if (num_threads < 1) num_threads = 1;
    if (num_threads > 64) num_threads = 64;
    float* brdf = (float*)calloc(DCRT_LUT_BRDF_COUNT, sizeof(float));
    float* brdfd = (float*)calloc(DCRT_LUT_BRDF_DIELECTRIC_COUNT, sizeof(float));
    float* bsdf = (float*)calloc(DCRT_LUT_BSDF_COUNT, sizeof(float));
    if (!brdf || !brdfd || !bsdf) { free(brdf); free(brdfd); free(bsdf); return DCRT_E_LIMIT; }
    float* outs[3] = { brdf, brdfd, bsdf };
    uint32_t counts[3] = { DCRT_LUT_BRDF_COUNT, DCRT_LUT_BRDF_DIELECTRIC_COUNT, DCRT_LUT_BSDF_COUNT };
    for (int which = 0; which < 3; ++which) {
        lut_job jobs[64]; pthread_t th[64];
        uint32_t chunk = (counts[which] + num_threads - 1) / num_threads;
        for (int i = 0; i < num_threads; ++i) {
            jobs[i].which = which; jobs[i].out = outs[which];
            jobs[i].begin = i * chunk < counts[which] ? i * chunk : counts[which];
            jobs[i].end = (i + 1) * chunk < counts[which] ? (i + 1) * chunk : counts[which];
        }
        for (int i = 0; i < num_threads; ++i) pthread_create(&th[i], NULL, lut_worker, &jobs[i]);
        for (int i = 0; i < num_threads; ++i) pthread_join(th[i], NULL);
    }
    oracle_lut_finalize(brdf, brdfd, bsdf, L);
    free(brdf); free(brdfd); free(bsdf);
    return DCRT_OK;
}

/* ------------------------------------------------------------------ */
/* Post-processing: SumLuminance.hlsl (two-stage log-luminance tree    */
/* reduction), PostProcessings.hlsl (exposure + Reinhard), and the     */
/* R8G8B8A8_UNORM_SRGB render-target encode (host-made thresholds).     */
/* ------------------------------------------------------------------ */
typedef struct float4_t { float x, y, z, w; } float4_t;
static float4_t film_load(const float* film, uint32_t W, uint32_t H, uint32_t x, uint32_t y)
{
    float4_t r = { 0.0f, 0.0f, 0.0f, 0.0f };          /* out-of-range Load returns 0 */
    if (x < W && y < H) { const float* p = film + ((size_t)y * W + x) * 4; r.x = p[0]; r.y = p[1]; r.z = p[2]; r.w = p[3]; }
    return r;
}
static float lum_log(float4_t s)                       /* SumLuminance.hlsl:29-44 */
{
    v3 c = V3(0.0f, 0.0f, 0.0f);
    if (s.w > 0.0f) c = V3(s.x / s.w, s.y / s.w, s.z / s.w);
    c.x = fminf(fmaxf(c.x, 0.0f), 65000.0f); c.y = fminf(fmaxf(c.y, 0.0f), 65000.0f); c.z = fminf(fmaxf(c.z, 0.0f), 65000.0f);
    const float lum = c.x * 0.299f + c.y * 0.587f + c.z * 0.114f;
    return det_logf(0.0001f + lum);
}
float oracle_sum_log_luminance(const float* film, uint32_t W, uint32_t H)
{
    const uint32_t bx = (((W + 7) / 8) + 1) / 2, by = (((H + 7) / 8) + 1) / 2;
    uint32_t count = bx * by;
    float* a = (float*)malloc(sizeof(float) * (count + 128));
    float* b = (float*)malloc(sizeof(float) * (count + 128));
    float acc[128];
    for (uint32_t gy = 0; gy < by; ++gy)
        for (uint32_t gx = 0; gx < bx; ++gx) {
            for (uint32_t t = 0; t < 64; ++t) {
                const uint32_t x = gx * 8 + (t % 8), y = gy * 8 + (t / 8);
                float v = lum_log(film_load(film, W, H, x, y));
                v = v + lum_log(film_load(film, W, H, x + 8 * bx, y));
                v = v + lum_log(film_load(film, W, H, x, y + 8 * by));
                v = v + lum_log(film_load(film, W, H, x + 8 * bx, y + 8 * by));
                acc[t] = v;
            }
            for (uint32_t k = 32; k >= 1; k >>= 1)
                for (uint32_t t = 0; t < k; ++t) acc[t] = acc[t] + acc[t + k];
            a[gy * bx + gx] = acc[0];
        }
    while (count != 1) {
        const uint32_t groups = (count + 127) / 128;
        for (uint32_t g = 0; g < groups; ++g) {
            for (uint32_t t = 0; t < 128; ++t) acc[t] = g * 128 + t < count ? a[g * 128 + t] : 0.0f;
            for (uint32_t k = 64; k >= 1; k >>= 1)
                for (uint32_t t = 0; t < k; ++t) acc[t] = acc[t] + acc[t + k];
            b[g] = acc[0];
        }
        float* tmp = a; a = b; b = tmp;
        count = groups;
    }
    const float r = a[0];
    free(a); free(b);
    return r;
}
void oracle_resolve_image(const float* film, uint32_t W, uint32_t H, int enabled, int autoExposure, float ev100,
                          float luminanceWhite, const float* srgbThresholds, uint8_t* out)
{
    float exposure = 1.0f;
    if (enabled) {
        float e = ev100;
        if (autoExposure) {
            const float recip = 1.0f / (float)(W * H);
            const float avgLum = det_expf(oracle_sum_log_luminance(film, W, H) * recip);
            e = det_logf(avgLum * 100.0f / 12.5f) * 1.44269504088896341f;   /* log2 */
        }
        const float maxLuminance = 1.2f * det_expf(e * 0.693147180559945309f);  /* pow(2, EV100) */
        exposure = 1.0f / maxLuminance;
    }
    const float maxWhiteSqr = luminanceWhite * luminanceWhite;
    for (uint32_t p = 0; p < W * H; ++p) {
        const float* f = film + (size_t)p * 4;
        float c[3] = { f[0] / f[3], f[1] / f[3], f[2] / f[3] };
        for (int k = 0; k < 3; ++k) {
            float v = c[k];
            if (enabled) {
                v = v * exposure;
                v = v * (1.0f + v / maxWhiteSqr) / (1.0f + v);
            }
            v = v != v ? 0.0f : fminf(fmaxf(v, 0.0f), 1.0f);
            uint32_t code = 0;
            for (int t = 0; t < 255; ++t) code += v >= srgbThresholds[t] ? 1u : 0u;
            out[(size_t)p * 4 + k] = (uint8_t)code;
        }
        out[(size_t)p * 4 + 3] = 255;
    }
}
