// xmath.cpp -- see xmath.h.
#include "xmath.h"

#include <cfloat>

namespace dcrt {

Float4x4 Inverse(const Float4x4& a, float* outDet)
{
    // Cofactor expansion in double, rounded once to float: exact for the
    // diagonal / axis-permutation / translation matrices the loaders emit.
    double m[16], inv[16];
    for (int i = 0; i < 16; ++i) m[i] = a.m[i / 4][i % 4];
    inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] + m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
    inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] - m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
    inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] + m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
    inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] - m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
    inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] - m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
    inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] + m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
    inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] - m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
    inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] + m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
    inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] + m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
    inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] - m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
    inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] + m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
    inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] - m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
    inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] - m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
    inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] + m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
    inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] - m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
    inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] + m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
    const double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
    if (outDet) *outDet = (float)det;
    Float4x4 r;
    const double s = det != 0.0 ? 1.0 / det : 0.0;
    for (int i = 0; i < 16; ++i) {
        double v = inv[i] * s;
        r.m[i / 4][i % 4] = (float)(v == 0.0 ? 0.0 : v);
    }
    return r;
}

// DirectXMath's sine / cosine: the argument reduced to [-pi, pi] by its nearest multiple of
// 2pi, reflected into [-pi/2, pi/2] (sin(pi - y) = sin(y), cos(pi - y) = -cos(y)), then an
// 11-degree odd minimax polynomial for sin and a 10-degree even one for cos, Horner order,
// every step a separate float multiply and add (the reference builds for x64 SSE2: no FMA).
namespace {
constexpr float kXM2Pi = 6.283185307f, kXM1Div2Pi = 0.159154943f, kXMPi = 3.141592654f, kXMPiDiv2 = 1.570796327f;
void SinCosPoly(float y, float sign, float* s, float* c)
{
    const float y2 = y * y;
    *s = (((((-2.3889859e-08f * y2 + 2.7525562e-06f) * y2 - 0.00019840874f) * y2 + 0.0083333310f) * y2 - 0.16666667f) * y2 + 1.0f) * y;
    const float p = ((((-2.6051615e-07f * y2 + 2.4760495e-05f) * y2 - 0.0013888378f) * y2 + 0.041666638f) * y2 - 0.5f) * y2 + 1.0f;
    *c = p * sign;
}
}  // namespace

void ScalarSinCos(float* s, float* c, float value)
{
    // XMScalarSinCos: the quotient rounded half away from zero (int truncation of q +- 0.5)
    float q = kXM1Div2Pi * value;
    q = value >= 0.0f ? (float)(int)(q + 0.5f) : (float)(int)(q - 0.5f);
    float y = value - kXM2Pi * q;
    float sign = 1.0f;
    if (y > kXMPiDiv2) { y = kXMPi - y; sign = -1.0f; }
    else if (y < -kXMPiDiv2) { y = -kXMPi - y; sign = -1.0f; }
    SinCosPoly(y, sign, s, c);
}

void VectorSinCos(float* s, float* c, float value)
{
    // XMVectorSinCos, one lane: XMVectorModAngles rounds the quotient half to even (SSE2
    // XMVectorRound: add and subtract 2^23 carrying the value's sign, for |q| <= 2^23), then
    // subtracts round * 2pi; the reflection keeps |x| <= pi/2 and maps the rest to +-pi - x.
    float q = value * kXM1Div2Pi;
    if (std::fabs(q) <= 8388608.0f) {
        const float magic = std::copysign(8388608.0f, q);
        volatile float t = q + magic;   // (two roundings, as addps / subps)
        q = t - magic;
    }
    float x = value - q * kXM2Pi;
    const float reflected = std::copysign(kXMPi, x) - x;
    const bool keep = std::fabs(x) <= kXMPiDiv2;
    SinCosPoly(keep ? x : reflected, keep ? 1.0f : -1.0f, s, c);
}

Float4x4 RotationNormal(Float3 n, float angle)
{
    // XMMatrixRotationNormal (SSE2): t = 1 - cos; V0 = t * (y, z, x) * (z, x, y);
    // R2 = t * n * n + cos; R1 = sin * n + V0; R0 = V0 - sin * n
    float s, c;
    ScalarSinCos(&s, &c, angle);
    const float t = 1.0f - c;
    const Float3 v0((t * n.y) * n.z, (t * n.z) * n.x, (t * n.x) * n.y);
    const Float3 r2((t * n.x) * n.x + c, (t * n.y) * n.y + c, (t * n.z) * n.z + c);
    const Float3 r1(s * n.x + v0.x, s * n.y + v0.y, s * n.z + v0.z);
    const Float3 r0(v0.x - s * n.x, v0.y - s * n.y, v0.z - s * n.z);
    Float4x4 M = Float4x4::Identity();
    M.m[0][0] = r2.x; M.m[0][1] = r1.z; M.m[0][2] = r0.y;
    M.m[1][0] = r0.z; M.m[1][1] = r2.y; M.m[1][2] = r1.x;
    M.m[2][0] = r1.y; M.m[2][1] = r0.x; M.m[2][2] = r2.z;
    return M;
}

Float3 Normalize3(Float3 v)
{
    // XMVector3Normalize (SSE2): v / sqrt((x*x + y*y) + z*z); a zero length gives 0, an
    // infinite one NaN
    const float len = std::sqrt(Dot(v, v));
    if (len == 0.0f) return Float3(0.0f, 0.0f, 0.0f);
    if (std::isinf(Dot(v, v))) return Float3(NAN, NAN, NAN);
    return Float3(v.x / len, v.y / len, v.z / len);
}

Float4x4 RotationRollPitchYaw(float pitch, float yaw, float roll)
{
    float cp, sp, cy, sy, cr, sr;
    VectorSinCos(&sp, &cp, pitch);
    VectorSinCos(&sy, &cy, yaw);
    VectorSinCos(&sr, &cr, roll);
    Float4x4 M;
    M.m[0][0] = cr * cy + sr * sp * sy;
    M.m[0][1] = sr * cp;
    M.m[0][2] = sr * sp * cy - cr * sy;
    M.m[0][3] = 0.0f;
    M.m[1][0] = cr * sp * sy - sr * cy;
    M.m[1][1] = cr * cp;
    M.m[1][2] = sr * sy + cr * sp * cy;
    M.m[1][3] = 0.0f;
    M.m[2][0] = cp * sy;
    M.m[2][1] = -sp;
    M.m[2][2] = cp * cy;
    M.m[2][3] = 0.0f;
    M.m[3][0] = 0.0f; M.m[3][1] = 0.0f; M.m[3][2] = 0.0f; M.m[3][3] = 1.0f;
    return M;
}

Float3 MatrixRotationToRollPitchYaw(const Float4x4& m)
{
    const float cy = std::sqrt(m.m[2][2] * m.m[2][2] + m.m[2][0] * m.m[2][0]);
    Float3 r;
    r.x = std::atan2(-m.m[2][1], cy);
    if (cy > 16.0f * FLT_EPSILON) {
        r.y = std::atan2(m.m[2][0], m.m[2][2]);
        r.z = std::atan2(m.m[0][1], m.m[1][1]);
    } else {
        r.y = 0.0f;
        r.z = std::atan2(-m.m[1][0], m.m[0][0]);
    }
    return r;
}

BoundingBox BoxTransform(const BoundingBox& box, const Float4x4& M)
{
    static const float kOffsets[8][3] = { { -1, -1, 1 }, { 1, -1, 1 }, { 1, 1, 1 }, { -1, 1, 1 },
                                          { -1, -1, -1 }, { 1, -1, -1 }, { 1, 1, -1 }, { -1, 1, -1 } };
    Float3 mn, mx;
    for (int i = 0; i < 8; ++i) {
        Float3 corner(box.extents.x * kOffsets[i][0] + box.center.x, box.extents.y * kOffsets[i][1] + box.center.y,
                      box.extents.z * kOffsets[i][2] + box.center.z);
        corner = TransformPoint(corner, M);
        if (i == 0) { mn = corner; mx = corner; }
        else { mn = VMin(mn, corner); mx = VMax(mx, corner); }
    }
    BoundingBox out;
    out.center = (mn + mx) * 0.5f;
    out.extents = (mx - mn) * 0.5f;
    return out;
}

}  // namespace dcrt
