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

Float4x4 RotationRollPitchYaw(float pitch, float yaw, float roll)
{
    const float cp = std::cos(pitch), sp = std::sin(pitch);
    const float cy = std::cos(yaw), sy = std::sin(yaw);
    const float cr = std::cos(roll), sr = std::sin(roll);
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
