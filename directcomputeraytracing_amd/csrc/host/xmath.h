// xmath.h -- the DirectXMath subset the reference host code relies on
// (XMFLOAT*, BoundingBox center/extents arithmetic, XMVector3Transform,
// XMMatrixRotationRollPitchYaw, XMMatrixInverse), restated in scalar C++ with
// the SSE code path's operation order (no FMA; DirectXMath is not available on
// Linux, SURVEY.md §7 "Hard parts").
#pragma once

#include <cmath>
#include <cstdint>
#include <cstring>

namespace dcrt {

struct Float2 { float x = 0, y = 0; };
struct Float3 {
    float x = 0, y = 0, z = 0;
    Float3() = default;
    Float3(float a, float b, float c) : x(a), y(b), z(c) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    float& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
inline Float3 operator+(Float3 a, Float3 b) { return { a.x + b.x, a.y + b.y, a.z + b.z }; }
inline Float3 operator-(Float3 a, Float3 b) { return { a.x - b.x, a.y - b.y, a.z - b.z }; }
inline Float3 operator*(Float3 a, float s) { return { a.x * s, a.y * s, a.z * s }; }
inline Float3 operator*(Float3 a, Float3 b) { return { a.x * b.x, a.y * b.y, a.z * b.z }; }
inline float Dot(Float3 a, Float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Float3 Cross(Float3 a, Float3 b) { return { a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x }; }
inline float Length(Float3 a) { return std::sqrt(Dot(a, a)); }
// XMVectorMin / XMVectorMax on SSE: minps(a, b) = a < b ? a : b
inline float XMin(float a, float b) { return a < b ? a : b; }
inline float XMax(float a, float b) { return a > b ? a : b; }
inline Float3 VMin(Float3 a, Float3 b) { return { XMin(a.x, b.x), XMin(a.y, b.y), XMin(a.z, b.z) }; }
inline Float3 VMax(Float3 a, Float3 b) { return { XMax(a.x, b.x), XMax(a.y, b.y), XMax(a.z, b.z) }; }

// Row-major 4x4, row-vector convention (XMFLOAT4X4).
struct Float4x4 {
    float m[4][4];
    static Float4x4 Identity()
    {
        Float4x4 r; std::memset(r.m, 0, sizeof(r.m));
        r.m[0][0] = r.m[1][1] = r.m[2][2] = r.m[3][3] = 1.0f;
        return r;
    }
};
// XMFLOAT4X3: 4 rows of 3 (row-major on the host).
struct Float4x3 {
    float m[4][3];
    static Float4x3 Identity()
    {
        Float4x3 r; std::memset(r.m, 0, sizeof(r.m));
        r.m[0][0] = r.m[1][1] = r.m[2][2] = 1.0f;
        return r;
    }
    static Float4x3 From4x4(const Float4x4& a)
    {
        Float4x3 r;
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][j];
        return r;
    }
    Float4x4 To4x4() const
    {
        Float4x4 r = Float4x4::Identity();
        for (int i = 0; i < 4; ++i) for (int j = 0; j < 3; ++j) r.m[i][j] = m[i][j];
        return r;
    }
};

// XMVector3Transform (SSE order): r = z*r2 + r3; r = y*r1 + r; r = x*r0 + r
inline Float3 TransformPoint(Float3 v, const Float4x4& M)
{
    Float3 r;
    for (int c = 0; c < 3; ++c) {
        float t = v.z * M.m[2][c] + M.m[3][c];
        t = v.y * M.m[1][c] + t;
        t = v.x * M.m[0][c] + t;
        r[c] = t;
    }
    return r;
}
// XMVector3TransformNormal: r = z*r2; r = y*r1 + r; r = x*r0 + r
inline Float3 TransformNormal(Float3 v, const Float4x4& M)
{
    Float3 r;
    for (int c = 0; c < 3; ++c) {
        float t = v.z * M.m[2][c];
        t = v.y * M.m[1][c] + t;
        t = v.x * M.m[0][c] + t;
        r[c] = t;
    }
    return r;
}

inline Float4x4 Multiply(const Float4x4& a, const Float4x4& b)
{
    Float4x4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float t = a.m[i][0] * b.m[0][j];
            t = t + a.m[i][1] * b.m[1][j];
            t = t + a.m[i][2] * b.m[2][j];
            t = t + a.m[i][3] * b.m[3][j];
            r.m[i][j] = t;
        }
    return r;
}
inline Float4x4 Transpose(const Float4x4& a)
{
    Float4x4 r;
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) r.m[i][j] = a.m[j][i];
    return r;
}

// General 4x4 inverse by cofactors (XMMatrixInverse; exact for the diagonal and
// rigid transforms the loaders produce).
Float4x4 Inverse(const Float4x4& a, float* outDet = nullptr);

// XMScalarSinCos / XMVectorSinCos (one lane): DirectXMath's minimax sine and cosine.
void ScalarSinCos(float* s, float* c, float value);
void VectorSinCos(float* s, float* c, float value);
// XMMatrixRotationNormal (XMMatrixRotationAxis after its XMVector3Normalize).
Float4x4 RotationNormal(Float3 normalAxis, float angle);
// XMVector3Normalize
Float3 Normalize3(Float3 v);

// XMMatrixRotationRollPitchYawFromVector(pitch = x, yaw = y, roll = z): sines and cosines
// from XMVectorSinCos; the products of the three-factor entries are taken in the scalar
// (_XM_NO_INTRINSICS_) order -- the SSE path's order is not pinned.
Float4x4 RotationRollPitchYaw(float pitch, float yaw, float roll);

// MathHelper::MatrixRotationToRollPitchYall (MathHelper.cpp:9-25)
Float3 MatrixRotationToRollPitchYaw(const Float4x4& m);

// DirectX::BoundingBox (center / extents).
struct BoundingBox {
    Float3 center{ 0.0f, 0.0f, 0.0f };
    Float3 extents{ 1.0f, 1.0f, 1.0f };
};
// BoundingBox::CreateFromPoints(out, pt1, pt2)
inline BoundingBox BoxFromPoints(Float3 p1, Float3 p2)
{
    Float3 mn = VMin(p1, p2), mx = VMax(p1, p2);
    BoundingBox b;
    b.center = (mn + mx) * 0.5f;
    b.extents = (mx - mn) * 0.5f;
    return b;
}
// BoundingBox::CreateMerged
inline BoundingBox BoxMerged(const BoundingBox& b1, const BoundingBox& b2)
{
    Float3 mn = b1.center - b1.extents;
    mn = VMin(mn, b2.center - b2.extents);
    Float3 mx = b1.center + b1.extents;
    mx = VMax(mx, b2.center + b2.extents);
    BoundingBox b;
    b.center = (mn + mx) * 0.5f;
    b.extents = (mx - mn) * 0.5f;
    return b;
}
// BoundingBox::Transform: the 8 corners through M.
BoundingBox BoxTransform(const BoundingBox& box, const Float4x4& M);

}  // namespace dcrt
