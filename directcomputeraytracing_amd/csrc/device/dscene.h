// dscene.h -- HBM-resident scene and its device-side accessors: two-level BVH
// traversal (BVHAccel.inc.hlsl:85-369), ray/box and ray/triangle tests
// (RayPrimitiveIntersect.inc.hlsl), hit reconstruction (HitShader.inc.hlsl,
// RayTracingCommon.inc.hlsl:88-116), lights (Light.inc.hlsl) and texture
// emulation (BxDFTextures.inc.hlsl, D3D12 SampleLevel at LOD 0).
#pragma once

#include "../../../include/dcrt.h"
#include "dmath.h"

namespace dcrt {
namespace dev {

// Scene capabilities a MATERIAL variant is compiled for (material_kernel<CAPS>). The host
// (dcrt_tracer::UploadScene) computes what the uploaded scene uses -- material types,
// multiscattering, textures, light types, an environment cube -- and launches the
// smallest compiled variant that covers it (kCapAll otherwise). A variant states its
// exclusions to the compiler (__builtin_assume) and so drops the code and the live
// registers of paths the scene cannot take; every path the scene does take is the same
// arithmetic in every variant, so results do not depend on the variant.
constexpr uint32_t kCapMatDiffuse = 1u << 0;       // bit = 1 << DCRT_MATERIAL_TYPE_*
constexpr uint32_t kCapMatPlastic = 1u << 1;
constexpr uint32_t kCapMatConductor = 1u << 2;
constexpr uint32_t kCapMatDielectric = 1u << 3;
constexpr uint32_t kCapMatThin = 1u << 4;
constexpr uint32_t kCapMultiscatter = 1u << 5;     // DCRT_MATERIAL_FLAG_MULTISCATTERING on some material
constexpr uint32_t kCapTextures = 1u << 6;         // albedo textures or the roughness checkerboard
constexpr uint32_t kCapLightPoint = 1u << 7;       // bit = DCRT_LIGHT_FLAGS_* << 7
constexpr uint32_t kCapLightMesh = 1u << 8;
constexpr uint32_t kCapLightDirectional = 1u << 9;
constexpr uint32_t kCapLightEnv = 1u << 10;
constexpr uint32_t kCapEnvCube = 1u << 11;
constexpr uint32_t kCapAll = (1u << 12) - 1u;
constexpr uint32_t kCapMaterialsMask = 0x1Fu;
constexpr uint32_t kCapLightShift = 7;
// Opaque delta-lit scenes (the Cornell configs): diffuse / plastic / conductor
// materials without multiscattering or textures, point and directional lights.
constexpr uint32_t kCapOpaqueDelta = kCapMatDiffuse | kCapMatPlastic | kCapMatConductor | kCapLightPoint | kCapLightDirectional;

// Light-type flags a variant admits (the reference's light flags are one type bit each).
template <uint32_t CAPS>
DEV void assume_light_caps(uint32_t flags)
{
    if constexpr (CAPS != kCapAll) __builtin_assume((flags & ~((CAPS >> kCapLightShift) & 0xFu) & 0xFu) == 0u);
}

struct TextureDesc {
    uint32_t width, height, format, offset;   // offset into the texel blob (bytes)
};

// Everything a kernel needs about the scene, passed by value (kernel argument).
struct DeviceScene {
    const float4* nodes;          // 2 x float4 per BVHNode (min.xyz,max.x | max.yz,right,misc)
    const float4* triVerts;       // 3 x float4 per triangle: BLAS positions (q0.w degenerate flag, q1.w material id bits)
    const float4* triShade;       // 6 x float4 per triangle: per vertex (normal.xyz, tangent.x), (tangent.yz, uv)
    const dcrt_vertex* vertices;
    const uint32_t* triangles;
    const uint32_t* materialIds;
    const float4* transforms;     // 3 x float4 per matrix, 2N matrices (forward, inverse)
    const uint32_t* instanceLightIndices;
    const uint32_t* instanceFlags;
    const uint32_t* instanceIdentity;   // 1: inverse transform is exactly the identity
    const uint32_t* overrides;
    const dcrt_material* materials;
    const dcrt_light* lights;
    const TextureDesc* textures;
    const uint8_t* texels;
    const float* srgbTable;       // 256 entries
    const float* envCube;         // 6 * n * n * 3, or nullptr
    const uint16_t* lutBrdf;
    const uint16_t* lutBrdfAvg;
    const uint16_t* lutBrdfDielectric;
    const uint16_t* lutBrdfDielectricAvg;
    const uint16_t* lutBsdf;
    const uint16_t* lutBsdfAvg;
    uint32_t instanceCount;
    uint32_t nodeCount;
    uint32_t triangleCount;
    uint32_t envCubeSize;
    uint32_t stackSize;           // per-lane traversal stack entries
    uint32_t stackRows;           // LDS stack rows per lane: stackSize + 2, or ringRows (RING kernels)
    // RING kernels (persistent_trace): the LDS holds a window of ringRows (a power of two, >= 8) of
    // the lane's stack as a ring -- entry e at row e mod ringRows -- and the entries below the
    // window live in `spill`, a [stackSize][lanes of the grid] column per lane (entry e of global
    // lane gl at spill[(e - 1) * lanes + gl]). 0: the whole stack in LDS.
    uint32_t ringRows;
    uint32_t* spill;
    uint32_t cachedNodes;         // nodes [0, cachedNodes) are mirrored in LDS (scene_cache_load)
    uint32_t cachedTris;          // triVerts of triangles [0, cachedTris) likewise, after the nodes
    uint32_t cachedInstances;     // 0, or instanceCount: every inverse transform + identity flag, after the triangles
    uint32_t singlePrimLeaves;    // 1: every BLAS leaf holds exactly one triangle (BVHAccel.cpp's builder always does)
    uint32_t pairLayout;          // node order: 0 PackBVH's (flat scene), 1 child pairs (kLayoutPairs)
    uint32_t skipRoot;            // 1: trav_skip_root at a ray's start (the non-counting trav_visit kernels)
    // MATERIAL's LDS scene copy (material_kernel<CAPS, true>, small scenes): the material and
    // light counts it copies (0 when the variant is not used)
    uint32_t ldsMaterials, ldsLights;
};

// MATERIAL's LDS scene copy, in 16-B units: triVerts (3 T), triShade (6 T), the forward
// instance transforms (3 I), then 4-B words: instance light indices (I), overrides (I),
// materials (13 M), lights (7 L). Bytes for T triangles, I instances, M materials, L lights.
__host__ __device__ inline uint32_t material_lds_bytes(uint32_t T, uint32_t I, uint32_t M, uint32_t L)
{
    return 16u * (9u * T + 3u * I) + 4u * (2u * I + 13u * M + 7u * L);
}

// Node orders on the device. kLayoutFlat is PackBVH's depth-first order, as in the flat
// scene: an interior node's left child is node + 1 and its `right` field the right child.
// kLayoutPairs (tracer.hip PairLayout, taken for scenes beyond an XCD's L2: the pair
// traversal's kernels) puts the two children side by side -- one 64-B line, fetched together
// when trav_visit_pair expands a node -- with `right` holding the left child's index, and the
// levels nearest the roots first (the prefix the LDS scene cache holds). kLayoutScene reads
// the order from the scene (kernels that serve either). The order changes no result.
enum : int { kLayoutFlat = 0, kLayoutPairs = 1, kLayoutScene = 2 };
// An interior node's children as packed references (with the node's BLAS bit); `right` is
// its record's `right` field (or the packed reference to it)
template <int LAYOUT>
DEV void node_children(const DeviceScene& sc, uint32_t node, uint32_t right, uint32_t* left, uint32_t* rightChild)
{
    const uint32_t r = right | (node & 0x80000000u);
    const bool pairs = LAYOUT == kLayoutPairs || (LAYOUT == kLayoutScene && sc.pairLayout != 0u);
    *left = pairs ? r : node + 1u;
    *rightChild = pairs ? r + 1u : r;
}

// LDS scene cache of the traversal kernels: after the per-lane stacks ([stackSize + 2]
// x blockDim words, see stack_at) the block holds a copy of the first cachedNodes BVH nodes and the
// first cachedTris pre-gathered triangles (the whole BVH and mesh of a small scene; the
// levels nearest the TLAS and BLAS roots of a large one, which the device node order puts
// first), so most node and triangle fetches are ds_read_b128 instead of vector-memory
// gathers through the texture path.

DEV float4* scene_cache(const DeviceScene& sc, uint32_t* stackMem, uint32_t shift)
{
    return (float4*)(stackMem + (sc.stackRows << shift));
}
// 16-B loads through address-space-qualified pointers (ds_read_b128 / global_load_dwordx4):
// where a node may come from the LDS cache or from memory, the two reads of one generic
// pointer became a flat load, whose waits count both counters. (The LDS offset is the low 32
// bits of a generic LDS address.)
typedef float LoadF4 __attribute__((ext_vector_type(4)));
DEV float4 lds_load4(const float4* genericLds, uint32_t i)
{
    const __attribute__((address_space(3))) LoadF4* p = (const __attribute__((address_space(3))) LoadF4*)(uint32_t)(uintptr_t)genericLds;
    const LoadF4 v = p[i];
    return make_float4(v.x, v.y, v.z, v.w);
}
DEV uint64_t global_load_u64(const uint64_t* g, size_t i)
{
    const __attribute__((address_space(1))) uint64_t* p = (const __attribute__((address_space(1))) uint64_t*)(uintptr_t)g;
    return p[i];
}
typedef float LoadF2 __attribute__((ext_vector_type(2)));
DEV float2 global_load2(const float2* g, size_t i)
{
    const __attribute__((address_space(1))) LoadF2* p = (const __attribute__((address_space(1))) LoadF2*)(uintptr_t)g;
    const LoadF2 v = p[i];
    return make_float2(v.x, v.y);
}
DEV float4 global_load4(const float4* g, size_t i)
{
    const __attribute__((address_space(1))) LoadF4* p = (const __attribute__((address_space(1))) LoadF4*)(uintptr_t)g;
    const LoadF4 v = p[i];
    return make_float4(v.x, v.y, v.z, v.w);
}
// Triangles of the cache-only variant (ALL_CACHED kernels) are stored three times, once
// per watertight-test axis permutation: copy z holds every vertex as (v[z+1], v[z+2], v[z])
// (mod 3) -- the (kx, ky, kz) of a ray whose dominant axis is z -- so the test reads its
// permuted coordinates instead of selecting them.
constexpr uint32_t kRotTriFloat4 = 9;   // float4 per triangle: 3 permutations x 3 vertices
template <bool ROTATED>
DEV uint32_t cache_tri_float4() { return ROTATED ? kRotTriFloat4 : 3u; }

// Every thread of the block: fill the cache, then a barrier.
template <bool ROTATED = false>
DEV void scene_cache_load(const DeviceScene& sc, uint32_t* stackMem, uint32_t shift)
{
    float4* c = scene_cache(sc, stackMem, shift);
    const uint32_t nn = sc.cachedNodes * 2u, nt = sc.cachedTris * cache_tri_float4<ROTATED>();
    for (uint32_t i = threadIdx.x; i < nn; i += blockDim.x) c[i] = sc.nodes[i];
    for (uint32_t i = threadIdx.x; i < nt; i += blockDim.x) {
        if (ROTATED) {
            const uint32_t tri = i / kRotTriFloat4, r = i - tri * kRotTriFloat4, z = r / 3u, k = r - z * 3u;
            const float4 q = sc.triVerts[(size_t)tri * 3 + k];
            const float v[3] = {q.x, q.y, q.z};
            const uint32_t x = z == 2u ? 0u : z + 1u, y = x == 2u ? 0u : x + 1u;
            c[nn + i] = make_float4(v[x], v[y], v[z], q.w);
        } else {
            c[nn + i] = sc.triVerts[i];
        }
    }
    // per instance: the inverse float4x3 (3 x float4), then (identity flag, 0, 0, 0)
    for (uint32_t i = threadIdx.x; i < sc.cachedInstances * 4u; i += blockDim.x) {
        const uint32_t inst = i >> 2, k = i & 3u;
        c[nn + nt + i] = k < 3u ? sc.transforms[(size_t)(sc.instanceCount + inst) * 3 + k]
                                : make_float4(__uint_as_float(sc.instanceIdentity[inst]), 0.0f, 0.0f, 0.0f);
    }
    __syncthreads();
}

// ---- ray / primitive tests ----------------------------------------------------
struct Shear {
    int kx, ky, kz;
    float sx, sy, sz;
    float ox, oy, oz;     // the ray origin permuted, (o[kx], o[ky], o[kz]) (rotated-triangle test)
};
// inv = (1/d.x, 1/d.y, 1/d.z) as the slab test already holds it: the shear's 1/d[kz] is
// the same IEEE quotient, so it is selected instead of divided again at every leaf
DEV Shear make_shear(V3 d, V3 inv)   // BVHAccel.inc.hlsl:72-83
{
    Shear s;
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int z = ax >= ay ? 0 : 1;
    z = (z == 0 ? ax : ay) >= az ? z : 2;
    int x = z + 1; x = x == 3 ? 0 : x;
    int y = x + 1; y = y == 3 ? 0 : y;
    s.kx = x; s.ky = y; s.kz = z;
    const float invZ = comp(inv, z);
    s.sx = -comp(d, x) * invZ;
    s.sy = -comp(d, y) * invZ;
    s.sz = invZ;
    s.ox = 0.0f; s.oy = 0.0f; s.oz = 0.0f;
    return s;
}
DEV Shear make_shear_rot(V3 d, V3 o, V3 inv)
{
    Shear s = make_shear(d, inv);
    s.ox = comp(o, s.kx); s.oy = comp(o, s.ky); s.oz = comp(o, s.kz);
    return s;
}

// Watertight test (RayPrimitiveIntersect.inc.hlsl:8-70).
// `degenerate` = (|cross(v1-v0, v2-v0)|^2 == 0), precomputed per triangle at upload
// with the same arithmetic (build_tri_verts_kernel) and stored in triVerts[3t].w.
DEV bool tri_watertight(V3 o, const Shear& sh, float tMin, float tMax, V3 v0, V3 v1, V3 v2, bool degenerate,
                        float* t, float* u, float* v, bool* backface)
{
    *t = 0.0f; *u = 0.0f; *v = 0.0f; *backface = false;
    if (degenerate) return false;
    const V3 a = v0 - o, b = v1 - o, c = v2 - o;
    float p0x = comp(a, sh.kx), p0y = comp(a, sh.ky), p0z = comp(a, sh.kz);
    float p1x = comp(b, sh.kx), p1y = comp(b, sh.ky), p1z = comp(b, sh.kz);
    float p2x = comp(c, sh.kx), p2y = comp(c, sh.ky), p2z = comp(c, sh.kz);
    p0x = p0x + sh.sx * p0z; p0y = p0y + sh.sy * p0z;
    p1x = p1x + sh.sx * p1z; p1y = p1y + sh.sy * p1z;
    p2x = p2x + sh.sx * p2z; p2y = p2y + sh.sy * p2z;
    const float e0 = p1x * p2y - p2x * p1y;
    const float e1 = p2x * p0y - p0x * p2y;
    const float e2 = p0x * p1y - p1x * p0y;
    if ((e0 < 0.0f || e1 < 0.0f || e2 < 0.0f) && (e0 > 0.0f || e1 > 0.0f || e2 > 0.0f)) return false;
    const float det = e0 + e1 + e2;
    p0z = p0z * sh.sz; p1z = p1z * sh.sz; p2z = p2z * sh.sz;
    const float tScaled = e0 * p0z + e1 * p1z + e2 * p2z;
    const float invDet = rcp_ieee(det);
    *t = tScaled * invDet;
    *u = e1 * invDet;
    *v = e2 * invDet;
    // fsign(sz) * det < 0 (the reference's form) as a sign-bit test: the two differ only
    // for det = +-0 or NaN, where the test below rejects the hit and `backface` is unused
    *backface = sh.sz != 0.0f && (int)(asu(sh.sz) ^ asu(det)) < 0;
    return det != 0.0f && *t >= tMin && *t < tMax;
}

// The same test on a rotated triangle copy (vertices already (v[kx], v[ky], v[kz])) and
// the permuted origin in the shear: identical operations, no component selects.
DEV bool tri_watertight_rot(const Shear& sh, float tMin, float tMax, float4 q0, float4 q1, float4 q2,
                            float* t, float* u, float* v, bool* backface)
{
    *t = 0.0f; *u = 0.0f; *v = 0.0f; *backface = false;
    // (the degenerate flag q0.w is tested with the edge signs below, not first: an early
    // exit on it made the three vertex reads wait for a separate read of q0.w)
    float p0x = q0.x - sh.ox, p0y = q0.y - sh.oy, p0z = q0.z - sh.oz;
    float p1x = q1.x - sh.ox, p1y = q1.y - sh.oy, p1z = q1.z - sh.oz;
    float p2x = q2.x - sh.ox, p2y = q2.y - sh.oy, p2z = q2.z - sh.oz;
    p0x = p0x + sh.sx * p0z; p0y = p0y + sh.sy * p0z;
    p1x = p1x + sh.sx * p1z; p1y = p1y + sh.sy * p1z;
    p2x = p2x + sh.sx * p2z; p2y = p2y + sh.sy * p2z;
    const float e0 = p1x * p2y - p2x * p1y;
    const float e1 = p2x * p0y - p0x * p2y;
    const float e2 = p0x * p1y - p1x * p0y;
    if (q0.w != 0.0f || ((e0 < 0.0f || e1 < 0.0f || e2 < 0.0f) && (e0 > 0.0f || e1 > 0.0f || e2 > 0.0f))) return false;
    const float det = e0 + e1 + e2;
    p0z = p0z * sh.sz; p1z = p1z * sh.sz; p2z = p2z * sh.sz;
    const float tScaled = e0 * p0z + e1 * p1z + e2 * p2z;
    const float invDet = rcp_ieee(det);
    *t = tScaled * invDet;
    *u = e1 * invDet;
    *v = e2 * invDet;
    // fsign(sz) * det < 0 (the reference's form) as a sign-bit test: the two differ only
    // for det = +-0 or NaN, where the test below rejects the hit and `backface` is unused
    *backface = sh.sz != 0.0f && (int)(asu(sh.sz) ^ asu(det)) < 0;
    return det != 0.0f && *t >= tMin && *t < tMax;
}

// Moller-Trumbore (RayPrimitiveIntersect.inc.hlsl:72-103).
DEV bool tri_moller(V3 o, V3 d, float tMin, float tMax, V3 v0, V3 v1, V3 v2, float* t, float* u, float* v, bool* backface)
{
    const V3 v0v1 = v1 - v0, v0v2 = v2 - v0;
    const V3 pvec = cross(d, v0v2);
    const float det = dot(v0v1, pvec);
    const float invDet = rcp_ieee(det);
    const V3 tvec = o - v0;
    *u = dot(tvec, pvec) * invDet;
    const V3 qvec = cross(tvec, v0v1);
    *v = dot(d, qvec) * invDet;
    *t = dot(v0v2, qvec) * invDet;
    *backface = det > -1e-10f;
    return fabsf(det) >= 1e-10f && *u >= 0.0f && *u <= 1.0f && *v >= 0.0f && *u + *v <= 1.0f && *t >= tMin && *t < tMax;
}

DEV V3 inv_dir(V3 d) { return mk(rcp_ieee(d.x), rcp_ieee(d.y), rcp_ieee(d.z)); }

struct HitRecord {
    float t, u, v;
    uint32_t tri;        // bit 31 = backface
    uint32_t inst;
};

// Two-level traversal (BVHIntersectNoInterp / BVHIntersect, BVHAccel.inc.hlsl:85-369)
// as a resumable per-lane state machine: one call = one node visit in the
// reference's order (test-on-visit, near child first by the split axis' direction
// sign, far child pushed), so hits, tie-breaking and the SRayTraversalCounters
// counts are the reference's. Kernels interleave steps with refills of finished
// lanes (persistent "while-while" with per-lane dynamic ray fetch), so a wave64
// does not idle until its slowest ray is done.
// The per-lane stack lives in LDS: column `lane` of a [stackSize][blockDim] array
// (consecutive lanes on consecutive banks); blockDim is a power of two and entry i of
// a lane sits at lds[i << shift], shift = log2(blockDim) (a shift, not a 32-bit multiply).
struct TraversalStats {
    uint32_t nodes;   // iterationCounter (BVHAccel.inc.hlsl:121)
    uint32_t tris;    // triangle tests
    uint32_t blas;    // TLAS -> BLAS entries
    uint32_t maxNodes;   // (merged cast, per ray kind) the longest ray's node visits
#ifdef DCRT_PHASE_CLOCKS
    // diagnostic build: node visits served by the LDS scene cache; pushes onto a stack
    // already 4 / 8 / 12 entries deep
    uint32_t cached, deep4, deep8, deep12;
#endif
};

struct TravState {
    V3 o, d, invW;        // world ray and 1/d (restored on BLAS -> TLAS without dividing again)
    // ray in the current space (world or instance): direction ld, origin and 1/d
    V3 ld;
    V3 lo_, inv_;
    DEV V3 lo() const { return lo_; }
    DEV V3 inv() const { return inv_; }
    DEV void set_space(V3 o, V3 i) { lo_ = o; inv_ = i; }
    float tMin, tMax;
    uint32_t node;        // node index | 0x80000000 in a BLAS (the stack entries' packing)
    uint32_t sp;          // stack entries x stride (bytes): see stack_at
    uint32_t base;        // RING kernels: entries spilled below the LDS window, x stride (ring_maintain)
    uint32_t inst;
    uint32_t leafRef, leafMisc;   // the visited leaf whose work is pending (parked; not kept with ALL_CACHED)
    bool found, parked, noZero;   // noZero: no component of o, d is +-0
    bool anyHit;          // merged cast kernel: this lane's ray is a shadow ray (first hit ends it)
    // trav_visit_pair: `node` is a hit interior node whose children are tested next
    // (expand), its right child (with the BLAS bit) and near-child choice
    bool expand, expNeg;
    uint32_t expRight;
    // Near/far choice of the current space: bit a = (ld[a] < 0) for the axes a = 0..2,
    // bit 3 = front-to-back order on (0: the whole mask is 0, near child = node + 1 always)
    uint32_t negMask;
    Shear sh;
    HitRecord hit;
    // ALLOW_ANYHIT_SHADER only (dead, and removed by the compiler, otherwise)
    float opacitySample;
    uint32_t matOverride;     // the current instance's material override
    bool opaque;              // the current instance's INSTANCE_FLAG_OPAQUE
};

// Slab test on PackBVH's node record (min.xyz, max.x) (max.yz, right, misc).
// (IDENT: the world ray's o / 1/d in every space -- see trav_visit)
DEV bool ray_aabb_raw(V3 o, V3 inv, float tMin, float tMax, float4 a, float4 b)
{
    const float tx0 = (a.x - o.x) * inv.x;
    const float tx1 = (a.w - o.x) * inv.x;
    float t0 = fminf(tx0, tx1);
    float t1 = fmaxf(tx0, tx1);
    const float ty0 = (a.y - o.y) * inv.y;
    const float ty1 = (b.x - o.y) * inv.y;
    t0 = fmaxf(t0, fminf(ty0, ty1));
    t1 = fminf(t1, fmaxf(ty0, ty1));
    const float tz0 = (a.z - o.z) * inv.z;
    const float tz1 = (b.y - o.z) * inv.z;
    t0 = fmaxf(t0, fminf(tz0, tz1));
    t1 = fminf(t1, fmaxf(tz0, tz1));
    return (t1 >= t0) & (t0 < tMax) & (t1 >= tMin);
}
DEV bool ray_aabb(const TravState& s, float4 a, float4 b)
{
    const float tMin = s.tMin, tMax = s.tMax;
    const V3 o = s.lo(), inv = s.inv();
    const float tx0 = (a.x - o.x) * inv.x;
    const float tx1 = (a.w - o.x) * inv.x;
    float t0 = fminf(tx0, tx1);
    float t1 = fmaxf(tx0, tx1);
    const float ty0 = (a.y - o.y) * inv.y;
    const float ty1 = (b.x - o.y) * inv.y;
    t0 = fmaxf(t0, fminf(ty0, ty1));
    t1 = fminf(t1, fmaxf(ty0, ty1));
    const float tz0 = (a.z - o.z) * inv.z;
    const float tz1 = (b.y - o.z) * inv.z;
    t0 = fmaxf(t0, fminf(tz0, tz1));
    t1 = fminf(t1, fmaxf(tz0, tz1));
    return (t1 >= t0) & (t0 < tMax) & (t1 >= tMin);   // (bitwise: no exec-mask branch per node)
}

// BVHAccel.inc.hlsl's near/far test `dir[axis] < 0` for all three axes at once, kept per
// space (world, instance) so a node visit selects one bit instead of comparing three signs
DEV uint32_t neg_mask(V3 d, uint32_t current)
{
    return (current & 8u) ? 8u | (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u) : 0u;
}

// f2b = false (DCRT_FEATURE_NO_FRONT_TO_BACK): near child is always node + 1
DEV void trav_init(TravState& s, V3 o, V3 d, float tMin, float tMax, bool f2b = true)
{
    s.negMask = neg_mask(d, f2b ? 8u : 0u);
    s.o = o; s.d = d; s.invW = inv_dir(d);
    s.ld = d; s.set_space(o, inv_dir(d));
    s.tMin = tMin; s.tMax = tMax;
    s.node = 0; s.sp = 0; s.base = 0; s.inst = 0;
    s.leafRef = 0; s.leafMisc = 0;
    s.found = false; s.parked = false; s.anyHit = false;
    s.expand = false; s.expNeg = false; s.expRight = 0;
    s.noZero = o.x != 0.0f && o.y != 0.0f && o.z != 0.0f && d.x != 0.0f && d.y != 0.0f && d.z != 0.0f;
    s.hit.t = 0.0f; s.hit.u = 0.0f; s.hit.v = 0.0f; s.hit.tri = 0u; s.hit.inst = 0u;
    s.opacitySample = 0.0f; s.matOverride = DCRT_INSTANCE_MATERIAL_OVERRIDE_NONE; s.opaque = false;
}

DEV void sample_texture_wrap(const DeviceScene& s, uint32_t index, float u, float v, float* out);

// AnyHitShader (HitShader.inc.hlsl:86-113): a hit on a non-opaque instance counts only
// when the ray's opacity sample is below the material's (texture-modulated) opacity.
DEV bool any_hit_shader(const DeviceScene& sc, uint32_t tri, uint32_t ov, float u, float v, float opacitySample)
{
    const uint32_t mid = ov != DCRT_INSTANCE_MATERIAL_OVERRIDE_NONE ? ov : sc.materialIds[tri];
    const dcrt_material& m = sc.materials[mid];
    float opacity = m.opacity;
    if (m.opacity_texture_index != -1) {
        const dcrt_vertex& V0 = sc.vertices[sc.triangles[tri * 3]];
        const dcrt_vertex& V1 = sc.vertices[sc.triangles[tri * 3 + 1]];
        const dcrt_vertex& V2 = sc.vertices[sc.triangles[tri * 3 + 2]];
        // VectorBaryCentric2 (Math.inc.hlsl:23-33), then texTiling
        float r1x = V1.texcoord[0] - V0.texcoord[0], r1y = V1.texcoord[1] - V0.texcoord[1];
        float r2x = V2.texcoord[0] - V0.texcoord[0], r2y = V2.texcoord[1] - V0.texcoord[1];
        r1x = r1x * u; r1y = r1y * u; r2x = r2x * v; r2y = r2y * v;
        r1x = r1x + V0.texcoord[0]; r1y = r1y + V0.texcoord[1];
        float tcx = r1x + r2x, tcy = r1y + r2y;
        tcx = tcx * m.tex_tiling[0]; tcy = tcy * m.tex_tiling[1];
        float rgba[4];
        sample_texture_wrap(sc, (uint32_t)m.opacity_texture_index, tcx, tcy, rgba);
        opacity = opacity * rgba[0];
    }
    return opacitySample < opacity;
}

// Per-lane traversal stack in LDS: row r of a lane's column sits at byte offset
// r * stride (stride = 4 * blockDim: consecutive lanes on consecutive banks). With
// `count` entries (sp = count * stride) the top entry is row count and a push goes to
// row count + 1; row 0 (read as the top of an empty stack) and row stackSize + 1 (the
// branch-free push of a full stack) are spares whose contents nothing uses.
DEV uint32_t& stack_at(uint32_t* lds, uint32_t byteOffset) { return *(uint32_t*)((char*)lds + byteOffset); }
// ALL_CACHED kernels run 256-thread workgroups (tracer.hip): a compile-time stride
// becomes the ds_write's immediate offset
template <bool ALL_CACHED>
DEV uint32_t stack_stride(uint32_t shift) { return ALL_CACHED ? 1024u : 4u << shift; }
// The LDS row of stack position `byteOffset` (entries x stride): itself, or in a RING kernel the
// position modulo the window (sc.ringRows rows; a power of two, so one AND with a uniform mask)
template <bool RING>
DEV uint32_t stack_row(const DeviceScene& sc, uint32_t byteOffset, uint32_t shift)
{
    return RING ? byteOffset & ((sc.ringRows << (shift + 2u)) - 1u) : byteOffset;
}

// Pop the next node (BVHAccel.inc.hlsl stack pop); true when the stack is empty.
template <bool IDENT = false, bool RING = false>
DEV bool trav_pop(const DeviceScene& sc, TravState& s, uint32_t* lds, uint32_t stride, uint32_t shift)
{
    if (s.sp == 0u) return true;
    const uint32_t packed = stack_at(lds, stack_row<RING>(sc, s.sp, shift));
    s.sp -= stride;
    s.expand = false;
    const bool restore = !IDENT && (int)s.node < 0 && (int)packed >= 0;   // BLAS -> TLAS
    s.node = packed;
    if (restore) {
        // component-wise: a struct copy inside the state becomes an alloca-local
        // memcpy that keeps SROA from promoting the state to registers
        s.ld = mk(s.d.x, s.d.y, s.d.z);
        s.set_space(s.o, s.invW);
        s.negMask = neg_mask(s.d, s.negMask);
    }
    return false;
}

// Phase A: visit one node (iterationCounter). A missed node pops; an interior node
// descends to the near child and pushes the far one; a leaf (TLAS or BLAS) parks
// the lane with its work pending. Returns true when the ray is finished.
// Written without divergent branches: the push always stores (slot `count`, or the
// spare slot `stackSize` past the end, which nothing reads), the pop always loads
// the top, and selects pick the outcome; the lanes of a wave stay convergent.
// ALL_CACHED: the whole BVH and every triangle sit in the LDS scene cache (small scenes),
// so node and triangle fetches are plain ds_read_b128 (no FLAT select, no global path).
// ENTER (the cache-only, non-opacity kernels): a hit TLAS leaf of an instance whose inverse is
// exactly the identity (misc bit 0, set at upload in the device node copy: a leaf's split-axis
// bits are otherwise unused) enters its BLAS here instead of parking for phase B -- for a ray
// with no zero component that entry changes nothing but the node and the instance (trav_leaf's
// identity branch), and the BLAS root is the next node visited either way, so the visits, the
// BLAS-entry count and the hits are the same.
constexpr uint32_t kMiscIdentityLeaf = 1u;
// IDENT (cache-only kernels of scenes whose instances all have exactly the identity inverse, every
// OBJ scene): no instance space is kept. The instance-space ray of such an instance is the world
// ray with -0 components turned into +0 (x*1 + y*0 + z*0 + w*0), and that changes no box test's
// outcome -- a zero direction component gives 1/d = +-inf, and with either sign the slab is
// (-inf, +inf) when the origin lies strictly inside it and empty otherwise; a -0 origin or
// plane coordinate changes only the sign of a zero t, which no comparison sees -- nor the
// near/far order (d < 0 is false for both zeros). So box tests use the world ray in every space,
// BLAS entries and exits change nothing but the node and instance, and only the triangle tests
// take the instance-space ray, formed where they need it (o + 0, d + 0: the same bits as the
// identity transform). The nine registers of the instance-space ray are then free.
template <bool INSTR, bool ALL_CACHED = false, int LAYOUT = kLayoutScene, bool ENTER = false, bool IDENT = false, bool RING = false>
DEV bool trav_visit(const DeviceScene& sc, TravState& s, uint32_t* lds, uint32_t shift, TraversalStats& st)
{
    if (INSTR) ++st.nodes;
    const uint32_t stride = stack_stride<ALL_CACHED>(shift);
#ifdef DCRT_PHASE_CLOCKS
    if (INSTR) {
        st.cached += (ALL_CACHED || (s.node & 0x7FFFFFFFu) < sc.cachedNodes) ? 1u : 0u;
    }
#endif
    // the stack top (read only by a pop) is issued together with the node fetch: this
    // visit's push writes the row above it, so the two LDS round trips of a visit overlap
    const uint32_t top = stack_at(lds, stack_row<RING>(sc, s.sp, shift));
    const uint32_t idx = s.node & 0x7FFFFFFFu;
    float4 a, b;
    if (ALL_CACHED) {
        const float4* c = scene_cache(sc, lds - threadIdx.x, shift);
        a = c[idx * 2];
        b = c[idx * 2 + 1];
    } else if (idx < sc.cachedNodes) {
        const float4* c = scene_cache(sc, lds - threadIdx.x, shift);
        a = lds_load4(c, idx * 2);
        b = lds_load4(c, idx * 2 + 1);
    } else {
        a = global_load4(sc.nodes, (size_t)idx * 2);
        b = global_load4(sc.nodes, (size_t)idx * 2 + 1);
    }
    const bool hit = IDENT ? ray_aabb_raw(s.o, s.invW, s.tMin, s.tMax, a, b) : ray_aabb(s, a, b);
    const uint32_t misc = asu(b.w);
    const uint32_t right = asu(b.z);
    // leaf: TLAS-leaf bit (4) or a primitive count (bits 3 and up); parked = hit && leaf
    // is formed as hit ^ descend below (a mask operation, not a second compare of misc)
    const bool descend = hit & (misc < 4u);
    const bool enter = ENTER && (hit & ((misc & (4u | kMiscIdentityLeaf)) == (4u | kMiscIdentityLeaf)) & (IDENT || s.noZero));
    // near/far by the split axis' direction sign (one bit of the space's sign mask);
    // children keep the BLAS bit of the packed node reference
    // (v_bfe takes its offset from the low 5 bits of misc: the split axis for an interior
    // node; for a leaf, whose neg is unused, a bit of negMask above bit 3, i.e. 0)
    const bool neg = __builtin_amdgcn_ubfe(s.negMask, misc, 1u) != 0u;
    uint32_t next, rightRef;
    node_children<LAYOUT>(sc, s.node, right, &next, &rightRef);
    const uint32_t nearChild = neg ? rightRef : next;
    const uint32_t farChild = neg ? next : rightRef;
    stack_at(lds, stack_row<RING>(sc, s.sp + stride, shift)) = farChild;
    const bool empty = s.sp == 0u;
    const bool pop = !hit && !empty;
    const bool done = !hit && empty;
    const bool restore = !IDENT && pop && (int)s.node < 0 && (int)top >= 0;    // BLAS -> TLAS: back to the world ray
#ifdef DCRT_PHASE_CLOCKS
    if (INSTR && descend) {
        st.deep4 += s.sp >= 4u * stride ? 1u : 0u;
        st.deep8 += s.sp >= 8u * stride ? 1u : 0u;
        st.deep12 += s.sp >= 12u * stride ? 1u : 0u;
    }
#endif
    // (three exclusive cases as a select chain on the stack top read at the step's start: as a
    // nested conditional the compiler branched and sank that read into the pop case -- a second
    // LDS round trip per popping step)
    uint32_t nextNode = pop ? top : s.node;
    nextNode = enter ? (right | 0x80000000u) : nextNode;
    nextNode = descend ? nearChild : nextNode;
    asm volatile("" : "+v"(nextNode));
    s.node = nextNode;
    s.sp = descend ? s.sp + stride : (pop ? s.sp - stride : s.sp);
    if (ENTER) {
        s.inst = enter ? (misc >> 3) & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT : s.inst;
        if (INSTR && enter) ++st.blas;
    }
    // rare (about once per ray): a branch the wave skips when no lane restores; as
    // selects it cost nine v_cndmask per visit (measured 2.5 % of the cast kernel)
    if (__builtin_expect(restore, 0)) {
        s.ld = mk(s.d.x, s.d.y, s.d.z);
        s.set_space(s.o, s.invW);
        s.negMask = neg_mask(s.d, s.negMask);
    }
    s.parked = hit ^ (descend | enter);
    if (!ALL_CACHED) {   // (ALL_CACHED: phase B reads them from the LDS copy of the node)
        s.leafRef = right;
        s.leafMisc = misc;
    }
    return done;
}

// A ray whose origin lies strictly inside the root's box (every ray of a scene that encloses its
// camera) hits that box: per axis one slab plane lies below the origin and one above, so the signs
// of (plane - o) are exact and every axis' interval holds 0 -- t0 <= 0 < t1 up to signed zeros and
// infinities, hence t1 >= t0, t0 < tMax (tMax > 0, or t0 < 0 = tMax) and t1 >= tMin = 0. Its first
// visit is then the root's descend, done here at the ray's start without the box test: the near
// child (split axis' direction sign) next, the far one pushed -- trav_visit's outcome bit for bit.
// (Non-counting kernels: the counting ones visit the root as the reference does.)
template <bool ALL_CACHED, int LAYOUT, bool IDENT>
DEV void trav_skip_root(const DeviceScene& sc, TravState& s, uint32_t* lds, uint32_t shift)
{
    // (and on down the near children while their boxes hold the origin strictly: each of those
    // visits is the same sure hit; sc.skipRoot levels at most, nodes of the LDS cache only)
    const uint32_t stride = stack_stride<ALL_CACHED>(shift);
    const V3 o = IDENT ? s.o : s.lo();
    const bool positive = s.tMax > 0.0f;
    uint32_t node = 0u;
    bool go = positive;
    for (uint32_t level = 0; level < sc.skipRoot; ++level) {
        const uint32_t idx = node & 0x7FFFFFFFu;
        if (!ALL_CACHED && idx >= sc.cachedNodes) go = false;
        if (__ballot(go) == 0ull) break;
        float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b = a;
        if (go) {
            const float4* c = scene_cache(sc, lds - threadIdx.x, shift);
            a = c[idx * 2];
            b = c[idx * 2 + 1];
        }
        const uint32_t misc = asu(b.w);
        go = go & (o.x > a.x) & (o.x < a.w) & (o.y > a.y) & (o.y < b.x) & (o.z > a.z) & (o.z < b.y) & (misc < 4u);
        if (go) {
            const bool neg = __builtin_amdgcn_ubfe(s.negMask, misc, 1u) != 0u;
            uint32_t left, right;
            node_children<LAYOUT>(sc, node, asu(b.z), &left, &right);
            stack_at(lds, s.sp + stride) = neg ? left : right;
            s.sp += stride;
            node = neg ? right : left;
            s.node = node;
        }
    }
}

// trav_skip_root for the pair traversal (trav_visit_pair): the root's sure hit leaves the lane
// about to expand the root -- both children fetched and tested at its first step -- as the root's
// own visit step would (take the root, an interior node: expand)
DEV void trav_skip_root_pair(const DeviceScene& sc, TravState& s, uint32_t* lds, uint32_t shift)
{
    if (sc.cachedNodes == 0u) return;
    const float4* c = scene_cache(sc, lds - threadIdx.x, shift);
    const float4 a = c[0], b = c[1];
    const V3 o = s.lo();
    const uint32_t misc = asu(b.w);
    const bool inside = (o.x > a.x) & (o.x < a.w) & (o.y > a.y) & (o.y < b.x) & (o.z > a.z) & (o.z < b.y) & (misc < 4u) &
                        (s.tMax > 0.0f);
    if (inside) {
        s.expand = true;
        s.expNeg = __builtin_amdgcn_ubfe(s.negMask, misc, 1u) != 0u;
        s.expRight = asu(b.z) | (s.node & 0x80000000u);
    }
}

// Phase A with one dependent fetch per hit interior node instead of one per visited node
// (the non-instrumented kernels; the counting kernels keep trav_visit). A node reached by
// a pop or a BLAS entry is visited as in trav_visit (its box tested with the current tMax);
// a hit interior node is then expanded: both child records are fetched together and both
// boxes tested with the current tMax. The near child (by the split axis' direction sign) is
// taken when it hits, the far one pushed when both hit, taken when only it hits.
// Same leaves, same order, same tMax at each leaf as BVHIntersect[NoInterp]
// (BVHAccel.inc.hlsl:119-229), hence the same hits bit for bit:
// * the near child is tested with the tMax the reference's next visit would use (no leaf
//   lies between the two tests);
// * a far child that misses at the parent would miss at its pop too: ray_aabb's only tMax
//   term is t0 < tMax and tMax never grows;
// * a far child that hits at the parent is pushed and tested again when popped (visit).
// The stack holds a subset of the reference's entries (a push needs both children to hit),
// so the uploaded stack size bounds it too.
template <bool ALL_CACHED = false, int LAYOUT = kLayoutScene, bool RING = false>
DEV bool trav_visit_pair(const DeviceScene& sc, TravState& s, uint32_t* lds, uint32_t shift)
{
    const uint32_t stride = stack_stride<ALL_CACHED>(shift);
    const uint32_t top = stack_at(lds, stack_row<RING>(sc, s.sp, shift));
    const uint32_t blasBit = s.node & 0x80000000u;
    // record A: the node itself (visit) or its near child (expand); record B: the far child
    // (expand only)
    // (expanding: s.node is the expanded node, s.expRight its `right` field with the BLAS bit)
    uint32_t nextRef, rightRef;
    node_children<LAYOUT>(sc, s.node, s.expRight, &nextRef, &rightRef);
    const uint32_t aRef = s.expand ? (s.expNeg ? rightRef : nextRef) : s.node;
    const uint32_t bRef = s.expNeg ? nextRef : rightRef;
    auto fetch = [&](uint32_t ref, float4& a, float4& b) __attribute__((always_inline)) {
        const uint32_t idx = ref & 0x7FFFFFFFu;
        if (ALL_CACHED || idx < sc.cachedNodes) {
            const float4* c = scene_cache(sc, lds - threadIdx.x, shift);
            a = c[idx * 2];
            b = c[idx * 2 + 1];
        } else {
            a = sc.nodes[idx * 2];
            b = sc.nodes[idx * 2 + 1];
        }
    };
    // (both fetches unconditional: a visit fetches its node twice, the second from L1, which
    // costs less than the exec-mask branch and the zeroed registers of a conditional fetch;
    // the LDS-or-memory choice stays one flat load here: split into ds_read / global_load
    // branches, as trav_visit has them, the pair kernel lost 5 %, profiles/r05_ab_split_loads.txt)
    float4 a0, b0, a1, b1;
    fetch(aRef, a0, b0);
    fetch(s.expand ? bRef : aRef, a1, b1);
    const bool hitA = ray_aabb(s, a0, b0);
    const bool hitB = s.expand && ray_aabb(s, a1, b1);
    // the node taken next: A if it hits, else B if it hits (push B when both hit)
    const bool take = hitA | hitB;
    const uint32_t takeRef = hitA ? aRef : bRef;
    const uint32_t right = asu(hitA ? b0.z : b1.z);
    const uint32_t misc = asu(hitA ? b0.w : b1.w);
    const bool push = hitA & hitB;
    // (the branch-free push: row count + 1 is written either way, and is unused unless pushed)
    stack_at(lds, stack_row<RING>(sc, s.sp + stride, shift)) = bRef;
    const bool empty = s.sp == 0u;
    const bool pop = !take && !empty;
    const bool done = !take && empty;
    const bool restore = pop && (int)s.node < 0 && (int)top >= 0;   // BLAS -> TLAS: back to the world ray
    const bool leaf = misc >= 4u;
    s.node = take ? takeRef : (pop ? top : s.node);
    s.sp = push ? s.sp + stride : (pop ? s.sp - stride : s.sp);
    s.expand = take & !leaf;
    s.expNeg = __builtin_amdgcn_ubfe(s.negMask, misc, 1u) != 0u;
    s.expRight = right | blasBit;
    if (__builtin_expect(restore, 0)) {
        s.ld = mk(s.d.x, s.d.y, s.d.z);
        s.set_space(s.o, s.invW);
        s.negMask = neg_mask(s.d, s.negMask);
    }
    s.parked = take & leaf;
    s.leafRef = right;
    s.leafMisc = misc;
    return done;
}

// Phase B: the parked leaf's work. TLAS leaf: move the ray into the instance and
// continue at its BLAS root. BLAS leaf: test triangles [ref, ref + count), then pop.
// LANE_ANY: any-hit is a per-lane choice (s.anyHit), for the merged ray-cast kernel
// FLAT (the entry-free node order of the cache-only IDENT kernel, tracer.hip EntryFreeLayout): no
// TLAS leaves -- a leaf is a BLAS triangle leaf whose count field holds its instance + 1
template <bool ANY_HIT, bool INSTR, bool OPACITY = false, bool LANE_ANY = false, bool ALL_CACHED = false, bool IDENT = false,
          bool RING = false, bool FLAT = false>
DEV bool trav_leaf(const DeviceScene& sc, TravState& s, bool watertight, uint32_t* lds, uint32_t shift, TraversalStats& st)
{
    s.parked = false;
    uint32_t leafRef = s.leafRef, leafMisc = s.leafMisc;
    if (ALL_CACHED) {   // the parked leaf is s.node (a leaf visit neither descends nor pops)
        const float4 b = scene_cache(sc, lds - threadIdx.x, shift)[(s.node & 0x7FFFFFFFu) * 2 + 1];
        leafRef = asu(b.z);
        leafMisc = asu(b.w);
    }
    const uint32_t primOrInst = (leafMisc >> 3) & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT;
    if (!FLAT && IDENT && (leafMisc & 0x4u)) {   // (every instance the identity: see trav_visit)
        s.inst = primOrInst;
        s.node = leafRef | 0x80000000u;
        if (INSTR) ++st.blas;
        return false;
    }
    if (!FLAT && (leafMisc & 0x4u)) {
        const float4* M;
        uint32_t identity;
        if (ALL_CACHED) {
            M = scene_cache(sc, lds - threadIdx.x, shift) + sc.cachedNodes * 2u + sc.cachedTris * kRotTriFloat4 + primOrInst * 4u;
            identity = __float_as_uint(M[3].x);
        } else {
            M = sc.transforms + (size_t)(sc.instanceCount + primOrInst) * 3;
            identity = sc.instanceIdentity[primOrInst];
        }
        if (s.noZero && identity) {
            // x*1 + y*0 + z*0 + w*0 == x exactly for finite nonzero components
            s.ld = mk(s.d.x, s.d.y, s.d.z);
            s.set_space(s.o, s.invW);
        } else {
            s.ld = mul43(s.d, 0.0f, M);
            s.set_space(mul43(s.o, 1.0f, M), inv_dir(s.ld));
        }
        s.negMask = neg_mask(s.ld, s.negMask);
        s.inst = primOrInst;
        s.node = leafRef | 0x80000000u;   // the BLAS root
        if (OPACITY) {   // BVHAccel.inc.hlsl:136-139
            s.opaque = (sc.instanceFlags[primOrInst] & DCRT_INSTANCE_FLAG_OPAQUE) != 0u;
            s.matOverride = sc.overrides[primOrInst];
        }
        if (INSTR) ++st.blas;
        return false;
    }
    // the shear of the current space, recomputed at every leaf instead of kept across
    // visits: fewer live registers (the cache-only kernel fits 7 waves/SIMD in 72 VGPRs:
    // 3.03 -> 2.96 ms/spp; coffee / lamp configs -1 to -2 %)
    // (IDENT: the instance-space ray formed here, o + 0 and d + 0; 1/d of its dominant axis --
    // the only one the shear reads -- is nonzero, so the world ray's)
    const V3 spO = IDENT ? mk(s.o.x + 0.0f, s.o.y + 0.0f, s.o.z + 0.0f) : s.lo();
    const V3 spD = IDENT ? mk(s.d.x + 0.0f, s.d.y + 0.0f, s.d.z + 0.0f) : s.ld;
    if (watertight) s.sh = ALL_CACHED ? make_shear_rot(spD, spO, IDENT ? s.invW : s.inv()) : make_shear(spD, IDENT ? s.invW : s.inv());
    // one triangle test: false = go on, true = the ray is finished (any-hit)
    auto test = [&](uint32_t p) __attribute__((always_inline)) {
        if (INSTR) ++st.tris;
        float t, u, v; bool bf, h;
        if (ALL_CACHED && watertight) {
            // (24-bit multiply: a full-rate v_mul_u32_u24 instead of the quarter-rate v_mul_lo_u32)
            const float4* c = scene_cache(sc, lds - threadIdx.x, shift) + sc.cachedNodes * 2u +
                              __umul24(p, kRotTriFloat4) + __umul24((uint32_t)s.sh.kz, 3u);
            const float4 q0 = c[0], q1 = c[1], q2 = c[2];
            // all three vertex reads issued before the degenerate / edge-sign exit (one LDS
            // round trip, not a read of q0 first and of q1, q2 behind the branch)
            asm volatile("" :: "v"(q0.w), "v"(q1.x), "v"(q2.x));
            h = tri_watertight_rot(s.sh, s.tMin, s.tMax, q0, q1, q2, &t, &u, &v, &bf);
        } else {
            float4 q0, q1, q2;
            if (ALL_CACHED) {
                const float4* c = scene_cache(sc, lds - threadIdx.x, shift) + sc.cachedNodes * 2u + __umul24(p, kRotTriFloat4) + 6u;
                q0 = c[0]; q1 = c[1]; q2 = c[2];   // permutation z = 2 is the identity
            } else if (p < sc.cachedTris) {
                const float4* c = scene_cache(sc, lds - threadIdx.x, shift) + sc.cachedNodes * 2u;
                q0 = lds_load4(c, p * 3); q1 = lds_load4(c, p * 3 + 1); q2 = lds_load4(c, p * 3 + 2);
            } else {
                q0 = global_load4(sc.triVerts, (size_t)p * 3);
                q1 = global_load4(sc.triVerts, (size_t)p * 3 + 1);
                q2 = global_load4(sc.triVerts, (size_t)p * 3 + 2);
            }
            const V3 v0 = mk(q0.x, q0.y, q0.z), v1 = mk(q1.x, q1.y, q1.z), v2 = mk(q2.x, q2.y, q2.z);
            h = watertight ? tri_watertight(spO, s.sh, s.tMin, s.tMax, v0, v1, v2, q0.w != 0.0f, &t, &u, &v, &bf)
                           : tri_moller(spO, spD, s.tMin, s.tMax, v0, v1, v2, &t, &u, &v, &bf);
        }
        if (OPACITY && h && !s.opaque) h = any_hit_shader(sc, p, s.matOverride, u, v, s.opacitySample);
        if (h) {
            s.found = true;
            if (ANY_HIT || (LANE_ANY && s.anyHit)) return true;
            s.tMax = t;
            s.hit.t = t; s.hit.u = u; s.hit.v = v;
            s.hit.tri = (p & 0x7FFFFFFFu) | (bf ? 0x80000000u : 0u);
            s.hit.inst = FLAT ? primOrInst - 1u : s.inst;
        }
        return false;
    };
    if (FLAT || sc.singlePrimLeaves) {   // (uniform: straight-line code, no loop)
        if (test(leafRef)) return true;
    } else {
        const uint32_t end = leafRef + primOrInst;
        for (uint32_t p = leafRef; p < end; ++p)
            if (test(p)) return true;
    }
    return trav_pop<IDENT, RING>(sc, s, lds, stack_stride<ALL_CACHED>(shift), shift);
}

// ---- texture emulation ----------------------------------------------------------
DEV float u16tex(const uint16_t* t, int x, int y, int w) { return (float)t[y * w + x] / 65535.0f; }
DEV int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
DEV float bilinear_u16(const uint16_t* tex, int w, int h, float u, float v)
{
    const float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const float fx = x - fx0, fy = y - fy0;
    const int x0 = clampi((int)fx0, 0, w - 1), x1 = clampi((int)fx0 + 1, 0, w - 1);
    const int y0 = clampi((int)fy0, 0, h - 1), y1 = clampi((int)fy0 + 1, 0, h - 1);
    const float a = u16tex(tex, x0, y0, w) * (1.0f - fx) + u16tex(tex, x1, y0, w) * fx;
    const float c = u16tex(tex, x0, y1, w) * (1.0f - fx) + u16tex(tex, x1, y1, w) * fx;
    return a * (1.0f - fy) + c * fy;
}
DEV int array_slice(float s, int slices)
{
    const float r = floorf(s + 0.5f);
    if (!(r > 0.0f)) return 0;
    if (r > (float)(slices - 1)) return slices - 1;
    return (int)r;
}
DEV float remap(uint32_t dim, float u) { return u * ((float)(dim - 1) / (float)dim) + 0.5f / (float)dim; }
DEV float sample_array(const uint16_t* tex, uint32_t w, uint32_t h, uint32_t slices, float uu, float vv, float ww, uint32_t dz, uint32_t off)
{
    const float slicePos = ww * ((float)dz - 1.0f);
    const float fraction = slicePos - floorf(slicePos);
    const float u = remap(w, uu), v = remap(h, vv);
    const uint32_t s0 = (uint32_t)(int32_t)slicePos + off;
    const uint32_t s1 = (uint32_t)(int32_t)slicePos + 1u + off;
    const int i0 = array_slice((float)s0, (int)slices), i1 = array_slice((float)s1, (int)slices);
    const float a = bilinear_u16(tex + (size_t)i0 * w * h, (int)w, (int)h, u, v);
    const float b = bilinear_u16(tex + (size_t)i1 * w * h, (int)w, (int)h, u, v);
    return lerp(a, b, fraction);
}
DEV float lut_brdf(const DeviceScene& s, float cosThetaO, float alpha)
{
    return bilinear_u16(s.lutBrdf, 32, 32, remap(32, cosThetaO), remap(32, alpha));
}
DEV float lut_brdf_avg(const DeviceScene& s, float alpha)
{
    const float u = remap(32, alpha);
    return bilinear_u16(s.lutBrdfAvg, 32, 1, u, u);
}
DEV float lut_brdf_dielectric(const DeviceScene& s, float cosThetaO, float alpha, float eta, bool entering)
{
    return sample_array(s.lutBrdfDielectric, 32, 16, 32, cosThetaO, alpha, (eta - 1.0f) / 2.0f, 16, entering ? 16u : 0u);
}
DEV float lut_brdf_dielectric_avg(const DeviceScene& s, float alpha, float eta, bool entering)
{
    return sample_array(s.lutBrdfDielectricAvg, 16, 16, 2, alpha, (eta - 1.0f) / 2.0f, 0.0f, 1, entering ? 1u : 0u);
}
DEV float lut_bsdf(const DeviceScene& s, float cosThetaO, float alpha, float eta, bool entering)
{
    return sample_array(s.lutBsdf, 32, 16, 32, cosThetaO, alpha, (eta - 1.0f) / 2.0f, 16, entering ? 16u : 0u);
}
DEV float lut_bsdf_avg(const DeviceScene& s, float alpha, float eta, bool entering)
{
    return sample_array(s.lutBsdfAvg, 16, 16, 2, alpha, (eta - 1.0f) / 2.0f, 0.0f, 1, entering ? 1u : 0u);
}

DEV int wrapi(int i, int n) { const int r = i % n; return r < 0 ? r + n : r; }
DEV void texel(const DeviceScene& s, const TextureDesc& t, int x, int y, float* o)
{
    if (t.format == DCRT_TEXTURE_FORMAT_R8_UNORM) {
        o[0] = (float)s.texels[t.offset + (size_t)y * t.width + x] / 255.0f; o[1] = 0.0f; o[2] = 0.0f; o[3] = 1.0f;
    } else {
        const uint8_t* p = s.texels + t.offset + ((size_t)y * t.width + x) * 4;
        o[0] = s.srgbTable[p[0]]; o[1] = s.srgbTable[p[1]]; o[2] = s.srgbTable[p[2]]; o[3] = (float)p[3] / 255.0f;
    }
}
DEV void sample_texture_wrap(const DeviceScene& s, uint32_t index, float u, float v, float* out)
{
    const TextureDesc t = s.textures[index];
    if (t.width == 0 || t.height == 0) { out[0] = out[1] = out[2] = out[3] = 0.0f; return; }   // null SRV reads 0
    const int w = (int)t.width, h = (int)t.height;
    const float x = u * (float)w - 0.5f, y = v * (float)h - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const float fx = x - fx0, fy = y - fy0;
    const int x0 = wrapi((int)fx0, w), x1 = wrapi((int)fx0 + 1, w);
    const int y0 = wrapi((int)fy0, h), y1 = wrapi((int)fy0 + 1, h);
    float a[4], b[4], c[4], d[4];
    texel(s, t, x0, y0, a); texel(s, t, x1, y0, b); texel(s, t, x0, y1, c); texel(s, t, x1, y1, d);
    for (int i = 0; i < 4; ++i) {
        const float top = a[i] * (1.0f - fx) + b[i] * fx;
        const float bot = c[i] * (1.0f - fx) + d[i] * fx;
        out[i] = top * (1.0f - fy) + bot * fy;
    }
}
DEV V3 sample_env(const DeviceScene& s, V3 d)
{
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    int face; float sc, tc, ma;
    if (ax >= ay && ax >= az) { ma = ax; if (d.x >= 0.0f) { face = 0; sc = -d.z; tc = -d.y; } else { face = 1; sc = d.z; tc = -d.y; } }
    else if (ay >= az) { ma = ay; if (d.y >= 0.0f) { face = 2; sc = d.x; tc = d.z; } else { face = 3; sc = d.x; tc = -d.z; } }
    else { ma = az; if (d.z >= 0.0f) { face = 4; sc = d.x; tc = -d.y; } else { face = 5; sc = -d.x; tc = -d.y; } }
    const float u = (sc / ma + 1.0f) * 0.5f, v = (tc / ma + 1.0f) * 0.5f;
    const int n = (int)s.envCubeSize;
    const float x = u * (float)n - 0.5f, y = v * (float)n - 0.5f;
    const float fx0 = floorf(x), fy0 = floorf(y);
    const float fx = x - fx0, fy = y - fy0;
    const int x0 = clampi((int)fx0, 0, n - 1), x1 = clampi((int)fx0 + 1, 0, n - 1);
    const int y0 = clampi((int)fy0, 0, n - 1), y1 = clampi((int)fy0 + 1, 0, n - 1);
    const float* base = s.envCube + (size_t)face * n * n * 3;
    float o[3];
    for (int i = 0; i < 3; ++i) {
        const float a = base[((size_t)y0 * n + x0) * 3 + i], b = base[((size_t)y0 * n + x1) * 3 + i];
        const float c = base[((size_t)y1 * n + x0) * 3 + i], e = base[((size_t)y1 * n + x1) * 3 + i];
        const float top = a * (1.0f - fx) + b * fx;
        const float bot = c * (1.0f - fx) + e * fx;
        o[i] = top * (1.0f - fy) + bot * fy;
    }
    return mk(o[0], o[1], o[2]);
}

// ---- hit reconstruction --------------------------------------------------------
struct Intersection {
    V3 albedo; float alpha;
    V3 position, normal, tangent, geometryNormal, ior;
    bool isTwoSided, backface, multiscattering;
    uint32_t internalScatteringMode, materialType, lightIndex, triangleIndex;
};

DEV V3 bary3(V3 p0, V3 p1, V3 p2, float u, float v)   // Math.inc.hlsl:35-43
{
    V3 r1 = p1 - p0, r2 = p2 - p0;
    r1 = r1 * u; r2 = r2 * v;
    r1 = r1 + p0; r1 = r1 + r2;
    return r1;
}

template <uint32_t CAPS = kCapAll>
DEV void hit_to_intersection(const DeviceScene& s, const HitRecord& h, Intersection& it)
{
    const uint32_t inst = h.inst, tri = h.tri & 0x7FFFFFFFu;
    it.lightIndex = s.instanceLightIndices[inst];
    it.triangleIndex = tri;
    const uint32_t ov = s.overrides[inst];
    // the triangle's vertices as pre-gathered at upload (build_tri_*_kernel): the same
    // values as vertices[triangles[3 tri + k]], one fetch level less
    const float4* P = s.triVerts + (size_t)tri * 3;
    const float4* Q = s.triShade + (size_t)tri * 6;
    const float4 q0 = P[0], q1 = P[1], q2 = P[2];
    const float4 a0 = Q[0], b0 = Q[1], a1 = Q[2], b1 = Q[3], a2 = Q[4], b2 = Q[5];
    const float u = h.u, v = h.v;
    const V3 p0 = mk(q0.x, q0.y, q0.z), p1 = mk(q1.x, q1.y, q1.z), p2 = mk(q2.x, q2.y, q2.z);
    it.position = bary3(p0, p1, p2, u, v);
    it.normal = normalize(bary3(mk(a0.x, a0.y, a0.z), mk(a1.x, a1.y, a1.z), mk(a2.x, a2.y, a2.z), u, v));
    V3 tangent = bary3(mk(a0.w, b0.x, b0.y), mk(a1.w, b1.x, b1.y), mk(a2.w, b2.x, b2.y), u, v);
    float tl = length(tangent);
    if (tl >= 0.000001f) {
        tangent = tangent - it.normal * dot(tangent, it.normal);
        tl = length(tangent);
    }
    if (tl < 0.000001f) {
        tangent = cross(it.normal, mk(0.0f, 1.0f, 0.0f));
        tl = length(tangent);
        tangent = tl >= 0.000001f ? tangent : mk(1.0f, 0.0f, 0.0f);
    }
    it.tangent = tangent / tl;
    it.geometryNormal = normalize(cross(p2 - p0, p1 - p0));
    const uint32_t mid = ov != DCRT_INSTANCE_MATERIAL_OVERRIDE_NONE ? ov : __float_as_uint(q1.w);
    const dcrt_material& m = s.materials[mid];
    if constexpr ((CAPS & kCapTextures) == 0u) {
        __builtin_assume(m.albedo_texture_index == -1);
        __builtin_assume((m.flags & DCRT_MATERIAL_FLAG_ROUGHNESS_TEXTURE) == 0u);
    }
    if constexpr ((CAPS & kCapMultiscatter) == 0u) __builtin_assume((m.flags & DCRT_MATERIAL_FLAG_MULTISCATTERING) == 0u);
    if constexpr ((CAPS & kCapMaterialsMask) != kCapMaterialsMask) {
        __builtin_assume((m.flags & DCRT_MATERIAL_FLAG_TYPE_MASK) <= DCRT_MATERIAL_TYPE_THIN_DIELECTRIC);
        __builtin_assume(((CAPS >> (m.flags & DCRT_MATERIAL_FLAG_TYPE_MASK)) & 1u) != 0u);
    }
    // VectorBaryCentric2 (Math.inc.hlsl:23-33)
    float r1x = b1.z - b0.z, r1y = b1.w - b0.w;
    float r2x = b2.z - b0.z, r2y = b2.w - b0.w;
    r1x = r1x * u; r1y = r1y * u; r2x = r2x * v; r2y = r2y * v;
    r1x = r1x + b0.z; r1y = r1y + b0.w;
    float tcx = r1x + r2x, tcy = r1y + r2y;
    tcx = tcx * m.tex_tiling[0]; tcy = tcy * m.tex_tiling[1];
    V3 albedo = ld3(m.albedo);
    if (m.albedo_texture_index != -1) {
        float rgba[4];
        sample_texture_wrap(s, (uint32_t)m.albedo_texture_index, tcx, tcy, rgba);
        albedo = albedo * mk(rgba[0], rgba[1], rgba[2]);
    }
    const float checker = ((f2u_sat(tcx * 2.0f) + f2u_sat(tcy * 2.0f)) & 0x1u) != 0 ? 1.0f : 0.0f;
    float roughness = m.roughness;
    roughness = roughness * ((m.flags & DCRT_MATERIAL_FLAG_ROUGHNESS_TEXTURE) != 0 ? checker : 1.0f);
    it.albedo = albedo;
    it.alpha = roughness * roughness;
    it.ior = ld3(m.ior);
    it.materialType = m.flags & DCRT_MATERIAL_FLAG_TYPE_MASK;
    it.isTwoSided = (m.flags & DCRT_MATERIAL_FLAG_IS_TWOSIDED) != 0;
    it.multiscattering = (m.flags & DCRT_MATERIAL_FLAG_MULTISCATTERING) != 0;
    it.internalScatteringMode = (m.flags & DCRT_MATERIAL_FLAG_INTERNAL_SCATTERING_MASK) >> DCRT_MATERIAL_FLAG_INTERNAL_SCATTERING_SHIFT;
    it.backface = (h.tri & 0x80000000u) != 0;
    const float4* M = s.transforms + (size_t)inst * 3;
    it.position = mul43(it.position, 1.0f, M);
    it.normal = normalize(mul43(it.normal, 0.0f, M));
    it.geometryNormal = normalize(mul43(it.geometryNormal, 0.0f, M));
    it.tangent = normalize(mul43(it.tangent, 0.0f, M));
}

// ---- lights (Light.inc.hlsl, RayTracingCommon.inc.hlsl:124-225) -------------------
struct LightSample {
    V3 radiance, wi;
    float pdf, distance;
    bool isDelta;
};
DEV V3 tri_pos(const DeviceScene& s, uint32_t tri, int k)
{
    const float4 q = s.triVerts[(size_t)tri * 3 + k];   // (the vertex position, gathered at upload)
    return mk(q.x, q.y, q.z);
}

template <uint32_t CAPS = kCapAll>
DEV LightSample sample_light(const DeviceScene& s, V3 p, uint32_t lightCount, Rng& rng)
{
    LightSample r;
    r.radiance = mk(0.0f, 0.0f, 0.0f); r.wi = mk(0.0f, 0.0f, 0.0f); r.pdf = 0.0f; r.distance = 0.0f; r.isDelta = false;
    const float sel = next1(rng);
    const uint32_t li = (uint32_t)floorf(sel * (float)lightCount);
    const dcrt_light& L = s.lights[li];
    assume_light_caps<CAPS>(L.flags);
    if constexpr ((CAPS & kCapEnvCube) == 0u) __builtin_assume(s.envCube == nullptr);
    if (L.flags & DCRT_LIGHT_FLAGS_POINT_LIGHT) {
        r.wi = ld3(L.position_or_triangle_range) - p;
        r.distance = length(r.wi);
        r.wi = r.wi / r.distance;
        r.radiance = ld3(L.radiance) / (r.distance * r.distance);
        r.pdf = 1.0f;
        r.isDelta = true;
    } else if (L.flags & DCRT_LIGHT_FLAGS_DIRECTIONAL_LIGHT) {
        r.wi = -ld3(L.position_or_triangle_range);
        r.distance = inf();
        r.radiance = ld3(L.radiance);
        r.pdf = 1.0f;
        r.isDelta = true;
    } else if (L.flags & DCRT_LIGHT_FLAGS_MESH_LIGHT) {
        const float triSel = next1(rng);
        const float ts0 = next1(rng), ts1 = next1(rng);
        const uint32_t triOffset = asu(L.position_or_triangle_range[0]);
        const uint32_t triCount = asu(L.position_or_triangle_range[1]);
        const uint32_t instance = asu(L.position_or_triangle_range[2]);
        const uint32_t tri = (uint32_t)((float)triOffset + floorf(triSel * (float)triCount));
        const V3 v0 = tri_pos(s, tri, 0), v1 = tri_pos(s, tri, 1), v2 = tri_pos(s, tri, 2);
        const float4* M = s.transforms + (size_t)instance * 3;
        const V3 w0 = mul43(v0, 1.0f, M), w1 = mul43(v1, 1.0f, M), w2 = mul43(v2, 1.0f, M);
        const float area = length(cross(w2 - w0, w1 - w0)) * 0.5f;
        const float sq = sqrtf(ts0);
        const float bu = 1.0f - sq, bv = ts1 * sq;
        V3 sp = bary3(v0, v1, v2, bu, bv);
        V3 nrm = normalize(cross(v2 - v0, v1 - v0));
        float pdf = area >= 1e-6f ? 1.0f / (area * 0.5f) : 0.0f;
        sp = mul43(sp, 1.0f, M);
        nrm = normalize(mul43(nrm, 0.0f, M));
        r.wi = sp - p;
        r.distance = length(r.wi);
        r.wi = r.wi / r.distance;
        const float WIdotN = -dot(r.wi, nrm);
        pdf = pdf * (r.distance * r.distance / WIdotN);
        r.radiance = (WIdotN > 0.0f && pdf > 0.0f) ? ld3(L.radiance) : mk(0.0f, 0.0f, 0.0f);
        r.pdf = WIdotN > 0.0f ? pdf : 0.0f;
        r.pdf = r.pdf / (float)triCount;
    } else if (L.flags & DCRT_LIGHT_FLAGS_ENVIRONMENT_LIGHT) {
        const float a = next1(rng), b = next1(rng);
        r.wi = uniform_sphere(a, b);
        r.pdf = uniform_sphere_pdf();
        r.radiance = s.envCube ? sample_env(s, r.wi) * ld3(L.radiance) : ld3(L.radiance);
        r.distance = inf();
    }
    r.pdf = r.pdf / (float)lightCount;
    if (r.distance != inf()) r.distance = r.distance * (1.0f - kShadowEpsilon);
    return r;
}

template <uint32_t CAPS = kCapAll>
DEV void evaluate_light(const DeviceScene& s, uint32_t li, uint32_t tri, V3 normal, V3 wi, float distance, uint32_t lightCount,
                        V3* radiance, float* pdf)
{
    *radiance = mk(0.0f, 0.0f, 0.0f);
    *pdf = 0.0f;
    const dcrt_light& L = s.lights[li];
    assume_light_caps<CAPS>(L.flags);
    if constexpr ((CAPS & kCapEnvCube) == 0u) __builtin_assume(s.envCube == nullptr);
    if (L.flags & DCRT_LIGHT_FLAGS_MESH_LIGHT) {
        const float4* M = s.transforms + (size_t)asu(L.position_or_triangle_range[2]) * 3;
        const V3 v0 = mul43(tri_pos(s, tri, 0), 1.0f, M), v1 = mul43(tri_pos(s, tri, 1), 1.0f, M), v2 = mul43(tri_pos(s, tri, 2), 1.0f, M);
        const float area = length(cross(v2 - v0, v1 - v0));
        float p = area >= 1e-6f ? 1.0f / (area * 0.5f) : 0.0f;
        const float WIdotN = -dot(wi, normal);
        *radiance = WIdotN > 0.0f ? ld3(L.radiance) : mk(0.0f, 0.0f, 0.0f);
        p = p * (WIdotN > 0.0f ? distance * distance / dot(-wi, normal) : 0.0f);
        *pdf = p / (float)asu(L.position_or_triangle_range[1]);
    } else if (L.flags & DCRT_LIGHT_FLAGS_ENVIRONMENT_LIGHT) {
        *radiance = s.envCube ? sample_env(s, wi) * ld3(L.radiance) : ld3(L.radiance);
        *pdf = uniform_sphere_pdf();
    }
    *pdf = *pdf / (float)lightCount;
}

}  // namespace dev
}  // namespace dcrt
