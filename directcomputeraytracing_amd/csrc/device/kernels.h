// kernels.h -- the wavefront path tracing kernels for gfx950
// (Shaders/WavefrontPathTracing.hlsl restated for 64-lane waves).
//
// Path pool is struct-of-arrays in HBM; queues are compacted with 64-bit wave
// ballots + mbcnt prefix counts and ONE atomic per workgroup (the reference
// issues one per 32-lane wave). CONTROL and NEW_PATH are fused: a fully idle
// wave claims an 8x8 pixel block and generates its camera rays in place.
#pragma once

#include "dbsdf.h"

namespace dcrt {
namespace dev {

constexpr uint32_t kFlagIdle = 0x80000000u;           // WavefrontPathTracing.hlsl:27-64
constexpr uint32_t kFlagShadowRayHit = 0x40000000u;
constexpr uint32_t kFlagTerminate = 0x20000000u;
constexpr uint32_t kFlagDelta = 0x10000000u;           // the path's last BSDF lobe was a delta (SPathAccumulation.isDelta)
constexpr uint32_t kFlagFirst = 0x08000000u;           // a new path's state record holds NEW_PATH's rng only (PathStateA)
constexpr uint32_t kFlagShadowPending = 0x04000000u;   // the path cast a shadow ray last pass: its result is at its position
constexpr uint32_t kBlockW = 8, kBlockH = 8;           // one wave64 = one 8x8 pixel block
#ifndef DCRT_CONTROL_BLOCK
#define DCRT_CONTROL_BLOCK 256
#endif
constexpr uint32_t kControlBlock = DCRT_CONTROL_BLOCK;  // CONTROL workgroup (the path pool is a multiple of it)
// the block appends keep per-wave counts in sm[16 q + wave] and the atomic's result in
// sm[16 q + 15]: at most 15 waves per workgroup
static_assert(kControlBlock % 64 == 0 && kControlBlock <= 960, "CONTROL workgroup: whole waves, at most 15");

// Queue counters are sharded: producer workgroup b appends to shard b % kShards,
// each shard counter on its own 256-B line. One returning device-scope atomic on
// a single word saturates at ~88 per microsecond on MI355X (MI355X_MICROARCH.md,
// "dequeue"), which would cap a 2M-path wavefront at ~100 us per queue per
// iteration; eight words spread that over eight memory-side atomic units.
constexpr uint32_t kShards = 8;
constexpr uint32_t kShardStride = 64;                  // uint32 words (256 B)
constexpr uint32_t kQExt = 0, kQShadow = 1, kQFinish = 2, kQueues = 3;
// Finish-queue counter shards: MATERIAL lists the paths it ends with a shadow ray still
// pending (the next CONTROL pass completes them). Each shard holds finCap entries.
#ifndef DCRT_FIN_SHARDS
#define DCRT_FIN_SHARDS 8
#endif
constexpr uint32_t kFinShards = DCRT_FIN_SHARDS;
constexpr uint32_t kCounterWords = 2 * kShards + kFinShards;   // ext, shadow, then finish shards
// One more word per parity (its own 256-B line): nonzero = this iteration's extension queue is
// a batch start's VIRTUAL queue -- item i is path slot i, whose camera ray the cast generates
// and whose NEW_PATH state the next MATERIAL pass recomputes (see control_kernel); its value is
// the number of items (the pool size; slots without a pixel are holes)
constexpr uint32_t kVirtualWord = kCounterWords;
constexpr uint32_t kNoPixel = 0xFFFFFFFFu;             // a virtual item (path slot) without a pixel
// And one more: nonzero = drain_kernel completed every path this iteration's queues held (the
// next MATERIAL / CONTROL pass has nothing to take from them)
constexpr uint32_t kDrainedWord = kCounterWords + 1;
// Extension-queue entry bit: the path's first MATERIAL pass follows (set by NEW_PATH), whose
// Li, light sampling result and throughput are the NEW_PATH constants, not stored or loaded
constexpr uint32_t kEntryFirst = 0x80000000u;

struct Counters {        // one set per iteration parity
    uint32_t w[(kCounterWords + 2) * kShardStride];
};
DEV uint32_t virtual_items(const Counters* c) { return c->w[kVirtualWord * kShardStride]; }
DEV bool drained(const Counters* c) { return c->w[kDrainedWord * kShardStride] != 0u; }
struct Globals {
    uint32_t nextBlock[kShards * kShardStride];        // per-shard pixel-block cursors
    uint32_t totalBlocks;
    uint32_t stackOverflow;
    // device-side image sequencing (RenderImages): no host round trip between images
    uint32_t imageComplete;   // SHADOW: every path idle after this iteration and nothing was claimed
    uint32_t poolIdle;        // the same, ignoring `stopped` (Render's IsImageComplete)
    uint32_t prevLive;        // paths live after the previous iteration (extension + finish queues)
    uint32_t stopped;         // all requested images are done: CONTROL claims nothing more
    uint32_t imagesDone, imageTarget, seedBase;
    uint32_t batchImages;     // images path-traced together in the current batch (image index in [0, batchImages))
    uint32_t batchCap;        // RenderImages' batch size
    // Batch start without atomics: RenderImages' first CONTROL pass of a batch finds every
    // slot idle, so wave j (in workgroup order) of shard s takes the shard's j-th pixel
    // block outright and the shard cursors are preset past those blocks (staticGrid =
    // CONTROL workgroups, 0 = off); cleared after that iteration.
    uint32_t staticFill, staticGrid;
    uint32_t skipFilm;        // RenderImages without the film pass: the caller convolves the images (accumulate_images)
    unsigned long long extRays, shadowRays, iterations;
};

DEV uint32_t* qctr(Counters* c, uint32_t q, uint32_t s) { return c->w + (q * kShards + s) * kShardStride; }
DEV uint32_t qctr_load(const Counters* c, uint32_t q, uint32_t s) { return c->w[(q * kShards + s) * kShardStride]; }
DEV uint32_t qtotal(const Counters* c, uint32_t q)
{
    uint32_t t = 0;
    for (uint32_t s = 0; s < kShards; ++s) t += qctr_load(c, q, s);
    return t;
}
// Concatenated view of the N shards of one queue: item i -> (shard, offset).
template <uint32_t N = kShards>
struct QueueMapN {
    uint32_t prefix[N + 1];
};
using QueueMap = QueueMapN<kShards>;
template <uint32_t N>
DEV void qmap(const Counters* c, uint32_t q, QueueMapN<N>* m)
{
    m->prefix[0] = 0;
    for (uint32_t s = 0; s < N; ++s) m->prefix[s + 1] = m->prefix[s] + qctr_load(c, q, s);
}
template <uint32_t N>
DEV uint32_t qentry(const uint32_t* queue, uint32_t cap, const QueueMapN<N>& m, uint32_t i)
{
    uint32_t s = 0, base = 0;                 // static indices only: no scratch for the map
#pragma unroll
    for (uint32_t k = 1; k < N; ++k) {
        const bool ge = i >= m.prefix[k];
        s += ge ? 1u : 0u;
        base = ge ? m.prefix[k] : base;
    }
    return queue[(size_t)s * cap + (i - base)];
}

// Position of item i of the concatenated shards: s * cap + (i - prefix[s]).
template <uint32_t N>
DEV uint32_t qpos(uint32_t cap, const QueueMapN<N>& m, uint32_t i)
{
    uint32_t s = 0, base = 0;
#pragma unroll
    for (uint32_t k = 1; k < N; ++k) {
        const bool ge = i >= m.prefix[k];
        s += ge ? 1u : 0u;
        base = ge ? m.prefix[k] : base;
    }
    return s * cap + (i - base);
}
// Extension-ray record `q` (q = shard * recCap + entry) through a 32-bit byte offset (one
// parity's records stay below 4 GiB: dcrt_tracer::Create checks it)
DEV float4* ext_rec(float4* recs, uint32_t q) { return (float4*)((char*)recs + (uint64_t)(q * 32u)); }
DEV const float4* ext_rec(const float4* recs, uint32_t q) { return (const float4*)((const char*)recs + (uint64_t)(q * 32u)); }

// Per-image constants, read from HBM so a captured graph can be replayed for
// every frame seed (SNewPathConstants / SMaterialConstants / SControlConstants).
struct FrameConstants {
    float camera[16];
    uint32_t resolution[2];
    float filmSize[2];
    float apertureRadius, focalDistance, filmDistance;
    uint32_t bladeCount;
    float bladeVertexPos[2];
    float apertureBaseAngle;
    uint32_t frameSeed;
    uint32_t maxBounce, lightCount, envLightIndex, features;
    uint32_t blocksX, bandCount;     // blocks per row, number of 8-row groups of the rendered rows
    uint32_t blocksPerImage;         // blocksX * bandCount
    uint32_t refillLanes, parkLanes; // persistent traversal thresholds (lanes of a wave64)
    uint32_t virtualStart;           // batch starts use the virtual extension queue (kVirtualWord)
    uint32_t drainPaths;             // drain_kernel completes the live paths once at most this many remain (0: off)
    uint32_t seedStride;             // image b of a batch has frame seed frameSeed + b * seedStride (interleaved pipelines)
};
// The frame seed of image `image` of the current batch (RenderImages: frameSeed is the batch's first)
DEV uint32_t image_seed(const FrameConstants& fc, uint32_t image) { return fc.frameSeed + __umul24(image, fc.seedStride); }

// SampleAperture + GenerateRay (RayTracingCommon.inc.hlsl:38-86).
DEV void generate_ray(const FrameConstants& f, float fsx, float fsy, float a0, float a1, float a2, V3* origin, V3* direction)
{
    V3 filmPos = mk(-fsx + 0.5f, fsy - 0.5f, -f.filmDistance);
    filmPos.x = filmPos.x * f.filmSize[0];
    filmPos.y = filmPos.y * f.filmSize[1];
    V3 o = mk(0.0f, 0.0f, 0.0f);
    V3 d = normalize(-filmPos);
    if (f.apertureRadius > 0.0f) {
        float apx, apy;
        if (f.bladeCount <= 2) {
            concentric_disk(a0, a1, &apx, &apy);
            apx = apx * f.apertureRadius;
            apy = apy * f.apertureRadius;
        } else {
            const float s = sqrtf(a0);
            const float u = 1.0f - s, v = a1 * s;
            const float px = f.bladeVertexPos[0] * (u + v);
            const float py = f.bladeVertexPos[1] * u - f.bladeVertexPos[1] * v;
            const float n = floorf(a2 * (float)f.bladeCount);
            const float theta = n * (kPiMul2 / (float)f.bladeCount) + f.apertureBaseAngle;
            float st, ct;
            det_sincos(theta, &st, &ct);
            apx = px * ct - py * st;
            apy = py * ct + px * st;
        }
        const V3 focus = d * (f.focalDistance / d.z);
        o = mk(apx, apy, 0.0f);
        d = normalize(focus - o);
    }
    *origin = mul44(o, 1.0f, f.camera);
    *direction = mul44(d, 0.0f, f.camera);
}

// Three floats, 12 B (dwordx3): path arrays whose fourth word would carry nothing
struct F3 {
    float x, y, z;
};
// four floats at 4-B alignment: a 16-B load at an F3 boundary (global_load_dwordx4 needs
// dword alignment only)
struct alignas(4) F4u {
    float x, y, z, w;
};

// Element i of a path-pool array through a 32-bit byte offset (every pool array is
// < 4 GiB): the access then takes the array base in SGPRs plus one VGPR offset
// (global_load v, v_off, s[base]) instead of a 64-bit VGPR address per array, which
// MATERIAL otherwise keeps live from a path's loads to its stores
template <typename T>
DEV T& slot(T* base, uint32_t i)
{
    return *(T*)((char*)base + (uint64_t)(i * (uint32_t)sizeof(T)));
}

// Element i of a film sample array (batch x W*H entries): a 64-bit byte offset -- a 4K
// batch of more than 32 images puts i * 16 past 2^32, which slot() would wrap onto
// another pixel
template <typename T>
DEV T& sample_at(T* base, uint32_t i)
{
    return *(T*)((char*)base + (uint64_t)i * (uint64_t)sizeof(T));
}
// The same element stored through a global-address-space pointer: a store through the
// generic pointer is a flat store, which the wait counters track out of order, so the compiler
// then waits for every outstanding memory operation before the next register reuse. (Through
// an integer and clang vector types: a generic -> global pointer cast is folded back into a
// flat store, and HIP's vector classes have no address-space-qualified assignment.)
typedef float GlobalF2 __attribute__((ext_vector_type(2)));
typedef float GlobalF4 __attribute__((ext_vector_type(4)));
DEV void store_global(float2* base, uint32_t i, float2 v)
{
    const GlobalF2 x = {v.x, v.y};
    *(__attribute__((address_space(1))) GlobalF2*)((uintptr_t)base + (uint64_t)i * 8u) = x;
}
DEV void store_global(float4* base, uint32_t i, float4 v)
{
    const GlobalF4 x = {v.x, v.y, v.z, v.w};
    *(__attribute__((address_space(1))) GlobalF4*)((uintptr_t)base + (uint64_t)i * 16u) = x;
}

// A live path's state travels with its extension ray: one 64-B record at the ray's
// extension-queue position q (beside the 32-B ray record), written densely by its producer
// (CONTROL for a new path, MATERIAL for a continuing one) and read densely by the next
// MATERIAL pass at the same position -- no slot-indexed state, so no access to a 128-B
// line half of which belongs to an ended path, and no load that waits for the slot.
// xoshiro state, (lsr.y, lsr.z, flags, path slot), throughput + bsdfPdf, Li + lsr.x, as two
// dense 32-B halves (two arrays, same positions). A new path writes half A only (CONTROL: rng
// and the misc word with kFlagFirst): its T = 1, bsdfPdf = 0, Li = 0, lsr = 0 are NEW_PATH's
// constants, which its first MATERIAL pass takes instead of half B. (As one 64-B record, a
// new path's half-written record cost a 32-B write request each: 33 M of a 4K batch start's
// 54 M, PMC.)
struct PathStateA {
    uint4 rng;
    float4 lsrMisc;  // lsr.y, lsr.z, asfloat(flags: first, delta, bounce), asfloat(path slot)
};
struct PathStateB {
    float4 thr;      // T.xyz, bsdfPdf
    float4 liLsr;    // Li.xyz, lsr.x
};
// A path MATERIAL ends with its shadow ray pending: what CONTROL's completion needs
// (Li += lsr when the shadow ray is unoccluded, WriteSample), at its finish-queue position.
struct FinishRec {
    float4 liLsr;    // Li.xyz, lsr.x
    float4 lsrSlot;  // lsr.y, lsr.z, asfloat(path slot), -
};
// Destination of a shadow ray's result (carried in its record's direction.w): the
// continuing path's extension-queue position, or its finish-queue position | kDestFinish
constexpr uint32_t kDestFinish = 0x80000000u;

struct PathPool {
    // the extension cast's result, indexed by the ray's item in the extension queue (its
    // index in the shards' prefix order, the same for the cast and the next MATERIAL pass):
    // 2 float4 per item, (t, u, v, asfloat(triangle | backface << 31)) and (the ray's
    // direction, asfloat(instance)) -- MATERIAL then needs nothing of the ray record
    float4* hit;
    // Shadow rays, like the extension rays, travel in their queue: entry e of shard s has
    // a 32-B record at 2 * (s * recCap + e) float4s, (origin, tMax) and (direction, the
    // result's destination), beside its path slot in shadowQueue[s * recCap + e]
    // (ALLOW_ANYHIT_SHADER's opacity samples are per slot)
    float4* shRec;
    uint32_t* pixel;     // per slot: sample index image * W*H + y * W + x (the sub-pixel
                         // position is recomputed from it: pixel_sample)
    uint32_t* flags;     // per slot: kFlagIdle (CONTROL's claims), else 0
    float* extOpacity;         // ALLOW_ANYHIT_SHADER: g_ExtensionRayOpacitySamples
    float* shadowOpacity;      //                      g_ShadowRayOpacitySamples
    // Queues (kShards x recCap entries each), alternating by iteration parity: the `*Rec`,
    // `state`, `shadowHit`, `finRec`, `finHit` pointers are this iteration's (written), the
    // `*Prev` ones the previous iteration's (MATERIAL / CONTROL work lists); the host sets
    // them per launch.
    // Extension rays travel IN the extension queue: entry e of shard s is a 32-B record at
    // 2 * (s * recCap + e) float4s, (origin, 0) and (direction, asfloat(path slot)); tMax =
    // inf, tMin = 0 implicit. Its producer (CONTROL, MATERIAL) writes it densely at its queue
    // position with the path's state record (`state`, same position), the cast reads it there
    // without an index load.
    float4* extRec;
    const float4* extPrevRec;
    PathStateA* stateA;          // kShards x recCap each (state_at: 32-bit offsets, as ext_rec)
    PathStateB* stateB;
    const PathStateA* stateAPrev;
    const PathStateB* stateBPrev;
    uint32_t* shadowHit;         // the shadow cast's result for ext position q (1 = occluded)
    const uint32_t* shadowHitPrev;
    uint32_t* shadowQueue;
    FinishRec* finRec;           // kFinShards x finCap
    const FinishRec* finPrevRec;
    uint32_t* finHit;            // the shadow cast's result for finish position f
    const uint32_t* finHitPrev;
    uint32_t size;
    uint32_t recCap;           // entries per extension-queue shard
    uint32_t finCap;           // entries per finish-queue shard
};
// State half of extension-queue position q (32 B: one parity's halves stay below 4 GiB like
// the extension records, dcrt_tracer::Create)
template <typename T>
DEV T& state_at(T* base, uint32_t q) { static_assert(sizeof(T) == 32, "state halves are 32 B"); return *(T*)((char*)base + (uint64_t)(q * 32u)); }

// Sample textures (m_SamplePositionTexture / m_SampleValueTexture) for every image of a
// batch: image b's sample of pixel (x, y) sits at b * W*H + y * W + x.
struct Film {
    float2* samplePosition;   // batch x W*H
    float4* sampleValue;      // batch x W*H
    uint4* debugRng;          // batch x W*H or nullptr
    float4* accum;            // W*H RGBA32F (sum w*L, sum w)
    const uint32_t* rowY;     // the rows this tracer path-traces (8 per block row), ascending
    const uint32_t* rowOwned; // per film row: 1 if this tracer convolves it (nullptr: all rows)
    uint32_t width, height, rowCount;
};

// Where MATERIAL writes the samples of the paths it ends (a device copy of the Film's
// sample pointers: read only on that path, so they hold no SGPRs across the shading code)
struct SampleOut {
    float2* samplePosition;
    float4* sampleValue;
    uint4* debugRng;
    uint32_t* rowRays;        // probe (dcrt_tracer_set_row_cost_probe): rays cast per film row, or nullptr
};

// A path's sub-pixel position (NEW_PATH's first two draws, WavefrontPathTracing.hlsl:213-214)
// recomputed from its sample index p = image * W*H + y * W + x when WriteSample needs it:
// the same rng_init and the same two draws, so the same bits as storing them per slot -- a
// 4-B pixel read per ending path instead of a 12-B one (two partly read sectors). Valid
// while the path's batch is live (fc's frame seed advances only once the batch completed);
// fc.resolution is the film's (EnsureFilm follows SetFrame).
DEV float2 pixel_sample(const FrameConstants& fc, uint32_t p)
{
    const uint32_t W = fc.resolution[0], wh = W * fc.resolution[1];
    const uint32_t image = p / wh, local = p - image * wh;
    const uint32_t py = local / W, px = local - py * W;
    Rng r = rng_init(px, py, image_seed(fc, image));
    const float psx = next1(r);
    const float psy = next1(r);
    return make_float2(psx, psy);
}

// NEW_PATH (WavefrontPathTracing.hlsl:211-237) of the path of sample index p = image * W*H + y *
// W + x: its rng after the pixel-sample and aperture draws and (RAY) its camera ray -- the same
// arithmetic control_kernel runs for a claimed pixel, so the same bits. A virtual batch start
// (kVirtualWord) runs it in the cast kernel (the ray) and in the path's first MATERIAL pass
// (the rng) instead of writing and reading them back.
template <bool RAY>
DEV Rng new_path(const FrameConstants& fc, uint32_t p, V3* o, V3* d)
{
    const uint32_t W = fc.resolution[0], wh = W * fc.resolution[1];
    const uint32_t image = p / wh, local = p - image * wh;
    const uint32_t py = local / W, px = local - py * W;
    Rng rng = rng_init(px, py, image_seed(fc, image));
    const float psx = next1(rng), psy = next1(rng);
    const float a0 = next1(rng), a1 = next1(rng), a2 = next1(rng);
    if (RAY) {
        const float fsx = (psx + (float)px) / (float)fc.resolution[0];
        const float fsy = (psy + (float)py) / (float)fc.resolution[1];
        generate_ray(fc, fsx, fsy, a0, a1, a2, o, d);
    }
    return rng;
}

// Pixel of lane `lane` in claimed block `block` of the batch: image, then 8-row group,
// then 8-column block. False for lanes outside the film or past the last rendered row.
DEV bool block_pixel(const FrameConstants& fc, const Film& film, uint32_t block, uint32_t lane, uint32_t* px, uint32_t* py,
                     uint32_t* image)
{
    *image = block / fc.blocksPerImage;
    const uint32_t local = block - *image * fc.blocksPerImage;
    const uint32_t band = local / fc.blocksX, bx = local - band * fc.blocksX;
    const uint32_t ri = band * kBlockH + lane / kBlockW;
    *px = bx * kBlockW + (lane % kBlockW);
    if (*px >= fc.resolution[0] || ri >= film.rowCount) return false;
    *py = film.rowY[ri];
    return *py < fc.resolution[1];
}

}  // namespace dev
}  // namespace dcrt
