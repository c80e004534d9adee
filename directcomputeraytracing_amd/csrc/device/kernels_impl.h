// kernels_impl.h -- MI355X (gfx950) kernels of the wavefront path tracer and the
// BxDF LUT integrator. Host orchestration lives in tracer.hip.
//
// Reference map (Shaders/WavefrontPathTracing.hlsl):
//   set_idle_kernel      SET_IDLE            :628-651
//   control_kernel       CONTROL + NEW_PATH  :483-607 + :176-255 (fused)
//   material_kernel      MATERIAL            :257-481
//   extension_kernel     EXTENSION_RAY_CAST  :66-122
//   shadow_kernel        SHADOW_RAY_CAST     :124-174
//   film_kernel          SampleConvolution.hlsl:67-106
//   lut_*_kernel         BxDFTexturesBuilding.hlsl:10-186
#include "kernels.h"
// (included once, by tracer.hip)

namespace dcrt {
namespace dev {

#ifdef DCRT_PHASE_CLOCKS
// Diagnostic build only (tools/phase_clocks.py): shader-clock cycles the cast kernels'
// waves spend per phase of the persistent loop, summed over all waves:
// [0] hand-over + result stores + ray set-up, [1] phase A (node visits), [2] phase B
// (leaf work), [3] loop trips, [4] phase-A checks, [5] phase-B entries.
// MATERIAL: [8] loads + Li update, [9] HitInfoToIntersection, [10] record / sample stores,
// [11] emission + NEE (BSDF frame, light sample, BSDF eval + pdf, shadow ray), [12] BSDF
// sample + new ray, [13] end-of-path loads, [14] queue appends (barriers + atomics), [15] items.
__device__ unsigned long long g_phaseClk[24];
#define DCRT_PHASE_INIT unsigned long long clk_[6] = {0, 0, 0, 0, 0, 0}; unsigned long long tP_ = __builtin_amdgcn_s_memtime()
#define DCRT_PHASE(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); clk_[i] += t_ - tP_; tP_ = t_; } while (0)
#define DCRT_PHASE_COUNT(i) (++clk_[i])
#define DCRT_PHASE_FLUSH() do { if ((threadIdx.x & 63u) == 0) for (int i_ = 0; i_ < 6; ++i_) atomicAdd(&g_phaseClk[i_], clk_[i_]); } while (0)
#define DCRT_MCLK_INIT unsigned long long mclk_[8] = {0, 0, 0, 0, 0, 0, 0, 0}; unsigned long long mT_ = __builtin_amdgcn_s_memtime()
#define DCRT_MCLK(i) do { const unsigned long long t_ = __builtin_amdgcn_s_memtime(); mclk_[i] += t_ - mT_; mT_ = t_; } while (0)
#define DCRT_MCLK_FLUSH(items) do { mclk_[7] += (items); if ((threadIdx.x & 63u) == 0) for (int i_ = 0; i_ < 8; ++i_) atomicAdd(&g_phaseClk[8 + i_], mclk_[i_]); } while (0)
// (shade_path's sections clock into its caller's MATERIAL clocks)
#define DCRT_MCLK_PARAMS , unsigned long long (&mclk_)[8], unsigned long long& mT_
#define DCRT_MCLK_ARGS , mclk_, mT_
#else
#define DCRT_MCLK_PARAMS
#define DCRT_MCLK_ARGS
#define DCRT_MCLK_INIT do {} while (0)
#define DCRT_MCLK(i) do {} while (0)
#define DCRT_MCLK_FLUSH(items) do {} while (0)
#define DCRT_PHASE_INIT do {} while (0)
#define DCRT_PHASE(i) do {} while (0)
#define DCRT_PHASE_COUNT(i) do {} while (0)
#define DCRT_PHASE_FLUSH() do {} while (0)
#endif

// One atomic per workgroup: wave ballot + mbcnt prefix, LDS scan over waves.
// Every thread of the block must call it (it contains barriers).
__device__ __forceinline__ uint32_t block_append(bool pred, uint32_t* counter, uint32_t* sm)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const unsigned long long mask = __ballot(pred);
    const uint32_t prefix = __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
    if (lane == 0) sm[wave] = (uint32_t)__popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t total = 0;
        const uint32_t waves = blockDim.x >> 6;
        for (uint32_t w = 0; w < waves; ++w) { const uint32_t c = sm[w]; sm[w] = total; total += c; }
        sm[32] = total ? atomicAdd(counter, total) : 0u;
    }
    __syncthreads();
    const uint32_t r = sm[32] + sm[wave] + prefix;
    __syncthreads();
    return r;
}

// Two appends at once (one barrier round for both queues): returns the slots of `pa` in
// counter a and of `pb` in counter b. sm needs 2 * (waves + 1) words; two calls in a row
// must use different sm halves (callers alternate), so no third barrier guards reuse.
__device__ __forceinline__ void block_append2(bool pa, uint32_t* ca, bool pb, uint32_t* cb, uint32_t* sm, uint32_t* ra, uint32_t* rb)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t waves = blockDim.x >> 6;
    const unsigned long long ma = __ballot(pa), mb = __ballot(pb);
    const uint32_t xa = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
    const uint32_t xb = __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
    if (lane == 0) { sm[wave] = (uint32_t)__popcll(ma); sm[16 + wave] = (uint32_t)__popcll(mb); }
    __syncthreads();
    if (threadIdx.x < 2) {   // thread 0: queue a, thread 1: queue b (their atomics overlap)
        uint32_t* q = sm + threadIdx.x * 16;
        uint32_t total = 0;
        for (uint32_t w = 0; w < waves; ++w) { const uint32_t c = q[w]; q[w] = total; total += c; }
        q[15] = total ? atomicAdd(threadIdx.x ? cb : ca, total) : 0u;
    }
    __syncthreads();
    *ra = sm[15] + sm[wave] + xa;
    *rb = sm[31] + sm[16 + wave] + xb;
}

// Three appends at once (MATERIAL: extension, shadow and finish queues): as block_append2,
// threads 0 / 1 / 2 issue the three atomics together. sm needs 48 words per call (callers
// alternate two halves of 96).
__device__ __forceinline__ void block_append3(bool pa, uint32_t* ca, bool pb, uint32_t* cb, bool pc, uint32_t* cc, uint32_t* sm,
                                              uint32_t* ra, uint32_t* rb, uint32_t* rc)
{
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t waves = blockDim.x >> 6;
    const unsigned long long ma = __ballot(pa), mb = __ballot(pb), mc = __ballot(pc);
    const uint32_t xa = __builtin_amdgcn_mbcnt_hi((uint32_t)(ma >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)ma, 0u));
    const uint32_t xb = __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
    const uint32_t xc = __builtin_amdgcn_mbcnt_hi((uint32_t)(mc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mc, 0u));
    if (lane == 0) { sm[wave] = (uint32_t)__popcll(ma); sm[16 + wave] = (uint32_t)__popcll(mb); sm[32 + wave] = (uint32_t)__popcll(mc); }
    __syncthreads();
    if (threadIdx.x < 3) {
        uint32_t* q = sm + threadIdx.x * 16;
        uint32_t total = 0;
        for (uint32_t w = 0; w < waves; ++w) { const uint32_t c = q[w]; q[w] = total; total += c; }
        q[15] = total ? atomicAdd(threadIdx.x == 0 ? ca : (threadIdx.x == 1 ? cb : cc), total) : 0u;
    }
    __syncthreads();
    *ra = sm[15] + sm[wave] + xa;
    *rb = sm[31] + sm[16 + wave] + xb;
    *rc = sm[47] + sm[32 + wave] + xc;
}

__device__ __forceinline__ unsigned long long wave_sum(uint32_t v)
{
    unsigned long long s = v;
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return s;
}

__global__ void set_frame_kernel(FrameConstants* dst, FrameConstants src) { *dst = src; }

__global__ void set_idle_kernel(PathPool pool, Counters* counters, Globals* g, uint32_t totalBlocks)
{
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    if (tid < pool.size) pool.flags[tid] = kFlagIdle;
    if (tid < 2 * (uint32_t)(sizeof(Counters) / 4)) ((uint32_t*)counters)[tid] = 0u;
    if (tid < kShards) g->nextBlock[tid * kShardStride] = 0u;
    if (tid == 0) {
        g->totalBlocks = totalBlocks;
        g->batchImages = 1u;
        g->batchCap = 1u;
        g->imageComplete = 0u;
        g->poolIdle = 0u;
        g->prevLive = 0u;
        g->stopped = 0u;
        g->imagesDone = 0u;
        g->imageTarget = 1u;
        g->staticFill = 0u;
        g->staticGrid = 0u;
        g->skipFilm = 0u;
    }
}

// Preset the shard cursors for a batch start (see Globals::staticFill): shard s's first
// min(waves of its CONTROL workgroups, its blocks) blocks are taken statically.
// Invariant the batch start relies on: every slot is idle when staticFill is set -- the two
// callers are begin_images_kernel (right after BeginImage's set_idle_kernel) and
// advance_image_kernel (only once the batch completed: no path was live entering the last
// iteration and none was started, end_iteration). The static claims (and the virtual start's
// pixel / flag writes, control_kernel) overwrite the slots without checking them.
__device__ __forceinline__ void begin_batch_claims(Globals* g)
{
    const uint32_t G = g->staticGrid, wavesPerGroup = kControlBlock >> 6;
    for (uint32_t s = 0; s < kShards; ++s) {
        const uint32_t blocks = g->totalBlocks > s ? (g->totalBlocks - s + kShards - 1) / kShards : 0u;
        const uint32_t waves = G > s ? ((G - s + kShards - 1) / kShards) * wavesPerGroup : 0u;
        g->nextBlock[s * kShardStride] = G ? min(blocks, waves) : 0u;
    }
    g->staticFill = G ? 1u : 0u;
}

// Upload-time gathers of the triangles' vertices (one fetch level less for the traversal
// and for MATERIAL's HitInfoToIntersection): positions (+ the degenerate flag and the
// per-triangle material id in the w words) and the shading attributes.
__global__ void build_tri_verts_kernel(const dcrt_vertex* vertices, const uint32_t* triangles, const uint32_t* materialIds,
                                       uint32_t count, float4* out, float4* shade)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= count) return;
    V3 p[3];
    for (int k = 0; k < 3; ++k) {
        const dcrt_vertex& v = vertices[triangles[t * 3 + k]];
        p[k] = mk(v.position[0], v.position[1], v.position[2]);
        shade[(size_t)t * 6 + 2 * k] = make_float4(v.normal[0], v.normal[1], v.normal[2], v.tangent[0]);
        shade[(size_t)t * 6 + 2 * k + 1] = make_float4(v.tangent[1], v.tangent[2], v.texcoord[0], v.texcoord[1]);
    }
    // RayTriangleIntersect's degenerate test (RayPrimitiveIntersect.inc.hlsl), hoisted to upload time
    const V3 cp = cross(p[1] - p[0], p[2] - p[0]);
    const float degenerate = dot(cp, cp) == 0.0f ? 1.0f : 0.0f;
    out[(size_t)t * 3] = make_float4(p[0].x, p[0].y, p[0].z, degenerate);
    out[(size_t)t * 3 + 1] = make_float4(p[1].x, p[1].y, p[1].z, __uint_as_float(materialIds[t]));
    out[(size_t)t * 3 + 2] = make_float4(p[2].x, p[2].y, p[2].z, 0.0f);
}

// ---- CONTROL (+ NEW_PATH) -------------------------------------------------------
// Live paths never pass through CONTROL: MATERIAL takes them from the previous
// iteration's extension queue and ends the paths it can (no shadow ray pending) itself.
// CONTROL (1) completes the paths MATERIAL ended with a shadow ray pending (listed in
// the previous iteration's finish queue): Li += light sampling result unless the shadow
// ray hit (:520-528) and WriteSample; (2) while its shard has pixel blocks to hand out,
// scans the slots for fully idle waves, which claim the next 8x8 block and start its
// paths (NEW_PATH). With every block claimed (the batch's first pass claims all of
// them) a pass is the finish list only, not a read of every slot's flags.
__global__ __launch_bounds__(kControlBlock) void control_kernel(PathPool pool, Film film, const FrameConstants* __restrict__ fc, Counters* cnt,
                                                       const Counters* prev, Globals* g, uint32_t debugRng)
{
    __shared__ uint32_t sm[64];
    if (g->stopped) return;                    // RenderImages finished: nothing live, nothing to claim
    {
        QueueMapN<kFinShards> fm;
        qmap(prev, kQFinish, &fm);
        const uint32_t nFin = drained(prev) ? 0u : fm.prefix[kFinShards];   // (drain_kernel completed them)
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nFin; i += gridDim.x * blockDim.x) {
            // the path's finish record and its shadow ray's result, both at its finish-queue
            // position (dense); only the pixel is per slot
            const uint32_t f = qpos(pool.finCap, fm, i);
            const FinishRec fr = pool.finPrevRec[f];
            const bool shadowHit = pool.finHitPrev[f] != 0u;
            const uint32_t path = asu(fr.lsrSlot.z);
            F3 li{fr.liLsr.x, fr.liLsr.y, fr.liLsr.z};
            const F3 lsr{fr.liLsr.w, fr.lsrSlot.x, fr.lsrSlot.y};
            li.x = li.x + (!shadowHit ? lsr.x : 0.0f);
            li.y = li.y + (!shadowHit ? lsr.y : 0.0f);
            li.z = li.z + (!shadowHit ? lsr.z : 0.0f);
            const uint32_t p = slot(pool.pixel, path);
            sample_at(film.samplePosition, p) = pixel_sample(*fc, p);
            sample_at(film.sampleValue, p) = make_float4(li.x, li.y, li.z, 0.0f);
            // (debug RNG: MATERIAL stored it when it ended the path)
            // last, after stores that consumed the loads: another workgroup's scan may see the
            // slot idle from here on and start a new path in it
            slot(pool.flags, path) = kFlagIdle;
        }
    }
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t shard = blockIdx.x % kShards;
    uint32_t* cursor = &g->nextBlock[shard * kShardStride];
    // pixel blocks of this shard: shard, shard + kShards, ...
    const uint32_t shardBlocks = g->totalBlocks > shard ? (g->totalBlocks - shard + kShards - 1) / kShards : 0u;
    const bool staticFill = g->staticFill != 0u;
    if (staticFill && fc->virtualStart) {
        // Virtual batch start: every slot is idle (the previous batch drained), wave j of the
        // shard takes the shard's block j, and NEW_PATH is deferred -- the cast generates slot
        // i's camera ray from its pixel (new_path<true>) and the path's first MATERIAL pass
        // recomputes its rng (new_path<false>), so the only per-slot writes are the pixel (or
        // kNoPixel: a hole in the virtual queue) and the busy flag. A 4K batch's start wrote
        // 72 B per path here and read 64 of them back.
        for (uint32_t base = blockIdx.x * blockDim.x; base < pool.size; base += gridDim.x * blockDim.x) {
            const uint32_t tid = base + threadIdx.x;
            const uint32_t vb = base / kControlBlock;
            const uint32_t claimed = (vb / kShards) * (kControlBlock >> 6) + (threadIdx.x >> 6);
            uint32_t pixel = kNoPixel, px = 0, py = 0, image = 0;
            if (claimed < shardBlocks && block_pixel(*fc, film, shard + claimed * kShards, lane, &px, &py, &image)) {
                pixel = image * (film.width * film.height) + py * film.width + px;
                pool.flags[tid] = 0u;   // busy
            }
            pool.pixel[tid] = pixel;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) cnt->w[kVirtualWord * kShardStride] = pool.size;
        return;
    }
    if (!staticFill) {
        // (one read for the workgroup: the scan below holds barriers, so the exit must be uniform)
        __shared__ uint32_t exhausted;
        if (threadIdx.x == 0) exhausted = __hip_atomic_load(cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= shardBlocks;
        __syncthreads();
        if (exhausted) return;
    }
    // (the grid is a multiple of kShards, or one round: every virtual workgroup vb of this
    // workgroup is in its shard)
    for (uint32_t base = blockIdx.x * blockDim.x; base < pool.size; base += gridDim.x * blockDim.x) {
    const uint32_t tid = base + threadIdx.x;
    const uint32_t vb = base / kControlBlock;
    const bool idle = (pool.flags[tid] & kFlagIdle) != 0;
    // A fully idle wave claims the next 8x8 block (one atomic per workgroup); at a batch
    // start (all slots idle, cursors preset) wave j of the shard takes block j outright.
    const bool waveIdle = __ballot(!idle) == 0ull;
    uint32_t claimed = 0;
    bool got = false;
    if (staticFill) {
        claimed = (vb / kShards) * (kControlBlock >> 6) + (threadIdx.x >> 6);
        got = waveIdle && claimed < shardBlocks;
    } else {
        bool want = false;
        if (waveIdle && lane == 0)
            want = __hip_atomic_load(cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < shardBlocks;
        uint32_t bslot, unused;
        block_append2(false, cursor, want, cursor, sm, &unused, &bslot);
        claimed = (uint32_t)__shfl((int)bslot, 0, 64);
        got = __shfl((int)want, 0, 64) != 0 && claimed < shardBlocks;
    }
    const uint32_t block = shard + claimed * kShards;
    bool newPath = false;
    V3 o = mk(0.0f, 0.0f, 0.0f), d = mk(0.0f, 0.0f, 0.0f);
    Rng rng;
    rng.s0 = rng.s1 = rng.s2 = rng.s3 = 0u;
    if (got) {
        uint32_t px = 0, py = 0, image = 0;
        if (block_pixel(*fc, film, block, lane, &px, &py, &image)) {
            // NEW_PATH :211-237 (image `image` of the batch has frame seed image_seed(fc, image))
            rng = rng_init(px, py, image_seed(*fc, image));
            const float psx = next1(rng), psy = next1(rng);
            const float fsx = (psx + (float)px) / (float)fc->resolution[0];
            const float fsy = (psy + (float)py) / (float)fc->resolution[1];
            const float a0 = next1(rng), a1 = next1(rng), a2 = next1(rng);
            generate_ray(*fc, fsx, fsy, a0, a1, a2, &o, &d);
            if (fc->features & DCRT_FEATURE_ALLOW_ANYHIT) pool.extOpacity[tid] = next1(rng);   // :223-226
            // (the sub-pixel position is recomputed from the pixel where WriteSample needs it:
            // pixel_sample)
            pool.pixel[tid] = image * (film.width * film.height) + py * film.width + px;
            pool.flags[tid] = 0u;   // busy
            newPath = true;
        }
    }
    // (the other half of sm: the next round's first append reuses the first half only
    // after every thread has passed this append's barriers)
    uint32_t eslot, unused;
    block_append2(newPath, qctr(cnt, kQExt, shard), false, qctr(cnt, kQExt, shard), sm + 32, &eslot, &unused);
    if (newPath) {
        const uint32_t q = shard * pool.recCap + eslot;
        float4* r = ext_rec(pool.extRec, q);
        r[0] = make_float4(o.x, o.y, o.z, 0.0f);
        r[1] = make_float4(d.x, d.y, d.z, asf(tid));
        // NEW_PATH's state (:227-237) beside the ray: the rng, isDelta = true, bounce 0, the
        // slot (32 B); Li = 0, light sampling result = 0, T = 1, bsdfPdf = 0 are implicit
        // (kFlagFirst: writing all 64 B cost the 4K batches' first passes 3 GB of writes)
        PathStateA& st = state_at(pool.stateA, q);
        st.rng = make_uint4(rng.s0, rng.s1, rng.s2, rng.s3);
        st.lsrMisc = make_float4(0.0f, 0.0f, asf(kFlagDelta | kFlagFirst), asf(tid));
    }
    }
}

// MATERIAL's shading of one path at its hit (WavefrontPathTracing.hlsl:302-441): emission with
// MIS, termination, next-event estimation (the shadow ray and its light sampling result), the
// BSDF sample (the next extension ray), the new throughput, bsdfPdf (thr.w) and flags. `li` is
// the path's Li after CONTROL's `Li += light sampling result`. Shared by material_kernel and
// the drain kernel (drain_kernel), so both run the same arithmetic in the same order.
template <uint32_t CAPS>
__device__ __forceinline__ void shade_path(const DeviceScene& sc, const FrameConstants& fc, const HitRecord& hit, V3 dir, Rng& rng,
                                           uint32_t& flags, float4& thr, const F3& li, V3& T, V3& L, V3& lsr, bool& terminate,
                                           bool& hasShadow, V3& nO, V3& nD, float4& sO, V3& sD, float& extOpacity,
                                           float& shadowOpacity DCRT_MCLK_PARAMS)
{
    const uint32_t bounce = flags & 0xFFu;
    const uint32_t features = fc.features;
    const bool vndf = (features & DCRT_FEATURE_GGX_SAMPLE_VNDF) != 0;
    const bool hasHit = hit.t != inf();
    Intersection it;
    it.lightIndex = DCRT_LIGHT_INDEX_INVALID; it.triangleIndex = 0;
    it.geometryNormal = mk(0.0f, 0.0f, 0.0f);
    if (hasHit) hit_to_intersection<CAPS>(sc, hit, it);
    DCRT_MCLK(1);
    T = mk(thr.x, thr.y, thr.z);
    L = mk(li.x, li.y, li.z);
    // Evaluate light :331-349
    {
        const uint32_t lightIndex = hasHit ? it.lightIndex : fc.envLightIndex;
        const bool visible = (features & DCRT_FEATURE_LIGHT_VISIBLE) != 0;
        if (visible ? lightIndex != DCRT_LIGHT_INDEX_INVALID : (bounce > 0 && lightIndex != DCRT_LIGHT_INDEX_INVALID)) {
            V3 radiance; float lightPdf;
            evaluate_light<CAPS>(sc, lightIndex, it.triangleIndex, it.geometryNormal, dir, hit.t, fc.lightCount, &radiance, &lightPdf);
            if (lightPdf > 0.0f) {
                const float weight = !(flags & kFlagDelta) ? power_heuristic(thr.w, lightPdf) : 1.0f;
                L = L + T * radiance * weight;
            }
        }
    }
    lsr = mk(0.0f, 0.0f, 0.0f);
    if (bounce > fc.maxBounce || !hasHit) {
        flags |= kFlagTerminate;
        terminate = true;
    } else {
        const V3 wo = -dir;
        const BsdfFrame bf = bsdf_frame(sc, wo, it);
        if (fc.lightCount != 0) {
            const LightSample ls = sample_light<CAPS>(sc, it.position, fc.lightCount, rng);
            if (any_pos(ls.radiance) && ls.pdf > 0.0f) {
                const V3 bsdf = evaluate_bsdf(sc, vndf, ls.wi, bf, it);
                const float NdotWI = fabsf(dot(it.normal, ls.wi));
                const float bsdfPdf = evaluate_bsdf_pdf(sc, vndf, ls.wi, bf, it);
                const float weight = ls.isDelta ? 1.0f : power_heuristic(ls.pdf, bsdfPdf);
                lsr = T * ls.radiance * bsdf * NdotWI * weight / ls.pdf;
                const V3 so = offset_ray_origin(it.position, it.geometryNormal, ls.wi);
                sO = make_float4(so.x, so.y, so.z, ls.distance);   // (written into the shadow
                sD = ls.wi;                                         //  queue after the append)
                hasShadow = true;
            }
        }
        DCRT_MCLK(3);
        float bsdfPdf = 0.0f;
        bool isDelta = false;
        {
            const float sel = next1(rng);
            const float sx = next1(rng), sy = next1(rng);
            V3 wi, bsdf;
            sample_bsdf(sc, vndf, bf, sx, sy, sel, it, &wi, &bsdf, &bsdfPdf, &isDelta);
            if ((bsdf.x != 0.0f || bsdf.y != 0.0f || bsdf.z != 0.0f) && bsdfPdf != 0.0f) {
                const float NdotWI = fabsf(dot(it.normal, wi));
                T = T * bsdf * NdotWI / bsdfPdf;
                nO = offset_ray_origin(it.position, it.geometryNormal, wi);
                nD = wi;   // (written into the extension queue after the append)
                flags = (flags & 0xFFFFFF00u) | ((bounce + 1) & 0xFFu);
            } else {
                flags |= kFlagTerminate;
                terminate = true;
            }
        }
        thr.w = bsdfPdf;
        flags = isDelta ? flags | kFlagDelta : flags & ~kFlagDelta;
        if (features & DCRT_FEATURE_ALLOW_ANYHIT) {   // :422-430 (the caller stores them)
            if (!terminate) extOpacity = next1(rng);
            if (hasShadow) shadowOpacity = next1(rng);
        }
    }
}

// ---- MATERIAL -----------------------------------------------------------------------
#ifndef DCRT_MATERIAL_BLOCK
#define DCRT_MATERIAL_BLOCK 256
#endif
static_assert(DCRT_MATERIAL_BLOCK % 64 == 0 && DCRT_MATERIAL_BLOCK <= 960, "MATERIAL workgroup: whole waves, at most 15 (block_append3)");
// The any-scene MATERIAL variant is held to 5 waves/SIMD (<= 96 VGPRs; 117 and 4 waves
// unbounded): it then spills 3 VGPRs and still gains, coffee 3.12 -> 3.02, lamp 7.78 ->
// 7.62 ms/spp (three / two A/B passes). The scene-specialised variants reach 5 waves by
// themselves (95 VGPRs); held to 5 the compiler schedules them into 91 and the Cornell
// bench loses 2 % (2.393 -> 2.447, four passes), so they are left unbounded.
#ifndef DCRT_MATERIAL_WAVES_PER_EU
#define DCRT_MATERIAL_WAVES_PER_EU 5
#endif
#ifndef DCRT_MATERIAL_OD_WAVES_PER_EU
#define DCRT_MATERIAL_OD_WAVES_PER_EU 1   // (the opaque / delta-light variants: the compiler's choice)
#endif
#define DCRT_MATERIAL_OCCUPANCY __attribute__((amdgpu_waves_per_eu(CAPS == kCapAll ? DCRT_MATERIAL_WAVES_PER_EU : DCRT_MATERIAL_OD_WAVES_PER_EU, 8)))
// CAPS: the scene capabilities this variant is compiled for (kCapAll = any scene; see
// kCapOpaqueDelta in dscene.h and dcrt_tracer::UploadScene).
// SCENE_LDS: the scene arrays MATERIAL's shading reads per item are copied into LDS by each
// workgroup first, so HitInfoToIntersection's dependent fetches are LDS reads -- 1: all of them
// (pre-gathered triangles, the forward instance transforms and instance words, materials,
// lights: small scenes, material_lds_bytes within the host's budget); 2: all but the triangles
// (larger scenes: the hit -> triangle fetch stays global, the triangle -> material one and the
// light sample's reads become LDS reads); 0: none.
// PROBE: counts the rays per film row (the row-cost probe); launched only while it is on.
template <uint32_t CAPS, int SCENE_LDS, bool PROBE = false>
__global__ __launch_bounds__(DCRT_MATERIAL_BLOCK) DCRT_MATERIAL_OCCUPANCY void material_kernel(PathPool pool, DeviceScene sc, const FrameConstants* __restrict__ fcr, Counters* cnt,
                                                                             const Counters* prev, const SampleOut* __restrict__ sampleOut)
{
#if defined(DCRT_MATERIAL_PRIO) && DCRT_MATERIAL_PRIO > 0
    __builtin_amdgcn_s_setprio(DCRT_MATERIAL_PRIO);   // (A/B: issue priority over a co-resident cast)
#endif
    __shared__ uint32_t sm[96];
    // the work list: the previous iteration's extension queue (its rays have been cast) -- or
    // a batch start's virtual queue (item i = path slot i, kVirtualWord)
    QueueMap qm;
    qmap(prev, kQExt, &qm);
    const uint32_t virt = virtual_items(prev);
    // (a work list drain_kernel already completed holds nothing)
    const uint32_t count = drained(prev) ? 0u : (virt ? virt : qm.prefix[kShards]);
    const uint32_t shard = blockIdx.x % kShards;
    const uint32_t fshard = blockIdx.x % kFinShards;
    // The frame constants through a restrict-qualified pointer: nothing this kernel stores
    // aliases them, so their reads in the item loop are scalar loads (scalar cache) -- through
    // the plain pointer they were vector loads, each waited on at once, several dependent round
    // trips per round.
    const FrameConstants& fcv = *fcr;
    if constexpr (SCENE_LDS != 0) {
        extern __shared__ float4 sceneLds[];
        if (blockIdx.x * blockDim.x >= count) return;   // (no item: no copy)
        const uint32_t T = SCENE_LDS == 1 ? sc.triangleCount : 0u, I = sc.instanceCount;
        float4* tv = sceneLds;
        float4* ts = tv + 3u * T;
        float4* tf = ts + 6u * T;
        uint32_t* w = (uint32_t*)(tf + 3u * I);
        uint32_t* li = w;
        uint32_t* ov = li + I;
        uint32_t* mt = ov + I;
        uint32_t* lt = mt + 13u * sc.ldsMaterials;
        for (uint32_t i = threadIdx.x; i < 3u * T; i += blockDim.x) tv[i] = sc.triVerts[i];
        for (uint32_t i = threadIdx.x; i < 6u * T; i += blockDim.x) ts[i] = sc.triShade[i];
        for (uint32_t i = threadIdx.x; i < 3u * I; i += blockDim.x) tf[i] = sc.transforms[i];
        for (uint32_t i = threadIdx.x; i < I; i += blockDim.x) { li[i] = sc.instanceLightIndices[i]; ov[i] = sc.overrides[i]; }
        for (uint32_t i = threadIdx.x; i < 13u * sc.ldsMaterials; i += blockDim.x) mt[i] = ((const uint32_t*)sc.materials)[i];
        for (uint32_t i = threadIdx.x; i < 7u * sc.ldsLights; i += blockDim.x) lt[i] = ((const uint32_t*)sc.lights)[i];
        __syncthreads();
        if constexpr (SCENE_LDS == 1) {
            sc.triVerts = tv;
            sc.triShade = ts;
        }
        sc.transforms = tf;
        sc.instanceLightIndices = li;
        sc.overrides = ov;
        sc.materials = (const dcrt_material*)mt;
        sc.lights = (const dcrt_light*)lt;
    }
    DCRT_MCLK_INIT;
    uint32_t itemsDone = 0;
    uint32_t round = 0;   // grid-stride round: alternates block_append2's sm halves
    for (uint32_t base = blockIdx.x * blockDim.x; base < count; base += gridDim.x * blockDim.x) {
    const uint32_t i = base + threadIdx.x;
    bool active = i < count;
    uint32_t newPixel = kNoPixel;   // a virtual item's pixel (a hole of the virtual queue has none)
    if (virt && active) {
        newPixel = slot(pool.pixel, i);
        active = newPixel != kNoPixel;
    }
    bool terminate = false, hasShadow = false, ends = false;
    uint32_t path = 0, pix = 0;
    float4 sample = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float2* outPos = nullptr;
    float4* outVal = nullptr;
    V3 nO = mk(0.0f, 0.0f, 0.0f), nD = mk(0.0f, 0.0f, 0.0f);   // the next extension ray
    float4 sO = make_float4(0.0f, 0.0f, 0.0f, 0.0f);            // the shadow ray (origin, tMax)
    V3 sD = mk(0.0f, 0.0f, 0.0f);
    // the path's state after this pass, stored at the positions the appends return
    uint32_t pathFlags = 0;
    float4 sThr = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    V3 sT = mk(0.0f, 0.0f, 0.0f), sL = mk(0.0f, 0.0f, 0.0f), sLsr = mk(0.0f, 0.0f, 0.0f);
    uint4 sRng = make_uint4(0u, 0u, 0u, 0u);
    if (active) {
        ++itemsDone;
        // Everything this pass reads is indexed by the item (no load waits for another):
        // the path's state record at its extension-queue position q, the cast's hit record
        // (with the ray's direction) at item i, the result of the path's last shadow ray at q
        // (only when it cast one: kFlagShadowPending)
        const float4 h4 = pool.hit[2 * i], hd = pool.hit[2 * i + 1];
        HitRecord hit;
        hit.t = h4.x; hit.u = h4.y; hit.v = h4.z; hit.tri = asu(h4.w); hit.inst = asu(hd.w);
        const V3 dir = mk(hd.x, hd.y, hd.z);
        Rng rng;
        uint32_t flags;
        float4 thr, l4, l2;
        bool shadowHit = false;
        if (virt) {
            // a virtual batch start's path (slot i): NEW_PATH's state (:227-237) recomputed from
            // its pixel -- the rng after the five camera draws, isDelta, bounce 0, T = 1,
            // bsdfPdf = 0, Li = 0, no light sampling result
            V3 unusedO, unusedD;
            rng = new_path<false>(fcv, newPixel, &unusedO, &unusedD);
            path = i;
            flags = kFlagDelta;
            thr = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
            l4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            l2 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        } else {
            const uint32_t q = qpos(pool.recCap, qm, i);
            const PathStateA& ps = state_at(pool.stateAPrev, q);
            const PathStateB& psB = state_at(pool.stateBPrev, q);
            // All of the item's loads in one round trip: both state halves and the shadow result
            // are read unconditionally (position q is always allocated; what the flags say is not
            // there is stale and not used) -- conditioned on the flags, the compiler issued them
            // only after the first half arrived, a second and third dependent round trip.
            const uint4 r4 = ps.rng;
            l2 = ps.lsrMisc;
            const float4 bThr = psB.thr, bLi = psB.liLsr;
            const uint32_t shRaw = pool.shadowHitPrev[q];
            rng.s0 = r4.x; rng.s1 = r4.y; rng.s2 = r4.z; rng.s3 = r4.w;
            path = asu(l2.w);
            flags = asu(l2.z);
            // a new path's first pass: NEW_PATH's constants, not the record's unwritten half
            const bool first = (flags & kFlagFirst) != 0u;
            thr = first ? make_float4(1.0f, 1.0f, 1.0f, 0.0f) : bThr;
            l4 = first ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : bLi;
            // the last shadow ray's result exists only if the path cast one (a position nothing
            // wrote this batch holds a stale value; its lsr is 0 then, but it is not read)
            shadowHit = (flags & kFlagShadowPending) != 0u && shRaw != 0u;
            flags &= ~(kFlagFirst | kFlagShadowPending);
        }
        F3 li{l4.x, l4.y, l4.z};
        {
            // CONTROL's Li += light sampling result (:520-528), done here for live paths (a
            // path without a shadow ray carries lsr = 0: Li + 0 either way)
            const F3 lsr0{l4.w, l2.x, l2.y};
            li.x = li.x + (!shadowHit ? lsr0.x : 0.0f);
            li.y = li.y + (!shadowHit ? lsr0.y : 0.0f);
            li.z = li.z + (!shadowHit ? lsr0.z : 0.0f);
        }
        // the slot index as a fresh value for the stores below: their addresses are then
        // formed where they are used instead of being shared with the loads' and kept
        // live in VGPR pairs across the whole shading code
        uint32_t out = path;
        asm volatile("" : "+v"(out));
        float extOpacity = 0.0f, shadowOpacity = 0.0f;
        V3 T, L, lsr;
        DCRT_MCLK(0);
        shade_path<CAPS>(sc, fcv, hit, dir, rng, flags, thr, li, T, L, lsr, terminate, hasShadow, nO, nD, sO, sD,
                         extOpacity, shadowOpacity DCRT_MCLK_ARGS);
        DCRT_MCLK(4);
        if (fcv.features & DCRT_FEATURE_ALLOW_ANYHIT) {   // :422-430
            if (!terminate) slot(pool.extOpacity, out) = extOpacity;
            if (hasShadow) slot(pool.shadowOpacity, out) = shadowOpacity;
        }
        ends = terminate && !hasShadow;
        // the row-cost probe (PROBE: the variant dcrt_tracer_set_row_cost_probe launches): the rays
        // of this pass per film row -- the extension ray this item shades and the shadow ray it
        // casts -- for cost-balanced film bands (partition.balanced_bands)
        if constexpr (PROBE) {
            uint32_t* rowRays = sampleOut->rowRays;
            const uint32_t p = virt ? newPixel : slot(pool.pixel, out);
            const uint32_t W = fcv.resolution[0], wh = W * fcv.resolution[1];
            atomicAdd(&rowRays[(p % wh) / W], hasShadow ? 2u : 1u);
        }
        // (the state written below goes to the queue positions the appends return)
        pathFlags = flags;
        sThr = thr;
        sT = T;
        sL = L;
        sLsr = lsr;
        sRng = make_uint4(rng.s0, rng.s1, rng.s2, rng.s3);
        if (ends || terminate) {
            // The path ends here with no shadow ray pending: all CONTROL would still do is
            // Li += light sampling result (0: the same bits as L + 0.0f) and WriteSample
            // (RayTracingCommon.inc.hlsl:118-122), so both happen in this pass and the slot
            // goes idle at once. (A path ending WITH a shadow ray pending goes to the finish
            // queue; CONTROL completes it. Its debug RNG state, final now, is stored here.)
            // The pixel is loaded here and the sample stored after the queue appends, whose
            // atomic round trip hides the load.
            const SampleOut so = *sampleOut;
            if (ends || so.debugRng) pix = slot(pool.pixel, out);
            if (ends) {
                sample = make_float4(L.x + 0.0f, L.y + 0.0f, L.z + 0.0f, 0.0f);
                // the sample pointers are read here too, not after the appends: read there
                // (behind the barriers and the atomic) they were one more round trip
                outPos = so.samplePosition;
                outVal = so.sampleValue;
            }
            if (so.debugRng) sample_at(so.debugRng, pix) = make_uint4(rng.s0, rng.s1, rng.s2, rng.s3);
        }
    }
    DCRT_MCLK(5);
    uint32_t es, ss;
    // (paths ended with a shadow ray pending: the next CONTROL pass completes them)
    const bool fin = active && terminate && hasShadow;
    uint32_t fb;
    block_append3(active && !terminate, qctr(cnt, kQExt, shard), active && hasShadow, qctr(cnt, kQShadow, shard),
                  fin, qctr(cnt, kQFinish, fshard), sm + (round & 1u) * 48u, &es, &ss, &fb);
    DCRT_MCLK(6);
    const uint32_t qNext = shard * pool.recCap + es;           // the continuing path's records
    const uint32_t fPos = fshard * pool.finCap + fb;           // a finishing path's record
    // An ended path's sample (and its slot's idle flag) is stored before the records: its
    // address needs the pixel load, and vmcnt counts loads and stores in issue order, so a
    // wait for the pixel issued after the record stores waited for all of them too. The empty
    // asm takes the pixel in every wave (whether or not one of its paths ended), so that wait
    // is placed here, ahead of every store, and not where the pixel's register is next reused.
    asm volatile("" ::"v"(pix));
    if (ends) {
        store_global(outPos, pix, pixel_sample(fcv, pix));
        store_global(outVal, pix, sample);
        slot(pool.flags, path) = kFlagIdle;
    }
    if (active && !terminate) {
        float4* r = ext_rec(pool.extRec, qNext);
        r[0] = make_float4(nO.x, nO.y, nO.z, 0.0f);
        r[1] = make_float4(nD.x, nD.y, nD.z, asf(path));
        PathStateA& st = state_at(pool.stateA, qNext);
        PathStateB& stB = state_at(pool.stateB, qNext);
        st.rng = sRng;
        stB.thr = make_float4(sT.x, sT.y, sT.z, sThr.w);
        stB.liLsr = make_float4(sL.x, sL.y, sL.z, sLsr.x);
        st.lsrMisc = make_float4(sLsr.y, sLsr.z, asf(pathFlags | (hasShadow ? kFlagShadowPending : 0u)), asf(path));
    }
    if (fin) {
        FinishRec& fr = pool.finRec[fPos];
        fr.liLsr = make_float4(sL.x, sL.y, sL.z, sLsr.x);
        fr.lsrSlot = make_float4(sLsr.y, sLsr.z, asf(path), 0.0f);
    }
    if (active && hasShadow) {
        const uint32_t sq = shard * pool.recCap + ss;
        float4* r = ext_rec(pool.shRec, sq);
        r[0] = sO;
        // where the shadow cast writes the result: the continuing path's next state, or its
        // finish record
        r[1] = make_float4(sD.x, sD.y, sD.z, asf(terminate ? (fPos | kDestFinish) : qNext));
        // the path slot beside it: only ALLOW_ANYHIT_SHADER's cast reads it (the shadow ray's
        // opacity sample is per slot)
        if (fcv.features & DCRT_FEATURE_ALLOW_ANYHIT) slot(pool.shadowQueue, sq) = path;
    }
    DCRT_MCLK(2);
    ++round;
    }
    DCRT_MCLK_FLUSH(itemsDone);
    (void)itemsDone;
}

// Cast-kernel occupancy: 5 waves per SIMD (<= 96 VGPRs; the compiler alone takes ~99,
// i.e. 4 waves). Measured on the 1080p Cornell bench, one pipeline: 4 waves 5.51,
// 5 waves 5.46, 6 waves 5.37, 7 waves 5.77 (spills), 8 waves 7.19 ms/spp; with the
// two concurrent pipelines of the default bench 5 waves leave the other pipeline's
// kernels room on the CU: 4.60 vs 4.66 ms/spp at 6 (3 repeats, tools/ab_libs.sh),
// although a lone launch is 3 % slower (106 vs 102.5 us).
#ifndef DCRT_CAST_WAVES_PER_EU
#define DCRT_CAST_WAVES_PER_EU 5
#endif
#if DCRT_CAST_WAVES_PER_EU > 0
#define DCRT_CAST_OCCUPANCY __attribute__((amdgpu_waves_per_eu(DCRT_CAST_WAVES_PER_EU, 8)))
#else
#define DCRT_CAST_OCCUPANCY
#endif
// The cache-only cast variant: 7 waves/SIMD (72 VGPRs, no spills; 6 waves at 74 VGPRs
// before the per-leaf shear: 2.96 vs 3.03 ms/spp, three A/B passes)
#ifndef DCRT_CACHED_CAST_WAVES_PER_EU
#define DCRT_CACHED_CAST_WAVES_PER_EU 7
#endif

// ---- EXTENSION_RAY_CAST / SHADOW_RAY_CAST ----------------------------------------------
// Persistent while-while loop with per-lane dynamic fetch: wave w owns items
// [w*chunk, (w+1)*chunk) of the queue; every step, lanes whose ray finished take
// the next items of the wave's range (ballot + mbcnt, no atomics), so all 64
// lanes keep traversing until the range is drained.

// log2(blockDim.x): traversal kernels run power-of-two workgroups (tracer.hip)
__device__ __forceinline__ uint32_t block_shift() { return 31u - (uint32_t)__clz((int)blockDim.x); }

#ifndef DCRT_VISITS_PER_CHECK
#define DCRT_VISITS_PER_CHECK 3
#endif
// node visits between two wave-level checks of the phase-A exit condition
constexpr int kVisitsPerCheck = DCRT_VISITS_PER_CHECK;
#ifndef DCRT_INTERLEAVE
#define DCRT_INTERLEAVE 64
#endif
// queue items per round-robin group of the cast kernels' static work split (power of two)
constexpr uint32_t kInterleave = DCRT_INTERLEAVE;
// PAIR (persistent_trace): phase A steps with trav_visit_pair instead of trav_visit. The
// tracer takes it for scenes whose nodes + triangles exceed an XCD's L2 (latency-bound
// fetches: spaceship 2.50 -> 2.46 ms/spp); on L2-resident scenes the second box test per
// step costs more than the shorter fetch chain saves (coffee 2.92 -> 3.02, lamp 7.21 ->
// 7.48). The test / megakernel paths always use it (the GPU parity tests cover it on every
// scene).

#ifdef DCRT_WAVE_TIMELINE
// Diagnostic build only (tools/wave_timeline.py): per-wave start/end realtime stamps
// and item counts of the cast kernels, 16 iteration slots x 8192 waves x 2 kernels.
__device__ unsigned long long g_waveLog[2][16][8192][2];
__device__ uint32_t g_waveItems[2][16][8192];
#define DCRT_WAVE_TAG(g) ((int)((g)->iterations & 15ull))
#else
#define DCRT_WAVE_TAG(g) (-1)
#endif


constexpr uint32_t kNoItem = 0xFFFFFFFFu;   // a fetch's "no ray for this item"
#ifndef DCRT_INLINE_ENTRY
#define DCRT_INLINE_ENTRY 1   // identity-instance BLAS entries in phase A (trav_visit ENTER)
#endif

// RING stacks: the lane's LDS stack is a window of sc.ringRows entries (dscene.h stack_row) over
// a per-lane global column (sc.spill). Before every batch of kVisitsPerCheck node visits the wave
// checks that each lane's window can take the batch: a visit writes the row above its top (push or
// not), so the window must hold at most ringRows - 1 entries before each visit, i.e. at most
// ringRows - kVisitsPerCheck before the batch; and a visit (or the following leaf work) pops at most one entry,
// so with entries spilled below the window it must hold at least kVisitsPerCheck + 1. A lane
// outside those bounds moves entries between the window and its spill column until the window
// holds ringRows / 2 (or every entry); the host keeps ringRows >= 2 * (kVisitsPerCheck + 1), so
// that window passes both checks (kMinRingRows). The entries' values and order are untouched: traversal,
// hits and counts are those of the whole-stack kernels bit for bit.
constexpr uint32_t kMinRingRows = 2u * ((uint32_t)kVisitsPerCheck + 1u);
template <bool RING>
__device__ __forceinline__ void ring_maintain(const DeviceScene& sc, TravState& s, bool active, uint32_t* lds, uint32_t shift)
{
    if constexpr (RING) {
        const uint32_t stride = 4u << shift;
        const uint32_t live = s.sp - s.base;
        const bool spill = active && live > (sc.ringRows - (uint32_t)kVisitsPerCheck) * stride;
        const bool fill = active && s.base != 0u && live <= (uint32_t)kVisitsPerCheck * stride;
        if (__builtin_expect(__ballot(spill | fill) != 0ull, 0)) {
            const uint32_t lanes = gridDim.x * blockDim.x;
            uint32_t* col = sc.spill + (size_t)blockIdx.x * blockDim.x + threadIdx.x;
            const uint32_t half = (sc.ringRows >> 1) * stride;
            const uint32_t target = s.sp > half ? s.sp - half : 0u;   // the new base
            if (spill) {
                // positions base + 1 .. target go to the column (entry e at col[(e - 1) * lanes])
                for (uint32_t p = s.base + stride; p <= target; p += stride)
                    col[(size_t)((p >> (shift + 2u)) - 1u) * lanes] = stack_at(lds, stack_row<true>(sc, p, shift));
                s.base = target;
            } else if (fill) {
                // positions target + 1 .. base come back into the window
                for (uint32_t p = target + stride; p <= s.base; p += stride)
                    stack_at(lds, stack_row<true>(sc, p, shift)) = col[(size_t)((p >> (shift + 2u)) - 1u) * lanes];
                s.base = target;
            }
        }
    }
}

template <bool ANY_HIT, bool INSTR, bool OPACITY, bool LANE_ANY = false, bool ALL_CACHED = false, bool PAIR = false,
          int LAYOUT = kLayoutScene, bool IDENT = false, bool RING = false, bool FLAT = false, typename Lookup, typename Fetch,
          typename Emit>
__device__ __forceinline__ void persistent_trace(const DeviceScene& sc, uint32_t n, uint32_t features, uint32_t kRefillLanes,
                                                 uint32_t kParkLanes, uint32_t* lds, uint32_t shift, Lookup lookup, Fetch fetch,
                                                 Emit emit, TraversalStats& st, int waveTag = -1)
{
    const bool watertight = (features & DCRT_FEATURE_WATERTIGHT) != 0;
    const bool f2b = (features & DCRT_FEATURE_NO_FRONT_TO_BACK) == 0;
    const uint32_t wavesPerBlock = blockDim.x >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t waves = gridDim.x * wavesPerBlock;
    const uint32_t waveId = blockIdx.x * wavesPerBlock + (threadIdx.x >> 6);
    // Work split: the queue is cut into groups of kInterleave consecutive items (one
    // region of the image / one producer workgroup each) dealt round-robin to the
    // waves, so every wave samples the whole queue and per-wave costs even out
    // (contiguous ranges follow the image's cost structure and leave the slowest
    // waves alone at the end). `cursor` and `end` count in the wave's own sequence.
    // A sparse queue (an image's drain: a few thousand long rays) is cut into smaller groups
    // -- the largest power of two <= n / (4 * waves), at least 1 -- so every wave gets some of
    // it: with 64-item groups the rays sat 64 to a wave on a few dozen waves (a handful of
    // CUs), and each of those waves took as long as its slowest lane plus every other lane's
    // leaf work. (At least 4 groups per wave keep the per-wave item counts within 5/4 of
    // each other.)
#ifndef DCRT_ADAPTIVE_GROUPS
#define DCRT_ADAPTIVE_GROUPS 1
#endif
    constexpr uint32_t kLgInterleave = 31u - __builtin_clz(kInterleave);
    const uint32_t perWave4 = n / (4u * waves);
    const uint32_t lg = !DCRT_ADAPTIVE_GROUPS || perWave4 >= kInterleave ? kLgInterleave : (perWave4 ? 31u - (uint32_t)__clz((int)perWave4) : 0u);
    const uint32_t gmask = (1u << lg) - 1u;
    const uint32_t groups = (n + gmask) >> lg;
    const uint32_t myGroups = groups > waveId ? (groups - waveId + waves - 1) / waves : 0u;
    uint32_t cursor = 0;
    const uint32_t end = myGroups << lg;
    const uint32_t chunk = end;   // (diagnostics)
    // (24-bit multiply: a 32-bit a * b + c becomes v_mad_u64_u32 with an arbitrary VGPR as
    // the unused high addend, which made the refill wait for the window's pending load)
    auto itemIndex = [&](uint32_t k) { return ((waveId + __umul24(k >> lg, waves)) << lg) + (k & gmask); };
    // lookup(i) is arithmetic only (a ray's record position in its queue): a refill waits for
    // the ray loads alone (the earlier 4-B queue entries needed a prefetch window of lookups
    // one refill ahead, a bpermute and a register)
    TravState s;
    // lane state, one integer (per-lane bools cost mask <-> register conversions per step):
    // kIdle no ray; kRun visiting nodes; kPark at a leaf (phase B work pending); kFin ray
    // finished, its result not yet written
    constexpr uint32_t kIdle = 0, kRun = 1, kPark = 2, kFin = 3;
    uint32_t ls = kIdle;
    uint32_t item = 0;
#ifdef DCRT_WAVE_TIMELINE
    const unsigned long long tStart = wall_clock64();
#endif
    DCRT_PHASE_INIT;
    for (;;) {
        DCRT_PHASE_COUNT(3);
        // refill only when at least kRefillLanes lanes are idle: the fetch (ray loads,
        // three IEEE divisions) is then shared by many lanes
        const bool free = ls == kIdle || ls == kFin;
        const unsigned long long need = __ballot(free);
        const uint32_t nNeed = (uint32_t)__popcll(need);
        const bool refill = nNeed >= kRefillLanes && cursor < end;
        const uint32_t k = cursor + __builtin_amdgcn_mbcnt_hi((uint32_t)(need >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)need, 0u));
        // Finished rays are written here, just before the ray loads (stores count in vmcnt
        // too: the loads are then not queued behind older stores' acknowledgements twice).
        if (ls == kFin) {
            emit(item, s);
            ls = kIdle;
        }
        if (refill) {
            const uint32_t idx = itemIndex(k);
            if (free && k < end && idx < n) {
                item = fetch(idx, lookup(idx), s);
                if (!f2b) s.negMask = 0u;
                if constexpr (!INSTR && !PAIR && !RING && !OPACITY) {
                    if (sc.skipRoot && item != kNoItem) trav_skip_root<ALL_CACHED, LAYOUT, IDENT>(sc, s, lds, shift);
                } else if constexpr (!INSTR && PAIR && !ALL_CACHED && !OPACITY) {
                    if (sc.skipRoot && item != kNoItem) trav_skip_root_pair(sc, s, lds, shift);
                }
                // (kNoItem: the queue item has no ray -- a hole of a virtual batch start)
                ls = item != kNoItem ? kRun : kIdle;
            }
            cursor += min(nNeed, end - cursor);
        }
        DCRT_PHASE(0);
        if (__ballot(ls != kIdle) == 0ull) break;
        // phase A: node visits only, until enough lanes are parked at leaves (or
        // enough are idle to refill, or none can advance)
        // (a lane whose ray ends here only flags it: the result is written at the next
        // refill point, which keeps the stores out of the unrolled visit steps)
        for (;;) {
            ring_maintain<RING>(sc, s, ls == kRun || ls == kPark, lds, shift);
#pragma unroll
            for (int k = 0; k < kVisitsPerCheck; ++k) {
                if (ls == kRun) {
                    const bool fin = PAIR && !INSTR && !ALL_CACHED ? trav_visit_pair<false, LAYOUT, RING>(sc, s, lds, shift)
                                                                   : trav_visit<INSTR, ALL_CACHED, LAYOUT, !FLAT && (ALL_CACHED || IDENT) && !OPACITY && DCRT_INLINE_ENTRY, IDENT, RING>(sc, s, lds, shift, st);
                    if (fin) ls = kFin;
                    else if (s.parked) ls = kPark;
                }
            }
            const unsigned long long runnable = __ballot(ls == kRun);
            const uint32_t parked = (uint32_t)__popcll(__ballot(ls == kPark));
            const uint32_t idle = 64u - (uint32_t)__popcll(runnable) - parked;
            DCRT_PHASE_COUNT(4);
#ifndef DCRT_ADAPTIVE_PARK
#define DCRT_ADAPTIVE_PARK 1
#endif
#ifndef DCRT_PARK_EIGHTHS
#define DCRT_PARK_EIGHTHS 4
#endif
            // leaf work once kParkLanes lanes wait at leaves -- or half of the wave's rays, when
            // it holds few (a drain's sparse waves: a lane parked at a leaf would otherwise wait
            // for every other ray to reach one)
            const uint32_t parkAt = DCRT_ADAPTIVE_PARK ? min(kParkLanes, max(1u, ((64u - idle) * DCRT_PARK_EIGHTHS) >> 3)) : kParkLanes;
            if (runnable == 0ull || parked >= parkAt || (idle >= kRefillLanes && cursor < end)) break;
        }
        DCRT_PHASE(1);
        // phase B: the parked lanes' leaf work, shared by many lanes at once
        if (__ballot(ls == kPark) != 0ull) DCRT_PHASE_COUNT(5);
        if (ls == kPark)
            ls = trav_leaf<ANY_HIT, INSTR, OPACITY, LANE_ANY, ALL_CACHED, IDENT, RING, FLAT>(sc, s, watertight, lds, shift, st) ? kFin : kRun;
        DCRT_PHASE(2);
    }
    DCRT_PHASE_FLUSH();
#ifdef DCRT_WAVE_TIMELINE
    if (waveTag >= 0 && n > 0 && (threadIdx.x & 63u) == 0 && waveId < 8192) {
        g_waveLog[ANY_HIT ? 1 : 0][waveTag & 15][waveId][0] = tStart;
        g_waveLog[ANY_HIT ? 1 : 0][waveTag & 15][waveId][1] = wall_clock64();
        g_waveItems[ANY_HIT ? 1 : 0][waveTag & 15][waveId] = chunk;
    }
#endif
}

// Kernel arguments the cast kernels select between per lane (extension vs shadow ray):
// pinned in SGPRs, so the select is a v_cndmask of two values and not a per-lane load
// of the pointer from the kernel-argument segment in front of every ray fetch.
// (The asm takes the pointer in the global address space and the result is cast back,
// so the loads through it stay global_load, not FLAT; the host pass only parses it.)
template <typename T>
__device__ __forceinline__ T* sgpr_ptr(T* p)
{
#if defined(__HIP_DEVICE_COMPILE__)
    __attribute__((address_space(1))) T* g = (__attribute__((address_space(1))) T*)p;
    asm volatile("" : "+s"(g));
    return (T*)g;
#else
    return p;
#endif
}

__device__ __forceinline__ void flush_stats(const TraversalStats& st, unsigned long long* dst)
{
    const unsigned long long a = wave_sum(st.nodes), b = wave_sum(st.tris), c = wave_sum(st.blas);
    if ((threadIdx.x & 63u) == 0 && (a | b | c)) { atomicAdd(&dst[0], a); atomicAdd(&dst[1], b); atomicAdd(&dst[2], c); }
}

// the wave's largest value into *dst (the longest ray's node visits)
__device__ __forceinline__ void flush_max(uint32_t v, unsigned long long* dst)
{
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
    if ((threadIdx.x & 63u) == 0 && v) atomicMax(dst, (unsigned long long)v);
}

// The extension cast's result at the ray's queue item: the hit and, for MATERIAL, the
// ray's direction and instance (so MATERIAL reads nothing of the ray record)
__device__ __forceinline__ void emit_hit(const PathPool& pool, uint32_t item, const TravState& s)
{
    float4* h = pool.hit + 2 * (size_t)item;
    h[0] = s.found ? make_float4(s.hit.t, s.hit.u, s.hit.v, asf(s.hit.tri)) : make_float4(inf(), 0.0f, 0.0f, 0.0f);
    h[1] = make_float4(s.d.x, s.d.y, s.d.z, asf(s.found ? s.hit.inst : 0u));
}
// The shadow cast's result where MATERIAL asked for it: the continuing path's next
// extension-queue position, or its finish-queue position (kDestFinish)
__device__ __forceinline__ void emit_occlusion(const PathPool& pool, uint32_t dest, const TravState& s)
{
    uint32_t* dst = (dest & kDestFinish) ? pool.finHit : pool.shadowHit;
    dst[dest & ~kDestFinish] = s.found ? 1u : 0u;
}

// OPACITY: the ALLOW_ANYHIT_SHADER variant (a separate instantiation, so the default
// kernels carry none of its state).
template <bool INSTR, bool OPACITY>
__global__ __launch_bounds__(256) DCRT_CAST_OCCUPANCY void extension_kernel(PathPool pool, DeviceScene sc, const FrameConstants* __restrict__ fc, const Counters* cnt,
                                                         Globals* g, unsigned long long* instr)
{
    extern __shared__ uint32_t stackMem[];
    scene_cache_load(sc, stackMem, block_shift());
    QueueMap qm;
    qmap(cnt, kQExt, &qm);
    TraversalStats st = {};
    persistent_trace<false, INSTR, OPACITY>(
        sc, qm.prefix[kShards], fc->features, fc->refillLanes, fc->parkLanes, stackMem + threadIdx.x, block_shift(),
        [&](uint32_t i) __attribute__((always_inline)) { return qpos(pool.recCap, qm, i); },
        [&](uint32_t i, uint32_t q, TravState& s) __attribute__((always_inline)) {
            const float4* r = ext_rec((const float4*)pool.extRec, q);
            const float4 o = r[0], d = r[1];
            trav_init(s, mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), 0.0f, inf());
            if (OPACITY) s.opacitySample = pool.extOpacity[asu(d.w) & ~kEntryFirst];
            return i;   // the result goes to the ray's queue item
        },
        [&](uint32_t item, const TravState& s) __attribute__((always_inline)) { emit_hit(pool, item, s); },
        st, DCRT_WAVE_TAG(g));
    if (INSTR) flush_stats(st, instr);
    (void)g;
}

// End of an iteration (after both casts): account it and clear the other parity's counters.
__device__ __forceinline__ void end_iteration(const Counters* cnt, Counters* nextCnt, Globals* g, uint32_t shadowRays)
{
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) {
            uint32_t fin = 0;
            for (uint32_t sh = 0; sh < kFinShards; ++sh) fin += qctr_load(cnt, kQFinish, sh);
            // (a virtual batch start's items: its cast counted the rays, holes excluded)
            const uint32_t virt = virtual_items(cnt);
            const uint32_t ext = virt ? virt : qtotal(cnt, kQExt);
            if (!virt) g->extRays += ext;
            g->shadowRays += shadowRays;
            g->iterations += 1ull;
            g->staticFill = 0u;   // only a batch's first CONTROL pass claims statically
            // IsImageComplete (WavefrontPathTracer.cpp:508-523), exact and on the device: no
            // path was live entering this iteration (so CONTROL's scan saw every slot idle)
            // and none was started
            const bool idle = g->prevLive == 0u && ext == 0u;
            g->poolIdle = idle ? 1u : 0u;
            g->imageComplete = (idle && !g->stopped) ? 1u : 0u;
            g->prevLive = ext + fin;
        }
        if (threadIdx.x < kCounterWords + 2) nextCnt->w[threadIdx.x * kShardStride] = 0u;   // (with kVirtual/kDrainedWord)
    }
}

template <bool INSTR, bool OPACITY>
__global__ __launch_bounds__(256) DCRT_CAST_OCCUPANCY void shadow_kernel(PathPool pool, DeviceScene sc, const FrameConstants* __restrict__ fc, Counters* cnt,
                                                      Counters* nextCnt, Globals* g, unsigned long long* instr)
{
    extern __shared__ uint32_t stackMem[];
    scene_cache_load(sc, stackMem, block_shift());
    QueueMap qm;
    qmap(cnt, kQShadow, &qm);
    const uint32_t n = qm.prefix[kShards];
    TraversalStats st = {};
    persistent_trace<true, INSTR, OPACITY>(
        sc, n, fc->features, fc->refillLanes, fc->parkLanes, stackMem + threadIdx.x, block_shift(),
        [&](uint32_t i) __attribute__((always_inline)) { return qpos(pool.recCap, qm, i); },
        [&](uint32_t i, uint32_t q, TravState& s) __attribute__((always_inline)) {
            const float4* r = ext_rec((const float4*)pool.shRec, q);
            const float4 o = r[0], d = r[1];
            trav_init(s, mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), 0.0f, o.w);
            if (OPACITY) s.opacitySample = pool.shadowOpacity[slot(pool.shadowQueue, q)];
            return asu(d.w);   // the result's destination (MATERIAL's kDestFinish code)
        },
        [&](uint32_t dest, const TravState& s) __attribute__((always_inline)) { emit_occlusion(pool, dest, s); },
        st, DCRT_WAVE_TAG(g));
    if (INSTR) flush_stats(st, instr + 3);
    end_iteration(cnt, nextCnt, g, n);
}

// EXTENSION_RAY_CAST + SHADOW_RAY_CAST in one persistent launch. The two queues are
// independent (MATERIAL filled both), so their items form one sequence (extension
// rays first) dealt to the waves like a single queue: one ramp and one drain per
// iteration instead of two, and a shadow ray can fill a lane an extension ray left
// idle. Per lane the ray keeps its own semantics (closest hit vs first hit), so the
// results are those of the two separate kernels.
// IDENT: the cache-only kernel of a scene whose instances all have the identity inverse
// (trav_visit): no instance-space ray, 8 waves/SIMD.
#ifndef DCRT_IDENT_CAST_WAVES_PER_EU
#define DCRT_IDENT_CAST_WAVES_PER_EU 8
#endif
// RING: the traversal stack as an LDS window over a per-lane global column (ring_maintain), for
// scenes whose whole stack would cost LDS occupancy (tracer.hip UploadScene).
// FLAT: the cache-only IDENT kernel over the entry-free node order (tracer.hip EntryFreeLayout)
template <bool INSTR, bool OPACITY, bool ALL_CACHED, bool PAIR, bool IDENT = false, bool RING = false, bool FLAT = false>
__global__ __launch_bounds__(256)
#ifndef DCRT_GLOBAL_CAST_WAVES_PER_EU
#define DCRT_GLOBAL_CAST_WAVES_PER_EU DCRT_CAST_WAVES_PER_EU   // (the global-memory, non-pair kernel; A/B)
#endif
__attribute__((amdgpu_waves_per_eu(ALL_CACHED && !OPACITY && !INSTR ? (IDENT ? DCRT_IDENT_CAST_WAVES_PER_EU : DCRT_CACHED_CAST_WAVES_PER_EU)
                                   : (!ALL_CACHED && !PAIR && !OPACITY && !INSTR ? DCRT_GLOBAL_CAST_WAVES_PER_EU : DCRT_CAST_WAVES_PER_EU), 8))) void cast_kernel(PathPool pool, DeviceScene sc, const FrameConstants* __restrict__ fc, Counters* cnt,
                                                                     Counters* nextCnt, Globals* g, unsigned long long* instr)
{
    extern __shared__ uint32_t stackMem[];
    scene_cache_load<ALL_CACHED>(sc, stackMem, block_shift());
    QueueMap qe, qs;
    qmap(cnt, kQExt, &qe);
    qmap(cnt, kQShadow, &qs);
    const uint32_t nExt = qe.prefix[kShards], nShadow = qs.prefix[kShards];
    const uint32_t* shQueue = sgpr_ptr(pool.shadowQueue);
    const float4* extRec = sgpr_ptr((const float4*)pool.extRec);
    const float4* shRec = sgpr_ptr((const float4*)pool.shRec);
    TraversalStats st = {};
    TraversalStats stExt = {}, stShadow = {};
    constexpr int kLayout = PAIR ? kLayoutPairs : (!INSTR || ALL_CACHED ? kLayoutFlat : kLayoutScene);
    const uint32_t virt = !OPACITY ? virtual_items(cnt) : 0u;
    if (!OPACITY && virt) {
        // A virtual batch start (control_kernel): item i is path slot i; its camera ray is
        // (the branch costs no registers: 74 / 72 / 77 VGPRs as without it, tools/vgprs.sh)
        // NEW_PATH's (new_path<true>) from the slot's pixel, its hit goes to item i. (The
        // shadow queue is empty: the previous batch drained.) The rays traced are counted
        // here -- the queue's holes are not rays.
        const FrameConstants& f = *fc;
        const uint32_t* pixels = sgpr_ptr((const uint32_t*)pool.pixel);
        uint32_t rays = 0;
        persistent_trace<false, INSTR, OPACITY, true, ALL_CACHED, PAIR, kLayout, IDENT, RING, FLAT>(
            sc, virt, f.features, f.refillLanes, f.parkLanes, stackMem + threadIdx.x, block_shift(),
            [&](uint32_t i) __attribute__((always_inline)) { return i; },
            [&](uint32_t i, uint32_t v, TravState& s) __attribute__((always_inline)) {
                const uint32_t p = slot(pixels, v);
                if (p == kNoPixel) return kNoItem;
                V3 o, d;
                (void)new_path<true>(f, p, &o, &d);
                trav_init(s, o, d, 0.0f, inf());
                s.anyHit = false;
                if (INSTR) st = TraversalStats{};
                ++rays;
                return i;
            },
            [&](uint32_t item, const TravState& s) __attribute__((always_inline)) {
                emit_hit(pool, item, s);
                if (INSTR) {
                    stExt.nodes += st.nodes; stExt.tris += st.tris; stExt.blas += st.blas;
                    stExt.maxNodes = max(stExt.maxNodes, st.nodes);
                }
            },
            st, DCRT_WAVE_TAG(g));
        const unsigned long long r = wave_sum(rays);
        if ((threadIdx.x & 63u) == 0 && r) atomicAdd(&g->extRays, r);
    } else {
    // (node order: the pair kernels run on pair-ordered scenes, the other non-counting ones on
    // PackBVH-ordered ones -- tracer.hip takes both from castPair -- the counting ones on either)
    persistent_trace<false, INSTR, OPACITY, true, ALL_CACHED, PAIR, kLayout, IDENT, RING, FLAT>(
        sc, nExt + nShadow, fc->features, fc->refillLanes, fc->parkLanes, stackMem + threadIdx.x, block_shift(),
        [&](uint32_t i) __attribute__((always_inline)) {
            // either kind: its record's position in its queue (no load)
            return i >= nExt ? qpos(pool.recCap, qs, i - nExt) : qpos(pool.recCap, qe, i);
        },
        [&](uint32_t i, uint32_t v, TravState& s) __attribute__((always_inline)) {
            const bool shadow = i >= nExt;
            // the ray's 32-B record at its queue position v (32-bit byte offsets: the records
            // stay below 4 GiB, dcrt_tracer::Create); a shadow ray's path slot beside it
            const float4* r = ext_rec(shadow ? shRec : extRec, v);
            const float4 o = r[0], d = r[1];
            trav_init(s, mk(o.x, o.y, o.z), mk(d.x, d.y, d.z), 0.0f, shadow ? o.w : inf());
            s.anyHit = shadow;
            if (OPACITY) {
                const uint32_t path = shadow ? slot(shQueue, v) : asu(d.w);
                s.opacitySample = shadow ? pool.shadowOpacity[path] : pool.extOpacity[path];
            }
            if (INSTR) st = TraversalStats{};
            // an extension ray's result goes to its queue item, a shadow ray's to the
            // destination MATERIAL put in its record
            return shadow ? asu(d.w) : i;
        },
        [&](uint32_t item, const TravState& s) __attribute__((always_inline)) {
            if (s.anyHit) emit_occlusion(pool, item, s);
            else emit_hit(pool, item, s);
            if (INSTR) {
                TraversalStats& dst = s.anyHit ? stShadow : stExt;
                dst.nodes += st.nodes; dst.tris += st.tris; dst.blas += st.blas;
                dst.maxNodes = max(dst.maxNodes, st.nodes);
#ifdef DCRT_PHASE_CLOCKS
                dst.cached += st.cached; dst.deep4 += st.deep4; dst.deep8 += st.deep8; dst.deep12 += st.deep12;
#endif
            }
        },
        st, DCRT_WAVE_TAG(g));
    }
    if (INSTR) {
        flush_stats(stExt, instr);
        flush_stats(stShadow, instr + 3);
        flush_max(stExt.maxNodes, instr + 6);
        flush_max(stShadow.maxNodes, instr + 7);
    }
#ifdef DCRT_PHASE_CLOCKS
    if (INSTR) {
        const unsigned long long c = wave_sum(stExt.cached + stShadow.cached), d4 = wave_sum(stExt.deep4 + stShadow.deep4),
                                 d8 = wave_sum(stExt.deep8 + stShadow.deep8), d12 = wave_sum(stExt.deep12 + stShadow.deep12);
        if ((threadIdx.x & 63u) == 0) {
            atomicAdd(&g_phaseClk[16], c); atomicAdd(&g_phaseClk[17], d4); atomicAdd(&g_phaseClk[18], d8); atomicAdd(&g_phaseClk[19], d12);
        }
    }
#endif
    end_iteration(cnt, nextCnt, g, nShadow);
}

// ---- GPU megakernel (MegakernelPathTracing.hlsl:65-208) -------------------------------------
// One lane traces one pixel's whole path; a fully finished wave claims the next 8x8
// pixel block (same per-shard cursors as CONTROL). Shares every device function with
// the wavefront kernels; differs from them only in the bounce-0 triangle-light
// emission, exactly like the reference's two tracers.
template <bool ANY_HIT, bool OPACITY>
__device__ __forceinline__ bool trace_full(const DeviceScene& sc, V3 o, V3 d, float tMax, bool watertight, bool f2b,
                                           float opacitySample, uint32_t* lds, uint32_t shift, HitRecord* hit)
{
    TravState s;
    trav_init(s, o, d, 0.0f, tMax, f2b);
    s.opacitySample = opacitySample;
    TraversalStats st = {};
    for (;;) {
        if (trav_visit_pair(sc, s, lds, shift)) break;
        if (s.parked && trav_leaf<ANY_HIT, false, OPACITY>(sc, s, watertight, lds, shift, st)) break;
    }
    *hit = s.hit;
    return s.found;
}

template <bool OPACITY>
__global__ __launch_bounds__(256) void megakernel(DeviceScene sc, const FrameConstants* __restrict__ fcp, Film film, Globals* g, uint32_t debugRng)
{
    extern __shared__ uint32_t stackMem[];
    scene_cache_load(sc, stackMem, block_shift());
    __shared__ uint32_t sm[64];
    const FrameConstants& fc = *fcp;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t shard = blockIdx.x % kShards;
    uint32_t* cursor = &g->nextBlock[shard * kShardStride];
    const uint32_t shardBlocks = g->totalBlocks > shard ? (g->totalBlocks - shard + kShards - 1) / kShards : 0u;
    const bool watertight = (fc.features & DCRT_FEATURE_WATERTIGHT) != 0;
    const bool f2b = (fc.features & DCRT_FEATURE_NO_FRONT_TO_BACK) == 0;
    const bool vndf = (fc.features & DCRT_FEATURE_GGX_SAMPLE_VNDF) != 0;
    const bool lightVisible = (fc.features & DCRT_FEATURE_LIGHT_VISIBLE) != 0;
    uint32_t* lds = stackMem + threadIdx.x;
    const uint32_t shift = block_shift();
    unsigned long long extRays = 0, shadowRays = 0;
    for (;;) {
        // every wave of the block claims one block per round (one atomic per workgroup)
        bool want = false;
        if (lane == 0) want = __hip_atomic_load(cursor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < shardBlocks;
        const uint32_t bslot = block_append(want, cursor, sm);
        const uint32_t claimed = (uint32_t)__shfl((int)bslot, 0, 64);
        const bool got = __shfl((int)want, 0, 64) != 0 && claimed < shardBlocks;
        if (__syncthreads_or(got ? 1 : 0) == 0) break;
        if (!got) continue;
        const uint32_t block = shard + claimed * kShards;
        uint32_t px = 0, py = 0, image = 0;
        if (!block_pixel(fc, film, block, lane, &px, &py, &image)) continue;
        Rng rng = rng_init(px, py, image_seed(fc, image));
        const float psx = next1(rng), psy = next1(rng);
        const float fsx = (psx + (float)px) / (float)fc.resolution[0];
        const float fsy = (psy + (float)py) / (float)fc.resolution[1];
        const float a0 = next1(rng), a1 = next1(rng), a2 = next1(rng);
        V3 ro, rd;
        generate_ray(fc, fsx, fsy, a0, a1, a2, &ro, &rd);
        V3 T = mk(1.0f, 1.0f, 1.0f), L = mk(0.0f, 0.0f, 0.0f);
        float bsdfPdfPrev = 0.0f;
        bool isDeltaPrev = true;
        uint32_t bounce = 0;
        for (;;) {
            HitRecord hit;
            ++extRays;
            // IntersectScene draws the ray's opacity sample (MegakernelPathTracing.hlsl:27-28)
            const float extOpacity = OPACITY ? next1(rng) : 0.0f;
            const bool hasHit = trace_full<false, OPACITY>(sc, ro, rd, inf(), watertight, f2b, extOpacity, lds, shift, &hit);
            const float hitT = hasHit ? hit.t : inf();
            Intersection it;
            it.lightIndex = DCRT_LIGHT_INDEX_INVALID; it.triangleIndex = 0;
            it.geometryNormal = mk(0.0f, 0.0f, 0.0f);
            if (hasHit) hit_to_intersection(sc, hit, it);
            {
                const uint32_t lightIndex = hasHit ? it.lightIndex : fc.envLightIndex;
                const bool doEval = lightVisible ? lightIndex != DCRT_LIGHT_INDEX_INVALID : (bounce > 0 && lightIndex != DCRT_LIGHT_INDEX_INVALID);
                if (doEval) {
                    if (bounce == 0) {
                        // MegakernelPathTracing.hlsl:135-140, 200-205
                        const dcrt_light& Lt = sc.lights[lightIndex];
                        const V3 rad = mk(Lt.radiance[0], Lt.radiance[1], Lt.radiance[2]);
                        if (hasHit) L = dot(-rd, it.geometryNormal) > 0.0f ? rad : mk(0.0f, 0.0f, 0.0f);
                        else L = sc.envCube ? sample_env(sc, rd) * rad : rad;
                    } else {
                        V3 radiance; float lightPdf;
                        evaluate_light(sc, lightIndex, it.triangleIndex, it.geometryNormal, rd, hitT, fc.lightCount, &radiance, &lightPdf);
                        if (lightPdf > 0.0f) {
                            const float weight = !isDeltaPrev ? power_heuristic(bsdfPdfPrev, lightPdf) : 1.0f;
                            L = L + T * radiance * weight;
                        }
                    }
                }
            }
            if (bounce > fc.maxBounce || !hasHit) break;
            const V3 wo = -rd;
            const BsdfFrame bf = bsdf_frame(sc, wo, it);
            V3 lsr = mk(0.0f, 0.0f, 0.0f);
            bool hasShadow = false;
            V3 so = mk(0.0f, 0.0f, 0.0f), sd = so;
            float sdist = 0.0f;
            if (fc.lightCount != 0) {
                const LightSample ls = sample_light(sc, it.position, fc.lightCount, rng);
                if (any_pos(ls.radiance) && ls.pdf > 0.0f) {
                    const V3 bsdf = evaluate_bsdf(sc, vndf, ls.wi, bf, it);
                    const float NdotWI = fabsf(dot(it.normal, ls.wi));
                    const float bsdfPdf = evaluate_bsdf_pdf(sc, vndf, ls.wi, bf, it);
                    const float weight = ls.isDelta ? 1.0f : power_heuristic(ls.pdf, bsdfPdf);
                    lsr = T * ls.radiance * bsdf * NdotWI * weight / ls.pdf;
                    so = offset_ray_origin(it.position, it.geometryNormal, ls.wi);
                    sd = ls.wi;
                    sdist = ls.distance;
                    hasShadow = true;
                }
            }
            // IsOcculuded draws its opacity sample before the BSDF sample (:57-58)
            const float shadowOpacity = OPACITY && hasShadow ? next1(rng) : 0.0f;
            bool terminate = false;
            {
                const float sel = next1(rng);
                const float sx = next1(rng), sy = next1(rng);
                V3 wi, bsdf;
                float bsdfPdf = 0.0f;
                bool isDelta = false;
                sample_bsdf(sc, vndf, bf, sx, sy, sel, it, &wi, &bsdf, &bsdfPdf, &isDelta);
                if ((bsdf.x != 0.0f || bsdf.y != 0.0f || bsdf.z != 0.0f) && bsdfPdf != 0.0f) {
                    const float NdotWI = fabsf(dot(it.normal, wi));
                    T = T * bsdf * NdotWI / bsdfPdf;
                    ro = offset_ray_origin(it.position, it.geometryNormal, wi);
                    rd = wi;
                    ++bounce;
                } else {
                    terminate = true;
                }
                bsdfPdfPrev = bsdfPdf;
                isDeltaPrev = isDelta;
            }
            if (hasShadow) {
                ++shadowRays;
                HitRecord sh;
                const bool occluded = trace_full<true, OPACITY>(sc, so, sd, sdist, watertight, f2b, shadowOpacity, lds, shift, &sh);
                if (!occluded) L = L + lsr;
            }
            if (terminate) break;
        }
        const size_t p = (size_t)image * film.width * film.height + (size_t)py * film.width + px;
        film.samplePosition[p] = make_float2(psx, psy);
        film.sampleValue[p] = make_float4(L.x, L.y, L.z, 0.0f);
        if (debugRng) film.debugRng[p] = make_uint4(rng.s0, rng.s1, rng.s2, rng.s3);
    }
    const unsigned long long e = wave_sum((uint32_t)extRays), sh = wave_sum((uint32_t)shadowRays);
    if (lane == 0) { atomicAdd(&g->extRays, e); atomicAdd(&g->shadowRays, sh); }
}

// ---- drain completion ----------------------------------------------------------------------
// Launched after every iteration's cast. Once a batch has no pixel block left to claim and
// at most fc.drainPaths paths are live, it runs each of them to its end in one lane, as the
// megakernel does, with the wavefront's arithmetic: the MATERIAL pass (shade_path) at the hit
// the cast just wrote, then the shadow ray, then the next extension ray, and so on, and the
// finish list's completion (CONTROL :520-528 + WriteSample) -- the same operations in the same
// order per path, so the same bits as the remaining iterations. A batch's drain iterations
// each took as long as their longest ray (a few thousand rays with 100-500 dependent node
// visits on the spaceship scene, 3 launches each); here a path's remaining rays follow each
// other in its lane and different paths overlap. The next iteration then finds the queues
// empty (kDrainedWord) and the batch complete.
template <uint32_t CAPS>
__global__ __launch_bounds__(256) void drain_kernel(PathPool pool, DeviceScene sc, const FrameConstants* __restrict__ fcp, Counters* cnt,
                                                    Globals* g, const SampleOut* __restrict__ sampleOut)
{
    const FrameConstants& fc = *fcp;
    if (!fc.drainPaths || g->stopped || virtual_items(cnt)) return;
    QueueMap qe;
    qmap(cnt, kQExt, &qe);
    QueueMapN<kFinShards> fm;
    qmap(cnt, kQFinish, &fm);
    const uint32_t nExt = qe.prefix[kShards], nFin = fm.prefix[kFinShards];
    if (nExt + nFin == 0u || nExt + nFin > fc.drainPaths) return;
    for (uint32_t sh = 0; sh < kShards; ++sh) {   // a block still to claim: new paths will follow
        const uint32_t blocks = g->totalBlocks > sh ? (g->totalBlocks - sh + kShards - 1) / kShards : 0u;
        if (__hip_atomic_load(&g->nextBlock[sh * kShardStride], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < blocks) return;
    }
    extern __shared__ uint32_t stackMem[];
    scene_cache_load(sc, stackMem, block_shift());
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        cnt->w[kDrainedWord * kShardStride] = 1u;   // the next MATERIAL / CONTROL pass: nothing to take
        g->prevLive = 0u;                           // (so the next iteration completes the batch)
    }
    const bool watertight = (fc.features & DCRT_FEATURE_WATERTIGHT) != 0;
    const bool f2b = (fc.features & DCRT_FEATURE_NO_FRONT_TO_BACK) == 0;
    uint32_t* lds = stackMem + threadIdx.x;
    const uint32_t shift = block_shift();
    const SampleOut so = *sampleOut;
    uint32_t extRays = 0, shadowRays = 0;
    // paths dealt to the waves first, lanes second (path w -> wave w mod waves, lane w / waves):
    // a wave runs a lane's path until that path ends, and its traversal and shading loops
    // last as long as their slowest lane, so few paths per wave let each path run at its own
    // chain's latency (the paths dealt to consecutive lanes had made every wave wait, bounce
    // by bounce, for its slowest path -- the wavefront's drain iterations again)
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    for (uint32_t w = (threadIdx.x & 63u) * waves + wave; w < nExt + nFin; w += 64u * waves) {
        if (w >= nExt) {
            // a path MATERIAL ended with its shadow ray pending (cast this iteration): CONTROL's
            // completion, as control_kernel does it
            const uint32_t f = qpos(pool.finCap, fm, w - nExt);
            const FinishRec fr = pool.finRec[f];
            const bool shadowHit = pool.finHit[f] != 0u;
            const uint32_t path = asu(fr.lsrSlot.z);
            F3 li{fr.liLsr.x, fr.liLsr.y, fr.liLsr.z};
            const F3 lsr{fr.liLsr.w, fr.lsrSlot.x, fr.lsrSlot.y};
            li.x = li.x + (!shadowHit ? lsr.x : 0.0f);
            li.y = li.y + (!shadowHit ? lsr.y : 0.0f);
            li.z = li.z + (!shadowHit ? lsr.z : 0.0f);
            const uint32_t p = slot(pool.pixel, path);
            sample_at(so.samplePosition, p) = pixel_sample(fc, p);
            sample_at(so.sampleValue, p) = make_float4(li.x, li.y, li.z, 0.0f);
            slot(pool.flags, path) = kFlagIdle;
            continue;
        }
        // a continuing path: its state at its extension-queue position, the hit at its item
        const uint32_t q = qpos(pool.recCap, qe, w);
        const PathStateA ps = state_at(pool.stateA, q);
        const float4 h4 = pool.hit[2 * w], hd = pool.hit[2 * w + 1];
        HitRecord hit;
        hit.t = h4.x; hit.u = h4.y; hit.v = h4.z; hit.tri = asu(h4.w); hit.inst = asu(hd.w);
        V3 dir = mk(hd.x, hd.y, hd.z);
        Rng rng;
        rng.s0 = ps.rng.x; rng.s1 = ps.rng.y; rng.s2 = ps.rng.z; rng.s3 = ps.rng.w;
        const uint32_t path = asu(ps.lsrMisc.w);
        uint32_t flags = asu(ps.lsrMisc.z);
        const bool first = (flags & kFlagFirst) != 0u;
        float4 thr = make_float4(1.0f, 1.0f, 1.0f, 0.0f), l4 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (!first) {
            const PathStateB psB = state_at(pool.stateB, q);
            thr = psB.thr;
            l4 = psB.liLsr;
        }
        bool shadowHit = (flags & kFlagShadowPending) ? pool.shadowHit[q] != 0u : false;
        flags &= ~(kFlagFirst | kFlagShadowPending);
        F3 li{l4.x, l4.y, l4.z};
        V3 lsr0 = mk(l4.w, ps.lsrMisc.x, ps.lsrMisc.y);
        for (;;) {
            li.x = li.x + (!shadowHit ? lsr0.x : 0.0f);
            li.y = li.y + (!shadowHit ? lsr0.y : 0.0f);
            li.z = li.z + (!shadowHit ? lsr0.z : 0.0f);
            bool terminate = false, hasShadow = false;
            V3 T, L, lsr, nO = mk(0.0f, 0.0f, 0.0f), nD = nO, sD = nO;
            float4 sO = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            float extOpacity = 0.0f, shadowOpacity = 0.0f;
            DCRT_MCLK_INIT;   // (the drain's sections are not reported)
            shade_path<CAPS>(sc, fc, hit, dir, rng, flags, thr, li, T, L, lsr, terminate, hasShadow, nO, nD, sO, sD,
                             extOpacity, shadowOpacity DCRT_MCLK_ARGS);
            shadowHit = false;
            if (hasShadow) {   // SHADOW_RAY_CAST
                HitRecord sh;
                shadowHit = trace_full<true, false>(sc, mk(sO.x, sO.y, sO.z), sD, sO.w, watertight, f2b, 0.0f, lds, shift, &sh);
                ++shadowRays;
            }
            if (terminate) {
                // MATERIAL's WriteSample (no shadow ray: L + 0) or CONTROL's (Li += lsr unless
                // the shadow ray hit)
                const uint32_t p = slot(pool.pixel, path);
                sample_at(so.samplePosition, p) = pixel_sample(fc, p);
                sample_at(so.sampleValue, p) = make_float4(L.x + (!shadowHit ? lsr.x : 0.0f), L.y + (!shadowHit ? lsr.y : 0.0f),
                                                           L.z + (!shadowHit ? lsr.z : 0.0f), 0.0f);
                if (so.debugRng) sample_at(so.debugRng, p) = make_uint4(rng.s0, rng.s1, rng.s2, rng.s3);
                slot(pool.flags, path) = kFlagIdle;
                break;
            }
            // EXTENSION_RAY_CAST of the next ray; the next MATERIAL pass's inputs
            if (!trace_full<false, false>(sc, nO, nD, inf(), watertight, f2b, 0.0f, lds, shift, &hit)) {
                hit.t = inf(); hit.u = 0.0f; hit.v = 0.0f; hit.tri = 0u; hit.inst = 0u;
            }
            ++extRays;
            dir = nD;
            thr = make_float4(T.x, T.y, T.z, thr.w);
            li = F3{L.x, L.y, L.z};
            lsr0 = lsr;
        }
    }
    const unsigned long long e = wave_sum(extRays), sr = wave_sum(shadowRays);
    if ((threadIdx.x & 63u) == 0) {
        if (e) atomicAdd(&g->extRays, e);
        if (sr) atomicAdd(&g->shadowRays, sr);
    }
}

// ---- kernel-level batch entry points (tests / roofline) -----------------------------------
// INSTR: count the reference's traversal (trav_visit); otherwise the kernels' trav_visit_pair
template <bool ANY, bool INSTR>
__global__ __launch_bounds__(256) void batch_trace_kernel(DeviceScene sc, const dcrt_ray* rays, uint32_t n, uint32_t features,
                                                           dcrt_ray_hit* hits, uint32_t* occluded, unsigned long long* instr)
{
    extern __shared__ uint32_t stackMem[];
    scene_cache_load(sc, stackMem, block_shift());
    TraversalStats st = {};
    persistent_trace<ANY, INSTR, false, false, false, !INSTR>(
        sc, n, features, 16u, 32u, stackMem + threadIdx.x, block_shift(),
        [&](uint32_t i) __attribute__((always_inline)) { return i; },
        [&](uint32_t i, uint32_t, TravState& s) __attribute__((always_inline)) {
            const dcrt_ray r = rays[i];
            trav_init(s, ld3(r.origin), ld3(r.direction), 0.0f, ANY ? r.t_max : inf());
            return i;
        },
        [&](uint32_t i, const TravState& s) __attribute__((always_inline)) {
            if (ANY) {
                occluded[i] = s.found ? 1u : 0u;
            } else {
                dcrt_ray_hit o;
                o.t = s.found ? s.hit.t : inf(); o.u = s.found ? s.hit.u : 0.0f; o.v = s.found ? s.hit.v : 0.0f;
                o.triangle_id = s.found ? s.hit.tri : 0u; o.instance_index = s.found ? s.hit.inst : 0u;
                hits[i] = o;
            }
        },
        st);
    if (INSTR) flush_stats(st, instr);
}

__global__ void math_eval_kernel(int function, const float* x, uint32_t n, float* y)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    switch (function) {
    case 0: y[i] = det_sin(x[i]); break;
    case 1: y[i] = det_cos(x[i]); break;
    case 2: y[i] = det_exp(x[i]); break;
    case 4: y[i] = det_log(x[i]); break;
    case 5: y[i] = rcp_ieee(x[i]); break;    // (the fast reciprocal against ...)
    case 6: y[i] = 1.0f / x[i]; break;       // (... the compiler's IEEE division)
    default: y[i] = det_atan(x[i]); break;
    }
}

// ---- SampleConvolution ----------------------------------------------------------------
struct FilterConsts { float radius, gaussianAlpha, gaussianExp, mf[7]; uint32_t tau, kind; };

__device__ __forceinline__ float filter_1d_sinc(float x) { x = fabsf(x); return x >= 1e-5f ? det_sin(3.1415926535f * x) / (3.1415926535f * x) : 1.0f; }
__device__ __forceinline__ float evaluate_filter(const FilterConsts& c, float px, float py)
{
    const float r = c.radius;
    switch (c.kind) {
    case DCRT_FILTER_TRIANGLE: return fmaxf(0.0f, r - fabsf(px)) * fmaxf(0.0f, r - fabsf(py));
    case DCRT_FILTER_GAUSSIAN: {
        const float gx = fmaxf(0.0f, det_exp(-c.gaussianAlpha * px * px) - c.gaussianExp);
        const float gy = fmaxf(0.0f, det_exp(-c.gaussianAlpha * py * py) - c.gaussianExp);
        return gx * gy;
    }
    case DCRT_FILTER_MITCHELL: {
        float v[2] = { px / c.radius, py / c.radius }, o[2];
        for (int k = 0; k < 2; ++k) {
            const float x = fabsf(2.0f * v[k]);
            float m = x < 1.0f ? c.mf[4] * x * x * x + c.mf[5] * x * x + c.mf[6]
                               : (x < 2.0f ? c.mf[0] * x * x * x + c.mf[1] * x * x + c.mf[2] * x + c.mf[3] : 0.0f);
            o[k] = m * (1.0f / 6.0f);
        }
        return o[0] * o[1];
    }
    case DCRT_FILTER_LANCZOS: {
        float o[2], v[2] = { px, py };
        for (int k = 0; k < 2; ++k) {
            const float x = fabsf(v[k]);
            const float lanczos = filter_1d_sinc(x / (float)c.tau);
            o[k] = x > r ? 0.0f : filter_1d_sinc(x) * lanczos;
        }
        return o[0] * o[1];
    }
    default: return (fabsf(px) <= r && fabsf(py) <= r) ? 1.0f : 0.0f;
    }
}

// SampleConvolution (SampleConvolution.hlsl:67-106), grid-stride over pixels. With
// `guard` set it runs only in the iteration that completed an image (RenderImages).
// One 16x16 pixel tile per workgroup: each image's samples of the tile plus the filter's
// halo are staged in LDS once (instead of every pixel fetching its (2r+1)^2 window from
// memory), then every pixel gathers its window from LDS. Per pixel the arithmetic and its
// order are those of the direct gather (images in order, window rows then columns).
#ifndef DCRT_FILM_TILE
#define DCRT_FILM_TILE 16
#endif
constexpr int kFilmTile = DCRT_FILM_TILE;   // (a workgroup per kFilmTile^2-pixel tile, one thread per pixel)
constexpr int kFilmThreads = kFilmTile * kFilmTile;
constexpr int kFilmMaxHalo = 4;
constexpr int kFilmSpan = kFilmTile + 2 * kFilmMaxHalo;
constexpr int kFilmStage = (kFilmSpan * kFilmSpan + kFilmThreads - 1) / kFilmThreads;   // staging elements per thread

__device__ __forceinline__ void film_pixel_window(const FilterConsts& c, uint32_t px, uint32_t py, uint32_t W, uint32_t H,
                                                  int* xs, int* xe, int* ys, int* ye)
{
    const float r = c.radius;
    const float cx = (float)px + 0.5f, cy = (float)py + 0.5f;
    *xs = (int)floorf(cx - r); *xs = *xs < 0 ? 0 : *xs;
    *xe = (int)floorf(cx + r); *xe = *xe > (int)W - 1 ? (int)W - 1 : *xe;
    *ys = (int)floorf(cy - r); *ys = *ys < 0 ? 0 : *ys;
    *ye = (int)floorf(cy + r); *ye = *ye > (int)H - 1 ? (int)H - 1 : *ye;
}

// posList / valList (accumulate_images): image b's sample textures sit at posList[b] / valList[b]
// (W*H each, e.g. other pipelines' slots) instead of at slot b of this film's.
__global__ __launch_bounds__(kFilmThreads) void film_kernel(Film film, const FilterConsts* fcon, uint32_t images, const Globals* guard,
                                                   const float2* const* __restrict__ posList,
                                                   const float4* const* __restrict__ valList)
{
    if (guard && (!guard->imageComplete || guard->skipFilm)) return;
    // the images of a completed batch, in order: per pixel the same additions as one
    // film pass per image
    const uint32_t count = guard ? guard->batchImages : images;
    const FilterConsts c = *fcon;
    const uint32_t W = film.width, H = film.height;
    const uint32_t total = W * H;
    const uint32_t tilesX = (W + kFilmTile - 1) / kFilmTile, tiles = tilesX * ((H + kFilmTile - 1) / kFilmTile);
    // two tile buffers: image b is convolved from buffer b & 1 while image b + 1's loads are in flight
    __shared__ float2 tPos[2][kFilmSpan * kFilmSpan];
    __shared__ float4 tVal[2][kFilmSpan * kFilmSpan];
    for (uint32_t tile = blockIdx.x; tile < tiles; tile += gridDim.x) {
        const int x0 = (int)(tile % tilesX) * kFilmTile, y0 = (int)(tile / tilesX) * kFilmTile;
        const uint32_t px = (uint32_t)x0 + (threadIdx.x % kFilmTile), py = (uint32_t)y0 + (threadIdx.x / kFilmTile);
        const bool mine = px < W && py < H && !(film.rowOwned && !film.rowOwned[py]);
        // a partitioned film's tiles without an owned pixel stage and convolve nothing
        // (at N ranks that is (N-1)/N of the tiles)
        if (film.rowOwned && !__syncthreads_or(mine)) continue;
        int xs = 0, xe = -1, ys = 0, ye = -1;
        float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (mine) {
            film_pixel_window(c, px, py, W, H, &xs, &xe, &ys, &ye);
            v = film.accum[(size_t)py * W + px];
        }
        // The tile's staged span is the union of its pixels' windows, taken from the
        // windows of its first and last pixel: floorf(p + 0.5 -/+ r) is monotone in p, so
        // every window of the tile lies inside, whatever the rounding of p + 0.5 + r does
        // (for r just below k + 0.5 a window can reach floor(r + 0.5) + 1 pixels out).
        int txs, txe, tys, tye, unused0, unused1;
        film_pixel_window(c, (uint32_t)x0, (uint32_t)y0, W, H, &txs, &unused0, &tys, &unused1);
        film_pixel_window(c, min((uint32_t)x0 + kFilmTile - 1u, W - 1u), min((uint32_t)y0 + kFilmTile - 1u, H - 1u), W, H,
                          &unused0, &txe, &unused1, &tye);
        const int spanX = txe - txs + 1, spanY = tye - tys + 1;
        if (spanX > kFilmSpan || spanY > kFilmSpan) {
            // wide filters: the direct gather from memory
            for (uint32_t b = 0; b < count && mine; ++b) {
                const float2* sPos = posList ? posList[b] : film.samplePosition + (size_t)b * total;
                const float4* sVal = valList ? valList[b] : film.sampleValue + (size_t)b * total;
                const float cx = (float)px + 0.5f, cy = (float)py + 0.5f;
                float wsum = 0.0f;
                V3 sum = mk(0.0f, 0.0f, 0.0f);
                for (int y = ys; y <= ye; ++y)
                    for (int x = xs; x <= xe; ++x) {
                        const size_t q = (size_t)y * W + x;
                        const float2 sp = sPos[q];
                        const float4 sv = sVal[q];
                        const float w = evaluate_filter(c, cx - (sp.x + (float)x), cy - (sp.y + (float)y));
                        sum = sum + mk(sv.x, sv.y, sv.z) * w;
                        wsum = wsum + w;
                    }
                v.x = v.x + sum.x; v.y = v.y + sum.y; v.z = v.z + sum.z; v.w = v.w + wsum;
            }
        } else {
            // staged span [txs, txe] x [tys, tye]: inside the film by construction
            const int span = spanX, ox = txs, oy = tys;
            // Software-pipelined over the images of a batch: image b + 1's tile is loaded into
            // registers while image b is convolved from its LDS buffer, and one barrier per image
            // separates the two buffers' writes from their reads. The barrier is s_barrier after
            // the LDS stores drain (lgkmcnt), not __syncthreads: that one's fence would also wait
            // for the next image's loads. (A buffer written at image b + 1 was last read at image
            // b - 1, which every thread finished before passing image b's barrier.)
            // (kFilmStage staging elements per thread, in registers: the loops below unroll)
            const int nStage = spanX * spanY;
            const size_t oFirst = (size_t)oy * W + (size_t)ox;
            size_t off[kFilmStage];
            float2 nP[kFilmStage];
            float4 nV[kFilmStage];
#pragma unroll
            for (int k = 0; k < kFilmStage; ++k) {
                const int i = (int)threadIdx.x + k * kFilmThreads;
                off[k] = i < nStage ? (size_t)(oy + i / spanX) * W + (size_t)(ox + i % spanX) : oFirst;
                nP[k] = make_float2(0.0f, 0.0f);
                nV[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            }
            // image b's sample textures: this film's slot b, or a list entry (accumulate_images),
            // read one image ahead with a vector load (the index made opaque to the uniformity
            // analysis: a scalar load would share lgkmcnt with the LDS traffic, whose waits would
            // then drain it too). The two sources run as two instances of the loop, so neither
            // carries the other's selects and register hazards.
            uint32_t lane0 = 0u;
            asm volatile("" : "+v"(lane0));
            auto run = [&](auto srcPos, auto srcVal) __attribute__((always_inline)) {
                // (unconditional loads: a thread without a third element loads the span's first
                // one again, so no branch splits the loads and their waits stay exact)
                auto stage_load = [&](const float2* lp, const float4* lv) __attribute__((always_inline)) {
#pragma unroll
                    for (int k = 0; k < kFilmStage; ++k) {
                        nP[k] = global_load2(lp, off[k]);
                        nV[k] = global_load4(lv, off[k]);
                    }
                };
                if (count > 0) stage_load(srcPos(0u), srcVal(0u));
                const float2* nextPos = count > 1 ? srcPos(1u) : nullptr;
                const float4* nextVal = count > 1 ? srcVal(1u) : nullptr;
                for (uint32_t b = 0; b < count; ++b) {
                    const uint32_t buf = b & 1u;
#pragma unroll
                    for (int k = 0; k < kFilmStage; ++k) {
                        const int i = (int)threadIdx.x + k * kFilmThreads;
                        if (i < nStage) {
                            tPos[buf][i] = nP[k];
                            tVal[buf][i] = nV[k];
                        }
                    }
                    if (b + 1 < count) {
                        stage_load(nextPos, nextVal);
                        if (b + 2 < count) { nextPos = srcPos(b + 2u); nextVal = srcVal(b + 2u); }
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                    if (mine) {
                        const float cx = (float)px + 0.5f, cy = (float)py + 0.5f;
                        float wsum = 0.0f;
                        V3 sum = mk(0.0f, 0.0f, 0.0f);
                        for (int y = ys; y <= ye; ++y)
                            for (int x = xs; x <= xe; ++x) {
                                const int i = (y - oy) * span + (x - ox);
                                const float2 sp = tPos[buf][i];
                                const float4 sv = tVal[buf][i];
                                const float w = evaluate_filter(c, cx - (sp.x + (float)x), cy - (sp.y + (float)y));
                                sum = sum + mk(sv.x, sv.y, sv.z) * w;
                                wsum = wsum + w;
                            }
                        v.x = v.x + sum.x; v.y = v.y + sum.y; v.z = v.z + sum.z; v.w = v.w + wsum;
                    }
                }
            };
            if (posList) {
                run([&](uint32_t b) __attribute__((always_inline)) { return (const float2*)global_load_u64((const uint64_t*)posList, b + lane0); },
                    [&](uint32_t b) __attribute__((always_inline)) { return (const float4*)global_load_u64((const uint64_t*)valList, b + lane0); });
            } else {
                run([&](uint32_t b) __attribute__((always_inline)) { return film.samplePosition + (size_t)b * total; },
                    [&](uint32_t b) __attribute__((always_inline)) { return film.sampleValue + (size_t)b * total; });
            }
        }
        if (mine) film.accum[(size_t)py * W + px] = v;
        __syncthreads();   // the tile buffers are reused by the next tile
    }
}

// film += src (dcrt_tracer_add_film_device): the films of disjoint film partitions
__global__ void add_film_kernel(float4* film, const float4* src, uint32_t n)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float4 a = film[i], b = src[i];
        film[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
}

// After the film pass of a completed batch: the next batch's first frame seed and
// size, rewind the block cursors.
__global__ void advance_image_kernel(FrameConstants* fc, Globals* g)
{
    if (threadIdx.x != 0 || !g->imageComplete) return;
    g->imageComplete = 0u;
    g->imagesDone += g->batchImages;
    if (g->imagesDone < g->imageTarget) {
        fc->frameSeed = g->seedBase + g->imagesDone * fc->seedStride;
        g->batchImages = min(g->batchCap, g->imageTarget - g->imagesDone);
        g->totalBlocks = fc->blocksPerImage * g->batchImages;
        begin_batch_claims(g);
    } else {
        g->stopped = 1u;
    }
}

__global__ void begin_images_kernel(Globals* g, const FrameConstants* fc, uint32_t count, uint32_t firstSeed, uint32_t batchCap,
                                    uint32_t staticGrid, uint32_t skipFilm)
{
    if (threadIdx.x != 0) return;
    g->skipFilm = skipFilm;
    g->imagesDone = 0u;
    g->imageTarget = count;
    g->seedBase = firstSeed;
    g->batchCap = batchCap;
    g->batchImages = min(batchCap, count);
    g->totalBlocks = fc->blocksPerImage * g->batchImages;
    g->stopped = count == 0u ? 1u : 0u;
    g->imageComplete = 0u;
    g->staticGrid = staticGrid;
    begin_batch_claims(g);
}

// ---- post-processing: SumLuminance.hlsl + PostProcessings.hlsl ---------------------------
__device__ __forceinline__ float4 film_load(const float4* film, uint32_t W, uint32_t H, uint32_t x, uint32_t y)
{
    return (x < W && y < H) ? film[(size_t)y * W + x] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // OOB Load -> 0
}
__device__ __forceinline__ float lum_log(float4 s)            // SumLuminance.hlsl:29-44
{
    V3 c = mk(0.0f, 0.0f, 0.0f);
    if (s.w > 0.0f) c = mk(s.x / s.w, s.y / s.w, s.z / s.w);
    c = mk(fminf(fmaxf(c.x, 0.0f), 65000.0f), fminf(fmaxf(c.y, 0.0f), 65000.0f), fminf(fmaxf(c.z, 0.0f), 65000.0f));
    const float lum = c.x * 0.299f + c.y * 0.587f + c.z * 0.114f;
    return det_log(0.0001f + lum);
}
// REDUCE_TO_1D: 8x8 groups, each thread four film texels, LDS tree 64 -> 1 (same order as the shader)
__global__ __launch_bounds__(64) void luminance_1d_kernel(const float4* film, uint32_t W, uint32_t H, uint32_t bx, uint32_t by, float* out)
{
    __shared__ float acc[64];
    const uint32_t tx = threadIdx.x & 7u, ty = threadIdx.x >> 3;
    const uint32_t x = blockIdx.x * 8 + tx, y = blockIdx.y * 8 + ty;
    float v = lum_log(film_load(film, W, H, x, y));
    v = v + lum_log(film_load(film, W, H, x + 8 * bx, y));
    v = v + lum_log(film_load(film, W, H, x, y + 8 * by));
    v = v + lum_log(film_load(film, W, H, x + 8 * bx, y + 8 * by));
    acc[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t k = 32; k >= 1; k >>= 1) {
        if (threadIdx.x < k) acc[threadIdx.x] = acc[threadIdx.x] + acc[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.y * bx + blockIdx.x] = acc[0];
}
// REDUCE_TO_SINGLE: 128-thread groups, LDS tree 128 -> 1
__global__ __launch_bounds__(128) void luminance_single_kernel(const float* in, uint32_t count, float* out)
{
    __shared__ float acc[128];
    const uint32_t i = blockIdx.x * 128 + threadIdx.x;
    acc[threadIdx.x] = i < count ? in[i] : 0.0f;
    __syncthreads();
    for (uint32_t k = 64; k >= 1; k >>= 1) {
        if (threadIdx.x < k) acc[threadIdx.x] = acc[threadIdx.x] + acc[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = acc[0];
}
// MainPS: rgb / w -> exposure -> Reinhard -> R8G8B8A8_UNORM_SRGB (encode by host-made thresholds)
__global__ __launch_bounds__(256) void postfx_kernel(const float4* film, uint32_t W, uint32_t H, int enabled, int autoExposure,
                                                     float ev100, float maxWhiteSqr, const float* sumLogLum,
                                                     const float* thresholds, uchar4* out)
{
    __shared__ float th[255];
    for (uint32_t t = threadIdx.x; t < 255; t += blockDim.x) th[t] = thresholds[t];
    __syncthreads();
    float exposure = 1.0f;
    if (enabled) {
        float e = ev100;
        if (autoExposure) {
            const float recip = 1.0f / (float)(W * H);
            const float avgLum = det_exp(sumLogLum[0] * recip);
            e = det_log(avgLum * 100.0f / 12.5f) * 1.44269504088896341f;
        }
        const float maxLuminance = 1.2f * det_exp(e * 0.693147180559945309f);
        exposure = 1.0f / maxLuminance;
    }
    for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < W * H; p += gridDim.x * blockDim.x) {
        const float4 f = film[p];
        float c[3] = { f.x / f.w, f.y / f.w, f.z / f.w };
        uint32_t code[3];
        for (int k = 0; k < 3; ++k) {
            float v = c[k];
            if (enabled) {
                v = v * exposure;
                v = v * (1.0f + v / maxWhiteSqr) / (1.0f + v);
            }
            v = v != v ? 0.0f : fminf(fmaxf(v, 0.0f), 1.0f);
            uint32_t n = 0;
            for (int t = 0; t < 255; ++t) n += v >= th[t] ? 1u : 0u;
            code[k] = n;
        }
        out[p] = make_uchar4((unsigned char)code[0], (unsigned char)code[1], (unsigned char)code[2], 255);
    }
}

// ---- BxDF LUT integration (BxDFTexturesBuilding.hlsl, "%f" defines) -------------------------
__global__ void lut_integrate_kernel(int which, uint32_t texels, float* out)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= texels) return;
    const float ix = 0.032258f;
    const float iy = which == 0 ? 0.032258f : 0.066667f;
    const float iz = which == 0 ? 1.0f : 0.133333f;
    const float sz = which == 0 ? 0.0f : 1.0f;
    const double weight = which == 2 ? 0.000010 : 0.000049;
    const uint32_t batches = which == 2 ? 24u : 5u;
    const uint32_t w = 32, h = which == 0 ? 32u : 16u;
    const uint32_t slice = t / (w * h), rem = t % (w * h);
    const uint32_t ty = rem / w, tx = rem % w;
    const bool entering = slice >= 16;
    const uint32_t tz = slice & 15u;
    const float cosThetaO = fmaxf((float)tx * ix, 0.0001f);
    const float alpha = (float)ty * iy;
    const float ior = (float)tz * iz + sz;
    const bool smooth = alpha < 0.00052441f;
    float acc = 0.0f;
    for (uint32_t batch = 0; batch < batches; ++batch) {
        Rng rng = rng_init(0, 0, batch);
        double result = batch == 0 ? 0.0 : (double)acc;
        for (uint32_t i = 0; i < 4096; ++i) {
            const V3 wo = mk(sqrtf(1.0f - cosThetaO * cosThetaO), 0.0f, cosThetaO);
            V3 wi = mk(0.0f, 0.0f, 0.0f);
            LCtx c; c.H = mk(0.0f, 0.0f, 0.0f); c.WOdotH = 0.0f;
            float value = 0.0f, pdf = 0.0f;
            if (which != 2) {
                if (smooth) {
                    wi = specular_brdf_sample(wo, &value, &pdf, c);
                } else {
                    const float sx = next1(rng), sy = next1(rng);
                    const V3 m = sample_vndf(wo, sx, sy, alpha);
                    wi = -reflect(wo, m);
                    c.H = m; c.WOdotH = dot(m, wo);
                    value = ct_brdf(wi, wo, alpha, c);
                    pdf = ct_brdf_pdf(true, wi, wo, alpha, c);
                }
                if (pdf > 0.0f) {
                    if (which == 1) {
                        const float etaO = entering ? ior : 1.0f, etaI = entering ? 1.0f : ior;
                        value = value * fresnel_dielectric(c.WOdotH, etaO, etaI);
                    }
                    result += weight * (double)value * (double)fabsf(wi.z) / (double)pdf;
                }
            } else {
                const float etaO = entering ? ior : 1.0f, etaI = entering ? 1.0f : ior;
                const float sel = next1(rng);
                if (smooth) {
                    wi = specular_bsdf_sample<true>(wo, sel, etaO, etaI, false, &value, &pdf, c);
                } else {
                    const float sx = next1(rng), sy = next1(rng);
                    wi = ct_bsdf_sample(true, wo, sel, sx, sy, alpha, etaO, etaI, c);
                    value = ct_bsdf<true>(wi, wo, alpha, etaO, etaI);
                    pdf = ct_bsdf_pdf(true, wi, wo, alpha, etaO, etaI);
                }
                if (pdf > 0.0f) result += weight * (double)value * (double)fabsf(wi.z) / (double)pdf;
            }
        }
        acc = (float)result;
    }
    out[t] = acc;
}

__device__ __forceinline__ uint16_t to_unorm16(float f) { return (uint16_t)rintf(saturate(f) * 65535.0f); }
__device__ __forceinline__ float average_row(const float* row)
{
    const uint32_t n = 31;
    const double fa = (double)(row[0] * 0.0001f);
    double sum = 0.0;
    for (uint32_t i = 1; i < n; ++i) {
        const double cosTheta = (double)((float)i * 0.032258f);
        sum += (double)saturate(row[i]) * cosTheta;
    }
    const double fb = (double)row[n];
    const double result = (sum + (fa + fb) * 0.5) * (double)(1.0f / (float)n);
    return (float)(result * 2.0);
}
__global__ void lut_finalize_kernel(const float* brdf, const float* brdfd, const float* bsdf, dcrt_bxdf_luts* L)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < DCRT_LUT_BRDF_COUNT) L->brdf[t] = to_unorm16(brdf[t]);
    if (t < DCRT_LUT_BRDF_DIELECTRIC_COUNT) { L->brdf_dielectric[t] = to_unorm16(brdfd[t]); L->bsdf[t] = to_unorm16(bsdf[t]); }
    if (t < 32) L->brdf_avg[t] = to_unorm16(average_row(brdf + t * 32));
    if (t < 512) {
        const uint32_t z = t / 16, y = t % 16;
        const uint32_t dest = (z / 16) * 256 + (z % 16) * 16 + y;
        L->brdf_dielectric_avg[dest] = to_unorm16(average_row(brdfd + (size_t)z * 512 + y * 32));
        L->bsdf_avg[dest] = to_unorm16(average_row(bsdf + (size_t)z * 512 + y * 32));
    }
}

// ---- explicit instantiations used by tracer.hip ---------------------------------------
template __global__ void extension_kernel<false, false>(PathPool, DeviceScene, const FrameConstants*, const Counters*, Globals*, unsigned long long*);
template __global__ void extension_kernel<false, true>(PathPool, DeviceScene, const FrameConstants*, const Counters*, Globals*, unsigned long long*);
template __global__ void extension_kernel<true, false>(PathPool, DeviceScene, const FrameConstants*, const Counters*, Globals*, unsigned long long*);
template __global__ void extension_kernel<true, true>(PathPool, DeviceScene, const FrameConstants*, const Counters*, Globals*, unsigned long long*);
template __global__ void shadow_kernel<false, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void shadow_kernel<false, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void shadow_kernel<true, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void shadow_kernel<true, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, false, false, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, false, true, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, true, false, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, true, true, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<true, false, false, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<true, false, true, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<true, true, false, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<true, true, true, false>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, false, false, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, true, false, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, false, true, false, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, false, true, false, true, false, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<true, false, true, false, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<false, false, false, false, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void cast_kernel<true, false, false, false, true>(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
template __global__ void megakernel<false>(DeviceScene, const FrameConstants*, Film, Globals*, uint32_t);
template __global__ void megakernel<true>(DeviceScene, const FrameConstants*, Film, Globals*, uint32_t);
template __global__ void batch_trace_kernel<false, false>(DeviceScene, const dcrt_ray*, uint32_t, uint32_t, dcrt_ray_hit*, uint32_t*, unsigned long long*);
template __global__ void batch_trace_kernel<true, false>(DeviceScene, const dcrt_ray*, uint32_t, uint32_t, dcrt_ray_hit*, uint32_t*, unsigned long long*);
template __global__ void batch_trace_kernel<false, true>(DeviceScene, const dcrt_ray*, uint32_t, uint32_t, dcrt_ray_hit*, uint32_t*, unsigned long long*);
template __global__ void batch_trace_kernel<true, true>(DeviceScene, const dcrt_ray*, uint32_t, uint32_t, dcrt_ray_hit*, uint32_t*, unsigned long long*);

}  // namespace dev
}  // namespace dcrt
