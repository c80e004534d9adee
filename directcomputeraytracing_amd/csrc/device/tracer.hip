// tracer.hip -- CWavefrontPathTracer on MI355X: pool allocation, scene upload,
// the per-iteration launch sequence (captured into a hipGraph), image
// completion, film accumulation, and the extern "C" tracer API of dcrt.h.
// Reference: Source/WavefrontPathTracer.cpp:70-1162, Source/Scene.cpp:273-608,
// Source/SampleConvolution.cpp:89-170, Source/BxDFTexturesBuilding.cpp:106-475.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <limits>
#include <vector>

#include "../../../include/dcrt.h"
#include "kernels_impl.h"

namespace dcrt {
void SetLastError(const std::string& s);
}
using dcrt::SetLastError;
using namespace dcrt::dev;

#define HIPCHECK(expr)                                                                              \
    do {                                                                                            \
        hipError_t e_ = (expr);                                                                     \
        if (e_ != hipSuccess) {                                                                     \
            SetLastError(std::string(#expr) + " failed: " + hipGetErrorString(e_));                 \
            return DCRT_E_HIP;                                                                      \
        }                                                                                           \
    } while (0)
#define CHECKED(expr)                      \
    do {                                   \
        const int r_ = (expr);             \
        if (r_ != DCRT_OK) return r_;      \
    } while (0)

namespace {

constexpr uint32_t kDefaultPoolSize = 1u << 20;      // 2^20 slots: 16 waves x 256 CUs x 256 (MI355X)
constexpr uint32_t kDefaultIterations = 8;
// RenderImages' chunks of iterations once its final batch is in flight: a chunk launched after
// the images completed finds no work, and two chunks are in flight when the host sees it
constexpr uint32_t kTailChunk = 4;
constexpr uint32_t kMaxImageBatch = 256;              // images in flight per RenderImages batch (sample textures: 24 B/px each)
#ifndef DCRT_MATERIAL_BLOCK
#define DCRT_MATERIAL_BLOCK 256
#endif
constexpr uint32_t kMaterialBlock = DCRT_MATERIAL_BLOCK;   // MATERIAL workgroup (one queue-append atomic each)
constexpr uint32_t kMaxPersistentBlocks = 256 * 8;   // CUs x resident workgroups

// (A/B knobs of AutoBatch)
uint32_t kMaxImageBatchAuto()
{
    static const uint32_t v = [] {
        const char* e = std::getenv("DCRT_MAX_BATCH");
        const int x = e ? std::atoi(e) : (int)kMaxImageBatch;
        return (uint32_t)std::min<int>(std::max<int>(x, 1), (int)kMaxImageBatch);
    }();
    return v;
}
bool BatchPoolLimit()
{
    static const bool v = [] { const char* e = std::getenv("DCRT_BATCH_POOL_LIMIT"); return !e || std::atoi(e) != 0; }();
    return v;
}

template <typename T>
int DeviceAlloc(T** p, size_t count, std::vector<void*>* owner)
{
    *p = nullptr;
    if (count == 0) count = 1;
    void* q = nullptr;
    HIPCHECK(hipMalloc(&q, count * sizeof(T)));
    *p = (T*)q;
    if (owner) owner->push_back(q);
    return DCRT_OK;
}
void FreeAll(std::vector<void*>* v)
{
    for (void* p : *v) (void)hipFree(p);
    v->clear();
}

FilterConsts MakeFilter(const dcrt_filter_params& p)   // SampleConvolution.cpp:100-130
{
    FilterConsts c;
    std::memset(&c, 0, sizeof(c));
    c.kind = p.filter;
    c.radius = p.radius;
    if (p.filter == DCRT_FILTER_GAUSSIAN) {
        c.gaussianAlpha = p.gaussian_alpha;
        c.gaussianExp = std::exp(-p.gaussian_alpha * p.radius * p.radius);
    } else if (p.filter == DCRT_FILTER_MITCHELL) {
        const float B = p.mitchell_b, C = p.mitchell_c;
        c.mf[0] = -B - 6 * C; c.mf[1] = 6 * B + 30 * C; c.mf[2] = -12 * B - 48 * C; c.mf[3] = 8 * B + 24 * C;
        c.mf[4] = 12 - 9 * B - 6 * C; c.mf[5] = -18 + 12 * B + 6 * C; c.mf[6] = 6 - 2 * B;
    } else if (p.filter == DCRT_FILTER_LANCZOS) {
        c.tau = p.lanczos_tau ? p.lanczos_tau : 3;
    }
    return c;
}

// Rows beyond its own that a film row's SampleConvolution window reaches
// (SampleConvolution.hlsl:77-81), with the kernel's float arithmetic
// (film_pixel_window): floor(r + 0.5) in exact arithmetic, one more where py + 0.5 + r
// rounds up to the next integer (r just below k + 0.5).
// roctx ranges around the host-side passes, named like the reference's PIX annotations
// (SCOPED_RENDER_ANNOTATION, WavefrontPathTracer.cpp:443-1083): visible in rocprofv3
// --marker-trace next to the kernels. rocprofiler-sdk's roctx (the one rocprofv3 intercepts;
// the legacy libroctx64 as a fallback) is opened at run time (no link dependency; absent, or
// DCRT_ROCTX=0: no ranges). Iterations captured into a hipGraph are annotated by
// their replay ("RenderImages" / graph chunks), not per kernel.
struct Roctx {
    int (*push)(const char*) = nullptr;
    int (*pop)() = nullptr;
    Roctx()
    {
        if (const char* e = std::getenv("DCRT_ROCTX")) {
            if (std::atoi(e) == 0) return;
        }
        void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
        pop = (int (*)())dlsym(h, "roctxRangePop");
        if (!push || !pop) push = nullptr, pop = nullptr;
    }
};
const Roctx& roctx()
{
    static const Roctx r;
    return r;
}
struct Annotation {
    bool on;
    explicit Annotation(const char* name, bool enabled = true) : on(enabled && roctx().push)
    {
        if (on) roctx().push(name);
    }
    ~Annotation()
    {
        if (on) roctx().pop();
    }
};

uint32_t FilterSupportRows(float r, uint32_t H)
{
    if (!(r < (float)H)) return H;
    uint32_t rows = 0;
    for (uint32_t py = 0; py < H; ++py) {
        const float cy = (float)py + 0.5f;
        int ys = (int)std::floor(cy - r), ye = (int)std::floor(cy + r);
        ys = std::max(ys, 0);
        ye = std::min(ye, (int)H - 1);
        rows = std::max<uint32_t>(rows, (uint32_t)std::max(ye - (int)py, (int)py - ys));
    }
    return rows;
}

using CastFn = void (*)(PathPool, DeviceScene, const FrameConstants*, Counters*, Counters*, Globals*, unsigned long long*);
// cast_kernel variant: instrumented counts x ALLOW_ANYHIT_SHADER x whole scene in the LDS cache
// x pair-expanding traversal (the non-counting kernels of scenes not in the LDS cache) x the
// world ray in every space (IDENT) x the spilling stack window (RING: non-counting, opaque,
// global-memory kernels)
CastFn CastKernel(bool instr, bool opacity, bool allCached, bool pair, bool ident = false, bool ring = false, bool flat = false)
{
    if (flat && ident && allCached && !opacity && !instr && !ring) return cast_kernel<false, false, true, false, true, false, true>;
    if (ring && !instr && !opacity && !allCached) {
        if (pair) return cast_kernel<false, false, false, true, false, true>;
        return ident ? cast_kernel<false, false, false, false, true, true> : cast_kernel<false, false, false, false, false, true>;
    }
    if (ident && allCached && !opacity) return instr ? cast_kernel<true, false, true, false, true> : cast_kernel<false, false, true, false, true>;
    if (ident && !opacity && (instr || !pair)) return instr ? cast_kernel<true, false, false, false, true> : cast_kernel<false, false, false, false, true>;
    static const CastFn table[8] = {
        cast_kernel<false, false, false, false>, cast_kernel<false, false, true, false>, cast_kernel<false, true, false, false>,
        cast_kernel<false, true, true, false>, cast_kernel<true, false, false, false>, cast_kernel<true, false, true, false>,
        cast_kernel<true, true, false, false>, cast_kernel<true, true, true, false>};
    if (pair && !instr && !allCached) return opacity ? cast_kernel<false, true, false, true> : cast_kernel<false, false, false, true>;
    return table[(instr ? 4 : 0) + (opacity ? 2 : 0) + (allCached ? 1 : 0)];
}

// Workgroups per CU that a workgroup's LDS allocation allows. hipOccupancyMaxActiveBlocksPerMultiprocessor
// rounds the allocation to 512 B, but gfx950 allocates LDS in 1280-B granules (160 KiB / 128). Measured
// on the persistent cast grid (one workgroup per resident slot): 6 x 26944 B and 5 x 32768 B per CU
// ran with 5 and 4 workgroups resident (the last one as a tail: cast launches +26 % / +29 %), while
// 6 x 26608 B ran with 6 -- the 1280-B rounding predicts all three (profiles/r04_ab_round4.txt).
// `lds` counts a workgroup's dynamic LDS; the kernel's static LDS (hipFuncAttributes
// sharedSizeBytes, e.g. the megakernel's claim words) comes on top of it. The per-CU total is the
// device's (maxSharedMemoryPerMultiProcessor: 160 KiB on gfx950, the only target this library is
// built for); the 1280-B granule is gfx950's.
size_t g_ldsPerCU = 163840;
constexpr size_t kLdsGranule = 1280;
int LdsResident(size_t lds, const void* kernel = nullptr)
{
    if (kernel) {
        hipFuncAttributes attr{};
        if (hipFuncGetAttributes(&attr, kernel) == hipSuccess) lds += attr.sharedSizeBytes;
    }
    return lds ? (int)(g_ldsPerCU / ((lds + kLdsGranule - 1) / kLdsGranule * kLdsGranule)) : 1 << 20;
}

// The LDS stack depth traversal of the uploaded tree needs: the most interior nodes on
// any root-to-leaf path through a TLAS leaf into its BLAS (each descent pushes the far
// child; BVHAccel.inc.hlsl:143-154). Children lie after their parent (depth-first
// layout), BLAS roots after the TLAS; anything else is malformed (false).
bool RequiredTraversalStack(const dcrt_flat_scene& s, uint32_t* out)
{
    const uint32_t n = s.bvh_node_count;
    *out = 0;
    if (n == 0) return true;
    std::vector<uint32_t> blasDepth(n, UINT32_MAX);   // memo: deepest path below a BLAS root
    // every node is reached at most once per walk: a tree. A node reached twice (a child
    // shared between parents, a cycle) is malformed -- and would make the walk exponential
    std::vector<uint32_t> seen(n, UINT32_MAX);        // the walk that last reached the node
    uint32_t walkId = 0;
    struct Item { uint32_t node, depth; };
    std::vector<Item> todo;
    auto walk = [&](uint32_t root, bool tlas, uint32_t* deepest) {
        ++walkId;
        todo.assign(1, { root, 0u });
        *deepest = 0;
        while (!todo.empty()) {
            const Item it = todo.back();
            todo.pop_back();
            if (seen[it.node] == walkId) return false;
            seen[it.node] = walkId;
            const dcrt_bvh_node& nd = s.bvh_nodes[it.node];
            if (nd.misc >= 4u) {   // a leaf
                uint32_t d = it.depth;
                if (tlas && (nd.misc & 4u)) {
                    const uint32_t b = nd.right_child_or_prim_index;
                    if (b >= n || b < s.tlas_node_count) return false;
                    d += blasDepth[b];
                }
                *deepest = std::max(*deepest, d);
                continue;
            }
            const uint32_t right = nd.right_child_or_prim_index;
            if (it.node + 1 >= n || right <= it.node || right >= n) return false;
            todo.push_back({ it.node + 1, it.depth + 1 });
            todo.push_back({ right, it.depth + 1 });
        }
        return true;
    };
    // BLAS roots: the TLAS leaves' targets
    for (uint32_t i = 0; i < std::min(s.tlas_node_count, n); ++i) {
        const dcrt_bvh_node& nd = s.bvh_nodes[i];
        if (!(nd.misc & 4u)) continue;
        const uint32_t b = nd.right_child_or_prim_index;
        if (b >= n || b < s.tlas_node_count) return false;
        if (blasDepth[b] != UINT32_MAX) continue;
        uint32_t d = 0;
        if (!walk(b, false, &d)) return false;
        blasDepth[b] = d;
    }
    return walk(0, true, out);
}

// The child-pair node order (dscene.h kLayoutPairs): an interior node's two children
// adjacent, its `right` field the first child's device index, a TLAS leaf's the BLAS root's.
// The levels nearest the roots come first -- the TLAS root and every BLAS root, breadth-first
// until at least `topNodes` nodes are placed: what the LDS scene cache (a prefix) and the L2
// hold -- then every subtree below them depth-first by child pairs. Each root gets a padded
// slot, so every pair starts at an even index (one 64-B aligned line). Traversal follows the
// tree, not the indices: hits, node counts and stack depths are those of the flat order.
// quads (the default; DCRT_NODE_QUADS=0: off): below the top levels the children pairs of a node's two children
// sit side by side in one 128-B aligned line (a padded half where a child is a leaf), so the
// fetch that expands one child brings its sibling's children into L2 with it; otherwise a
// node's left child's pair follows the node's own pair depth-first.
// Call after RequiredTraversalStack (which checks every reference); false if a node would be
// placed twice (a child shared between parents).
bool PairLayout(const dcrt_flat_scene& s, uint32_t topNodes, std::vector<dcrt_bvh_node>* out, bool quads = false)
{
    constexpr uint32_t kNone = UINT32_MAX;
    const dcrt_bvh_node* nd = s.bvh_nodes;
    std::vector<uint32_t> pos(s.bvh_node_count, kNone);   // flat index -> device index
    std::vector<uint32_t> order;                          // device index -> flat index (kNone: padding)
    order.reserve((size_t)s.bvh_node_count + 64);
    auto isLeaf = [&](uint32_t i) { return nd[i].misc >= 4u; };
    auto place = [&](uint32_t i) {
        if (pos[i] != kNone) return false;
        pos[i] = (uint32_t)order.size();
        order.push_back(i);
        return true;
    };
    // an interior node's children, left then right, at the next (even) device index
    auto placeChildren = [&](uint32_t p) { return place(p + 1) && place(nd[p].right_child_or_prim_index); };
    std::vector<uint32_t> level, next, stack;
    auto addRoot = [&](uint32_t r) {
        if (pos[r] != kNone) return;   // a BLAS shared by several instances
        place(r);
        order.push_back(kNone);
        if (!isLeaf(r)) level.push_back(r);
    };
    addRoot(0);
    for (uint32_t i = 0; i < std::min(s.tlas_node_count, s.bvh_node_count); ++i)
        if ((nd[i].misc & 4u) && nd[i].misc >= 4u) addRoot(nd[i].right_child_or_prim_index);
    while (!level.empty() && order.size() < topNodes) {
        next.clear();
        for (const uint32_t p : level) {
            if (!placeChildren(p)) return false;
            if (!isLeaf(p + 1)) next.push_back(p + 1);
            if (!isLeaf(nd[p].right_child_or_prim_index)) next.push_back(nd[p].right_child_or_prim_index);
        }
        level.swap(next);
    }
    for (const uint32_t root : level) {
        stack.assign(1, root);
        if (quads) {
            // stack: nodes whose children are placed; expanding one places its children's pairs
            if (!placeChildren(root)) return false;
            while (!stack.empty()) {
                const uint32_t p = stack.back();
                stack.pop_back();
                const uint32_t c0 = p + 1, c1 = nd[p].right_child_or_prim_index;
                if (isLeaf(c0) && isLeaf(c1)) continue;
                while (order.size() & 3u) order.push_back(kNone);   // one 128-B line
                if (!isLeaf(c0) && !placeChildren(c0)) return false;
                if (!isLeaf(c1) && !placeChildren(c1)) return false;
                if (!isLeaf(c1)) stack.push_back(c1);
                if (!isLeaf(c0)) stack.push_back(c0);   // the left subtree first
            }
            continue;
        }
        while (!stack.empty()) {
            const uint32_t p = stack.back();
            stack.pop_back();
            if (!placeChildren(p)) return false;
            if (!isLeaf(nd[p].right_child_or_prim_index)) stack.push_back(nd[p].right_child_or_prim_index);
            if (!isLeaf(p + 1)) stack.push_back(p + 1);   // the left subtree's pairs first
        }
    }
    out->assign(order.size(), dcrt_bvh_node{});
    for (size_t k = 0; k < order.size(); ++k) {
        if (order[k] == kNone) continue;
        dcrt_bvh_node v = nd[order[k]];
        if (v.misc < 4u) v.right_child_or_prim_index = pos[order[k] + 1];
        else if (v.misc & 4u) v.right_child_or_prim_index = pos[v.right_child_or_prim_index];
        (*out)[k] = v;
    }
    return true;
}

// The entry-free node order of the cache-only IDENT kernel (cast_kernel<..., FLAT>; every instance's
// inverse exactly the identity, single-triangle leaves). A TLAS leaf whose box is its BLAS root's bit
// for bit is replaced by (a copy of) that root: the root's visit would repeat the leaf's box test with
// the same world ray and tMax (IDENT), so skipping it changes no hit. Any other TLAS leaf becomes an interior node (misc 3:
// its near child is taken by negMask bit 3, the front-to-back flag) whose children are an empty node
// and a copy of its instance's BLAS; the BLAS triangle leaves carry instance + 1 in their count field.
// The kernel then has no BLAS-entry step in its node visit: the TLAS leaf's box is tested as before,
// the BLAS root is visited next (or after the empty node, which no ray hits: all its planes are +inf,
// so its slab interval is empty or starts at +inf), and hits, their order and their tMax are the
// reference's bit for bit -- the empty node adds a visit and a stack entry (the kernel's stack has
// one row more), no triangle test. (The counting kernels keep PackBVH's order and their counts are
// the reference's.) False if a leaf holds more than one triangle.
bool EntryFreeLayout(const dcrt_flat_scene& s, std::vector<dcrt_bvh_node>* out, bool merge = true)
{
    const dcrt_bvh_node* nd = s.bvh_nodes;
    const uint32_t n = s.bvh_node_count;
    out->clear();
    out->reserve((size_t)n + 2u * s.instance_count);
    bool ok = true;
    // (explicit stack: (node, instance + 1 or 0 in the TLAS, the slot whose `right` field takes it))
    struct Item { uint32_t node, inst1, parent; };
    std::vector<Item> todo{{0u, 0u, UINT32_MAX}};
    while (!todo.empty() && ok) {
        const Item it = todo.back();
        todo.pop_back();
        if (it.node >= n) { ok = false; break; }
        const uint32_t idx = (uint32_t)out->size();
        if (it.parent != UINT32_MAX) (*out)[it.parent].right_child_or_prim_index = idx;
        dcrt_bvh_node v = nd[it.node];
        if (it.inst1 == 0u && (v.misc & 0x4u)) {
            const uint32_t inst = (v.misc >> 3) & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT;
            const uint32_t blas = v.right_child_or_prim_index;
            if (merge && blas < n && inst + 1u <= DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT &&
                std::memcmp(v.bbox_min, nd[blas].bbox_min, sizeof(v.bbox_min)) == 0 &&
                std::memcmp(v.bbox_max, nd[blas].bbox_max, sizeof(v.bbox_max)) == 0) {
                // the BLAS root's box is the TLAS leaf's bit for bit (an identity instance's bounds
                // usually are): its visit would repeat the leaf's test with the same ray and tMax,
                // so the root takes the leaf's place and the ray enters with no visit of its own
                todo.push_back({blas, inst + 1u, it.parent});
                continue;
            }
        }
        if (it.inst1 == 0u && (v.misc & 0x4u)) {
            // TLAS leaf -> interior node: left child the empty node, right child the BLAS copy
            const uint32_t inst = (v.misc >> 3) & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT;
            if (inst + 1u > DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT) { ok = false; break; }
            const uint32_t blas = v.right_child_or_prim_index;
            v.misc = 3u;
            out->push_back(v);
            dcrt_bvh_node empty{};
            const float inf = std::numeric_limits<float>::infinity();
            empty.bbox_min[0] = empty.bbox_min[1] = empty.bbox_min[2] = inf;
            empty.bbox_max[0] = empty.bbox_max[1] = empty.bbox_max[2] = inf;
            empty.misc = 0u;
            out->push_back(empty);
            todo.push_back({blas, inst + 1u, idx});
        } else if (v.misc >= 4u) {
            // BLAS triangle leaf (a TLAS-level triangle leaf cannot exist)
            if (it.inst1 == 0u || ((v.misc >> 3) & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT) != 1u) { ok = false; break; }
            v.misc = (v.misc & 0x7u) | (it.inst1 << 3);
            out->push_back(v);
        } else {
            // interior: the left child (node + 1) right behind it, the right child after its subtree
            out->push_back(v);
            todo.push_back({v.right_child_or_prim_index, it.inst1, idx});
            todo.push_back({it.node + 1u, it.inst1, UINT32_MAX});
        }
        if (out->size() > (size_t)n * 4u + 64u) { ok = false; break; }   // (a malformed tree: refuse)
    }
    return ok && !out->empty();
}

}  // namespace

struct dcrt_tracer {
    int device = 0;
    hipStream_t stream = nullptr;
    bool ownsStream = false;
    uint32_t poolSize = 0;
    // CONTROL / MATERIAL grids (ResidentGrid): workgroups that loop over the pool's 256-slot
    // "virtual workgroups" vb = blockIdx.x + round * gridDim.x
    uint32_t controlGrid = 0, materialGrid = 0;
    uint32_t materialLds = 0;          // MATERIAL's dynamic LDS: the scene copy's bytes (0: the global-memory variant)
    uint32_t materialLdsMode = 0;      // material_kernel<CAPS, mode>: 0 no copy, 1 whole shading data, 2 all but the triangles
    bool castIdent = false;            // cache-only cast kernel without instance space (every instance the identity: dscene.h IDENT)
    uint32_t iterationsPerRender = kDefaultIterations;
    bool debugRng = false;
    // cast-kernel refill / park thresholds (persistent_trace): refill when 36 lanes are idle
    // in the LDS-only kernel, 28 in the global-memory one (round 3 sweep with the adaptive
    // park threshold); park at 24 (profiles/r01_tune_sweep.txt); DCRT_TRAVERSAL_TUNE=
    // "refill,park" overrides both
    uint32_t refillLanes = 36, parkLanes = 24;
    bool tuneOverride = false;
    uint64_t imagesCompleted = 0;                // since the last ResetStats (counters())

    std::vector<void*> poolAllocs, sceneAllocs, filmAllocs, sampleAllocs, rowAllocs;
    PathPool pool{};                   // (queue pointers set per launch: LaunchIteration)
    float4* extRecs = nullptr;         // 2 parities x kShards x recCap extension-ray records (2 float4)
    PathStateA* stateRecsA = nullptr;  // 2 parities x kShards x recCap path state halves
    PathStateB* stateRecsB = nullptr;
    uint32_t* shadowHits = nullptr;    // 2 parities x kShards x recCap shadow results
    FinishRec* finRecs = nullptr;      // 2 parities x kFinShards x pool.finCap
    uint32_t* finHits = nullptr;       // 2 parities x kFinShards x pool.finCap
    DeviceScene scene{};
    bool hasScene = false;
    uint32_t castBlock = 256;
    size_t castLds = 0;
    size_t castLdsFull = 0;            // the layout of every kernel but the ring cast: stackSize + 2 rows + the cache
    uint32_t ringRows = 0;             // the ring cast kernel's LDS stack window (0: whole stack in LDS)
    DeviceScene sceneRing{};           // the scene as the ring cast kernel sees it (stackRows = ringRows, spill column)
    bool castFlat = false;             // the cache-only IDENT cast runs on the entry-free node order (EntryFreeLayout)
    DeviceScene sceneFlat{};           // the scene as that kernel sees it (its nodes, one more stack row)
    size_t castLdsFlat = 0;
    uint32_t castPerCU = 0;            // resident cast workgroups per CU
    bool castAllCached = false;        // the scene fits the LDS cache: cast_kernel<., ., true, .>
    bool castPair = false;             // trav_visit_pair: the scene outgrows an XCD's L2 (UploadScene)
    bool mergedCasts = true;           // one cast_kernel per iteration (DCRT_SPLIT_CASTS=1: EXT then SHADOW)
    bool virtualStart = true;          // virtual batch starts where the cast kernel has them (DCRT_VIRTUAL_START=0: off)
    uint32_t sceneCaps = kCapAll;      // what the uploaded scene uses (kCap* of dscene.h)
    uint32_t materialCaps = kCapAll;   // the MATERIAL variant launched for it

    dcrt_bxdf_luts* dLuts = nullptr;
    Film film{};
    uint32_t filmW = 0, filmH = 0;
    uint32_t rowCount = 0;             // rows this tracer path-traces (film.rowY)
    uint32_t bandCount = 0;            // ceil(rowCount / 8): block rows of an image
    uint32_t sampleImages = 0;         // images the sample textures hold (batch capacity)
    uint32_t batchImages = 0;          // RenderImages batch size (0: automatic)
    uint32_t lastSlot = 0;             // sample slot of the last completed image
    uint32_t seedStride = 1;           // RenderImages: image k has frame seed first + k * seedStride
    bool keptSlots = false;            // the last RenderImages left image k's samples in slot k (no film pass)
    uint32_t keptImages = 0;
    void** dSourceLists = nullptr;     // accumulate_images: device copies of the caller's pointer lists
    uint32_t sourceCap = 0;
    dcrt_film_partition partition{ 1, 0, 64, 0 };
    std::vector<uint32_t> bands;       // explicit film bands [y0, y1) pairs (dcrt_tracer_set_film_bands), or empty

    dcrt_frame_params frame{};
    bool hasFrame = false;
    FrameConstants* dFrame = nullptr;
    Counters* dCounters = nullptr;     // [2]
    Globals* dGlobals = nullptr;
    SampleOut* dSampleOut = nullptr;   // MATERIAL's copy of the sample pointers (EnsureSamples)
    SampleOut hSampleOut = {};
    unsigned long long* dInstr = nullptr;   // [8]
    Counters* hCounters = nullptr;     // pinned [2]

    bool newImage = true;
    bool capturing = false;            // LaunchIteration is being captured into a graph (no host annotations)
    bool imageComplete = false;
    bool filmClearTrigger = false;
    uint32_t parity = 0;

    // graphs of `iters` iterations (even), rebuilt when launch parameters change;
    // [0] = plain iterations (Render), [1] = with the guarded film pass and image
    // advance (RenderImages)
    struct GraphCache {
        hipGraphExec_t exec = nullptr;
        uint32_t iters = 0;
    } graphs[3];   // unsequenced (Render), sequenced (RenderImages), sequenced tail chunks
    FilterConsts* dFilter = nullptr;
    FilterConsts* hFilter = nullptr;   // pinned staging
    uint32_t* hStop = nullptr;         // pinned [4][2]: Globals::stopped, imagesDone per poll
    hipEvent_t stopEvents[4] = {};
    bool instrCounters = false;
    bool extTiming = false;
    bool rowProbe = false;             // the row-cost probe: MATERIAL's PROBE variant counts rays per film row
    uint32_t* dRowRays = nullptr;      // [filmH] (rowAllocs: follows the film)
    // timed launches (ext_timing): start / stop event pairs and the kernel each pair timed
    enum TimedKind : uint8_t { kTimedCast = 0, kTimedMaterial = 1, kTimedControl = 2, kTimedKinds = 3 };
    std::vector<hipEvent_t> events;
    std::vector<uint8_t> eventKinds;   // per pair
    size_t eventsUsed = 0;
    double kindMs[kTimedKinds] = {};
    uint64_t kindLaunches[kTimedKinds] = {};
    int TimedPair(TimedKind kind, hipEvent_t* e0, hipEvent_t* e1)
    {
        while (events.size() < eventsUsed + 2) {
            hipEvent_t e;
            HIPCHECK(hipEventCreate(&e));
            events.push_back(e);
        }
        eventKinds.resize(events.size() / 2);
        eventKinds[eventsUsed / 2] = kind;
        *e0 = events[eventsUsed++];
        *e1 = events[eventsUsed++];
        return DCRT_OK;
    }
    int CollectTimes()   // fold the recorded pairs into kindMs / kindLaunches
    {
        for (size_t i = 0; i + 1 < eventsUsed; i += 2) {
            float e = 0.0f;
            HIPCHECK(hipEventElapsedTime(&e, events[i], events[i + 1]));
            kindMs[eventKinds[i / 2]] += e;
            ++kindLaunches[eventKinds[i / 2]];
        }
        eventsUsed = 0;
        return DCRT_OK;
    }

    ~dcrt_tracer();
    int Create(const dcrt_tracer_config& cfg);
    int BuildLuts();
    int UploadScene(const dcrt_flat_scene& s);
    int SetFrame(const dcrt_frame_params& p);
    int SetPartition(const dcrt_film_partition& p);
    int SetBands(const uint32_t* b, uint32_t count, uint32_t halo);
    int EnsureFilm(uint32_t w, uint32_t h);
    int BuildRows();
    int UploadSampleOut();
    int SetRowProbe(bool on);
    int EnsureSamples(uint32_t images);
    uint32_t AutoBatch(uint32_t count) const;
    int BeginImage();
    int LaunchIteration(uint32_t par, bool timed, bool sequenced);
    int LaunchGraph(bool sequenced, uint32_t iters);
    int BuildGraph(bool sequenced, uint32_t iters);
    int PrepareImages(uint32_t count);
    int RunIterations(uint32_t n);
    int UploadFilter(const dcrt_filter_params& f);
    int ReadCompletion(bool* complete);
    int Render(uint32_t maxIterations);
    int RenderImages(uint32_t firstSeed, uint32_t count, const dcrt_filter_params& filter, uint32_t stride = 1,
                     bool convolve = true);
    int AccumulateImages(const void* const* pos, const void* const* val, uint32_t count, const dcrt_filter_params& filter);
    int Accumulate(const dcrt_filter_params& filter);
    void InvalidateGraph()
    {
        for (GraphCache& g : graphs) {
            if (g.exec) (void)hipGraphExecDestroy(g.exec);
            g.exec = nullptr;
            g.iters = 0;
        }
    }
    // film_kernel: one 16x16 tile per workgroup (grid-stride beyond the cap)
    uint32_t FilmGrid() const
    {
        const uint32_t T = (uint32_t)kFilmTile;
        return std::max<uint32_t>(1u, std::min<uint32_t>(((filmW + T - 1) / T) * ((filmH + T - 1) / T), 8u * kMaxPersistentBlocks * (256u / kFilmThreads)));
    }
    uint32_t castResident = 0;         // persistent cast grid: resident workgroups on the whole chip
    uint32_t castResidentOpacity = 0;  // the same for the ALLOW_ANYHIT_SHADER variant
    uint32_t megaResident = 0;         // persistent megakernel grid
    uint32_t drainResident = 0;        // drain_kernel grid (resident workgroups)
    uint32_t drainPaths = 0;           // drain_kernel threshold (DCRT_DRAIN_PATHS; 0: no drain launches -- the default: profiles/r04_ab_virtual_drain.txt)
    int mode = 0;                      // 0 wavefront (WavefrontPathTracer), 1 megakernel (MegakernelPathTracer)
    uint32_t castResidentInstr = 0;    // the same for the counting kernels (whole stack: castLdsFull)
    uint32_t castResidentInstrOpacity = 0;
    uint32_t CastGrid(uint32_t block, bool opacity) const
    {
        const uint32_t resident = instrCounters ? (opacity ? castResidentInstrOpacity : castResidentInstr)
                                                : (opacity ? castResidentOpacity : castResident);
        return std::min<uint32_t>((poolSize + block - 1) / block, resident);
    }
};

dcrt_tracer::~dcrt_tracer()
{
    (void)hipSetDevice(device);
    if (stream) (void)hipStreamSynchronize(stream);
    InvalidateGraph();
    for (hipEvent_t e : events) (void)hipEventDestroy(e);
    for (hipEvent_t e : stopEvents) if (e) (void)hipEventDestroy(e);
    if (hFilter) (void)hipHostFree(hFilter);
    if (dSourceLists) (void)hipFree(dSourceLists);
    if (hStop) (void)hipHostFree(hStop);
    FreeAll(&poolAllocs);
    FreeAll(&sceneAllocs);
    FreeAll(&filmAllocs);
    FreeAll(&sampleAllocs);
    FreeAll(&rowAllocs);
    if (hCounters) (void)hipHostFree(hCounters);
    if (ownsStream && stream) (void)hipStreamDestroy(stream);
}

int dcrt_tracer::Create(const dcrt_tracer_config& cfg)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        SetLastError("no HIP device visible");
        return DCRT_E_NO_DEVICE;
    }
    device = cfg.device;
    if (device < 0 || device >= count) { SetLastError("invalid device ordinal"); return DCRT_E_INVALID_ARG; }
    HIPCHECK(hipSetDevice(device));
    if (cfg.stream) {
        stream = (hipStream_t)cfg.stream;
    } else {
        HIPCHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        ownsStream = true;
    }
    poolSize = cfg.path_pool_size ? cfg.path_pool_size : kDefaultPoolSize;
    // whole CONTROL workgroups of whole waves, and at least one CONTROL workgroup per
    // pixel-block shard (workgroup b claims the blocks of shard b % kShards)
    poolSize = std::max<uint32_t>(poolSize, kControlBlock * kShards);
    poolSize = (poolSize + kControlBlock - 1) / kControlBlock * kControlBlock;
    iterationsPerRender = cfg.iterations_per_render ? cfg.iterations_per_render : kDefaultIterations;
    debugRng = cfg.debug_rng != 0;
    if (const char* split = std::getenv("DCRT_SPLIT_CASTS")) mergedCasts = std::atoi(split) == 0;
    if (const char* vs = std::getenv("DCRT_VIRTUAL_START")) virtualStart = std::atoi(vs) != 0;
    if (const char* dp = std::getenv("DCRT_DRAIN_PATHS")) drainPaths = (uint32_t)std::max(0, std::atoi(dp));
    if (const char* tune = std::getenv("DCRT_TRAVERSAL_TUNE")) {
        unsigned r = 0, p = 0;
        if (std::sscanf(tune, "%u,%u", &r, &p) == 2 && r >= 1 && r <= 64 && p >= 1 && p <= 64) {
            refillLanes = r;
            parkLanes = p;
            tuneOverride = true;
        }
    }
    // pool arrays are addressed through 32-bit byte offsets (slot(): at most 16 B per slot), and
    // one parity's extension-ray records and path-state halves (ext_rec(), state_at(): 32 B at
    // position q = shard * recCap + entry) as well; this check bounds the pool at 2^26 slots,
    // the recCap check below keeps recCap * kShards * 32 B within 4 GiB
    if ((uint64_t)poolSize * 64u > (1ull << 32)) {
        SetLastError("path pool too large: at most 2^26 slots (32-bit pool offsets)");
        return DCRT_E_LIMIT;
    }
    // WavefrontPathTracer.cpp:120-264 (SoA instead of AoS)
    const size_t P = poolSize;
    CHECKED(DeviceAlloc(&pool.hit, 2 * P, &poolAllocs));   // 2 float4 per extension-queue item
    CHECKED(DeviceAlloc(&pool.pixel, P, &poolAllocs));
    CHECKED(DeviceAlloc(&pool.flags, P, &poolAllocs));
    CHECKED(DeviceAlloc(&pool.extOpacity, P, &poolAllocs));
    CHECKED(DeviceAlloc(&pool.shadowOpacity, P, &poolAllocs));
    // the extension and finish queues: one per iteration parity (extRecs / finRecs)
    static_assert(kControlBlock == 256u && kMaterialBlock == 256u, "queue capacities assume 256-slot workgroups");
    const uint32_t V = poolSize / 256u;   // virtual workgroups (256 slots / items each)
    {
        // One workgroup per virtual workgroup would make a pass over an idle or nearly empty
        // pool cost the dispatch of P / 256 workgroups (2^26 slots: 262144 workgroups,
        // CONTROL 91 us and MATERIAL 57 us with nothing to do). The grids hold what is
        // resident instead, a multiple of kShards (= kFinShards), so a workgroup's virtual
        // workgroups all belong to its own shard: vb mod kShards = blockIdx.x mod kShards.
        // DCRT_CONTROL_GRID / DCRT_MATERIAL_GRID = k: k x resident; 0: one workgroup per virtual
        // workgroup (A/B overrides).
        hipDeviceProp_t prop;
        HIPCHECK(hipGetDeviceProperties(&prop, device));
        if (prop.maxSharedMemoryPerMultiProcessor > 0) g_ldsPerCU = prop.maxSharedMemoryPerMultiProcessor;
        int cPerCU = 0, mPerCU = 0;
        HIPCHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&cPerCU, control_kernel, (int)kControlBlock, 0));
        HIPCHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&mPerCU, material_kernel<kCapAll, 0>, (int)kMaterialBlock, 0));
        auto resident = [&](int perCU, const char* knob, uint32_t mul) {
            if (const char* g = std::getenv(knob)) mul = (uint32_t)std::max(0, std::atoi(g));
            if (mul == 0) return V;
            const uint64_t r = (uint64_t)std::max(1, perCU) * (uint64_t)std::max(1, prop.multiProcessorCount) * mul;
            const uint32_t g = (uint32_t)std::max<uint64_t>(kShards, r / kShards * kShards);
            return std::min(g, V);   // (= V: one round, any V)
        };
        // 2x / 4x resident (two A/B passes of the default bench on cornell / spaceship / coffee,
        // ms/spp: one workgroup per virtual workgroup 2.40 / 2.84 / 2.96; 1x / 1x 2.28-2.38 /
        // 2.63 / 3.02; 1x / 4x 2.37 / 2.58 / 2.95; 2x / 4x 2.35-2.38 / 2.54 / 2.92; 4x / 4x
        // 2.37 / 2.55 / 2.95; 2x / 8x 2.37-2.39 / 2.55 / 2.92)
        controlGrid = resident(cPerCU, "DCRT_CONTROL_GRID", 2);
        materialGrid = resident(mPerCU, "DCRT_MATERIAL_GRID", 4);
        static_assert(kFinShards == kShards, "MATERIAL's grid is a multiple of both shard counts");
    }
    // The extension queue's shard s receives the new paths of CONTROL's virtual workgroups
    // vb = s mod kShards and the continuing paths of MATERIAL's (at most 256 each): at most
    // 2 ceil(V / kShards) 256 entries
    pool.recCap = std::min<uint32_t>(poolSize, 2u * ((V + kShards - 1) / kShards) * 256u);
    // (32-bit byte offsets address one parity's records: at most 2^32 bytes, e.g. 2^26 slots)
    if ((uint64_t)pool.recCap * kShards * 32u > (1ull << 32)) { SetLastError("path pool too large for the extension-queue records"); return DCRT_E_LIMIT; }
    CHECKED(DeviceAlloc(&extRecs, (size_t)pool.recCap * kShards * 2 * 2, &poolAllocs));
    // the paths' state records and their shadow rays' results, at the same positions
    CHECKED(DeviceAlloc(&stateRecsA, (size_t)pool.recCap * kShards * 2, &poolAllocs));
    CHECKED(DeviceAlloc(&stateRecsB, (size_t)pool.recCap * kShards * 2, &poolAllocs));
    CHECKED(DeviceAlloc(&shadowHits, (size_t)pool.recCap * kShards * 2, &poolAllocs));
    // the shadow queue (filled and cast within one iteration): records + path slots
    CHECKED(DeviceAlloc(&pool.shRec, (size_t)pool.recCap * kShards * 2, &poolAllocs));
    CHECKED(DeviceAlloc(&pool.shadowQueue, (size_t)pool.recCap * kShards, &poolAllocs));

    // MATERIAL's virtual workgroup vb appends the paths it ends with a shadow ray pending to
    // finish shard vb mod kFinShards
    pool.finCap = ((V + kFinShards - 1) / kFinShards) * kMaterialBlock;
    CHECKED(DeviceAlloc(&finRecs, (size_t)pool.finCap * kFinShards * 2, &poolAllocs));
    CHECKED(DeviceAlloc(&finHits, (size_t)pool.finCap * kFinShards * 2, &poolAllocs));
    pool.size = poolSize;
    CHECKED(DeviceAlloc(&dFrame, 1, &poolAllocs));
    CHECKED(DeviceAlloc(&dSampleOut, 1, &poolAllocs));
    CHECKED(DeviceAlloc(&dCounters, 2, &poolAllocs));
    CHECKED(DeviceAlloc(&dGlobals, 1, &poolAllocs));
    CHECKED(DeviceAlloc(&dInstr, 8, &poolAllocs));
    CHECKED(DeviceAlloc(&dLuts, 1, &poolAllocs));
    HIPCHECK(hipMemsetAsync(dCounters, 0, 2 * sizeof(Counters), stream));
    HIPCHECK(hipMemsetAsync(dGlobals, 0, sizeof(Globals), stream));
    HIPCHECK(hipMemsetAsync(dInstr, 0, 8 * sizeof(unsigned long long), stream));
    HIPCHECK(hipHostMalloc((void**)&hCounters, 2 * sizeof(Counters), hipHostMallocDefault));
    CHECKED(DeviceAlloc(&dFilter, 1, &poolAllocs));
    HIPCHECK(hipHostMalloc((void**)&hFilter, sizeof(FilterConsts), hipHostMallocDefault));
    HIPCHECK(hipHostMalloc((void**)&hStop, 8 * sizeof(uint32_t), hipHostMallocDefault));
    for (hipEvent_t& e : stopEvents) HIPCHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CHECKED(BuildLuts());
    HIPCHECK(hipStreamSynchronize(stream));
    return DCRT_OK;
}

// BxDFTexturesBuilding::Build (BxDFTexturesBuilding.cpp:106-475) as three
// integration launches + one conversion/average launch.
// The LUTs depend on nothing but the integration constants, so a process integrates
// them once per device (≈ 0.24 s of GPU time) and every further tracer copies them
// (the cache's device copies live until the process exits).
static std::mutex g_lutMutex;
static std::map<int, dcrt_bxdf_luts*> g_lutCache;

int dcrt_tracer::BuildLuts()
{
    std::lock_guard<std::mutex> lock(g_lutMutex);
    auto hit = g_lutCache.find(device);
    if (hit != g_lutCache.end()) {
        HIPCHECK(hipMemcpyAsync(dLuts, hit->second, sizeof(dcrt_bxdf_luts), hipMemcpyDeviceToDevice, stream));
        HIPCHECK(hipStreamSynchronize(stream));
        return DCRT_OK;
    }
    std::vector<void*> tmp;
    float *brdf = nullptr, *brdfd = nullptr, *bsdf = nullptr;
    CHECKED(DeviceAlloc(&brdf, DCRT_LUT_BRDF_COUNT, &tmp));
    CHECKED(DeviceAlloc(&brdfd, DCRT_LUT_BRDF_DIELECTRIC_COUNT, &tmp));
    CHECKED(DeviceAlloc(&bsdf, DCRT_LUT_BSDF_COUNT, &tmp));
    hipLaunchKernelGGL(lut_integrate_kernel, dim3((DCRT_LUT_BRDF_COUNT + 63) / 64), dim3(64), 0, stream, 0, (uint32_t)DCRT_LUT_BRDF_COUNT, brdf);
    hipLaunchKernelGGL(lut_integrate_kernel, dim3((DCRT_LUT_BRDF_DIELECTRIC_COUNT + 63) / 64), dim3(64), 0, stream, 1,
                       (uint32_t)DCRT_LUT_BRDF_DIELECTRIC_COUNT, brdfd);
    hipLaunchKernelGGL(lut_integrate_kernel, dim3((DCRT_LUT_BSDF_COUNT + 63) / 64), dim3(64), 0, stream, 2, (uint32_t)DCRT_LUT_BSDF_COUNT, bsdf);
    hipLaunchKernelGGL(lut_finalize_kernel, dim3((DCRT_LUT_BRDF_DIELECTRIC_COUNT + 255) / 256), dim3(256), 0, stream, brdf, brdfd, bsdf, dLuts);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(stream));
    FreeAll(&tmp);
    dcrt_bxdf_luts* cached = nullptr;
    if (hipMalloc((void**)&cached, sizeof(dcrt_bxdf_luts)) == hipSuccess) {
        if (hipMemcpy(cached, dLuts, sizeof(dcrt_bxdf_luts), hipMemcpyDeviceToDevice) == hipSuccess) g_lutCache[device] = cached;
        else (void)hipFree(cached);
    }
    return DCRT_OK;
}

int dcrt_tracer::UploadScene(const dcrt_flat_scene& s)
{
    Annotation an("UploadScene");
    if (!s.vertices || !s.triangles || !s.bvh_nodes || !s.material_ids || !s.instance_transforms || !s.materials ||
        !s.instance_light_indices || !s.instance_flags || !s.instance_material_overrides || s.triangle_count == 0 ||
        s.bvh_node_count == 0 || s.instance_count == 0 || s.material_count == 0) {
        SetLastError("incomplete flat scene");
        return DCRT_E_INVALID_ARG;
    }
    if (s.light_count > DCRT_MAX_LIGHT_COUNT) { SetLastError("more than 5000 lights"); return DCRT_E_LIMIT; }
    HIPCHECK(hipStreamSynchronize(stream));
    InvalidateGraph();
    FreeAll(&sceneAllocs);
    hasScene = false;
    DeviceScene d{};
    auto upload = [&](auto** dst, const auto* src, size_t count) -> int {
        using T = std::remove_const_t<std::remove_pointer_t<decltype(src)>>;
        T* p = nullptr;
        CHECKED(DeviceAlloc(&p, count, &sceneAllocs));
        if (count && src) HIPCHECK(hipMemcpyAsync(p, src, count * sizeof(T), hipMemcpyHostToDevice, stream));
        *dst = p;
        return DCRT_OK;
    };
    dcrt_vertex* vtx = nullptr;
    uint32_t* tris = nullptr;
    dcrt_bvh_node* nodes = nullptr;
    dcrt_float4x3* xf = nullptr;
    CHECKED(upload(&vtx, s.vertices, s.vertex_count));
    CHECKED(upload(&tris, s.triangles, (size_t)s.triangle_count * 3));
    // the traversal pushes without a bound check: refuse a stack size below what the
    // uploaded tree needs (TLAS leaf depth + BLAS depth, Scene.cpp:199-207); the walk also
    // checks every node reference
    uint32_t stackNeed = 0;
    if (!RequiredTraversalStack(s, &stackNeed)) { SetLastError("malformed BVH node references"); return DCRT_E_INVALID_ARG; }
    if (s.bvh_traversal_stack_size < stackNeed) {
        SetLastError("bvh_traversal_stack_size " + std::to_string(s.bvh_traversal_stack_size) +
                     " is below the uploaded BVH's depth " + std::to_string(stackNeed));
        return DCRT_E_INVALID_ARG;
    }
    uint32_t* mids = nullptr; uint32_t* lidx = nullptr; uint32_t* iflags = nullptr; uint32_t* ovr = nullptr;
    dcrt_material* mats = nullptr; dcrt_light* lights = nullptr;
    CHECKED(upload(&mids, s.material_ids, s.triangle_count));
    CHECKED(upload(&xf, s.instance_transforms, (size_t)s.instance_count * 2));
    CHECKED(upload(&lidx, s.instance_light_indices, s.instance_count));
    CHECKED(upload(&iflags, s.instance_flags, s.instance_count));
    CHECKED(upload(&ovr, s.instance_material_overrides, s.instance_count));
    // instances whose world->instance matrix is exactly the identity (every OBJ shape):
    // traversal then reuses the world ray instead of transforming it (bit-identical
    // when no ray component is zero, which the kernel checks per ray)
    std::vector<uint32_t> identity(s.instance_count, 0u);
    for (uint32_t i = 0; i < s.instance_count; ++i) {
        const float* m = s.instance_transforms[s.instance_count + i].m;
        bool id = true;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 4; ++c) id = id && m[r * 4 + c] == (r == c ? 1.0f : 0.0f);
        identity[i] = id ? 1u : 0u;
    }
    uint32_t* ident = nullptr;
    CHECKED(upload(&ident, identity.data(), s.instance_count));
    CHECKED(upload(&mats, s.materials, s.material_count));
    CHECKED(upload(&lights, s.lights, std::max<uint32_t>(s.light_count, 1)));
    float4* triVerts = nullptr;
    float4* triShade = nullptr;
    CHECKED(DeviceAlloc(&triVerts, (size_t)s.triangle_count * 3, &sceneAllocs));
    CHECKED(DeviceAlloc(&triShade, (size_t)s.triangle_count * 6, &sceneAllocs));
    if (s.triangle_count)
        hipLaunchKernelGGL(build_tri_verts_kernel, dim3((s.triangle_count + 255) / 256), dim3(256), 0, stream, vtx, tris, mids,
                           s.triangle_count, triVerts, triShade);
    HIPCHECK(hipGetLastError());
    // textures: one texel blob + descriptors (Scene.cpp:586-608)
    std::vector<TextureDesc> descs(std::max<uint32_t>(s.texture_count, 1));
    std::vector<uint8_t> blob;
    for (uint32_t i = 0; i < s.texture_count; ++i) {
        const dcrt_texture& t = s.textures[i];
        TextureDesc& td = descs[i];
        const size_t bpp = t.format == DCRT_TEXTURE_FORMAT_R8_UNORM ? 1 : 4;
        td.width = t.pixels ? t.width : 0; td.height = t.pixels ? t.height : 0; td.format = t.format;
        td.offset = (uint32_t)blob.size();
        if (t.pixels) blob.insert(blob.end(), t.pixels, t.pixels + (size_t)t.width * t.height * bpp);
        while (blob.size() % 4) blob.push_back(0);
    }
    if (blob.empty()) blob.resize(4, 0);
    TextureDesc* dDescs = nullptr; uint8_t* dBlob = nullptr; float* dSrgb = nullptr;
    CHECKED(upload(&dDescs, descs.data(), descs.size()));
    CHECKED(upload(&dBlob, blob.data(), blob.size()));
    float srgb[256];
    for (int i = 0; i < 256; ++i) {
        const double c = i / 255.0;
        srgb[i] = (float)(c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4));
    }
    CHECKED(upload(&dSrgb, srgb, 256));
    float* dEnv = nullptr;
    if (s.env_cube_rgb && s.env_cube_size) CHECKED(upload(&dEnv, s.env_cube_rgb, (size_t)6 * s.env_cube_size * s.env_cube_size * 3));
    d.triVerts = triVerts;
    d.triShade = triShade;
    d.vertices = vtx;
    d.triangles = tris;
    d.materialIds = mids;
    d.transforms = (const float4*)xf;
    d.instanceLightIndices = lidx;
    d.instanceFlags = iflags;
    d.instanceIdentity = ident;
    d.overrides = ovr;
    d.materials = mats;
    d.lights = lights;
    d.textures = dDescs;
    d.texels = dBlob;
    d.srgbTable = dSrgb;
    d.envCube = dEnv;
    d.envCubeSize = dEnv ? s.env_cube_size : 0;
    d.lutBrdf = dLuts->brdf;
    d.lutBrdfAvg = dLuts->brdf_avg;
    d.lutBrdfDielectric = dLuts->brdf_dielectric;
    d.lutBrdfDielectricAvg = dLuts->brdf_dielectric_avg;
    d.lutBsdf = dLuts->bsdf;
    d.lutBsdfAvg = dLuts->bsdf_avg;
    d.instanceCount = s.instance_count;
    d.triangleCount = s.triangle_count;
    d.stackSize = std::max<uint32_t>(s.bvh_traversal_stack_size, 1u);
    // BLAS leaves (no TLAS-leaf bit, a primitive count) all with one triangle
    d.singlePrimLeaves = 1u;
    for (uint32_t i = 0; i < s.bvh_node_count; ++i) {
        const uint32_t misc = s.bvh_nodes[i].misc;
        if (!(misc & 0x4u) && ((misc >> 3) & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT) > 1u) { d.singlePrimLeaves = 0u; break; }
    }
    scene = d;
    // MATERIAL variant: the smallest compiled one whose capabilities cover the scene
    sceneCaps = dEnv ? kCapEnvCube : 0u;
    for (uint32_t i = 0; i < s.material_count; ++i) {
        const dcrt_material& m = s.materials[i];
        const uint32_t type = m.flags & DCRT_MATERIAL_FLAG_TYPE_MASK;
        sceneCaps |= type <= DCRT_MATERIAL_TYPE_THIN_DIELECTRIC ? (1u << type) : kCapAll;
        if (m.flags & DCRT_MATERIAL_FLAG_MULTISCATTERING) sceneCaps |= kCapMultiscatter;
        if (m.albedo_texture_index != -1 || (m.flags & DCRT_MATERIAL_FLAG_ROUGHNESS_TEXTURE)) sceneCaps |= kCapTextures;
    }
    for (uint32_t i = 0; i < s.light_count; ++i) sceneCaps |= (s.lights[i].flags & 0xFu) << kCapLightShift;
    materialCaps = (sceneCaps & ~kCapOpaqueDelta) == 0u ? kCapOpaqueDelta : kCapAll;
    // MATERIAL's LDS scene copy (material_kernel<CAPS, mode>): the whole shading data of a small
    // scene (mode 1), else everything but the triangles (mode 2) -- DCRT_MATERIAL_LDS = bytes
    // budget, 0: off; DCRT_MATERIAL_LDS_PARTIAL=0: no mode 2
    {
        uint32_t budget = 16384;
        if (const char* e = std::getenv("DCRT_MATERIAL_LDS")) budget = (uint32_t)std::max(0, std::atoi(e));
        bool partial = true;
        if (const char* e = std::getenv("DCRT_MATERIAL_LDS_PARTIAL")) partial = std::atoi(e) != 0;
        const bool counts = s.triangle_count > 0 && s.triangle_count < (1u << 20) && s.instance_count < (1u << 20) &&
                            s.material_count < (1u << 20) && s.light_count < (1u << 20);
        const uint64_t whole = material_lds_bytes(s.triangle_count, s.instance_count, s.material_count, s.light_count);
        const uint64_t rest = material_lds_bytes(0u, s.instance_count, s.material_count, s.light_count);
        materialLdsMode = !counts ? 0u : whole <= budget ? 1u : (partial && rest <= budget ? 2u : 0u);
        materialLds = materialLdsMode == 1 ? (uint32_t)whole : materialLdsMode == 2 ? (uint32_t)rest : 0u;
        d.ldsMaterials = materialLdsMode ? s.material_count : 0u;
        d.ldsLights = materialLdsMode ? s.light_count : 0u;
        scene = d;
    }
    if (const char* g = std::getenv("DCRT_MATERIAL_GENERIC")) {   // A/B: always the generic variant
        if (std::atoi(g)) materialCaps = kCapAll;
    }
    // LDS stack: [stackSize + 2][block] u32 (two spare rows per lane, see stack_at in
    // dscene.h); keep a workgroup's stack <= 32 KiB
    castBlock = 256;
    while (castBlock > 64 && (size_t)(d.stackSize + 2) * castBlock * 4 > 32768) castBlock >>= 1;
    if (const char* e = std::getenv("DCRT_CAST_BLOCK")) {   // (A/B: 64 / 128 / 256, at most the default)
        const uint32_t v = (uint32_t)std::atoi(e);
        if ((v == 64 || v == 128 || v == 256) && v <= castBlock) castBlock = v;
    }
    d.stackRows = d.stackSize + 2u;
    d.ringRows = 0u;
    d.spill = nullptr;
    ringRows = 0;
    castLds = (size_t)(d.stackSize + 2) * castBlock * 4;
    if (castLds > 65536) { SetLastError("BVH traversal stack too deep for LDS"); return DCRT_E_LIMIT; }
    // resident workgroups per CU of a cast kernel with `lds` bytes of dynamic LDS: registers and
    // LDS (gfx950's 1280-B allocation granule, LdsResident)
    auto castOccupancy = [&](CastFn k, size_t lds, int* out) -> int {
        int n = 0;
        if (mergedCasts) HIPCHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, (int)castBlock, lds));
        else HIPCHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, extension_kernel<false, false>, (int)castBlock, lds));
        *out = std::min(n, LdsResident(lds, mergedCasts ? (const void*)k : (const void*)extension_kernel<false, false>));
        return DCRT_OK;
    };
    {
        // LDS scene cache in what the cast kernel's register-limited occupancy leaves of the
        // CU's 160 KiB per workgroup: BVH nodes first, then pre-gathered triangles
        int regPerCU = 0;
        CHECKED(castOccupancy(cast_kernel<false, false, false, false>, castLds, &regPerCU));
        const size_t perBlock = (g_ldsPerCU / (size_t)std::max(1, regPerCU)) & ~(size_t)15;
        size_t budget = castLds < perBlock ? perBlock - castLds : 0;
        uint32_t nodeCount = s.bvh_node_count;
        d.cachedNodes = (uint32_t)std::min<size_t>(nodeCount, budget / 32);
        d.cachedTris = (uint32_t)std::min<size_t>(s.triangle_count, (budget - d.cachedNodes * 32) / 48);
        bool noCache = false;
        if (const char* off = std::getenv("DCRT_NO_LDS_CACHE")) noCache = std::atoi(off) != 0;   // A/B experiments, tests
        if (noCache) d.cachedNodes = d.cachedTris = 0;
        // (the LDS-only variant assumes 256-thread workgroups: its stack stride is a constant)
        // (the cache-only variant keeps three permuted copies of every triangle: 144 B each)
        castAllCached = castBlock == 256 && d.cachedNodes == nodeCount && d.cachedTris == s.triangle_count &&
                        (size_t)d.cachedNodes * 32 + (size_t)s.triangle_count * 144 + (size_t)s.instance_count * 64 <= budget;
        d.cachedInstances = castAllCached ? s.instance_count : 0u;
        // trav_visit_pair where the traversal's fetches miss L2: nodes + triangles beyond an
        // XCD's 4 MiB L2 (DCRT_PAIR_TRAVERSAL=0/1 forces it off / on, A/B and tests)
        castPair = !castAllCached && (size_t)nodeCount * 32 + (size_t)s.triangle_count * 48 > ((size_t)4 << 20);
        if (const char* pv = std::getenv("DCRT_PAIR_TRAVERSAL")) castPair = !castAllCached && std::atoi(pv) != 0;
        // the node order goes with it (dscene.h kLayoutPairs: the pair kernels assume it, the
        // other non-counting cast kernels assume PackBVH's)
        std::vector<dcrt_bvh_node> pairNodes;
        if (castPair) {
            uint32_t topNodes = 4096;
            if (const char* e = std::getenv("DCRT_TOP_NODES")) topNodes = (uint32_t)std::atoi(e);   // A/B experiments
            // quads (profiles/r06_ab_log.md: spaceship -1.6 %, close framing -0.1 / -1.4 %)
            bool quads = true;
            if (const char* e = std::getenv("DCRT_NODE_QUADS")) quads = std::atoi(e) != 0;   // A/B experiments
            if (!PairLayout(s, topNodes, &pairNodes, quads)) { SetLastError("malformed BVH: a node with two parents"); return DCRT_E_INVALID_ARG; }
            nodeCount = (uint32_t)pairNodes.size();
        }
        std::vector<dcrt_bvh_node> devNodes = castPair ? std::move(pairNodes) : std::vector<dcrt_bvh_node>(s.bvh_nodes, s.bvh_nodes + nodeCount);
        // every instance the identity: the cache-only kernel keeps no instance space (IDENT;
        // DCRT_IDENT_CAST=0: off, A/B)
        // (bitwise: +1 and +0 entries only -- with a -0 entry the transform of a -0 component could
        // stay -0, where IDENT's o + 0 gives +0)
        castIdent = (castAllCached || !castPair) && mergedCasts && s.instance_count > 0;
        for (uint32_t i = 0; castIdent && i < s.instance_count; ++i) {
            const float* m = s.instance_transforms[s.instance_count + i].m;
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 4; ++c) {
                    uint32_t bits;
                    std::memcpy(&bits, &m[r * 4 + c], 4);
                    castIdent = castIdent && bits == (r == c ? 0x3F800000u : 0u);
                }
        }
        if (const char* e = std::getenv("DCRT_IDENT_CAST")) castIdent = castIdent && std::atoi(e) != 0;
        // The spilling stack (cast_kernel<..., RING>: an LDS window of K rows over a per-lane global
        // column, kernels_impl.h ring_maintain) where the whole stack costs the launched kernel
        // resident workgroups: a deep BVH (spaceship: 30 entries = 32 KiB per 256-lane workgroup,
        // 4 workgroups per CU where its registers allow 6). DCRT_STACK_RING = K (a power of two,
        // 8..64) forces a window of K rows (tests: K below the scene's depth spills), 0: never.
        if (!castAllCached && mergedCasts) {
            int forced = -1;
            if (const char* e = std::getenv("DCRT_STACK_RING")) forced = std::atoi(e);
            const uint32_t K = forced > 0 ? (uint32_t)forced : 16u;
            // (the window must take a batch of kVisitsPerCheck visits after a refill to half: kMinRingRows)
            const bool validK = K >= std::max(8u, kMinRingRows) && K <= 64u && (K & (K - 1u)) == 0u;
            if (forced > 0 && !validK) {
                SetLastError("DCRT_STACK_RING: a power of two in [max(8, 2 * (visits per check + 1)), 64]");
                return DCRT_E_INVALID_ARG;
            }
            if (forced > 0) {
                ringRows = K;
            } else if (forced < 0 && validK && K < d.stackSize + 2u) {
                int whole = 0, ring = 0;
                CHECKED(castOccupancy(CastKernel(false, false, false, castPair, castIdent, false), castLds, &whole));
                CHECKED(castOccupancy(CastKernel(false, false, false, castPair, castIdent, true), (size_t)K * castBlock * 4, &ring));
                if (ring > whole) ringRows = K;
            }
        }
        // A scene the cache does not hold whole: the cache leaves `reserve` bytes of each CU's LDS
        // free, so workgroups of the other pipeline's kernels (MATERIAL, CONTROL) can be resident
        // beside the cast's -- with the cache sized to the last byte they could not
        // (DCRT_CAST_LDS_RESERVE, bytes per CU)
#ifndef DCRT_CAST_LDS_RESERVE
#define DCRT_CAST_LDS_RESERVE 12288   // (A/B: coffee -2 to -3 %, lamp -1 %; profiles/r04_ab_round4.txt)
#endif
        size_t reserve = DCRT_CAST_LDS_RESERVE;
        if (const char* e = std::getenv("DCRT_CAST_LDS_RESERVE")) reserve = (size_t)std::max(0, std::atoi(e));
        reserve = std::min<size_t>(reserve, g_ldsPerCU);
        const CastFn launched = CastKernel(false, false, castAllCached, castPair, castIdent, ringRows != 0);
        // the launched kernel's stack bytes: the ring window, or the whole stack
        const size_t stackLds = ringRows ? (size_t)ringRows * castBlock * 4 : castLds;
        if (!castAllCached) {
            // the cache budget from the occupancy of the kernel that launches
            int perCU = 0;
            CHECKED(castOccupancy(launched, stackLds, &perCU));
            const size_t perBlockR = ((g_ldsPerCU - reserve) / (size_t)std::max(1, perCU)) & ~(size_t)15;
            budget = stackLds < perBlockR ? perBlockR - stackLds : 0;
            d.cachedNodes = (uint32_t)std::min<size_t>(nodeCount, budget / 32);
            d.cachedTris = (uint32_t)std::min<size_t>(s.triangle_count, (budget - d.cachedNodes * 32) / 48);
            if (noCache) d.cachedNodes = d.cachedTris = 0;
        }
        // the cache-only kernels enter identity instances' BLASes in phase A (dscene.h
        // kMiscIdentityLeaf): TLAS leaves carry the flag in their otherwise unused axis bits
        if (castAllCached || castIdent) {
            for (dcrt_bvh_node& n : devNodes) {
                if (!(n.misc & 0x4u)) continue;
                const uint32_t inst = (n.misc >> 3) & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT;
                n.misc = (n.misc & ~0x3u) | (inst < s.instance_count && identity[inst] ? kMiscIdentityLeaf : 0u);
            }
        }
        CHECKED(upload(&nodes, devNodes.data(), nodeCount));
        HIPCHECK(hipStreamSynchronize(stream));   // (devNodes ends with this block)
        d.nodes = (const float4*)nodes;
        d.nodeCount = nodeCount;
        d.pairLayout = castPair ? 1u : 0u;
        // trav_skip_root: levels of sure hits taken at a ray's start without their box tests
        d.skipRoot = 1u;
        if (const char* e = std::getenv("DCRT_SKIP_ROOT")) d.skipRoot = (uint32_t)std::max(0, std::min(16, std::atoi(e)));   // (A/B, tests)
        const size_t cacheBytes = [&] { return (size_t)d.cachedNodes * 32 + (size_t)d.cachedTris * (castAllCached ? 144 : 48) + (size_t)d.cachedInstances * 64; }();
        size_t launchLds = stackLds + cacheBytes;
        // The budget above divides 160 KiB evenly among the workgroups the registers allow; the
        // LDS is allocated in granules (and the kernel's static LDS comes on top), so the cache
        // could cost a workgroup per CU (the spaceship pair kernel ran 5 of its 6). Trim the
        // cache -- triangles first, then nodes, a granule at a time -- until the launched kernel
        // keeps the occupancy the stack alone allows.
        bool trim = true;
        if (const char* e = std::getenv("DCRT_LDS_TRIM")) trim = std::atoi(e) != 0;   // (A/B)
        if (!castAllCached && trim) {
            int target = 0, now = 0;
            CHECKED(castOccupancy(launched, stackLds, &target));
            for (;;) {
                CHECKED(castOccupancy(launched, launchLds, &now));
                if (now >= target || (d.cachedTris == 0 && d.cachedNodes == 0)) break;
                if (d.cachedTris > 0) d.cachedTris -= std::min<uint32_t>(d.cachedTris, 11);   // 528 B
                else d.cachedNodes -= std::min<uint32_t>(d.cachedNodes, 16);                  // 512 B
                launchLds = stackLds + (size_t)d.cachedNodes * 32 + (size_t)d.cachedTris * 48;
            }
        }
        scene = d;
        // every kernel but the ring cast launches with the whole stack (stackSize + 2 rows) in
        // front of the same cache
        castLdsFull = castLds + (launchLds - stackLds);
        castLds = launchLds;
        // The entry-free node order for the cache-only IDENT kernel (EntryFreeLayout: no BLAS-entry
        // step per node visit), where its nodes, the triangles and one more stack row still fit
        // the LDS the IDENT kernel runs at (DCRT_FLAT_CAST=0: off, A/B and tests)
        castFlat = false;
        bool flatWanted = true;
        if (const char* e = std::getenv("DCRT_FLAT_CAST")) flatWanted = std::atoi(e) != 0;
        if (flatWanted && castAllCached && castIdent && mergedCasts && d.singlePrimLeaves) {
            std::vector<dcrt_bvh_node> flat;
            bool merge = true;   // (DCRT_FLAT_MERGE=0: every TLAS leaf over an empty node -- tests)
            if (const char* e = std::getenv("DCRT_FLAT_MERGE")) merge = std::atoi(e) != 0;
            if (EntryFreeLayout(s, &flat, merge)) {
                const size_t flatLds = (size_t)(d.stackSize + 3u) * castBlock * 4 + flat.size() * 32 + (size_t)s.triangle_count * 144;
                int identPerCU = 0, flatPerCU = 0;
                CHECKED(castOccupancy(CastKernel(false, false, true, false, true, false), castLds, &identPerCU));
                CHECKED(castOccupancy(CastKernel(false, false, true, false, true, false, true), flatLds, &flatPerCU));
                if (flatPerCU >= identPerCU && flatLds <= 65536) {
                    dcrt_bvh_node* fn = nullptr;
                    CHECKED(upload(&fn, flat.data(), flat.size()));
                    HIPCHECK(hipStreamSynchronize(stream));   // (flat ends with this block)
                    sceneFlat = scene;
                    sceneFlat.nodes = (const float4*)fn;
                    sceneFlat.nodeCount = (uint32_t)flat.size();
                    sceneFlat.cachedNodes = (uint32_t)flat.size();
                    sceneFlat.cachedInstances = 0u;
                    sceneFlat.stackSize = d.stackSize + 1u;
                    sceneFlat.stackRows = d.stackSize + 3u;
                    castLdsFlat = flatLds;
                    castFlat = true;
                }
            }
        }
    }
    {
        // The persistent traversal kernels run exactly one resident wave of workgroups.
        hipDeviceProp_t prop;
        HIPCHECK(hipGetDeviceProperties(&prop, device));
        int perCU = 0;
        if (castFlat) CHECKED(castOccupancy(CastKernel(false, false, true, false, true, false, true), castLdsFlat, &perCU));
        else CHECKED(castOccupancy(CastKernel(false, false, castAllCached, castPair, castIdent, ringRows != 0), castLds, &perCU));
        if (const char* b = std::getenv("DCRT_CAST_BLOCKS_PER_CU")) {   // tuning experiments
            const int v = std::atoi(b);
            if (v >= 1 && v < perCU) perCU = v;
        }
        castPerCU = (uint32_t)std::max(1, perCU);
        castResident = castPerCU * (uint32_t)std::max(1, prop.multiProcessorCount);
        if (const char* m = std::getenv("DCRT_CAST_GRID_MUL")) {   // (A/B: k x resident, workgroups retire in k rounds)
            const int k = std::atoi(m);
            if (k >= 2 && k <= 16) castResident *= (uint32_t)k;
        }
        int opacityPerCU = 0;
        CHECKED(castOccupancy(CastKernel(false, true, castAllCached, castPair), castLdsFull, &opacityPerCU));
        castResidentOpacity = (uint32_t)std::max(1, std::min(opacityPerCU, perCU)) * (uint32_t)std::max(1, prop.multiProcessorCount);
        // the counting kernels keep the whole stack (castLdsFull): their own resident grid, so an
        // instrumented run has no second partial round of workgroups the shipped kernel lacks
        int instrPerCU = 0, instrOpacityPerCU = 0;
        CHECKED(castOccupancy(CastKernel(true, false, castAllCached, castPair, castIdent, false), castLdsFull, &instrPerCU));
        CHECKED(castOccupancy(CastKernel(true, true, castAllCached, castPair), castLdsFull, &instrOpacityPerCU));
        castResidentInstr = (uint32_t)std::max(1, std::min(instrPerCU, perCU)) * (uint32_t)std::max(1, prop.multiProcessorCount);
        castResidentInstrOpacity = (uint32_t)std::max(1, std::min(instrOpacityPerCU, perCU)) * (uint32_t)std::max(1, prop.multiProcessorCount);
        int megaPerCU = 0;
        HIPCHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&megaPerCU, megakernel<false>, (int)castBlock, castLdsFull));
        megaResident = (uint32_t)std::max(1, std::min(megaPerCU, LdsResident(castLdsFull, (const void*)megakernel<false>))) *
                       (uint32_t)std::max(1, prop.multiProcessorCount);
        int drainPerCU = 0;
        HIPCHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&drainPerCU, materialCaps == kCapOpaqueDelta ? drain_kernel<kCapOpaqueDelta> : drain_kernel<kCapAll>,
                                                              (int)castBlock, castLdsFull));
        drainResident = (uint32_t)std::max(1, std::min(drainPerCU, LdsResident(castLdsFull, materialCaps == kCapOpaqueDelta
                                                                                                 ? (const void*)drain_kernel<kCapOpaqueDelta>
                                                                                                 : (const void*)drain_kernel<kCapAll>))) *
                        (uint32_t)std::max(1, prop.multiProcessorCount);
        if (ringRows) {
            // the spill columns: stackSize entries per lane of the persistent ring grid
            uint32_t* spill = nullptr;
            CHECKED(DeviceAlloc(&spill, (size_t)castResident * castBlock * scene.stackSize, &sceneAllocs));
            HIPCHECK(hipMemsetAsync(spill, 0, (size_t)castResident * castBlock * scene.stackSize * 4, stream));
            sceneRing = scene;
            sceneRing.stackRows = ringRows;
            sceneRing.ringRows = ringRows;
            sceneRing.spill = spill;
        }
    }
    HIPCHECK(hipStreamSynchronize(stream));
    hasScene = true;
    newImage = true;
    return DCRT_OK;
}

int dcrt_tracer::EnsureFilm(uint32_t w, uint32_t h)
{
    if (w == filmW && h == filmH && film.accum) return DCRT_OK;
    if (w == 0 || h == 0 || w > 65535 || h > 65535) { SetLastError("invalid film resolution"); return DCRT_E_INVALID_ARG; }
    HIPCHECK(hipStreamSynchronize(stream));
    InvalidateGraph();
    FreeAll(&filmAllocs);
    FreeAll(&sampleAllocs);
    sampleImages = 0;
    const size_t n = (size_t)w * h;
    CHECKED(DeviceAlloc(&film.accum, n, &filmAllocs));
    HIPCHECK(hipMemsetAsync(film.accum, 0, n * sizeof(float4), stream));
    filmW = w; filmH = h;
    film.width = w; film.height = h;
    CHECKED(EnsureSamples(1));
    return BuildRows();
}

// Sample textures for `images` images (a RenderImages batch); grows only.
int dcrt_tracer::EnsureSamples(uint32_t images)
{
    if (images <= sampleImages) return DCRT_OK;
    HIPCHECK(hipStreamSynchronize(stream));
    InvalidateGraph();
    FreeAll(&sampleAllocs);
    const size_t n = (size_t)filmW * filmH * images;
    CHECKED(DeviceAlloc(&film.samplePosition, n, &sampleAllocs));
    CHECKED(DeviceAlloc(&film.sampleValue, n, &sampleAllocs));
    film.debugRng = nullptr;
    if (debugRng) CHECKED(DeviceAlloc(&film.debugRng, n, &sampleAllocs));
    HIPCHECK(hipMemsetAsync(film.samplePosition, 0, n * sizeof(float2), stream));
    HIPCHECK(hipMemsetAsync(film.sampleValue, 0, n * sizeof(float4), stream));
    if (film.debugRng) HIPCHECK(hipMemsetAsync(film.debugRng, 0, n * sizeof(uint4), stream));
    hSampleOut = SampleOut{film.samplePosition, film.sampleValue, film.debugRng, rowProbe ? dRowRays : nullptr};
    HIPCHECK(hipMemcpyAsync(dSampleOut, &hSampleOut, sizeof(SampleOut), hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    sampleImages = images;
    return DCRT_OK;
}

// Images per RenderImages batch: as many as the path pool holds at once, so that a rank
// of a partitioned film (a fraction of every image) still runs full wavefronts. A batch
// that overflows the pool by a little is avoided: its last pixel blocks would start only
// when the first paths end and stretch the batch by a whole path length. Every batch ends
// in a drain (iterations with a shrinking path population), so large pools and batches of
// many images amortise it: a rank of an N-GPU film renders 1/N of each image, and gets N
// times as many images per batch.
uint32_t dcrt_tracer::AutoBatch(uint32_t count) const
{
    uint32_t b = batchImages;
    // (sample index p = image * W*H + y * W + x stays below 2^31)
    const uint32_t cap = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kMaxImageBatchAuto(), ((uint64_t)1 << 31) / ((uint64_t)filmW * filmH)));
    if (b == 0) {
        // the slots an image takes: whole 8x8 pixel blocks (a wave each), partial bands and
        // columns included, so a batch that "fits" never waits for slots to free up
        const uint64_t pixels = std::max<uint64_t>(1, (uint64_t)bandCount * kBlockH * ((filmW + kBlockW - 1) / kBlockW) * kBlockW);
        b = (uint32_t)std::min<uint64_t>(cap, std::max<uint64_t>(1, poolSize / pixels));
        if (!BatchPoolLimit()) b = cap;
        // equal batches: as many batches as the cap needs, each as large as the others (a
        // small last batch would pay a whole drain for a sparse wavefront)
        const uint32_t batches = (count + b - 1) / b;
        b = (count + batches - 1) / batches;
    }
    return std::max<uint32_t>(1, std::min(std::min(b, cap), count));
}

// Rows this tracer renders. One tracer: every row. Partitioned film: the
// film is cut into K = N * k stripes of floor/ceil(H / K) rows, k = round(H / (N * S))
// for the target stripe height S, stripe j belongs to rank j mod N (every rank gets k
// stripes, equal row counts to one row); a rank renders its rows plus `halo` rows on
// either side of each stripe and convolves only its own rows. The rows are packed 8 per
// block row in ascending order (directcomputeraytracing_amd/partition.py mirrors this).
int dcrt_tracer::BuildRows()
{
    const uint32_t H = filmH;
    std::vector<uint32_t> rows;
    std::vector<uint32_t> owned;
    if (!bands.empty()) {
        // explicit film bands (dcrt_tracer_set_film_bands): their rows plus the halo beyond each
        const uint32_t halo = partition.halo_rows ? partition.halo_rows : 2u;
        owned.assign(H, 0);
        std::vector<uint8_t> need(H, 0);
        for (size_t i = 0; i + 1 < bands.size(); i += 2) {
            const uint32_t y0 = std::min(bands[i], H), y1 = std::min(bands[i + 1], H);
            for (uint32_t y = y0; y < y1; ++y) owned[y] = 1;
            if (y0 >= y1) continue;
            const uint32_t lo = y0 >= halo ? y0 - halo : 0, hi = std::min(H, y1 + halo);
            for (uint32_t y = lo; y < hi; ++y) need[y] = 1;
        }
        for (uint32_t y = 0; y < H; ++y) if (need[y]) rows.push_back(y);
    } else if (partition.world_size <= 1) {
        for (uint32_t y = 0; y < H; ++y) rows.push_back(y);
    } else {
        const uint32_t N = partition.world_size, halo = partition.halo_rows ? partition.halo_rows : 2u;
        const uint32_t k = std::max<uint32_t>(1, (uint32_t)((H + (N * partition.stripe_height) / 2) / (N * partition.stripe_height)));
        const uint64_t K = std::min<uint64_t>((uint64_t)N * k, H);
        owned.assign(H, 0);
        std::vector<uint8_t> need(H, 0);
        for (uint64_t j = partition.rank; j < K; j += N) {
            const uint32_t y0 = (uint32_t)(j * H / K), y1 = (uint32_t)((j + 1) * H / K);
            for (uint32_t y = y0; y < y1; ++y) owned[y] = 1;
            const uint32_t lo = y0 >= halo ? y0 - halo : 0, hi = std::min(H, y1 + halo);
            for (uint32_t y = lo; y < hi; ++y) need[y] = 1;
        }
        for (uint32_t y = 0; y < H; ++y) if (need[y]) rows.push_back(y);
    }
    if (rows.empty()) rows.push_back(0);
    HIPCHECK(hipStreamSynchronize(stream));
    FreeAll(&rowAllocs);
    rowCount = (uint32_t)rows.size();
    bandCount = (rowCount + kBlockH - 1) / kBlockH;
    uint32_t* dRows = nullptr;
    CHECKED(DeviceAlloc(&dRows, rows.size(), &rowAllocs));
    HIPCHECK(hipMemcpyAsync(dRows, rows.data(), rows.size() * 4, hipMemcpyHostToDevice, stream));
    uint32_t* dOwned = nullptr;
    if (!owned.empty()) {
        CHECKED(DeviceAlloc(&dOwned, owned.size(), &rowAllocs));
        HIPCHECK(hipMemcpyAsync(dOwned, owned.data(), owned.size() * 4, hipMemcpyHostToDevice, stream));
    }
    HIPCHECK(hipStreamSynchronize(stream));
    film.rowY = dRows;
    film.rowOwned = dOwned;
    film.rowCount = rowCount;
    dRowRays = nullptr;
    if (rowProbe) {   // (the probe's counters follow the film's height)
        CHECKED(DeviceAlloc(&dRowRays, filmH, &rowAllocs));
        HIPCHECK(hipMemsetAsync(dRowRays, 0, (size_t)filmH * 4, stream));
        CHECKED(UploadSampleOut());
    }
    return DCRT_OK;
}

int dcrt_tracer::UploadSampleOut()
{
    hSampleOut.rowRays = rowProbe ? dRowRays : nullptr;
    HIPCHECK(hipMemcpyAsync(dSampleOut, &hSampleOut, sizeof(SampleOut), hipMemcpyHostToDevice, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    return DCRT_OK;
}

// The row-cost probe: while on, MATERIAL's PROBE variant adds each pass's rays (the extension ray
// it shades, the shadow ray it casts) to a counter per film row -- the per-row cost that
// partition.balanced_bands cuts equal-cost film bands from. Turning it on or off re-captures
// the iteration graphs; on clears the counters.
int dcrt_tracer::SetRowProbe(bool on)
{
    HIPCHECK(hipStreamSynchronize(stream));
    InvalidateGraph();
    rowProbe = on;
    if (on && filmH) return BuildRows();   // (allocates and clears the counters)
    return UploadSampleOut();
}

int dcrt_tracer::SetFrame(const dcrt_frame_params& p)
{
    if (p.resolution[0] == 0 || p.resolution[1] == 0 || p.max_bounce_count > DCRT_MAX_RAY_BOUNCE) {
        SetLastError("invalid frame parameters");
        return DCRT_E_INVALID_ARG;
    }
    CHECKED(EnsureFilm(p.resolution[0], p.resolution[1]));
    if ((frame.features ^ p.features) & DCRT_FEATURE_ALLOW_ANYHIT) {   // captured graphs hold the other kernel variant
        HIPCHECK(hipStreamSynchronize(stream));
        InvalidateGraph();
    }
    frame = p;
    hasFrame = true;
    return DCRT_OK;
}

int dcrt_tracer::SetPartition(const dcrt_film_partition& p)
{
    if (p.world_size == 0 || p.rank >= p.world_size || (p.world_size > 1 && p.stripe_height == 0)) {
        SetLastError("invalid film partition");
        return DCRT_E_INVALID_ARG;
    }
    partition = p;
    bands.clear();
    if (filmW) {
        HIPCHECK(hipStreamSynchronize(stream));
        InvalidateGraph();
        CHECKED(BuildRows());
    }
    newImage = true;
    return DCRT_OK;
}

// Explicit film bands: this tracer owns rows [b[2i], b[2i+1]) (ascending, disjoint, non-empty),
// path-traces them plus `halo` rows beyond each band and convolves only its own rows. Any cut
// of the film into bands dealt to tracers sums to the one-tracer film bit for bit, as the
// stripes do; cost-balanced cuts come from the row-cost probe (partition.balanced_bands).
int dcrt_tracer::SetBands(const uint32_t* b, uint32_t count, uint32_t halo)
{
    if (count == 0 || !b) { SetLastError("no film bands"); return DCRT_E_INVALID_ARG; }
    for (uint32_t i = 0; i < count; ++i) {
        if (b[2 * i] >= b[2 * i + 1] || (i > 0 && b[2 * i] < b[2 * i - 1])) {
            SetLastError("film bands: ascending, disjoint, non-empty [y0, y1) ranges");
            return DCRT_E_INVALID_ARG;
        }
    }
    bands.assign(b, b + 2 * count);
    partition = dcrt_film_partition{1, 0, 64, halo};
    if (filmW) {
        HIPCHECK(hipStreamSynchronize(stream));
        InvalidateGraph();
        CHECKED(BuildRows());
    }
    newImage = true;
    return DCRT_OK;
}

// ResetImage + SET_IDLE + constant upload for one image (WavefrontPathTracer.cpp:441-468)
int dcrt_tracer::BeginImage()
{
    Annotation an("Reset", !capturing);
    FrameConstants fc;
    std::memset(&fc, 0, sizeof(fc));
    std::memcpy(fc.camera, frame.camera_transform, sizeof(fc.camera));
    fc.resolution[0] = frame.resolution[0]; fc.resolution[1] = frame.resolution[1];
    fc.filmSize[0] = frame.film_size[0]; fc.filmSize[1] = frame.film_size[1];
    fc.apertureRadius = frame.aperture_radius;
    fc.focalDistance = frame.focal_distance;
    fc.filmDistance = frame.film_distance;
    fc.bladeCount = frame.blade_count;
    fc.bladeVertexPos[0] = frame.blade_vertex_pos[0]; fc.bladeVertexPos[1] = frame.blade_vertex_pos[1];
    fc.apertureBaseAngle = frame.aperture_base_angle;
    fc.frameSeed = frame.frame_seed;
    fc.seedStride = seedStride;
    fc.maxBounce = frame.max_bounce_count;
    fc.lightCount = frame.light_count;
    fc.envLightIndex = frame.environment_light_index;
    fc.features = frame.features;
    fc.blocksX = (frame.resolution[0] + kBlockW - 1) / kBlockW;
    fc.bandCount = bandCount;
    fc.blocksPerImage = fc.blocksX * bandCount;
#ifndef DCRT_REFILL_GLOBAL
#define DCRT_REFILL_GLOBAL 28
#endif
    fc.refillLanes = tuneOverride || castAllCached ? refillLanes : DCRT_REFILL_GLOBAL;
    fc.parkLanes = parkLanes;
    // virtual batch starts (control_kernel): the merged cast kernels carry the camera-ray fetch;
    // not with ALLOW_ANYHIT_SHADER (NEW_PATH's opacity draw)
    fc.virtualStart = virtualStart && mergedCasts && !(frame.features & DCRT_FEATURE_ALLOW_ANYHIT) ? 1u : 0u;
    // drain completion (drain_kernel): not with ALLOW_ANYHIT_SHADER, and not while the cast
    // kernels are instrumented (the roofline leg's counts and launch times are the wavefront's)
    fc.drainPaths = !(frame.features & DCRT_FEATURE_ALLOW_ANYHIT) && !instrCounters && !extTiming && !rowProbe ? drainPaths : 0u;
    hipLaunchKernelGGL(set_frame_kernel, dim3(1), dim3(1), 0, stream, dFrame, fc);
    const uint32_t total = fc.blocksPerImage;
    const uint32_t idleThreads = std::max<uint32_t>(poolSize, 2u * (uint32_t)(sizeof(Counters) / 4));
    hipLaunchKernelGGL(set_idle_kernel, dim3((idleThreads + 255) / 256), dim3(256), 0, stream, pool, dCounters, dGlobals, total);
    HIPCHECK(hipGetLastError());
    parity = 0;
    newImage = false;
    imageComplete = false;
    return DCRT_OK;
}

// RenderOneIteration (WavefrontPathTracer.cpp:622-1162): CONTROL(+NEW_PATH) ->
// MATERIAL -> EXTENSION_RAY_CAST -> SHADOW_RAY_CAST. Queue sizes are read on the
// device, so no indirect-argument pass and no host round trip is needed.
// `sequenced` appends the film pass and the image advance, both no-ops unless
// this iteration completed an image (RenderImages runs images back to back).
int dcrt_tracer::LaunchIteration(uint32_t par, bool timed, bool sequenced)
{
    Annotation an("Iteration", !capturing);
    Counters* cnt = dCounters + par;
    Counters* next = dCounters + (par ^ 1u);   // (the previous iteration's; the casts clear them for the next)
    PathPool pool = this->pool;
    pool.extRec = extRecs + (size_t)par * kShards * pool.recCap * 2;
    pool.extPrevRec = extRecs + (size_t)(par ^ 1u) * kShards * pool.recCap * 2;
    pool.stateA = stateRecsA + (size_t)par * kShards * pool.recCap;
    pool.stateB = stateRecsB + (size_t)par * kShards * pool.recCap;
    pool.stateAPrev = stateRecsA + (size_t)(par ^ 1u) * kShards * pool.recCap;
    pool.stateBPrev = stateRecsB + (size_t)(par ^ 1u) * kShards * pool.recCap;
    pool.shadowHit = shadowHits + (size_t)par * kShards * pool.recCap;
    pool.shadowHitPrev = shadowHits + (size_t)(par ^ 1u) * kShards * pool.recCap;
    pool.finRec = finRecs + (size_t)par * kFinShards * pool.finCap;
    pool.finPrevRec = finRecs + (size_t)(par ^ 1u) * kFinShards * pool.finCap;
    pool.finHit = finHits + (size_t)par * kFinShards * pool.finCap;
    pool.finHitPrev = finHits + (size_t)(par ^ 1u) * kFinShards * pool.finCap;
    const bool opacity = (frame.features & DCRT_FEATURE_ALLOW_ANYHIT) != 0;
    const uint32_t castGrid = CastGrid(castBlock, opacity);
    // Timed launches take their start/stop timestamps from the dispatch itself
    // (hipExtLaunchKernelGGL), so the duration is the kernel's, as rocprofv3 reports it.
    hipEvent_t c0 = nullptr, c1 = nullptr, m0 = nullptr, m1 = nullptr, e0 = nullptr, e1 = nullptr;
    if (timed) CHECKED(TimedPair(kTimedControl, &c0, &c1));
    {
        Annotation a("Control", !capturing);
        hipExtLaunchKernelGGL(control_kernel, dim3(controlGrid), dim3(kControlBlock), 0, stream, c0, c1, 0, pool, film,
                              (const FrameConstants*)dFrame, cnt, (const Counters*)next, dGlobals, (uint32_t)(film.debugRng != nullptr));
    }
    auto material = rowProbe ? material_kernel<kCapAll, 0, true>
                  : materialCaps == kCapOpaqueDelta
                        ? (materialLdsMode == 1 ? material_kernel<kCapOpaqueDelta, 1>
                                                : materialLdsMode == 2 ? material_kernel<kCapOpaqueDelta, 2> : material_kernel<kCapOpaqueDelta, 0>)
                        : (materialLdsMode == 1 ? material_kernel<kCapAll, 1>
                                                : materialLdsMode == 2 ? material_kernel<kCapAll, 2> : material_kernel<kCapAll, 0>);
    if (timed) CHECKED(TimedPair(kTimedMaterial, &m0, &m1));
    {
        Annotation a("Material", !capturing);
        hipExtLaunchKernelGGL(material, dim3(materialGrid), dim3(kMaterialBlock), rowProbe ? 0u : materialLds, stream, m0, m1, 0, pool, scene,
                              (const FrameConstants*)dFrame, cnt, (const Counters*)next, (const SampleOut*)dSampleOut);
    }
    if (timed) CHECKED(TimedPair(kTimedCast, &e0, &e1));
    // kernel variant: instrumented counts x ALLOW_ANYHIT_SHADER
    Annotation castAnnotation(mergedCasts ? "Extension + shadow ray cast" : "Extension ray cast, shadow ray cast", !capturing);
    if (mergedCasts) {
        const bool ring = ringRows != 0 && !instrCounters && !opacity;   // (the ring kernel; the counting and
                                                                        // any-hit kernels keep the whole stack)
        const bool flat = castFlat && !instrCounters && !opacity;
        auto cast = CastKernel(instrCounters, opacity, castAllCached, castPair, castIdent, ring, flat);
        hipExtLaunchKernelGGL(cast, dim3(castGrid), dim3(castBlock), flat ? castLdsFlat : ring ? castLds : castLdsFull, stream, e0,
                              e1, 0, pool, flat ? sceneFlat : ring ? sceneRing : scene,
                              (const FrameConstants*)dFrame, cnt, next, dGlobals, dInstr);
    } else {
        auto ext = instrCounters ? (opacity ? extension_kernel<true, true> : extension_kernel<true, false>)
                                 : (opacity ? extension_kernel<false, true> : extension_kernel<false, false>);
        auto shadow = instrCounters ? (opacity ? shadow_kernel<true, true> : shadow_kernel<true, false>)
                                    : (opacity ? shadow_kernel<false, true> : shadow_kernel<false, false>);
        hipExtLaunchKernelGGL(ext, dim3(castGrid), dim3(castBlock), castLdsFull, stream, e0, e1, 0, pool, scene,
                              (const FrameConstants*)dFrame, (const Counters*)cnt, dGlobals, dInstr);
        hipLaunchKernelGGL(shadow, dim3(castGrid), dim3(castBlock), castLdsFull, stream, pool, scene, (const FrameConstants*)dFrame, cnt,
                           next, dGlobals, dInstr);
    }
    if (drainPaths) {
        // (returns at once unless the batch's last paths are few enough: fc.drainPaths)
        auto drain = materialCaps == kCapOpaqueDelta ? drain_kernel<kCapOpaqueDelta> : drain_kernel<kCapAll>;
        hipLaunchKernelGGL(drain, dim3(drainResident), dim3(castBlock), castLdsFull, stream, pool, scene, (const FrameConstants*)dFrame, cnt,
                           dGlobals, (const SampleOut*)dSampleOut);
    }
    if (sequenced) {
        hipLaunchKernelGGL(film_kernel, dim3(FilmGrid()), dim3(kFilmThreads), 0, stream, film, (const FilterConsts*)dFilter, 1u,
                           (const Globals*)dGlobals, (const float2* const*)nullptr, (const float4* const*)nullptr);
        hipLaunchKernelGGL(advance_image_kernel, dim3(1), dim3(64), 0, stream, dFrame, dGlobals);
    }
    HIPCHECK(hipGetLastError());
    return DCRT_OK;
}

// Replay `iters` iterations (even, starting at parity 0) as one captured graph.
// RenderImages' graph of tail chunks (its final batch) holds kTailChunk iterations
static uint32_t GraphSlot(bool sequenced, uint32_t iters) { return !sequenced ? 0u : (iters == kTailChunk ? 2u : 1u); }
int dcrt_tracer::LaunchGraph(bool sequenced, uint32_t iters)
{
    Annotation an(sequenced ? "Iterations (graph, sequenced images)" : "Iterations (graph)");
    CHECKED(BuildGraph(sequenced, iters));
    HIPCHECK(hipGraphLaunch(graphs[GraphSlot(sequenced, iters)].exec, stream));
    return DCRT_OK;
}

// Capture (once) the graph of `iters` iterations; kernels take the buffers by value, so
// a reallocation (EnsureSamples) invalidates it.
int dcrt_tracer::BuildGraph(bool sequenced, uint32_t iters)
{
    GraphCache& gc = graphs[GraphSlot(sequenced, iters)];
    if (!gc.exec || gc.iters != iters) {
        if (gc.exec) (void)hipGraphExecDestroy(gc.exec);
        gc.exec = nullptr;
        hipGraph_t g = nullptr;
        HIPCHECK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
        int rc = DCRT_OK;
        capturing = true;
        for (uint32_t i = 0; i < iters && rc == DCRT_OK; ++i) rc = LaunchIteration(i & 1u, false, sequenced);
        capturing = false;
        hipError_t ec = hipStreamEndCapture(stream, &g);
        if (rc != DCRT_OK) return rc;
        HIPCHECK(ec);
        HIPCHECK(hipGraphInstantiate(&gc.exec, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
        gc.iters = iters;
    }
    return DCRT_OK;
}

// What RenderImages(count) would allocate or capture on its first call: the batch's
// sample textures and the sequenced graph. Lets a caller keep both out of a timed region.
int dcrt_tracer::PrepareImages(uint32_t count)
{
    if (!hasScene) { SetLastError("no scene uploaded"); return DCRT_E_NO_SCENE; }
    if (!hasFrame) { SetLastError("no frame parameters"); return DCRT_E_INVALID_ARG; }
    if (count == 0 || mode == 1) return DCRT_OK;
    // (also the slots of a render without the film pass, which keeps every image: slot k = image k)
    const uint64_t keptCap = std::min<uint64_t>(kMaxImageBatch, ((uint64_t)1 << 31) / ((uint64_t)filmW * filmH));
    CHECKED(EnsureSamples(std::max<uint32_t>(AutoBatch(count), count <= keptCap ? count : 0u)));
    if (!extTiming) {
        const uint32_t chunk = std::max<uint32_t>(2, iterationsPerRender & ~1u);
        CHECKED(BuildGraph(true, chunk));
        if (chunk > kTailChunk) CHECKED(BuildGraph(true, kTailChunk));
    }
    HIPCHECK(hipStreamSynchronize(stream));
    return DCRT_OK;
}

// n plain iterations (Render); even chunks replay a captured graph.
int dcrt_tracer::RunIterations(uint32_t n)
{
    const uint32_t chunk = std::max<uint32_t>(2, iterationsPerRender & ~1u);
    while (n > 0) {
        if (!extTiming && parity == 0 && n >= chunk) {
            CHECKED(LaunchGraph(false, chunk));
            n -= chunk;
        } else {
            CHECKED(LaunchIteration(parity, extTiming, false));
            parity ^= 1u;
            --n;
        }
    }
    return DCRT_OK;
}

// IsImageComplete (WavefrontPathTracer.cpp:508-523): no path was live entering the last
// iteration and none was started (Globals::poolIdle). Here exact, not 2 frames late.
int dcrt_tracer::ReadCompletion(bool* complete)
{
    uint32_t* h = (uint32_t*)hCounters;   // (pinned staging)
    HIPCHECK(hipMemcpyAsync(h, &dGlobals->poolIdle, sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
    HIPCHECK(hipStreamSynchronize(stream));
    *complete = *h != 0;
    return DCRT_OK;
}

int dcrt_tracer::Render(uint32_t maxIterations)
{
    if (!hasScene) { SetLastError("no scene uploaded"); return DCRT_E_NO_SCENE; }
    if (!hasFrame) { SetLastError("no frame parameters"); return DCRT_E_INVALID_ARG; }
    if (newImage) CHECKED(BeginImage());
    lastSlot = 0;
    CHECKED(RunIterations(maxIterations ? maxIterations : iterationsPerRender));
    bool complete = false;
    CHECKED(ReadCompletion(&complete));
    if (complete) ++imagesCompleted;
    imageComplete = complete;
    newImage = complete;   // WavefrontPathTracer.cpp:500
    return DCRT_OK;
}

int dcrt_tracer::UploadFilter(const dcrt_filter_params& f)
{
    HIPCHECK(hipStreamSynchronize(stream));     // the pinned staging buffer is reused
    *hFilter = MakeFilter(f);
    HIPCHECK(hipMemcpyAsync(dFilter, hFilter, sizeof(FilterConsts), hipMemcpyHostToDevice, stream));
    return DCRT_OK;
}

int dcrt_tracer::Accumulate(const dcrt_filter_params& f)
{
    Annotation an("SampleConvolution");
    if (!film.accum) { SetLastError("no film"); return DCRT_E_INVALID_ARG; }
    CHECKED(UploadFilter(f));
    hipLaunchKernelGGL(film_kernel, dim3(FilmGrid()), dim3(kFilmThreads), 0, stream, film, (const FilterConsts*)dFilter, 1u,
                       (const Globals*)nullptr, (const float2* const*)nullptr, (const float4* const*)nullptr);
    HIPCHECK(hipGetLastError());
    return DCRT_OK;
}

// Images firstSeed .. firstSeed+count-1 back to back: the device detects each
// image's completion, convolves it into the film and starts the next one, so the
// host only enqueues graphs and polls a pinned "stopped" word two graphs behind.
int dcrt_tracer::RenderImages(uint32_t firstSeed, uint32_t count, const dcrt_filter_params& filter, uint32_t stride, bool convolve)
{
    seedStride = std::max<uint32_t>(1u, stride);
    keptSlots = false;
    Annotation an("RenderImages");
    if (!hasScene) { SetLastError("no scene uploaded"); return DCRT_E_NO_SCENE; }
    if (!hasFrame) { SetLastError("no frame parameters"); return DCRT_E_INVALID_ARG; }
    if (count == 0) return DCRT_OK;
    if (partition.world_size > 1 || !bands.empty()) {
        // a partitioned film's convolution reads the filter's window rows beyond its stripes
        const uint32_t halo = partition.halo_rows ? partition.halo_rows : 2u;
        if (!(filter.radius >= 0.0f) || FilterSupportRows(filter.radius, filmH) > halo) {
            SetLastError("filter radius needs more halo rows than the film partition renders");
            return DCRT_E_INVALID_ARG;
        }
    }
    lastSlot = 0;
    if (mode == 1) {   // MegakernelPathTracer::Render: one persistent launch + SampleConvolution per image
        if (!convolve) { SetLastError("the megakernel mode convolves every image"); return DCRT_E_INVALID_ARG; }
        CHECKED(UploadFilter(filter));
        for (uint32_t img = 0; img < count; ++img) {
            frame.frame_seed = firstSeed + img * seedStride;
            CHECKED(BeginImage());
            hipEvent_t e0 = nullptr, e1 = nullptr;
            if (extTiming) CHECKED(TimedPair(kTimedCast, &e0, &e1));
            auto mk = (frame.features & DCRT_FEATURE_ALLOW_ANYHIT) ? megakernel<true> : megakernel<false>;
            hipExtLaunchKernelGGL(mk, dim3(megaResident), dim3(castBlock), castLdsFull, stream, e0, e1, 0, scene,
                                  (const FrameConstants*)dFrame, film, dGlobals, (uint32_t)(film.debugRng != nullptr));
            hipLaunchKernelGGL(film_kernel, dim3(FilmGrid()), dim3(kFilmThreads), 0, stream, film, (const FilterConsts*)dFilter, 1u,
                               (const Globals*)nullptr, (const float2* const*)nullptr, (const float4* const*)nullptr);
            HIPCHECK(hipGetLastError());
        }
        HIPCHECK(hipStreamSynchronize(stream));
        imageComplete = true;
        newImage = true;
        imagesCompleted += count;
        return DCRT_OK;
    }
    uint32_t batch = AutoBatch(count);
    if (!convolve) {
        // every image keeps its samples (slot k = image k) for the caller's film pass: one batch
        const uint64_t cap = std::min<uint64_t>(kMaxImageBatch, ((uint64_t)1 << 31) / ((uint64_t)filmW * filmH));
        if (count > cap) { SetLastError("render_images without the film pass: too many images for one batch"); return DCRT_E_LIMIT; }
        batch = count;
    }
    CHECKED(EnsureSamples(batch));
    frame.frame_seed = firstSeed;
    CHECKED(UploadFilter(filter));
    CHECKED(BeginImage());
    // static batch-start claims: one per wave of CONTROL's virtual workgroups
    const uint32_t staticGrid = poolSize / kControlBlock;
    hipLaunchKernelGGL(begin_images_kernel, dim3(1), dim3(64), 0, stream, dGlobals, (const FrameConstants*)dFrame, count, firstSeed, batch,
                       staticGrid, convolve ? 0u : 1u);
    HIPCHECK(hipGetLastError());
    // a path needs maxBounce + 3 iterations; cap the total so a broken scene cannot spin forever
    const uint64_t maxIterations = ((uint64_t)count + 2) * (frame.max_bounce_count + 8) * (1 + (filmW * (uint64_t)filmH) / poolSize) + 64;
    uint64_t launched = 0;
    bool stopped = false;
    {
        // chunks of `chunk` iterations (a replayed graph, or plain timed launches when the
        // EXT kernel is being timed), the "stopped" word polled two chunks behind; once the
        // final batch is in flight (imagesDone + batch >= count, polled with it), chunks of
        // kTailChunk: the chunks launched after the last image completes find no work
        // (32 empty iterations after a one-batch call took 0.4 ms with 16-iteration chunks)
        const uint32_t bigChunk = std::max<uint32_t>(2, iterationsPerRender & ~1u);
        bool finalBatch = count <= batch;
        uint32_t inflight[4];
        uint32_t head = 0, size = 0, slot = 0;
        while (!stopped && launched < maxIterations) {
            const uint32_t chunk = finalBatch ? std::min(bigChunk, kTailChunk) : bigChunk;
            if (extTiming) {
                for (uint32_t i = 0; i < chunk; ++i) {
                    CHECKED(LaunchIteration(parity, true, true));
                    parity ^= 1u;
                }
            } else {
                CHECKED(LaunchGraph(true, chunk));
            }
            launched += chunk;
            static_assert(offsetof(Globals, imagesDone) == offsetof(Globals, stopped) + 4, "polled together");
            HIPCHECK(hipMemcpyAsync(&hStop[2 * slot], &dGlobals->stopped, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
            HIPCHECK(hipEventRecord(stopEvents[slot], stream));
            inflight[(head + size) % 4] = slot;
            ++size;
            slot = (slot + 1) % 4;
            if (size >= 2) {
                const uint32_t s0 = inflight[head];
                HIPCHECK(hipEventSynchronize(stopEvents[s0]));
                stopped = hStop[2 * s0] != 0;
                finalBatch = finalBatch || (uint64_t)hStop[2 * s0 + 1] + batch >= count;
                head = (head + 1) % 4;
                --size;
            }
        }
        // graphs still in flight after `stopped` find no work (CONTROL returns at once)
    }
    HIPCHECK(hipStreamSynchronize(stream));
    if (!stopped) {
        HIPCHECK(hipMemcpy(hStop, &dGlobals->stopped, sizeof(uint32_t), hipMemcpyDeviceToHost));
        if (!hStop[0]) { SetLastError("images did not complete"); return DCRT_E_LIMIT; }
    }
    imageComplete = true;
    newImage = true;
    imagesCompleted += count;
    lastSlot = (count - 1) % batch;
    keptSlots = !convolve;
    keptImages = keptSlots ? count : 0u;
    return DCRT_OK;
}

// The film pass over `count` images whose sample textures (W*H each, this film's size) sit at
// the caller's device pointers -- e.g. the slots of several pipelines that rendered interleaved
// images (render_images without the film pass): image b of the list is convolved b-th, so the
// film is the one-pipeline film bit for bit when the list is in image order.
int dcrt_tracer::AccumulateImages(const void* const* pos, const void* const* val, uint32_t count, const dcrt_filter_params& f)
{
    Annotation an("SampleConvolution (image list)");
    if (!film.accum) { SetLastError("no film"); return DCRT_E_INVALID_ARG; }
    if (count == 0) return DCRT_OK;
    if (count > sourceCap) {
        HIPCHECK(hipStreamSynchronize(stream));
        if (dSourceLists) (void)hipFree(dSourceLists);
        dSourceLists = nullptr;
        sourceCap = 0;
        HIPCHECK(hipMalloc(&dSourceLists, (size_t)count * 2 * sizeof(void*)));
        sourceCap = count;
    }
    std::vector<const void*> lists((size_t)count * 2);
    for (uint32_t i = 0; i < count; ++i) {
        if (!pos[i] || !val[i]) { SetLastError("null sample texture pointer"); return DCRT_E_INVALID_ARG; }
        lists[i] = pos[i];
        lists[count + i] = val[i];
    }
    CHECKED(UploadFilter(f));   // (synchronises: the list's staging below is reused safely)
    HIPCHECK(hipMemcpyAsync(dSourceLists, lists.data(), lists.size() * sizeof(void*), hipMemcpyHostToDevice, stream));
    hipLaunchKernelGGL(film_kernel, dim3(FilmGrid()), dim3(kFilmThreads), 0, stream, film, (const FilterConsts*)dFilter, count,
                       (const Globals*)nullptr, (const float2* const*)dSourceLists, (const float4* const*)(dSourceLists + count));
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(stream));   // (the host list is released on return)
    return DCRT_OK;
}

// ============================ C ABI ========================================
#define TRACER_GUARD(t)                                         \
    if (!(t)) return DCRT_E_INVALID_ARG;                        \
    if (hipSetDevice((t)->device) != hipSuccess) {              \
        SetLastError("hipSetDevice failed");                    \
        return DCRT_E_HIP;                                      \
    }

extern "C" {

DCRT_API int dcrt_device_count(int* out)
{
    if (!out) return DCRT_E_INVALID_ARG;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_create(const dcrt_tracer_config* config, dcrt_tracer** out)
{
    if (!out) return DCRT_E_INVALID_ARG;
    *out = nullptr;
    dcrt_tracer_config cfg{};
    if (config) cfg = *config;
    dcrt_tracer* t = new (std::nothrow) dcrt_tracer();
    if (!t) return DCRT_E_LIMIT;
    const int rc = t->Create(cfg);
    if (rc != DCRT_OK) { delete t; return rc; }
    *out = t;
    return DCRT_OK;
}

DCRT_API void dcrt_tracer_destroy(dcrt_tracer* t) { delete t; }

DCRT_API int dcrt_tracer_upload_scene(dcrt_tracer* t, const dcrt_flat_scene* s)
{
    TRACER_GUARD(t);
    if (!s) return DCRT_E_INVALID_ARG;
    return t->UploadScene(*s);
}

DCRT_API int dcrt_tracer_set_frame_params(dcrt_tracer* t, const dcrt_frame_params* p)
{
    TRACER_GUARD(t);
    if (!p) return DCRT_E_INVALID_ARG;
    return t->SetFrame(*p);
}

DCRT_API int dcrt_tracer_set_film_partition(dcrt_tracer* t, const dcrt_film_partition* p)
{
    TRACER_GUARD(t);
    if (!p) return DCRT_E_INVALID_ARG;
    return t->SetPartition(*p);
}

DCRT_API int dcrt_tracer_set_film_bands(dcrt_tracer* t, const uint32_t* bands, uint32_t band_count, uint32_t halo_rows)
{
    TRACER_GUARD(t);
    return t->SetBands(bands, band_count, halo_rows);
}

DCRT_API int dcrt_tracer_render(dcrt_tracer* t, uint32_t max_iterations)
{
    TRACER_GUARD(t);
    return t->Render(max_iterations);
}

DCRT_API int dcrt_tracer_render_images(dcrt_tracer* t, uint32_t first_seed, uint32_t count, const dcrt_filter_params* f)
{
    TRACER_GUARD(t);
    if (!f) return DCRT_E_INVALID_ARG;
    return t->RenderImages(first_seed, count, *f);
}

DCRT_API int dcrt_tracer_render_images_strided(dcrt_tracer* t, uint32_t first_seed, uint32_t seed_stride, uint32_t count,
                                               int convolve, const dcrt_filter_params* f)
{
    TRACER_GUARD(t);
    if (!f || seed_stride == 0) return DCRT_E_INVALID_ARG;
    return t->RenderImages(first_seed, count, *f, seed_stride, convolve != 0);
}

DCRT_API int dcrt_tracer_image_sample_ptrs(dcrt_tracer* t, uint32_t image, void** pos, void** val)
{
    TRACER_GUARD(t);
    if (!pos || !val) return DCRT_E_INVALID_ARG;
    if (!t->keptSlots || image >= t->keptImages) {
        SetLastError("no such image: its samples are kept only by render_images without the film pass");
        return DCRT_E_INVALID_ARG;
    }
    const size_t o = (size_t)t->filmW * t->filmH * image;
    *pos = (void*)(t->film.samplePosition + o);
    *val = (void*)(t->film.sampleValue + o);
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_accumulate_images(dcrt_tracer* t, const void* const* d_positions, const void* const* d_values,
                                           uint32_t image_count, const dcrt_filter_params* f)
{
    TRACER_GUARD(t);
    if (!f || (image_count && (!d_positions || !d_values))) return DCRT_E_INVALID_ARG;
    return t->AccumulateImages(d_positions, d_values, image_count, *f);
}

DCRT_API int dcrt_tracer_reset_image(dcrt_tracer* t)
{
    TRACER_GUARD(t);
    t->newImage = true;
    t->imageComplete = false;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_is_image_complete(dcrt_tracer* t, int* out)
{
    TRACER_GUARD(t);
    if (!out) return DCRT_E_INVALID_ARG;
    *out = t->imageComplete ? 1 : 0;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_acquire_film_clear_trigger(dcrt_tracer* t, int* out)
{
    TRACER_GUARD(t);
    if (!out) return DCRT_E_INVALID_ARG;
    *out = t->filmClearTrigger ? 1 : 0;
    t->filmClearTrigger = false;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_clear_film(dcrt_tracer* t)
{
    TRACER_GUARD(t);
    if (!t->film.accum) return DCRT_E_INVALID_ARG;
    HIPCHECK(hipMemsetAsync(t->film.accum, 0, (size_t)t->filmW * t->filmH * sizeof(float4), t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_accumulate_film(dcrt_tracer* t, const dcrt_filter_params* f)
{
    TRACER_GUARD(t);
    if (!f) return DCRT_E_INVALID_ARG;
    return t->Accumulate(*f);
}

DCRT_API int dcrt_tracer_read_film(dcrt_tracer* t, float* out)
{
    TRACER_GUARD(t);
    if (!out || !t->film.accum) return DCRT_E_INVALID_ARG;
    HIPCHECK(hipMemcpyAsync(out, t->film.accum, (size_t)t->filmW * t->filmH * sizeof(float4), hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_read_samples(dcrt_tracer* t, float* pos, float* val)
{
    TRACER_GUARD(t);
    if (!t->film.sampleValue) return DCRT_E_INVALID_ARG;
    const size_t n = (size_t)t->filmW * t->filmH, o = n * t->lastSlot;   // the last image's samples
    if (pos) HIPCHECK(hipMemcpyAsync(pos, t->film.samplePosition + o, n * sizeof(float2), hipMemcpyDeviceToHost, t->stream));
    if (val) HIPCHECK(hipMemcpyAsync(val, t->film.sampleValue + o, n * sizeof(float4), hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_read_rng(dcrt_tracer* t, uint32_t* out)
{
    TRACER_GUARD(t);
    if (!out || !t->film.debugRng) { SetLastError("tracer was created without debug_rng"); return DCRT_E_INVALID_ARG; }
    const size_t n = (size_t)t->filmW * t->filmH;
    HIPCHECK(hipMemcpyAsync(out, t->film.debugRng + n * t->lastSlot, n * sizeof(uint4), hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_film_device_ptr(dcrt_tracer* t, void** out)
{
    TRACER_GUARD(t);
    if (!out) return DCRT_E_INVALID_ARG;
    *out = t->film.accum;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_sample_device_ptrs(dcrt_tracer* t, void** pos, void** val)
{
    TRACER_GUARD(t);
    if (!pos || !val) return DCRT_E_INVALID_ARG;
    if (!t->film.sampleValue) { SetLastError("no frame parameters: the sample textures are not allocated"); return DCRT_E_INVALID_ARG; }
    const size_t o = (size_t)t->filmW * t->filmH * t->lastSlot;   // the last image's slot
    *pos = (void*)(t->film.samplePosition + o);
    *val = (void*)(t->film.sampleValue + o);
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_set_row_cost_probe(dcrt_tracer* t, int enable)
{
    TRACER_GUARD(t);
    if (enable && t->mode != 0) { SetLastError("the row-cost probe counts the wavefront's MATERIAL passes"); return DCRT_E_INVALID_ARG; }
    return t->SetRowProbe(enable != 0);
}

DCRT_API int dcrt_tracer_read_row_cost(dcrt_tracer* t, uint32_t* out_rows)
{
    TRACER_GUARD(t);
    if (!out_rows) return DCRT_E_INVALID_ARG;
    if (!t->rowProbe || !t->dRowRays) { SetLastError("the row-cost probe is off"); return DCRT_E_INVALID_ARG; }
    HIPCHECK(hipMemcpyAsync(out_rows, t->dRowRays, (size_t)t->filmH * 4, hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_copy_film_device(dcrt_tracer* t, void* d_dst)
{
    TRACER_GUARD(t);
    if (!d_dst || !t->film.accum) return DCRT_E_INVALID_ARG;
    HIPCHECK(hipMemcpyAsync(d_dst, t->film.accum, (size_t)t->filmW * t->filmH * sizeof(float4), hipMemcpyDeviceToDevice,
                            t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_add_film_device(dcrt_tracer* t, const void* d_src)
{
    TRACER_GUARD(t);
    if (!d_src || !t->film.accum) return DCRT_E_INVALID_ARG;
    const uint32_t n = t->filmW * t->filmH;
    hipLaunchKernelGGL(add_film_kernel, dim3(std::min<uint32_t>((n + 255) / 256, kMaxPersistentBlocks)), dim3(256), 0, t->stream,
                       t->film.accum, (const float4*)d_src, n);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_counters(dcrt_tracer* t, dcrt_ray_stats* out)
{
    TRACER_GUARD(t);
    if (!out) return DCRT_E_INVALID_ARG;
    Globals g;
    HIPCHECK(hipMemcpyAsync(&g, t->dGlobals, sizeof(Globals), hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    out->extension_rays = g.extRays;
    out->shadow_rays = g.shadowRays;
    // every rendered pixel (film rows of this tracer, halo included) starts one path per image
    out->new_paths = t->imagesCompleted * (uint64_t)t->rowCount * t->filmW;
    out->iterations = g.iterations;
    out->images_completed = t->imagesCompleted;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_set_instrumentation(dcrt_tracer* t, int counters, int ext_timing)
{
    TRACER_GUARD(t);
    if ((counters != 0) != t->instrCounters) t->InvalidateGraph();
    t->instrCounters = counters != 0;
    t->extTiming = ext_timing != 0;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_get_info(dcrt_tracer* t, dcrt_tracer_info* out)
{
    TRACER_GUARD(t);
    if (!out) return DCRT_E_INVALID_ARG;
    out->path_pool_size = t->poolSize;
    out->scene_in_lds = t->hasScene && t->castAllCached ? 1u : 0u;
    out->cached_nodes = t->hasScene ? t->scene.cachedNodes : 0u;
    out->cached_triangles = t->hasScene ? t->scene.cachedTris : 0u;
    out->cast_block = t->castBlock;
    out->traversal_stack = t->hasScene ? t->scene.stackSize : 0u;
    out->material_generic = t->materialCaps == kCapAll ? 1u : 0u;
    out->pair_traversal = t->hasScene && t->castPair ? 1u : 0u;
    out->control_grid = t->controlGrid;
    out->material_grid = t->materialGrid;
    out->cast_grid = t->castResident;
    out->material_lds = t->materialLds;
    out->cast_identity = t->castIdent ? (t->castFlat ? 2u : 1u) : 0u;
    out->stack_lds_rows = t->hasScene ? (t->ringRows ? t->ringRows : t->castFlat ? t->sceneFlat.stackRows : t->scene.stackRows) : 0u;
    out->ring_rows = t->hasScene ? t->ringRows : 0u;
    out->cast_waves_per_cu = t->castPerCU * (t->castBlock / 64u);
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_debug_ring_spills(dcrt_tracer* t, uint64_t* out)
{
    TRACER_GUARD(t);
    if (!out) return DCRT_E_INVALID_ARG;
    *out = 0;
    if (!t->hasScene || !t->ringRows) return DCRT_OK;
    const size_t n = (size_t)t->castResident * t->castBlock * t->scene.stackSize;
    std::vector<uint32_t> h(n);
    HIPCHECK(hipStreamSynchronize(t->stream));
    HIPCHECK(hipMemcpy(h.data(), t->sceneRing.spill, n * 4, hipMemcpyDeviceToHost));
    for (const uint32_t w : h) *out += w != 0u;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_traversal_stats(dcrt_tracer* t, dcrt_traversal_stats* out)
{
    TRACER_GUARD(t);
    if (!out) return DCRT_E_INVALID_ARG;
    unsigned long long v[8];
    HIPCHECK(hipMemcpyAsync(v, t->dInstr, sizeof(v), hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    CHECKED(t->CollectTimes());
    out->ext_node_visits = v[0]; out->ext_triangle_tests = v[1]; out->ext_blas_entries = v[2];
    out->shadow_node_visits = v[3]; out->shadow_triangle_tests = v[4]; out->shadow_blas_entries = v[5];
    out->ext_launches = t->kindLaunches[dcrt_tracer::kTimedCast];
    out->ext_kernel_ms = t->kindMs[dcrt_tracer::kTimedCast];
    out->ext_max_node_visits = v[6]; out->shadow_max_node_visits = v[7];
    out->material_launches = t->kindLaunches[dcrt_tracer::kTimedMaterial];
    out->material_kernel_ms = t->kindMs[dcrt_tracer::kTimedMaterial];
    out->control_launches = t->kindLaunches[dcrt_tracer::kTimedControl];
    out->control_kernel_ms = t->kindMs[dcrt_tracer::kTimedControl];
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_reset_stats(dcrt_tracer* t)
{
    TRACER_GUARD(t);
    HIPCHECK(hipStreamSynchronize(t->stream));
    HIPCHECK(hipMemsetAsync(t->dInstr, 0, 8 * sizeof(unsigned long long), t->stream));
    Globals g;
    HIPCHECK(hipMemcpyAsync(&g, t->dGlobals, sizeof(Globals), hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    g.extRays = g.shadowRays = g.iterations = 0;
    t->imagesCompleted = 0;
    HIPCHECK(hipMemcpyAsync(t->dGlobals, &g, sizeof(Globals), hipMemcpyHostToDevice, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    t->eventsUsed = 0;
    for (int k = 0; k < dcrt_tracer::kTimedKinds; ++k) {
        t->kindMs[k] = 0.0;
        t->kindLaunches[k] = 0;
    }
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_synchronize(dcrt_tracer* t)
{
    TRACER_GUARD(t);
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_get_luts(dcrt_tracer* t, dcrt_bxdf_luts* out)
{
    TRACER_GUARD(t);
    if (!out) return DCRT_E_INVALID_ARG;
    HIPCHECK(hipMemcpyAsync(out, t->dLuts, sizeof(dcrt_bxdf_luts), hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_set_luts(dcrt_tracer* t, const dcrt_bxdf_luts* luts)
{
    TRACER_GUARD(t);
    if (!luts) return DCRT_E_INVALID_ARG;
    HIPCHECK(hipMemcpyAsync(t->dLuts, luts, sizeof(dcrt_bxdf_luts), hipMemcpyHostToDevice, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

static int TraceBatch(dcrt_tracer* t, const dcrt_ray* d_rays, uint32_t n, dcrt_ray_hit* d_hits, uint32_t* d_occ, bool any, uint32_t features)
{
    if (!t->hasScene) { SetLastError("no scene uploaded"); return DCRT_E_NO_SCENE; }
    const uint32_t grid = std::min<uint32_t>((n + t->castBlock - 1) / t->castBlock, t->castResident);
    if (n == 0) return DCRT_OK;
    unsigned long long* instr = t->instrCounters ? t->dInstr : nullptr;
    auto kernel = any ? (instr ? batch_trace_kernel<true, true> : batch_trace_kernel<true, false>)
                      : (instr ? batch_trace_kernel<false, true> : batch_trace_kernel<false, false>);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(t->castBlock), t->castLdsFull, t->stream, t->scene, d_rays, n, features, d_hits, d_occ, instr);
    HIPCHECK(hipGetLastError());
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_trace_rays(dcrt_tracer* t, const dcrt_ray* rays, uint32_t n, dcrt_ray_hit* out, uint32_t features)
{
    TRACER_GUARD(t);
    if ((!rays || !out) && n) return DCRT_E_INVALID_ARG;
    std::vector<void*> tmp;
    dcrt_ray* dr = nullptr; dcrt_ray_hit* dh = nullptr;
    CHECKED(DeviceAlloc(&dr, n, &tmp));
    CHECKED(DeviceAlloc(&dh, n, &tmp));
    int rc = DCRT_OK;
    if (hipMemcpyAsync(dr, rays, (size_t)n * sizeof(dcrt_ray), hipMemcpyHostToDevice, t->stream) != hipSuccess) rc = DCRT_E_HIP;
    if (rc == DCRT_OK) rc = TraceBatch(t, dr, n, dh, nullptr, false, features);
    if (rc == DCRT_OK && hipMemcpyAsync(out, dh, (size_t)n * sizeof(dcrt_ray_hit), hipMemcpyDeviceToHost, t->stream) != hipSuccess) rc = DCRT_E_HIP;
    if (hipStreamSynchronize(t->stream) != hipSuccess) rc = DCRT_E_HIP;
    FreeAll(&tmp);
    return rc;
}

DCRT_API int dcrt_tracer_occluded(dcrt_tracer* t, const dcrt_ray* rays, uint32_t n, uint32_t* out, uint32_t features)
{
    TRACER_GUARD(t);
    if ((!rays || !out) && n) return DCRT_E_INVALID_ARG;
    std::vector<void*> tmp;
    dcrt_ray* dr = nullptr; uint32_t* dOcc = nullptr;
    CHECKED(DeviceAlloc(&dr, n, &tmp));
    CHECKED(DeviceAlloc(&dOcc, n, &tmp));
    int rc = DCRT_OK;
    if (hipMemcpyAsync(dr, rays, (size_t)n * sizeof(dcrt_ray), hipMemcpyHostToDevice, t->stream) != hipSuccess) rc = DCRT_E_HIP;
    if (rc == DCRT_OK) rc = TraceBatch(t, dr, n, nullptr, dOcc, true, features);
    if (rc == DCRT_OK && hipMemcpyAsync(out, dOcc, (size_t)n * 4, hipMemcpyDeviceToHost, t->stream) != hipSuccess) rc = DCRT_E_HIP;
    if (hipStreamSynchronize(t->stream) != hipSuccess) rc = DCRT_E_HIP;
    FreeAll(&tmp);
    return rc;
}

DCRT_API int dcrt_tracer_trace_rays_device(dcrt_tracer* t, const void* d_rays, uint32_t n, void* d_hits, uint32_t features)
{
    TRACER_GUARD(t);
    if ((!d_rays || !d_hits) && n) return DCRT_E_INVALID_ARG;
    return TraceBatch(t, (const dcrt_ray*)d_rays, n, (dcrt_ray_hit*)d_hits, nullptr, false, features);
}

DCRT_API int dcrt_tracer_prepare_images(dcrt_tracer* t, uint32_t image_count)
{
    TRACER_GUARD(t);
    return t->PrepareImages(image_count);
}

DCRT_API int dcrt_tracer_set_image_batch(dcrt_tracer* t, uint32_t images)
{
    TRACER_GUARD(t);
    if (images > kMaxImageBatch) { SetLastError("image batch too large (max 256)"); return DCRT_E_INVALID_ARG; }
    t->batchImages = images;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_set_mode(dcrt_tracer* t, int mode)
{
    TRACER_GUARD(t);
    if (mode != 0 && mode != 1) return DCRT_E_INVALID_ARG;
    t->mode = mode;
    return DCRT_OK;
}

DCRT_API int dcrt_tracer_resolve_image(dcrt_tracer* t, const dcrt_postfx_params* prm, uint8_t* out, float* outSumLogLum)
{
    TRACER_GUARD(t);
    if (!prm || !out || !t->film.accum) return DCRT_E_INVALID_ARG;
    const uint32_t W = t->filmW, H = t->filmH;
    float hth[255];
    dcrt_srgb_encode_thresholds(hth);
    std::vector<void*> tmp;
    struct Free { std::vector<void*>* v; ~Free() { FreeAll(v); } } guard{ &tmp };
    float* dth = nullptr;
    CHECKED(DeviceAlloc(&dth, 255, &tmp));
    HIPCHECK(hipMemcpyAsync(dth, hth, sizeof(hth), hipMemcpyHostToDevice, t->stream));
    // SumLuminance: REDUCE_TO_1D then REDUCE_TO_SINGLE until one value (SceneLuminance.cpp:110-190)
    const uint32_t bx = (((W + 7) / 8) + 1) / 2, by = (((H + 7) / 8) + 1) / 2;
    float *la = nullptr, *lb = nullptr;
    CHECKED(DeviceAlloc(&la, (size_t)bx * by + 1, &tmp));
    CHECKED(DeviceAlloc(&lb, (size_t)bx * by + 1, &tmp));
    hipLaunchKernelGGL(luminance_1d_kernel, dim3(bx, by), dim3(64), 0, t->stream, (const float4*)t->film.accum, W, H, bx, by, la);
    uint32_t count = bx * by;
    while (count != 1) {
        const uint32_t groups = (count + 127) / 128;
        hipLaunchKernelGGL(luminance_single_kernel, dim3(groups), dim3(128), 0, t->stream, (const float*)la, count, lb);
        std::swap(la, lb);
        count = groups;
    }
    uchar4* dout = nullptr;
    CHECKED(DeviceAlloc(&dout, (size_t)W * H, &tmp));
    const uint32_t grid = std::max<uint32_t>(1u, std::min<uint32_t>((W * H + 255) / 256, kMaxPersistentBlocks));
    hipLaunchKernelGGL(postfx_kernel, dim3(grid), dim3(256), 0, t->stream, (const float4*)t->film.accum, W, H, prm->enabled,
                       prm->auto_exposure, prm->ev100, prm->luminance_white * prm->luminance_white, (const float*)la,
                       (const float*)dth, dout);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpyAsync(out, dout, (size_t)W * H * 4, hipMemcpyDeviceToHost, t->stream));
    if (outSumLogLum) HIPCHECK(hipMemcpyAsync(outSumLogLum, la, sizeof(float), hipMemcpyDeviceToHost, t->stream));
    HIPCHECK(hipStreamSynchronize(t->stream));
    return DCRT_OK;
}

DCRT_API int dcrt_device_math_eval(dcrt_tracer* t, int function, const float* x, uint32_t n, float* y)
{
    TRACER_GUARD(t);
    if ((!x || !y) && n) return DCRT_E_INVALID_ARG;
    std::vector<void*> tmp;
    float *dx = nullptr, *dy = nullptr;
    CHECKED(DeviceAlloc(&dx, n, &tmp));
    CHECKED(DeviceAlloc(&dy, n, &tmp));
    int rc = DCRT_OK;
    if (hipMemcpyAsync(dx, x, (size_t)n * 4, hipMemcpyHostToDevice, t->stream) != hipSuccess) rc = DCRT_E_HIP;
    if (rc == DCRT_OK && n) {
        hipLaunchKernelGGL(math_eval_kernel, dim3((n + 255) / 256), dim3(256), 0, t->stream, function, dx, n, dy);
        if (hipGetLastError() != hipSuccess) rc = DCRT_E_HIP;
    }
    if (rc == DCRT_OK && hipMemcpyAsync(y, dy, (size_t)n * 4, hipMemcpyDeviceToHost, t->stream) != hipSuccess) rc = DCRT_E_HIP;
    if (hipStreamSynchronize(t->stream) != hipSuccess) rc = DCRT_E_HIP;
    FreeAll(&tmp);
    return rc;
}

}  // extern "C"

#ifdef DCRT_WAVE_TIMELINE
// Diagnostic build only: copy the per-wave cast timeline (see kernels_impl.h).
extern "C" DCRT_API int dcrt_debug_wave_timeline(dcrt_tracer* t, unsigned long long* stamps, uint32_t* items)
{
    TRACER_GUARD(t);
    HIPCHECK(hipStreamSynchronize(t->stream));
    HIPCHECK(hipMemcpyFromSymbol(stamps, HIP_SYMBOL(g_waveLog), sizeof(g_waveLog)));
    HIPCHECK(hipMemcpyFromSymbol(items, HIP_SYMBOL(g_waveItems), sizeof(g_waveItems)));
    return DCRT_OK;
}
#endif

#ifdef DCRT_PHASE_CLOCKS
// Diagnostic build only: read and clear the cast kernels' per-phase wave cycles.
extern "C" DCRT_API int dcrt_debug_phase_clocks(dcrt_tracer* t, unsigned long long* out)
{
    TRACER_GUARD(t);
    HIPCHECK(hipStreamSynchronize(t->stream));
    HIPCHECK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phaseClk), sizeof(g_phaseClk)));
    const unsigned long long zero[24] = {};
    HIPCHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_phaseClk), zero, sizeof(zero)));
    return DCRT_OK;
}
#endif
