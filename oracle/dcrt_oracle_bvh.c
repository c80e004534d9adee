/* TEST INFRASTRUCTURE (oracle) -- never part of the product, never measured.
 *
 * An independent C restatement of the reference's BVH build -- BVHAccel::BuildNodes /
 * BuildBLAS / BuildTLAS / PackBVH (Source/BVHAccel.cpp:7-30,76-447) -- written against
 * the reference source, not against the product's csrc/host/bvh_accel.cpp, so the
 * product's node order, boxes, reordered triangles, depth and stack size are checked
 * against a second derivation (tests/test_bvh_pin.py, and the GPU parity tests render
 * against the BVH this file builds).
 *
 * Semantics reproduced:
 *  - DirectX::BoundingBox is center/extents. CreateFromPoints / CreateMerged form
 *    (min + max) * 0.5 and (max - min) * 0.5 from SSE minps / maxps (a < b ? a : b,
 *    a > b ? a : b); BoundingBox::Transform runs the 8 corners ext * offset + center
 *    (no FMA: the reference builds without /arch:AVX2) through XMVector3Transform
 *    (((z * r2 + r3) + y * r1) + x * r0) and re-boxes them.
 *  - std::nth_element on the <= 4 primitives that reach it (BVHAccel.cpp:232-236) is
 *    MSVC's: for ranges of at most 32 (_ISORT_MAX) it is one insertion sort with the
 *    "new earliest element moves to the front" shortcut (Appendix A.8).
 *  - std::partition is the two-ended swap loop (MSVC and libstdc++ agree).
 *  - float -> uint32 conversions of the bucket index go through a 64-bit truncation,
 *    as x86-64 code generation for `uint32_t(float)` does.
 *  - the value-initialised node of emplace_back(): axis 0, count 0, not a leaf.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "dcrt_oracle.h"

typedef struct { float c[3], e[3]; } xbox;          /* DirectX::BoundingBox        */
typedef struct { xbox box; uint32_t prim, bucket; } xprim;   /* SPrimitiveInfo   */
typedef struct { int parent; uint32_t begin, end, depth; } xjob;   /* BVHNodeInfo   */

static float sse_min(float a, float b) { return a < b ? a : b; }
static float sse_max(float a, float b) { return a > b ? a : b; }

/* BoundingBox::CreateFromPoints(out, p1, p2) */
static xbox box_of_points(const float* p1, const float* p2)
{
    xbox b;
    for (int k = 0; k < 3; ++k) {
        const float lo = sse_min(p1[k], p2[k]), hi = sse_max(p1[k], p2[k]);
        b.c[k] = (lo + hi) * 0.5f;
        b.e[k] = (hi - lo) * 0.5f;
    }
    return b;
}

/* BoundingBox::CreateMerged(out, a, b) */
static xbox box_union(const xbox* a, const xbox* b)
{
    float lo[3], hi[3];
    for (int k = 0; k < 3; ++k) {
        lo[k] = sse_min(a->c[k] - a->e[k], b->c[k] - b->e[k]);
        hi[k] = sse_max(a->c[k] + a->e[k], b->c[k] + b->e[k]);
    }
    xbox r;
    for (int k = 0; k < 3; ++k) {
        r.c[k] = (lo[k] + hi[k]) * 0.5f;
        r.e[k] = (hi[k] - lo[k]) * 0.5f;
    }
    return r;
}

/* BoundingBoxSurfaceArea (BVHAccel.cpp:23-30) */
static float box_area(const xbox* b)
{
    return 8.f * (b->e[0] * b->e[1] + b->e[0] * b->e[2] + b->e[1] * b->e[2]);
}

/* BoundingBox::Transform by XMLoadFloat4x3(m): rows r0..r3 of 3, w column (0,0,0,1) */
static xbox box_transformed(const xbox* b, const float* m12)
{
    static const float corner_sign[8][3] = { { -1, -1, 1 }, { 1, -1, 1 }, { 1, 1, 1 }, { -1, 1, 1 },
                                             { -1, -1, -1 }, { 1, -1, -1 }, { 1, 1, -1 }, { -1, 1, -1 } };
    float lo[3] = { 0, 0, 0 }, hi[3] = { 0, 0, 0 };
    for (int i = 0; i < 8; ++i) {
        float p[3], q[3];
        for (int k = 0; k < 3; ++k) p[k] = b->e[k] * corner_sign[i][k] + b->c[k];
        for (int k = 0; k < 3; ++k) {
            float t = p[2] * m12[2 * 3 + k] + m12[3 * 3 + k];
            t = p[1] * m12[1 * 3 + k] + t;
            q[k] = p[0] * m12[0 * 3 + k] + t;
        }
        for (int k = 0; k < 3; ++k) {
            if (i == 0) { lo[k] = q[k]; hi[k] = q[k]; }
            else { lo[k] = sse_min(lo[k], q[k]); hi[k] = sse_max(hi[k], q[k]); }
        }
    }
    xbox r;
    for (int k = 0; k < 3; ++k) {
        r.c[k] = (lo[k] + hi[k]) * 0.5f;
        r.e[k] = (hi[k] - lo[k]) * 0.5f;
    }
    return r;
}

/* MSVC _Insertion_sort_unchecked on center[axis] with operator< */
static void msvc_insertion_sort(xprim* a, uint32_t n, int axis)
{
    for (uint32_t mid = 1; mid < n; ++mid) {
        const xprim v = a[mid];
        if (v.box.c[axis] < a[0].box.c[axis]) {
            memmove(a + 1, a, sizeof(xprim) * mid);
            a[0] = v;
        } else {
            uint32_t hole = mid;
            while (v.box.c[axis] < a[hole - 1].box.c[axis]) { a[hole] = a[hole - 1]; --hole; }
            a[hole] = v;
        }
    }
}

/* std::partition(first, last, bucket <= split): index of the first "false" element */
static uint32_t two_ended_partition(xprim* a, uint32_t first, uint32_t last, uint32_t split)
{
    for (;;) {
        for (;;) {
            if (first == last) return first;
            if (!(a[first].bucket <= split)) break;
            ++first;
        }
        do {
            --last;
            if (first == last) return first;
        } while (!(a[last].bucket <= split));
        const xprim t = a[first]; a[first] = a[last]; a[last] = t;
        ++first;
    }
}

/* float -> uint32 as x86-64 converts it (cvttss2si through a 64-bit register) */
static uint32_t to_u32(float f)
{
    if (!(f > -9.2e18f && f < 9.2e18f)) return 0u;
    return (uint32_t)(int64_t)f;
}

typedef struct {
    oracle_bvh_node* nodes; uint32_t count;
    xjob* stack; uint32_t depth_of_stack, stack_cap;
    uint32_t placed;            /* reorderedPrimitiveCount */
} xbuild;

static void push_job(xbuild* b, xjob j)
{
    if (b->depth_of_stack == b->stack_cap) {
        b->stack_cap = b->stack_cap ? b->stack_cap * 2 : 64;
        b->stack = (xjob*)realloc(b->stack, sizeof(xjob) * b->stack_cap);
    }
    b->stack[b->depth_of_stack++] = j;
}

/* BuildNodes<...> (BVHAccel.cpp:76-371). triangles: 3 indices per primitive or NULL. */
static void build_nodes(xprim* prims, uint32_t prim_count, uint32_t max_in_leaf, const uint32_t* triangles,
                        uint32_t* out_triangles, uint32_t* out_prim_order, oracle_bvh_node* nodes, uint32_t* node_count,
                        uint32_t* max_depth, uint32_t* max_stack, uint32_t* leaf_depths)
{
    xbuild b;
    memset(&b, 0, sizeof(b));
    b.nodes = nodes;
    xjob cur = { -1, 0, prim_count, 0 };
    for (;;) {
        const uint32_t self = b.count;
        if (cur.parent != -1) b.nodes[cur.parent].child_or_prim = self;
        oracle_bvh_node* node = &b.nodes[b.count++];
        memset(node, 0, sizeof(*node));
        xbox box = prims[cur.begin].box;
        for (uint32_t i = cur.begin + 1; i < cur.end; ++i) box = box_union(&box, &prims[i].box);
        memcpy(node->center, box.c, sizeof(box.c));
        memcpy(node->extents, box.e, sizeof(box.e));
        const uint32_t n = cur.end - cur.begin;
        int make_leaf = n == 1;
        uint32_t mid = (cur.begin + cur.end) / 2;
        int halve = 0;
        if (!make_leaf) {
            float cmin[3], cmax[3];
            memcpy(cmin, prims[cur.begin].box.c, sizeof(cmin));
            memcpy(cmax, cmin, sizeof(cmax));
            for (uint32_t i = cur.begin + 1; i < cur.end; ++i)
                for (int k = 0; k < 3; ++k) {
                    cmax[k] = sse_max(cmax[k], prims[i].box.c[k]);
                    cmin[k] = sse_min(cmin[k], prims[i].box.c[k]);
                }
            const xbox cbox = box_of_points(cmin, cmax);
            int axis = 0;
            float widest = cbox.e[0];
            if (cbox.e[1] > widest) { widest = cbox.e[1]; axis = 1; }
            if (cbox.e[2] > widest) axis = 2;
            node->split_axis = (uint32_t)axis;
            const float area = box_area(&box);
            if (area == 0.f || cbox.e[axis] == 0.f) {
                /* all degenerate or coincident centroids (BVHAccel.cpp:186-230) */
                if (n < max_in_leaf) make_leaf = 1;
                else halve = 1;
            } else if (n <= 4) {
                msvc_insertion_sort(prims + cur.begin, n, axis);   /* nth_element */
            } else {
                uint32_t bucket_n[12] = { 0 };
                xbox bucket_box[12];
                memset(bucket_box, 0, sizeof(bucket_box));
                for (uint32_t i = cur.begin; i < cur.end; ++i) {
                    const float lo = cbox.c[axis] - cbox.e[axis];
                    const float size = cbox.e[axis] * 2.0f;
                    uint32_t k = to_u32((float)12 * (prims[i].box.c[axis] - lo) / size);
                    if (k >= 12) k = 11;
                    prims[i].bucket = k;
                    bucket_box[k] = bucket_n[k] == 0 ? prims[i].box : box_union(&bucket_box[k], &prims[i].box);
                    bucket_n[k]++;
                }
                float cost[11];
                for (int s = 0; s < 11; ++s) {
                    uint32_t n0 = 0, n1 = 0;
                    xbox b0 = { { 0, 0, 0 }, { 1, 1, 1 } }, b1 = { { 0, 0, 0 }, { 1, 1, 1 } };   /* BoundingBox() */
                    int have0 = 0, have1 = 0;
                    for (int j = 0; j <= s; ++j)
                        if (bucket_n[j]) {
                            b0 = have0 ? box_union(&b0, &bucket_box[j]) : bucket_box[j];
                            have0 = 1;
                            n0 += bucket_n[j];
                        }
                    for (int j = s + 1; j < 12; ++j)
                        if (bucket_n[j]) {
                            b1 = have1 ? box_union(&b1, &bucket_box[j]) : bucket_box[j];
                            have1 = 1;
                            n1 += bucket_n[j];
                        }
                    cost[s] = .125f + ((float)n0 * box_area(&b0) + (float)n1 * box_area(&b1)) / area;
                }
                uint32_t best = 0;
                for (uint32_t s = 1; s < 11; ++s)
                    if (cost[s] < cost[best]) best = s;
                if (n > max_in_leaf || cost[best] < (float)n) {
                    mid = two_ended_partition(prims, cur.begin, cur.end, best);
                } else {
                    make_leaf = 1;   /* unreachable for the reference's leaf sizes */
                }
            }
        }
        if (make_leaf) {
            for (uint32_t i = 0; i < n; ++i) {
                const uint32_t p = prims[cur.begin + i].prim;
                if (triangles)
                    for (int k = 0; k < 3; ++k) out_triangles[(b.placed + i) * 3 + k] = triangles[p * 3 + k];
                out_prim_order[b.placed + i] = p;
            }
            node->child_or_prim = b.placed;
            node->count_or_instance = n;
            node->is_leaf = 1;
            if (leaf_depths) leaf_depths[b.placed] = cur.depth;
            b.placed += n;
            if (b.depth_of_stack == 0) break;
            cur = b.stack[--b.depth_of_stack];
            continue;
        }
        (void)halve;
        cur.depth++;
        push_job(&b, (xjob){ (int)self, mid, cur.end, cur.depth });
        cur.parent = -1;
        cur.end = mid;
        if (cur.depth > *max_depth) *max_depth = cur.depth;
        if (b.depth_of_stack > *max_stack) *max_stack = b.depth_of_stack;
    }
    free(b.stack);
    *node_count = b.count;
}

int oracle_bvh_build_blas(const dcrt_vertex* vertices, const uint32_t* indices, uint32_t tri_count, oracle_bvh_node* nodes,
                          uint32_t* node_count, uint32_t* reordered_indices, uint32_t* tri_order, uint32_t* max_depth,
                          uint32_t* max_stack)
{
    if (!tri_count) return -1;
    xprim* prims = (xprim*)malloc(sizeof(xprim) * tri_count);
    for (uint32_t t = 0; t < tri_count; ++t) {
        const float* p0 = vertices[indices[t * 3]].position;
        const float* p1 = vertices[indices[t * 3 + 1]].position;
        const float* p2 = vertices[indices[t * 3 + 2]].position;
        float lo[3], hi[3];
        for (int k = 0; k < 3; ++k) {
            lo[k] = sse_min(p2[k], sse_min(p0[k], p1[k]));
            hi[k] = sse_max(p2[k], sse_max(p0[k], p1[k]));
        }
        prims[t].box = box_of_points(lo, hi);
        prims[t].prim = t;
        prims[t].bucket = 0;
    }
    *max_depth = 0;
    *max_stack = 0;
    build_nodes(prims, tri_count, 2, indices, reordered_indices, tri_order, nodes, node_count, max_depth, max_stack, NULL);
    free(prims);
    return 0;
}

int oracle_bvh_build_tlas(const float* blas_root_boxes, const float* transforms, uint32_t instance_count, oracle_bvh_node* nodes,
                          uint32_t* node_count, uint32_t* instance_order, uint32_t* max_depth, uint32_t* max_stack,
                          uint32_t* instance_depths)
{
    if (!instance_count) return -1;
    xprim* prims = (xprim*)malloc(sizeof(xprim) * instance_count);
    for (uint32_t i = 0; i < instance_count; ++i) {
        xbox b;
        memcpy(b.c, blas_root_boxes + i * 6, sizeof(b.c));
        memcpy(b.e, blas_root_boxes + i * 6 + 3, sizeof(b.e));
        prims[i].box = box_transformed(&b, transforms + i * 12);
        prims[i].prim = i;
        prims[i].bucket = 0;
    }
    *max_depth = 0;
    *max_stack = 0;
    build_nodes(prims, instance_count, 1, NULL, NULL, instance_order, nodes, node_count, max_depth, max_stack,
                instance_depths);
    free(prims);
    return 0;
}

/* PackBVH (BVHAccel.cpp:413-447) */
void oracle_bvh_pack(const oracle_bvh_node* nodes, uint32_t count, int is_blas, dcrt_bvh_node* out, uint32_t node_offset,
                     uint32_t prim_offset)
{
    for (uint32_t i = 0; i < count; ++i) {
        const oracle_bvh_node* u = &nodes[i];
        dcrt_bvh_node* p = &out[i];
        for (int k = 0; k < 3; ++k) {
            p->bbox_min[k] = u->center[k] - u->extents[k];
            p->bbox_max[k] = u->center[k] + u->extents[k];
        }
        p->right_child_or_prim_index = u->child_or_prim;
        p->misc = (u->count_or_instance & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT) << 3;
        p->misc |= u->split_axis & 0x3u;
        if (!u->is_leaf) p->right_child_or_prim_index += node_offset;
        else if (is_blas) p->right_child_or_prim_index += prim_offset;
        if (!is_blas && u->is_leaf) p->misc |= 0x4u;
    }
}
