// bvh_accel.cpp -- BVHAccel restated (Source/BVHAccel.cpp:51-491).
//
// Binned SAH, 12 buckets on the max-extent centroid axis, depth-first node
// order (left child = node + 1, right child stored), 2..4-primitive ranges split
// at the median with MSVC's nth_element (a stable insertion sort for ranges of
// at most 32 elements), std::partition with the two-ended bidirectional scheme.
// With maxPrim = 2 (BLAS) / 1 (TLAS) every leaf holds exactly one primitive
// (SURVEY.md §8 a28). Large builds split their top levels across threads and splice
// the subtrees back in depth-first order: the output is bit-identical to the
// single-threaded reference build (parity mode).
#include "bvh_accel.h"

#include <algorithm>
#include <cstdlib>
#include <exception>
#include <stack>
#include <thread>

namespace dcrt {
namespace bvh {
namespace {

struct PrimInfo {
    BoundingBox box;
    uint32_t primIndex = 0;
    uint32_t bucketIndex = 0;
};

struct NodeInfo {
    int parentIndex;
    uint32_t primBegin;
    uint32_t primEnd;
    uint32_t depth;
};

// BVHAccel.cpp:67-74
float SurfaceArea(const BoundingBox& b)
{
    return 8.0f * (b.extents.x * b.extents.y + b.extents.x * b.extents.z + b.extents.y * b.extents.z);
}

// MSVC _Insertion_sort_unchecked: stable, strict-less predicate.
void InsertionSortByCenter(PrimInfo* first, PrimInfo* last, int axis)
{
    if (first == last) return;
    for (PrimInfo* mid = first + 1; mid != last; ++mid) {
        PrimInfo val = *mid;
        const float key = val.box.center[axis];
        if (key < first->box.center[axis]) {
            std::move_backward(first, mid, mid + 1);
            *first = val;
        } else {
            PrimInfo* hole = mid;
            for (PrimInfo* prev = hole - 1; key < prev->box.center[axis]; --prev) {
                *hole = *prev;
                hole = prev;
            }
            *hole = val;
        }
    }
}

// Two-ended std::partition for bidirectional iterators (MSVC and libstdc++ agree).
PrimInfo* PartitionByBucket(PrimInfo* first, PrimInfo* last, uint32_t split)
{
    for (;;) {
        for (;;) {
            if (first == last) return first;
            if (!(first->bucketIndex <= split)) break;
            ++first;
        }
        do {
            --last;
            if (first == last) return first;
        } while (!(last->bucketIndex <= split));
        std::swap(*first, *last);
        ++first;
    }
}

// The build's fixed inputs and outputs, shared by all subtree builders.
struct BuildContext {
    std::vector<PrimInfo>& infos;
    const uint32_t* primitives;            // index triples of a BLAS (nullptr for the TLAS)
    uint32_t maxPrim;
    uint32_t* reorderedPrimitives;
    uint32_t* reorderedPrimitiveIndices;
    uint32_t* leafDepths;
};

// A subtree's nodes in depth-first order with subtree-local child indices.
struct Subtree {
    std::vector<Node> nodes;
    uint32_t maxDepth = 0;
    uint32_t maxStackSize = 0;
};

// Leaves are emitted left to right over the primitive ranges, so a leaf's first
// reordered slot is its range begin: subtrees write disjoint slots.
void EmitLeaf(const BuildContext& c, Node* node, const NodeInfo& info, uint32_t count)
{
    for (uint32_t i = 0; i < count; ++i) {
        const uint32_t prim = c.infos[info.primBegin + i].primIndex;
        const uint32_t slot = info.primBegin + i;
        if (c.primitives) {
            c.reorderedPrimitives[slot * 3 + 0] = c.primitives[prim * 3 + 0];
            c.reorderedPrimitives[slot * 3 + 1] = c.primitives[prim * 3 + 1];
            c.reorderedPrimitives[slot * 3 + 2] = c.primitives[prim * 3 + 2];
        }
        c.reorderedPrimitiveIndices[slot] = prim;
    }
    node->childOrPrimIndex = info.primBegin;
    node->primCountOrInstance = count;
    node->isLeaf = true;
    if (c.leafDepths) c.leafDepths[info.primBegin] = info.depth;
}

// One node of BVHAccel.cpp:120-415 (BuildNodes): bounds, split axis, SAH or median
// split, or a leaf. Returns true (and the split point) when the node is interior.
bool ProcessNode(const BuildContext& c, const NodeInfo& cur, Node* node, uint32_t* primMiddle)
{
    std::vector<PrimInfo>& infos = c.infos;
    node->primCountOrInstance = 0;
    node->isLeaf = false;
    node->box = infos[cur.primBegin].box;
    for (uint32_t i = cur.primBegin + 1; i < cur.primEnd; ++i) node->box = BoxMerged(node->box, infos[i].box);

    const uint32_t count = cur.primEnd - cur.primBegin;
    *primMiddle = (cur.primBegin + cur.primEnd) / 2;
    if (count == 1) {
        EmitLeaf(c, node, cur, 1);
        return false;
    }
    Float3 cmin = infos[cur.primBegin].box.center, cmax = cmin;
    for (uint32_t i = cur.primBegin + 1; i < cur.primEnd; ++i) {
        cmax = VMax(cmax, infos[i].box.center);
        cmin = VMin(cmin, infos[i].box.center);
    }
    const BoundingBox centroidBox = BoxFromPoints(cmin, cmax);
    int axis = 0;
    {
        float mx = centroidBox.extents.x;
        if (centroidBox.extents.y > mx) { mx = centroidBox.extents.y; axis = 1; }
        if (centroidBox.extents.z > mx) axis = 2;
    }
    node->splitAxis = (uint8_t)axis;
    const float nodeArea = SurfaceArea(node->box);
    if (nodeArea == 0.0f || centroidBox.extents[axis] == 0.0f) {
        if (count < c.maxPrim) {
            EmitLeaf(c, node, cur, count);
            return false;
        }
        return true;   // split at the middle without sorting (BVHAccel.cpp:264-273)
    }
    if (count <= 4) {
        InsertionSortByCenter(&infos[cur.primBegin], &infos[cur.primBegin] + count, axis);
        return true;
    }
    constexpr uint32_t kBuckets = 12;
    struct Bucket { uint32_t count = 0; BoundingBox box{ { 0, 0, 0 }, { 0, 0, 0 } }; };
    Bucket buckets[kBuckets];
    for (uint32_t i = cur.primBegin; i < cur.primEnd; ++i) {
        const float mn = centroidBox.center[axis] - centroidBox.extents[axis];
        const float size = centroidBox.extents[axis] * 2.0f;
        const float f = (float)kBuckets * (infos[i].box.center[axis] - mn) / size;
        uint32_t n = f > 0.0f ? (uint32_t)f : 0u;
        if (n >= kBuckets) n = kBuckets - 1;
        infos[i].bucketIndex = n;
        if (buckets[n].count == 0) buckets[n].box = infos[i].box;
        else buckets[n].box = BoxMerged(buckets[n].box, infos[i].box);
        buckets[n].count++;
    }
    float cost[kBuckets - 1];
    for (uint32_t i = 0; i < kBuckets - 1; ++i) {
        uint32_t c0 = 0, c1 = 0;
        BoundingBox b0, b1;
        bool init0 = false, init1 = false;
        for (uint32_t j = 0; j <= i; ++j) {
            if (!buckets[j].count) continue;
            b0 = init0 ? BoxMerged(b0, buckets[j].box) : buckets[j].box;
            init0 = true;
            c0 += buckets[j].count;
        }
        for (uint32_t j = i + 1; j < kBuckets; ++j) {
            if (!buckets[j].count) continue;
            b1 = init1 ? BoxMerged(b1, buckets[j].box) : buckets[j].box;
            init1 = true;
            c1 += buckets[j].count;
        }
        cost[i] = 0.125f + ((float)c0 * SurfaceArea(b0) + (float)c1 * SurfaceArea(b1)) / nodeArea;
    }
    uint32_t minIndex = 0;
    for (uint32_t i = 1; i < kBuckets - 1; ++i)
        if (cost[i] < cost[minIndex]) minIndex = i;
    const float minCost = cost[minIndex];
    if (count > c.maxPrim || minCost < (float)count) {
        PrimInfo* base = infos.data();
        PrimInfo* p = PartitionByBucket(base + cur.primBegin, base + cur.primEnd, minIndex);
        *primMiddle = (uint32_t)(p - base);
        return true;
    }
    EmitLeaf(c, node, cur, count);
    return false;
}

// The reference's iterative depth-first loop over one subtree. `pending` = entries
// the reference's traversal-order stack already holds when it reaches this subtree's
// root (right siblings of left-side ancestors), so maxStackSize comes out the same.
void BuildSequential(const BuildContext& c, NodeInfo cur, uint32_t pending, Subtree* out)
{
    std::vector<Node>& nodes = out->nodes;
    std::stack<NodeInfo> stack;
    cur.parentIndex = -1;
    for (;;) {
        const uint32_t nodeIndex = (uint32_t)nodes.size();
        if (cur.parentIndex != -1) nodes[(size_t)cur.parentIndex].childOrPrimIndex = nodeIndex;
        nodes.emplace_back();
        uint32_t primMiddle = 0;
        if (!ProcessNode(c, cur, &nodes.back(), &primMiddle)) {
            if (stack.empty()) break;
            cur = stack.top();
            stack.pop();
            continue;
        }
        cur.depth++;
        stack.push({ (int)nodeIndex, primMiddle, cur.primEnd, cur.depth });
        cur.parentIndex = -1;
        cur.primEnd = primMiddle;
        out->maxDepth = std::max(out->maxDepth, cur.depth);
        out->maxStackSize = std::max(out->maxStackSize, pending + (uint32_t)stack.size());
    }
}

// Parallel parity build: the top `budget` levels split on the calling thread and
// hand the right subtree to a new thread; subtrees are spliced in depth-first order
// (node, left subtree, right subtree), which is exactly the sequential node order.
// Every node's own arithmetic stays sequential, so the result is bit-identical.
constexpr uint32_t kParallelMinPrims = 8192;

void BuildParallel(const BuildContext& c, NodeInfo cur, uint32_t pending, int budget, Subtree* out)
{
    if (budget <= 0 || cur.primEnd - cur.primBegin < kParallelMinPrims) {
        BuildSequential(c, cur, pending, out);
        return;
    }
    Node node;
    uint32_t primMiddle = 0;
    if (!ProcessNode(c, cur, &node, &primMiddle)) {
        out->nodes.push_back(node);
        return;
    }
    const uint32_t depth = cur.depth + 1;
    Subtree left, right;
    std::exception_ptr error;
    std::thread worker([&] {
        try {
            BuildParallel(c, { -1, primMiddle, cur.primEnd, depth }, pending, budget - 1, &right);
        } catch (...) {
            error = std::current_exception();
        }
    });
    try {
        BuildParallel(c, { -1, cur.primBegin, primMiddle, depth }, pending + 1, budget - 1, &left);
    } catch (...) {
        worker.join();
        throw;
    }
    worker.join();
    if (error) std::rethrow_exception(error);
    out->maxDepth = std::max({ depth, left.maxDepth, right.maxDepth });
    out->maxStackSize = std::max({ pending + 1, left.maxStackSize, right.maxStackSize });
    const uint32_t leftCount = (uint32_t)left.nodes.size();
    node.childOrPrimIndex = 1 + leftCount;
    out->nodes.reserve(1 + left.nodes.size() + right.nodes.size());
    out->nodes.push_back(node);
    for (Node n : left.nodes) {
        if (!n.isLeaf) n.childOrPrimIndex += 1;
        out->nodes.push_back(n);
    }
    for (Node n : right.nodes) {
        if (!n.isLeaf) n.childOrPrimIndex += 1 + leftCount;
        out->nodes.push_back(n);
    }
}

int BuildThreadBudget()
{
    unsigned threads = std::thread::hardware_concurrency();
    if (const char* e = std::getenv("DCRT_BUILD_THREADS")) threads = (unsigned)std::max(1, std::atoi(e));
    threads = std::min(threads ? threads : 1u, 16u);
    int budget = 0;
    while ((1u << budget) < threads) ++budget;
    return budget;
}

void BuildNodes(std::vector<PrimInfo>& infos, const uint32_t* primitives, NodeInfo root, uint32_t maxPrim,
                uint32_t* reorderedPrimitives, uint32_t* reorderedPrimitiveIndices, uint32_t* leafDepths,
                BuildResult* out)
{
    const BuildContext c{ infos, primitives, maxPrim, reorderedPrimitives, reorderedPrimitiveIndices, leafDepths };
    Subtree tree;
    BuildParallel(c, root, 0, BuildThreadBudget(), &tree);
    out->nodes = std::move(tree.nodes);
    out->maxDepth = tree.maxDepth;
    out->maxStackSize = tree.maxStackSize;
}

}  // namespace

void BuildBLAS(const dcrt_vertex* vertices, const uint32_t* indices, uint32_t triangleCount, uint32_t* reorderedIndices,
               uint32_t* reorderedTriangleIndices, BuildResult* out)
{
    std::vector<PrimInfo> infos(triangleCount);
    for (uint32_t i = 0; i < triangleCount; ++i) {
        const float* p0 = vertices[indices[i * 3 + 0]].position;
        const float* p1 = vertices[indices[i * 3 + 1]].position;
        const float* p2 = vertices[indices[i * 3 + 2]].position;
        const Float3 v0(p0[0], p0[1], p0[2]), v1(p1[0], p1[1], p1[2]), v2(p2[0], p2[1], p2[2]);
        // CalculateTriangleBoundingBox (BVHAccel.cpp:7-15)
        const Float3 mn = VMin(v2, VMin(v0, v1));
        const Float3 mx = VMax(v2, VMax(v0, v1));
        infos[i].box = BoxFromPoints(mn, mx);
        infos[i].primIndex = i;
    }
    out->nodes.clear();
    if (triangleCount == 0) return;
    BuildNodes(infos, indices, { -1, 0, triangleCount, 0 }, 2, reorderedIndices, reorderedTriangleIndices, nullptr, out);
}

void BuildTLAS(const Instance* instances, uint32_t instanceCount, uint32_t* reorderedInstanceIndices,
               uint32_t* instanceDepths, BuildResult* out)
{
    std::vector<PrimInfo> infos(instanceCount);
    for (uint32_t i = 0; i < instanceCount; ++i) {
        infos[i].box = BoxTransform(instances[i].box, instances[i].transform);
        infos[i].primIndex = i;
    }
    out->nodes.clear();
    if (instanceCount == 0) return;
    BuildNodes(infos, nullptr, { -1, 0, instanceCount, 0 }, 1, nullptr, reorderedInstanceIndices, instanceDepths, out);
}

void PackBVH(const Node* nodes, uint32_t nodeCount, bool isBLAS, dcrt_bvh_node* packed, uint32_t nodeIndexOffset,
             uint32_t primitiveIndexOffset)
{
    for (uint32_t i = 0; i < nodeCount; ++i) {
        const Node& n = nodes[i];
        dcrt_bvh_node& p = packed[i];
        const Float3 mn = n.box.center - n.box.extents;
        const Float3 mx = n.box.center + n.box.extents;
        p.bbox_min[0] = mn.x; p.bbox_min[1] = mn.y; p.bbox_min[2] = mn.z;
        p.bbox_max[0] = mx.x; p.bbox_max[1] = mx.y; p.bbox_max[2] = mx.z;
        p.right_child_or_prim_index = n.childOrPrimIndex;
        p.misc = (n.primCountOrInstance & DCRT_BVHNODE_MISC_MASK_PRIMITIVE_COUNT) << 3;
        p.misc |= n.splitAxis & 0x3u;
        if (!n.isLeaf) p.right_child_or_prim_index += nodeIndexOffset;
        else if (isBLAS) p.right_child_or_prim_index += primitiveIndexOffset;
        if (!isBLAS && n.isLeaf) p.misc |= 0x4u;
    }
}

}  // namespace bvh
}  // namespace dcrt
