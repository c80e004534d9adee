// bvh_accel.h -- binned-SAH BVH builder with the reference's exact node order
// and leaf rules (Source/BVHAccel.cpp:76-491, Source/BVHAccel.h:9-45).
#pragma once

#include <cstdint>
#include <vector>

#include "../../../include/dcrt.h"
#include "xmath.h"

namespace dcrt {
namespace bvh {

// BVHAccel::BVHNode (BVHAccel.h:12-27): childIndex/primIndex and
// primCount/instanceIndex share storage exactly as the reference's unions.
struct Node {
    BoundingBox box;
    uint32_t childOrPrimIndex = 0;   // right child (interior) or first primitive (leaf)
    uint32_t primCountOrInstance = 0;
    bool isLeaf = false;
    uint8_t splitAxis = 0;
};

struct Instance {
    BoundingBox box;      // BLAS root box
    Float4x4 transform;   // instance to world
};

struct BuildResult {
    std::vector<Node> nodes;
    uint32_t maxDepth = 0;
    uint32_t maxStackSize = 0;
};

// BVHAccel::BuildBLAS (BVHAccel.cpp:376-394): builds over triangles, writes the
// BVH-ordered index triples and the new->old triangle map.
void BuildBLAS(const dcrt_vertex* vertices, const uint32_t* indices, uint32_t triangleCount,
               uint32_t* reorderedIndices, uint32_t* reorderedTriangleIndices, BuildResult* out);

// BVHAccel::BuildTLAS (BVHAccel.cpp:396-411): instance boxes transformed to world.
void BuildTLAS(const Instance* instances, uint32_t instanceCount, uint32_t* reorderedInstanceIndices,
               uint32_t* instanceDepths, BuildResult* out);

// BVHAccel::PackBVH (BVHAccel.cpp:413-447).
void PackBVH(const Node* nodes, uint32_t nodeCount, bool isBLAS, dcrt_bvh_node* packed,
             uint32_t nodeIndexOffset = 0, uint32_t primitiveIndexOffset = 0);

}  // namespace bvh
}  // namespace dcrt
