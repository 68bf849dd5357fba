// octree_gpu.h — device octree builder.
//
// Builds, in HBM, exactly the tree the host builder (scene_build.cpp) and the
// oracle define (DESIGN.md "Octree build"): same effective root box, same
// breadth-first node records, same ascending leaf lists, bit for bit.  The
// reference's intended entry is setOctree(min, max, res)
// (include/renderer.cuh:35, src/renderer.cu:134-138), which has no builder.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtamd {

struct GpuBuildResult {
    uint32_t n_nodes = 0, n_prims = 0, n_leaves = 0, depth_reached = 0;
    uint32_t n_invalid = 0;  // spheres with r <= 0 or a non-finite value (build refused)
    uint64_t ref_overflow = 0;  // references of the level that exceeded the 32-bit slots (refused)
    float rmin[3] = {0, 0, 0}, rmax[3] = {0, 0, 0};
    uint2 root = {0, 0};
    bool root_is_leaf = true;
};

// Per-sphere bounds of a sphere list: min(c - r), max(c + r) per axis in
// double, and the number of invalid spheres.  `out` is 6 doubles + 1 count.
struct SphereBounds {
    double lo[3], hi[3];
    uint32_t n_invalid;
};

class GpuOctreeBuilder {
public:
    GpuOctreeBuilder() = default;
    GpuOctreeBuilder(const GpuOctreeBuilder&) = delete;
    GpuOctreeBuilder& operator=(const GpuOctreeBuilder&) = delete;
    ~GpuOctreeBuilder() { release(); }

    // Reduce a device sphere list (4 floats per sphere) to its bounds; syncs `st`.
    hipError_t bounds(const float4* spheres, uint32_t n, hipStream_t st, SphereBounds* out);
    // Build the octree of `spheres` (device) over the configured box grown to
    // enclose every sphere.  Outputs stay in this object's buffers (nodes(),
    // prim_sp(), prim_idx()); syncs `st` once per level.
    hipError_t build(const float4* spheres, uint32_t n, const float cfg_min[3],
                     const float cfg_max[3], uint32_t max_depth, uint32_t leaf_cap,
                     hipStream_t st, GpuBuildResult* res);
    void release();

    const uint2* nodes() const { return nodes_; }
    const float4* prim_sp() const { return prim_sp_; }
    const uint32_t* prim_idx() const { return prim_idx_; }

private:
    template <typename T>
    struct Buf {
        T* p = nullptr;
        size_t cap = 0;
    };
    template <typename T>
    hipError_t reserve(Buf<T>& b, size_t n, size_t keep, hipStream_t st);
    hipError_t scan_flags(uint32_t n, hipStream_t st);

    uint2* nodes_ = nullptr;
    float4* prim_sp_ = nullptr;
    uint32_t* prim_idx_ = nullptr;
    Buf<uint2> nodes_b_;
    Buf<float4> prim_sp_b_;
    Buf<uint32_t> prim_idx_b_;
    // level scratch: cells (x, y, z, count), ref offsets, child masks, tuples
    Buf<uint4> cell_[2];
    Buf<uint32_t> off_[2];
    Buf<uint32_t> refs_[2], rpar_[2];
    Buf<uint32_t> mask_;
    Buf<uint4> tup_in_, tup_ex_;
    Buf<uint32_t> flags_, pos_;
    Buf<unsigned char> temp_;
    Buf<double> partial_;
    Buf<uint4> totals_;
    uint4* totals_host_ = nullptr;
};

// Depth-K cell table over a built octree (cell_table.hip): one uint2 entry per
// depth-K cell naming the node that covers it, so a walk can reach depth K in
// one load.  k_req: kCellTableAuto (choose K from the tree), kCellTableOff, or
// a depth (clamped to the tree).  k() == 0 means no table (root leaf, or a
// leaf list longer than the packed entry holds).
class CellTable {
public:
    CellTable() = default;
    CellTable(const CellTable&) = delete;
    CellTable& operator=(const CellTable&) = delete;
    ~CellTable() { release(); }
    hipError_t build(const uint2* nodes, uint2 root, bool root_is_leaf, uint32_t max_depth,
                     uint32_t depth_reached, uint32_t k_req, hipStream_t st);
    void release();
    const uint2* table() const { return k_ ? tab_ : nullptr; }
    uint32_t k() const { return k_; }

private:
    hipError_t run(const uint2* nodes, uint2 root, uint32_t K, bool write, hipStream_t st,
                   unsigned long long* hist_host, uint32_t* overflow_host);
    uint2* tab_ = nullptr;
    size_t cap_ = 0;
    unsigned long long* scratch_ = nullptr;
    uint32_t k_ = 0;
};

}  // namespace rtamd
