// cell_table.hip — the depth-K cell table over the octree (DESIGN.md §5.1
// "Cell table").
//
// One uint2 entry per cell of the 2^K x 2^K x 2^K grid at depth K: the node
// that covers the cell, found by descending from the root —
//   * the internal node AT depth K whose cell it is,
//   * or the leaf at depth <= K that contains it,
//   * or "empty" with the depth of the empty child that contains it.
// Entry: x = the node record's x, y = record.y (24 bits) | depth << 24 |
// kind << 29 (kCell* in rt_params.h).  The walk uses it to get from an
// ancestor above depth K straight to the cell at depth K (one load instead of
// a chain of record reads); the tree itself is unchanged, so images and the
// oracle's node/sphere counters are too.
//
// K is chosen per tree: the area-weighted mean depth of the cells' covering
// nodes (a ray meets a cell of depth d in proportion to its cross-section,
// 4^-d, and a depth-d node covers 8^(Kmax-d) finest table cells), rounded.
// That is where ray walks leave one leaf for the next (C3: 5, C5: 6).
#include <hip/hip_runtime.h>

#include "octree_gpu.h"
#include "rt_params.h"

namespace rtamd {
namespace {

constexpr uint32_t kThreads = 256;
constexpr uint32_t kHistBins = kMaxDepth + 1;

// One thread per depth-K cell (real coordinates, x fastest).  `tab` may be
// null (histogram only); `hist` counts cells per covering depth.
__global__ void __launch_bounds__(kThreads)
    cell_table_kernel(const uint2* __restrict__ nodes, uint2 root, uint32_t K, uint32_t n_cells,
                      uint2* __restrict__ tab, unsigned long long* __restrict__ hist,
                      uint32_t* __restrict__ overflow) {
    __shared__ uint32_t h[kHistBins];
    if (threadIdx.x < kHistBins) h[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t idx = blockIdx.x * kThreads + threadIdx.x;
    if (idx < n_cells) {
        const uint32_t m = (1u << K) - 1u;
        const uint32_t c0 = idx & m, c1 = (idx >> K) & m, c2 = idx >> (2u * K);
        uint2 node = root, rec = root;
        uint32_t depth = 0, kind = kCellInternal;
        while (depth < K) {
            const uint32_t sh = K - depth - 1u;
            const uint32_t ch = ((c0 >> sh) & 1u) | (((c1 >> sh) & 1u) << 1) | (((c2 >> sh) & 1u) << 2);
            const uint32_t valid = node.y & 0xFFu;
            depth += 1;
            if (!(valid & (1u << ch))) {
                kind = kCellEmpty;
                rec = make_uint2(0u, 0u);
                break;
            }
            rec = nodes[node.x + __builtin_popcount(valid & ((1u << ch) - 1u))];
            if ((node.y >> 8) & (1u << ch)) {
                kind = kCellLeaf;
                break;
            }
            node = rec;
        }
        if (rec.y > kCellRecMask && kind != kCellEmpty) atomicOr(overflow, 1u);
        if (tab)
            tab[idx] = make_uint2(rec.x, (rec.y & kCellRecMask) | (depth << kCellDepthShift) |
                                             (kind << kCellKindShift));
        atomicAdd(&h[depth], 1u);
    }
    __syncthreads();
    if (threadIdx.x < kHistBins && h[threadIdx.x])
        atomicAdd(&hist[threadIdx.x], static_cast<unsigned long long>(h[threadIdx.x]));
}

}  // namespace

void CellTable::release() {
    if (tab_) (void)hipFree(tab_);
    if (scratch_) (void)hipFree(scratch_);
    tab_ = nullptr;
    scratch_ = nullptr;
    cap_ = 0;
    k_ = 0;
}

hipError_t CellTable::run(const uint2* nodes, uint2 root, uint32_t K, bool write, hipStream_t st,
                          unsigned long long* hist_host, uint32_t* overflow_host) {
    hipError_t e;
    if (!scratch_) {
        e = hipMalloc(reinterpret_cast<void**>(&scratch_), 32 * sizeof(unsigned long long));
        if (e != hipSuccess) return e;
    }
    const uint32_t n_cells = 1u << (3u * K);
    if (write && cap_ < n_cells) {
        if (tab_) (void)hipFree(tab_);
        tab_ = nullptr;
        cap_ = 0;
        e = hipMalloc(reinterpret_cast<void**>(&tab_), sizeof(uint2) * n_cells);
        if (e != hipSuccess) return e;
        cap_ = n_cells;
    }
    e = hipMemsetAsync(scratch_, 0, 32 * sizeof(unsigned long long), st);
    if (e != hipSuccess) return e;
    unsigned long long* hist = scratch_;
    uint32_t* overflow = reinterpret_cast<uint32_t*>(scratch_ + kHistBins);
    hipLaunchKernelGGL(cell_table_kernel, dim3((n_cells + kThreads - 1) / kThreads), dim3(kThreads),
                       0, st, nodes, root, K, n_cells, write ? tab_ : nullptr, hist, overflow);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    unsigned long long buf[kHistBins + 1];
    e = hipMemcpyAsync(buf, scratch_, sizeof(buf), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return e;
    for (uint32_t i = 0; i < kHistBins; ++i) hist_host[i] = buf[i];
    *overflow_host = static_cast<uint32_t>(buf[kHistBins] & 0xFFFFFFFFu);
    return hipSuccess;
}

hipError_t CellTable::build(const uint2* nodes, uint2 root, bool root_is_leaf, uint32_t max_depth,
                            uint32_t depth_reached, uint32_t k_req, hipStream_t st) {
    k_ = 0;
    if (root_is_leaf || k_req == kCellTableOff || max_depth == 0) return hipSuccess;
    uint32_t kmax = max_depth < kCellTableMaxK ? max_depth : kCellTableMaxK;
    if (depth_reached >= 1 && depth_reached < kmax) kmax = depth_reached;
    unsigned long long hist[kHistBins];
    uint32_t overflow = 0;
    uint32_t K;
    hipError_t e;
    if (k_req != kCellTableAuto) {
        K = k_req < kmax ? k_req : kmax;
    } else {
        // covering-depth histogram at kmax, weighted 2^d per finest cell
        if ((e = run(nodes, root, kmax, false, st, hist, &overflow)) != hipSuccess) return e;
        double num = 0.0, den = 0.0;
        for (uint32_t d = 0; d < kHistBins; ++d) {
            const double w = static_cast<double>(hist[d]) * static_cast<double>(1u << d);
            num += w * d;
            den += w;
        }
        const double mean = den > 0.0 ? num / den : 1.0;
        K = static_cast<uint32_t>(mean + 0.5);
        if (K < 1) K = 1;
        if (K > kmax) K = kmax;
    }
    if ((e = run(nodes, root, K, true, st, hist, &overflow)) != hipSuccess) return e;
    if (overflow) return hipSuccess;  // a leaf list too long for the packed entry: no table
    k_ = K;
    return hipSuccess;
}

}  // namespace rtamd
