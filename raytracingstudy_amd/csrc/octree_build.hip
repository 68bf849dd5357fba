// octree_build.hip — breadth-first octree build in HBM.
//
// One pass per depth over the current level, flat over sphere references
// (not one workgroup per cell), so the root level's n references and the
// deep levels' many small cells load the chip alike:
//
//   flags    one thread per reference of an internal cell tests the sphere
//            against the 8 children (the f64 overlap of scene_build.cpp) and
//            writes 8 flags at [8*off + child*cnt + pos]: parent-major,
//            child-major, list order;
//   scan     an exclusive scan of the flags (hipCUB) gives every surviving
//            (reference, child) its slot in the next level: child lists come
//            out contiguous, in next-level node order, ascending sphere index;
//   nodes    one thread per cell: child counts from the scan, valid/leaf masks;
//            a scan of (children, leaf refs, leaves) tuples assigns child
//            blocks and leaf list offsets in breadth-first order;
//   write    node records + the next level's cells;
//   scatter  references into the next level, or into the leaf lists.
//
// Every double operation is the host builder's, in the same order
// (-ffp-contract=off, IEEE f64 on CDNA4), so the tree is identical bit for
// bit: tests/test_gpu_build.py compares it with the host build and with the
// oracle's tree.  One 16-byte readback per level sizes the next one.
#include <hipcub/hipcub.hpp>

#include "octree_gpu.h"
#include "rt_params.h"

namespace rtamd {
namespace {

constexpr uint32_t kThreads = 256;

struct Geo {
    double lo[3], ext[3], margin;
    uint32_t depth;     // depth of the level being processed
    uint32_t max_depth, cap;
};

__device__ inline double plane(const Geo& g, int ax, uint32_t k, double cells) {
    return g.lo[ax] + g.ext[ax] * (static_cast<double>(k) / cells);
}

// scene_build.cpp Geometry::overlaps: squared distance from the centre to the
// closed box <= (r + margin)^2, accumulated x, y, z (adding +0.0 for an axis
// the centre lies within leaves the sum unchanged, as the host's skip does).
__device__ inline double axis_d2(double c, double lo, double hi) {
    double e = 0.0;
    if (c < lo) e = lo - c;
    else if (c > hi) e = c - hi;
    return e * e;
}

__device__ inline bool valid_sphere(float4 s) {
    return s.w > 0.0f && isfinite(s.x) && isfinite(s.y) && isfinite(s.z) && isfinite(s.w);
}

// ---- bounds ------------------------------------------------------------------
__global__ void __launch_bounds__(kThreads) bounds_partial(const float4* __restrict__ sp,
                                                           uint32_t n, double* __restrict__ part) {
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    double bad = 0.0;
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        const float4 s = sp[i];
        if (!valid_sphere(s)) {
            bad += 1.0;
            continue;
        }
        const double r = static_cast<double>(s.w);
        const double c[3] = {static_cast<double>(s.x), static_cast<double>(s.y),
                             static_cast<double>(s.z)};
        for (int a = 0; a < 3; ++a) {
            lo[a] = fmin(lo[a], c[a] - r);
            hi[a] = fmax(hi[a], c[a] + r);
        }
    }
    __shared__ double red[7][kThreads];
    for (int a = 0; a < 3; ++a) {
        red[a][threadIdx.x] = lo[a];
        red[3 + a][threadIdx.x] = hi[a];
    }
    red[6][threadIdx.x] = bad;
    __syncthreads();
    for (uint32_t w = kThreads / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            const uint32_t o = threadIdx.x + w;
            for (int a = 0; a < 3; ++a) {
                red[a][threadIdx.x] = fmin(red[a][threadIdx.x], red[a][o]);
                red[3 + a][threadIdx.x] = fmax(red[3 + a][threadIdx.x], red[3 + a][o]);
            }
            red[6][threadIdx.x] += red[6][o];
        }
        __syncthreads();
    }
    if (threadIdx.x < 7) part[blockIdx.x * 8 + threadIdx.x] = red[threadIdx.x][0];
}

__global__ void __launch_bounds__(kThreads) bounds_final(const double* __restrict__ part,
                                                         uint32_t nb, double* __restrict__ out) {
    // 7 independent reductions over nb partials, one wave each
    const uint32_t k = threadIdx.x / 64, lane = threadIdx.x % 64;
    for (uint32_t q = k; q < 7; q += kThreads / 64) {
        double v = q < 3 ? INFINITY : (q < 6 ? -INFINITY : 0.0);
        for (uint32_t b = lane; b < nb; b += 64) {
            const double x = part[b * 8 + q];
            v = q < 3 ? fmin(v, x) : (q < 6 ? fmax(v, x) : v + x);
        }
        for (int o = 32; o > 0; o >>= 1) {
            const double x = __shfl_xor(v, o);
            v = q < 3 ? fmin(v, x) : (q < 6 ? fmax(v, x) : v + x);
        }
        if (lane == 0) out[q] = v;
    }
}

// ---- root level ----------------------------------------------------------------
__global__ void root_flags(const float4* __restrict__ sp, uint32_t n, Geo g,
                           uint32_t* __restrict__ flags) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i > n) return;
    if (i == n) {
        flags[n] = 0;  // scan sentinel: pos[n] = number of root references
        return;
    }
    const float4 s = sp[i];
    const double c[3] = {static_cast<double>(s.x), static_cast<double>(s.y),
                         static_cast<double>(s.z)};
    double d2 = 0.0;
    for (int a = 0; a < 3; ++a) d2 += axis_d2(c[a], plane(g, a, 0u, 1.0), plane(g, a, 1u, 1.0));
    const double r = static_cast<double>(s.w) + g.margin;
    flags[i] = d2 <= r * r ? 1u : 0u;
}

__global__ void root_scatter(uint32_t n, const uint32_t* __restrict__ flags,
                             const uint32_t* __restrict__ pos, uint32_t* __restrict__ refs,
                             uint32_t* __restrict__ rpar, uint4* __restrict__ cell,
                             uint32_t* __restrict__ off) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i == 0) {
        cell[0] = make_uint4(0, 0, 0, pos[n]);
        off[0] = 0;
    }
    if (i < n && flags[i]) {
        refs[pos[i]] = i;
        rpar[pos[i]] = 0;
    }
}

// ---- one level -------------------------------------------------------------------
__device__ inline bool is_leaf(uint32_t cnt, uint32_t depth, const Geo& g) {
    return cnt <= g.cap || depth >= g.max_depth;
}

__global__ void __launch_bounds__(kThreads) level_flags(
    const float4* __restrict__ sp, const uint32_t* __restrict__ refs,
    const uint32_t* __restrict__ rpar, const uint4* __restrict__ cell,
    const uint32_t* __restrict__ off, uint32_t R, Geo g, uint32_t* __restrict__ flags) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j > R) return;
    if (j == R) {
        flags[8u * R] = 0;  // scan sentinel
        return;
    }
    const uint32_t p = rpar[j];
    const uint4 cl = cell[p];
    const uint32_t o = off[p], cnt = cl.w;
    uint32_t* f = flags + 8u * o + (j - o);
    if (is_leaf(cnt, g.depth, g)) {
        for (uint32_t ch = 0; ch < 8; ++ch) f[ch * cnt] = 0;
        return;
    }
    const float4 s = sp[refs[j]];
    const double c[3] = {static_cast<double>(s.x), static_cast<double>(s.y),
                         static_cast<double>(s.z)};
    const double cells = static_cast<double>(1u << (g.depth + 1));
    const uint32_t cc[3] = {cl.x, cl.y, cl.z};
    // squared axis distances to the lower (bit 0) and upper (bit 1) child slab
    double e[3][2];
    for (int a = 0; a < 3; ++a) {
        const double p0 = plane(g, a, 2u * cc[a], cells);
        const double p1 = plane(g, a, 2u * cc[a] + 1u, cells);
        const double p2 = plane(g, a, 2u * cc[a] + 2u, cells);
        e[a][0] = axis_d2(c[a], p0, p1);
        e[a][1] = axis_d2(c[a], p1, p2);
    }
    const double r = static_cast<double>(s.w) + g.margin;
    const double rr = r * r;
    for (uint32_t ch = 0; ch < 8; ++ch) {
        double d2 = 0.0;
        d2 += e[0][ch & 1u];
        d2 += e[1][(ch >> 1) & 1u];
        d2 += e[2][(ch >> 2) & 1u];
        f[ch * cnt] = d2 <= rr ? 1u : 0u;
    }
}

__global__ void __launch_bounds__(kThreads) level_nodes(
    const uint4* __restrict__ cell, const uint32_t* __restrict__ off,
    const uint32_t* __restrict__ pos, uint32_t M, Geo g, uint32_t* __restrict__ mask,
    uint4* __restrict__ tup) {
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= M) return;
    const uint32_t cnt = cell[p].w, o = off[p];
    if (is_leaf(cnt, g.depth, g)) {
        mask[p] = 0;
        tup[p] = make_uint4(0, cnt, 1, 0);
        return;
    }
    uint32_t valid = 0, leafm = 0;
    const uint32_t* q = pos + 8u * o;
    uint32_t a = q[0];
    for (uint32_t ch = 0; ch < 8; ++ch) {
        const uint32_t b = q[(ch + 1) * cnt];
        const uint32_t k = b - a;
        if (k) {
            valid |= 1u << ch;
            if (is_leaf(k, g.depth + 1, g)) leafm |= 1u << ch;
        }
        a = b;
    }
    mask[p] = valid | (leafm << 8);
    tup[p] = make_uint4(__popc(valid), 0, 0, 0);
}

struct Add4 {
    __host__ __device__ uint4 operator()(const uint4& a, const uint4& b) const {
        return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
};

// totals of the level: x = next-level cells, y = leaf references, z = leaves,
// w = next-level references
__global__ void level_totals(const uint4* __restrict__ tin, const uint4* __restrict__ tex,
                             uint32_t M, const uint32_t* __restrict__ pos, uint32_t R,
                             uint4* __restrict__ tot) {
    const uint4 a = tin[M - 1], b = tex[M - 1];
    *tot = make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, pos[8u * R]);
}

__global__ void __launch_bounds__(kThreads) level_write(
    const uint4* __restrict__ cell, const uint32_t* __restrict__ off,
    const uint32_t* __restrict__ pos, const uint32_t* __restrict__ mask,
    const uint4* __restrict__ tex, uint32_t M, uint32_t level_start, uint32_t next_start,
    uint32_t prim_base, Geo g, uint2* __restrict__ nodes, uint4* __restrict__ ncell,
    uint32_t* __restrict__ noff) {
    const uint32_t p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= M) return;
    const uint4 cl = cell[p];
    const uint32_t cnt = cl.w, o = off[p];
    const uint4 ex = tex[p];
    if (is_leaf(cnt, g.depth, g)) {
        nodes[level_start + p] = make_uint2(prim_base + ex.y, cnt);
        return;
    }
    const uint32_t m = mask[p];
    nodes[level_start + p] = make_uint2(next_start + ex.x, m);
    const uint32_t* q = pos + 8u * o;
    uint32_t k = ex.x;
    for (uint32_t ch = 0; ch < 8; ++ch) {
        if (!(m & (1u << ch))) continue;
        const uint32_t a = q[ch * cnt], b = q[(ch + 1) * cnt];
        ncell[k] = make_uint4(2u * cl.x + (ch & 1u), 2u * cl.y + ((ch >> 1) & 1u),
                              2u * cl.z + ((ch >> 2) & 1u), b - a);
        noff[k] = a;
        ++k;
    }
}

__global__ void __launch_bounds__(kThreads) level_scatter(
    const uint32_t* __restrict__ refs, const uint32_t* __restrict__ rpar,
    const uint4* __restrict__ cell, const uint32_t* __restrict__ off,
    const uint32_t* __restrict__ flags, const uint32_t* __restrict__ pos,
    const uint32_t* __restrict__ mask, const uint4* __restrict__ tex, uint32_t R,
    uint32_t prim_base, Geo g, uint32_t* __restrict__ prim_idx, uint32_t* __restrict__ nrefs,
    uint32_t* __restrict__ nrpar) {
    const uint32_t j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= R) return;
    const uint32_t p = rpar[j];
    const uint32_t cnt = cell[p].w, o = off[p], at = j - o;
    const uint32_t id = refs[j];
    if (is_leaf(cnt, g.depth, g)) {
        prim_idx[prim_base + tex[p].y + at] = id;
        return;
    }
    const uint32_t m = mask[p] & 0xFFu;
    uint32_t k = tex[p].x;
    const uint32_t base = 8u * o + at;
    for (uint32_t ch = 0; ch < 8; ++ch) {
        if (!(m & (1u << ch))) continue;
        const uint32_t x = base + ch * cnt;
        if (flags[x]) {
            nrefs[pos[x]] = id;
            nrpar[pos[x]] = k;
        }
        ++k;
    }
}

__global__ void gather_prims(const float4* __restrict__ sp, const uint32_t* __restrict__ idx,
                             uint32_t n, float4* __restrict__ out) {
    const uint32_t i = blockIdx.x * kThreads + threadIdx.x;
    if (i < n) out[i] = sp[idx[i]];
}

inline uint32_t blocks_for(uint64_t n) { return static_cast<uint32_t>((n + kThreads - 1) / kThreads); }

}  // namespace

#define RT_TRY(x)                              \
    do {                                       \
        hipError_t e_ = (x);                   \
        if (e_ != hipSuccess) return e_;       \
    } while (0)

template <typename T>
hipError_t GpuOctreeBuilder::reserve(Buf<T>& b, size_t n, size_t keep, hipStream_t st) {
    if (n <= b.cap && b.p) return hipSuccess;
    size_t cap = b.cap ? b.cap : 256;
    while (cap < n) cap += cap / 2 + 256;
    T* p = nullptr;
    RT_TRY(hipMalloc(reinterpret_cast<void**>(&p), cap * sizeof(T)));
    if (keep && b.p) {
        hipError_t e = hipMemcpyAsync(p, b.p, keep * sizeof(T), hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) {
            (void)hipFree(p);
            return e;
        }
    }
    if (b.p) RT_TRY(hipFree(b.p));
    b.p = p;
    b.cap = cap;
    return hipSuccess;
}

void GpuOctreeBuilder::release() {
    auto fr = [](auto& b) {
        if (b.p) (void)hipFree(b.p);
        b.p = nullptr;
        b.cap = 0;
    };
    fr(nodes_b_), fr(prim_sp_b_), fr(prim_idx_b_);
    for (int i = 0; i < 2; ++i) fr(cell_[i]), fr(off_[i]), fr(refs_[i]), fr(rpar_[i]);
    fr(mask_), fr(tup_in_), fr(tup_ex_), fr(flags_), fr(pos_), fr(temp_), fr(partial_),
        fr(totals_);
    if (totals_host_) (void)hipHostFree(totals_host_);
    totals_host_ = nullptr;
    nodes_ = nullptr;
    prim_sp_ = nullptr;
    prim_idx_ = nullptr;
}

// exclusive sum of flags_[0..n) into pos_ (n includes the zero sentinel)
hipError_t GpuOctreeBuilder::scan_flags(uint32_t n, hipStream_t st) {
    size_t bytes = 0;
    RT_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, flags_.p, pos_.p, n, st));
    RT_TRY(reserve(temp_, bytes, 0, st));
    return hipcub::DeviceScan::ExclusiveSum(temp_.p, bytes, flags_.p, pos_.p, n, st);
}

hipError_t GpuOctreeBuilder::bounds(const float4* sp, uint32_t n, hipStream_t st,
                                    SphereBounds* out) {
    const uint32_t nb = n ? std::min<uint32_t>(blocks_for(n), 1024u) : 1u;
    RT_TRY(reserve(partial_, nb * 8 + 8, 0, st));
    if (!totals_host_) RT_TRY(hipHostMalloc(reinterpret_cast<void**>(&totals_host_), 64));
    hipLaunchKernelGGL(bounds_partial, dim3(nb), dim3(kThreads), 0, st, sp, n, partial_.p);
    RT_TRY(hipGetLastError());
    hipLaunchKernelGGL(bounds_final, dim3(1), dim3(kThreads), 0, st, partial_.p, nb,
                       partial_.p + nb * 8);
    RT_TRY(hipGetLastError());
    double* h = reinterpret_cast<double*>(totals_host_);
    RT_TRY(hipMemcpyAsync(h, partial_.p + nb * 8, 7 * sizeof(double), hipMemcpyDeviceToHost, st));
    RT_TRY(hipStreamSynchronize(st));
    for (int a = 0; a < 3; ++a) {
        out->lo[a] = h[a];
        out->hi[a] = h[3 + a];
    }
    out->n_invalid = static_cast<uint32_t>(h[6]);
    return hipSuccess;
}

hipError_t GpuOctreeBuilder::build(const float4* sp, uint32_t n, const float cfg_min[3],
                                   const float cfg_max[3], uint32_t max_depth, uint32_t leaf_cap,
                                   hipStream_t st, GpuBuildResult* res) {
    *res = GpuBuildResult();
    SphereBounds sb;
    RT_TRY(bounds(sp, n, st, &sb));
    res->n_invalid = sb.n_invalid;
    if (sb.n_invalid) return hipSuccess;  // the caller refuses the scene

    // effective root box: scene_build.cpp build_octree, same double expressions
    double um = 0.0;
    for (int a = 0; a < 3; ++a)
        um = std::max(um, static_cast<double>(cfg_max[a]) - static_cast<double>(cfg_min[a]));
    Geo g;
    double m = 0.0;
    for (int a = 0; a < 3; ++a) {
        const double lo = std::min(static_cast<double>(cfg_min[a]), sb.lo[a]);
        const double hi = std::max(static_cast<double>(cfg_max[a]), sb.hi[a]);
        res->rmin[a] = lo < static_cast<double>(cfg_min[a]) ? static_cast<float>(lo - 1e-6 * um)
                                                            : cfg_min[a];
        res->rmax[a] = hi > static_cast<double>(cfg_max[a]) ? static_cast<float>(hi + 1e-6 * um)
                                                            : cfg_max[a];
        g.lo[a] = static_cast<double>(res->rmin[a]);
        g.ext[a] = static_cast<double>(res->rmax[a]) - static_cast<double>(res->rmin[a]);
        m = std::max(m, g.ext[a]);
    }
    g.margin = 1e-6 * m;
    g.max_depth = max_depth;
    g.cap = leaf_cap;
    g.depth = 0;

    // root level: the spheres overlapping the root box (all of them, as it is
    // grown to enclose every sphere; tested anyway, as the host does)
    RT_TRY(reserve(flags_, size_t(n) + 1, 0, st));
    RT_TRY(reserve(pos_, size_t(n) + 1, 0, st));
    RT_TRY(reserve(refs_[0], std::max<size_t>(n, 1), 0, st));
    RT_TRY(reserve(rpar_[0], std::max<size_t>(n, 1), 0, st));
    RT_TRY(reserve(cell_[0], 1, 0, st));
    RT_TRY(reserve(off_[0], 1, 0, st));
    RT_TRY(reserve(totals_, 4, 0, st));
    hipLaunchKernelGGL(root_flags, dim3(blocks_for(size_t(n) + 1)), dim3(kThreads), 0, st, sp, n,
                       g, flags_.p);
    RT_TRY(hipGetLastError());
    RT_TRY(scan_flags(n + 1, st));
    hipLaunchKernelGGL(root_scatter, dim3(blocks_for(std::max<uint32_t>(n, 1))), dim3(kThreads), 0,
                       st, n, flags_.p, pos_.p, refs_[0].p, rpar_[0].p, cell_[0].p, off_[0].p);
    RT_TRY(hipGetLastError());
    RT_TRY(hipMemcpyAsync(totals_host_, pos_.p + n, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    RT_TRY(hipStreamSynchronize(st));
    uint32_t R = totals_host_->x;  // root references
    res->root_is_leaf = R <= leaf_cap || max_depth == 0;
    uint32_t M = 1;                // cells in the level
    uint32_t level_start = 0, next_start = 1, prim_total = 0;
    RT_TRY(reserve(nodes_b_, std::max<size_t>(1024, n / 2), 0, st));
    RT_TRY(reserve(prim_idx_b_, std::max<size_t>(1024, size_t(n) * 2), 0, st));
    int cur = 0;
    for (uint32_t depth = 0; M > 0; ++depth) {
        g.depth = depth;
        if (uint64_t(R) * 8u + 1u >= (uint64_t(1) << 32)) {  // 8 flag slots per reference
            res->ref_overflow = R;
            return hipErrorInvalidValue;
        }
        const uint32_t nf = 8u * R + 1u;
        RT_TRY(reserve(flags_, nf, 0, st));
        RT_TRY(reserve(pos_, nf, 0, st));
        RT_TRY(reserve(mask_, M, 0, st));
        RT_TRY(reserve(tup_in_, M, 0, st));
        RT_TRY(reserve(tup_ex_, M, 0, st));
        hipLaunchKernelGGL(level_flags, dim3(blocks_for(size_t(R) + 1)), dim3(kThreads), 0, st, sp,
                           refs_[cur].p, rpar_[cur].p, cell_[cur].p, off_[cur].p, R, g, flags_.p);
        RT_TRY(hipGetLastError());
        RT_TRY(scan_flags(nf, st));
        hipLaunchKernelGGL(level_nodes, dim3(blocks_for(M)), dim3(kThreads), 0, st, cell_[cur].p,
                           off_[cur].p, pos_.p, M, g, mask_.p, tup_in_.p);
        RT_TRY(hipGetLastError());
        {
            size_t bytes = 0;
            RT_TRY(hipcub::DeviceScan::ExclusiveScan(nullptr, bytes, tup_in_.p, tup_ex_.p, Add4(),
                                                     make_uint4(0, 0, 0, 0), M, st));
            RT_TRY(reserve(temp_, bytes, 0, st));
            RT_TRY(hipcub::DeviceScan::ExclusiveScan(temp_.p, bytes, tup_in_.p, tup_ex_.p, Add4(),
                                                     make_uint4(0, 0, 0, 0), M, st));
        }
        hipLaunchKernelGGL(level_totals, dim3(1), dim3(1), 0, st, tup_in_.p, tup_ex_.p, M, pos_.p,
                           R, totals_.p);
        RT_TRY(hipGetLastError());
        RT_TRY(hipMemcpyAsync(totals_host_, totals_.p, sizeof(uint4), hipMemcpyDeviceToHost, st));
        RT_TRY(hipStreamSynchronize(st));
        const uint4 t = *totals_host_;  // x next cells, y leaf refs, z leaves, w next refs
        // node slots and leaf-list offsets are 32-bit record fields: refuse
        // (the caller then builds on the host, which refuses the same way)
        // rather than wrap
        if (uint64_t(prim_total) + t.y + kPrimPad >= (uint64_t(1) << 32) ||
            uint64_t(next_start) + t.x >= (uint64_t(1) << 32)) {
            res->ref_overflow = uint64_t(prim_total) + t.y;
            return hipErrorInvalidValue;
        }
        const int nxt = cur ^ 1;
        RT_TRY(reserve(nodes_b_, size_t(next_start) + t.x, next_start, st));
        RT_TRY(reserve(prim_idx_b_, size_t(prim_total) + t.y + 1, prim_total, st));
        RT_TRY(reserve(cell_[nxt], std::max<uint32_t>(t.x, 1), 0, st));
        RT_TRY(reserve(off_[nxt], std::max<uint32_t>(t.x, 1), 0, st));
        RT_TRY(reserve(refs_[nxt], std::max<uint32_t>(t.w, 1), 0, st));
        RT_TRY(reserve(rpar_[nxt], std::max<uint32_t>(t.w, 1), 0, st));
        hipLaunchKernelGGL(level_write, dim3(blocks_for(M)), dim3(kThreads), 0, st, cell_[cur].p,
                           off_[cur].p, pos_.p, mask_.p, tup_ex_.p, M, level_start, next_start,
                           prim_total, g, nodes_b_.p, cell_[nxt].p, off_[nxt].p);
        RT_TRY(hipGetLastError());
        if (R) {
            hipLaunchKernelGGL(level_scatter, dim3(blocks_for(R)), dim3(kThreads), 0, st,
                               refs_[cur].p, rpar_[cur].p, cell_[cur].p, off_[cur].p, flags_.p,
                               pos_.p, mask_.p, tup_ex_.p, R, prim_total, g, prim_idx_b_.p,
                               refs_[nxt].p, rpar_[nxt].p);
            RT_TRY(hipGetLastError());
        }
        res->n_leaves += t.z;
        if (t.z) res->depth_reached = depth;
        prim_total += t.y;
        level_start = next_start;
        next_start += t.x;
        M = t.x;
        R = t.w;
        cur = nxt;
    }
    // + kPrimPad: the scalar leaf path may read up to 3 spheres past a leaf's end
    RT_TRY(reserve(prim_sp_b_, size_t(prim_total) + kPrimPad, 0, st));
    if (prim_total) {
        hipLaunchKernelGGL(gather_prims, dim3(blocks_for(prim_total)), dim3(kThreads), 0, st, sp,
                           prim_idx_b_.p, prim_total, prim_sp_b_.p);
        RT_TRY(hipGetLastError());
    }
    RT_TRY(hipMemcpyAsync(totals_host_, nodes_b_.p, sizeof(uint2), hipMemcpyDeviceToHost, st));
    RT_TRY(hipStreamSynchronize(st));
    const uint2 root = *reinterpret_cast<const uint2*>(totals_host_);
    res->root = root;
    res->n_nodes = next_start;
    res->n_prims = prim_total;
    nodes_ = nodes_b_.p;
    prim_idx_ = prim_idx_b_.p;
    prim_sp_ = prim_sp_b_.p;
    return hipSuccess;
}

}  // namespace rtamd
