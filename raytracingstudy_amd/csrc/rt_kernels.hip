// rt_kernels.hip — hand-written HIP kernels for gfx950 (MI355X, CDNA4).
//
// Replaces the reference's single CUDA kernel `raytracing`
// (src/renderer.cu:57-82, grid (W/32+1, H/32+1) x block (32,32)) and its
// <<<1,1>>> setup kernels (src/renderer.cu:84-109):
//   * compat_kernel : byte-exact restatement of `raytracing` (root-box slab
//                     test, R = Octree::traverse() = 200, miss colour).
//   * scene_kernel  : the build-defined octree path (DESIGN.md "Scene mode").
//   * unpack_kernel : scatters packed per-rank tiles into the frame.
// Compiled with -ffp-contract=off: every f32/f64 expression is evaluated in
// source order with IEEE division/sqrt, exactly like oracle/oracle.c.
#include <hip/hip_runtime.h>

#include "rt_params.h"

namespace rtamd {

__device__ __forceinline__ float sat(float x) { return x > 0.0f ? (x < 1.0f ? x : 1.0f) : 0.0f; }

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ float u01(uint32_t x) {
    return static_cast<float>(x >> 8) * (1.0f / 16777216.0f);
}

// include/camera.h:24-41 — Camera::getRay, camera passed by value.
__device__ __forceinline__ void get_ray(const CamArgs& c, float u, float v, float& wx, float& wy,
                                        float& wz) {
    const float dx = (u - c.K[2]) / c.K[0];
    const float dy = (v - c.K[5]) / c.K[4];
    const float dz = 1.0f;
    wx = c.R[0] * dx + c.R[3] * dy + c.R[6] * dz;
    wy = c.R[1] * dx + c.R[4] * dy + c.R[7] * dz;
    wz = c.R[2] * dx + c.R[5] * dy + c.R[8] * dz;
    const float len = sqrtf(wx * wx + wy * wy + wz * wz);
    wx /= len;
    wy /= len;
    wz /= len;
}

// src/renderer.cu:3-55 — `hit_sphere`: slab test of the root box [0,1.28]^3
// with the negative-direction axes mirrored about the centre 0.64 (f32
// origin/inverse widened to f64, f64 slab products rounded to f32, NaN-dropping
// fmaxf/fminf, no t >= 0 test).
__device__ __forceinline__ double mirror_o(float o, float d) {
    return d < 0.0f ? static_cast<double>(0.64f * 2.0f - o) : static_cast<double>(o);
}
__device__ __forceinline__ double mirror_inv(float d) {
    return d < 0.0f ? static_cast<double>(-(1.0f / d)) : static_cast<double>(1.0f / d);
}
__device__ __forceinline__ bool hit_root_box(const float o[3], float d0, float d1, float d2) {
    const double bmin = static_cast<double>(0.0f);
    const double bmax = static_cast<double>(1.28f);
    const double rx = mirror_o(o[0], d0), ry = mirror_o(o[1], d1), rz = mirror_o(o[2], d2);
    const double ix = mirror_inv(d0), iy = mirror_inv(d1), iz = mirror_inv(d2);
    const float tx0 = static_cast<float>((bmin - rx) * ix);
    const float tx1 = static_cast<float>((bmax - rx) * ix);
    const float ty0 = static_cast<float>((bmin - ry) * iy);
    const float ty1 = static_cast<float>((bmax - ry) * iy);
    const float tz0 = static_cast<float>((bmin - rz) * iz);
    const float tz1 = static_cast<float>((bmax - rz) * iz);
    return fmaxf(fmaxf(tx0, ty0), tz0) < fminf(fminf(tx1, ty1), tz1);
}

__device__ __forceinline__ uint32_t compat_pixel(const CamArgs& cam, uint32_t x, uint32_t y) {
    float d0, d1, d2;
    get_ray(cam, static_cast<float>(x), static_cast<float>(y), d0, d1, d2);
    if (hit_root_box(cam.o, d0, d1, d2)) return 0xFFFFFFFFu;
    const uint32_t g = static_cast<uint32_t>(sat(d1) * 255.0f);
    const uint32_t b = static_cast<uint32_t>(sat(d2) * 255.0f);
    return 200u | (g << 8) | (b << 16) | (255u << 24);
}

// One wave = 64 consecutive pixels of a row; one packed 32-bit store per lane.
__global__ void __launch_bounds__(kBlockThreads) compat_kernel(FrameArgs a) {
    const uint32_t x = blockIdx.x * 64u + (threadIdx.x & 63u);
    const uint32_t y = blockIdx.y * 4u + (threadIdx.x >> 6);
    if (x >= a.W || y >= a.H) return;
    __builtin_nontemporal_store(compat_pixel(a.cam, x, y), a.out8 + (size_t)y * a.W + x);
}

// Tile-packed compat: block = 64 x 4 strip of one tile.
__global__ void __launch_bounds__(kBlockThreads) compat_tiles_kernel(FrameArgs a) {
    const uint32_t ts = a.tile_size;
    const uint32_t strips = ts / 4u * (ts / 64u);
    const uint32_t k = blockIdx.x / strips;
    const uint32_t sidx = blockIdx.x % strips;
    const uint32_t lx = (sidx % (ts / 64u)) * 64u + (threadIdx.x & 63u);
    const uint32_t ly = (sidx / (ts / 64u)) * 4u + (threadIdx.x >> 6);
    const uint32_t tile = a.tiles[k];
    const uint32_t x = (tile % a.tiles_x) * ts + lx;
    const uint32_t y = (tile / a.tiles_x) * ts + ly;
    const uint32_t v = (x < a.W && y < a.H) ? compat_pixel(a.cam, x, y) : 0u;
    a.out8[(size_t)k * ts * ts + ly * ts + lx] = v;
}

// ---------------------------------------------------------------------------
// Scene mode
// ---------------------------------------------------------------------------

// Nearest root with the perpendicular-distance discriminant; tmin < t < tmax.
__device__ __forceinline__ bool isect(float o0, float o1, float o2, float d0, float d1, float d2,
                                      float4 sp, float tmin, float tmax, float& tout) {
    const float ocx = o0 - sp.x;
    const float ocy = o1 - sp.y;
    const float ocz = o2 - sp.z;
    const float b = ocx * d0 + ocy * d1 + ocz * d2;
    const float qx = ocx - b * d0;
    const float qy = ocy - b * d1;
    const float qz = ocz - b * d2;
    const float h = sp.w * sp.w - (qx * qx + qy * qy + qz * qz);
    if (h < 0.0f) return false;
    const float sq = sqrtf(h);
    float t = -b - sq;
    if (!(t > tmin)) t = -b + sq;
    if (!(t > tmin) || !(t < tmax)) return false;
    tout = t;
    return true;
}

// Grid-space octree walk (DESIGN.md "Octree walk"): mirrored origin so every
// direction component is >= 0 (the Revelles entry step of hit_sphere,
// src/renderer.cu:23-43), cell planes at integer grid coordinates, descend by
// mid-plane tests at the current t, leave a cell through its exit planes, and
// pop to the common ancestor found from the highest flipped coordinate bit.
// The per-thread ancestor stack lives in LDS, [depth-1][thread] (conflict-free).
template <bool kAnyHit>
__device__ __forceinline__ bool walk(const SceneArgs& S, float o0, float o1, float o2, float d0,
                                     float d1, float d2, float tmin, float tmax, float& tout,
                                     uint32_t& iout, uint32_t& n_nodes, uint32_t& n_prims,
                                     uint2* __restrict__ stk) {
    const uint32_t G = 1u << S.max_depth;
    const float o[3] = {o0, o1, o2};
    const float d[3] = {d0, d1, d2};
    float og[3], inv[3];
    uint32_t mask = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float g = (o[i] - S.rmin[i]) * S.scale[i];
        const bool neg = d[i] < 0.0f;
        float a = fabsf(d[i]);
        if (a < 1e-20f) a = 1e-20f;
        og[i] = neg ? S.G - g : g;
        inv[i] = 1.0f / (a * S.scale[i]);
        mask |= static_cast<uint32_t>(neg) << i;
    }
    auto plane = [&](int i, uint32_t k) { return (static_cast<float>(k) - og[i]) * inv[i]; };
    float t0 = plane(0, 0), t1 = plane(0, G);
#pragma unroll
    for (int i = 1; i < 3; ++i) {
        const float a0 = plane(i, 0), a1 = plane(i, G);
        if (a0 > t0) t0 = a0;
        if (a1 < t1) t1 = a1;
    }
    if (t0 < tmin) t0 = tmin;
    if (t1 > tmax) t1 = tmax;
    if (!(t0 < t1)) return false;

    float best_t = tmax;
    uint32_t best = kNoHit;
    n_nodes += 1;

    auto leaf = [&](uint32_t off, uint32_t cnt) -> bool {
        for (uint32_t j = 0; j < cnt; ++j) {
            const float4 sp = S.prim_sp[off + j];
            n_prims += 1;
            float th;
            if (isect(o0, o1, o2, d0, d1, d2, sp, tmin, tmax, th)) {
                if (kAnyHit) {
                    tout = th;
                    return true;
                }
                const uint32_t idx = S.prim_idx[off + j];
                if (th < best_t || (th == best_t && idx < best)) {
                    best_t = th;
                    best = idx;
                }
            }
        }
        return false;
    };

    if (S.root_is_leaf) {
        if (leaf(S.root.x, S.root.y)) return true;
    } else {
        uint2 node = S.root;
        uint32_t depth = 0, c0 = 0, c1 = 0, c2 = 0;
        float t = t0;
        // Hard cap (never reached by a correct walk: a ray crosses < 3*G cells
        // and each crossing costs at most one descent): no input can hang the GPU.
        for (uint32_t it = 0, cap = 8u * G + 64u; it < cap; ++it) {
            const uint32_t half = G >> (depth + 1);
            uint32_t bits = 0;
            if (plane(0, (2u * c0 + 1u) * half) <= t) bits |= 1u;
            if (plane(1, (2u * c1 + 1u) * half) <= t) bits |= 2u;
            if (plane(2, (2u * c2 + 1u) * half) <= t) bits |= 4u;
            const uint32_t child = bits ^ mask;
            c0 = 2u * c0 + (bits & 1u);
            c1 = 2u * c1 + ((bits >> 1) & 1u);
            c2 = 2u * c2 + (bits >> 2);
            depth += 1;
            const uint32_t valid = node.y & 0xFFu;
            if (valid & (1u << child)) {
                const uint32_t slot = node.x + __builtin_popcount(valid & ((1u << child) - 1u));
                const uint2 rec = S.nodes[slot];
                n_nodes += 1;
                if (!((node.y >> 8) & (1u << child))) {
                    node = rec;
                    stk[(depth - 1) * kBlockThreads] = rec;
                    continue;
                }
                if (leaf(rec.x, rec.y)) return true;
            }
            const uint32_t size = G >> depth;
            const float e0 = plane(0, (c0 + 1u) * size);
            const float e1 = plane(1, (c1 + 1u) * size);
            const float e2 = plane(2, (c2 + 1u) * size);
            float texit = e0 < e1 ? e0 : e1;
            texit = texit < e2 ? texit : e2;
            if (!kAnyHit && best_t < texit) break;
            if (texit >= t1) break;
            uint32_t diff = 0;
            const uint32_t lim = 1u << depth;
            bool out = false;
            if (e0 == texit) { diff |= c0 ^ (c0 + 1u); c0 += 1u; out |= c0 >= lim; }
            if (e1 == texit) { diff |= c1 ^ (c1 + 1u); c1 += 1u; out |= c1 >= lim; }
            if (e2 == texit) { diff |= c2 ^ (c2 + 1u); c2 += 1u; out |= c2 >= lim; }
            if (out) break;
            const uint32_t m = 32u - __builtin_clz(diff);
            depth -= m;
            c0 >>= m;
            c1 >>= m;
            c2 >>= m;
            node = depth ? stk[(depth - 1) * kBlockThreads] : S.root;
            t = texit;
        }
    }
    if (!kAnyHit && best != kNoHit) {
        tout = best_t;
        iout = best;
        return true;
    }
    return false;
}

struct PixelOut {
    float r, g, b;
};

__device__ __forceinline__ PixelOut scene_pixel(const FrameArgs& a, uint32_t x, uint32_t y,
                                                uint32_t& n_shadow, uint32_t& n_nodes,
                                                uint32_t& n_prims, uint2* stk) {
    const SceneArgs& S = a.sc;
    const uint32_t pid = y * a.W + x;
    const uint32_t hp = mix32(a.seedmix ^ pid);
    const float miss_r = 200.0f / 255.0f;
    float ar = 0.0f, ag = 0.0f, ab = 0.0f;
    for (uint32_t s = 0; s < a.spp; ++s) {
        float u = static_cast<float>(x), v = static_cast<float>(y);
        if (a.jitter) {
            u = u + u01(mix32(hp ^ (s << 1)));
            v = v + u01(mix32(hp ^ ((s << 1) | 1u)));
        }
        float d0, d1, d2;
        get_ray(a.cam, u, v, d0, d1, d2);
        float t;
        uint32_t idx;
        float cr, cg, cb;
        if (!walk<false>(S, a.cam.o[0], a.cam.o[1], a.cam.o[2], d0, d1, d2, 0.0f, INFINITY, t, idx,
                         n_nodes, n_prims, stk)) {
            cr = miss_r;
            cg = sat(d1);
            cb = sat(d2);
        } else {
            const float4 sp = S.spheres[idx];
            const float p0 = a.cam.o[0] + t * d0;
            const float p1 = a.cam.o[1] + t * d1;
            const float p2 = a.cam.o[2] + t * d2;
            const float ir = 1.0f / sp.w;
            const float n0 = (p0 - sp.x) * ir;
            const float n1 = (p1 - sp.y) * ir;
            const float n2 = (p2 - sp.z) * ir;
            const float ndl = n0 * a.L[0] + n1 * a.L[1] + n2 * a.L[2];
            float lam = ndl > 0.0f ? ndl : 0.0f;
            if (ndl > 0.0f && a.shadows) {
                const float s0 = p0 + n0 * kShadowEps;
                const float s1 = p1 + n1 * kShadowEps;
                const float s2 = p2 + n2 * kShadowEps;
                n_shadow += 1;
                float ts;
                uint32_t is;
                if (walk<true>(S, s0, s1, s2, a.L[0], a.L[1], a.L[2], 0.0f, INFINITY, ts, is,
                               n_nodes, n_prims, stk))
                    lam = 0.0f;
            }
            const float f = a.ambient + (1.0f - a.ambient) * lam;
            const uint32_t al = S.albedo[idx];
            cr = static_cast<float>(al & 0xFFu) * (1.0f / 255.0f) * f;
            cg = static_cast<float>((al >> 8) & 0xFFu) * (1.0f / 255.0f) * f;
            cb = static_cast<float>((al >> 16) & 0xFFu) * (1.0f / 255.0f) * f;
        }
        ar += cr;
        ag += cg;
        ab += cb;
    }
    return {ar * a.inv_spp, ag * a.inv_spp, ab * a.inv_spp};
}

__device__ __forceinline__ uint32_t pack_rgba8(const PixelOut& p) {
    const uint32_t r = static_cast<uint32_t>(sat(p.r) * 255.0f);
    const uint32_t g = static_cast<uint32_t>(sat(p.g) * 255.0f);
    const uint32_t b = static_cast<uint32_t>(sat(p.b) * 255.0f);
    return r | (g << 8) | (b << 16) | (255u << 24);
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ void flush_counters(const FrameArgs& a, uint32_t prim, uint32_t shadow,
                                               uint32_t nodes, uint32_t prims) {
    const unsigned long long s0 = wave_sum(prim);
    const unsigned long long s1 = wave_sum(shadow);
    const unsigned long long s2 = wave_sum(nodes);
    const unsigned long long s3 = wave_sum(prims);
    if ((threadIdx.x & 63u) == 0) {
        atomicAdd(a.counters + 0, s0);
        atomicAdd(a.counters + 1, s1);
        atomicAdd(a.counters + 2, s2);
        atomicAdd(a.counters + 3, s3);
    }
}

// 16x16 pixels per workgroup; wave w covers the 8x8 quadrant (w&1, w>>1),
// lane -> (lane&7, lane>>3), so one wave's rays are a compact screen block.
template <bool kTiles>
__global__ void __launch_bounds__(kBlockThreads) scene_kernel(FrameArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint2 lds_stack[];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t qx = (wave & 1u) * 8u + (lane & 7u);
    const uint32_t qy = (wave >> 1) * 8u + (lane >> 3);
    uint32_t x, y, k = 0, lx = 0, ly = 0;
    if (kTiles) {
        const uint32_t per = (a.tile_size / kTileSide) * (a.tile_size / kTileSide);
        k = blockIdx.x / per;
        const uint32_t sub = blockIdx.x % per;
        lx = (sub % (a.tile_size / kTileSide)) * kTileSide + qx;
        ly = (sub / (a.tile_size / kTileSide)) * kTileSide + qy;
        const uint32_t tile = a.tiles[k];
        x = (tile % a.tiles_x) * a.tile_size + lx;
        y = (tile / a.tiles_x) * a.tile_size + ly;
    } else {
        x = blockIdx.x * kTileSide + qx;
        y = blockIdx.y * kTileSide + qy;
    }
    uint32_t n_shadow = 0, n_nodes = 0, n_prims = 0, n_primary = 0;
    const bool inside = x < a.W && y < a.H;
    if (inside) {
        const PixelOut p = scene_pixel(a, x, y, n_shadow, n_nodes, n_prims, lds_stack + threadIdx.x);
        n_primary = a.spp;
        const uint32_t rgba = pack_rgba8(p);
        if (kTiles) {
            a.out8[(size_t)k * a.tile_size * a.tile_size + ly * a.tile_size + lx] = rgba;
        } else {
            a.out8[(size_t)y * a.W + x] = rgba;
            if (a.out32) a.out32[(size_t)y * a.W + x] = make_float4(p.r, p.g, p.b, 1.0f);
        }
    } else if (kTiles) {
        a.out8[(size_t)k * a.tile_size * a.tile_size + ly * a.tile_size + lx] = 0u;
    }
    flush_counters(a, n_primary, n_shadow, n_nodes, n_prims);
}

__global__ void __launch_bounds__(kBlockThreads)
    unpack_kernel(const uint32_t* __restrict__ packed, const uint32_t* __restrict__ tiles,
                  uint32_t n_tiles, uint32_t ts, uint32_t tiles_x, uint32_t W, uint32_t H,
                  uint32_t* __restrict__ img) {
    const size_t i = (size_t)blockIdx.x * kBlockThreads + threadIdx.x;
    const size_t per = (size_t)ts * ts;
    if (i >= per * n_tiles) return;
    const uint32_t k = static_cast<uint32_t>(i / per);
    const uint32_t r = static_cast<uint32_t>(i % per);
    const uint32_t tile = tiles[k];
    const uint32_t x = (tile % tiles_x) * ts + r % ts;
    const uint32_t y = (tile / tiles_x) * ts + r / ts;
    if (x < W && y < H) img[(size_t)y * W + x] = packed[i];
}

// ---------------------------------------------------------------------------
// launchers (called from rt_capi.cpp)
// ---------------------------------------------------------------------------

size_t scene_lds_bytes(uint32_t max_depth) {
    const uint32_t levels = max_depth > 1 ? max_depth - 1 : 1;
    return static_cast<size_t>(levels) * kBlockThreads * sizeof(uint2);
}

hipError_t launch_compat(const FrameArgs& a, hipStream_t st) {
    if (a.tiles) {
        const uint32_t strips = a.tile_size / 4u * (a.tile_size / 64u);
        hipLaunchKernelGGL(compat_tiles_kernel, dim3(a.n_tiles * strips), dim3(kBlockThreads), 0,
                           st, a);
    } else {
        hipLaunchKernelGGL(compat_kernel, dim3((a.W + 63) / 64, (a.H + 3) / 4), dim3(kBlockThreads),
                           0, st, a);
    }
    return hipGetLastError();
}

hipError_t launch_scene(const FrameArgs& a, hipStream_t st) {
    const size_t lds = scene_lds_bytes(a.sc.max_depth);
    if (a.tiles) {
        const uint32_t per = (a.tile_size / kTileSide) * (a.tile_size / kTileSide);
        hipLaunchKernelGGL(scene_kernel<true>, dim3(a.n_tiles * per), dim3(kBlockThreads), lds, st,
                           a);
    } else {
        hipLaunchKernelGGL(scene_kernel<false>,
                           dim3((a.W + kTileSide - 1) / kTileSide, (a.H + kTileSide - 1) / kTileSide),
                           dim3(kBlockThreads), lds, st, a);
    }
    return hipGetLastError();
}

hipError_t launch_unpack(const uint32_t* packed, const uint32_t* tiles, uint32_t n_tiles,
                         uint32_t ts, uint32_t tiles_x, uint32_t W, uint32_t H, uint32_t* img,
                         hipStream_t st) {
    const size_t total = (size_t)ts * ts * n_tiles;
    const uint32_t blocks = static_cast<uint32_t>((total + kBlockThreads - 1) / kBlockThreads);
    if (blocks) {
        hipLaunchKernelGGL(unpack_kernel, dim3(blocks), dim3(kBlockThreads), 0, st, packed, tiles,
                           n_tiles, ts, tiles_x, W, H, img);
    }
    return hipGetLastError();
}

}  // namespace rtamd
