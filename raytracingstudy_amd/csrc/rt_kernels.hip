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

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <utility>
#include <vector>

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

// getRay under ONE CANDIDATE contraction of include/camera.h:31-34 (dz = 1
// folds; an fadd of two products fused through its first operand), a guess at
// what nvcc's default -fmad=true does to the reference binary.  Which order
// that binary really uses cannot be checked without nvcc: unpinned
// (DESIGN.md 2.1).  The default (get_ray) is the SOURCE semantics.  Same
// operations as the oracle's contracted getRay, contract = 1.
__device__ __forceinline__ void get_ray_fma(const CamArgs& c, float u, float v, float& wx,
                                            float& wy, float& wz) {
    const float dx = (u - c.K[2]) / c.K[0];
    const float dy = (v - c.K[5]) / c.K[4];
    wx = fmaf(c.R[0], dx, c.R[3] * dy) + c.R[6];
    wy = fmaf(c.R[1], dx, c.R[4] * dy) + c.R[7];
    wz = fmaf(c.R[2], dx, c.R[5] * dy) + c.R[8];
    const float len = sqrtf(fmaf(wz, wz, fmaf(wx, wx, wy * wy)));
    wx /= len;
    wy /= len;
    wz /= len;
}

__device__ __forceinline__ uint32_t compat_pixel(const CamArgs& cam, uint32_t x, uint32_t y,
                                                 uint32_t contract) {
    float d0, d1, d2;
    if (contract)
        get_ray_fma(cam, static_cast<float>(x), static_cast<float>(y), d0, d1, d2);
    else
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
    __builtin_nontemporal_store(compat_pixel(a.cam, x, y, a.contract), a.out8 + (size_t)y * a.W + x);
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
    const uint32_t v = (x < a.W && y < a.H) ? compat_pixel(a.cam, x, y, a.contract) : 0u;
    a.out8[(size_t)k * ts * ts + ly * ts + lx] = v;
}

// ---------------------------------------------------------------------------
// Scene mode
// ---------------------------------------------------------------------------

#ifdef RT_BLOCK_STATS
// Diagnostic build: the first active lane counts one execution of block i by
// the wave, and the active lanes (BlockStat, rt_params.h).
__device__ __forceinline__ void bs_count(uint32_t* bs, uint32_t i) {
    const uint64_t m = __ballot(1);
    if (__lane_id() == static_cast<uint32_t>(__builtin_ctzll(m))) {
        bs[2 * i] += 1u;
        bs[2 * i + 1] += static_cast<uint32_t>(__popcll(m));
    }
}
#define RT_BS(i) bs_count(bs, (i))
#else
#define RT_BS(i) ((void)0)
#endif

// Nearest root with the perpendicular-distance discriminant, explicit FMAs
// (13 VALU to the h < 0 test); accepted iff tmin < t < tmax.  Same operations
// as oracle.c:isect.  isect_oc takes o - c already formed (in the same f32
// operations: the camera-relative records hold it), isect forms it.
__device__ __forceinline__ bool isect_oc(float ocx, float ocy, float ocz, float d0, float d1,
                                         float d2, float r, float tmin, float tmax, float& tout,
                                         uint32_t* bs = nullptr) {
    const float b = fmaf(ocz, d2, fmaf(ocy, d1, ocx * d0));
    const float qx = fmaf(-b, d0, ocx);
    const float qy = fmaf(-b, d1, ocy);
    const float qz = fmaf(-b, d2, ocz);
    const float qq = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
    const float h = fmaf(r, r, -qq);
    if (h < 0.0f) return false;
    RT_BS(kBsSqrt);
    const float sq = sqrtf(h);
    float t = -b - sq;
    if (!(t > tmin)) t = -b + sq;
    if (!(t > tmin) || !(t < tmax)) return false;
    tout = t;
    return true;
}
__device__ __forceinline__ bool isect(float o0, float o1, float o2, float d0, float d1, float d2,
                                      float4 sp, float tmin, float tmax, float& tout,
                                      uint32_t* bs = nullptr) {
    const float ocx = o0 - sp.x;
    const float ocy = o1 - sp.y;
    const float ocz = o2 - sp.z;
    return isect_oc(ocx, ocy, ocz, d0, d1, d2, sp.w, tmin, tmax, tout, bs);
}

// v_readlane of a float's bits (the builtin is int-typed: a float argument
// would be converted to an integer value)
__device__ __forceinline__ float readlane_f(float x, uint32_t lane) {
    return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(x), lane));
}

// isect's discriminant h alone (same operations): h < 0 <=> isect rejects
// the sphere before its square root.
__device__ __forceinline__ float isect_h_oc(float ocx, float ocy, float ocz, float d0, float d1,
                                            float d2, float r) {
    const float b = fmaf(ocz, d2, fmaf(ocy, d1, ocx * d0));
    const float qx = fmaf(-b, d0, ocx);
    const float qy = fmaf(-b, d1, ocy);
    const float qz = fmaf(-b, d2, ocz);
    const float qq = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
    return fmaf(r, r, -qq);
}
__device__ __forceinline__ float isect_h(float o0, float o1, float o2, float d0, float d1,
                                         float d2, float4 sp) {
    const float ocx = o0 - sp.x;
    const float ocy = o1 - sp.y;
    const float ocz = o2 - sp.z;
    return isect_h_oc(ocx, ocy, ocz, d0, d1, d2, sp.w);
}

// Camera-relative records (SceneArgs::prim_cam): 0 off; 1 =
// {o - c, C'} with the slack screen fma(b, b, -C') >= 0 and the exact tests
// reloading the chunk's spheres; 2 = {o - c, r}, the exact discriminant from
// the stored o - c (isect's own operations, 10 VALU: no slack, no reload)
#ifndef RT_CAM_MODE
#define RT_CAM_MODE 1
#endif
constexpr int kCamMode = RT_CAM_MODE;

// The kernel's FrameArgs as memory (the kernarg segment, scalar-cached),
// behind an opaque pointer: a field read through it is a fresh s_load at that
// point instead of a value kept live in an SGPR across the walk (the register
// allocator would spill it into VGPR lanes: v_writelane / v_readlane, VALU
// work per pixel).  Used for the per-sample camera, shading and output fields.
typedef __attribute__((address_space(4))) const FrameArgs KernArgs;
__device__ __forceinline__ KernArgs* kernargs() {
    KernArgs* p = (KernArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return p;
}

// An incomplete frame (FrameArgs::qerr): this frame's id into the renderer's
// pinned host word, a plain system-scope store (no atomic over the host
// link), visible to the host without a copy.  Called by a wave's lead lane.
__device__ __forceinline__ void frame_failed() {
    KernArgs* ka = kernargs();
    __hip_atomic_store(ka->qerr, ka->frame_id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

constexpr uint32_t kSortMaxRounds = 4;  // up to 256 samples per pixel
constexpr uint32_t kSortMax = 64u * kSortMaxRounds;
// per wave: per sample a slot {t, sphere} -> {lam | miss g, albedo | miss b}
// and a kind byte; the tracing order and the list of lit samples (u8 each)
constexpr uint32_t kSortCellBits = 3;  // jitter cells per axis: 2^3 (8 x 8, Morton order)
constexpr uint32_t kSortCells = 1u << (2u * kSortCellBits);
constexpr uint32_t kSortWaveBytes = kSortMax * 8u + 3u * kSortMax + kSortCells * 4u;
static_assert(kSortWaveBytes % 16u == 0u, "per-wave regions stay float4-aligned");

// rank of this lane among the lanes set in m
__device__ __forceinline__ uint32_t lane_rank(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}

// LDS leaf staging (RT_LDS_LEAF): a per-wave buffer of
// kLeafBuf spheres after the rest of the workgroup's LDS (pixel sums and
// stacks, or the sorted path's stacks and per-wave regions).
#ifndef RT_LDS_LEAF
#define RT_LDS_LEAF 1
#endif
// Leaves of fewer spheres read them directly: staging adds an LDS round trip
// to the first chunk, which a leaf of one or two chunks does not win back.
// Measured (profiles/r05/ldsmin_ab.log, 3 alternating rounds, against no
// staging): from 1 / 4 / 6 / 8 spheres C3 +1.0 / -0.7 / -1.7 / +0.2%, C5
// -6.9 / -7.8 / -7.8 / -5.3%, C5d +4.0 / +2.5 / +2.3 / +2.5%.  Round 6, with
// shadow walks no longer staging (kLdsShadow), against 6: from 2 / 3 / 4 / 5
// spheres C3 +0.2 / -0.4 / -0.5 / -1.0%, C5 -0.8 / -1.1 / -1.2 / -1.3%, C5d
// +1.0 / +0.5 / +0.3 / +0.1%, 8: C3 +3.5%, C5 +4.6%
// (profiles/r06/ab_r6_lmin2_lmin3_lmin4_lmin5.log, ab_r6_lmin4_lmin8.log).
#ifndef RT_LDS_MIN
#define RT_LDS_MIN 5
#endif
constexpr uint32_t kLdsLeafMin = RT_LDS_MIN;
// Only nearest-hit (primary) walks stage their leaves: a shadow ray may stop
// at a leaf's first chunk, after a staging load fetched all of the leaf's
// lines, and its chunked reads stop with it.  Against staging shadow leaves
// too (RT_LDS_SHADOW=1, A/B): C5d -1.3%, C5 -0.5%, C3 -0.1%
// (profiles/r06/ab_ctr3_noshst_sbo.log, 3 alternating rounds).
#ifndef RT_LDS_SHADOW
#define RT_LDS_SHADOW 0
#endif
constexpr bool kLdsShadow = RT_LDS_SHADOW != 0;
// Shading by leaf reference (SceneArgs::prim_al): a nearest walk's `iout` is
// the hit's reference, and shading reads prim_sp[ref] / prim_al[ref]; 0 keeps
// the sphere index (prim_idx[ref]) and the by-index spheres / albedo arrays.
// Measured (profiles/r06/ab_ref_shade.log, 3 alternating rounds): C3 -0.7%,
// C5 -0.5%, C5d -0.2%, C2 0; L2 misses C3 -7.5%, C5d -11.5% (pmc_l2_*.json)
#ifndef RT_REF_SHADE
#define RT_REF_SHADE 1
#endif
// Light-plane records in 8 bytes (SceneArgs::prim_shd8): a shadow chunk's two
// spheres in ONE dwordx4 (the texture path charges a load by instruction,
// not by bytes: 16 cycles for a dwordx2 or a dwordx4), screened against the
// scene's largest radius term.  C3 -2.0%, C5 -2.4%, C2 -2.8%, C5d -0.1%; the
// looser radius sends 2% (C3, C5) to 6% (C5d) more shadow chunks down the
// exact path (profiles/r06/ab_shd8.log, bstats_shd8.log).  0: 16-byte records
#ifndef RT_SHD8
#define RT_SHD8 1
#endif
// Image-plane screen for primary rays in 8 bytes (SceneArgs::prim_cam8,
// DESIGN.md 5.1 round 6): the primary walks screen a chunk's two spheres
// from ONE dwordx4 instead of two 16-byte camera-relative records, and stage
// no leaves in LDS.  C3 -2.9%, C5 -2.4%, C5d -2.1%, C2 -1.9% (unsorted and
// sorted walks, profiles/r06/ab_cam8_sorted.log); RT_CAM8=0: the 16-byte
// camera-relative screen and its LDS staging
#ifndef RT_CAM8
#define RT_CAM8 1
#endif
// ... LDS staging of the 8-byte records, pairs per float4, from
// kLdsLeafMin8 spheres: C3 +1.2 / +1.3 / +3.4% from 8 / 5 / 3 against none
// (ab_cam8_staging.log), so off
#ifndef RT_CAM8_LDS
#define RT_CAM8_LDS 0
#endif
// ... for the sorted walks (C5, C5d) too
#ifndef RT_CAM8_SORTED
#define RT_CAM8_SORTED 1
#endif
#ifndef RT_CAM8_LDS_MIN
#define RT_CAM8_LDS_MIN 5
#endif
constexpr uint32_t kLdsLeafMin8 = RT_CAM8_LDS_MIN;
// ... each sphere's own rr' as bf16 in the records' low bytes (RT_SHD8_PER)
// instead of the scene's largest
#ifndef RT_SHD8_PER
#define RT_SHD8_PER 0
#endif
// spheres per chunk of the shadow walks (with 8-byte records: two per dwordx4);
// 4 spills 48-100 B and runs C3 +6%, C5 +8%, C5d +5% (profiles/r06/ab_shd_chunk4.log)
#ifndef RT_SHD_CHUNK
#define RT_SHD_CHUNK 2
#endif
constexpr size_t kLeafBufBytes = RT_LDS_LEAF ? (kBlockThreads / 64u) * kLeafBuf * sizeof(float4) : 0u;

// Ancestor-stack levels per thread: depths 1..D-1, or K..D-1 with a cell table
// (a pop above depth K jumps through the table instead).
// Per-thread ancestor-stack levels.  Internal nodes sit at depths <
// stack_depth (the deepest leaf), and with a cell table only depths >= K are
// pushed: K .. stack_depth - 1 (C5: its tree stops at depth 8 under a
// depth-12 grid, so 2 levels, not 6).  The stackless walk (kNoStack, sorted
// pixels) keeps none when there is a table: an ancestor that is not the
// current node re-enters through the table.
__host__ __device__ inline uint32_t stack_levels(const SceneArgs& S, bool no_stack = false) {
    if (no_stack && S.tab_k) return 0u;
    const uint32_t sb = S.tab_k ? S.tab_k - 1u : 0u;
    return S.stack_depth > 1u + sb ? S.stack_depth - 1u - sb : 1u;
}

// First float4 of this wave's LDS leaf buffer (the layout of scene_lds_bytes
// and sort_lds_bytes).
__device__ __forceinline__ uint32_t leaf_buf_base(const SceneArgs& S, bool sorted) {
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t head = sorted ? (stack_levels(S, true) * kBlockThreads * 8u +
                                    (kBlockThreads / 64u) * kSortWaveBytes) / 16u
                                 : kBlockThreads + stack_levels(S) * kBlockThreads / 2u;
    return head + wave * kLeafBuf;
}

#ifndef RT_CAP_VALU
#define RT_CAP_VALU 0
#endif

// LDS leaf staging by gfx950's direct global -> LDS load (RT_GLDS, VERDICT r05
// item 5): ONE global_load_lds_dwordx4 writes spheres 0 .. cnt - 1 of the leaf
// at src into dst[0 .. cnt - 1] without a VGPR round trip or a ds_write.  Its
// LDS destination is M0 + 16 x lane id, so it needs cnt consecutive active
// lanes: from the wave's first active lane l0, lane l0 + k fetches sphere k
// into (dst - l0)[l0 + k].  Returns false (the caller stages through
// registers) when lanes l0 .. l0 + cnt - 1 are not all active.  (Widening
// exec to lanes 0 .. cnt - 1 inside an asm statement instead, the first
// build, was wrong: the address temporary's VGPR then changes in lanes the
// compiler keeps other lanes' loop-exit values in; plain frames differed.)
// The explicit vmcnt(0) retires the DMA before the chunks' ds_reads (the
// issuing wave is the reader: no barrier, MI355X_MICROARCH.md item 7).
#ifndef RT_GLDS
#define RT_GLDS 0
#endif
__device__ __forceinline__ bool glds_leaf(const float4* src, float4* dst, uint32_t cnt) {
    typedef __attribute__((address_space(3))) void LdsV;
    const uint64_t act = __ballot(1);
    const uint32_t l0 = static_cast<uint32_t>(__builtin_ctzll(act));
    const uint64_t run = ((1ull << cnt) - 1ull) << l0;  // cnt < kLeafBuf = 32
    if (l0 + cnt > 64u || (act & run) != run) return false;
    const uint32_t k = __lane_id() - l0;
    if (k < cnt) __builtin_amdgcn_global_load_lds(src + k, (LdsV*)(dst - l0), 16, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return true;
}

// Grid-space octree walk (DESIGN.md "Octree walk"): mirrored origin so every
// direction component is >= 0 (the Revelles entry step of hit_sphere,
// src/renderer.cu:23-43), cell planes at integer grid coordinates, descend by
// mid-plane tests at the current t, leave a cell through its exit planes, and
// pop to the common ancestor found from the highest flipped coordinate bit.
// The per-thread ancestor stack lives in LDS, [depth-1][thread] (conflict-free).
// kAnyHit: compile-time any-hit; with kDynAny the mode comes from `any_rt`
// instead, so ONE inlined walk serves both the primary and the shadow ray.
// kShadowL: this walk's any-hit rays are the frame's shadow rays, whose
// direction is FrameArgs::L in every lane: only then may it use
// the light-plane screen and keep its reciprocals wave-uniform.  Any other
// any-hit walk (a per-lane direction: ambient occlusion, area lights) keeps
// the full discriminant screen.
template <bool kAnyHitT, int kChunk = 2, bool kDynAny = false, bool kStats = true,
          bool kNoStack = false, bool kShadowL = false, bool kCam8 = false>
__device__ __forceinline__ bool walk(const SceneArgs& S, float o0, float o1, float o2, float d0,
                                     float d1, float d2, float tmin, float tmax, float& tout,
                                     uint32_t& iout, uint32_t& n_nodes, uint32_t& n_prims,
                                     uint2* __restrict__ stk, bool any_rt = false,
                                     uint32_t* bs = nullptr, uint32_t lb_u = ~0u) {
    static_assert(!kShadowL || kAnyHitT || kDynAny, "a shadow walk along L is an any-hit walk");
    const bool kAnyHit = kDynAny ? any_rt : kAnyHitT;
    const uint32_t D = S.max_depth;
    const uint32_t G = 1u << D;
    // Camera-relative screen: a nearest-hit walk is a primary
    // ray, whose origin is the frame's camera origin, so its screen reads the
    // per-frame records {o - c, C'} and tests fma(b, b, -C') >= 0 (4 VALU a
    // sphere) instead of the full discriminant (13 VALU); the exact tests of a
    // chunk that passes load the chunk's own sphere records (through a fresh
    // kernel-argument read: no second array pointer lives in the walk).
    // Shadow (any-hit) walks start at hit points and keep the full screen.
    const bool cam = kCamMode != 0 && !kAnyHit;
    const bool cam_exact = cam && kCamMode == 2;  // records {o - c, r}: the tests use them as they are
    // 8-byte image-plane records (RT_CAM8, unsorted nearest walks): the
    // lane's point s = (Bd).xy / (Bd).z, once per walk
    const bool cam8 = kCam8 && cam && !cam_exact && kChunk % 2 == 0;
    float s8x = 0.0f, s8y = 0.0f;
    if (cam8) {
        KernArgs* kb = kernargs();
        const float px = fmaf(kb->cam8_B[2], d2, fmaf(kb->cam8_B[1], d1, kb->cam8_B[0] * d0));
        const float py = fmaf(kb->cam8_B[5], d2, fmaf(kb->cam8_B[4], d1, kb->cam8_B[3] * d0));
        const float pz = fmaf(kb->cam8_B[8], d2, fmaf(kb->cam8_B[7], d1, kb->cam8_B[6] * d0));
        const float iz = __builtin_amdgcn_rcpf(pz);
        s8x = px * iz;
        s8y = py * iz;
    }
    // Light-plane screen: a shadow walk's direction is the
    // frame's L in every lane, so a sphere is near the ray iff its centre is
    // near the ray's origin in the plane perpendicular to L.  The records
    // hold each centre's {u, v} there and a radius grown by the rounding
    // bound, the lane its origin's {up, vp}: 5 VALU a sphere instead of 13.
#ifdef RT_NO_SHADOW_SCREEN
    constexpr bool kShdOk = false;
#else
    constexpr bool kShdOk = true;
#endif
    const bool shd = kShdOk && kShadowL && kAnyHit;  // a shadow ray along L (the caller says so)
    float up = 0.0f, vp = 0.0f;
    const bool shd8 = RT_SHD8 && kChunk % 2 == 0 && shd;
    const float2* __restrict__ shd8_base = shd8 ? S.prim_shd8 : nullptr;
    const float2* __restrict__ cam8_base = cam8 ? kernargs()->sc.prim_cam8 : nullptr;
    const float shd_rr = shd8 ? kernargs()->shd_rr : 0.0f;
    if (shd) {
        KernArgs* ke = kernargs();
        up = fmaf(o2, ke->shd_e[2], fmaf(o1, ke->shd_e[1], o0 * ke->shd_e[0]));
        vp = fmaf(o2, ke->shd_e[5], fmaf(o1, ke->shd_e[4], o0 * ke->shd_e[3]));
    }
    const float4* __restrict__ prim_sp = cam ? S.prim_cam : shd ? S.prim_shd : S.prim_sp;
    const uint2* __restrict__ nodes = S.nodes;
    const float o[3] = {o0, o1, o2};
    const float d[3] = {d0, d1, d2};
    float inv[3], nog[3];
    // Mirror mask packed in the cell table's index layout: field i (K bits,
    // 1 without a table) is all ones iff axis i is mirrored, so a table
    // index is the packed l >> (D - K) XOR mt (top - c == c ^ top for c <=
    // top), and the descent's child mirror bits are each field's low bit.
    const uint32_t kf = S.tab_k ? S.tab_k : 1u;
    const uint32_t ftop = (1u << kf) - 1u;
    uint32_t mt = 0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float g = (o[i] - S.rmin[i]) * S.scale[i];
        const bool neg = d[i] < 0.0f;
        float a = fabsf(d[i]);
        if (a < 1e-20f) a = 1e-20f;
        const float og = neg ? S.G - g : g;
        inv[i] = 1.0f / (a * S.scale[i]);
        // a shadow walk's direction is the frame's light direction, the same
        // in every lane (sample_color_unified): its reciprocals live in SGPRs
        if (kShadowL && kAnyHitT && !kDynAny)
            inv[i] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(
                                                   __builtin_bit_cast(uint32_t, inv[i])));
        nog[i] = -(og * inv[i]);
        mt |= neg ? ftop << (i * kf) : 0u;
    }
    // t of the grid plane at (mirrored) integer k: one FMA (oracle.c:plane)
    auto plane = [&](int i, uint32_t k) { return fmaf(static_cast<float>(k), inv[i], nog[i]); };
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
    RT_BS(kBsWalk);

    float best_t = tmax;
    if (kStats) n_nodes += 1;

    // Nearest keeps the best leaf *reference*; the sphere index is loaded only
    // for an exact t tie (rare) and once at the end, so no dependent load sits
    // in the hot loop.  Same result as the oracle's (min t, then min index).
    uint32_t best_ref = kNoHit;
    auto test = [&](const float4& sp, uint32_t ref) -> bool {
        if (kStats) n_prims += 1;
        RT_BS(kBsTest);
        if (kAnyHit) RT_BS(kBsTestShadow);
        float th;
        if (cam_exact ? isect_oc(sp.x, sp.y, sp.z, d0, d1, d2, sp.w, tmin, tmax, th, bs)
                      : isect(o0, o1, o2, d0, d1, d2, sp, tmin, tmax, th, bs)) {
            RT_BS(kBsAccept);
            if (kAnyHit) {
                tout = th;
                return true;
            }
            if (th < best_t) {
                best_t = th;
                best_ref = ref;
            } else if (th == best_t) {
                RT_BS(kBsTieLoad);
                if (S.prim_idx[ref] < S.prim_idx[best_ref]) best_ref = ref;
            }
        }
        return false;
    };
    // Leaf spheres in list order (same order, hence same counters, as the
    // oracle): each lane loads its own, kChunk loads in flight.
    // The chunk loop over one leaf's spheres (offset off, count cnt), each
    // read as load(k), k counted from the leaf's first reference.
    // plb: with 8-byte image-plane records staged in LDS (RT_CAM8_LDS), the
    // wave's buffer, pairs of records per float4; ~0u: records from global
    auto chunks = [&](auto&& load, uint32_t off, uint32_t cnt, uint32_t plb = ~0u) -> bool {
        // cnt >= 1 (a leaf is a non-empty cell; the root leaf is guarded by
        // its caller): a do-while skips the loop-entry test and its branch
        uint32_t j = 0;
        // Slot q of a chunk holds one of the leaf's spheres iff j + q < cnt.
        // Slot 0 always does (j < cnt inside the do-while), and for q >= 1
        // the test is j < cnt - q against a per-leaf bound: no per-chunk
        // m = cnt - j, no second loop counter and no mask for slot 0.
        const auto in_leaf = [&](int q) -> bool {
            return q == 0 || static_cast<int>(j) < static_cast<int>(cnt) - q;
        };
        do {
            RT_BS(kBsLeafChunk);
            if (kAnyHit) RT_BS(kBsChunkShadow);
            // kChunk unconditional dwordx4 loads in flight at fixed offsets; a
            // slot past the leaf's end reads the next leaf or the array's
            // kPrimPad tail (in bounds) and is never tested
            float4 sv[kChunk];
            // slot q >= 1 is fetched only when some lane's leaf still holds
            // it (RT_SKIP_PAST_END, a wave-uniform branch): a wave-wide load
            // costs the texture path as much for one lane as for 64, and at
            // a leaf's odd end the whole wave usually has no slot 1
            bool fetched[kChunk];
            if (shd8 || cam8) {
                // two slots' 8-byte records per dwordx4 (8-byte aligned:
                // global loads need dword alignment only; an even kChunk)
#pragma unroll
                for (int h = 0; h < kChunk / 2; ++h) {
                    extern __shared__ __attribute__((aligned(16))) float4 lds_pairs[];
                    const float4 pr = cam8 && plb != ~0u
                                          ? lds_pairs[plb + (j >> 1) + h]
                                          : *reinterpret_cast<const float4*>((cam8 ? cam8_base : shd8_base) +
                                                                             (off + j + 2u * h));
                    sv[2 * h] = make_float4(pr.x, pr.y, 0.0f, 0.0f);
                    sv[2 * h + 1] = make_float4(pr.z, pr.w, 0.0f, 0.0f);
                    fetched[2 * h] = fetched[2 * h + 1] = true;
                }
            } else
#pragma unroll
            for (int q = 0; q < kChunk; ++q) {
#ifdef RT_SKIP_PAST_END
                fetched[q] = q == 0 || __any(in_leaf(q));
                if (fetched[q]) sv[q] = load(j + q);
                else sv[q] = sv[0];
#else
                fetched[q] = true;
                sv[q] = load(j + q);
#endif
                // issue in list order, so the first test waits for its own
                // sphere only (vmcnt(kChunk-1)), not for the whole chunk
                __builtin_amdgcn_sched_barrier(0);
            }
            // Uniform screen: every lane's discriminants first, with no branch;
            // only when some lane's h is >= 0 (or NaN) does the wave run the
            // exact per-lane tests (which recompute them), one branch for the
            // chunk instead of a divergent branch per test.  h < 0 is exactly
            // where isect returns false, so the same spheres are accepted.
            bool maybe = false;
#pragma unroll
            for (int q = 0; q < kChunk; ++q) {
                // unconditional and unmasked: a slot past the leaf's end holds
                // a real sphere record too, and if it passes the screen the
                // exact tests below still skip it (in_leaf), so it can only
                // send the chunk down the exact path for nothing
                bool pos;
                if (cam_exact) {
                    pos = !(isect_h_oc(sv[q].x, sv[q].y, sv[q].z, d0, d1, d2, sv[q].w) < 0.0f);
                } else if (cam8) {
                    // the lane's image-plane distance from the centre's
                    // projection against rho^2 (bf16 in the records' low bytes)
                    const float rho2 = __uint_as_float(__builtin_amdgcn_perm(
                        __float_as_uint(sv[q].x), __float_as_uint(sv[q].y), 0x04000C0Cu));
                    const float dx = s8x - sv[q].x, dy = s8y - sv[q].y;
                    pos = !(fmaf(dy, dy, dx * dx) > rho2);
                } else if (cam) {
                    // b exactly as isect computes it ({x,y,z} = o - c in the
                    // same f32 operations); C' undercuts |o-c|^2 - r^2 by the
                    // rounding bound, so every sphere isect accepts passes
                    const float b = fmaf(sv[q].z, d2, fmaf(sv[q].y, d1, sv[q].x * d0));
                    pos = !(fmaf(b, b, -sv[q].w) < 0.0f);
                } else if (shd) {
                    // the centre's light-plane distance from the origin; rr'
                    // covers the rounding, so every sphere isect accepts passes
                    const float du = up - sv[q].x, dv = vp - sv[q].y;
                    const float rr8 = RT_SHD8_PER ? __uint_as_float(__builtin_amdgcn_perm(
                                                         __float_as_uint(sv[q].x), __float_as_uint(sv[q].y),
                                                         0x04000C0Cu))
                                                   : shd_rr;
                    pos = !(fmaf(dv, dv, du * du) > (shd8 ? rr8 : sv[q].z));
                } else {
                    pos = !(isect_h(o0, o1, o2, d0, d1, d2, sv[q]) < 0.0f);
                }
                maybe |= fetched[q] && pos;
            }
            // marked unlikely (it is: most chunks pass no lane): the exact
            // tests are laid out off the fall-through path (C3 -0.6%, C5
            // -0.7%, profiles/r02/branch_hint_ab.log)
#ifdef RT_BLOCK_STATS
            if (j + 1u >= cnt) RT_BS(kBsPastEnd);
#endif
            if (__builtin_expect(__any(maybe), 0)) {
                if ((cam && !cam_exact) || shd) {  // the exact tests need the spheres themselves (cam8 too)
                    RT_BS(kBsExactLoad);
                    const float4* __restrict__ ex = kernargs()->sc.prim_sp + off;
#pragma unroll
                    for (int q = 0; q < kChunk; ++q) sv[q] = ex[j + q];
                }
#pragma unroll
                for (int q = 0; q < kChunk; ++q)
                    if (in_leaf(q) && test(sv[q], off + j + q)) return true;
            } else if (kStats) {
                n_prims += min(cnt - j, static_cast<uint32_t>(kChunk));
            }
            j += kChunk;
        } while (j < cnt);
        return false;
    };
    auto leaf = [&](uint32_t off, uint32_t cnt) -> bool {
        static_assert(kChunk <= kPrimPad + 1, "leaf loads may run kChunk-1 spheres past a leaf");
        RT_BS(kBsLeaf);
#if RT_LDS_LEAF
        // A leaf the whole wave is at (the common case: one pixel's samples
        // walk together): its spheres cross the texture path ONCE, each
        // active lane fetching one into the wave's LDS leaf buffer, and the
        // chunks read them back by LDS broadcast (every lane the same
        // address): one dwordx4 texture instruction per leaf visit instead
        // of two per chunk (DESIGN.md 5.1 "LDS leaf staging").  The buffer
        // is a typed LDS array, never a generic pointer (round 3's flat
        // loads).  A slot past the leaf's end holds a stale sphere, which
        // the exact tests skip as before.
        const uint32_t off_u = __builtin_amdgcn_readfirstlane(off);
        const uint32_t cnt_u = __builtin_amdgcn_readfirstlane(cnt);
        if ((kLdsShadow || !kAnyHit) && !cam8 && cnt_u >= kLdsLeafMin && cnt_u < kernargs()->sc.lds_max &&
            __all(off == off_u)) {
            RT_BS(kBsLdsLeaf);
            extern __shared__ __attribute__((aligned(16))) float4 lds_leaf[];
            // (lb_u: the caller's wave-uniform copy, an SGPR; else from threadIdx)
            const uint32_t lb = lb_u != ~0u ? lb_u : leaf_buf_base(S, kNoStack);
            const float4* __restrict__ pu = prim_sp + off_u;
            if (!RT_GLDS || !glds_leaf(pu, lds_leaf + lb, cnt_u)) {
                const uint64_t act = __ballot(1);
                const uint32_t na = static_cast<uint32_t>(__popcll(act));
                for (uint32_t k = lane_rank(act); k < cnt_u; k += na) lds_leaf[lb + k] = pu[k];
            }
            // (a wave's LDS operations complete in order: the reads below see
            // the writes, and the compiler keeps them in order: same array)
            return chunks([&](uint32_t k) { return lds_leaf[lb + k]; }, off_u, cnt_u);
        }
        // the same for 8-byte image-plane records: pairs of records, one
        // float4 per active lane, the chunks reading a pair per ds_read_b128
        if (RT_CAM8_LDS && cam8 && cnt_u >= kLdsLeafMin8 && cnt_u < 2u * kernargs()->sc.lds_max &&
            __all(off == off_u)) {
            RT_BS(kBsLdsLeaf);
            extern __shared__ __attribute__((aligned(16))) float4 lds_leaf[];
            const uint32_t lb = lb_u != ~0u ? lb_u : leaf_buf_base(S, kNoStack);
            const float4* __restrict__ pu = reinterpret_cast<const float4*>(cam8_base + off_u);
            const uint32_t np = (cnt_u + 1u) >> 1;  // pairs (an odd leaf's last pair reads one past it)
            const uint64_t act = __ballot(1);
            const uint32_t na = static_cast<uint32_t>(__popcll(act));
            for (uint32_t k = lane_rank(act); k < np; k += na) lds_leaf[lb + k] = pu[k];
            return chunks([&](uint32_t k) { return lds_leaf[lb + k]; }, off_u, cnt_u, lb);
        }
#endif
        const float4* __restrict__ ps = prim_sp + off;
        return chunks([&](uint32_t k) { return ps[k]; }, off, cnt);
    };

    if (S.root_is_leaf) {
        if (S.root.y && leaf(S.root.x, S.root.y)) return true;  // an empty scene's root holds 0
    } else {
        uint2 node = S.root;
        // Cell = (depth, lower corner l* in finest-grid units, size = G >> depth):
        // mid plane = l + size/2, exit plane = l + size: the same integers (hence
        // the same plane values) as the oracle's c * size forms, 3 VALU a plane.
        uint32_t depth = 0, l0 = 0, l1 = 0, l2 = 0, size = G;
        float t = t0;
        // Cell table: the walk enters at depth K through one
        // table load, and a step whose common ancestor lies above depth K
        // jumps the same way instead of re-reading the records down to K.
        const uint2* __restrict__ tab = S.tab;
        const uint32_t K = S.tab_k;
        bool jump = tab != nullptr;
        uint32_t from = 0;  // depth the oracle re-descends from (stats)
        // with a table, only depths >= K are ever on the stack (stack_levels);
        // the stackless walk (kNoStack) keeps one only without a table
        const uint32_t sb = K ? K - 1u : 0u;
        // Hard cap (never reached by a correct walk: a ray crosses < 3*G cells
        // and each crossing costs at most one descent): no input can hang the GPU.
        // One exit per trip (`stop`): the any-hit, nearest-done, ray-left and
        // root-left conditions are OR-ed into one flag, so the wave's exec
        // bookkeeping is one loop-exit mask update per trip (the scalar pipe is
        // this kernel's busiest unit, profiles/r02/pmc_sq_screen.json).
        bool any_hit = false;
#if RT_CAP_VALU
        // the trip counter as a lane value (an opaque v_mov): the cap test is
        // one VALU compare feeding the exit mask, not SALU add / compare /
        // select on the scalar pipe (A/B)
        uint32_t it;
        asm volatile("v_mov_b32 %0, 0" : "=v"(it));
        for (const uint32_t cap = 8u * G + 64u;; ++it) {
#else
        for (uint32_t it = 0, cap = 8u * G + 64u;; ++it) {
#endif
            RT_BS(kBsIter);
            if (kAnyHit) RT_BS(kBsIterShadow);
            uint2 rec = make_uint2(0u, 0u);
            bool have = false;   // rec is a leaf record (else the cell is empty)
            bool inner = false;  // stepped into an internal node: descend next trip
            if (jump) {
                RT_BS(kBsJump);
                jump = false;
                // mid-plane tests at t from `depth` down to K (no loads: the
                // descent's child choices), then the cell's table entry
                while (depth < K) {
                    RT_BS(kBsJumpDescend);
                    if (kAnyHit) RT_BS(kBsJumpDescendShadow);
                    const uint32_t half = size >> 1;
                    l0 += plane(0, l0 + half) <= t ? half : 0u;
                    l1 += plane(1, l1 + half) <= t ? half : 0u;
                    l2 += plane(2, l2 + half) <= t ? half : 0u;
                    size = half;
                    depth += 1;
                }
                const uint32_t sh = D - K;
                // real cell coordinates: mirrored axes count from the far side
                // (the XOR with mt flips every mirrored field at once)
                const uint32_t c = ((((l2 >> sh) << K) | (l1 >> sh)) << K | (l0 >> sh)) ^ mt;
                const uint2 e = tab[c];
                const uint32_t kind = e.y >> kCellKindShift;
                depth = (e.y >> kCellDepthShift) & 31u;
                size = G >> depth;
                l0 &= ~(size - 1u);
                l1 &= ~(size - 1u);
                l2 &= ~(size - 1u);
                rec = make_uint2(e.x, e.y & kCellRecMask);
                // the oracle reads one record per level from `from` down to
                // the covering node (an empty child's own level reads none)
                // (a re-entry below K re-reads levels the oracle pops: none counted)
                if (kStats) {
                    const uint32_t cd = kind == kCellEmpty ? depth - 1u : depth;
                    n_nodes += cd > from ? cd - from : 0u;
                }
                inner = kind == kCellInternal;
                have = kind == kCellLeaf;
            } else {
                RT_BS(kBsDescend);
                const uint32_t half = size >> 1;
                const bool b0 = plane(0, l0 + half) <= t;
                const bool b1 = plane(1, l1 + half) <= t;
                const bool b2 = plane(2, l2 + half) <= t;
                const uint32_t bits = (b0 ? 1u : 0u) | (b1 ? 2u : 0u) | (b2 ? 4u : 0u);
                const uint32_t mbits = (mt & 1u) | ((mt >> (kf - 1u)) & 2u) |
                                       ((mt >> (2u * kf - 2u)) & 4u);
                const uint32_t child = bits ^ mbits;
                l0 += b0 ? half : 0u;
                l1 += b1 ? half : 0u;
                l2 += b2 ? half : 0u;
                size = half;
                depth += 1;
                const uint32_t valid = node.y & 0xFFu;
                have = (valid & (1u << child)) != 0;
                if (have) {
                    const uint32_t slot = node.x + __builtin_popcount(valid & ((1u << child) - 1u));
                    rec = nodes[slot];
#ifdef RT_BLOCK_STATS
                    if (depth > from) RT_BS(kBsNodeRead);
                    else RT_BS(kBsNodeReread);
#endif
                    // records down to a re-entered ancestor are the oracle's
                    // stack pops, not reads
                    if (kStats && depth > from) n_nodes += 1;
                    inner = !((node.y >> 8) & (1u << child));
                    have = !inner;
                }
            }
            // An internal node: descend next trip.  No `continue` and no break
            // inside the step: the rest of the trip is the else branch, and the
            // loop's one exit is `stop` at the end of the trip (a stopped lane's
            // step state is garbage it never uses; its pop is masked off), so
            // the structurizer keeps no exit-code variable: C3 -3.3%, C5 -3.3%,
            // C5d -3.8% (profiles/r02/inner_else_ab.log).
            bool stop = false;
            if (inner) {
                RT_BS(kBsInternal);
                node = rec;
                if (!kNoStack || !tab) stk[(depth - 1 - sb) * kBlockThreads] = rec;
            } else {
                if (have) any_hit = leaf(rec.x, rec.y);
                RT_BS(kBsExit);
                const float e0 = plane(0, l0 + size);
                const float e1 = plane(1, l1 + size);
                const float e2 = plane(2, l2 + size);
                // one v_min3_f32 (the oracle's ternaries can differ only in the sign
                // of a zero, and texit is only ever compared: identical walks)
                const float texit = fminf(fminf(e0, e1), e2);
                // step every axis whose exit plane is texit; the flipped bits give the
                // common ancestor (oracle.c: diff of the cell coordinates)
                const uint32_t n0 = e0 == texit ? l0 + size : l0;
                const uint32_t n1 = e1 == texit ? l1 + size : l1;
                const uint32_t n2 = e2 == texit ? l2 + size : l2;
                // leave on an any-hit, a nearest hit before this cell's exit, or
                // the ray's end.  The oracle's root-boundary test (a stepped
                // coordinate reaching G) needs no term of its own: an axis that
                // steps to G exits through plane(i, G), the very value t1 is
                // the minimum of, so texit >= t1 already holds there.
                stop = any_hit | (!kAnyHit & (best_t < texit)) | (texit >= t1);
                const uint32_t diff = (l0 ^ n0) | (l1 ^ n1) | (l2 ^ n2);
                const uint32_t top = 31u - __builtin_clz(diff);  // highest flipped bit
                t = texit;
                // The common ancestor: size 2^(top+1), depth D - (top+1).  With a
                // table the walk re-enters through it unless the ancestor is the
                // node it iterates (m == 1): above depth K, or (no ancestor stack)
                // two or more levels up.  A cell at depth >= K indexes the table
                // straight from the neighbour's corner (`keep`) and re-descends
                // by records; a shallower one resolves down to K from the
                // ancestor's cell.  Without a table it pops to the ancestor.
                // Selects, not branches: every lane ends the trip with the same
                // instructions (the scalar pipe carries the branches' exec-mask
                // updates, and it is the kernel's busiest unit).
                const uint32_t adepth = D - (top + 1u);
                const uint32_t m = depth - adepth;  // levels up to the ancestor
                const bool above = adepth < K || (kNoStack && K != 0u && m > 1u);
                const bool keep = above && depth >= K;
                const uint32_t asize = 2u << top;
                const uint32_t am = keep ? 0xFFFFFFFFu : ~(asize - 1u);
                l0 = n0 & am;
                l1 = n1 & am;
                l2 = n2 & am;
                size = keep ? size : asize;
                depth = keep ? depth : adepth;
                if (kStats && above) from = adepth;
                jump = above;
                // m == 1: the ancestor is the node we are iterating (still in `node`)
                if (!stop && !above && m > 1) {  // (the stackless walk: only without a table)
                    RT_BS(kBsPop);
                    node = depth ? stk[(depth - 1 - sb) * kBlockThreads] : S.root;
                }
            }
            // the safety cap shares the one exit (C3 -0.3%, profiles/r02/cap_exit_ab.log)
            if (stop || it + 1u >= cap) break;
        }
        if (any_hit) return true;
    }
    if (!kAnyHit && best_ref != kNoHit) {
        if (!RT_REF_SHADE) RT_BS(kBsHitIdx);
        tout = best_t;
        iout = RT_REF_SHADE ? best_ref : S.prim_idx[best_ref];
        return true;
    }
    return false;
}

// ---------------------------------------------------------------------------
// Frame mapping, shading, ordered accumulation
//
// A wave owns `ppw` pixels x `spw` samples (host: spw = min(spp, 64),
// ppw = pow2floor(64 / spw)); lane l works on pixel l / spw, sample
// round * spw + l % spw.  At spp >= 64 all 64 lanes of a wave trace jittered
// samples of ONE pixel: their primary rays stay within one pixel footprint and
// their shadow rays start from nearly the same point with the same direction,
// so the wave's lanes follow nearly the same octree path (little SIMD
// divergence, and coherent packets).  The per-pixel mean keeps the oracle's
// exact summation order: every lane parks its sample colour in LDS and the
// pixel's leader lane adds them in sample order.
// ---------------------------------------------------------------------------

struct PixelOut {
    float r, g, b;
};

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

// Stats frames only.  Every wave adds its counts as it exits, so the adds
// all land in the frame's tail: on ONE cache line they serialise there and
// stall the last waves' loads behind them (plain frames that still flushed
// were 4.3% slower on C3 and 17% on a 1/8 tile share, profiles/r02/flush_ab.log).
// One line per XCD group cuts the queue per line 8x; the host sums the lines.
__device__ __forceinline__ void flush_counters(const FrameArgs& a, uint32_t prim, uint32_t shadow,
                                               uint32_t nodes, uint32_t prims) {
    // ray counts are wave-uniform already (ballot counts); the work counters
    // are per lane
    const unsigned long long s0 = prim;
    const unsigned long long s1 = shadow;
    const unsigned long long s2 = wave_sum(nodes);
    const unsigned long long s3 = wave_sum(prims);
    if ((threadIdx.x & 63u) == 0) {
        unsigned long long* c = a.counters + kStatLineBase + (blockIdx.x & 7u) * kStatLineStride;
        atomicAdd(c + 0, s0);
        atomicAdd(c + 1, s1);
        atomicAdd(c + 2, s2);
        atomicAdd(c + 3, s3);
    }
}

// The hit record a nearest walk returned (`iout`: a leaf reference under
// RT_REF_SHADE, else a sphere index): its sphere and its packed albedo.
// (SA: SceneArgs, or the kernel arguments' copy behind kernargs())
template <typename SA>
__device__ __forceinline__ float4 hit_sphere_rec(SA& S, uint32_t h) {
    return RT_REF_SHADE ? S.prim_sp[h] : S.spheres[h];
}
template <typename SA>
__device__ __forceinline__ uint32_t hit_albedo(SA& S, uint32_t h) {
    return RT_REF_SHADE ? S.prim_al[h] : S.albedo[h];
}

// Unified lane path: one walk instance run twice (primary, then the shadow ray
// of the lanes that need one), so the register allocator sees one walk.
template <int kChunk, bool kStats, bool kCam8 = false>
__device__ __forceinline__ PixelOut sample_color_unified(const FrameArgs& a, uint32_t x,
                                                         uint32_t y, uint32_t hp, uint32_t s,
                                                         bool valid, uint32_t& n_shadow,
                                                         uint32_t& n_nodes, uint32_t& n_prims,
                                                         void* stk, uint32_t* bs = nullptr,
                                                         uint32_t lbs = ~0u) {
    const SceneArgs& S = a.sc;
    KernArgs* ka = kernargs();
    float u = static_cast<float>(x), v = static_cast<float>(y);
    if (ka->jitter) {
        u = u + u01(mix32(hp ^ (s << 1)));
        v = v + u01(mix32(hp ^ ((s << 1) | 1u)));
    }
    float r0 = ka->cam.o[0], r1 = ka->cam.o[1], r2 = ka->cam.o[2];
    float d0, d1, d2;
    {
        CamArgs cam;
        for (int i = 0; i < 9; ++i) cam.K[i] = ka->cam.K[i], cam.R[i] = ka->cam.R[i];
        get_ray(cam, u, v, d0, d1, d2);
    }
    const float miss_g = sat(d1), miss_b = sat(d2);
    bool active = valid, hit0 = false;
    float lam = 0.0f;
    uint32_t al = 0;
    // the primary and the shadow walk as two instances (the phase loop was
    // always unrolled into two copies; written out so that the primary one
    // keeps the camera-relative screen, a compile-time choice)
#pragma unroll
    for (int phase = 0; phase < 2; ++phase) {
        float t = 0.0f;
        uint32_t idx = 0;
        bool hit = false;
        if (active) {
            RT_BS(kBsPhase);
            if (phase) RT_BS(kBsPhaseShadow);
            if (phase == 0)
                hit = walk<false, kChunk, false, kStats, false, false, kCam8>(S, r0, r1, r2, d0, d1, d2, 0.0f, INFINITY, t,
                                                         idx, n_nodes, n_prims,
                                                         static_cast<uint2*>(stk), false, bs, lbs);
            else {
                // the shadow direction L is the frame's, the same in every
                // lane: read afresh from the kernel arguments (SGPRs), not the
                // lanes' d registers
                KernArgs* kl = kernargs();
                hit = walk<true, RT_SHD_CHUNK, false, kStats, false, true>(
                    S, r0, r1, r2, kl->L[0], kl->L[1], kl->L[2], 0.0f, INFINITY, t, idx, n_nodes,
                    n_prims, static_cast<uint2*>(stk), true, bs, lbs);
            }
        }
        if (phase == 0) {
            hit0 = active && hit;
            bool want_shadow = false;
            KernArgs* kb = kernargs();
            if (hit0) {
                RT_BS(kBsShadeLoad);  // the sphere record
                RT_BS(kBsShadeLoad);  // the albedo
                const float4 sp = hit_sphere_rec(kb->sc, idx);
                const float p0 = r0 + t * d0;
                const float p1 = r1 + t * d1;
                const float p2 = r2 + t * d2;
                const float ir = 1.0f / sp.w;
                const float n0 = (p0 - sp.x) * ir;
                const float n1 = (p1 - sp.y) * ir;
                const float n2 = (p2 - sp.z) * ir;
                const float ndl = n0 * kb->L[0] + n1 * kb->L[1] + n2 * kb->L[2];
                lam = ndl > 0.0f ? ndl : 0.0f;
                want_shadow = ndl > 0.0f && kb->shadows;
                al = hit_albedo(kb->sc, idx);
                r0 = p0 + n0 * kShadowEps;
                r1 = p1 + n1 * kShadowEps;
                r2 = p2 + n2 * kShadowEps;
                d0 = kb->L[0];
                d1 = kb->L[1];
                d2 = kb->L[2];
            }
            active = want_shadow;
            n_shadow += static_cast<uint32_t>(__popcll(__ballot(active)));  // wave-uniform
            if (!__any(active)) break;
        } else if (active && hit) {
            lam = 0.0f;
        }
    }
    PixelOut c{200.0f / 255.0f, miss_g, miss_b};
    if (hit0) {
        const float amb = kernargs()->ambient;
        const float f = amb + (1.0f - amb) * lam;
        c.r = static_cast<float>(al & 0xFFu) * (1.0f / 255.0f) * f;
        c.g = static_cast<float>((al >> 8) & 0xFFu) * (1.0f / 255.0f) * f;
        c.b = static_cast<float>((al >> 16) & 0xFFu) * (1.0f / 255.0f) * f;
    }
    return c;
}

// Wave tile (tw x th pixels x spw samples, launch_scene) at pixel origin
// (ox, oy); for a packed tile list also obase: image pixel (x, y) of this
// tile is packed word obase + y * tile_size + x (mod 2^32; one value kept
// live across the walks instead of the slot and the tile-local origin).
// Rounds of spw samples, pairwise butterfly per round, rounds added in
// order in the leader's LDS slot, then the mean is written.
template <bool kTiles, int kChunk, bool kStats, bool kProg, bool kCam8 = false>
__device__ __forceinline__ void shade_wave_tile(const FrameArgs& a, float4* acc, void* stk,
                                                uint32_t ox, uint32_t oy, uint32_t obase,
                                                uint32_t& n_primary,
                                                uint32_t& n_shadow, uint32_t& n_nodes,
                                                uint32_t& n_prims, uint32_t* bs = nullptr,
                                                uint32_t lbs = ~0u) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t spw = a.spw, g = a.g;
    const uint32_t pix = lane / g, sub = lane & (g - 1u);
    const uint32_t qx = pix % a.tw, qy = pix / a.tw;
    const uint32_t x = ox + qx, y = oy + qy;
    const bool lane_pix = pix < a.ppw && x < a.W && y < a.H;
    const bool leader = lane_pix && sub == 0;
    const uint32_t pid = y * a.W + x;
    const uint32_t hp = mix32(a.seedmix ^ pid);
    // progressive: the stored sum seeds the leader's LDS slot, so round 0
    // adds onto it like any later round (nothing extra live in the walk)
    if (kProg && a.accum_in && leader) acc[threadIdx.x] = a.accum[(size_t)y * a.W + x];
    // sample index across accumulated frames: s_base + r*spw + sub
    const uint32_t s_base = kProg ? a.s_base : 0u;
    const uint32_t sub_base = s_base + sub;
    const uint32_t s_end = s_base + a.spp;
    const bool lane_ok = lane_pix && sub < spw;
    for (uint32_t r = 0; r < a.rounds; ++r) {
        const uint32_t sg = r * spw + sub_base;
        const bool valid = lane_ok && sg < s_end;
        n_primary += static_cast<uint32_t>(__popcll(__ballot(valid)));  // wave-uniform
        PixelOut c = sample_color_unified<kChunk, kStats, kCam8>(a, x, y, hp, sg, valid, n_shadow,
                                                          n_nodes, n_prims, stk, bs, lbs);
        // Pixel sum of this round: pairwise butterfly over the pixel's g
        // lanes (missing samples are 0) = oracle.c:tree_sum; rounds are then
        // added in order in the leader's LDS slot.
        if (!valid) c = PixelOut{0.0f, 0.0f, 0.0f};
        for (uint32_t m = 1; m < g; m <<= 1) {
            c.r += __shfl_xor(c.r, static_cast<int>(m), 64);
            c.g += __shfl_xor(c.g, static_cast<int>(m), 64);
            c.b += __shfl_xor(c.b, static_cast<int>(m), 64);
        }
        if (leader) {
            if (r || (kProg && a.accum_in)) {
                const float4 A = acc[threadIdx.x];
                c.r = A.x + c.r;
                c.g = A.y + c.g;
                c.b = A.z + c.b;
            }
            acc[threadIdx.x] = make_float4(c.r, c.g, c.b, 0.0f);
        }
    }
    // outputs: fields read afresh (kernargs()), not kept live across the walks
    KernArgs* ko = kernargs();
    if (leader) {
        const float4 A = acc[threadIdx.x];
        if (kProg) ko->accum[(size_t)y * ko->W + x] = A;
        const float isp = ko->inv_spp;
        const PixelOut p{A.x * isp, A.y * isp, A.z * isp};
        const uint32_t rgba = pack_rgba8(p);
        if (kTiles) {
            ko->out8[obase + y * ko->tile_size + x] = rgba;
        } else {
            ko->out8[(size_t)y * ko->W + x] = rgba;
            if (ko->out32) ko->out32[(size_t)y * ko->W + x] = make_float4(p.r, p.g, p.b, 1.0f);
        }
    } else if (kTiles && sub == 0 && pix < ko->ppw) {
        ko->out8[obase + y * ko->tile_size + x] = 0u;  // off-image pixel of an edge tile
    }
}

// ---------------------------------------------------------------------------
// Quadrant-sorted rounds (DESIGN.md 5.1 "Sorted rounds")
//
// At spp > 64 a pixel's samples run in rounds of 64, and a round costs its
// slowest lane.  Where a pixel is about one sphere wide (C5: pixel 0.0017,
// sphere diameter ~0.003 world units) its samples hit different spheres and
// their walks diverge; the oracle's walks put the slowest lane at 1.6x the
// mean (tools/shadow_sim.py).  Samples whose jitter falls in the same pixel
// quadrant are closer, so this path traces a pixel's samples grouped by
// quadrant (stable: a quadrant's samples in index order), 64 at a time,
// parks each colour in the wave's LDS under its sample index, and then sums
// the rounds exactly as shade_wave_tile does: round r = samples 64r..64r+63,
// pairwise, rounds in order.  Same colours, same sums, same image; the model
// predicts 11% fewer primary and 13% fewer shadow trips on C5.
// ---------------------------------------------------------------------------


// Morton cell of sample sg's jitter on a 2^kSortCellBits grid per axis (the
// top bits of each hash are its u01 in those steps): the top two bits are
// the quadrant, and so on down
__device__ __forceinline__ uint32_t jitter_cell(uint32_t hp, uint32_t sg) {
    const uint32_t qu = mix32(hp ^ (sg << 1)) >> (32u - kSortCellBits);
    const uint32_t qv = mix32(hp ^ ((sg << 1) | 1u)) >> (32u - kSortCellBits);
    uint32_t c = 0;
#pragma unroll
    for (uint32_t b = 0; b < kSortCellBits; ++b)
        c |= (((qu >> b) & 1u) << (2u * b)) | (((qv >> b) & 1u) << (2u * b + 1u));
    return c;
}

// Primary ray direction of sample sg of pixel (x, y) (sample_color_unified's).
__device__ __forceinline__ void sample_dir(uint32_t x, uint32_t y, uint32_t hp, uint32_t sg,
                                           float& d0, float& d1, float& d2) {
    KernArgs* ka = kernargs();
    float u = static_cast<float>(x), v = static_cast<float>(y);
    if (ka->jitter) {
        u = u + u01(mix32(hp ^ (sg << 1)));
        v = v + u01(mix32(hp ^ ((sg << 1) | 1u)));
    }
    CamArgs cam;
    for (int i = 0; i < 9; ++i) cam.K[i] = ka->cam.K[i], cam.R[i] = ka->cam.R[i];
    get_ray(cam, u, v, d0, d1, d2);
}

// Hit point and normal of a primary hit (sample_color_unified's shading prep).
struct HitShade {
    float p0, p1, p2, n0, n1, n2, ndl;
};
__device__ __forceinline__ HitShade hit_shade(float d0, float d1, float d2, float t, uint32_t idx,
                                              uint32_t* bs = nullptr) {
    KernArgs* kb = kernargs();
    const float4 sp = hit_sphere_rec(kb->sc, idx);
    RT_BS(kBsShadeLoad);
    HitShade h;
    h.p0 = kb->cam.o[0] + t * d0;
    h.p1 = kb->cam.o[1] + t * d1;
    h.p2 = kb->cam.o[2] + t * d2;
    const float ir = 1.0f / sp.w;
    h.n0 = (h.p0 - sp.x) * ir;
    h.n1 = (h.p1 - sp.y) * ir;
    h.n2 = (h.p2 - sp.z) * ir;
    h.ndl = h.n0 * kb->L[0] + h.n1 * kb->L[1] + h.n2 * kb->L[2];
    return h;
}

// One pixel (spw = 64: the wave is one pixel), 2..4 rounds, at pixel (x, y):
//  1. order: the pixel's samples grouped by jitter quadrant;
//  2. primary rays 64 at a time in that order; a miss or an unlit hit is
//     final (its slot holds the colour's inputs), a lit hit parks {t, sphere}
//     and joins the list of lit samples;
//  3. the lit samples' shadow rays 64 at a time (dense: one pixel's lit
//     samples of all rounds together, in quadrant order), each recomputing
//     its hit point from {t, sphere} with the same operations;
//  4. per round in sample order: colours, pairwise sums, rounds in order.
template <bool kTiles, int kChunk, bool kStats, bool kProg>
__device__ __forceinline__ void shade_pixel_sorted(const FrameArgs& a, float* wl, void* stk,
                                                   uint32_t x, uint32_t y, uint32_t obase,
                                                   uint32_t& n_primary, uint32_t& n_shadow,
                                                   uint32_t& n_nodes, uint32_t& n_prims,
                                                   uint32_t* bs, uint32_t lbs) {
    const SceneArgs& S = a.sc;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t R = a.rounds;
    const bool lane_pix = x < a.W && y < a.H;
    const uint32_t n = lane_pix ? a.spp : 0u;  // this pixel's samples (local indices)
    const uint32_t hp = mix32(a.seedmix ^ (y * a.W + x));
    const uint32_t s_base = kProg ? a.s_base : 0u;
    uint2* slot = reinterpret_cast<uint2*>(wl);
    uint8_t* kind = reinterpret_cast<uint8_t*>(slot + kSortMax);  // 0 miss, 1 hit, 2 lit (in flight)
    uint8_t* ord = kind + kSortMax;
    uint8_t* lit = ord + kSortMax;
    // 1. tracing order: local samples s = 64 j + lane grouped by 4x4 Morton
    //    cell of their jitter (quadrants first): a counting sort over LDS
    //    counters (an LDS atomic gives a sample its place in its cell)
    uint32_t* bcnt = reinterpret_cast<uint32_t*>(lit + kSortMax);
    const bool jit = kernargs()->jitter != 0u;
    if (lane < kSortCells) bcnt[lane] = 0u;
    // (cell << 8 | place in the cell) parked in the sample's slot until placed
    for (uint32_t j = 0; j < R; ++j) {
        const uint32_t sl = 64u * j + lane;
        if (sl < n) {
            const uint32_t cell = jit ? jitter_cell(hp, s_base + sl) : 0u;
            slot[sl].x = (cell << 8) | atomicAdd(bcnt + cell, 1u);
        }
    }
    {  // exclusive prefix of the cells' counts (one per lane)
        const uint32_t v = lane < kSortCells ? bcnt[lane] : 0u;
        uint32_t incl = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t o = __shfl_up(incl, static_cast<unsigned>(d), 64);
            if (static_cast<int>(lane) >= d) incl += o;
        }
        if (lane < kSortCells) bcnt[lane] = incl - v;
    }
    for (uint32_t j = 0; j < R; ++j) {
        const uint32_t sl = 64u * j + lane;
        if (sl < n) {
            const uint32_t kp = slot[sl].x;
            ord[bcnt[kp >> 8] + (kp & 0xFFu)] = static_cast<uint8_t>(sl);
        }
    }
    // (a wave's LDS operations complete in order: no barrier needed)
    // 2. primary rays in that order
    uint32_t nl = 0;  // lit samples listed (wave-uniform)
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t i = 64u * r + lane;
        const bool valid = i < n;
        const uint32_t sl = valid ? static_cast<uint32_t>(ord[i]) : 0u;
        n_primary += static_cast<uint32_t>(__popcll(__ballot(valid)));  // wave-uniform
        float d0, d1, d2;
        sample_dir(x, y, hp, s_base + sl, d0, d1, d2);
        float t = 0.0f;
        uint32_t idx = 0;
        bool hit = false;
        if (valid) {
            RT_BS(kBsPhase);
            KernArgs* kc = kernargs();
            hit = walk<false, kChunk, true, kStats, true, false, RT_CAM8_SORTED != 0>(S, kc->cam.o[0], kc->cam.o[1], kc->cam.o[2],
                                                          d0, d1, d2, 0.0f, INFINITY, t, idx, n_nodes,
                                                          n_prims, static_cast<uint2*>(stk), false, bs,
                                                          lbs);
        }
        bool is_lit = false;
        if (valid) {
            uint2 sv = make_uint2(__float_as_uint(sat(d1)), __float_as_uint(sat(d2)));
            uint8_t kd = 0;
            if (hit) {
                const HitShade h = hit_shade(d0, d1, d2, t, idx, bs);
                is_lit = h.ndl > 0.0f && kernargs()->shadows;
                if (is_lit) {
                    sv = make_uint2(__float_as_uint(t), idx);
                    kd = 2;
                } else {
                    RT_BS(kBsShadeLoad);
                    sv = make_uint2(__float_as_uint(h.ndl > 0.0f ? h.ndl : 0.0f),
                                    hit_albedo(kernargs()->sc, idx));
                    kd = 1;
                }
            }
            slot[sl] = sv;
            kind[sl] = kd;
        }
        const uint64_t lm = __ballot(is_lit);
        if (is_lit) lit[nl + lane_rank(lm)] = static_cast<uint8_t>(sl);
        nl += static_cast<uint32_t>(__popcll(lm));
    }
    n_shadow += nl;
    // 3. the lit samples' shadow rays, 64 at a time
    for (uint32_t c0 = 0; c0 < nl; c0 += 64u) {
        const uint32_t j = c0 + lane;
        const bool has = j < nl;
        const uint32_t sl = has ? static_cast<uint32_t>(lit[j]) : 0u;
        float o0 = 0.f, o1 = 0.f, o2 = 0.f, lam = 0.0f;
        uint32_t idx = 0;
        if (has) {
            float d0, d1, d2;
            sample_dir(x, y, hp, s_base + sl, d0, d1, d2);
            const uint2 sv = slot[sl];
            idx = sv.y;
            const HitShade h = hit_shade(d0, d1, d2, __uint_as_float(sv.x), idx, bs);
            lam = h.ndl > 0.0f ? h.ndl : 0.0f;
            o0 = h.p0 + h.n0 * kShadowEps;
            o1 = h.p1 + h.n1 * kShadowEps;
            o2 = h.p2 + h.n2 * kShadowEps;
        }
        bool occ = false;
        if (has) {
            RT_BS(kBsPhase);
            RT_BS(kBsPhaseShadow);
            KernArgs* kl = kernargs();
            float ts;
            uint32_t is;
            occ = walk<false, RT_SHD_CHUNK, true, kStats, true, true>(
                S, o0, o1, o2, kl->L[0], kl->L[1], kl->L[2], 0.0f, INFINITY, ts, is, n_nodes,
                n_prims, static_cast<uint2*>(stk), true, bs, lbs);
        }
        if (has) {
            RT_BS(kBsShadeLoad);
            slot[sl] = make_uint2(__float_as_uint(occ ? 0.0f : lam), hit_albedo(kernargs()->sc, idx));
            kind[sl] = 1;
        }
    }
    // 4. the rounds in sample order: colours, pairwise sums (oracle.c:tree_sum),
    //    added in order (shade_wave_tile's arithmetic)
    KernArgs* ko = kernargs();
    float4 A = make_float4(0.f, 0.f, 0.f, 0.f);
    for (uint32_t r = 0; r < R; ++r) {
        const uint32_t i = 64u * r + lane;
        PixelOut c{0.0f, 0.0f, 0.0f};
        if (i < n) {
            const uint2 sv = slot[i];
            if (kind[i]) {
                const float lam = __uint_as_float(sv.x);
                const uint32_t al = sv.y;
                const float amb = ko->ambient;
                const float f = amb + (1.0f - amb) * lam;
                c.r = static_cast<float>(al & 0xFFu) * (1.0f / 255.0f) * f;
                c.g = static_cast<float>((al >> 8) & 0xFFu) * (1.0f / 255.0f) * f;
                c.b = static_cast<float>((al >> 16) & 0xFFu) * (1.0f / 255.0f) * f;
            } else {
                c = PixelOut{200.0f / 255.0f, __uint_as_float(sv.x), __uint_as_float(sv.y)};
            }
        }
        for (uint32_t m = 1; m < 64u; m <<= 1) {
            c.r += __shfl_xor(c.r, static_cast<int>(m), 64);
            c.g += __shfl_xor(c.g, static_cast<int>(m), 64);
            c.b += __shfl_xor(c.b, static_cast<int>(m), 64);
        }
        if (r == 0u) {
            if (kProg && ko->accum_in && lane_pix) {
                const float4 P = ko->accum[(size_t)y * ko->W + x];
                A = make_float4(P.x + c.r, P.y + c.g, P.z + c.b, 0.0f);
            } else {
                A = make_float4(c.r, c.g, c.b, 0.0f);
            }
        } else {
            A = make_float4(A.x + c.r, A.y + c.g, A.z + c.b, 0.0f);
        }
    }
    if (lane == 0u) {
        if (lane_pix) {
            if (kProg) ko->accum[(size_t)y * ko->W + x] = A;
            const float isp = ko->inv_spp;
            const PixelOut p{A.x * isp, A.y * isp, A.z * isp};
            const uint32_t rgba = pack_rgba8(p);
            if (kTiles) {
                ko->out8[obase + y * ko->tile_size + x] = rgba;
            } else {
                ko->out8[(size_t)y * ko->W + x] = rgba;
                if (ko->out32) ko->out32[(size_t)y * ko->W + x] = make_float4(p.r, p.g, p.b, 1.0f);
            }
        } else if (kTiles) {
            ko->out8[obase + y * ko->tile_size + x] = 0u;  // off-image pixel of an edge tile
        }
    }
}

// Work scheduling (persistent workgroups: grid = resident workgroups):
//
// kWaveQ = false: workgroups pull bts x bts block tiles from ONE device-wide
//   queue head (a returning atomic per tile); the tile's wave tiles are dealt
//   to the 4 waves round-robin, and the workgroup syncs per tile.
// kWaveQ = true: every WAVE pulls tickets of 1-4 wave tiles on its own.  The
//   wave tiles are numbered in 8x8 blocks (spatially coherent) of 8x8-block
//   superblocks; whole superblocks go to XCD groups (blockIdx % 8: blocks are
//   dealt round-robin over the 8 XCDs, MI355X_MICROARCH.md "Workgroup
//   dispatch") in claim order, and each XCD has its own ticket head on its
//   own cache line (one head saturates near 88 dequeues/us) over the
//   superblocks it claimed: the two-level queue below.  No workgroup barrier;
//   the tail is one ticket.
//
// kMinW = minimum waves per SIMD requested from the register allocator.
// kProg: progressive frame (a.accum set); compiled separately so plain frames
// keep their register budget.
// Residency of the wave-queue builds is set by SGPRs, not VGPRs: at 60-65
// VGPRs and 94 SGPRs (112 allocated) a SIMD holds 7 waves.  The 8-wave build
// caps its SGPRs at 80 (the rest spill into VGPR lanes, no scratch), and 8
// waves fit: C3 -1.9%, its tile path -3.3%, C5 -2.4% (84: 8 do not fit; 76
// and 72: the extra spills cost more; profiles/r02/sgpr_ab.log).
// scene_kernel_w8 below is that build of the timed default.
template <bool kTiles, int kChunk, bool kStats = true, bool kProg = false, bool kWaveQ = false,
          bool kSort = false>
__device__ __forceinline__ void scene_body(FrameArgs a) {
    extern __shared__ __attribute__((aligned(16))) float4 lds[];
    float4* acc = lds;  // [256] running pixel sums (leader lanes' slots)
    const uint32_t wave = threadIdx.x >> 6;
    // sorted rounds: no per-thread pixel sums; stacks first, then each wave's
    // colours and tracing order (sort_lds_bytes)
    void* stk = reinterpret_cast<uint2*>(lds + (kSort ? 0u : kBlockThreads)) + threadIdx.x;
    float* wl = kSort ? reinterpret_cast<float*>(reinterpret_cast<uint2*>(lds) +
                                                 stack_levels(a.sc, true) * kBlockThreads) +
                            wave * (kSortWaveBytes / 4u)
                      : nullptr;
    // the walks' LDS leaf buffer base as a wave-uniform value (an SGPR, or a
    // lane of the SGPR spill VGPR), handed down to walk(): computed from
    // threadIdx inside the walk it lived in a VGPR, which the sorted 64-VGPR
    // build spilled to scratch and reloaded (a scratch load and a vmcnt(0)
    // wait) on every staged leaf.  C5 -1.2%, C5d -0.3% (sorted), C3 -0.4%
    // (profiles/r06/ab_leaf_base_*.log); RT_LB_SGPR=0: as before
#ifndef RT_LB_SGPR
#define RT_LB_SGPR 1
#endif
    const uint32_t lbs = RT_LB_SGPR ? __builtin_amdgcn_readfirstlane(leaf_buf_base(a.sc, kSort)) : ~0u;
    // the next frame's counters, queue heads and slot table (the other set,
    // FrameArgs::ctr_next): zeroed here by the first workgroup, so frames run
    // back to back with no memset launch between them.  The previous frame,
    // which used that set, completed before this one started.
    // (fields read through kernargs(): nothing of this stays live in SGPRs)
    if (blockIdx.x == 0) {
        KernArgs* kz = kernargs();
        for (uint32_t i = threadIdx.x; i < kz->ctr_next_words; i += kBlockThreads) kz->ctr_next[i] = 0ull;
    }
    const uint32_t tw = a.tw, th = a.th;
    uint32_t n_shadow = 0, n_nodes = 0, n_prims = 0, n_primary = 0;
#ifdef RT_BLOCK_STATS
    uint32_t bs[2 * kBlockStats] = {};
#else
    uint32_t* bs = nullptr;
#endif
#ifdef RT_TIMELINE
    // diagnostic build only (tools/timeline.sh): per-wave {start, first empty
    // range, exit, units} in wall-clock ticks
    const unsigned long long tl_start = wall_clock64();
    unsigned long long tl_empty = 0, tl_units = 0;
#endif
    if (kWaveQ) {
        // wave-tile grid of the frame, or of one packed tile
        const uint32_t gw = kTiles ? a.tile_size / tw : (a.W + tw - 1) / tw;
        const uint32_t gh = kTiles ? a.tile_size / th : (a.H + th - 1) / th;
        const uint32_t nbx = (gw + 7u) / 8u, nby = (gh + 7u) / 8u;
        // superblock = 8x8 blocks of 8x8 wave tiles (one 64x64 tile at 64 spp)
        const uint32_t nsx = (nbx + 7u) / 8u, nsy = (nby + 7u) / 8u;
        const uint32_t sb_grid = nsx * nsy;  // superblocks per grid
        const uint32_t n_sb = kTiles ? a.n_tiles * sb_grid : sb_grid;
        // Two-level queue.  Level 1 hands whole superblocks (4096 wave tiles,
        // one 64x64 tile at 64 spp) to XCDs in claim order from one counter;
        // level 2 is a per-XCD ticket head over the XCD's own sequence of
        // superblocks ("slots": slot s = units [4096 s, 4096 s + 4096) of that
        // head).  An XCD's waves thus share one image region at a time (its
        // L2 holds that region's part of the scene), no unit ever runs on
        // another XCD (a stolen unit runs 3-6x slower, L2-cold), and the XCDs
        // still balance dynamically at superblock granularity (uneven scenes).
        // The ticket holding the middle unit of slot s claims slot s + 1 half
        // a slot early, so waves arriving at a new slot find it published;
        // ticket 0 claims slot 0.  A claim past the last superblock publishes
        // kSlotNone and the waves that reach it exit.  Launches of fewer
        // than 192 superblocks (a multi-GPU tile share, small frames) claim
        // single 8x8 blocks instead (slot = 64 units), numbered over the
        // blocks that hold wave tiles: the XCDs then run dry within a block
        // of each other, not within a superblock (1/8 C3 share -4%), and a
        // small frame never dequeues a superblock of padding.
        const uint32_t q = blockIdx.x & 7u;  // this workgroup's XCD (round-robin dispatch)
        unsigned long long* head = a.counters + kWaveQueueBase + q * kWaveQueueStride;
        unsigned long long* claims = a.counters + kWaveQueueClaim;
        uint32_t* slots = a.wq_slots + q * a.wq_slot_stride;
        const uint32_t chunk = a.wq_chunk;  // wave tiles per ticket (divides 32)
        const uint32_t ks = a.wq_slot_shift;  // 12: superblock slots, 6: block slots
        const uint32_t nbb = nbx * nby;       // blocks per grid
        const uint32_t n1 = ks == 12u ? n_sb : (kTiles ? a.n_tiles : 1u) * nbb;  // level-1 units
        const uint32_t half = 1u << (ks - 1u);
        // the current slot's grid (packed tile) and origin in wave tiles
        uint32_t cached_s = ~0u, k = 0, sx0 = 0, sy0 = 0, tox = 0, toy = 0, obase = 0;
        uint32_t owed = 0;  // the last real slot this wave claimed (see below)
        for (;;) {
            uint32_t t = 0;
            if ((threadIdx.x & 63u) == 0) t = static_cast<uint32_t>(atomicAdd(head, 1ull));
            const uint32_t u0 = __builtin_amdgcn_readfirstlane(t) * chunk;
            const uint32_t s = u0 >> ks, w0 = u0 & ((1u << ks) - 1u);
            const bool lead = (threadIdx.x & 63u) == 0;
            // The ticket holding slot s's middle unit claims slot s + 1 as soon
            // as it has its ticket (ticket 0 claims slot 0), before it waits
            // on anything, so claims run in parallel and land half a slot
            // early.  Two claims of one XCD can then be taken from the
            // counter out of slot order: at the counter's end slot s may hold
            // kSlotNone while slot s + 1 holds the last block.  Round 4's
            // waves all left at their first empty slot, and that block was
            // lost when every wave of the XCD had drawn one of slot s's
            // tickets (13 of 1,800 first frames; test_gpu_variants.py
            // test_wave_queue_claims_in_slot_order).  Now the wave that
            // claimed a real slot t (`owed` = t) does not leave before its
            // tickets reach slot t: every ticket up to there is drawn by a
            // live wave, so slot t's units all run.  The other waves leave at
            // their first empty slot as before.  Claiming in slot order (each
            // claim after the previous slot is published) is correct too but
            // chains the claims into serial memory round trips, C2 +5..19%;
            // keeping every wave until two empty slots in a row costs C2
            // +12% in head atomics (profiles/r05/queue_order_ab.log).
            uint32_t mine = 0;  // the slot this ticket claimed, if it got a real one
            if (lead && (u0 == 0u || (w0 <= half && half < w0 + chunk))) {
                // (test only: hold XCD 0's first claim back until the other
                // claims of its first slots would have been taken)
                if (q == 0u && u0 == 0u) {
                    for (uint32_t d = kernargs()->wq_claim_delay; d; --d) __builtin_amdgcn_s_sleep(127);
                    // (test only, RT_TEST_FAULT=queue:k: report this frame as failed)
                    if (kernargs()->test_fault_queue) frame_failed();
                }
                const uint32_t slot = u0 == 0u ? 0u : s + 1u;
                const uint32_t g = static_cast<uint32_t>(atomicAdd(claims, 1ull));
                if (slot < a.wq_slot_stride)
                    __hip_atomic_store(slots + slot, g < n1 ? g + 1u : kSlotNone, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                if (g < n1) mine = slot;
            }
            owed = max(owed, __builtin_amdgcn_readfirstlane(mine));
            uint32_t e = kSlotNone;
            if (s != cached_s) {  // resolve the slot's superblock or block (published, or soon)
                if (lead && s < a.wq_slot_stride) {
                    // the claimer holds a ticket already and publishes before it
                    // waits on anything; the cap (~1 s) only turns a broken
                    // invariant into a flagged, visibly wrong frame, not a hang
                    for (uint32_t spin = 0;; ++spin) {
                        e = __hip_atomic_load(slots + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (e != 0u) break;
                        if (spin == (1u << 22)) {
                            frame_failed();
                            e = kSlotNone;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(8);
                    }
                }
                e = __builtin_amdgcn_readfirstlane(e);
#ifndef RT_TEST_CLAIM_RULE_R4  // (test-only build of round 4's rule: the negative
                               // control of tests/test_gpu_queue_report.py)
                if (e == kSlotNone && s < owed) continue;  // a slot this wave claimed is ahead
#endif
            }
            if (s != cached_s) {
#ifdef RT_TIMELINE
                if (e == kSlotNone && !tl_empty) tl_empty = wall_clock64();
#endif
                if (e == kSlotNone) break;
                cached_s = s;
                const uint32_t g = e - 1u;
                if (ks == 12u) {
                    k = kTiles ? g / sb_grid : 0u;
                    uint32_t sg = g - k * sb_grid;
                    // claim order -> superblock: row-major, or a space-filling
                    // order (FrameArgs::sb_order, RT_SB_ORDER) in which an
                    // XCD's successive claims lie near each other
                    if (!kTiles) {
                        const uint32_t* so = kernargs()->sb_order;
                        if (so) sg = so[sg];
                    }
                    sx0 = (sg % nsx) * 64u;
                    sy0 = (sg / nsx) * 64u;
                } else {
                    // the grid's blocks that hold wave tiles, numbered
                    // superblock by superblock (row-major superblocks; edge
                    // superblocks hold vr x vc blocks)
                    k = kTiles ? g / nbb : 0u;
                    const uint32_t r = g - k * nbb;
                    const uint32_t sy = r / (8u * nbx);
                    const uint32_t vr = min(8u, nby - sy * 8u);
                    const uint32_t r1 = r - sy * 8u * nbx;
                    const uint32_t sx = r1 / (vr * 8u);
                    const uint32_t vc = min(8u, nbx - sx * 8u);
                    const uint32_t r2 = r1 - sx * vr * 8u;
                    sx0 = (sx * 8u + r2 % vc) * 8u;
                    sy0 = (sy * 8u + r2 / vc) * 8u;
                }
                if (kTiles) {  // the packed tile's origin in the image, once per slot
                    const uint32_t tile = a.tiles[k];
                    const uint32_t ts = a.tile_size;
                    tox = (tile % a.tiles_x) * ts;
                    toy = (tile / a.tiles_x) * ts;
                    obase = k * ts * ts - toy * ts - tox;
                }
            }
            for (uint32_t cur = w0; cur < w0 + chunk; ++cur) {
                const uint32_t b = cur >> 6, w = cur & 63u;  // b = 0 in block slots
                const uint32_t wx = sx0 + (b & 7u) * 8u + (w & 7u);
                const uint32_t wy = sy0 + (b >> 3) * 8u + (w >> 3);
                if (wx >= gw || wy >= gh) continue;  // padding of an edge block
                const uint32_t olx = wx * tw, oly = wy * th;
                const uint32_t ox = olx + tox, oy = oly + toy;
#ifdef RT_TIMELINE
                const unsigned long long tu0 = wall_clock64();
#endif
                if (kSort)
                    shade_pixel_sorted<kTiles, kChunk, kStats, kProg>(
                        a, wl, stk, ox, oy, obase, n_primary, n_shadow, n_nodes, n_prims, bs, lbs);
                else
                    shade_wave_tile<kTiles, kChunk, kStats, kProg, RT_CAM8 != 0 && !kSort>(
                        a, acc, stk, ox, oy, obase, n_primary, n_shadow, n_nodes, n_prims, bs, lbs);
#ifdef RT_TIMELINE
                // per unit {start, end, hw_id << 32 | xcc << 16 | wave index}
                // after the 65536 per-wave records
                const uint32_t sbt = k * sb_grid + (wy >> 6) * nsx + (wx >> 6);
                const unsigned long long uid = (unsigned long long)sbt * 4096u +
                                               (((wy >> 3) & 7u) * 8u + ((wx >> 3) & 7u)) * 64u +
                                               (wy & 7u) * 8u + (wx & 7u);
                if (a.timeline && (threadIdx.x & 63u) == 0 && uid < (1ull << 22)) {
                    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
                    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID
                    a.timeline[4ull * 65536 + 3 * uid] = tu0;
                    a.timeline[4ull * 65536 + 3 * uid + 1] = wall_clock64();
                    a.timeline[4ull * 65536 + 3 * uid + 2] =
                        ((unsigned long long)hw << 32) | (xcc << 16) | (blockIdx.x * 4u + wave);
                }
#endif
            }
        }
    } else {
        __shared__ uint32_t tile_slot;
        const uint32_t bts = a.bts;  // block-tile side (16, or 8/4 for small frames)
        const uint32_t wtx = bts / tw, wtiles = wtx * (bts / th);
        const uint32_t per_tile = kTiles ? (a.tile_size / bts) * (a.tile_size / bts) : 0u;
        const uint32_t bx_n = (a.W + bts - 1) / bts;
        const uint32_t n_bt = kTiles ? a.n_tiles * per_tile : bx_n * ((a.H + bts - 1) / bts);
        for (;;) {
            __syncthreads();  // every wave is done with the previous tile_slot
            if (threadIdx.x == 0)
                tile_slot = static_cast<uint32_t>(atomicAdd(a.counters + kQueueSlot, 1ull));
            __syncthreads();
            const uint32_t bt = tile_slot;
            if (bt >= n_bt) break;
            uint32_t ox, oy, obase = 0;  // block-tile origin (frame / packed tile)
            if (kTiles) {
                const uint32_t ts = a.tile_size, tpr = ts / bts;
                const uint32_t k = bt / per_tile;
                const uint32_t b = bt - k * per_tile;
                const uint32_t tile = a.tiles[k];
                const uint32_t tox = (tile % a.tiles_x) * ts, toy = (tile / a.tiles_x) * ts;
                ox = tox + (b % tpr) * bts;
                oy = toy + (b / tpr) * bts;
                obase = k * ts * ts - toy * ts - tox;
            } else {
                ox = (bt % bx_n) * bts;
                oy = (bt / bx_n) * bts;
            }
            for (uint32_t wt = wave; wt < wtiles; wt += kBlockThreads / 64) {
                const uint32_t wox = (wt % wtx) * tw, woy = (wt / wtx) * th;
#ifdef RT_TIMELINE
                const unsigned long long tu0 = wall_clock64();
#endif
                shade_wave_tile<kTiles, kChunk, kStats, kProg>(
                    a, acc, stk, ox + wox, oy + woy, obase, n_primary, n_shadow, n_nodes,
                    n_prims, bs, lbs);
#ifdef RT_TIMELINE
                // per wave tile of a block tile: {start, end, hw_id << 32 | xcc << 16 |
                // wave index}, unit id = block tile * 16 + wave tile (tools/timeline.py)
                const unsigned long long uid = (unsigned long long)bt * 16u + wt;
                if (a.timeline && (threadIdx.x & 63u) == 0 && uid < (1ull << 22)) {
                    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
                    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // XCC_ID
                    a.timeline[4ull * 65536 + 3 * uid] = tu0;
                    a.timeline[4ull * 65536 + 3 * uid + 1] = wall_clock64();
                    a.timeline[4ull * 65536 + 3 * uid + 2] =
                        ((unsigned long long)hw << 32) | (xcc << 16) | (blockIdx.x * 4u + wave);
                }
#endif
            }
        }
    }
    if (kStats) flush_counters(a, n_primary, n_shadow, n_nodes, n_prims);
#ifdef RT_BLOCK_STATS
    if (a.bstats) {
#pragma unroll
        for (uint32_t i = 0; i < 2 * kBlockStats; ++i) {
            const unsigned long long v = wave_sum(bs[i]);
            if ((threadIdx.x & 63u) == 0) atomicAdd(a.bstats + i, v);
        }
    }
#endif
#ifdef RT_TIMELINE
    tl_units = n_primary / 64u;  // samples cast by the wave / 64
    if (a.timeline && (threadIdx.x & 63u) == 0) {
        unsigned long long* e = a.timeline + 4ull * (blockIdx.x * (kBlockThreads / 64) + wave);
        e[0] = tl_start;
        e[1] = tl_empty;
        e[2] = wall_clock64();
        e[3] = tl_units;
    }
#endif
}

template <bool kTiles, int kMinW, int kChunk, bool kStats = true, bool kProg = false,
          bool kWaveQ = false, bool kSort = false>
__global__ void __launch_bounds__(kBlockThreads, kMinW) scene_kernel(FrameArgs a) {
    scene_body<kTiles, kChunk, kStats, kProg, kWaveQ, kSort>(a);
}

// The timed default for spp >= 8 (variant 13, plain frames): 8 waves per SIMD,
// SGPRs capped so that they fit (see above).
template <bool kTiles, bool kProg = false, bool kSort = false>
__global__ void __launch_bounds__(kBlockThreads, 8) __attribute__((amdgpu_num_sgpr(80)))
    scene_kernel_w8(FrameArgs a) {
    scene_body<kTiles, 2, false, kProg, true, kSort>(a);
}

// Camera-relative screen records of every leaf reference (and the kPrimPad
// tail) for camera origin o (SceneArgs::prim_cam):
// {o - c in f32, exactly isect's oc}, and C' = |o - c|^2 - r^2 minus the
// slack, computed in f64 and rounded toward -inf, so C' <= the bound the
// screen's soundness needs.  One thread per reference: 16 B read, 16 B written.
__global__ void __launch_bounds__(kBlockThreads)
    cam_screen_kernel(const float4* __restrict__ prim_sp, uint32_t n, float ox, float oy, float oz,
                      float4* __restrict__ out) {
    const uint32_t i = blockIdx.x * kBlockThreads + threadIdx.x;
    if (i >= n) return;
    const float4 c = prim_sp[i];
    const float x = ox - c.x, y = oy - c.y, z = oz - c.z;
    const double oo = static_cast<double>(x) * x + static_cast<double>(y) * y + static_cast<double>(z) * z;
    const double rr = static_cast<double>(c.w) * c.w;
    const double u = 1.0 / 16777216.0;  // 2^-24, the f32 unit roundoff
    const double cd = oo - rr - (kScreenSlackOc * u) * oo - (kScreenSlackR * u) * rr;
    out[i] = make_float4(x, y, z, kCamMode == 2 ? c.w : __double2float_rd(cd));
}

// Light-plane screen records (SceneArgs::prim_shd): per
// reference the centre's {u, v} = {c.e1, c.e2} (f64, rounded to nearest) and
// rr' = ((r (1 + 4u) + delta)^2 (1 + 4u)) rounded up, delta = the slack for
// this scene (kShadowSlackM u M).  One thread per reference.
__global__ void __launch_bounds__(kBlockThreads)
    shd_screen_kernel(const float4* __restrict__ prim_sp, uint32_t n, float e0, float e1, float e2,
                      float e3, float e4, float e5, double delta, float4* __restrict__ out,
                      float2* __restrict__ out8, uint32_t* __restrict__ rr_max) {
    const uint32_t i = blockIdx.x * kBlockThreads + threadIdx.x;
    uint32_t rb = 0u;
    if (i < n) {
        const float4 c = prim_sp[i];
        const double u = static_cast<double>(c.x) * e0 + static_cast<double>(c.y) * e1 + static_cast<double>(c.z) * e2;
        const double v = static_cast<double>(c.x) * e3 + static_cast<double>(c.y) * e4 + static_cast<double>(c.z) * e5;
        const double ur = 1.0 / 16777216.0;
        const double rg = static_cast<double>(c.w) * (1.0 + 4.0 * ur) + delta;
        const float rr = __double2float_ru(rg * rg * (1.0 + 4.0 * ur));
        out[i] = make_float4(static_cast<float>(u), static_cast<float>(v), rr, 0.0f);
        if (out8) {
            const float uf = static_cast<float>(u), vf = static_cast<float>(v);
            if (RT_SHD8_PER) {
                // this sphere's rr', grown by the stored centre's error (its
                // 8 low mantissa bits a coordinate carry rr': <= 2^-15 |u|
                // each), rounded up to bf16 (its soundness test: tests/test_cam_screen.py)
                const double ec = (1.0 / 16384.0) * (fabs(static_cast<double>(uf)) + fabs(static_cast<double>(vf)));
                const double rg8 = rg + ec;
                const float r8 = __double2float_ru(rg8 * rg8 * (1.0 + 4.0 * ur));
                uint32_t b8 = __float_as_uint(r8);
                if (b8 & 0xFFFFu) b8 = (b8 & 0xFFFF0000u) + 0x10000u;
                if (!(isfinite(r8) && b8 < 0x7F800000u)) b8 = 0x7F800000u;  // always pass
                out8[i] = make_float2(__uint_as_float((__float_as_uint(uf) & ~0xFFu) | (b8 >> 24)),
                                      __uint_as_float((__float_as_uint(vf) & ~0xFFu) | ((b8 >> 16) & 0xFFu)));
            } else {
                out8[i] = make_float2(uf, vf);
            }
        }
        rb = __float_as_uint(rr);
    }
    if (out8) {
        // the largest rr' (non-negative floats order as their bits; a NaN
        // radius, the test-only pad fill, orders above every number): the
        // block's maximum into rr_max[blockIdx.x], reduced by
        // max_bits_kernel (atomics on one word serialise across the XCDs:
        // one per record, or one per wave, took C5d's 4.9 M records 0.87 ms)
        __shared__ uint32_t wmax[kBlockThreads / 64];
        for (int d = 32; d > 0; d >>= 1) rb = max(rb, static_cast<uint32_t>(__shfl_xor(static_cast<int>(rb), d, 64)));
        if ((threadIdx.x & 63u) == 0u) wmax[threadIdx.x >> 6] = rb;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t m = 0u;
            for (uint32_t w = 0; w < kBlockThreads / 64; ++w) m = max(m, wmax[w]);
            rr_max[blockIdx.x] = m;
        }
    }
}

// out[0] = the largest of in[0 .. n) (one block)
__global__ void __launch_bounds__(kBlockThreads)
    max_bits_kernel(const uint32_t* __restrict__ in, uint32_t n, uint32_t* __restrict__ out) {
    __shared__ uint32_t wmax[kBlockThreads / 64];
    uint32_t m = 0u;
    for (uint32_t i = threadIdx.x; i < n; i += kBlockThreads) m = max(m, in[i]);
    for (int d = 32; d > 0; d >>= 1) m = max(m, static_cast<uint32_t>(__shfl_xor(static_cast<int>(m), d, 64)));
    if ((threadIdx.x & 63u) == 0u) wmax[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (uint32_t w = 1; w < kBlockThreads / 64; ++w) m = max(m, wmax[w]);
        out[0] = m;
    }
}

hipError_t launch_shd_screen(const float4* prim_sp, uint32_t n, const float e[6], double delta,
                             float4* out, float2* out8, uint32_t* rr_max, hipStream_t st) {
    // rr_max: (blocks + 1) words, the scene's largest rr' bits in the last
    if (n) {
        const uint32_t nb = (n + kBlockThreads - 1) / kBlockThreads;
        hipLaunchKernelGGL(shd_screen_kernel, dim3(nb), dim3(kBlockThreads), 0, st, prim_sp, n, e[0],
                           e[1], e[2], e[3], e[4], e[5], delta, out, out8, rr_max);
        if (out8)
            hipLaunchKernelGGL(max_bits_kernel, dim3(1), dim3(kBlockThreads), 0, st, rr_max, nb, rr_max + nb);
    }
    return hipGetLastError();
}

hipError_t launch_cam_screen(const float4* prim_sp, uint32_t n, const float o[3], float4* out,
                             hipStream_t st) {
    if (n) {
        hipLaunchKernelGGL(cam_screen_kernel, dim3((n + kBlockThreads - 1) / kBlockThreads),
                           dim3(kBlockThreads), 0, st, prim_sp, n, o[0], o[1], o[2], out);
    }
    return hipGetLastError();
}

// Image-plane screen records (SceneArgs::prim_cam8).
// For basis B (f32 rows, orthonormal to f32 rounding) and camera origin o,
// a sphere's centre direction a = B(c - o)/|c - o| projects to q = a.xy/a.z.
// A ray the exact test accepts passes within r' = r (1 + 1e-6) of c, so its
// direction b is within theta (sin theta = r'/|c - o|) of a, and for unit
// vectors |q_a - q_b| <= |a x b| / (a_z b_z) <= sin theta / (a_z cos(beta +
// theta)), beta the angle of a from B's z axis.  rho adds the f32 errors of
// the lane's point (4e-6 (1 + |q| + rho)^2, ~5x the bound), the stored
// centre's (its 8 low mantissa bits carry rho^2: <= 2^-14 |q| a component)
// and 1e-5 relative; rho^2 is rounded up to bf16.  Spheres near or behind
// the camera plane, or a frame whose rays B does not keep in front (ok = 0),
// get rho^2 = +inf: always passed.
__global__ void __launch_bounds__(kBlockThreads)
    cam8_screen_kernel(const float4* __restrict__ prim_sp, uint32_t n, float ox, float oy, float oz,
                       float b0, float b1, float b2, float b3, float b4, float b5, float b6, float b7,
                       float b8, uint32_t ok, float2* __restrict__ out) {
    const uint32_t i = blockIdx.x * kBlockThreads + threadIdx.x;
    if (i >= n) return;
    const float4 c = prim_sp[i];
    const double vx = static_cast<double>(c.x) - ox, vy = static_cast<double>(c.y) - oy,
                 vz = static_cast<double>(c.z) - oz;
    const double X = static_cast<double>(b0) * vx + static_cast<double>(b1) * vy + static_cast<double>(b2) * vz;
    const double Y = static_cast<double>(b3) * vx + static_cast<double>(b4) * vy + static_cast<double>(b5) * vz;
    const double Z = static_cast<double>(b6) * vx + static_cast<double>(b7) * vy + static_cast<double>(b8) * vz;
    const double dist = sqrt(vx * vx + vy * vy + vz * vz);
    const double rp = static_cast<double>(c.w) * (1.0 + 1e-6);
    uint32_t hx = 0u, hy = 0u, rb = 0x7F800000u;  // rho^2 = +inf: always pass
    bool pass_all = !ok || !(dist > rp * 1.0001) || !(Z > 0.0) || !isfinite(dist) || !(c.w >= 0.0f);
    if (!pass_all) {
        const double az = Z / dist;
        const double beta = acos(fmin(1.0, az));
        const double th = asin(fmin(1.0, rp / dist));
        if (!(beta + th < 1.45)) {  // ~83 degrees: the bound's cos(beta + theta) too small
            pass_all = true;
        } else {
            const float qx = static_cast<float>(X / Z), qy = static_cast<float>(Y / Z);
            const double q = fabs(static_cast<double>(qx)) + fabs(static_cast<double>(qy));
            const double rho_g = sin(th) / (az * cos(beta + th));
            const double eps_c = 1.5 * (1.0 / 16384.0) * q;
            const double m = 1.0 + q + rho_g;
            const double rho = rho_g * (1.0 + 1e-5) + eps_c + 4e-6 * m * m;
            const float r2 = __double2float_ru(rho * rho * (1.0 + 1e-6));
            uint32_t bits = __float_as_uint(r2);
            if (bits & 0xFFFFu) bits = (bits & 0xFFFF0000u) + 0x10000u;  // bf16, rounded up
            if (isfinite(r2) && bits < 0x7F800000u) {
                rb = bits;
                hx = __float_as_uint(qx);
                hy = __float_as_uint(qy);
            } else {
                pass_all = true;
            }
        }
    }
    // low bytes: rho^2's bf16, high byte in x, low byte in y
    const uint32_t sx = (hx & ~0xFFu) | (rb >> 24), sy = (hy & ~0xFFu) | ((rb >> 16) & 0xFFu);
    out[i] = make_float2(__uint_as_float(sx), __uint_as_float(sy));
}

hipError_t launch_cam8_screen(const float4* prim_sp, uint32_t n, const float o[3], const float B[9],
                              uint32_t ok, float2* out, hipStream_t st) {
    if (n) {
        hipLaunchKernelGGL(cam8_screen_kernel, dim3((n + kBlockThreads - 1) / kBlockThreads),
                           dim3(kBlockThreads), 0, st, prim_sp, n, o[0], o[1], o[2], B[0], B[1], B[2],
                           B[3], B[4], B[5], B[6], B[7], B[8], ok, out);
    }
    return hipGetLastError();
}

// Albedo by leaf reference (SceneArgs::prim_al): out[i] = albedo[prim_idx[i]]
// for the n real reference slots (a packed layout's gaps name sphere 0).
__global__ void __launch_bounds__(kBlockThreads)
    albedo_refs_kernel(const uint32_t* __restrict__ prim_idx, const uint32_t* __restrict__ albedo,
                       uint32_t n, uint32_t n_spheres, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * kBlockThreads + threadIdx.x;
    if (i >= n) return;
    const uint32_t k = prim_idx[i];
    out[i] = k < n_spheres ? albedo[k] : 0u;
}

hipError_t launch_albedo_refs(const uint32_t* prim_idx, const uint32_t* albedo, uint32_t n,
                              uint32_t n_spheres, uint32_t* out, hipStream_t st) {
    if (n) {
        hipLaunchKernelGGL(albedo_refs_kernel, dim3((n + kBlockThreads - 1) / kBlockThreads),
                           dim3(kBlockThreads), 0, st, prim_idx, albedo, n, n_spheres, out);
    }
    return hipGetLastError();
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
    if (tile == 0xFFFFFFFFu) return;  // RT_TILE_SKIP: a padding slot
    const uint32_t x = (tile % tiles_x) * ts + r % ts;
    const uint32_t y = (tile / tiles_x) * ts + r / ts;
    if (x < W && y < H) img[(size_t)y * W + x] = packed[i];
}

// ---------------------------------------------------------------------------
// launchers (called from rt_capi.cpp)
// ---------------------------------------------------------------------------

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

size_t scene_lds_bytes(const FrameArgs& a) {
    const size_t colours = kBlockThreads * sizeof(float4);  // pixel sums
    const uint32_t levels = stack_levels(a.sc);
    return colours + static_cast<size_t>(levels) * kBlockThreads * sizeof(uint2) + kLeafBufBytes;
}

// Resident workgroups on the device for a kernel at a given LDS size.  The
// occupancy query is a host call: cache it per (kernel, LDS bytes, device) so
// the launch path stays a single hipLaunchKernelGGL.
template <typename K>
static uint32_t resident_blocks(K kernel, size_t lds) {
    struct Key {
        const void* k;
        size_t lds;
        int dev;
    };
    static std::mutex mu;
    static std::vector<std::pair<Key, uint32_t>> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    const void* kp = reinterpret_cast<const void*>(kernel);
    {
        std::lock_guard<std::mutex> g(mu);
        for (const auto& e : cache)
            if (e.first.k == kp && e.first.lds == lds && e.first.dev == dev) return e.second;
    }
    hipDeviceProp_t prop;
    int cus = 256;
    if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlockThreads, lds) != hipSuccess ||
        per_cu <= 0)
        per_cu = 4;
    const uint32_t n = static_cast<uint32_t>(cus * per_cu);
    std::lock_guard<std::mutex> g(mu);
    cache.push_back({{kp, lds, dev}, n});
    return n;
}

static uint32_t cus_of_device() {
    static std::mutex mu;
    static std::vector<std::pair<int, uint32_t>> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> g(mu);
    for (const auto& e : cache)
        if (e.first == dev) return e.second;
    hipDeviceProp_t prop;
    const uint32_t n = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
    cache.push_back({dev, n});
    return n;
}

constexpr size_t kOneSppLds = (160u * 1024u / 3u) & ~size_t(15);  // 3 workgroups per CU

// Block tiles in the frame (or in the packed tile list) for block-tile side b.
static uint32_t count_block_tiles(const FrameArgs& a, uint32_t b) {
    if (a.tiles) return a.n_tiles * (a.tile_size / b) * (a.tile_size / b);
    return ((a.W + b - 1) / b) * ((a.H + b - 1) / b);
}

// Persistent launch: grid = resident workgroups; the block-tile side shrinks
// (16 -> 8 -> 4 pixels, never below two wave tiles) until the tile queue holds
// >= 8 tiles per resident workgroup, so the dynamic queue can even out costly
// image regions to the end (A/B, profiles/r01/bts_ab.log: 1080p 64 spp picks
// 8x8 tiles, -6.4% vs 16x16; a 1/4 or 1/8 multi-GPU share picks 4x4).
template <typename K>
static void launch_persistent(K kernel, const FrameArgs& a_in, uint32_t, size_t lds,
                              hipStream_t st) {
    FrameArgs a = a_in;
    // 1 spp: a wave's 64 lanes are 64 different pixels, whose walks thrash
    // the L1 when 5 workgroups share a CU; the dynamic LDS is padded so that
    // at most 3 are resident (C2: 0.358 -> 0.274 ms; 2 or 4 per CU slower,
    // 4 spp unchanged; profiles/r01/c2_wg_cap_ab.log)
    if (a.spw == 1u && !(a.sc.opt & kOptNoWgCap)) lds = std::max(lds, kOneSppLds);
    const uint32_t res = resident_blocks(kernel, lds);
    const uint32_t min_side = 2u * std::max(a.tw, a.th);
    a.bts = kTileSide;
    const uint32_t force = (a.sc.opt >> kOptBtsShift) & 7u;
    if (force && (kTileSide >> (force - 1u)) >= min_side)
        a.bts = kTileSide >> (force - 1u);
    else
        while (a.bts / 2u >= min_side && count_block_tiles(a, a.bts) < 8u * res) a.bts /= 2u;
    const uint32_t grid = std::min(count_block_tiles(a, a.bts), res);
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlockThreads), lds, st, a);
}

// Per-wave queue launch: grid = resident workgroups, capped by the work.
template <typename K>
static void launch_waveq(K kernel, const FrameArgs& a, size_t lds, hipStream_t st,
                         uint32_t per_simd = 7) {
    const uint32_t res = resident_blocks(kernel, lds);
    uint64_t units;
    if (a.tiles)
        units = (uint64_t)a.n_tiles * (a.tile_size / a.tw) * (a.tile_size / a.th);
    else
        units = (uint64_t)((a.W + a.tw - 1) / a.tw) * ((a.H + a.th - 1) / a.th);
    // (the grid only sizes the launch; padding units of edge blocks are skipped)
    const uint64_t want = (units + kBlockThreads / 64 - 1) / (kBlockThreads / 64);
    // The occupancy query counts 8 workgroups per CU for the 7-wave builds
    // (60-65 VGPRs), but their 94 SGPRs leave room for 7: the 8th per CU
    // only starts when another exits, finds nothing and adds 8 queue atomics
    // to the tail (profiles/r02/timeline_hwid.log).  Capped at the build's
    // waves per SIMD: C3 -0.8%, 1/8 share -5% (profiles/r02/steal_ab.log,
    // measured with the static per-XCD ranges that preceded the two-level queue)
    const uint64_t cap = per_simd ? static_cast<uint64_t>(cus_of_device()) * per_simd : res;
    const uint32_t grid =
        static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>(std::min<uint64_t>(res, cap), want)));
    FrameArgs b = a;
    if (!((a.sc.opt >> kOptChunkShift) & 7u)) {
        // auto ticket size, second half: a small launch (a multi-GPU share)
        // has few units per wave, and big tickets lengthen its tail. N-way
        // C3 shares: 4 per ticket best at 1/2 and 1/4, 2 at 1/8 (36 units a
        // wave; profiles/r01/shard_chunk.log)
        const uint64_t per_wave = units / (static_cast<uint64_t>(grid) * (kBlockThreads / 64));
        const uint32_t cap = per_wave >= 64 ? 4u : per_wave >= 16 ? 2u : 1u;
        b.wq_chunk = std::min(b.wq_chunk, cap);
    }
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlockThreads), lds, st, b);
}

// Sorted rounds (above): a wave-queue frame of one pixel per wave and 2..4
// rounds, wherever the per-wave LDS still lets 8 workgroups share a CU.
// RT_SORT=0 turns it off (A/B; images and counters are the same).
static uint32_t env_u32(const char* name, uint32_t dflt) {
    const char* e = getenv(name);
    return e && *e ? static_cast<uint32_t>(strtoul(e, nullptr, 10)) : dflt;
}
size_t sort_lds_bytes(const FrameArgs& a) {
    return static_cast<size_t>(stack_levels(a.sc, true)) * kBlockThreads * sizeof(uint2) +
           (kBlockThreads / 64) * kSortWaveBytes + kLeafBufBytes;
}
static bool sorted_rounds(const FrameArgs& a) {
    static const uint32_t on = env_u32("RT_SORT", 1u);
    return on && a.spp >= 8u && a.spw == 64u && a.rounds >= 2u && a.rounds <= kSortMaxRounds &&
           sort_lds_bytes(a) * 8u <= 160u * 1024u &&
           (a.accum != nullptr || a.variant == kVariantWaveQ);
}

template <bool kTiles>
static void launch_scene_t(const FrameArgs& a, uint32_t n_bt, size_t lds, hipStream_t st) {
    if (sorted_rounds(a)) {
        const size_t sl = sort_lds_bytes(a);
        if (a.accum) {
            if (a.count_work)
                launch_waveq(scene_kernel<kTiles, 7, 2, true, true, true, true>, a, sl, st);
            else
                launch_waveq(scene_kernel_w8<kTiles, true, true>, a, sl, st, 8);
        } else if (a.count_work) {
            launch_waveq(scene_kernel<kTiles, 7, 2, true, false, true, true>, a, sl, st);
        } else {
            launch_waveq(scene_kernel_w8<kTiles, false, true>, a, sl, st, 8);
        }
        return;
    }
    if (a.accum) {  // progressive frames: the unified walk, whatever the variant
        if (a.spp >= 8u) {  // the wave queue, like variant 13
            if (a.count_work)
                launch_waveq(scene_kernel<kTiles, 7, 2, true, true, true>, a, lds, st);
            else
                launch_waveq(scene_kernel_w8<kTiles, true>, a, lds, st, 8);
        } else if (a.count_work) {
            launch_persistent(scene_kernel<kTiles, 1, 2, true, true>, a, n_bt, lds, st);
        } else {
            launch_persistent(scene_kernel<kTiles, 1, 2, false, true>, a, n_bt, lds, st);
        }
        return;
    }
    switch (a.variant) {
        case kVariantLaneUnified:  // block-tile queue, counting in every frame
            launch_persistent(scene_kernel<kTiles, 1, 2>, a, n_bt, lds, st);
            break;
        case kVariantLaneUnified2NoStats:  // the spp < 8 default: 7 with counters only in stats frames
            if (a.count_work)
                launch_persistent(scene_kernel<kTiles, 1, 2, true>, a, n_bt, lds, st);
            else
                launch_persistent(scene_kernel<kTiles, 1, 2, false>, a, n_bt, lds, st);
            break;
        case kVariantWaveQLow:  // the spp < 8 default (round 4): the per-wave queue, 8 waves/SIMD
            // No workgroup barrier per block tile: the timeline of the block-tile
            // queue (variant 10) showed waves idle 28% of the C2 launch, mostly
            // waiting at that barrier for the slowest of a tile's 4 wave tiles
            // (gaps p90 5.2 us against units of p50 5.8 us,
            // profiles/r04/c2_timeline.log).  With it C2 0.155 -> 0.107 ms; the
            // 3-workgroups-per-CU cap of the block-tile queue costs it again
            // here (0.152 ms), so it has none (profiles/r04/c2_waveq_ab.log).
            if (a.count_work)
                launch_waveq(scene_kernel<kTiles, 7, 2, true, false, true>, a, lds, st);
            else
                launch_waveq(scene_kernel_w8<kTiles>, a, lds, st, 8);
            break;
        case kVariantWaveQ:  // the spp >= 8 default: per-wave scheduling over per-XCD queues.
            // Timed (plain) frames: 8 waves/SIMD with SGPRs capped at 80
            // (kSceneSgprs); stats frames keep 7 (their counters need the
            // registers; C3 -2.8%, C5 -5.4% against 6, profiles/r01/occupancy_ab.log)
            if (a.count_work)
                launch_waveq(scene_kernel<kTiles, 7, 2, true, false, true>, a, lds, st);
            else
                launch_waveq(scene_kernel_w8<kTiles>, a, lds, st, 8);
            break;
        default:  // rejected by variant_available() before any launch
            break;
    }
}

// Variants compiled into this build (rt_create refuses the others).  The
// measured-and-rejected alternatives of DESIGN.md 5.1 (packets, LDS / scalar /
// one-lane uniform leaves, bundle prefilter, 6- and 8-wave builds) were
// removed in round 3; their A/B logs stay under profiles/.
bool variant_available(uint32_t v) {
    return v == 0 || v == kVariantLaneUnified || v == kVariantLaneUnified2NoStats ||
           v == kVariantWaveQ || v == kVariantWaveQLow;
}

hipError_t launch_scene(const FrameArgs& a_in, hipStream_t st) {
    FrameArgs a = a_in;
    if (a.accum) a.variant = kVariantLaneUnified;  // what launch_scene_t runs (LDS sizing)
    // wave mapping: spw samples x ppw pixels per wave (see scene_kernel)
    wave_tile_shape(a.spp, a.spw, a.g, a.ppw, a.tw, a.th);
    a.rounds = (a.spp + a.spw - 1) / a.spw;
    // wave-queue ticket size: adjacent wave tiles back to back on one wave
    // reuse its CU's L1; a ticket of about four rounds of work balances that
    // against the queue tail (C3, 1 round: 4 per ticket -4.1%; C5, 4 rounds:
    // 1 per ticket, more is slower; profiles/r01/chunk_ab.log)
    const uint32_t ck = (a.sc.opt >> kOptChunkShift) & 7u;
    a.wq_chunk = ck ? 1u << (ck - 1u) : std::max(1u, 4u / std::max(1u, std::min(a.rounds, 4u)));
    const size_t lds = scene_lds_bytes(a);
    if (a.tiles)
        launch_scene_t<true>(a, 0, lds, st);
    else
        launch_scene_t<false>(a, 0, lds, st);
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
