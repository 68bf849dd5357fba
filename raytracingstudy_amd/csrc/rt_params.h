// rt_params.h — kernel-argument structs shared by the C-ABI host code and the
// HIP kernels.  Everything the hot loop needs travels BY VALUE in one kernel
// argument block (SGPR-resident), replacing the reference's device-heap
// Camera/Octree objects reached through thrust::device_ptr<T*> double
// indirection (src/renderer.cu:57,65-66,84-109).
#pragma once
#include <stdint.h>

namespace rtamd {

constexpr int kBlockThreads = 256;  // 4 waves of 64
constexpr uint32_t kTileSide = 16;  // scene kernel: largest block tile (16x16 pixels per workgroup)
constexpr uint32_t kMaxDepth = 16;  // octree depth limit (grid coordinates stay < 2^16, exact in f32)
constexpr float kShadowEps = 1e-5f; // shadow-ray origin offset along the normal (world units)
constexpr uint32_t kNoHit = 0xFFFFFFFFu;

// scene kernel variants (rt_config.flags bits 16..19, RT_FLAG_VARIANT_SHIFT);
// 0 picks 13 for spp >= 8, else 10.  Numbers of the variants measured and
// removed are not reused.
constexpr uint32_t kVariantLaneUnified = 7;   // one walk instance for primary + shadow, 2 in flight
constexpr uint32_t kVariantLaneUnified2NoStats = 10; // spp < 8 default: 7 with counters only in stats frames
constexpr uint32_t kVariantWaveQ = 13;     // unified walk scheduled per wave over per-XCD queues
                                           // (default for spp >= 8)
constexpr uint32_t kVariantWaveQLow = 4;   // the per-wave queue for spp < 8 too (no workgroup
                                           // barrier per block tile; the spp < 8 default
                                           // since round 4)
// prim_sp padding after the last leaf list: the leaf loads run kChunk - 1 = 1
// sphere past a leaf's end (rt_capi.cpp fills it)
constexpr uint32_t kPrimPad = 4;

// A/B toggles (rt_config.flags bits 20..27), results identical either way
constexpr uint32_t kOptDeviceBuildRefuse = 1u << 0;  // bit 0: the device build reports running out
                                                     // of HBM (tests its host fallback)
constexpr uint32_t kOptBtsShift = 1;       // bits 1..3: force the block-tile side (A/B):
                                           // 0 auto, 1 = 16, 2 = 8, 3 = 4, 4 = 2 pixels
constexpr uint32_t kOptNoWgCap = 1u << 7; // bit 7: 1-spp frames without the 3-workgroups-per-CU cap
constexpr uint32_t kOptChunkShift = 4;     // bits 4..6: wave-queue tiles per ticket: 0 auto
                                           // (4 / rounds, at least 1), k = 1..4 -> 1 << (k - 1);
                                           // 5..7 are refused (a ticket must not span half
                                           // a slot: the two-level queue's claim rule)
constexpr uint32_t kOptChunkMax = 4;

// Depth-K cell table (cell_table.hip): entry = {record.x, record.y (24 bits) |
// depth << 24 | kind << 29} of the node covering each depth-K cell.
constexpr uint32_t kCellInternal = 0;  // internal node at depth K
constexpr uint32_t kCellLeaf = 1;      // leaf at depth <= K containing the cell
constexpr uint32_t kCellEmpty = 2;     // empty child (depth <= K) containing the cell
constexpr uint32_t kCellRecMask = 0xFFFFFFu;
constexpr uint32_t kCellDepthShift = 24;
constexpr uint32_t kCellKindShift = 29;
constexpr uint32_t kCellTableMaxK = 7;        // 2^21 entries, 16 MiB
constexpr uint32_t kCellTableAuto = 0xFFFFFFFFu;
constexpr uint32_t kCellTableOff = 0;

// counters[] layout: [0..7] unused, [kQueueSlot] block-tile queue head (own
// cache line), then 8 per-XCD wave-queue heads, one per 128-byte line
constexpr uint32_t kQueueSlot = 8;
constexpr uint32_t kWaveQueueBase = 16;
constexpr uint32_t kWaveQueueStride = 16;
// two-level wave queue: superblocks handed to XCDs (claim counter, own line)
constexpr uint32_t kWaveQueueClaim = kWaveQueueBase + 8 * kWaveQueueStride;
// stats frames: work counters {primary, shadow, nodes, prims} per XCD group
// (blockIdx % 8), one 128-byte line each, summed by the host
constexpr uint32_t kStatLineBase = kWaveQueueClaim + 16;
constexpr uint32_t kStatLineStride = 16;
constexpr uint32_t kCounterWords = kStatLineBase + 8 * kStatLineStride;
constexpr uint32_t kSlotNone = 0xFFFFFFFFu;  // slot table: no superblock left

// Diagnostic build (-DRT_BLOCK_STATS, tools/block_stats.py): how many times a
// wave executed each block of the walk (a block runs once for the wave when
// any lane is in it), and how many lanes were active.  [2*i] = executions of
// block i, [2*i+1] = active lanes summed over those executions.
enum BlockStat : uint32_t {
    kBsIter = 0,      // walk loop trips
    kBsJump,          // trips taking the cell-table jump path
    kBsJumpDescend,   // mid-plane steps inside a jump (while depth < K)
    kBsDescend,       // trips taking the record-descent path
    kBsInternal,      // descents into an internal child (continue)
    kBsLeaf,          // leaves entered
    kBsLeafChunk,     // leaf chunk trips (kChunk spheres each)
    kBsTest,          // sphere tests (one per slot of a chunk)
    kBsSqrt,          // tests past h >= 0 (square root path)
    kBsAccept,        // tests returning a hit
    kBsExit,          // exit-plane steps
    kBsPop,           // pops reading the LDS stack (m > 1)
    kBsWalk,          // walks started (root box entered)
    kBsPhase,         // sample phases (primary / shadow) run by the wave
    kBsIterShadow,    // walk loop trips of shadow (any-hit) walks
    kBsTestShadow,    // sphere tests of shadow walks
    kBsPhaseShadow,   // shadow phases run by the wave
    // vector-memory loads by class (round 5; one wave
    // execution = one load instruction): sphere pairs are 2 x kBsLeafChunk and
    // table entries kBsJump; these add the rest
    kBsNodeRead,      // child record reads of a descent (oracle-counted)
    kBsNodeReread,    // child record re-reads below a re-entered ancestor (not counted by the oracle)
    kBsExactLoad,     // chunks whose camera-relative screen passed: 2 sphere loads for the exact tests
    kBsPastEnd,       // chunks whose slot 1 lies past the leaf's end (lanes: how many)
    kBsTieLoad,       // exact-t ties: 2 prim_idx loads
    kBsHitIdx,        // nearest walks ending on a hit: 1 prim_idx load
    kBsShadeLoad,     // shading reads of a hit's sphere record / albedo (1 load each)
    kBsChunkShadow,   // leaf chunk trips of shadow (any-hit) walks
    kBsJumpDescendShadow,  // jump mid-plane steps of shadow walks
    kBsLdsLeaf,       // leaf visits staged through the wave's LDS buffer (RT_LDS_LEAF)
    kBlockStats
};

// Wave mapping of the scene kernel: spw = min(spp, 64) samples of a pixel on
// g = pow2ceil(spw) lanes, ppw = 64 / g pixels per wave as a tw x th tile.
inline void wave_tile_shape(uint32_t spp, uint32_t& spw, uint32_t& g, uint32_t& ppw,
                            uint32_t& tw, uint32_t& th) {
    spw = spp >= 64u ? 64u : (spp ? spp : 1u);
    g = 1;
    while (g < spw) g *= 2u;
    ppw = 64u / g;
    uint32_t lg = 0;
    while ((1u << lg) < ppw) ++lg;
    tw = 1u << ((lg + 1) / 2);
    th = 1u << (lg / 2);
}

// Superblocks (8x8 blocks of 8x8 wave tiles) of a scene frame's wave-tile
// grid, or of n_tiles packed tiles.
inline uint32_t scene_superblocks(uint32_t W, uint32_t H, uint32_t spp, uint32_t n_tiles,
                                  uint32_t tile_size) {
    uint32_t spw, g, ppw, tw, th;
    wave_tile_shape(spp, spw, g, ppw, tw, th);
    const uint32_t gw = n_tiles ? tile_size / tw : (W + tw - 1) / tw;
    const uint32_t gh = n_tiles ? tile_size / th : (H + th - 1) / th;
    const uint32_t nsx = ((gw + 7u) / 8u + 7u) / 8u, nsy = ((gh + 7u) / 8u + 7u) / 8u;
    return (n_tiles ? n_tiles : 1u) * nsx * nsy;
}

// 8x8-wave-tile blocks of the same grid(s) that hold at least one wave tile.
inline uint32_t scene_blocks(uint32_t W, uint32_t H, uint32_t spp, uint32_t n_tiles,
                             uint32_t tile_size) {
    uint32_t spw, g, ppw, tw, th;
    wave_tile_shape(spp, spw, g, ppw, tw, th);
    const uint32_t gw = n_tiles ? tile_size / tw : (W + tw - 1) / tw;
    const uint32_t gh = n_tiles ? tile_size / th : (H + th - 1) / th;
    return (n_tiles ? n_tiles : 1u) * ((gw + 7u) / 8u) * ((gh + 7u) / 8u);
}

// The wave queue's level-1 unit (scene_kernel): superblocks when there are
// enough of them that one superblock is a small part of an XCD's share
// (>= 192: C3 full frame (510), block slots cost it 0.6-3.4%; C4 8-way share
// (255), equal within noise) and they are mostly wave
// tiles (a packed 64x64 tile below 64 spp fills 1/4 of one or less), else
// 8x8 blocks (1/8 and 1/4 C3 tile shares, 64 and 128: -4% and -2%,
// profiles/r02/slot_size_ab.log).
#ifndef RT_SLOT_SB_MIN
#define RT_SLOT_SB_MIN 192u
#endif
inline uint32_t wave_queue_slot_shift(uint32_t superblocks, uint32_t blocks) {
    return superblocks >= RT_SLOT_SB_MIN && 4ull * blocks >= 3ull * 64u * superblocks ? 12u : 6u;
}

// Pinhole camera (include/camera.h:9-56): K and R column-major like glm.
struct CamArgs {
    float K[9];  // K[c*3+r]
    float R[9];  // rot = mat3(pose): R[c*3+r] = pose[c*4+r]
    float o[3];  // origin = pose[3].xyz
};

// Octree in HBM (DESIGN.md "Data layout"):
//   nodes[]   : uint2 records.  internal: {first child slot, valid | leaf<<8}
//                               leaf    : {first prim ref, prim count}
//               children of a node occupy consecutive slots, only the valid
//               ones, in real child order (bit0 x, bit1 y, bit2 z);
//               breadth-first, so the top levels are contiguous.
//   prim_sp[] : float4 (cx, cy, cz, r), one per leaf reference (leaf-contiguous)
//   prim_idx[]: sphere index of each reference (nearest-hit tie-break, shading)
struct SceneArgs {
    const uint2* nodes;
    const float4* prim_sp;
    const uint32_t* prim_idx;
    const float4* spheres;   // by sphere index (shading)
    const uint32_t* albedo;  // packed RGBA8 by sphere index
    uint2 root;              // nodes[0], also passed by value
    uint32_t root_is_leaf;
    uint32_t max_depth;      // D: grid is G = 2^D cells per axis
    float rmin[3];
    float scale[3];          // G / (rmax - rmin), f32
    float G;
    uint32_t opt;            // kOpt* toggles (A/B only; 0 = all optimisations on)
    const uint2* tab;        // depth-tab_k cell table, or null (cell_table.hip)
    uint32_t tab_k;          // 0: no table
    uint32_t stack_depth;    // deepest leaf (sizes the per-lane ancestor stack)
    // Camera-relative screen records (DESIGN.md 5.1 "Camera-relative screen"):
    // per leaf reference {o - c (f32, as isect computes it), C'} with
    // C' <= |o - c|^2 - r^2 - slack, for the camera origin o of the frame
    // (cam_screen_kernel, refreshed when the origin or the scene changes).
    // Primary rays screen a sphere by fma(b, b, -C') >= 0 with b = (o - c).d.
    const float4* prim_cam;
    // Light-plane screen records (DESIGN.md 5.1 "Light-plane screen"): per leaf
    // reference {u, v} = the centre's coordinates in the plane perpendicular
    // to the light direction L (basis FrameArgs::shd_e) and rr' >= (r + slack)^2,
    // made once per scene and light (shd_screen_kernel).  Shadow rays (any-hit,
    // direction L) screen a sphere by (u_p - u)^2 + (v_p - v)^2 <= rr'.
    const float4* prim_shd;
    // The same records in 8 bytes, {u, v} per reference (RT_SHD8): one
    // dwordx4 carries a chunk's two; the radius term is the scene's largest
    // rr' (FrameArgs::shd_rr), so the screen passes a superset still
    const float2* prim_shd8;
    // Image-plane screen records of primary rays in 8 bytes (RT_CAM8): per
    // reference {qx, qy}, the sphere centre's gnomonic projection in the
    // basis FrameArgs::cam8_B, with a bf16 bound rho^2 on the image-plane
    // distance of every ray the exact test may accept folded into the low
    // bytes (cam8_screen_kernel); one dwordx4 a chunk
    const float2* prim_cam8;
    // Albedo by leaf reference (albedo[prim_idx[ref]], made once per scene,
    // albedo_refs_kernel): a nearest walk returns its hit's REFERENCE, and the
    // hit is shaded from prim_sp[ref] and prim_al[ref], lines the walk's own
    // exact test and its neighbours just read, instead of three dependent
    // loads of lines by sphere index (prim_idx, spheres, albedo) that miss the
    // L2 (RT_REF_SHADE)
    const uint32_t* prim_al;
    // LDS leaf staging: leaves of kLdsLeafMin .. lds_max - 1
    // spheres are staged; kLeafBuf, or 0 (off) under RT_LDS_STAGE=0 (A/B:
    // off at run time loses on every config, C5d included,
    // profiles/r05/stage_switch_ab.log)
    uint32_t lds_max;
};

// Spheres per wave in the LDS leaf buffer (a leaf of >= kLeafBuf uses global loads)
constexpr uint32_t kLeafBuf = 32;

// Slack of the camera-relative screen, in units of 2^-24: the
// screen may only pass MORE spheres than the exact test, so C' undercuts
// |o - c|^2 - r^2 by the bound on the two forms' rounding difference
// (13 u |o - c|^2 + 5 u r^2 derived there; 16 and 8 kept).
constexpr double kScreenSlackOc = 16.0;
constexpr double kScreenSlackR = 8.0;
// Slack of the light-plane screen: an accepted sphere's
// centre lies within r (1 + 3.5 u) + 7.8 u M of the shadow ray's origin in
// the light plane (M bounds |origin| and |centre|: the root box's farthest
// corner); the records use r (1 + 4 u) + 64 u M.
constexpr double kShadowSlackM = 64.0;

struct FrameArgs {
    CamArgs cam;
    SceneArgs sc;
    uint32_t W, H;
    uint32_t spp;
    uint32_t seedmix;   // mix32(seed ^ 0x9E3779B9)
    uint32_t jitter;
    uint32_t shadows;
    uint32_t contract;  // compat: 1 = getRay with nvcc-style FMA contraction (RT_FLAG_COMPAT_FMA)
    float L[3];         // unit vector toward the light
    float shd_e[6];     // light-plane basis {e1, e2} (orthonormal, perpendicular to L; f32)
    float shd_rr;       // the largest light-plane rr' of the scene (SceneArgs::prim_shd8)
    float cam8_B[9];    // orthonormal basis of the image-plane screen, rows x, y, z (f32)
    float ambient;
    float inv_spp;      // 1 / samples in the image (all accumulated frames)
    // progressive accumulation (RT_FLAG_PROGRESSIVE)
    float4* accum;      // per-pixel running radiance sums (frame layout), or null
    uint32_t s_base;    // first sample index of this frame (frame index * spp)
    uint32_t accum_in;  // 1: add this frame's rounds onto the stored sums
    // output
    uint32_t* out8;     // RGBA8 (R in the low byte), frame- or tile-packed
    float4* out32;      // optional mean radiance (frame layout only), may be null
    // tile mode (out8 packed per tile)
    const uint32_t* tiles;
    uint32_t n_tiles;
    uint32_t tile_size;
    uint32_t tiles_x;   // ceil(W / tile_size)
    unsigned long long* counters;  // this frame's set: stat lines, queue heads, slot table
    // the other set, which this frame's kernel zeroes (ctr_next_words words)
    // for the next frame: frames need no memset launch between them
    unsigned long long* ctr_next;
    uint32_t ctr_next_words;
    uint32_t variant;   // scene kernel variant (kVariant*)
    // wave mapping (set by launch_scene): a wave = ppw pixels (tw x th) x spw samples
    uint32_t spw, g, ppw, tw, th, rounds;  // g = pow2ceil(spw) lanes per pixel
    uint32_t count_work;  // 1: also count node visits / sphere tests (stats frames)
    uint32_t bts;         // block-tile side in pixels (set by the launcher)
    uint32_t wq_chunk;    // wave-queue scheduling: wave tiles per dequeue ticket (launch_scene)
    uint32_t* wq_slots;        // two-level wave queue: per XCD, the superblock of each slot + 1
    uint32_t wq_slot_stride;   //   (0 = not claimed yet, kSlotNone = none left); zeroed per frame
    uint32_t wq_slot_shift;    //   slot = 2^shift wave tiles: 12 a superblock, 6 one 8x8 block
    const uint32_t* sb_order;  // frame superblock slots: claim index -> superblock (a
                               //   Hilbert order over the superblock grid), or null: row-major
    uint32_t wq_claim_delay;   // test only (RT_TEST_CLAIM_DELAY): XCD 0's ticket-0 wave sleeps
                               //   this many s_sleep 127 before claiming slot 0; 0 in product
    // Wave-queue failure report: a wave whose slot was never published (the
    // bounded wait below gave up) stores frame_id into this word of pinned,
    // host-coherent memory (rt_renderer::qerr_host), which the host reads
    // without a copy or a sync: the next rt_render reports it (the Displayer
    // never reads back, src/window/displayer.cpp:51-53), as do rt_synchronize,
    // rt_readback and stats frames.
    uint32_t* qerr;
    uint32_t frame_id;         // nonzero, per renderer
    uint32_t test_fault_queue; // test only (RT_TEST_FAULT=queue:k): the frame reports itself failed
#ifdef RT_TIMELINE
    unsigned long long* timeline;  // diagnostic build: 4 words per wave
#endif
#ifdef RT_BLOCK_STATS
    unsigned long long* bstats;    // diagnostic build: kBlockStats wave-execution counters
#endif
};

}  // namespace rtamd
