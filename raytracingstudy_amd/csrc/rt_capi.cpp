// rt_capi.cpp — the C-ABI (include/rt.h) over the HIP kernels.
//
// Host runtime that replaces KernelRenderer (include/renderer.cuh:25-50,
// src/renderer.cu:111-198): camera/octree state lives on the host and goes to
// the kernels by value; device buffers are owned here (the reference leaks
// its device-heap Camera/Octree, src/renderer.cu:189-198); every call returns
// a status (the reference's render path checks nothing, :145-151).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>  // types only: the functions are resolved at run time (rccl_api)
#include <stdio.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/rt.h"
#include "octree_gpu.h"
#include "rt_params.h"
#include "scene_build.h"

namespace rtamd {
hipError_t launch_compat(const FrameArgs& a, hipStream_t st);
hipError_t launch_scene(const FrameArgs& a, hipStream_t st);
bool variant_available(uint32_t v);
hipError_t launch_unpack(const uint32_t* packed, const uint32_t* tiles, uint32_t n_tiles,
                         uint32_t ts, uint32_t tiles_x, uint32_t W, uint32_t H, uint32_t* img,
                         hipStream_t st);
hipError_t launch_cam_screen(const float4* prim_sp, uint32_t n, const float o[3], float4* out,
                             hipStream_t st);
hipError_t launch_shd_screen(const float4* prim_sp, uint32_t n, const float e[6], double delta,
                             float4* out, float2* out8, uint32_t* rr_max, hipStream_t st);
hipError_t launch_albedo_refs(const uint32_t* prim_idx, const uint32_t* albedo, uint32_t n,
                              uint32_t n_spheres, uint32_t* out, hipStream_t st);
hipError_t launch_cam8_screen(const float4* prim_sp, uint32_t n, const float o[3], const float B[9],
                              uint32_t ok, float2* out, hipStream_t st);
}  // namespace rtamd

using namespace rtamd;

// rt_create_multi: the frame's tiles over several
// devices of this process; `r` (the handle) is devices[0]'s renderer
struct MultiState {
    static constexpr int F = 2;            // frames in flight
    static constexpr uint32_t kTs = 64;    // tile side
    std::vector<int> devs;                 // devs[0] = the handle's device
    std::vector<rt_renderer*> peers;       // peers[k] renders device k's tiles (peers[0] = the handle)
    uint32_t transport = 0;                // RT_TRANSPORT_RCCL / RT_TRANSPORT_PEER
    std::vector<ncclComm_t> comms;         // one per device (ncclCommInitAll)
    std::vector<hipStream_t> cs;           // per-device comm stream
    // devices[0]'s output stream: what a NULL stream argument means for the
    // handle (rt_stream).  Not devices[0]'s render stream, so that the wait
    // for frame j's unpack does not hold frame j+1's tiles on device 0.
    hipStream_t out = nullptr;
    // per frame slot f: each device's packed slab, devices[0]'s receive buffer
    // of n slabs end to end, and the events that order their reuse (all
    // timing-disabled: they are waited on every frame)
    std::vector<void*> slab[F];
    void* recv[F] = {nullptr, nullptr};
    std::vector<hipEvent_t> rendered[F], sent[F];
    hipEvent_t recvd[F] = {nullptr, nullptr}, unpacked[F] = {nullptr, nullptr}, out_ready = nullptr;
    bool used[F] = {false, false};
    // rt_get_multi_timing: timing events, recorded only once the caller has
    // asked for timing: device k's render start / end, devices[0]'s
    // unpack end; timed[f] = slot f's frame recorded them
    bool timing = false;
    bool timed[F] = {false, false};
    std::vector<hipEvent_t> t_start[F], t_end[F];
    hipEvent_t t_unpacked[F] = {nullptr, nullptr};
    uint64_t frame = 0;
    // a resize that failed part-way leaves the devices at different sizes:
    // rt_render refuses the handle until a resize succeeds
    bool broken = false;
    // test-only fault injection (RT_TEST_FAULT with RT_FLAG_TEST_HOOKS, read
    // once by rt_create_multi): "create:k" peer k's rt_create fails, "comm"
    // ncclCommInitAll fails, "slab:k" the slab allocation on peer k fails,
    // "queue:k" peer k's plain frames report themselves incomplete (as a
    // slot that was never published: rt_renderer::test_fault_queue)
    enum Fault { kNone = 0, kCreate, kComm, kSlab, kQueue };
    int fault = kNone;
    uint32_t fault_k = 0;
    // tile plan for the current size
    uint32_t W = 0, H = 0, S = 0;          // S = slab tiles
    size_t slab_bytes = 0;
    std::vector<std::vector<uint32_t>> ids;
    std::vector<uint32_t> all_ids;         // n * S, padding slots RT_TILE_SKIP
    uint32_t* d_all_ids = nullptr;         // on devices[0]
};

namespace {
thread_local std::string g_last_error;

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;  // elements
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};
}  // namespace

struct rt_renderer {
    rt_config cfg;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // completion of the renderer's last queued work (render, tiles, unpack) on
    // whichever stream it ran: a launch on another stream is ordered after it
    // (the counters, queue heads and buffers are shared), and
    // rt_synchronize / rt_readback wait for it
    hipEvent_t done = nullptr;
    hipStream_t last_stream = nullptr;
    bool pending = false;
    // wave-queue failure report (FrameArgs::qerr): a pinned host-coherent word
    // the kernel stores a failed frame's id into; the host reports each new
    // value once (queue_report), from rt_render without any copy or sync
    uint32_t* qerr_host = nullptr;
    uint32_t* qerr_dev = nullptr;
    uint32_t frame_seq = 0;   // last frame id handed out (never 0)
    uint32_t qerr_seen = 0;   // last reported value of *qerr_host
    // test only (RT_TEST_FAULT=queue:k, RT_FLAG_TEST_HOOKS): plain frames
    // report themselves failed
    bool test_fault_queue = false;
    float pose[16];
    float K[9];
    uint32_t W = 0, H = 0;
    DevBuf<uint32_t> fb;
    DevBuf<float4> rad;
    DevBuf<float4> accum;            // RT_FLAG_PROGRESSIVE running sums
    uint32_t frames_accum = 0;       // frames in `accum` (0: next frame starts over)
    uint64_t accum_sig = 0;          // which pixels the sums belong to (frame / tile list)
    DevBuf<unsigned long long> counters;
    // the counters, queue heads and slot table in two sets of ctr_stride
    // words: a scene frame uses set ctr_set and its kernel zeroes the other
    // one for the next frame (FrameArgs::ctr_next), so no memset launch sits
    // between frames; ctr_zero[s] = leading words of set s known to be zero
    size_t ctr_stride = 0;
    uint32_t ctr_set = 0;
    size_t ctr_zero[2] = {0, 0};
    // superblock claim order of full frames (FrameArgs::sb_order) and the
    // superblock grid it was made for
    DevBuf<uint32_t> sb_order;
    uint32_t sb_nx = 0, sb_ny = 0;
    // device copies of recently used tile lists (rt_render_tiles: this rank's
    // list; rt_unpack_tiles on rank 0: one list per peer), least recently used
    // evicted; each host vector stays alive as the source of its async upload
    struct TileList {
        std::vector<uint32_t> host;
        DevBuf<uint32_t> dev;
        uint64_t used = 0;
    };
    std::vector<TileList> tile_lists;
    uint64_t tile_clock = 0;
    // display buffer mapped per frame: the Displayer's
    // registered GL PBO through the HIP graphics ops, or a caller's ops
    rt_display_ops disp{};
    void* disp_user = nullptr;
    bool gl_disp = false;  // disp are the built-in HIP graphics-interop ops
    // scene: the sphere list lives in d_spheres/d_albedo; `spheres` is a host
    // copy when the scene came from host memory (host builder input)
    uint32_t n_spheres = 0;
    std::vector<float> spheres;
    bool host_copy = false;
    // leaf-reference arrays' length (prim_sp / prim_idx / the screen records):
    // info.n_prim_refs, plus the gaps of the line-packed layout (pack_leaf_lines)
    uint32_t prim_slots = 0;
    bool leaf_packed = false;
    // test only: RT_TEST_CLAIM_DELAY at rt_create with RT_FLAG_TEST_HOOKS
    // (FrameArgs::wq_claim_delay)
    uint32_t test_claim_delay = 0;
    rt_octree_params oct;
    bool has_scene = false;
    GpuOctreeBuilder gpu_build;
    CellTable cell_table;
    DevBuf<uint2> d_nodes;
    DevBuf<float4> d_prim_sp;
    DevBuf<uint32_t> d_prim_idx;
    DevBuf<float4> d_spheres;
    DevBuf<uint32_t> d_albedo;
    SceneArgs sc{};
    // camera-relative screen records (SceneArgs::prim_cam) and what they were
    // made for: the scene build and the camera origin
    DevBuf<float4> d_prim_cam;
    uint64_t scene_gen = 0, cam_gen = ~0ull;
    // light-plane screen records (SceneArgs::prim_shd) and the basis and
    // scene they were made for
    DevBuf<float4> d_prim_shd;
    uint64_t shd_gen = ~0ull;
    float shd_e[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float cam_o[3] = {0.f, 0.f, 0.f};
    // the light-plane records in 8 bytes (SceneArgs::prim_shd8) and their
    // radius term (FrameArgs::shd_rr; rr_dev: the kernel's max, in bits)
    DevBuf<float2> d_prim_shd8;
    DevBuf<uint32_t> d_shd_rr;
    float shd_rr = 0.0f;
    // image-plane screen records (SceneArgs::prim_cam8) and what they were
    // made for: the scene, the camera origin and the basis (with its check)
    DevBuf<float2> d_prim_cam8;
    uint64_t cam8_gen = ~0ull;
    float cam8_key[13] = {};
    // albedo by leaf reference (SceneArgs::prim_al) and the scene it was made for
    DevBuf<uint32_t> d_prim_al;
    uint64_t al_gen = ~0ull;
    rt_scene_info info{};
    std::string err;
    // multi-device handle (rt_create_multi): this renderer is devices[0]'s
    // part; the state holds the other devices' renderers and the transport
    MultiState* multi = nullptr;
};

namespace {

// multi-device handle internals (defined with rt_create_multi below)
int multi_render(rt_renderer* r, uint32_t* out, hipStream_t hs, rt_stats* stats);
int multi_wait(rt_renderer* r);
int multi_synchronize(rt_renderer* r);
int multi_queue_report(rt_renderer* r);
void multi_destroy(rt_renderer* r);
int multi_set_scene_device(rt_renderer* r, uint32_t n, const rt_octree_params* oct);
// " (device <ordinal>, peer <k>)": names the device in a multi-device error
std::string peer_name(const MultiState& m, size_t k) {
    return " (device " + std::to_string(m.devs[k]) + ", peer " + std::to_string(k) + ")";
}
// apply `fn` to every other device's renderer of a multi-device handle
template <typename Fn>
int for_peers(rt_renderer* r, Fn fn) {
    if (!r || !r->multi) return RT_OK;
    for (size_t k = 1; k < r->multi->peers.size(); ++k) {
        const int st = fn(r->multi->peers[k]);
        if (st) {
            r->err = r->multi->peers[k]->err + peer_name(*r->multi, k);
            return st;
        }
    }
    return RT_OK;
}
// the stream a NULL stream argument means: the renderer's own, or a
// multi-device handle's output stream on devices[0]
hipStream_t own_stream(const rt_renderer* r) { return r->multi ? r->multi->out : r->stream; }

int fail(rt_renderer* r, int code, const std::string& msg) {
    g_last_error = msg;
    if (r) r->err = msg;
    return code;
}

int hip_fail(rt_renderer* r, hipError_t e, const char* what) {
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return fail(r, RT_E_HIP, m);
}

#define RT_HIP(r, call)                                   \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail((r), e_, #call); \
    } while (0)

template <typename T>
int ensure(rt_renderer* r, DevBuf<T>& b, size_t n) {
    if (b.n >= n && b.p) return RT_OK;
    b.release();
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&b.p), n * sizeof(T));
    if (e != hipSuccess) {
        b.p = nullptr;
        return hip_fail(r, e, "hipMalloc");
    }
    b.n = n;
    return RT_OK;
}

int render_tiles_one(rt_renderer* r, const uint32_t* tile_ids, uint32_t n_tiles, uint32_t ts,
                     void* dev_packed, void* stream, rt_stats* stats);
int unpack_tiles_one(rt_renderer* r, const void* dev_packed, const uint32_t* tile_ids,
                     uint32_t n_tiles, uint32_t ts, void* dev_rgba8, void* stream);

int set_device(rt_renderer* r) {
    RT_HIP(r, hipSetDevice(r->device));
    return RT_OK;
}

void fill_frame_args(rt_renderer* r, FrameArgs& a) {
    memset(&a, 0, sizeof(a));
    memcpy(a.cam.K, r->K, sizeof(r->K));
    for (int c = 0; c < 3; ++c)
        for (int row = 0; row < 3; ++row) a.cam.R[c * 3 + row] = r->pose[c * 4 + row];
    a.cam.o[0] = r->pose[12];
    a.cam.o[1] = r->pose[13];
    a.cam.o[2] = r->pose[14];
    a.sc = r->sc;
    a.W = r->W;
    a.H = r->H;
    a.spp = r->cfg.spp ? r->cfg.spp : 1;
    a.seedmix = mix32(r->cfg.seed ^ 0x9E3779B9u);
    bool jitter = a.spp > 1;
    if (r->cfg.flags & RT_FLAG_JITTER) jitter = true;
    if (r->cfg.flags & RT_FLAG_NO_JITTER) jitter = false;
    a.jitter = jitter ? 1u : 0u;
    a.shadows = (r->cfg.flags & RT_FLAG_NO_SHADOWS) ? 0u : 1u;
    a.contract = (r->cfg.flags & RT_FLAG_COMPAT_FMA) ? 1u : 0u;
    const float* ld = r->cfg.light_dir;
    const float ll = sqrtf(ld[0] * ld[0] + ld[1] * ld[1] + ld[2] * ld[2]);
    a.L[0] = -(ld[0] / ll);
    a.L[1] = -(ld[1] / ll);
    a.L[2] = -(ld[2] / ll);
    a.ambient = r->cfg.ambient;
    a.inv_spp = 1.0f / static_cast<float>(a.spp);
    if ((r->cfg.flags & RT_FLAG_PROGRESSIVE) && r->cfg.mode == RT_MODE_SCENE) {
        // frame k traces samples [k*spp, (k+1)*spp) and adds them onto the
        // stored sums: after K frames the image is the mean of K*spp samples
        // (identical to one K*spp frame when spp is a multiple of 64)
        if (uint64_t(r->frames_accum + 1) * a.spp >= (1ull << 31)) r->frames_accum = 0;
        a.accum = r->accum.p;
        a.s_base = r->frames_accum * a.spp;
        a.accum_in = r->frames_accum ? 1u : 0u;
        a.inv_spp = 1.0f / static_cast<float>((r->frames_accum + 1) * a.spp);
    }
    a.counters = r->counters.p;
    a.sc.opt = (r->cfg.flags >> RT_FLAG_OPT_SHIFT) & 0xFFu;
    a.wq_claim_delay = r->test_claim_delay;
    a.qerr = r->qerr_dev;
    if (++r->frame_seq == 0) r->frame_seq = 1;
    a.frame_id = r->frame_seq;
    const uint32_t v = (r->cfg.flags >> RT_FLAG_VARIANT_SHIFT) & 0xFu;
    // default: multi-sample frames are scheduled per wave over per-XCD queues
    // (variant 13: C5 -15%, equal on C3, better on multi-GPU shares); 1-spp
    // frames (8x8-pixel wave tiles) keep the block-tile queue (tools/variants.py A/B,
    // profiles/r01/wave_queue_ab.log)
    // spp < 8: the block-tile queue with counters only in stats frames (C2
    // 0.185 -> 0.168 ms against the always-counting build 7,
    // profiles/r02/c2_variant_ab.log)
    // round 4: spp < 8 frames take the per-wave queue too (variant 4, no
    // workgroup barrier per block tile: C2 0.155 -> 0.107 ms,
    // profiles/r04/c2_waveq_ab.log)
    a.variant = v ? v : (a.spp >= 8u ? kVariantWaveQ : kVariantWaveQLow);
}

// An A/B switch read from the environment ("0" off, anything else on), or dflt.
bool env_flag(const char* name, bool dflt) {
    const char* v = getenv(name);
    return v && *v ? atoi(v) != 0 : dflt;
}
#ifndef RT_LEAF_PACK_DEFAULT
#define RT_LEAF_PACK_DEFAULT 0
#endif

// A test hook's environment variable (RT_TEST_*): its value when the config
// carries RT_FLAG_TEST_HOOKS, else NULL.  Either way a set variable is named
// on stderr once per process, so a stray one is visible.
const char* test_env(uint32_t flags, const char* name) {
    const char* v = getenv(name);
    if (!v || !*v) return nullptr;
    const bool on = (flags & RT_FLAG_TEST_HOOKS) != 0;
    static std::mutex mu;
    static std::vector<std::string> said;
    {
        std::lock_guard<std::mutex> g(mu);
        const std::string key = std::string(name) + (on ? "+" : "-");
        if (std::find(said.begin(), said.end(), key) == said.end()) {
            said.push_back(key);
            fprintf(stderr, on ? "librt_amd: test hook %s=%s active (RT_FLAG_TEST_HOOKS)\n"
                               : "librt_amd: %s=%s ignored (test hooks need RT_FLAG_TEST_HOOKS)\n",
                    name, v);
        }
    }
    return on ? v : nullptr;
}

// Superblock claim order (FrameArgs::sb_order, RT_SB_ORDER): the cells of a
// Hilbert curve over the next power-of-two square, those inside the nx x ny
// superblock grid in curve order, as row-major indices.  The level-1 counter
// hands claims to the XCDs in turn, so an XCD's successive superblocks lie a
// few steps apart along the curve, near each other in the image, instead of
// eight columns apart in row-major order.
std::vector<uint32_t> hilbert_order(uint32_t nx, uint32_t ny) {
    uint32_t n = 1;
    while (n < nx || n < ny) n *= 2u;
    std::vector<uint32_t> out;
    out.reserve(size_t(nx) * ny);
    for (uint64_t d = 0; d < uint64_t(n) * n; ++d) {
        uint32_t x = 0, y = 0;
        uint64_t t = d;
        for (uint32_t s = 1; s < n; s *= 2u) {
            const uint32_t rx = 1u & static_cast<uint32_t>(t / 2), ry = 1u & static_cast<uint32_t>(t ^ rx);
            if (ry == 0) {
                if (rx == 1) {
                    x = s - 1u - x;
                    y = s - 1u - y;
                }
                std::swap(x, y);
            }
            x += s * rx;
            y += s * ry;
            t /= 4;
        }
        if (x < nx && y < ny) out.push_back(y * nx + x);
    }
    return out;
}
#ifndef RT_SB_ORDER_DEFAULT
#define RT_SB_ORDER_DEFAULT 0
#endif

// Leaf records of a breadth-first tree: a record's kind is in
// its parent's leaf mask, and children come after their parent, so one
// forward pass over the records finds them all.  Returned in record order.
std::vector<uint32_t> leaf_records(const std::vector<uint2>& nodes) {
    std::vector<uint8_t> internal(nodes.size(), 0);
    std::vector<uint32_t> leaves;
    if (!nodes.empty()) internal[0] = 1;  // (callers skip a root leaf)
    for (size_t i = 0; i < nodes.size(); ++i) {
        if (!internal[i]) continue;
        const uint32_t valid = nodes[i].y & 0xFFu, leafm = (nodes[i].y >> 8) & 0xFFu;
        uint32_t k = nodes[i].x;
        for (uint32_t c = 0; c < 8; ++c) {
            if (!((valid >> c) & 1u)) continue;
            if ((leafm >> c) & 1u) leaves.push_back(k);
            else internal[k] = 1;
            ++k;
        }
    }
    std::sort(leaves.begin(), leaves.end(), [&](uint32_t a, uint32_t b) { return nodes[a].x < nodes[b].x; });
    return leaves;
}

// Line-packed leaf lists: the builders store the leaf
// lists back to back, so a leaf of n spheres (16 B each) straddles a 128-byte
// cache line whenever it does not fit in the rest of one: 1.44-1.57 lines per
// leaf on C3 / C5 / C5d against 1.05-1.12 when no leaf that fits a line
// crosses one.  This relays the lists out so that it never does: a leaf whose
// footprint (n, plus the slot past its end that a two-sphere chunk reads when
// n is odd) fits in 8 slots starts in the current line if it fits there, else
// at the next line; a longer leaf starts at a line.  The gaps hold what the
// kPrimPad tail holds (zero spheres, or the test-only pad-fill spheres);
// leaf records point at the new offsets; images and counters are unchanged
// (the layout is not part of the spec).  The arrays grow by ~1.28x.
int pack_leaf_lines(rt_renderer* r, SceneArgs& sc, rt_scene_info& in, const float4& pad) {
    const size_t nn = in.n_nodes, np = in.n_prim_refs;
    std::vector<uint2> nodes(nn);
    RT_HIP(r, hipMemcpy(nodes.data(), sc.nodes, nn * sizeof(uint2), hipMemcpyDeviceToHost));
    const std::vector<uint32_t> leaves = leaf_records(nodes);
    std::vector<uint32_t> nf(leaves.size());
    uint64_t off = 0;
    for (size_t i = 0; i < leaves.size(); ++i) {
        const uint32_t n = nodes[leaves[i]].y, f = n + (n & 1u), w = static_cast<uint32_t>(off & 7u);
        if (w && (f > 8u || w + f > 8u)) off += 8u - w;
        nf[i] = static_cast<uint32_t>(off);
        off += n;
    }
    if (off + kPrimPad >= (uint64_t(1) << 32)) return RT_OK;  // (keep the compact layout)
    const uint32_t slots = static_cast<uint32_t>(off);
    std::vector<float4> sp(np), spn(slots, pad);
    std::vector<uint32_t> ix(np), ixn(slots, 0u);
    if (np) {
        RT_HIP(r, hipMemcpy(sp.data(), sc.prim_sp, np * sizeof(float4), hipMemcpyDeviceToHost));
        RT_HIP(r, hipMemcpy(ix.data(), sc.prim_idx, np * sizeof(uint32_t), hipMemcpyDeviceToHost));
    }
    for (size_t i = 0; i < leaves.size(); ++i) {
        uint2& rec = nodes[leaves[i]];
        std::copy(sp.begin() + rec.x, sp.begin() + rec.x + rec.y, spn.begin() + nf[i]);
        std::copy(ix.begin() + rec.x, ix.begin() + rec.x + rec.y, ixn.begin() + nf[i]);
        rec.x = nf[i];
    }
    int st;
    if ((st = ensure(r, r->d_prim_sp, (size_t)slots + kPrimPad))) return st;
    if ((st = ensure(r, r->d_prim_idx, slots))) return st;
    if (slots) {
        RT_HIP(r, hipMemcpy(r->d_prim_sp.p, spn.data(), slots * sizeof(float4), hipMemcpyHostToDevice));
        RT_HIP(r, hipMemcpy(r->d_prim_idx.p, ixn.data(), slots * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    RT_HIP(r, hipMemcpy(const_cast<uint2*>(sc.nodes), nodes.data(), nn * sizeof(uint2),
                        hipMemcpyHostToDevice));
    sc.prim_sp = r->d_prim_sp.p;
    sc.prim_idx = r->d_prim_idx.p;
    r->prim_slots = slots;
    r->leaf_packed = true;
    return RT_OK;
}

// Build the octree of the device sphere list (d_spheres) and point the
// kernel's scene arguments at it.  The device builder is the default; the
// host builder (RT_FLAG_HOST_BUILD) yields the identical tree.
int build_scene(rt_renderer* r) {
    const uint32_t n = r->n_spheres;
    rt_octree_params& p = r->oct;
    uint32_t depth = p.max_depth ? p.max_depth : depth_for_resolution(p.min, p.max, p.resolution);
    if (depth > kMaxDepth) depth = kMaxDepth;
    const uint32_t cap = p.leaf_capacity ? p.leaf_capacity : 8;
    int st;
    if ((st = set_device(r))) return st;
    // buffers of the previous tree may still be read by frames in flight on
    // any stream: the rebuild waits for the device
    RT_HIP(r, hipDeviceSynchronize());
    r->has_scene = false;
    r->frames_accum = 0;
    rt_scene_info& in = r->info;
    const double upload_ms = in.upload_ms;
    in = rt_scene_info();
    in.upload_ms = upload_ms;
    SceneArgs& sc = r->sc;
    float rmin[3], rmax[3];
    auto t0 = std::chrono::steady_clock::now();
    bool host = (r->cfg.flags & RT_FLAG_HOST_BUILD) != 0;
    if (!host) {
        GpuBuildResult res;
        hipError_t e = r->gpu_build.build(r->d_spheres.p, n, p.min, p.max, depth, cap, r->stream, &res);
        if (res.n_invalid)
            return fail(r, RT_E_INVALID, "scene has spheres with radius <= 0 or non-finite values");
        // (test only: kOptDeviceBuildRefuse makes the device build report
        // running out of HBM, the one case that falls back to the host)
        if ((r->cfg.flags >> RT_FLAG_OPT_SHIFT) & kOptDeviceBuildRefuse) e = hipErrorOutOfMemory;
        if (res.ref_overflow) {
            // The device builder's 32-bit per-level slots overflowed: that
            // level holds >= 2^29 references (octree_build.hip), which the
            // host builder would need >= 2^29 x ~64 B = 32 GiB for (index,
            // sphere record, per-level lists) and would grind through for
            // minutes.  Always refused, at once; the
            // host fallback covers only the device build running out of HBM.
            (void)hipGetLastError();
            return fail(r, RT_E_NOMEM,
                        "scene too large for the octree: the device builder overflowed at " +
                            std::to_string(res.ref_overflow) +
                            " references (a host build would need about " +
                            std::to_string((res.ref_overflow * 64ull) >> 30) +
                            " GiB); lower max_depth or raise leaf_capacity");
        }
        if (e == hipErrorOutOfMemory) {
            // HBM cannot hold the device build's working set: build the
            // identical tree on the host instead (rt_scene_info.builder then
            // reports RT_BUILDER_HOST); build_octree refuses past 2^31
            // references and reports host allocation failure as RT_E_NOMEM
            (void)hipGetLastError();
            host = true;
        } else if (e != hipSuccess) {
            return hip_fail(r, e, "device octree build");
        } else {
            sc.nodes = r->gpu_build.nodes();
            sc.prim_sp = r->gpu_build.prim_sp();
            sc.prim_idx = r->gpu_build.prim_idx();
            sc.root = res.root;
            sc.root_is_leaf = res.root_is_leaf ? 1u : 0u;
            in.n_nodes = res.n_nodes;
            in.n_leaves = res.n_leaves;
            in.n_prim_refs = res.n_prims;
            in.depth_reached = res.depth_reached;
            in.builder = RT_BUILDER_DEVICE;
            memcpy(rmin, res.rmin, sizeof(rmin));
            memcpy(rmax, res.rmax, sizeof(rmax));
        }
    }
    if (host) {
        if (!r->host_copy) {
            r->spheres.resize(4u * n);
            if (n)
                RT_HIP(r, hipMemcpy(r->spheres.data(), r->d_spheres.p, n * sizeof(float4),
                                    hipMemcpyDeviceToHost));
            r->host_copy = true;
        }
        BuiltOctree tree;
        try {
            build_octree(r->spheres.data(), n, p.min, p.max, depth, cap, tree);
        } catch (const std::length_error& ex) {  // past the 32-bit record fields
            return fail(r, RT_E_INVALID, std::string("scene too large for the octree: ") + ex.what() +
                                             "; lower max_depth or raise leaf_capacity");
        } catch (const std::exception& ex) {  // bad_alloc: never through the C-ABI
            return fail(r, RT_E_NOMEM, std::string("host octree build: ") + ex.what());
        }
        const size_t nn = tree.nodes.size(), np = tree.prim_idx.size();
        if ((st = ensure(r, r->d_nodes, nn))) return st;
        if ((st = ensure(r, r->d_prim_sp, np + kPrimPad))) return st;  // scalar-read padding
        if ((st = ensure(r, r->d_prim_idx, np))) return st;
        RT_HIP(r, hipMemcpy(r->d_nodes.p, tree.nodes.data(), nn * sizeof(uint2),
                            hipMemcpyHostToDevice));
        if (np) {
            RT_HIP(r, hipMemcpy(r->d_prim_sp.p, tree.prim_sp.data(), np * sizeof(float4),
                                hipMemcpyHostToDevice));
            RT_HIP(r, hipMemcpy(r->d_prim_idx.p, tree.prim_idx.data(), np * sizeof(uint32_t),
                                hipMemcpyHostToDevice));
        }
        sc.nodes = r->d_nodes.p;
        sc.prim_sp = r->d_prim_sp.p;
        sc.prim_idx = r->d_prim_idx.p;
        sc.root = make_uint2(tree.nodes[0].x, tree.nodes[0].y);
        sc.root_is_leaf = tree.root_is_leaf ? 1u : 0u;
        in.n_nodes = static_cast<uint32_t>(nn);
        in.n_leaves = tree.n_leaves;
        in.n_prim_refs = static_cast<uint32_t>(np);
        in.depth_reached = tree.depth_reached;
        in.builder = RT_BUILDER_HOST;
        memcpy(rmin, tree.rmin, sizeof(rmin));
        memcpy(rmax, tree.rmax, sizeof(rmax));
    }
    {
        // The kPrimPad tail after the last leaf list is read by the leaf loads
        // (a chunk's slot past the end of the LAST leaf) and joins the leaf
        // screen unmasked; its tests are skipped, so only time could depend on
        // it.  Neither builder writes it: fill it here so that nothing a frame
        // does depends on what the allocation held before.  Zero spheres
        // (r = 0) by default; the test-only fill modes put spheres there that
        // pass the screen (NaN, or one covering the root box) to prove the
        // images and counters do not depend on the tail.
        const uint32_t mode = (r->cfg.flags >> RT_FLAG_PAD_FILL_SHIFT) & 3u;
        float4 p1 = make_float4(0.f, 0.f, 0.f, 0.f);
        if (mode == 1) {
            p1 = make_float4(NAN, NAN, NAN, NAN);
        } else if (mode == 2) {
            const float c = 0.5f * (rmin[0] + rmax[0]);
            p1 = make_float4(c, 0.5f * (rmin[1] + rmax[1]), 0.5f * (rmin[2] + rmax[2]),
                             4.0f * (rmax[0] - rmin[0] + rmax[1] - rmin[1] + rmax[2] - rmin[2]));
        }
        float4 pad[kPrimPad];
        for (uint32_t i = 0; i < kPrimPad; ++i) pad[i] = p1;
        // the line-packed layout's gaps hold the same (RT_LEAF_PACK=1, an A/B
        // switch read here; off by default: measured no faster)
        r->prim_slots = in.n_prim_refs;
        r->leaf_packed = false;
        if (!sc.root_is_leaf && env_flag("RT_LEAF_PACK", RT_LEAF_PACK_DEFAULT) &&
            (st = pack_leaf_lines(r, sc, in, p1)))
            return st;
        float4* tail = const_cast<float4*>(sc.prim_sp) + r->prim_slots;
        RT_HIP(r, hipMemcpyAsync(tail, pad, sizeof(pad), hipMemcpyHostToDevice, r->stream));
        RT_HIP(r, hipStreamSynchronize(r->stream));
    }
    {
        // depth-K cell table over the tree (flags bits 28..31: 0 auto, 15 off, else K)
        const uint32_t f = (r->cfg.flags >> RT_FLAG_CELL_TABLE_SHIFT) & 0xFu;
        const uint32_t k_req = f == 0 ? kCellTableAuto : f == 15 ? kCellTableOff : f;
        hipError_t e = r->cell_table.build(sc.nodes, sc.root, sc.root_is_leaf != 0, depth,
                                           in.depth_reached, k_req, r->stream);
        if (e != hipSuccess) return hip_fail(r, e, "cell table build");
        sc.tab = r->cell_table.table();
        sc.tab_k = r->cell_table.k();
        in.cell_table_depth = sc.tab_k;
    }
    auto t1 = std::chrono::steady_clock::now();
    sc.spheres = r->d_spheres.p;
    sc.albedo = r->d_albedo.p;
    sc.max_depth = depth;
    sc.stack_depth = std::max(1u, std::min(depth, in.depth_reached));
    {
        // LDS leaf staging on every scene; RT_LDS_STAGE=0
        // turns it off (A/B and the on/off parity test)
        const char* ls = getenv("RT_LDS_STAGE");
        sc.lds_max = ls && *ls && atoi(ls) == 0 ? 0u : kLeafBuf;
    }
    sc.G = static_cast<float>(1u << depth);
    for (int i = 0; i < 3; ++i) {
        sc.rmin[i] = rmin[i];
        sc.scale[i] = sc.G / (rmax[i] - rmin[i]);
        in.root_min[i] = rmin[i];
        in.root_max[i] = rmax[i];
    }
    in.n_spheres = n;
    in.max_depth = depth;
    in.node_bytes = sizeof(uint2);
    in.prim_bytes = sizeof(float4) + sizeof(uint32_t);
    in.build_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    ++r->scene_gen;  // the camera-relative screen records are remade at the next frame
    r->has_scene = true;
    return RT_OK;
}

int check_octree_params(rt_renderer* r, const rt_octree_params* oct, const char* who) {
    if (!oct) return RT_OK;
    for (int i = 0; i < 3; ++i)
        if (!(oct->max[i] > oct->min[i]))
            return fail(r, RT_E_INVALID, std::string(who) + ": empty octree root box");
    if (oct->max_depth > kMaxDepth) return fail(r, RT_E_INVALID, std::string(who) + ": max_depth > 16");
    if (oct->max_depth == 0 && !(oct->resolution > 0.0f))
        return fail(r, RT_E_INVALID, std::string(who) + ": need max_depth or resolution > 0");
    return RT_OK;
}

int check_tiles(rt_renderer* r, const uint32_t* ids, uint32_t n_tiles, uint32_t ts,
                bool allow_skip = false) {
    if (ts == 0 || ts % 64 != 0 || ts > 4096)
        return fail(r, RT_E_INVALID, "tile_size must be a multiple of 64 in [64, 4096]");
    const uint32_t tx = (r->W + ts - 1) / ts, ty = (r->H + ts - 1) / ts;
    for (uint32_t i = 0; i < n_tiles; ++i)
        if (ids[i] >= tx * ty && !(allow_skip && ids[i] == RT_TILE_SKIP))
            return fail(r, RT_E_INVALID, "tile id out of range");
    return RT_OK;
}

// Device copy of a tile list: found in the cache when the same list was used
// recently (steady-state frames never copy or synchronise), else uploaded
// asynchronously into the least recently used slot.
constexpr size_t kTileListSlots = 16;

int tile_list(rt_renderer* r, const uint32_t* ids, uint32_t n, hipStream_t s, const uint32_t** out) {
    rt_renderer::TileList* hit = nullptr;
    for (auto& e : r->tile_lists)
        if (e.host.size() == n && e.dev.p && memcmp(e.host.data(), ids, n * sizeof(uint32_t)) == 0) {
            hit = &e;
            break;
        }
    if (!hit) {
        if (r->tile_lists.size() < kTileListSlots) {
            r->tile_lists.emplace_back();
            hit = &r->tile_lists.back();
        } else {
            hit = &r->tile_lists[0];
            for (auto& e : r->tile_lists)
                if (e.used < hit->used) hit = &e;
            // its previous upload may still be in flight on some stream
            RT_HIP(r, hipDeviceSynchronize());
        }
        int st;
        if ((st = ensure(r, hit->dev, n))) return st;
        hit->host.assign(ids, ids + n);
        RT_HIP(r, hipMemcpyAsync(hit->dev.p, hit->host.data(), n * sizeof(uint32_t),
                                 hipMemcpyHostToDevice, s));
    }
    hit->used = ++r->tile_clock;
    *out = hit->dev.p;
    return RT_OK;
}

// Progressive sums belong to one pixel set: the full frame (sig 1) or one
// tile list; rendering another set starts the accumulation over.
void accum_pixels(rt_renderer* r, const uint32_t* ids, uint32_t n, uint32_t ts) {
    uint64_t sig = 1;
    if (ids) {
        sig = 1469598103934665603ull ^ ts;
        for (uint32_t i = 0; i < n; ++i) sig = (sig ^ ids[i]) * 1099511628211ull;
        sig = (sig ^ n) * 1099511628211ull | 2u;
    }
    if (sig != r->accum_sig) r->frames_accum = 0;
    r->accum_sig = sig;
}

// Order work about to be queued on `st` after the renderer's last queued work
// when that ran on another stream (caller streams are typically non-blocking).
int order_after_last(rt_renderer* r, hipStream_t st) {
    if (r->pending && r->last_stream != st) RT_HIP(r, hipStreamWaitEvent(st, r->done, 0));
    return RT_OK;
}

int mark_queued(rt_renderer* r, hipStream_t st) {
    RT_HIP(r, hipEventRecord(r->done, st));
    r->last_stream = st;
    r->pending = true;
    return RT_OK;
}

// A frame the kernel found incomplete (its wave queue's bounded slot wait
// gave up, rt_kernels.hip) stored its id in the renderer's pinned word; each
// new value is reported once.  A plain host read: rt_render calls it before
// every frame with no sync, rt_synchronize / rt_readback / stats frames after
// theirs.
int queue_report(rt_renderer* r) {
    const uint32_t v = __atomic_load_n(r->qerr_host, __ATOMIC_ACQUIRE);
    if (v == r->qerr_seen) return RT_OK;
    r->qerr_seen = v;
    return fail(r, RT_E_HIP, "scene kernel: wave-queue slot never published: frame " +
                                 std::to_string(v) + " of this renderer is incomplete");
}

// RT_FLAG_TEST_POISON: the frame's outputs filled with a sentinel first
// (rt.h), so a pixel no kernel writes shows in the readback.
int poison_outputs(rt_renderer* r, const FrameArgs& a, hipStream_t st) {
    if (!(r->cfg.flags & RT_FLAG_TEST_POISON)) return RT_OK;
    const size_t px = a.tiles ? (size_t)a.n_tiles * a.tile_size * a.tile_size : (size_t)a.W * a.H;
    RT_HIP(r, hipMemsetAsync(a.out8, 0xAB, px * 4, st));
    // (the compat kernel writes RGBA8 only: no radiance to check there)
    if (a.out32 && r->cfg.mode == RT_MODE_SCENE)
        RT_HIP(r, hipMemsetAsync(a.out32, 0xFF, (size_t)a.W * a.H * 16, st));
    if (a.accum && !a.accum_in) RT_HIP(r, hipMemsetAsync(a.accum, 0xFF, (size_t)a.W * a.H * 16, st));
    return RT_OK;
}

// The image-plane screen's basis (SceneArgs::prim_cam8, DESIGN.md 5.1 round
// 6): rows x, y, z, orthonormal in f64 and rounded to f32, z along the ray
// through the image centre (getRay's K and R, include/camera.h:24-41).
// Returns 1 when every primary ray of the W x H frame keeps (B d).z >= 0.1
// |B d| (checked at the image corners: the rays' directions are the cone
// they span, and the ratio is kept under positive combinations), else 0:
// the records then pass every sphere.
uint32_t cam8_basis(const FrameArgs& a, float B[9]) {
    auto ray = [&](double u, double v, double w[3]) {
        const double dx = (u - a.cam.K[2]) / a.cam.K[0], dy = (v - a.cam.K[5]) / a.cam.K[4];
        for (int i = 0; i < 3; ++i) w[i] = a.cam.R[i] * dx + a.cam.R[3 + i] * dy + a.cam.R[6 + i];
    };
    double z[3], x[3] = {a.cam.R[0], a.cam.R[1], a.cam.R[2]}, y[3];
    ray(0.5 * a.W, 0.5 * a.H, z);
    const double zn = sqrt(z[0] * z[0] + z[1] * z[1] + z[2] * z[2]);
    if (!(zn > 0.0) || !std::isfinite(zn)) {
        for (int i = 0; i < 9; ++i) B[i] = i % 4 == 0 ? 1.0f : 0.0f;
        return 0u;
    }
    for (double& t : z) t /= zn;
    const double xz = x[0] * z[0] + x[1] * z[1] + x[2] * z[2];
    for (int i = 0; i < 3; ++i) x[i] -= xz * z[i];
    double xn = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    if (!(xn > 1e-3)) {  // R's first column along the view: any perpendicular
        x[0] = fabs(z[0]) < 0.9 ? 1.0 : 0.0;
        x[1] = fabs(z[0]) < 0.9 ? 0.0 : 1.0;
        x[2] = 0.0;
        const double t = x[0] * z[0] + x[1] * z[1];
        for (int i = 0; i < 3; ++i) x[i] -= t * z[i];
        xn = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    }
    for (double& t : x) t /= xn;
    y[0] = z[1] * x[2] - z[2] * x[1];
    y[1] = z[2] * x[0] - z[0] * x[2];
    y[2] = z[0] * x[1] - z[1] * x[0];
    for (int i = 0; i < 3; ++i) {
        B[i] = static_cast<float>(x[i]);
        B[3 + i] = static_cast<float>(y[i]);
        B[6 + i] = static_cast<float>(z[i]);
    }
    uint32_t ok = 1u;
    for (int k = 0; k < 4; ++k) {
        double w[3], p[3];
        ray((k & 1) ? a.W : 0.0, (k & 2) ? a.H : 0.0, w);
        for (int i = 0; i < 3; ++i)
            p[i] = (double)B[3 * i] * w[0] + (double)B[3 * i + 1] * w[1] + (double)B[3 * i + 2] * w[2];
        const double pn = sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
        if (!(p[2] >= 0.1 * pn) || !std::isfinite(pn)) ok = 0u;
    }
    return ok;
}

int do_render(rt_renderer* r, FrameArgs& a, void* stream, rt_stats* stats) {
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : r->stream;
    if (r->cfg.mode == RT_MODE_SCENE && !r->has_scene)
        return fail(r, RT_E_NOSCENE, "RT_MODE_SCENE render without rt_set_scene");
    int ost;
    if ((ost = order_after_last(r, st))) return ost;
    // the counters and, for the wave queue, its per-XCD slot table (8 x
    // (superblocks + 2) words after them): one set of `words`
    size_t words = kCounterWords;
    a.wq_slots = nullptr;
    a.wq_slot_stride = 0;
    if (r->cfg.mode == RT_MODE_SCENE) {
        const uint32_t nt = a.tiles ? a.n_tiles : 0u;
        const uint32_t nsb = scene_superblocks(a.W, a.H, a.spp, nt, a.tile_size);
        const uint32_t nbk = scene_blocks(a.W, a.H, a.spp, nt, a.tile_size);
        a.wq_slot_shift = wave_queue_slot_shift(nsb, nbk);
        a.wq_slot_stride = (a.wq_slot_shift == 12u ? nsb : nbk) + 2u;
        words += (8u * static_cast<size_t>(a.wq_slot_stride) + 1u) / 2u;
    }
    if (r->ctr_stride < words) {  // (re)allocate both sets and zero them
        if ((ost = ensure(r, r->counters, 2 * words))) return ost;
        r->ctr_stride = r->counters.n / 2;
        RT_HIP(r, hipMemsetAsync(r->counters.p, 0, r->counters.n * sizeof(unsigned long long), st));
        r->ctr_zero[0] = r->ctr_zero[1] = r->ctr_stride;
    }
    const uint32_t cs = r->ctr_set;
    unsigned long long* ctr = r->counters.p + cs * r->ctr_stride;
    if (r->ctr_zero[cs] < words)  // (after a failed launch, or a frame needing more words)
        RT_HIP(r, hipMemsetAsync(ctr, 0, words * sizeof(unsigned long long), st));
    if (a.wq_slot_stride) a.wq_slots = reinterpret_cast<uint32_t*>(ctr + kCounterWords);
    a.sb_order = nullptr;
    if (r->cfg.mode == RT_MODE_SCENE && !a.tiles && a.wq_slot_shift == 12u &&
        env_flag("RT_SB_ORDER", RT_SB_ORDER_DEFAULT)) {
        // the superblock grid of this frame (scene_body's nsx x nsy)
        uint32_t spw, g, ppw, tw, th;
        wave_tile_shape(a.spp, spw, g, ppw, tw, th);
        const uint32_t gw = (a.W + tw - 1u) / tw, gh = (a.H + th - 1u) / th;
        const uint32_t nx = ((gw + 7u) / 8u + 7u) / 8u, ny = ((gh + 7u) / 8u + 7u) / 8u;
        if (r->sb_nx != nx || r->sb_ny != ny || !r->sb_order.p) {
            const std::vector<uint32_t> ord = hilbert_order(nx, ny);
            if ((ost = ensure(r, r->sb_order, ord.size()))) return ost;
            RT_HIP(r, hipMemcpy(r->sb_order.p, ord.data(), ord.size() * sizeof(uint32_t),
                                hipMemcpyHostToDevice));
            r->sb_nx = nx;
            r->sb_ny = ny;
        }
        a.sb_order = r->sb_order.p;
    }
    if (r->cfg.mode == RT_MODE_SCENE) {
        // the camera-relative screen records of this frame's camera origin
        // (DESIGN.md 5.1): remade on this stream, after the renderer's earlier
        // frames (order_after_last), when the origin or the scene changed
        const uint32_t nr = r->prim_slots + kPrimPad;
        const float4* before = r->d_prim_cam.p;
        if ((ost = ensure(r, r->d_prim_cam, nr))) return ost;
        if (r->d_prim_cam.p != before || r->cam_gen != r->scene_gen ||
            memcmp(r->cam_o, a.cam.o, sizeof(r->cam_o)) != 0) {
            hipError_t e = launch_cam_screen(a.sc.prim_sp, nr, a.cam.o, r->d_prim_cam.p, st);
            if (e != hipSuccess) return hip_fail(r, e, "camera-relative screen records");
            memcpy(r->cam_o, a.cam.o, sizeof(r->cam_o));
            r->cam_gen = r->scene_gen;
        }
        a.sc.prim_cam = r->d_prim_cam.p;
        // the image-plane records of this frame's camera (origin, basis)
        {
            const uint32_t ok = cam8_basis(a, a.cam8_B);
            float key[13];
            memcpy(key, a.cam.o, sizeof(a.cam.o));
            memcpy(key + 3, a.cam8_B, sizeof(a.cam8_B));
            key[12] = ok ? 1.0f : 0.0f;
            const float2* before8 = r->d_prim_cam8.p;
            if ((ost = ensure(r, r->d_prim_cam8, nr))) return ost;
            if (r->d_prim_cam8.p != before8 || r->cam8_gen != r->scene_gen ||
                memcmp(r->cam8_key, key, sizeof(key)) != 0) {
                hipError_t e = launch_cam8_screen(a.sc.prim_sp, nr, a.cam.o, a.cam8_B, ok,
                                                  r->d_prim_cam8.p, st);
                if (e != hipSuccess) return hip_fail(r, e, "image-plane screen records");
                memcpy(r->cam8_key, key, sizeof(key));
                r->cam8_gen = r->scene_gen;
            }
            a.sc.prim_cam8 = r->d_prim_cam8.p;
        }
        // the light-plane screen: an orthonormal basis {e1, e2} of the plane
        // perpendicular to the shadow direction a.L (in f64 from the f32 L the
        // kernel uses, then rounded), and the records of its centres, remade
        // when the scene or the basis changes
        double l[3] = {a.L[0], a.L[1], a.L[2]};
        const double ln = sqrt(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]);
        for (double& x : l) x /= ln;
        int kmin = 0;
        for (int i = 1; i < 3; ++i)
            if (fabs(l[i]) < fabs(l[kmin])) kmin = i;
        double e1[3] = {0.0, 0.0, 0.0};
        e1[kmin] = 1.0;
        const double al = l[kmin];
        for (int i = 0; i < 3; ++i) e1[i] -= al * l[i];
        const double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
        for (double& x : e1) x /= n1;
        const double e2[3] = {l[1] * e1[2] - l[2] * e1[1], l[2] * e1[0] - l[0] * e1[2],
                              l[0] * e1[1] - l[1] * e1[0]};
        for (int i = 0; i < 3; ++i) {
            a.shd_e[i] = static_cast<float>(e1[i]);
            a.shd_e[3 + i] = static_cast<float>(e2[i]);
        }
        const float4* before_s = r->d_prim_shd.p;
        const float2* before_s8 = r->d_prim_shd8.p;
        if ((ost = ensure(r, r->d_prim_shd, nr))) return ost;
        if ((ost = ensure(r, r->d_prim_shd8, nr))) return ost;
        const uint32_t nbk = (nr + kBlockThreads - 1u) / kBlockThreads;  // shd_screen_kernel's blocks
        if ((ost = ensure(r, r->d_shd_rr, nbk + 1u))) return ost;
        if (r->d_prim_shd.p != before_s || r->d_prim_shd8.p != before_s8 || r->shd_gen != r->scene_gen ||
            memcmp(r->shd_e, a.shd_e, sizeof(r->shd_e)) != 0) {
            // M bounds |origin| and |centre| of every shadow test: the root
            // box holds every sphere, and a shadow origin is a hit point
            // moved 1e-5 off its sphere
            double m = 0.0;
            for (int c = 0; c < 8; ++c) {
                double q = 0.0;
                for (int i = 0; i < 3; ++i) {
                    const double v = (c >> i) & 1 ? r->info.root_max[i] : r->info.root_min[i];
                    q += v * v;
                }
                m = std::max(m, sqrt(q));
            }
            const double delta = kShadowSlackM / 16777216.0 * (m + 1e-4);
            RT_HIP(r, hipMemsetAsync(r->d_shd_rr.p, 0, (nbk + 1u) * sizeof(uint32_t), st));
            hipError_t e = launch_shd_screen(a.sc.prim_sp, nr, a.shd_e, delta, r->d_prim_shd.p,
                                             r->d_prim_shd8.p, r->d_shd_rr.p, st);
            if (e != hipSuccess) return hip_fail(r, e, "light-plane screen records");
            // the 8-byte records' radius term, once per scene and light (a sync)
            uint32_t bits = 0;
            RT_HIP(r, hipMemcpyAsync(&bits, r->d_shd_rr.p + nbk, sizeof(bits), hipMemcpyDeviceToHost, st));
            RT_HIP(r, hipStreamSynchronize(st));
            memcpy(&r->shd_rr, &bits, sizeof(bits));
            memcpy(r->shd_e, a.shd_e, sizeof(r->shd_e));
            r->shd_gen = r->scene_gen;
        }
        a.sc.prim_shd = r->d_prim_shd.p;
        a.sc.prim_shd8 = r->d_prim_shd8.p;
        a.shd_rr = r->shd_rr;
        // the albedo of every leaf reference, made once per scene
        const uint32_t* before_a = r->d_prim_al.p;
        if ((ost = ensure(r, r->d_prim_al, nr))) return ost;
        if (r->d_prim_al.p != before_a || r->al_gen != r->scene_gen) {
            hipError_t e = launch_albedo_refs(a.sc.prim_idx, a.sc.albedo, r->prim_slots, r->n_spheres,
                                              r->d_prim_al.p, st);
            if (e != hipSuccess) return hip_fail(r, e, "albedo by leaf reference");
            r->al_gen = r->scene_gen;
        }
        a.sc.prim_al = r->d_prim_al.p;
    }
    a.counters = ctr;
    const bool scene = r->cfg.mode == RT_MODE_SCENE;
    a.ctr_next = scene ? r->counters.p + (1u - cs) * r->ctr_stride : nullptr;
    a.ctr_next_words = scene ? static_cast<uint32_t>(words) : 0u;
    if ((ost = poison_outputs(r, a, st))) return ost;
    a.count_work = stats ? 1u : 0u;
    a.test_fault_queue = r->test_fault_queue && !stats ? 1u : 0u;
    if (stats) RT_HIP(r, hipEventRecord(r->ev0, st));
#ifdef RT_TIMELINE
    // diagnostic build (tools/timeline.sh): every stats frame appends its
    // per-wave timeline to $RT_TIMELINE_FILE
    static unsigned long long* tl = nullptr;
    const size_t tl_waves = 1u << 16;
    const size_t tl_words = tl_waves * 4 + (3u << 22) + tl_waves * 2;  // per wave, per unit, phases
    const char* tl_file = getenv("RT_TIMELINE_FILE");
    if (tl_file) {
        if (!tl) RT_HIP(r, hipMalloc(reinterpret_cast<void**>(&tl), tl_words * 8));
        RT_HIP(r, hipMemsetAsync(tl, 0, tl_words * 8, st));
        a.timeline = tl;
    }
#endif
#ifdef RT_BLOCK_STATS
    // diagnostic build (tools/block_stats.py): stats frames count the wave
    // executions of every walk block and append them to $RT_BLOCK_STATS_FILE
    static unsigned long long* bsd = nullptr;
    const char* bs_file = stats ? getenv("RT_BLOCK_STATS_FILE") : nullptr;
    a.bstats = nullptr;
    if (bs_file) {
        if (!bsd) RT_HIP(r, hipMalloc(reinterpret_cast<void**>(&bsd), 2 * kBlockStats * 8));
        RT_HIP(r, hipMemsetAsync(bsd, 0, 2 * kBlockStats * 8, st));
        a.bstats = bsd;
    }
#endif
    hipError_t e = r->cfg.mode == RT_MODE_SCENE ? launch_scene(a, st) : launch_compat(a, st);
    if (e != hipSuccess) {
        r->ctr_zero[0] = r->ctr_zero[1] = 0;  // neither set is known to be zero
        return hip_fail(r, e, "kernel launch");
    }
    if (scene) {  // this frame dirtied its set and zeroes the other one
        r->ctr_zero[cs] = 0;
        r->ctr_zero[1u - cs] = words;
        r->ctr_set = 1u - cs;
    }
#ifdef RT_BLOCK_STATS
    if (bs_file) {
        unsigned long long h[2 * kBlockStats];
        RT_HIP(r, hipStreamSynchronize(st));
        RT_HIP(r, hipMemcpy(h, bsd, sizeof(h), hipMemcpyDeviceToHost));
        if (FILE* f = fopen(bs_file, "a")) {
            fprintf(f, "{\"W\": %u, \"H\": %u, \"spp\": %u, \"counts\": [", a.W, a.H, a.spp);
            for (uint32_t i = 0; i < 2 * kBlockStats; ++i)
                fprintf(f, "%s%llu", i ? ", " : "", h[i]);
            fprintf(f, "]}\n");
            fclose(f);
        }
    }
#endif
    if ((ost = mark_queued(r, st))) return ost;
#ifdef RT_TIMELINE
    if (tl_file) {
        std::vector<unsigned long long> h(tl_words);
        RT_HIP(r, hipStreamSynchronize(st));
        RT_HIP(r, hipMemcpy(h.data(), tl, tl_words * 8, hipMemcpyDeviceToHost));
        if (FILE* f = fopen(tl_file, "ab")) {
            fwrite(h.data(), 8, h.size(), f);
            fclose(f);
        }
    }
#endif
    if (a.accum) ++r->frames_accum;
    if (stats) {
        RT_HIP(r, hipEventRecord(r->ev1, st));
        RT_HIP(r, hipEventSynchronize(r->ev1));
        unsigned long long lines[8 * kStatLineStride], c[4] = {0, 0, 0, 0};
        RT_HIP(r, hipMemcpy(lines, ctr + kStatLineBase, sizeof(lines), hipMemcpyDeviceToHost));
        for (uint32_t q = 0; q < 8; ++q)
            for (uint32_t i = 0; i < 4; ++i) c[i] += lines[q * kStatLineStride + i];
        float ms = 0.f;
        RT_HIP(r, hipEventElapsedTime(&ms, r->ev0, r->ev1));
        memset(stats, 0, sizeof(*stats));
        const uint64_t px = a.tiles ? 0 : (uint64_t)a.W * a.H;
        stats->primary_rays = r->cfg.mode == RT_MODE_SCENE ? c[0] : px;
        stats->shadow_rays = c[1];
        stats->nodes_visited = c[2];
        stats->prims_tested = c[3];
        stats->ms = ms;
        stats->samples_per_pixel = r->cfg.mode != RT_MODE_SCENE ? 1u
                                   : a.accum ? a.spp * r->frames_accum : a.spp;
        if ((ost = queue_report(r))) return ost;
    }
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }

int rt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

void rt_config_default(rt_config* c) {
    memset(c, 0, sizeof(*c));
    c->width = 1280;  // main.cpp:6
    c->height = 720;
    c->spp = 1;
    c->seed = 0x2545F491u;
    c->device = -1;
    c->mode = RT_MODE_COMPAT;
    c->flags = 0;
    c->light_dir[0] = 1.0f;  // normalize(1,1,-1)
    c->light_dir[1] = 1.0f;
    c->light_dir[2] = -1.0f;
    c->ambient = 0.1f;
}

void rt_octree_params_default(rt_octree_params* p) {
    memset(p, 0, sizeof(*p));
    for (int i = 0; i < 3; ++i) {
        p->min[i] = 0.0f;   // src/renderer.cu:134
        p->max[i] = 1.28f;  // src/renderer.cu:135
    }
    p->resolution = 0.01f;  // src/renderer.cu:136
    p->max_depth = 0;
    p->leaf_capacity = 8;
}

void rt_resize_intrinsic(uint32_t width, uint32_t height, float K[9]) {
    // src/renderer.cu:162-170 (float arithmetic, integer cx/cy)
    const float rad = 80.f * 0.01745329251994329576923690768489f;
    const float f = static_cast<float>(width) / (2.0f * tanf(rad / 2.0f));
    for (int i = 0; i < 9; ++i) K[i] = 0.0f;
    K[0] = f;
    K[4] = f;
    K[8] = 1.0f;
    K[2] = static_cast<float>(width / 2u);
    K[5] = static_cast<float>(height / 2u);
}

int rt_create(const rt_config* cfg, rt_renderer** out) {
    if (!cfg || !out) return fail(nullptr, RT_E_INVALID, "rt_create: null argument");
    *out = nullptr;
    if (cfg->width == 0 || cfg->height == 0 || cfg->width > 32768 || cfg->height > 32768)
        return fail(nullptr, RT_E_INVALID, "rt_create: width/height out of range");
    if (cfg->mode != RT_MODE_COMPAT && cfg->mode != RT_MODE_SCENE)
        return fail(nullptr, RT_E_INVALID, "rt_create: unknown mode");
    if (!variant_available((cfg->flags >> RT_FLAG_VARIANT_SHIFT) & 0xFu))
        return fail(nullptr, RT_E_INVALID,
                    "rt_create: scene-kernel variant not in this build (0, 4, 7, 10 or 13)");
    if (((cfg->flags >> (RT_FLAG_OPT_SHIFT + kOptChunkShift)) & 7u) > kOptChunkMax)
        return fail(nullptr, RT_E_INVALID,
                    "rt_create: wave-queue ticket size field (flags bits 24..26) must be 0..4");
    rt_renderer* r = new (std::nothrow) rt_renderer();
    if (!r) return fail(nullptr, RT_E_NOMEM, "rt_create: out of host memory");
    r->cfg = *cfg;
    if (r->cfg.spp == 0) r->cfg.spp = 1;
    int dev = cfg->device;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    }
    r->device = dev;
    r->W = cfg->width;
    r->H = cfg->height;
    // test only (tests/test_gpu_variants.py, test_gpu_queue_report.py)
    if (const char* cd = test_env(cfg->flags, "RT_TEST_CLAIM_DELAY"))
        r->test_claim_delay = static_cast<uint32_t>(std::min(100000ul, strtoul(cd, nullptr, 10)));
    if (const char* fe = test_env(cfg->flags, "RT_TEST_FAULT"))
        r->test_fault_queue = strcmp(fe, "queue:0") == 0;
    // src/renderer.cu:87-89: K0 = mat3(1000,0,640, 0,1000,340, 0,0,1), pose = mat4(1)
    const float K0[9] = {1000.f, 0.f, 640.f, 0.f, 1000.f, 340.f, 0.f, 0.f, 1.f};
    memcpy(r->K, K0, sizeof(K0));
    for (int i = 0; i < 16; ++i) r->pose[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    rt_octree_params_default(&r->oct);
    int st;
    hipError_t e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&r->ev0);
    if (e == hipSuccess) e = hipEventCreate(&r->ev1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&r->done, hipEventDisableTiming);
    // the frame-failure word: pinned, host-coherent, mapped for the kernels
    if (e == hipSuccess)
        e = hipHostMalloc(reinterpret_cast<void**>(&r->qerr_host), sizeof(uint32_t),
                          hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
        *r->qerr_host = 0;
        e = hipHostGetDevicePointer(reinterpret_cast<void**>(&r->qerr_dev), r->qerr_host, 0);
    }
    if (e != hipSuccess) {
        st = hip_fail(nullptr, e, "rt_create");
        rt_destroy(r);
        return st;
    }
    if ((st = ensure(r, r->fb, (size_t)r->W * r->H)) ||
        (st = ensure(r, r->counters, kCounterWords))) {
        g_last_error = r->err;
        rt_destroy(r);
        return st;
    }
    if (cfg->flags & RT_FLAG_PROGRESSIVE) {
        if ((st = ensure(r, r->accum, (size_t)r->W * r->H))) {
            g_last_error = r->err;
            rt_destroy(r);
            return st;
        }
    }
    if (cfg->flags & RT_FLAG_RADIANCE) {
        if ((st = ensure(r, r->rad, (size_t)r->W * r->H))) {
            g_last_error = r->err;
            rt_destroy(r);
            return st;
        }
    }
    *out = r;
    return RT_OK;
}

int rt_destroy(rt_renderer* r) {
    if (!r) return RT_OK;
    if (r->multi) multi_destroy(r);
    (void)hipSetDevice(r->device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    if (r->pending) (void)hipEventSynchronize(r->done);  // work on a caller's stream
    r->fb.release();
    r->rad.release();
    r->accum.release();
    r->counters.release();
    for (auto& e : r->tile_lists) e.dev.release();
    r->d_nodes.release();
    r->d_prim_sp.release();
    r->d_prim_idx.release();
    r->d_spheres.release();
    r->d_albedo.release();
    r->d_prim_cam.release();
    r->d_prim_al.release();
    r->d_prim_cam8.release();
    r->d_prim_shd8.release();
    r->d_shd_rr.release();
    r->d_prim_shd.release();
    r->sb_order.release();
    r->gpu_build.release();
    r->cell_table.release();
    if (r->ev0) (void)hipEventDestroy(r->ev0);
    if (r->ev1) (void)hipEventDestroy(r->ev1);
    if (r->done) (void)hipEventDestroy(r->done);
    if (r->stream) (void)hipStreamDestroy(r->stream);
    if (r->qerr_host) (void)hipHostFree(r->qerr_host);
    delete r;
    return RT_OK;
}

int rt_set_pose(rt_renderer* r, const float pose[16]) {
    if (!r || !pose) return fail(r, RT_E_INVALID, "rt_set_pose: null argument");
    if (memcmp(r->pose, pose, sizeof(r->pose)) != 0) r->frames_accum = 0;
    memcpy(r->pose, pose, sizeof(r->pose));
    return for_peers(r, [&](rt_renderer* p) { return rt_set_pose(p, pose); });
}

int rt_set_intrinsic(rt_renderer* r, const float K[9]) {
    if (!r || !K) return fail(r, RT_E_INVALID, "rt_set_intrinsic: null argument");
    if (memcmp(r->K, K, sizeof(r->K)) != 0) r->frames_accum = 0;
    memcpy(r->K, K, sizeof(r->K));
    return for_peers(r, [&](rt_renderer* p) { return rt_set_intrinsic(p, K); });
}

int rt_get_camera(const rt_renderer* r, float pose_out[16], float K_out[9]) {
    if (!r) return RT_E_INVALID;
    if (pose_out) memcpy(pose_out, r->pose, sizeof(r->pose));
    if (K_out) memcpy(K_out, r->K, sizeof(r->K));
    return RT_OK;
}

int rt_resize(rt_renderer* r, uint32_t width, uint32_t height) {
    if (!r) return fail(r, RT_E_INVALID, "rt_resize: null handle");
    if (width == 0 || height == 0 || width > 32768 || height > 32768)
        return fail(r, RT_E_INVALID, "rt_resize: width/height out of range");
    int st;
    // every queued frame that may still write the buffers released below has
    // finished first, on whichever stream it ran (a caller's, a multi-device
    // handle's comm and output streams)
    if (r->multi && (st = multi_wait(r))) return st;
    if ((st = set_device(r))) return st;
    RT_HIP(r, hipStreamSynchronize(r->stream));
    if (r->pending) RT_HIP(r, hipEventSynchronize(r->done));
    // a multi-device handle is inconsistent until every device has resized
    if (r->multi) r->multi->broken = true;
    r->W = width;
    r->H = height;
    r->frames_accum = 0;
    if ((st = ensure(r, r->fb, (size_t)width * height))) return st;
    if (r->cfg.flags & RT_FLAG_PROGRESSIVE)
        if ((st = ensure(r, r->accum, (size_t)width * height))) return st;
    if (r->cfg.flags & RT_FLAG_RADIANCE)
        if ((st = ensure(r, r->rad, (size_t)width * height))) return st;
    rt_resize_intrinsic(width, height, r->K);
    if ((st = for_peers(r, [&](rt_renderer* p) { return rt_resize(p, width, height); }))) return st;
    if (r->multi) r->multi->broken = false;  // the slabs are re-planned at the next frame
    return RT_OK;
}

int rt_set_scene(rt_renderer* r, const float* spheres, const uint32_t* albedo, uint32_t n,
                 const rt_octree_params* oct) {
    if (!r) return fail(r, RT_E_INVALID, "rt_set_scene: null handle");
    if (n && !spheres) return fail(r, RT_E_INVALID, "rt_set_scene: null spheres");
    int st;
    if ((st = check_octree_params(r, oct, "rt_set_scene"))) return st;
    for (uint32_t i = 0; i < n; ++i) {
        const float* s = spheres + 4u * i;
        if (!(s[3] > 0.0f) || !isfinite(s[0]) || !isfinite(s[1]) || !isfinite(s[2]) ||
            !isfinite(s[3]))
            return fail(r, RT_E_INVALID,
                        "rt_set_scene: sphere with radius <= 0 or non-finite values");
    }
    if (oct) r->oct = *oct;
    if ((st = set_device(r))) return st;
    RT_HIP(r, hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    r->spheres.assign(spheres, spheres + 4u * n);
    r->host_copy = true;
    r->n_spheres = n;
    std::vector<uint32_t> alb(n);
    for (uint32_t i = 0; i < n; ++i) alb[i] = albedo ? albedo[i] : 0xFFCCCCCCu;
    if ((st = ensure(r, r->d_spheres, n))) return st;
    if ((st = ensure(r, r->d_albedo, n))) return st;
    if (n) {
        RT_HIP(r, hipMemcpy(r->d_spheres.p, spheres, n * sizeof(float4), hipMemcpyHostToDevice));
        RT_HIP(r, hipMemcpy(r->d_albedo.p, alb.data(), n * sizeof(uint32_t), hipMemcpyHostToDevice));
    }
    r->info.upload_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if ((st = build_scene(r))) return st;
    return for_peers(r, [&](rt_renderer* p) { return rt_set_scene(p, spheres, albedo, n, oct); });
}

int rt_set_scene_device(rt_renderer* r, const void* dev_spheres, const void* dev_albedo,
                        uint32_t n, const rt_octree_params* oct, void* stream) {
    if (!r) return fail(r, RT_E_INVALID, "rt_set_scene_device: null handle");
    if (n && !dev_spheres) return fail(r, RT_E_INVALID, "rt_set_scene_device: null spheres");
    int st;
    if ((st = check_octree_params(r, oct, "rt_set_scene_device"))) return st;
    if ((st = set_device(r))) return st;
    if (stream) RT_HIP(r, hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    const float4* src = static_cast<const float4*>(dev_spheres);
    if (n) {
        SphereBounds sb;
        hipError_t e = r->gpu_build.bounds(src, n, r->stream, &sb);
        if (e != hipSuccess) return hip_fail(r, e, "rt_set_scene_device: validation");
        if (sb.n_invalid)
            return fail(r, RT_E_INVALID,
                        "rt_set_scene_device: sphere with radius <= 0 or non-finite values");
    }
    if (oct) r->oct = *oct;
    RT_HIP(r, hipDeviceSynchronize());
    auto t0 = std::chrono::steady_clock::now();
    if ((st = ensure(r, r->d_spheres, n))) return st;
    if ((st = ensure(r, r->d_albedo, n))) return st;
    if (n) {
        RT_HIP(r, hipMemcpyAsync(r->d_spheres.p, src, n * sizeof(float4), hipMemcpyDeviceToDevice,
                                 r->stream));
        if (dev_albedo)
            RT_HIP(r, hipMemcpyAsync(r->d_albedo.p, dev_albedo, n * sizeof(uint32_t),
                                     hipMemcpyDeviceToDevice, r->stream));
        else
            RT_HIP(r, hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(r->d_albedo.p),
                                        0xFFCCCCCCu, n, r->stream));
        RT_HIP(r, hipStreamSynchronize(r->stream));
    }
    r->n_spheres = n;
    r->spheres.clear();
    r->host_copy = false;
    r->info.upload_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if ((st = build_scene(r))) return st;
    // a multi-device handle: the validated list (now in d_spheres / d_albedo
    // on devices[0]) is broadcast to the other devices, which build their trees
    return r->multi ? multi_set_scene_device(r, n, oct) : RT_OK;
}

int rt_set_octree(rt_renderer* r, const float mn[3], const float mx[3], float resolution) {
    if (!r || !mn || !mx) return fail(r, RT_E_INVALID, "rt_set_octree: null argument");
    rt_octree_params p = r->oct;
    for (int i = 0; i < 3; ++i) {
        p.min[i] = mn[i];
        p.max[i] = mx[i];
        if (!(mx[i] > mn[i])) return fail(r, RT_E_INVALID, "rt_set_octree: empty box");
    }
    if (!(resolution > 0.0f)) return fail(r, RT_E_INVALID, "rt_set_octree: resolution <= 0");
    p.resolution = resolution;
    p.max_depth = 0;
    r->oct = p;
    int st;
    if (r->has_scene && (st = build_scene(r))) return st;
    return for_peers(r, [&](rt_renderer* q) { return rt_set_octree(q, mn, mx, resolution); });
}

int rt_get_scene_info(const rt_renderer* r, rt_scene_info* info) {
    if (!r || !info) return RT_E_INVALID;
    if (!r->has_scene) return RT_E_NOSCENE;
    *info = r->info;
    return RT_OK;
}

int rt_export_octree(rt_renderer* r, uint32_t* nodes_out, float* prim_sp_out,
                     uint32_t* prim_idx_out) {
    if (!r) return fail(r, RT_E_INVALID, "rt_export_octree: null handle");
    if (!r->has_scene) return fail(r, RT_E_NOSCENE, "rt_export_octree: no scene");
    int st;
    if ((st = set_device(r))) return st;
    RT_HIP(r, hipDeviceSynchronize());
    const size_t nn = r->info.n_nodes, np = r->info.n_prim_refs;
    if (r->leaf_packed) {
        // the builders' record-for-record tree: the line-packed lists
        // (pack_leaf_lines) put back to back again, in the same order
        std::vector<uint2> nodes(nn);
        RT_HIP(r, hipMemcpy(nodes.data(), r->sc.nodes, nn * sizeof(uint2), hipMemcpyDeviceToHost));
        std::vector<float4> sp(r->prim_slots);
        std::vector<uint32_t> ix(r->prim_slots);
        if (r->prim_slots) {
            RT_HIP(r, hipMemcpy(sp.data(), r->sc.prim_sp, sp.size() * sizeof(float4), hipMemcpyDeviceToHost));
            RT_HIP(r, hipMemcpy(ix.data(), r->sc.prim_idx, ix.size() * sizeof(uint32_t),
                                hipMemcpyDeviceToHost));
        }
        uint32_t off = 0;
        for (uint32_t i : leaf_records(nodes)) {
            uint2& rec = nodes[i];
            if (prim_sp_out)
                memcpy(prim_sp_out + 4u * size_t(off), sp.data() + rec.x, rec.y * sizeof(float4));
            if (prim_idx_out) memcpy(prim_idx_out + off, ix.data() + rec.x, rec.y * sizeof(uint32_t));
            rec.x = off;
            off += rec.y;
        }
        if (nodes_out) memcpy(nodes_out, nodes.data(), nn * sizeof(uint2));
        return RT_OK;
    }
    if (nodes_out)
        RT_HIP(r, hipMemcpy(nodes_out, r->sc.nodes, nn * sizeof(uint2), hipMemcpyDeviceToHost));
    if (prim_sp_out && np)
        RT_HIP(r, hipMemcpy(prim_sp_out, r->sc.prim_sp, np * sizeof(float4), hipMemcpyDeviceToHost));
    if (prim_idx_out && np)
        RT_HIP(r, hipMemcpy(prim_idx_out, r->sc.prim_idx, np * sizeof(uint32_t),
                            hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_save_spheres(const char* path, const float* spheres, const uint32_t* albedo, uint32_t n) {
    if (!path || (n && !spheres)) return fail(nullptr, RT_E_INVALID, "rt_save_spheres: null argument");
    std::string err;
    if (!save_sphere_file(path, spheres, albedo, n, &err)) return fail(nullptr, RT_E_INVALID, err);
    return RT_OK;
}

int rt_load_spheres(const char* path, float* spheres_out, uint32_t* albedo_out, uint32_t capacity,
                    uint32_t* n_out) {
    if (!path || !n_out) return fail(nullptr, RT_E_INVALID, "rt_load_spheres: null argument");
    std::string err;
    if (!load_sphere_file(path, spheres_out, albedo_out, capacity, n_out, &err))
        return fail(nullptr, RT_E_INVALID, err);
    return RT_OK;
}

int rt_generate_spheres(uint32_t n, uint32_t seed, float* spheres_out, uint32_t* albedo_out) {
    if (n && !spheres_out) return fail(nullptr, RT_E_INVALID, "rt_generate_spheres: null output");
    generate_spheres(n, seed, spheres_out, albedo_out);
    return RT_OK;
}

int rt_render(rt_renderer* r, void* dev_rgba8, void* stream, rt_stats* stats) {
    if (!r) return fail(r, RT_E_INVALID, "rt_render: null handle");
    int st;
    // an earlier frame the kernel found incomplete: reported here, before
    // anything is queued, by a host read (no sync: the Displayer's frames
    // into a mapped PBO are never read back)
    if (r->multi) {
        if ((st = multi_queue_report(r))) return st;
    } else if ((st = queue_report(r))) {
        return st;
    }
    if ((st = set_device(r))) return st;
    // (a multi-device handle's renderers accumulate per tile list, in multi_render)
    if (!r->multi) accum_pixels(r, nullptr, 0, 0);
    FrameArgs a;
    fill_frame_args(r, a);
    a.out8 = dev_rgba8 ? static_cast<uint32_t*>(dev_rgba8) : r->fb.p;
    a.out32 = (r->cfg.flags & RT_FLAG_RADIANCE) ? r->rad.p : nullptr;
    // (a resize whose allocation failed leaves no internal framebuffer)
    if (!a.out8 || ((r->cfg.flags & RT_FLAG_RADIANCE) && !a.out32))
        return fail(r, RT_E_STATE, "rt_render: no framebuffer (a resize failed): resize again");
    const auto render_into = [&](hipStream_t hs) -> int {
        return r->multi ? multi_render(r, a.out8, hs, stats) : do_render(r, a, hs, stats);
    };
    if (dev_rgba8 || !r->disp.map) return render_into(static_cast<hipStream_t>(stream));
    // the reference's render(): map the PBO, launch into it, unmap
    // (src/renderer.cu:145-151)
    hipStream_t hs = stream ? static_cast<hipStream_t>(stream) : own_stream(r);
    if ((st = order_after_last(r, hs))) return st;
    void* ptr = nullptr;
    size_t bytes = 0;
    const int em = r->disp.map(r->disp_user, hs, &ptr, &bytes);
    if (em != 0) {
        std::string m = "rt_render: display buffer map failed (" + std::to_string(em) + ")";
        if (r->gl_disp) m += std::string(": ") + hipGetErrorString(static_cast<hipError_t>(em));
        return fail(r, RT_E_HIP, m);
    }
    if (!ptr || bytes < (size_t)r->W * r->H * 4) {
        (void)r->disp.unmap(r->disp_user, hs);
        return fail(r, RT_E_INVALID, "rt_render: display buffer smaller than W*H*4 bytes");
    }
    a.out8 = static_cast<uint32_t*>(ptr);
    st = render_into(hs);
    const int eu = r->disp.unmap(r->disp_user, hs);
    if (st) return st;
    if (eu != 0) {
        std::string m = "rt_render: display buffer unmap failed (" + std::to_string(eu) + ")";
        if (r->gl_disp) m += std::string(": ") + hipGetErrorString(static_cast<hipError_t>(eu));
        return fail(r, RT_E_HIP, m);
    }
    return RT_OK;
}

namespace {
// built-in ops over a hipGraphicsResource_t (hipGraphicsGLRegisterBuffer);
// the status is the hipError_t
int gl_map(void* user, void* stream, void** ptr, size_t* bytes) {
    hipGraphicsResource_t res = static_cast<hipGraphicsResource_t>(user);
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipGraphicsMapResources(1, &res, s);
    if (e != hipSuccess) return static_cast<int>(e);
    e = hipGraphicsResourceGetMappedPointer(ptr, bytes, res);
    if (e != hipSuccess) (void)hipGraphicsUnmapResources(1, &res, s);
    return static_cast<int>(e);
}
int gl_unmap(void* user, void* stream) {
    hipGraphicsResource_t res = static_cast<hipGraphicsResource_t>(user);
    return static_cast<int>(hipGraphicsUnmapResources(1, &res, static_cast<hipStream_t>(stream)));
}
}  // namespace

int rt_bind_display(rt_renderer* r, const rt_display_ops* ops, void* user) {
    if (!r) return fail(r, RT_E_INVALID, "rt_bind_display: null handle");
    if (ops && (!ops->map || !ops->unmap))
        return fail(r, RT_E_INVALID, "rt_bind_display: map and unmap are both required");
    r->disp = ops ? *ops : rt_display_ops{};
    r->disp_user = ops ? user : nullptr;
    r->gl_disp = false;
    return RT_OK;
}

int rt_bind_graphics_resource(rt_renderer* r, void* resource) {
    if (!r) return fail(r, RT_E_INVALID, "rt_bind_graphics_resource: null handle");
    static const rt_display_ops kGl = {gl_map, gl_unmap};
    const int st = rt_bind_display(r, resource ? &kGl : nullptr, resource);
    r->gl_disp = resource != nullptr;
    return st;
}

int rt_render_tiles(rt_renderer* r, const uint32_t* tile_ids, uint32_t n_tiles, uint32_t ts,
                    void* dev_packed, void* stream, rt_stats* stats) {
    if (!r) return fail(r, RT_E_INVALID, "rt_render_tiles: null handle");
    if (r->multi)
        return fail(r, RT_E_STATE, "rt_render_tiles: a multi-device handle renders whole frames");
    return render_tiles_one(r, tile_ids, n_tiles, ts, dev_packed, stream, stats);
}

int rt_unpack_tiles(rt_renderer* r, const void* dev_packed, const uint32_t* tile_ids,
                    uint32_t n_tiles, uint32_t ts, void* dev_rgba8, void* stream) {
    if (!r) return fail(r, RT_E_INVALID, "rt_unpack_tiles: null handle");
    if (r->multi)
        return fail(r, RT_E_STATE, "rt_unpack_tiles: a multi-device handle renders whole frames");
    return unpack_tiles_one(r, dev_packed, tile_ids, n_tiles, ts, dev_rgba8, stream);
}

}  // extern "C"

namespace {
int render_tiles_one(rt_renderer* r, const uint32_t* tile_ids, uint32_t n_tiles, uint32_t ts,
                     void* dev_packed, void* stream, rt_stats* stats) {
    if (n_tiles && (!tile_ids || !dev_packed))
        return fail(r, RT_E_INVALID, "rt_render_tiles: null argument");
    int st;
    if ((st = check_tiles(r, tile_ids, n_tiles, ts))) return st;
    const uint32_t tx = (r->W + ts - 1) / ts;
    if ((st = set_device(r))) return st;
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->stream;
    if (n_tiles == 0) {
        if (stats) memset(stats, 0, sizeof(*stats));
        return RT_OK;
    }
    const uint32_t* dev_ids = nullptr;
    if ((st = order_after_last(r, s))) return st;
    if ((st = tile_list(r, tile_ids, n_tiles, s, &dev_ids))) return st;
    accum_pixels(r, tile_ids, n_tiles, ts);
    FrameArgs a;
    fill_frame_args(r, a);
    a.out8 = static_cast<uint32_t*>(dev_packed);
    a.out32 = nullptr;
    a.tiles = dev_ids;
    a.n_tiles = n_tiles;
    a.tile_size = ts;
    a.tiles_x = tx;
    st = do_render(r, a, s, stats);
    if (!st && stats && r->cfg.mode != RT_MODE_SCENE) {
        uint64_t px = 0;
        for (uint32_t i = 0; i < n_tiles; ++i) {
            const uint32_t x0 = (tile_ids[i] % tx) * ts, y0 = (tile_ids[i] / tx) * ts;
            const uint64_t w = std::min<uint64_t>(ts, r->W - x0), h = std::min<uint64_t>(ts, r->H - y0);
            px += w * h;
        }
        stats->primary_rays = px;
    }
    return st;
}

int unpack_tiles_one(rt_renderer* r, const void* dev_packed, const uint32_t* tile_ids,
                     uint32_t n_tiles, uint32_t ts, void* dev_rgba8, void* stream) {
    if (n_tiles && (!tile_ids || !dev_packed)) return fail(r, RT_E_INVALID, "rt_unpack_tiles: null argument");
    int st;
    if ((st = check_tiles(r, tile_ids, n_tiles, ts, /*allow_skip=*/true))) return st;
    if (n_tiles == 0) return RT_OK;
    const uint32_t tx = (r->W + ts - 1) / ts;
    if ((st = set_device(r))) return st;
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : r->stream;
    const uint32_t* dev_ids = nullptr;
    if ((st = order_after_last(r, s))) return st;
    if ((st = tile_list(r, tile_ids, n_tiles, s, &dev_ids))) return st;
    hipError_t e = launch_unpack(static_cast<const uint32_t*>(dev_packed), dev_ids, n_tiles, ts, tx,
                                 r->W, r->H, dev_rgba8 ? static_cast<uint32_t*>(dev_rgba8) : r->fb.p, s);
    if (e != hipSuccess) return hip_fail(r, e, "rt_unpack_tiles");
    return mark_queued(r, s);
}
}  // namespace

extern "C" {

int rt_reset_accumulation(rt_renderer* r) {
    if (!r) return fail(r, RT_E_INVALID, "rt_reset_accumulation: null handle");
    r->frames_accum = 0;
    return for_peers(r, [](rt_renderer* p) { return rt_reset_accumulation(p); });
}

// After the renderer's work has completed: the wave queue's bounded wait
// (rt_kernels.hip) marks a frame whose slot was never published instead of
// hanging; every such frame not reported yet is reported now.
int rt_synchronize(rt_renderer* r) {
    if (!r) return RT_E_INVALID;
    int st;
    if (r->multi && (st = multi_synchronize(r))) return st;
    if ((st = set_device(r))) return st;
    RT_HIP(r, hipStreamSynchronize(r->stream));
    if (r->pending) RT_HIP(r, hipEventSynchronize(r->done));
    return queue_report(r);
}

int rt_readback(rt_renderer* r, uint8_t* host_rgba8, float* host_rgba32f) {
    if (!r) return RT_E_INVALID;
    int st;
    if (r->multi && (st = multi_synchronize(r))) return st;
    if ((st = set_device(r))) return st;
    // the frame may have been queued on a caller's stream
    RT_HIP(r, hipStreamSynchronize(r->stream));
    if (r->pending) RT_HIP(r, hipEventSynchronize(r->done));
    if ((st = queue_report(r))) return st;
    const size_t px = (size_t)r->W * r->H;
    if (host_rgba8) RT_HIP(r, hipMemcpy(host_rgba8, r->fb.p, px * 4, hipMemcpyDeviceToHost));
    if (host_rgba32f) {
        if (!(r->cfg.flags & RT_FLAG_RADIANCE))
            return fail(r, RT_E_STATE, "rt_readback: radiance buffer needs RT_FLAG_RADIANCE");
        RT_HIP(r, hipMemcpy(host_rgba32f, r->rad.p, px * 16, hipMemcpyDeviceToHost));
    }
    return RT_OK;
}

void* rt_framebuffer(rt_renderer* r) { return r ? r->fb.p : nullptr; }

void* rt_stream(rt_renderer* r) { return r ? static_cast<void*>(own_stream(r)) : nullptr; }

const char* rt_last_error(const rt_renderer* r) {
    if (r) return r->err.c_str();
    return g_last_error.c_str();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Multi-device handle (rt_create_multi; SURVEY 8b B2 "device ids", 8e E1)
//
// One process drives n devices.  Frame j uses slot f = j mod 2:
//   device k, its renderer's stream : [wait sent[f][k]]  render its tiles -> slab[f][k]
//                                      record rendered[f][k]
//   device k, comm stream cs[k]     : wait rendered[f][k]; send slab[f][k] to device 0
//                                      record sent[f][k]
//   device 0, comm stream cs[0]     : [wait unpacked[f]]; receive slab k into
//                                      recv[f] + k * slab; record recvd[f]
//   device 0, output stream hs      : record out_ready; cs[0] waits it and recvd[f], unpacks
//                                      the n slabs in ONE launch into the frame; hs waits
//                                      unpacked[f]
// so frame j+1's tiles render while frame j's slabs travel and unpack, and a
// slab or receive buffer is rewritten only after its previous frame let go of
// it.  Transport: RCCL (grouped ncclSend / ncclRecv over one ncclCommInitAll
// communicator, device 0 receiving from itself too) or peer copies
// (hipMemcpyPeerAsync: distinct devices over xGMI, or the same device in a
// rehearsal of the n-way plan on one GPU).
// ---------------------------------------------------------------------------
namespace {

// RCCL resolved at run time: librt_amd.so does not link it, so a process that
// already holds one (torch's) shares it, and single-device use never loads it.
struct RcclApi {
    bool ok = false;
    std::string why;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t,
                              hipStream_t) = nullptr;
    const char* (*ErrorString)(ncclResult_t) = nullptr;
};

RcclApi& rccl_api() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            api.why = std::string("librccl.so.1 not loadable: ") + dlerror();
            return;
        }
        bool all = true;
        auto sym = [&](const char* n) {
            void* p = dlsym(h, n);
            if (!p) all = false;
            return p;
        };
        api.CommInitAll = reinterpret_cast<decltype(api.CommInitAll)>(sym("ncclCommInitAll"));
        api.CommDestroy = reinterpret_cast<decltype(api.CommDestroy)>(sym("ncclCommDestroy"));
        api.GroupStart = reinterpret_cast<decltype(api.GroupStart)>(sym("ncclGroupStart"));
        api.GroupEnd = reinterpret_cast<decltype(api.GroupEnd)>(sym("ncclGroupEnd"));
        api.Send = reinterpret_cast<decltype(api.Send)>(sym("ncclSend"));
        api.Recv = reinterpret_cast<decltype(api.Recv)>(sym("ncclRecv"));
        api.Broadcast = reinterpret_cast<decltype(api.Broadcast)>(sym("ncclBroadcast"));
        api.ErrorString = reinterpret_cast<decltype(api.ErrorString)>(sym("ncclGetErrorString"));
        api.ok = all;
        if (!all) api.why = "librccl.so.1 lacks a required symbol";
    });
    return api;
}

int nccl_fail(rt_renderer* r, ncclResult_t e, const char* what) {
    const char* m = rccl_api().ErrorString ? rccl_api().ErrorString(e) : "?";
    return fail(r, RT_E_HIP, std::string(what) + ": RCCL error " + std::to_string((int)e) + " (" + m + ")");
}

#define RT_NCCL(r, call)                                         \
    do {                                                         \
        ncclResult_t e_ = (call);                                \
        if (e_ != ncclSuccess) return nccl_fail((r), e_, #call); \
    } while (0)

// (Re)plan the tiles and the buffers for the handle's current size: tile t to
// device t mod n (interleaved, so a centred scene balances), slabs
// of S = ceil(T / n) tiles, the gathered slabs unpacked with padding slots
// skipped.  Waits for in-flight frames before it frees anything.
int multi_plan(rt_renderer* r) {
    MultiState& m = *r->multi;
    if (m.W == r->W && m.H == r->H && m.recv[0]) return RT_OK;
    int st;
    if ((st = multi_wait(r))) return st;
    const uint32_t n = static_cast<uint32_t>(m.devs.size()), ts = MultiState::kTs;
    const uint32_t T = ((r->W + ts - 1) / ts) * ((r->H + ts - 1) / ts);
    m.S = (T + n - 1) / n;
    m.slab_bytes = (size_t)m.S * ts * ts * 4;
    m.ids.assign(n, {});
    for (uint32_t t = 0; t < T; ++t) m.ids[t % n].push_back(t);
    m.all_ids.assign((size_t)n * m.S, RT_TILE_SKIP);
    for (uint32_t k = 0; k < n; ++k)
        std::copy(m.ids[k].begin(), m.ids[k].end(), m.all_ids.begin() + (size_t)k * m.S);
    for (int f = 0; f < MultiState::F; ++f) {
        for (uint32_t k = 0; k < n; ++k) {
            RT_HIP(r, hipSetDevice(m.devs[k]));
            if (m.slab[f][k]) (void)hipFree(m.slab[f][k]);
            m.slab[f][k] = nullptr;
            hipError_t e = m.fault == MultiState::kSlab && k == m.fault_k
                               ? hipErrorOutOfMemory  // RT_TEST_FAULT=slab:k
                               : hipMalloc(&m.slab[f][k], m.slab_bytes);
            if (e != hipSuccess) {
                m.slab[f][k] = nullptr;
                return hip_fail(r, e, ("tile slab allocation" + peer_name(m, k)).c_str());
            }
        }
        RT_HIP(r, hipSetDevice(m.devs[0]));
        if (m.recv[f]) (void)hipFree(m.recv[f]);
        m.recv[f] = nullptr;
        RT_HIP(r, hipMalloc(&m.recv[f], m.slab_bytes * n));
        m.used[f] = false;
    }
    RT_HIP(r, hipSetDevice(m.devs[0]));
    if (m.d_all_ids) (void)hipFree(m.d_all_ids);
    m.d_all_ids = nullptr;
    RT_HIP(r, hipMalloc(reinterpret_cast<void**>(&m.d_all_ids), m.all_ids.size() * sizeof(uint32_t)));
    RT_HIP(r, hipMemcpy(m.d_all_ids, m.all_ids.data(), m.all_ids.size() * sizeof(uint32_t),
                        hipMemcpyHostToDevice));
    m.W = r->W;
    m.H = r->H;
    return RT_OK;
}

// Wait for all of the handle's queued work: every device's render and comm
// streams, devices[0]'s output stream and the unpacks.
int multi_wait(rt_renderer* r) {
    MultiState& m = *r->multi;
    for (size_t k = 0; k < m.devs.size(); ++k) {
        RT_HIP(r, hipSetDevice(m.devs[k]));
        if (k < m.cs.size() && m.cs[k]) RT_HIP(r, hipStreamSynchronize(m.cs[k]));
        // (a creation that failed part-way leaves later peers unmade)
        rt_renderer* p = m.peers[k];
        if (!p) continue;
        RT_HIP(r, hipStreamSynchronize(p->stream));
        if (p->pending) RT_HIP(r, hipEventSynchronize(p->done));
    }
    RT_HIP(r, hipSetDevice(m.devs[0]));
    if (m.out) RT_HIP(r, hipStreamSynchronize(m.out));
    for (int f = 0; f < MultiState::F; ++f)
        if (m.unpacked[f]) RT_HIP(r, hipEventSynchronize(m.unpacked[f]));
    return RT_OK;
}

// Every device's failure word (queue_report): a device whose frame the wave
// queue's bounded wait marked incomplete had its slab gathered and unpacked
// incomplete, so the handle reports RT_E_HIP naming that device, as a
// single-device renderer does for itself.  A host read, no sync.
int multi_queue_report(rt_renderer* r) {
    MultiState& m = *r->multi;
    for (size_t k = 0; k < m.peers.size(); ++k) {
        rt_renderer* p = m.peers[k];
        if (!p) continue;
        if (const int st = queue_report(p)) return fail(r, st, p->err + peer_name(m, k));
    }
    return RT_OK;
}

// multi_wait, then every device's failure word.
int multi_synchronize(rt_renderer* r) {
    int st;
    if ((st = multi_wait(r))) return st;
    if ((st = multi_queue_report(r))) return st;
    return set_device(r);
}

int multi_render(rt_renderer* r, uint32_t* out, hipStream_t hs, rt_stats* stats) {
    MultiState& m = *r->multi;
    int st;
    if (r->cfg.mode == RT_MODE_SCENE && !r->has_scene)
        return fail(r, RT_E_NOSCENE, "RT_MODE_SCENE render without rt_set_scene");
    if (m.broken)
        return fail(r, RT_E_STATE, "rt_render: a resize failed on one of the devices: resize again");
    if ((st = multi_plan(r))) return st;
    if (!hs) hs = m.out;
    const uint32_t n = static_cast<uint32_t>(m.devs.size()), ts = MultiState::kTs;
    const int f = static_cast<int>(m.frame % MultiState::F);
    const auto t0 = std::chrono::steady_clock::now();
    const bool timed = m.timing;
    m.timed[f] = false;
    rt_stats sum{};
    // 1. every device renders its tiles into its slab of slot f
    for (uint32_t k = 0; k < n; ++k) {
        rt_renderer* p = m.peers[k];
        RT_HIP(r, hipSetDevice(m.devs[k]));
        if (m.used[f]) RT_HIP(r, hipStreamWaitEvent(p->stream, m.sent[f][k], 0));
        if (timed) RT_HIP(r, hipEventRecord(m.t_start[f][k], p->stream));
        rt_stats sk{};
        st = render_tiles_one(p, m.ids[k].data(), static_cast<uint32_t>(m.ids[k].size()), ts,
                              m.slab[f][k], p->stream, stats ? &sk : nullptr);
        if (st) {
            r->err = p->err + peer_name(m, k);
            return st;
        }
        if (stats) {
            sum.primary_rays += sk.primary_rays;
            sum.shadow_rays += sk.shadow_rays;
            sum.nodes_visited += sk.nodes_visited;
            sum.prims_tested += sk.prims_tested;
            sum.samples_per_pixel = sk.samples_per_pixel;
        }
        if (timed) RT_HIP(r, hipEventRecord(m.t_end[f][k], p->stream));
        RT_HIP(r, hipEventRecord(m.rendered[f][k], p->stream));
        RT_HIP(r, hipStreamWaitEvent(m.cs[k], m.rendered[f][k], 0));
    }
    // 2. the slabs to devices[0]: recv[f] + k * slab
    RT_HIP(r, hipSetDevice(m.devs[0]));
    if (m.used[f]) RT_HIP(r, hipStreamWaitEvent(m.cs[0], m.unpacked[f], 0));
    char* rb = static_cast<char*>(m.recv[f]);
    if (m.transport == RT_TRANSPORT_RCCL) {
        RcclApi& api = rccl_api();
        RT_NCCL(r, api.GroupStart());
        for (uint32_t k = 0; k < n; ++k) {
            ncclResult_t e = api.Send(m.slab[f][k], m.slab_bytes, ncclUint8, 0, m.comms[k], m.cs[k]);
            if (e == ncclSuccess)
                e = api.Recv(rb + k * m.slab_bytes, m.slab_bytes, ncclUint8, static_cast<int>(k),
                             m.comms[0], m.cs[0]);
            if (e != ncclSuccess) {
                (void)api.GroupEnd();
                return nccl_fail(r, e, "ncclSend/ncclRecv");
            }
        }
        RT_NCCL(r, api.GroupEnd());
        for (uint32_t k = 0; k < n; ++k) {
            RT_HIP(r, hipSetDevice(m.devs[k]));
            RT_HIP(r, hipEventRecord(m.sent[f][k], m.cs[k]));
        }
    } else {
        for (uint32_t k = 0; k < n; ++k) {
            RT_HIP(r, hipSetDevice(m.devs[k]));
            // the copy writes devices[0]'s receive buffer from device k's stream:
            // after frame j-2's unpack has read it
            if (k && m.used[f]) RT_HIP(r, hipStreamWaitEvent(m.cs[k], m.unpacked[f], 0));
            RT_HIP(r, hipMemcpyPeerAsync(rb + k * m.slab_bytes, m.devs[0], m.slab[f][k], m.devs[k],
                                         m.slab_bytes, m.cs[k]));
            RT_HIP(r, hipEventRecord(m.sent[f][k], m.cs[k]));
        }
        RT_HIP(r, hipSetDevice(m.devs[0]));
        for (uint32_t k = 1; k < n; ++k) RT_HIP(r, hipStreamWaitEvent(m.cs[0], m.sent[f][k], 0));
    }
    // 3. one unpack of all slabs on devices[0], after the output stream's
    //    earlier work (a mapped display buffer is ready) and the slabs' arrival
    RT_HIP(r, hipSetDevice(m.devs[0]));
    RT_HIP(r, hipEventRecord(m.recvd[f], m.cs[0]));
    // (RT_FLAG_TEST_POISON: the frame's pixels all come from the unpack)
    if (r->cfg.flags & RT_FLAG_TEST_POISON)
        RT_HIP(r, hipMemsetAsync(out, 0xAB, (size_t)r->W * r->H * 4, hs));
    RT_HIP(r, hipEventRecord(m.out_ready, hs));
    RT_HIP(r, hipStreamWaitEvent(m.cs[0], m.out_ready, 0));
    hipError_t e = launch_unpack(static_cast<const uint32_t*>(m.recv[f]), m.d_all_ids, n * m.S, ts,
                                 (r->W + ts - 1) / ts, r->W, r->H, out, m.cs[0]);
    if (e != hipSuccess) return hip_fail(r, e, "multi-device unpack");
    if (timed) RT_HIP(r, hipEventRecord(m.t_unpacked[f], m.cs[0]));
    RT_HIP(r, hipEventRecord(m.unpacked[f], m.cs[0]));
    RT_HIP(r, hipStreamWaitEvent(hs, m.unpacked[f], 0));
    m.used[f] = true;
    m.timed[f] = timed;
    ++m.frame;
    if (stats) {
        RT_HIP(r, hipStreamSynchronize(hs));
        sum.ms = static_cast<float>(
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        if (r->cfg.mode != RT_MODE_SCENE) sum.primary_rays = (uint64_t)r->W * r->H;
        *stats = sum;
    }
    return RT_OK;
}

int multi_set_scene_device(rt_renderer* r, uint32_t n, const rt_octree_params* oct) {
    MultiState& m = *r->multi;
    const uint32_t nd = static_cast<uint32_t>(m.devs.size());
    if (nd < 2) return RT_OK;
    // each other device receives the list into a scratch pair, then builds
    std::vector<void*> sp(nd, nullptr), al(nd, nullptr);
    int st = RT_OK;
    auto release = [&] {
        for (uint32_t k = 1; k < nd; ++k) {
            (void)hipSetDevice(m.devs[k]);
            if (sp[k]) (void)hipFree(sp[k]);
            if (al[k]) (void)hipFree(al[k]);
        }
        (void)hipSetDevice(m.devs[0]);
    };
    const size_t nb = std::max<size_t>(1, (size_t)n) * sizeof(float4);
    const size_t ab = std::max<size_t>(1, (size_t)n) * sizeof(uint32_t);
    for (uint32_t k = 1; k < nd && !st; ++k) {
        hipError_t e = hipSetDevice(m.devs[k]);
        if (e == hipSuccess) e = hipMalloc(&sp[k], nb);
        if (e == hipSuccess) e = hipMalloc(&al[k], ab);
        if (e != hipSuccess) st = hip_fail(r, e, "rt_set_scene_device: broadcast buffers");
    }
    if (!st && n) {
        if (m.transport == RT_TRANSPORT_RCCL) {
            // ncclBroadcast from devices[0]: spheres as 4n floats, albedo as n words
            RcclApi& api = rccl_api();
            ncclResult_t e = api.GroupStart();
            for (uint32_t k = 0; k < nd && e == ncclSuccess; ++k) {
                void* dst = k ? sp[k] : r->d_spheres.p;
                e = api.Broadcast(r->d_spheres.p, dst, (size_t)n * 4, ncclFloat32, 0, m.comms[k], m.cs[k]);
                if (e == ncclSuccess)
                    e = api.Broadcast(r->d_albedo.p, k ? al[k] : r->d_albedo.p, n, ncclUint32, 0,
                                      m.comms[k], m.cs[k]);
            }
            const ncclResult_t e2 = api.GroupEnd();
            if (e == ncclSuccess) e = e2;
            if (e != ncclSuccess) st = nccl_fail(r, e, "ncclBroadcast");
        } else {
            for (uint32_t k = 1; k < nd && !st; ++k) {
                hipError_t e = hipSetDevice(m.devs[k]);
                if (e == hipSuccess)
                    e = hipMemcpyPeerAsync(sp[k], m.devs[k], r->d_spheres.p, m.devs[0], nb, m.cs[k]);
                if (e == hipSuccess)
                    e = hipMemcpyPeerAsync(al[k], m.devs[k], r->d_albedo.p, m.devs[0], ab, m.cs[k]);
                if (e != hipSuccess) st = hip_fail(r, e, "rt_set_scene_device: peer copy");
            }
        }
    }
    for (uint32_t k = 1; k < nd && !st; ++k) {
        st = rt_set_scene_device(m.peers[k], sp[k], al[k], n, oct, m.cs[k]);
        if (st) r->err = m.peers[k]->err + " (device " + std::to_string(m.devs[k]) + ")";
    }
    release();
    return st;
}

void multi_destroy(rt_renderer* r) {
    MultiState* m = r->multi;
    (void)multi_wait(r);
    r->multi = nullptr;
    const size_t n = m->devs.size();
    for (size_t k = 0; k < n; ++k) {
        (void)hipSetDevice(m->devs[k]);
        for (int f = 0; f < MultiState::F; ++f) {
            if (k < m->slab[f].size() && m->slab[f][k]) (void)hipFree(m->slab[f][k]);
            for (auto* ev : {&m->rendered[f], &m->sent[f], &m->t_start[f], &m->t_end[f]})
                if (k < ev->size() && (*ev)[k]) (void)hipEventDestroy((*ev)[k]);
        }
        if (k < m->comms.size() && m->comms[k]) (void)rccl_api().CommDestroy(m->comms[k]);
        if (k < m->cs.size() && m->cs[k]) (void)hipStreamDestroy(m->cs[k]);
        if (k && m->peers[k]) rt_destroy(m->peers[k]);
    }
    (void)hipSetDevice(m->devs[0]);
    for (int f = 0; f < MultiState::F; ++f) {
        if (m->recv[f]) (void)hipFree(m->recv[f]);
        if (m->recvd[f]) (void)hipEventDestroy(m->recvd[f]);
        if (m->unpacked[f]) (void)hipEventDestroy(m->unpacked[f]);
        if (m->t_unpacked[f]) (void)hipEventDestroy(m->t_unpacked[f]);
    }
    if (m->out) (void)hipStreamDestroy(m->out);
    if (m->out_ready) (void)hipEventDestroy(m->out_ready);
    if (m->d_all_ids) (void)hipFree(m->d_all_ids);
    delete m;
}

}  // namespace

extern "C" {

int rt_create_multi(const rt_config* cfg, const int32_t* devices, uint32_t n_devices,
                    uint32_t transport, rt_renderer** out) {
    if (!cfg || !devices || !out) return fail(nullptr, RT_E_INVALID, "rt_create_multi: null argument");
    *out = nullptr;
    if (n_devices == 0 || n_devices > RT_MAX_DEVICES)
        return fail(nullptr, RT_E_INVALID, "rt_create_multi: n_devices must be 1..16");
    if (transport > RT_TRANSPORT_PEER) return fail(nullptr, RT_E_INVALID, "rt_create_multi: unknown transport");
    const int ndev = rt_device_count();
    bool distinct = true;
    for (uint32_t i = 0; i < n_devices; ++i) {
        if (devices[i] < 0 || devices[i] >= ndev)
            return fail(nullptr, RT_E_INVALID, "rt_create_multi: device ordinal out of range");
        for (uint32_t j = 0; j < i; ++j)
            if (devices[j] == devices[i]) distinct = false;
    }
    if (transport == RT_TRANSPORT_RCCL && !distinct)
        return fail(nullptr, RT_E_INVALID,
                    "rt_create_multi: RCCL needs distinct devices (a repeated ordinal is a "
                    "peer-copy rehearsal)");
    if (transport == RT_TRANSPORT_AUTO) transport = distinct && rccl_api().ok ? RT_TRANSPORT_RCCL : RT_TRANSPORT_PEER;
    if (transport == RT_TRANSPORT_RCCL && !rccl_api().ok)
        return fail(nullptr, RT_E_INVALID, "rt_create_multi: " + rccl_api().why);
    // the handle renders through packed tile slabs, which carry RGBA8 only
    if (cfg->flags & RT_FLAG_RADIANCE)
        return fail(nullptr, RT_E_INVALID,
                    "rt_create_multi: RT_FLAG_RADIANCE is not supported on a multi-device handle");
    // test-only fault injection (MultiState::Fault, RT_FLAG_TEST_HOOKS)
    int fault = MultiState::kNone;
    uint32_t fault_k = 0;
    if (const char* fe = test_env(cfg->flags, "RT_TEST_FAULT")) {
        const std::string f(fe);
        const size_t c = f.find(':');
        const std::string kind = f.substr(0, c);
        fault_k = c == std::string::npos ? 0u : static_cast<uint32_t>(strtoul(f.c_str() + c + 1, nullptr, 10));
        fault = kind == "create" ? MultiState::kCreate : kind == "comm" ? MultiState::kComm
              : kind == "slab" ? MultiState::kSlab : kind == "queue" ? MultiState::kQueue
              : MultiState::kNone;
    }
    rt_config c0 = *cfg;
    c0.device = devices[0];
    rt_renderer* r = nullptr;
    int st = rt_create(&c0, &r);
    if (st) return st;
    MultiState* m = new (std::nothrow) MultiState();
    if (!m) {
        rt_destroy(r);
        return fail(nullptr, RT_E_NOMEM, "rt_create_multi: out of host memory");
    }
    r->multi = m;
    m->transport = transport;
    m->fault = fault;
    m->fault_k = fault_k;
    m->devs.assign(devices, devices + n_devices);
    m->peers.assign(n_devices, nullptr);
    m->peers[0] = r;
    m->cs.assign(n_devices, nullptr);
    for (int f = 0; f < MultiState::F; ++f) {
        m->slab[f].assign(n_devices, nullptr);
        m->rendered[f].assign(n_devices, nullptr);
        m->sent[f].assign(n_devices, nullptr);
        m->t_start[f].assign(n_devices, nullptr);
        m->t_end[f].assign(n_devices, nullptr);
    }
    auto bail = [&](int code) {
        g_last_error = r->err.empty() ? g_last_error : r->err;
        rt_destroy(r);  // frees the multi state and the peers made so far
        return code;
    };
    for (uint32_t k = 1; k < n_devices; ++k) {
        rt_config ck = *cfg;
        ck.device = devices[k];
        st = m->fault == MultiState::kCreate && k == m->fault_k
                 ? fail(nullptr, RT_E_NOMEM, "rt_create: injected failure (RT_TEST_FAULT)")
                 : rt_create(&ck, &m->peers[k]);
        if (st) {
            r->err = "rt_create_multi: " + g_last_error + peer_name(*m, k);
            return bail(st);
        }
    }
    // RT_TEST_FAULT=queue:k: peer k's plain frames report themselves failed
    // (rt_create honoured a "queue:0" on every peer: only peer k keeps it)
    for (uint32_t k = 0; k < n_devices; ++k)
        m->peers[k]->test_fault_queue = m->fault == MultiState::kQueue && k == m->fault_k;
    for (uint32_t k = 0; k < n_devices; ++k) {
        hipError_t e = hipSetDevice(devices[k]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->cs[k], hipStreamNonBlocking);
        for (int f = 0; f < MultiState::F && e == hipSuccess; ++f) {
            e = hipEventCreateWithFlags(&m->rendered[f][k], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&m->sent[f][k], hipEventDisableTiming);
            // t_start / t_end time device k's render (rt_get_multi_timing)
            if (e == hipSuccess) e = hipEventCreate(&m->t_start[f][k]);
            if (e == hipSuccess) e = hipEventCreate(&m->t_end[f][k]);
        }
        if (e != hipSuccess)
            return bail(hip_fail(r, e, ("rt_create_multi: streams/events" + peer_name(*m, k)).c_str()));
        if (k && transport == RT_TRANSPORT_PEER && devices[k] != devices[0]) {
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devices[0], devices[k]) == hipSuccess && can) {
                (void)hipSetDevice(devices[0]);
                (void)hipDeviceEnablePeerAccess(devices[k], 0);  // already enabled is fine
                (void)hipGetLastError();
            }
        }
    }
    {
        hipError_t e = hipSetDevice(devices[0]);
        if (e == hipSuccess) e = hipStreamCreateWithFlags(&m->out, hipStreamNonBlocking);
        for (int f = 0; f < MultiState::F && e == hipSuccess; ++f) {
            e = hipEventCreateWithFlags(&m->recvd[f], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&m->unpacked[f], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreate(&m->t_unpacked[f]);
        }
        if (e == hipSuccess) e = hipEventCreateWithFlags(&m->out_ready, hipEventDisableTiming);
        if (e != hipSuccess) return bail(hip_fail(r, e, "rt_create_multi: events"));
    }
    if (transport == RT_TRANSPORT_RCCL) {
        m->comms.assign(n_devices, nullptr);
        const ncclResult_t e = m->fault == MultiState::kComm
                                   ? ncclInternalError  // RT_TEST_FAULT=comm
                                   : rccl_api().CommInitAll(m->comms.data(), static_cast<int>(n_devices), devices);
        if (e != ncclSuccess) {
            m->comms.clear();
            std::string devs;
            for (uint32_t k = 0; k < n_devices; ++k) devs += (k ? "," : "") + std::to_string(devices[k]);
            return bail(nccl_fail(r, e, ("ncclCommInitAll over devices [" + devs + "]").c_str()));
        }
    }
    // the tile plan and its slabs for the configured size, now: an allocation
    // failure surfaces here, not at the first frame (a resize re-plans)
    if ((st = multi_plan(r))) return bail(st);
    (void)hipSetDevice(devices[0]);
    *out = r;
    return RT_OK;
}

int rt_get_multi_timing(rt_renderer* r, rt_multi_timing* t) {
    if (!r || !t) return fail(r, RT_E_INVALID, "rt_get_multi_timing: null argument");
    if (!r->multi) return fail(r, RT_E_STATE, "rt_get_multi_timing: not a multi-device handle");
    MultiState& m = *r->multi;
    // from now on frames record their timing events
    const bool was_on = m.timing;
    m.timing = true;
    if (!m.frame) return fail(r, RT_E_STATE, "rt_get_multi_timing: no frame rendered yet");
    const int f = static_cast<int>((m.frame - 1) % MultiState::F);
    if (!m.timed[f])
        return fail(r, RT_E_STATE,
                    was_on ? "rt_get_multi_timing: the last frame was not timed"
                           : "rt_get_multi_timing: timing starts with the next frame (frames "
                             "record timing events once it has been asked for)");
    int st;
    if ((st = multi_wait(r))) return st;
    memset(t, 0, sizeof(*t));
    t->n_devices = static_cast<uint32_t>(m.devs.size());
    t->frame = m.frame - 1;
    for (size_t k = 0; k < m.devs.size(); ++k) {
        RT_HIP(r, hipSetDevice(m.devs[k]));
        RT_HIP(r, hipEventElapsedTime(&t->render_ms[k], m.t_start[f][k], m.t_end[f][k]));
    }
    RT_HIP(r, hipSetDevice(m.devs[0]));
    RT_HIP(r, hipEventElapsedTime(&t->deliver_ms, m.t_end[f][0], m.t_unpacked[f]));
    return RT_OK;
}

int rt_get_multi_info(const rt_renderer* r, rt_multi_info* info) {
    if (!r || !info) return RT_E_INVALID;
    memset(info, 0, sizeof(*info));
    info->tile_size = MultiState::kTs;
    if (!r->multi) {
        info->n_devices = 1;
        info->devices[0] = r->device;
        return RT_OK;
    }
    const MultiState& m = *r->multi;
    info->n_devices = static_cast<uint32_t>(m.devs.size());
    for (size_t k = 0; k < m.devs.size(); ++k) info->devices[k] = m.devs[k];
    info->transport = m.transport;
    const uint32_t ts = MultiState::kTs, n = info->n_devices;
    info->slab_tiles = (((r->W + ts - 1) / ts) * ((r->H + ts - 1) / ts) + n - 1) / n;
    info->frames_in_flight = MultiState::F;
    info->frames = m.frame;
    return RT_OK;
}

}  // extern "C"
