/*
 * rt.h — C-ABI of the MI355X-native render path (drop-in for the reference's
 * KernelRenderer, randomwons/RayTracingStudy).
 *
 * Plain C: opaque handle, plain pointers and sizes, int status (0 = ok,
 * negative = error).  No HIP, GL or torch types appear in any signature; a HIP
 * stream is passed as `void*` (a hipStream_t), device buffers as `void*`.
 *
 * Every entry point names the reference interface it replaces (file:line is
 * relative to the reference repository root):
 *
 *   reference                                            this ABI
 *   ---------------------------------------------------  ---------------------------
 *   KernelRenderer(cudaGraphicsResource_t,w,h)            rt_create
 *     include/renderer.cuh:29, src/renderer.cu:124-141
 *   ~KernelRenderer()  include/renderer.cuh:28,           rt_destroy
 *     src/renderer.cu:189-198 (leaks device objects)
 *   setPosition(glm::mat4)  include/renderer.cuh:32,      rt_set_pose
 *     src/renderer.cu:111-113, 93-97
 *   setIntrinsic(glm::mat3) include/renderer.cuh:33,      rt_set_intrinsic
 *     src/renderer.cu:115-117, 99-103
 *   resize(int,int) include/renderer.cuh:31,              rt_resize
 *     src/renderer.cu:155-187
 *   setOctree(vec3,vec3,float) include/renderer.cuh:35    rt_set_octree
 *     (declared, never defined: src/renderer.cu:119-121)
 *   (none: Octree::traverse is a stub,                    rt_set_scene
 *     include/octree.h:19-21)
 *   render() include/renderer.cuh:30,                     rt_render
 *     src/renderer.cu:143-153 (raytracing<<<>>> :149)
 *   cudaGraphicsResourceGetMappedPointer + unmap          rt_render(dev_rgba8 = mapped ptr)
 *     src/renderer.cu:145-151
 *   (none: single device)                                 rt_render_tiles / rt_unpack_tiles
 *   (none: single device; SURVEY 8b B2 "device ids",      rt_create_multi / rt_get_multi_info /
 *     8e E1 ncclCommInitAll)                                rt_get_multi_timing
 *   (none: no error reporting, all void)                  rt_last_error
 *
 * Threading: one handle per host thread / stream; calls on one handle are not
 * re-entrant.  Ownership: the caller owns every buffer it passes in; the
 * renderer owns its internal device buffers (freed by rt_destroy).
 */
#ifndef RT_AMD_RT_H
#define RT_AMD_RT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_ABI_VERSION 4

typedef struct rt_renderer rt_renderer;

/* status codes */
enum {
    RT_OK = 0,
    RT_E_INVALID = -1,  /* bad argument */
    RT_E_HIP = -2,      /* HIP runtime error (message in rt_last_error) */
    RT_E_NOMEM = -3,    /* host or device allocation failed */
    RT_E_NOSCENE = -4,  /* RT_MODE_SCENE render without rt_set_scene */
    RT_E_STATE = -5     /* call not valid in the current state */
};

/* render modes */
enum {
    /* Byte-exact restatement of the reference kernel `raytracing`
     * (src/renderer.cu:57-82): R = Octree::traverse() = 200, root-box slab test
     * `hit_sphere` (src/renderer.cu:3-55), miss colour from the direction. */
    RT_MODE_COMPAT = 0,
    /* Build-defined octree scene: nearest sphere hit, Lambert + one shadow ray,
     * `spp` jittered samples averaged (DESIGN.md "Scene mode"). */
    RT_MODE_SCENE = 1
};

/* rt_config.flags */
enum {
    RT_FLAG_JITTER = 1u << 0,      /* per-sample sub-pixel jitter (default: on iff spp > 1) */
    RT_FLAG_NO_JITTER = 1u << 1,   /* force jitter off */
    RT_FLAG_RADIANCE = 1u << 2,    /* also keep the float4 mean radiance buffer */
    RT_FLAG_NO_SHADOWS = 1u << 3,  /* skip shadow rays (Lambert without visibility) */
    RT_FLAG_HOST_BUILD = 1u << 4,  /* build the octree on the host (default: on the GPU);
                                      both builders produce the identical tree */
    RT_FLAG_PROGRESSIVE = 1u << 5, /* scene mode: accumulate samples across frames while the
                                      camera, size, scene and tile list stay unchanged; every
                                      frame adds spp samples */
    RT_FLAG_COMPAT_FMA = 1u << 6,  /* compat mode: evaluate getRay (include/camera.h:31-34) with
                                      ONE CANDIDATE of the FMA contraction nvcc's default
                                      -fmad=true may apply to the reference binary; which order
                                      that binary really uses is unpinned here (no nvcc).  Off
                                      (default) = the reference's SOURCE semantics, in source
                                      order */
    /* bits 8..9, test-only: what fills the padding after the last leaf list
     * (DESIGN.md §4): 0 zero spheres (default), 1 NaN spheres, 2 spheres
     * covering the root box.  Images and counters are the same for all three. */
    RT_FLAG_PAD_FILL_SHIFT = 8,
    /* Test-only: rt_create / rt_create_multi honour the RT_TEST_* environment
     * variables (RT_TEST_FAULT fault injection, RT_TEST_CLAIM_DELAY); without
     * this flag they are ignored (a set one is named on stderr once). */
    RT_FLAG_TEST_HOOKS = 1u << 10,
    /* Test-only: before every frame, fill the frame's outputs with a sentinel
     * (RGBA8 bytes 0xAB, frame or packed tiles; radiance and a first
     * progressive frame's sums all-ones bits, a NaN), so a pixel the kernels
     * do not write shows in any readback.  Costs a memset per frame. */
    RT_FLAG_TEST_POISON = 1u << 11,
    /* bits 16..19: scene-kernel variant for A/B runs (0 = default: 13, the
     * per-wave queue, for spp >= 8, else 7; others in DESIGN.md 5.1); images
     * and counters are identical across variants (packets: images only) */
    RT_FLAG_VARIANT_SHIFT = 16,
    /* bits 20..27: A/B toggles that switch single optimisations off or on (0 = defaults) */
    RT_FLAG_OPT_SHIFT = 20,
    /* bits 28..31: depth of the octree's cell table (DESIGN.md 5.1 "Cell table"):
     * 0 = chosen from the tree (default), 1..7 = that depth (clamped to the
     * tree), 15 = no table.  Images and counters are the same either way. */
    RT_FLAG_CELL_TABLE_SHIFT = 28
};

typedef struct rt_config {
    uint32_t width;        /* framebuffer width  (reference: KernelRenderer::width)  */
    uint32_t height;       /* framebuffer height (reference: KernelRenderer::height) */
    uint32_t spp;          /* samples per pixel (scene mode; compat ignores it: 1)   */
    uint32_t seed;         /* sampling seed (scene mode)                              */
    int32_t device;        /* HIP device ordinal, -1 = the calling thread's current   */
    uint32_t mode;         /* RT_MODE_*                                               */
    uint32_t flags;        /* RT_FLAG_*                                               */
    float light_dir[3];    /* direction the directional light TRAVELS (need not be unit) */
    float ambient;         /* ambient term of the Lambert shade, [0,1]                */
} rt_config;

/* Octree parameters.  Defaults (rt_octree_params_default) are the reference's
 * hard-coded root, src/renderer.cu:134-136: min (0,0,0), max (1.28)^3,
 * resolution 0.01 => max_depth = ceil(log2(1.28/0.01)) = 7. */
typedef struct rt_octree_params {
    float min[3];
    float max[3];
    float resolution;       /* smallest cell edge; used when max_depth == 0            */
    uint32_t max_depth;     /* 0 = derive from resolution; else 1..16                  */
    uint32_t leaf_capacity; /* split a cell while it holds more spheres than this (8) */
} rt_octree_params;

typedef struct rt_stats {
    uint64_t primary_rays;   /* camera rays cast (pixels * spp)                         */
    uint64_t shadow_rays;    /* shadow rays cast (lit-facing primary hits)              */
    uint64_t nodes_visited;  /* octree node records read (DESIGN.md counter definition) */
    uint64_t prims_tested;   /* ray-sphere tests                                        */
    float ms;                /* device time of the render launch(es), hipEvent          */
    uint32_t samples_per_pixel; /* samples in the image: spp, or the accumulated total  */
} rt_stats;

typedef struct rt_scene_info {
    uint32_t n_spheres;
    uint32_t n_nodes;        /* node records (internal + leaf)                          */
    uint32_t n_leaves;
    uint32_t n_prim_refs;    /* total length of all leaf sphere lists                   */
    uint32_t max_depth;      /* depth limit the tree was built with                     */
    uint32_t depth_reached;  /* deepest leaf                                            */
    uint32_t node_bytes;     /* sizeof one node record                                  */
    uint32_t prim_bytes;     /* bytes read per sphere test                              */
    float root_min[3];       /* effective root box: the configured box grown to          */
    float root_max[3];       /*   enclose every sphere (equal to it when none protrudes)  */
    double build_ms;         /* time to a device-resident octree (GPU build, or host
                                build + upload with RT_FLAG_HOST_BUILD)                 */
    double upload_ms;        /* time to place the sphere list in device memory          */
    uint32_t builder;        /* RT_BUILDER_* that built the current tree                */
    uint32_t cell_table_depth; /* K of the depth-K cell table the walk uses, 0 = none   */
} rt_scene_info;

enum { RT_BUILDER_DEVICE = 0, RT_BUILDER_HOST = 1 };

/* ---- version / discovery -------------------------------------------------- */
int rt_abi_version(void);
/* Number of visible HIP devices (0 when no GPU); never initialises a context. */
int rt_device_count(void);

/* ---- lifecycle ------------------------------------------------------------ */
void rt_config_default(rt_config* cfg);
void rt_octree_params_default(rt_octree_params* p);
/* Reference ctor: camera K0 = mat3(1000,0,640, 0,1000,340, 0,0,1) and identity
 * pose (src/renderer.cu:84-91), octree root from rt_octree_params_default. */
int rt_create(const rt_config* cfg, rt_renderer** out);
int rt_destroy(rt_renderer* r);

/* ---- camera --------------------------------------------------------------- */
/* pose: glm-style column-major mat4; origin = pose[3].xyz, rot = mat3(pose)
 * (include/camera.h:43-46).  K: column-major mat3, K[0][0]=fx, K[1][1]=fy,
 * K[0][2]=cx, K[1][2]=cy, i.e. K[c*3+r] (include/camera.h:24-26). */
int rt_set_pose(rt_renderer* r, const float pose[16]);
int rt_set_intrinsic(rt_renderer* r, const float K[9]);
int rt_get_camera(const rt_renderer* r, float pose_out[16], float K_out[9]);
/* Reference resize (src/renderer.cu:155-170): f = W/(2 tan(radians(80)/2)),
 * cx = W/2, cy = H/2 (integer division); reallocates internal buffers. */
int rt_resize(rt_renderer* r, uint32_t width, uint32_t height);
/* The intrinsic rt_resize would set, without a renderer (for hosts/tests). */
void rt_resize_intrinsic(uint32_t width, uint32_t height, float K_out[9]);

/* ---- scene ---------------------------------------------------------------- */
/* spheres: 4*n floats (cx, cy, cz, radius); albedo: n packed RGBA8 (R in the low
 * byte) or NULL (every sphere 0.8 grey).  oct == NULL keeps the current octree
 * parameters.  Builds the octree on the host and uploads it. */
int rt_set_scene(rt_renderer* r, const float* spheres, const uint32_t* albedo, uint32_t n,
                 const rt_octree_params* oct);
/* Same, from a sphere list already in device memory (e.g. produced by a
 * simulation on the GPU): dev_spheres = 4*n floats, dev_albedo = n RGBA8 words
 * or NULL.  `stream` (or NULL) is the stream that produced them; the call waits
 * for it.  The octree is built on the GPU unless RT_FLAG_HOST_BUILD is set.
 * Invalid spheres (r <= 0, non-finite values) are found on the device and the
 * call fails with RT_E_INVALID, keeping the previous scene.  SURVEY.md 8f F1;
 * the reference's intended entry is setOctree (include/renderer.cuh:35). */
int rt_set_scene_device(rt_renderer* r, const void* dev_spheres, const void* dev_albedo,
                        uint32_t n, const rt_octree_params* oct, void* stream);
/* Mirror of the reference's setOctree(min, max, resolution): rebuilds the
 * octree of the current spheres with a new root box / resolution. */
int rt_set_octree(rt_renderer* r, const float min[3], const float max[3], float resolution);
int rt_get_scene_info(const rt_renderer* r, rt_scene_info* info);
/* Copy the current octree to host memory (sizes from rt_get_scene_info):
 * nodes_out 2*n_nodes words (uint2 records), prim_sp_out
 * 4*n_prim_refs floats, prim_idx_out n_prim_refs words; any may be NULL. */
int rt_export_octree(rt_renderer* r, uint32_t* nodes_out, float* prim_sp_out,
                     uint32_t* prim_idx_out);
/* Synthetic scene generator: splitmix64 -> PCG32 from `seed`;
 * centres U[0,1.28)^3, radius 0.02*(1000/n)^(1/3)*U[0.5,1), albedo U[0.2,1). */
int rt_generate_spheres(uint32_t n, uint32_t seed, float* spheres_out, uint32_t* albedo_out);

/* ---- scene files (binary sphere list) --------------------- */
/* Write n spheres (4 floats each) and, if albedo != NULL, their RGBA8 words. */
int rt_save_spheres(const char* path, const float* spheres, const uint32_t* albedo, uint32_t n);
/* Read a sphere file.  *n_out = its sphere count; with spheres_out == NULL only
 * the count is returned.  Otherwise capacity must be >= the count; albedo_out
 * (may be NULL) gets the file's colours or 0.8 grey when it has none. */
int rt_load_spheres(const char* path, float* spheres_out, uint32_t* albedo_out,
                    uint32_t capacity, uint32_t* n_out);

/* ---- render --------------------------------------------------------------- */
/* Render one frame.  dev_rgba8: W*H*4 device bytes (e.g. the pointer a GL PBO
 * maps to), or NULL to render into the renderer's internal framebuffer.
 * stream: a hipStream_t or NULL (the renderer's own stream).  Asynchronous
 * unless stats != NULL (then it waits for the frame and fills the counters).
 * An earlier frame that the kernel found incomplete (its work queue's bounded
 * wait gave up: a broken invariant, never a normal frame) is reported by the
 * first call that sees it, without a sync: this rt_render returns RT_E_HIP
 * naming that frame and renders nothing, so a caller that never reads back
 * (the reference's Displayer, src/window/displayer.cpp:51-53) still learns
 * of it; rt_synchronize, rt_readback and stats frames report it too. */
int rt_render(rt_renderer* r, void* dev_rgba8, void* stream, rt_stats* stats);
/* GL interop.  The Displayer registers its PBO with
 * hipGraphicsGLRegisterBuffer (where it called cudaGraphicsGLRegisterBuffer,
 * src/window/displayer.cpp:13-17, and again after a resize, :61-70) and binds
 * the resource here.  Then rt_render(r, NULL, stream, stats) maps it, renders
 * into the mapped pointer and unmaps it: the reference's render()
 * (src/renderer.cu:145-151).  NULL unbinds (render into the internal
 * framebuffer).  The resource stays owned by the caller. */
int rt_bind_graphics_resource(rt_renderer* r, void* hip_graphics_resource);
/* The same per-frame map -> render -> unmap cycle for a display buffer the
 * caller's toolkit owns (a GL PBO, Vulkan/EGL external memory, a swap-chain
 * image): rt_render(r, NULL, stream, stats) calls ops->map(user, stream, &ptr,
 * &bytes) on the frame's stream, fails with RT_E_INVALID (after unmapping) if
 * bytes < W*H*4, renders into ptr and calls ops->unmap(user, stream) after
 * the launch, also when the render itself failed.  map/unmap return 0 on
 * success; a failing map must leave the buffer unmapped, and rt_render then
 * returns RT_E_HIP.  rt_bind_graphics_resource(r, res) is this call with the
 * built-in HIP graphics-interop ops (hipGraphicsMapResources, ...GetMappedPointer,
 * hipGraphicsUnmapResources) and user = res.  ops == NULL unbinds; *ops is
 * copied.  SURVEY.md 8f F2; replaces src/renderer.cu:145-151. */
typedef struct rt_display_ops {
    int (*map)(void* user, void* stream, void** dev_ptr, size_t* bytes);
    int (*unmap)(void* user, void* stream);
} rt_display_ops;
int rt_bind_display(rt_renderer* r, const rt_display_ops* ops, void* user);
/* Render only the listed image tiles (tile_size x tile_size, row-major tile
 * ids over ceil(W/ts) x ceil(H/ts)) into a packed device buffer of
 * n_tiles*ts*ts*4 bytes: tile k's pixel (lx,ly) at byte 4*(k*ts*ts + ly*ts + lx);
 * pixels outside the image are written as 0.  Used to shard a frame over GPUs. */
int rt_render_tiles(rt_renderer* r, const uint32_t* tile_ids, uint32_t n_tiles,
                    uint32_t tile_size, void* dev_packed_rgba8, void* stream, rt_stats* stats);
/* Scatter a packed tile buffer (layout above) into a W*H*4 device image.
 * A tile id of RT_TILE_SKIP marks a padding slot that is not copied, so the
 * equal-size slabs of all ranks, gathered into one buffer, unpack in one call. */
#define RT_TILE_SKIP 0xFFFFFFFFu
int rt_unpack_tiles(rt_renderer* r, const void* dev_packed_rgba8, const uint32_t* tile_ids,
                    uint32_t n_tiles, uint32_t tile_size, void* dev_rgba8, void* stream);
/* RT_FLAG_PROGRESSIVE: start the next frame from zero samples (any change of
 * pose, intrinsic, size, scene or tile list does this by itself; setting the
 * same pose again, as the reference's Displayer does every frame, does not). */
int rt_reset_accumulation(rt_renderer* r);
/* Wait for all work queued by this renderer, on its own stream or on the
 * caller streams passed to rt_render / rt_render_tiles / rt_unpack_tiles.
 * (Work queued on a stream other than the previous call's is ordered after
 * that previous call's work: the renderer's counters and buffers are shared.) */
int rt_synchronize(rt_renderer* r);
/* Copy the internal framebuffer (and the float4 radiance buffer when
 * RT_FLAG_RADIANCE is set) to host memory; either pointer may be NULL.
 * Waits for the renderer's queued work first, whatever stream it is on. */
int rt_readback(rt_renderer* r, uint8_t* host_rgba8, float* host_rgba32f);
/* Device pointer of the internal framebuffer (W*H*4 bytes). */
void* rt_framebuffer(rt_renderer* r);
/* The renderer's own stream (a hipStream_t made with the handle), the one a
 * NULL stream argument means (a multi-device handle: its output stream on
 * devices[0]).  Extension: the reference launches on the legacy
 * default stream (src/renderer.cu:149).  Renderers made one after another get
 * streams on different hardware queues, so frames in flight on them overlap. */
void* rt_stream(rt_renderer* r);

/* ---- one process, several devices (SURVEY 8b B2 "device ids", 8e E1) ------ */
/* A renderer handle that renders every frame across n_devices GPUs of this
 * process: one renderer per device (same config, same scene: replicated), the
 * frame's 64x64 tiles dealt round-robin (tile t to device t mod n), each
 * device rendering its tiles into a packed slab on its own stream, the slabs
 * moved to devices[0] (RCCL: one ncclCommInitAll communicator over the
 * devices, grouped ncclSend / ncclRecv on per-device comm streams; or peer
 * copies) and unpacked there by ONE launch into the frame.  Two frames are in
 * flight: frame k+1's tiles render while frame k's slabs travel and unpack.
 * Every other entry point works on the handle as on a single-device one
 * (rt_set_pose / rt_set_intrinsic / rt_resize / rt_set_scene / rt_set_octree
 * / rt_reset_accumulation apply to every device; rt_set_scene_device takes a
 * sphere list on devices[0] and broadcasts it (ncclBroadcast); rt_render,
 * rt_bind_graphics_resource / rt_bind_display, rt_readback, rt_framebuffer,
 * rt_stream, rt_get_scene_info and rt_export_octree are devices[0]'s), except
 * rt_render_tiles / rt_unpack_tiles (RT_E_STATE: the handle renders whole
 * frames).  rt_render with stats renders the devices one after another and
 * sums their counters (ms = host wall time of the frame).  The reference's
 * Displayer (src/window/displayer.cpp:28) constructs the renderer this way
 * and calls render() unchanged.
 * devices: HIP ordinals; a repeated ordinal (e.g. {0,0,0,0}) rehearses the
 * n-way plan on fewer GPUs (peer-copy transport only: RCCL refuses a device
 * twice in one communicator).  cfg->device is ignored. */
enum {
    RT_TRANSPORT_AUTO = 0, /* RCCL when the devices are distinct and librccl loads, else peer */
    RT_TRANSPORT_RCCL = 1, /* grouped ncclSend / ncclRecv over one ncclCommInitAll communicator */
    RT_TRANSPORT_PEER = 2  /* hipMemcpyPeerAsync on the comm streams (xGMI, or a local copy) */
};
#define RT_MAX_DEVICES 16
typedef struct rt_multi_info {
    uint32_t n_devices;              /* 1 for a single-device handle                     */
    int32_t devices[RT_MAX_DEVICES]; /* HIP ordinals, devices[0] holds the frame           */
    uint32_t transport;              /* RT_TRANSPORT_RCCL or RT_TRANSPORT_PEER (0: single)  */
    uint32_t tile_size;              /* 64                                                */
    uint32_t slab_tiles;             /* tiles per device slab (ceil(tiles / n_devices))   */
    uint32_t frames_in_flight;       /* 2                                                 */
    uint64_t frames;                 /* frames rendered by the handle                     */
} rt_multi_info;
/* Refuses RT_FLAG_RADIANCE (RT_E_INVALID: the slabs carry RGBA8 only).  The
 * tile plan and its slabs are allocated here for cfg's size (again at the
 * first frame after a resize), so an allocation failure is reported by this
 * call.  A NULL stream argument (rt_render, rt_stream) means the handle's
 * output stream on devices[0], which is not devices[0]'s render stream, so
 * frame j+1's tiles there do not wait for frame j's unpack.  A failure on one
 * device names it in rt_last_error: "(device <ordinal>, peer <k>)".
 * Test-only (with RT_FLAG_TEST_HOOKS): the environment variable RT_TEST_FAULT,
 * read here, injects one failure: "create:k" (peer k's renderer), "comm"
 * (ncclCommInitAll), "slab:k" (peer k's slab allocation) or "queue:k" (peer
 * k's plain frames report themselves incomplete, which the next rt_render,
 * rt_synchronize or rt_readback returns as RT_E_HIP naming the peer); rt_create
 * honours "queue:0" for a single-device renderer. */
int rt_create_multi(const rt_config* cfg, const int32_t* devices, uint32_t n_devices,
                    uint32_t transport, rt_renderer** out);
int rt_get_multi_info(const rt_renderer* r, rt_multi_info* info);
/* Device times of the handle's last frame (waits for the handle's queued
 * work): render_ms[k] = device k rendering its tiles into its slab (HIP
 * events on its render stream); deliver_ms = on devices[0], from the end of
 * its own tiles to the frame unpacked (the other slabs' arrival over the
 * transport, then the one unpack).  Frames record timing events only after
 * the handle's first rt_get_multi_timing call (the frame path's own
 * synchronisation events stay timing-free), so that first call, like one for
 * a single-device handle or an untimed last frame, returns RT_E_STATE. */
typedef struct rt_multi_timing {
    uint32_t n_devices;
    uint64_t frame;                   /* 0-based index of the frame timed           */
    float render_ms[RT_MAX_DEVICES];
    float deliver_ms;
} rt_multi_timing;
int rt_get_multi_timing(rt_renderer* r, rt_multi_timing* t);

/* ---- errors --------------------------------------------------------------- */
/* Last error message for this handle (r may be NULL: last global error). */
const char* rt_last_error(const rt_renderer* r);

#ifdef __cplusplus
}
#endif

#endif /* RT_AMD_RT_H */
