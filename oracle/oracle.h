/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, contraction off, IEEE f32/f64) of the reference's
 * render path and of the build-defined scene mode.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and
 * only as the checker / the timed CPU baseline — never as the product path.
 *
 * Parity pin: compat mode is pinned by the hand-derived known answers of
 * SURVEY.md 8(c) C4 (tests/golden/).  The reference itself cannot be built
 * here (needs nvcc + glm/GLFW/glad fetched from the network),
 * and it has no tests, so scene mode (which the reference does not
 * implement: Octree::traverse is a stub, include/octree.h:19-21) is pinned by
 * this file's own spec + brute-force cross-checks only.
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- compat mode (reference-exact) --------------------------------------- */
void orc_resize_intrinsic(uint32_t width, uint32_t height, float K[9]);
void orc_get_ray(const float pose[16], const float K[9], float u, float v, float dir_out[3]);
int orc_hit_root_box(const float origin[3], const float dir[3]);
void orc_render_compat(uint32_t width, uint32_t height, const float pose[16], const float K[9],
                       uint8_t* out_rgba8);
/* nvcc-style FMA contraction of getRay (contract 1 or 2; 0 = as above) */
void orc_get_ray_fma(const float pose[16], const float K[9], float u, float v, int contract,
                     float dir_out[3]);
void orc_render_compat_fma(uint32_t width, uint32_t height, const float pose[16], const float K[9],
                           int contract, uint8_t* out_rgba8);

/* ---- synthetic scene ----------------------------------------------------- */
void orc_generate_spheres(uint32_t n, uint32_t seed, float* spheres, uint32_t* albedo);
uint32_t orc_sample_hash(uint32_t seed, uint32_t pid, uint32_t s, uint32_t dim);

/* ---- octree -------------------------------------------------------------- */
typedef struct orc_scene orc_scene;
orc_scene* orc_scene_build(const float* spheres, const uint32_t* albedo, uint32_t n,
                           const float root_min[3], const float root_max[3],
                           uint32_t max_depth, uint32_t leaf_capacity);
void orc_scene_free(orc_scene* s);
/* info[0]=nodes (internal+leaf), [1]=leaves, [2]=prim refs, [3]=deepest leaf */
void orc_scene_info(const orc_scene* s, uint32_t info[4]);
/* effective root box (configured box grown to enclose every sphere) */
void orc_scene_root(const orc_scene* s, float rmin[3], float rmax[3]);
/* The tree in the product's breadth-first record layout:
 * nodes_out 2*info[0] words, prim_idx_out info[2] words.  Lets tests compare
 * a built octree with this one record for record. */
void orc_scene_export_bfs(const orc_scene* s, uint32_t* nodes_out, uint32_t* prim_idx_out);
uint32_t orc_depth_for_resolution(const float root_min[3], const float root_max[3], float res);

/* counters[0]=primary rays, [1]=shadow rays, [2]=nodes visited, [3]=prims tested */
int orc_trace(const orc_scene* s, const float o[3], const float d[3], float tmin, float tmax,
              int any_hit, float* t_out, uint32_t* idx_out, uint64_t counters[4]);
int orc_trace_brute(const orc_scene* s, const float o[3], const float d[3], float tmin,
                    float tmax, int any_hit, float* t_out, uint32_t* idx_out);

/* Scene render of the pixels whose rows satisfy (y % row_step) == row_phase and
 * x in [x0,x1), y in [y0,y1) (row_step = 1: the whole rectangle).  Outputs are
 * full-frame (W*H*4) buffers; out_f32 may be NULL.  flags: bit0 jitter,
 * bit3 no-shadows (same bits as rt.h).  n_threads <= 0: OpenMP default. */
void orc_render_scene(const orc_scene* s, uint32_t width, uint32_t height, const float pose[16],
                      const float K[9], uint32_t spp, uint32_t seed, uint32_t flags,
                      const float light_dir[3], float ambient, uint32_t x0, uint32_t y0,
                      uint32_t x1, uint32_t y1, uint32_t row_step, uint32_t row_phase,
                      uint8_t* out_rgba8, float* out_f32, uint64_t counters[4], int n_threads);

/* Progressive frame `frame` (0, 1, ...) of RT_FLAG_PROGRESSIVE: samples
 * [frame*spp, (frame+1)*spp) are added onto accum (W*H*4 running sums,
 * in/out; ignored and zero-started at frame 0); the outputs are the mean over
 * (frame+1)*spp samples.  accum == NULL is orc_render_scene. */
void orc_render_scene_frame(const orc_scene* s, uint32_t width, uint32_t height,
                            const float pose[16], const float K[9], uint32_t spp, uint32_t seed,
                            uint32_t flags, const float light_dir[3], float ambient, uint32_t x0,
                            uint32_t y0, uint32_t x1, uint32_t y1, uint32_t row_step,
                            uint32_t row_phase, uint32_t frame, float* accum, uint8_t* out_rgba8,
                            float* out_f32, uint64_t counters[4], int n_threads);

int orc_max_threads(void);

#ifdef __cplusplus
}
#endif
#endif
