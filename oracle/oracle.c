/*
 * oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Plain-C CPU restatement of:
 *   - the reference kernel `raytracing` (src/renderer.cu:57-82) with
 *     Camera::getRay (include/camera.h:24-41), hit_sphere
 *     (src/renderer.cu:3-55) and the resize intrinsic (src/renderer.cu:155-170);
 *   - the build-defined scene mode (DESIGN.md "Scene mode"): sphere generator,
 *     octree builder, grid-space octree walk, Lambert + shadow ray, spp mean.
 *
 * Compiled with -O2 -ffp-contract=off (no FMA contraction, SSE f32/f64, no
 * excess precision): every expression below is evaluated exactly in source
 * order, which is the semantics the HIP kernels reproduce bit for bit.
 * Never compile with -ffast-math.
 */
#include "oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ========================================================================== */
/* compat mode                                                                */
/* ========================================================================== */

/* src/renderer.cu:162-170: intrinsic = mat3(1); f = width/(2*tan(radians(80.f)/2))
 * (glm::radians multiplies by the float constant, glm::tan = tanf, the
 * arithmetic is float; the double f is then stored back into a float);
 * intrinsic[0][2] = width/2, intrinsic[1][2] = height/2 in integer arithmetic. */
void orc_resize_intrinsic(uint32_t width, uint32_t height, float K[9]) {
    const float rad = 80.f * 0.01745329251994329576923690768489f;
    const float f = (float)width / (2.0f * tanf(rad / 2.0f));
    for (int i = 0; i < 9; ++i) K[i] = 0.0f;
    K[0] = f;                      /* [0][0] */
    K[4] = f;                      /* [1][1] */
    K[8] = 1.0f;                   /* [2][2] */
    K[2] = (float)(width / 2u);    /* [0][2] */
    K[5] = (float)(height / 2u);   /* [1][2] */
}

/* include/camera.h:24-41 (u, v already floats; the reference converts its
 * uint32 pixel index to float in `u - intrinsic[0][2]`).  glm storage is
 * column-major: rot[c][r] = pose[c*4+r], K[c][r] = K[c*3+r]. */
void orc_get_ray(const float pose[16], const float K[9], float u, float v, float dir_out[3]) {
    const float dx = (u - K[2]) / K[0];
    const float dy = (v - K[5]) / K[4];
    const float dz = 1.0f;
    float wdx = pose[0] * dx + pose[4] * dy + pose[8] * dz;
    float wdy = pose[1] * dx + pose[5] * dy + pose[9] * dz;
    float wdz = pose[2] * dx + pose[6] * dy + pose[10] * dz;
    const float len = sqrtf(wdx * wdx + wdy * wdy + wdz * wdz);
    wdx /= len;
    wdy /= len;
    wdz /= len;
    dir_out[0] = wdx;
    dir_out[1] = wdy;
    dir_out[2] = wdz;
}

/* include/camera.h:31-34 as nvcc would compile it with its default
 * -fmad=true (the reference's CMakeLists.txt:2,16 sets no -fmad=false): the
 * `a*b + c*d + e*1` sums contract into FMAs.  `rot[2][i] * dz` with the
 * constant dz = 1 folds to rot[2][i] (x * 1.0 == x), and LLVM's DAG combiner
 * (NVVM) fuses an fadd of two products through its FIRST operand:
 *   contract = 1: wd = fmaf(rot[0][i], dx, rot[1][i] * dy) + rot[2][i]
 *                 len = sqrtf(fmaf(wdz, wdz, fmaf(wdx, wdx, wdy * wdy)))
 *   contract = 2: the other operand order (a bound on the ambiguity)
 *                 wd = fmaf(rot[1][i], dy, rot[0][i] * dx) + rot[2][i]
 *                 len = sqrtf(fmaf(wdz, wdz, fmaf(wdy, wdy, wdx * wdx)))
 * contract = 0 is orc_get_ray (source order, no contraction).  Used to
 * bound how far the reference BINARY can differ from its source semantics
 * (tools/compat_fma_gap.py). */
void orc_get_ray_fma(const float pose[16], const float K[9], float u, float v, int contract,
                     float dir_out[3]) {
    if (contract == 0) {
        orc_get_ray(pose, K, u, v, dir_out);
        return;
    }
    const float dx = (u - K[2]) / K[0];
    const float dy = (v - K[5]) / K[4];
    float w[3];
    for (int i = 0; i < 3; ++i)
        w[i] = contract == 1 ? fmaf(pose[i], dx, pose[4 + i] * dy) + pose[8 + i]
                             : fmaf(pose[4 + i], dy, pose[i] * dx) + pose[8 + i];
    const float l2 = contract == 1 ? fmaf(w[2], w[2], fmaf(w[0], w[0], w[1] * w[1]))
                                   : fmaf(w[2], w[2], fmaf(w[1], w[1], w[0] * w[0]));
    const float len = sqrtf(l2);
    for (int i = 0; i < 3; ++i) dir_out[i] = w[i] / len;
}

/* src/renderer.cu:3-55.  Box min (0,0,0), max glm::vec3(1.28) (doubles -> f32),
 * centre glm::vec3(0.64) passed from :70.  Mixed f32/f64 exactly as written:
 * the mirrored origin is a float expression widened to double, the inverse is
 * a float division widened to double, the slab products are double and
 * rounded to float; fmaxf/fminf drop NaN (0*inf). No t >= 0 test. */
int orc_hit_root_box(const float origin[3], const float dir[3]) {
    const float bmin = 0.0f;
    const float bmax = (float)1.28;
    const float center = (float)0.64;
    double ro[3], inv[3];
    for (int i = 0; i < 3; ++i) {
        if (dir[i] < 0.0f) {
            ro[i] = (double)(center * 2.0f - origin[i]);
            inv[i] = (double)(-(1.0f / dir[i]));
        } else {
            ro[i] = (double)origin[i];
            inv[i] = (double)(1.0f / dir[i]);
        }
    }
    const float tx0 = (float)(((double)bmin - ro[0]) * inv[0]);
    const float tx1 = (float)(((double)bmax - ro[0]) * inv[0]);
    const float ty0 = (float)(((double)bmin - ro[1]) * inv[1]);
    const float ty1 = (float)(((double)bmax - ro[1]) * inv[1]);
    const float tz0 = (float)(((double)bmin - ro[2]) * inv[2]);
    const float tz1 = (float)(((double)bmax - ro[2]) * inv[2]);
    return fmaxf(fmaxf(tx0, ty0), tz0) < fminf(fminf(tx1, ty1), tz1);
}

/* __saturatef: clamp to [0,1], NaN -> 0 */
static inline float sat(float x) { return x > 0.0f ? (x < 1.0f ? x : 1.0f) : 0.0f; }

/* src/renderer.cu:57-82.  Row-major uchar4, pid = y*W + x.  `contract`
 * selects orc_get_ray_fma's evaluation of getRay (0 = source order). */
void orc_render_compat_fma(uint32_t width, uint32_t height, const float pose[16], const float K[9],
                           int contract, uint8_t* out) {
    const float origin[3] = {pose[12], pose[13], pose[14]};
    for (uint32_t y = 0; y < height; ++y) {
        for (uint32_t x = 0; x < width; ++x) {
            uint8_t* px = out + 4u * ((size_t)y * width + x);
            float dir[3];
            orc_get_ray_fma(pose, K, (float)x, (float)y, contract, dir);
            if (orc_hit_root_box(origin, dir)) {
                px[0] = px[1] = px[2] = px[3] = 255;
                continue;
            }
            px[0] = (uint8_t)200.0; /* (unsigned char)Octree::traverse() */
            px[1] = (uint8_t)(sat(dir[1]) * 255.0f);
            px[2] = (uint8_t)(sat(dir[2]) * 255.0f);
            px[3] = 255;
        }
    }
}

void orc_render_compat(uint32_t width, uint32_t height, const float pose[16], const float K[9],
                       uint8_t* out) {
    orc_render_compat_fma(width, height, pose, K, 0, out);
}

/* ========================================================================== */
/* synthetic scene                                          */
/* ========================================================================== */

static uint64_t splitmix64(uint64_t* x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef struct { uint64_t state, inc; } pcg32_t;

static uint32_t pcg32_next(pcg32_t* g) {
    const uint64_t old = g->state;
    g->state = old * 6364136223846793005ull + g->inc;
    const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
    const uint32_t rot = (uint32_t)(old >> 59u);
    return (xs >> rot) | (xs << ((-rot) & 31u));
}

static float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

void orc_generate_spheres(uint32_t n, uint32_t seed, float* sp, uint32_t* albedo) {
    uint64_t sm = (uint64_t)seed;
    pcg32_t g;
    g.state = splitmix64(&sm);
    g.inc = splitmix64(&sm) | 1ull;
    const float rscale = n ? (float)(0.02 * cbrt(1000.0 / (double)n)) : 0.0f;
    for (uint32_t i = 0; i < n; ++i) {
        const float cx = u01(pcg32_next(&g)) * 1.28f;
        const float cy = u01(pcg32_next(&g)) * 1.28f;
        const float cz = u01(pcg32_next(&g)) * 1.28f;
        const float ru = u01(pcg32_next(&g));
        sp[4 * i + 0] = cx;
        sp[4 * i + 1] = cy;
        sp[4 * i + 2] = cz;
        sp[4 * i + 3] = rscale * (0.5f + 0.5f * ru);
        uint32_t a = 0xFF000000u;
        for (int c = 0; c < 3; ++c) {
            const float v = 0.2f + 0.8f * u01(pcg32_next(&g));
            a |= ((uint32_t)(v * 255.0f) & 0xFFu) << (8 * c);
        }
        if (albedo) albedo[i] = a;
    }
}

static inline uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

uint32_t orc_sample_hash(uint32_t seed, uint32_t pid, uint32_t s, uint32_t dim) {
    return mix32(mix32(mix32(seed ^ 0x9E3779B9u) ^ pid) ^ ((s << 1) | dim));
}

/* ========================================================================== */
/* octree                                                                     */
/* ========================================================================== */

typedef struct {
    int32_t child[8]; /* real child index (bit0 x, bit1 y, bit2 z) -> node, -1 empty */
    int32_t leaf;
    uint32_t off, cnt; /* leaf: range in prim list */
} onode;

struct orc_scene {
    const float* spheres; /* borrowed copy (owned below) */
    float* sp;
    uint32_t* albedo;
    uint32_t n;
    float rmin[3], rmax[3];
    uint32_t max_depth, leaf_cap;
    onode* nodes;
    uint32_t n_nodes, cap_nodes;
    uint32_t* prims;
    uint32_t n_prims, cap_prims;
    uint32_t n_leaves, depth_reached;
    /* traversal constants */
    float scale[3];
    float G;
};

/* The oracle is test infrastructure: a scene whose tree outgrows 32-bit
 * counts or host memory stops the process with a message instead of
 * corrupting memory (the product's builders report such scenes as errors). */
static void* grow(void* p, uint32_t* cap, uint32_t first, size_t elem, const char* what) {
    const uint64_t next = *cap ? 2ull * *cap : first;
    void* q = next < (1ull << 31) ? realloc(p, elem * (size_t)next) : NULL;
    if (!q) {
        fprintf(stderr, "oracle: octree %s exceed %llu entries or host memory\n", what,
                (unsigned long long)next);
        abort();
    }
    *cap = (uint32_t)next;
    return q;
}

static uint32_t new_node(orc_scene* s) {
    if (s->n_nodes == s->cap_nodes)
        s->nodes = (onode*)grow(s->nodes, &s->cap_nodes, 1024, sizeof(onode), "nodes");
    onode* nd = &s->nodes[s->n_nodes];
    for (int i = 0; i < 8; ++i) nd->child[i] = -1;
    nd->leaf = 0;
    nd->off = nd->cnt = 0;
    return s->n_nodes++;
}

static void push_prim(orc_scene* s, uint32_t idx) {
    if (s->n_prims == s->cap_prims)
        s->prims = (uint32_t*)grow(s->prims, &s->cap_prims, 4096, sizeof(uint32_t), "references");
    s->prims[s->n_prims++] = idx;
}

/* Conservative sphere/cell overlap in double: squared distance from the centre
 * to the closed cell box <= (r + margin)^2, margin = 1e-6 * largest extent. */
static int overlaps(const float* sp, const double lo[3], const double hi[3], double margin) {
    double d2 = 0.0;
    for (int i = 0; i < 3; ++i) {
        const double c = (double)sp[i];
        if (c < lo[i]) {
            const double e = lo[i] - c;
            d2 += e * e;
        } else if (c > hi[i]) {
            const double e = c - hi[i];
            d2 += e * e;
        }
    }
    const double r = (double)sp[3] + margin;
    return d2 <= r * r;
}

static void cell_bounds(const orc_scene* s, uint32_t depth, const uint32_t c[3], double lo[3],
                        double hi[3]) {
    const double cells = (double)(1u << depth);
    for (int i = 0; i < 3; ++i) {
        const double ext = (double)s->rmax[i] - (double)s->rmin[i];
        lo[i] = (double)s->rmin[i] + ext * ((double)c[i] / cells);
        hi[i] = (double)s->rmin[i] + ext * ((double)(c[i] + 1u) / cells);
    }
}

static double margin_of(const orc_scene* s) {
    double m = 0.0;
    for (int i = 0; i < 3; ++i) {
        const double e = (double)s->rmax[i] - (double)s->rmin[i];
        if (e > m) m = e;
    }
    return 1e-6 * m;
}

/* Recursive build: split while count > leaf_cap and depth < max_depth; a
 * child is kept only when some sphere overlaps it; leaf lists ascending. */
static void build_rec(orc_scene* s, uint32_t node, uint32_t depth, const uint32_t c[3],
                      const uint32_t* list, uint32_t cnt) {
    if (cnt <= s->leaf_cap || depth >= s->max_depth) {
        s->nodes[node].leaf = 1;
        s->nodes[node].off = s->n_prims;
        s->nodes[node].cnt = cnt;
        for (uint32_t i = 0; i < cnt; ++i) push_prim(s, list[i]);
        s->n_leaves++;
        if (depth > s->depth_reached) s->depth_reached = depth;
        return;
    }
    const double margin = margin_of(s);
    uint32_t* sub = (uint32_t*)malloc(sizeof(uint32_t) * (cnt ? cnt : 1));
    for (uint32_t ch = 0; ch < 8; ++ch) {
        const uint32_t cc[3] = {2 * c[0] + (ch & 1u), 2 * c[1] + ((ch >> 1) & 1u),
                                2 * c[2] + ((ch >> 2) & 1u)};
        double lo[3], hi[3];
        cell_bounds(s, depth + 1, cc, lo, hi);
        uint32_t m = 0;
        for (uint32_t i = 0; i < cnt; ++i)
            if (overlaps(s->sp + 4u * list[i], lo, hi, margin)) sub[m++] = list[i];
        if (!m) continue;
        const uint32_t k = new_node(s);
        s->nodes[node].child[ch] = (int32_t)k;
        build_rec(s, k, depth + 1, cc, sub, m);
    }
    free(sub);
}

uint32_t orc_depth_for_resolution(const float rmin[3], const float rmax[3], float res) {
    float ext = 0.0f;
    for (int i = 0; i < 3; ++i)
        if (rmax[i] - rmin[i] > ext) ext = rmax[i] - rmin[i];
    if (!(res > 0.0f)) return 7;
    uint32_t d = 0;
    while (d < 16 && (double)ext / (double)(1u << d) > (double)res * (1.0 + 1e-6)) ++d;
    return d;
}

orc_scene* orc_scene_build(const float* spheres, const uint32_t* albedo, uint32_t n,
                           const float root_min[3], const float root_max[3], uint32_t max_depth,
                           uint32_t leaf_capacity) {
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    s->n = n;
    s->sp = (float*)malloc(sizeof(float) * 4u * (n ? n : 1));
    memcpy(s->sp, spheres, sizeof(float) * 4u * n);
    s->spheres = s->sp;
    s->albedo = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    for (uint32_t i = 0; i < n; ++i) s->albedo[i] = albedo ? albedo[i] : 0xFFCCCCCCu;
    /* Effective root: the configured box, grown (only where needed, by a
     * margin) to enclose every sphere's AABB, so protruding spheres stay
     * reachable by the walk. */
    double um = 0.0;
    for (int i = 0; i < 3; ++i) {
        const double e = (double)root_max[i] - (double)root_min[i];
        if (e > um) um = e;
    }
    for (int i = 0; i < 3; ++i) {
        double lo = (double)root_min[i], hi = (double)root_max[i];
        for (uint32_t k = 0; k < n; ++k) {
            const double c = (double)spheres[4 * k + i], r = (double)spheres[4 * k + 3];
            if (c - r < lo) lo = c - r;
            if (c + r > hi) hi = c + r;
        }
        s->rmin[i] = lo < (double)root_min[i] ? (float)(lo - 1e-6 * um) : root_min[i];
        s->rmax[i] = hi > (double)root_max[i] ? (float)(hi + 1e-6 * um) : root_max[i];
    }
    s->max_depth = max_depth > 16 ? 16 : max_depth;
    s->leaf_cap = leaf_capacity;
    s->G = (float)(1u << s->max_depth);
    for (int i = 0; i < 3; ++i) s->scale[i] = s->G / (s->rmax[i] - s->rmin[i]);

    const double margin = margin_of(s);
    const uint32_t zero[3] = {0, 0, 0};
    double lo[3], hi[3];
    cell_bounds(s, 0, zero, lo, hi);
    uint32_t* list = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; ++i)
        if (overlaps(s->sp + 4u * i, lo, hi, margin)) list[m++] = i;
    const uint32_t root = new_node(s);
    build_rec(s, root, 0, zero, list, m);
    free(list);
    return s;
}

void orc_scene_free(orc_scene* s) {
    if (!s) return;
    free(s->sp);
    free(s->albedo);
    free(s->nodes);
    free(s->prims);
    free(s);
}

void orc_scene_info(const orc_scene* s, uint32_t info[4]) {
    info[0] = s->n_nodes;
    info[1] = s->n_leaves;
    info[2] = s->n_prims;
    info[3] = s->depth_reached;
}

/* Breadth-first renumbering of the recursive tree: a node's children get
 * consecutive slots in child order, leaf lists are laid out in slot order;
 * internal record {first child slot, valid | leaf mask << 8}, leaf record
 * {list offset, count}. */
void orc_scene_export_bfs(const orc_scene* s, uint32_t* nodes_out, uint32_t* prim_idx_out) {
    uint32_t* queue = (uint32_t*)malloc(sizeof(uint32_t) * (s->n_nodes ? s->n_nodes : 1));
    uint32_t head = 0, tail = 0, prim = 0;
    queue[tail++] = 0;
    while (head < tail) {
        const uint32_t slot = head;
        const onode* nd = &s->nodes[queue[head++]];
        if (nd->leaf) {
            nodes_out[2 * slot] = prim;
            nodes_out[2 * slot + 1] = nd->cnt;
            for (uint32_t i = 0; i < nd->cnt; ++i) prim_idx_out[prim++] = s->prims[nd->off + i];
            continue;
        }
        uint32_t valid = 0, leafm = 0;
        const uint32_t first = tail;
        for (int ch = 0; ch < 8; ++ch) {
            if (nd->child[ch] < 0) continue;
            valid |= 1u << ch;
            if (s->nodes[nd->child[ch]].leaf) leafm |= 1u << ch;
            queue[tail++] = (uint32_t)nd->child[ch];
        }
        nodes_out[2 * slot] = first;
        nodes_out[2 * slot + 1] = valid | (leafm << 8);
    }
    free(queue);
}

void orc_scene_root(const orc_scene* s, float rmin[3], float rmax[3]) {
    for (int i = 0; i < 3; ++i) {
        rmin[i] = s->rmin[i];
        rmax[i] = s->rmax[i];
    }
}

/* ---- ray / sphere ---------------------------------------------------------- */

/* Nearest root of |o + t d - c| = r with the perpendicular-distance
 * discriminant (no b*b - c cancellation), written with explicit fmaf so the
 * kernel evaluates the identical operations; accepted iff tmin < t < tmax. */
static inline int isect(const float o[3], const float d[3], const float* sp, float tmin,
                        float tmax, float* tout) {
    const float ocx = o[0] - sp[0];
    const float ocy = o[1] - sp[1];
    const float ocz = o[2] - sp[2];
    const float b = fmaf(ocz, d[2], fmaf(ocy, d[1], ocx * d[0]));
    const float qx = fmaf(-b, d[0], ocx);
    const float qy = fmaf(-b, d[1], ocy);
    const float qz = fmaf(-b, d[2], ocz);
    const float qq = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
    const float r = sp[3];
    const float h = fmaf(r, r, -qq);
    if (h < 0.0f) return 0;
    const float sq = sqrtf(h);
    float t = -b - sq;
    if (!(t > tmin)) t = -b + sq;
    if (!(t > tmin) || !(t < tmax)) return 0;
    *tout = t;
    return 1;
}

/* Test-only check of the PRODUCT's camera-relative screen (not part of the
 * spec: the screen decides only which chunks run the exact tests, DESIGN.md
 * 5.1).  Pair k is ray (o, dirs[3k..]) against sphere sp[4 idx[k]..]: the
 * screen record is {o - c in f32, C' = |o - c|^2 - r^2 - slack_oc u |o - c|^2
 * - slack_r u r^2 in f64 rounded toward -inf}, u = 2^-24 (rt_kernels.hip
 * cam_screen_kernel), and the screen passes iff !(fmaf(b, b, -C') < 0) with b
 * isect's b.  out[0] = pairs isect's discriminant accepts (h >= 0) that the
 * screen rejects (a sound screen has none), out[1] = pairs the screen passes,
 * out[2] = pairs with h >= 0. */
void orc_cam_screen_check(const float o[3], const float* dirs, const float* sp, const uint32_t* idx,
                          uint32_t m, double slack_oc, double slack_r, uint64_t out[3]) {
    const double u = 1.0 / 16777216.0;
    out[0] = out[1] = out[2] = 0;
    for (uint32_t k = 0; k < m; ++k) {
        const float* d = dirs + 3u * k;
        const float* s = sp + 4u * idx[k];
        const float ocx = o[0] - s[0], ocy = o[1] - s[1], ocz = o[2] - s[2];
        const float b = fmaf(ocz, d[2], fmaf(ocy, d[1], ocx * d[0]));
        const float qx = fmaf(-b, d[0], ocx);
        const float qy = fmaf(-b, d[1], ocy);
        const float qz = fmaf(-b, d[2], ocz);
        const float qq = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
        const float h = fmaf(s[3], s[3], -qq);
        const double oo = (double)ocx * ocx + (double)ocy * ocy + (double)ocz * ocz;
        const double rr = (double)s[3] * s[3];
        const double cd = oo - rr - slack_oc * u * oo - slack_r * u * rr;
        float c = (float)cd;
        if ((double)c > cd) c = nextafterf(c, -INFINITY);  /* toward -inf */
        const int pass = !(fmaf(b, b, -c) < 0.0f);
        const int exact = !(h < 0.0f);
        out[0] += (uint64_t)(exact && !pass);
        out[1] += (uint64_t)pass;
        out[2] += (uint64_t)exact;
    }
}

/* Test-only: the product's image-plane screen of primary rays (rt_kernels.hip
 * cam8_screen_kernel and walk<>'s cam8 chunk screen; rt_capi.cpp cam8_basis
 * makes the basis B, rows x, y, z in f32) against the exact discriminant of
 * isect, for m (direction, sphere) pairs from camera origin o.  The record
 * is made as the kernel makes it (f64, rho^2 as bf16 in the low bytes of
 * {qx, qy}); the lane's point from its f32 direction with each of the three
 * f32 values next to 1/pz (the GPU's v_rcp_f32 is within 1 ulp), and a pair
 * counts as passed only if all three pass.  shrink scales rho (1 = the
 * product; < 1 must be seen to miss).  out[0] = pairs the exact test accepts
 * and the screen rejects (must be 0), out[1] = pairs passed, out[2] = pairs
 * the exact test accepts. */
void orc_cam8_screen_check(const float o[3], const float B[9], uint32_t ok, const float* dirs,
                           const float* sp, const uint32_t* idx, uint32_t m, double shrink,
                           uint64_t out[3]) {
    out[0] = out[1] = out[2] = 0;
    for (uint32_t k = 0; k < m; ++k) {
        const float* d = dirs + 3u * k;
        const float* s = sp + 4u * idx[k];
        /* the record (cam8_screen_kernel) */
        const double vx = (double)s[0] - o[0], vy = (double)s[1] - o[1], vz = (double)s[2] - o[2];
        const double X = (double)B[0] * vx + (double)B[1] * vy + (double)B[2] * vz;
        const double Y = (double)B[3] * vx + (double)B[4] * vy + (double)B[5] * vz;
        const double Z = (double)B[6] * vx + (double)B[7] * vy + (double)B[8] * vz;
        const double dist = sqrt(vx * vx + vy * vy + vz * vz);
        const double rp = (double)s[3] * (1.0 + 1e-6);
        uint32_t hx = 0u, hy = 0u, rb = 0x7F800000u;
        int pass_all = !ok || !(dist > rp * 1.0001) || !(Z > 0.0) || !isfinite(dist) || !(s[3] >= 0.0f);
        if (!pass_all) {
            const double az = Z / dist;
            const double beta = acos(fmin(1.0, az));
            const double th = asin(fmin(1.0, rp / dist));
            if (!(beta + th < 1.45)) {
                pass_all = 1;
            } else {
                const float qx = (float)(X / Z), qy = (float)(Y / Z);
                const double q = fabs((double)qx) + fabs((double)qy);
                const double rho_g = sin(th) / (az * cos(beta + th));
                const double eps_c = 1.5 * (1.0 / 16384.0) * q;
                const double mm = 1.0 + q + rho_g;
                const double rho = (rho_g * (1.0 + 1e-5) + eps_c + 4e-6 * mm * mm) * shrink;
                const double r2d = rho * rho * (1.0 + 1e-6);
                float r2 = (float)r2d;
                if ((double)r2 < r2d) r2 = nextafterf(r2, INFINITY); /* toward +inf */
                uint32_t bits;
                memcpy(&bits, &r2, 4);
                if (bits & 0xFFFFu) bits = (bits & 0xFFFF0000u) + 0x10000u;
                if (isfinite(r2) && bits < 0x7F800000u) {
                    rb = bits;
                    memcpy(&hx, &qx, 4);
                    memcpy(&hy, &qy, 4);
                } else {
                    pass_all = 1;
                }
            }
        }
        const uint32_t sxb = (hx & ~0xFFu) | (rb >> 24), syb = (hy & ~0xFFu) | ((rb >> 16) & 0xFFu);
        float rqx, rqy, rho2;
        memcpy(&rqx, &sxb, 4);
        memcpy(&rqy, &syb, 4);
        const uint32_t rbits = ((sxb & 0xFFu) << 24) | ((syb & 0xFFu) << 16); /* v_perm_b32 0x04000C0C */
        memcpy(&rho2, &rbits, 4);
        /* the lane (walk<> cam8) */
        const float px = fmaf(B[2], d[2], fmaf(B[1], d[1], B[0] * d[0]));
        const float py = fmaf(B[5], d[2], fmaf(B[4], d[1], B[3] * d[0]));
        const float pz = fmaf(B[8], d[2], fmaf(B[7], d[1], B[6] * d[0]));
        const float iz0 = 1.0f / pz;
        const float izs[3] = {nextafterf(iz0, -INFINITY), iz0, nextafterf(iz0, INFINITY)};
        int pass = 1;
        for (int v = 0; v < 3; ++v) {
            const float s8x = px * izs[v], s8y = py * izs[v];
            const float dx = s8x - rqx, dy = s8y - rqy;
            pass &= !(fmaf(dy, dy, dx * dx) > rho2);
        }
        (void)pass_all;
        /* the exact discriminant (isect) */
        const float ocx = o[0] - s[0], ocy = o[1] - s[1], ocz = o[2] - s[2];
        const float b = fmaf(ocz, d[2], fmaf(ocy, d[1], ocx * d[0]));
        const float qx = fmaf(-b, d[0], ocx);
        const float qy = fmaf(-b, d[1], ocy);
        const float qz = fmaf(-b, d[2], ocz);
        const float qq = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
        const float h = fmaf(s[3], s[3], -qq);
        const int exact = !(h < 0.0f);
        out[0] += (uint64_t)(exact && !pass);
        out[1] += (uint64_t)pass;
        out[2] += (uint64_t)exact;
    }
}

/* Test-only: the light-plane screen with 8-byte records carrying each
 * sphere's own rr' as bf16 in the low bytes of {u, v} (rt_kernels.hip
 * shd_screen_kernel and walk<> under RT_SHD8_PER): as orc_shd_screen_check,
 * the radius grown by the stored centre's error 2^-14 (|u| + |v|) and the
 * result scaled by shrink (1 = the product). */
void orc_shd8_screen_check(const float* origins, const float L[3], const float* sp,
                           const uint32_t* idx, uint32_t m, double big_m, double slack_m,
                           double grow, double shrink, uint64_t out[3]) {
    const double u = 1.0 / 16777216.0;
    double l[3] = {L[0], L[1], L[2]};
    const double ln = sqrt(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]);
    for (int i = 0; i < 3; ++i) l[i] /= ln;
    int kmin = 0;
    for (int i = 1; i < 3; ++i)
        if (fabs(l[i]) < fabs(l[kmin])) kmin = i;
    double e1[3] = {0.0, 0.0, 0.0};
    e1[kmin] = 1.0;
    const double al = l[kmin];
    for (int i = 0; i < 3; ++i) e1[i] -= al * l[i];
    const double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    for (int i = 0; i < 3; ++i) e1[i] /= n1;
    const double e2[3] = {l[1] * e1[2] - l[2] * e1[1], l[2] * e1[0] - l[0] * e1[2],
                          l[0] * e1[1] - l[1] * e1[0]};
    float e[6];
    for (int i = 0; i < 3; ++i) {
        e[i] = (float)e1[i];
        e[3 + i] = (float)e2[i];
    }
    const double delta = slack_m * u * (big_m + 1e-4);
    out[0] = out[1] = out[2] = 0;
    for (uint32_t k = 0; k < m; ++k) {
        const float* o = origins + 3u * k;
        const float* s = sp + 4u * idx[k];
        const float ocx = o[0] - s[0], ocy = o[1] - s[1], ocz = o[2] - s[2];
        const float b = fmaf(ocz, L[2], fmaf(ocy, L[1], ocx * L[0]));
        const float qx = fmaf(-b, L[0], ocx);
        const float qy = fmaf(-b, L[1], ocy);
        const float qz = fmaf(-b, L[2], ocz);
        const float qq = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
        const float h = fmaf(s[3], s[3], -qq);
        /* the packed record (shd_screen_kernel) */
        const double cu = (double)s[0] * e[0] + (double)s[1] * e[1] + (double)s[2] * e[2];
        const double cv = (double)s[0] * e[3] + (double)s[1] * e[4] + (double)s[2] * e[5];
        const float cuf = (float)cu, cvf = (float)cv;
        const double ec = (1.0 / 16384.0) * (fabs((double)cuf) + fabs((double)cvf));
        const double rg = ((double)s[3] * (1.0 + grow * u) + delta + ec) * shrink;
        const double rr = rg * rg * (1.0 + grow * u);
        float rrf = (float)rr;
        if ((double)rrf < rr) rrf = nextafterf(rrf, INFINITY);
        uint32_t rb, hu, hv;
        memcpy(&rb, &rrf, 4);
        if (rb & 0xFFFFu) rb = (rb & 0xFFFF0000u) + 0x10000u;
        if (!(isfinite(rrf) && rb < 0x7F800000u)) rb = 0x7F800000u;
        memcpy(&hu, &cuf, 4);
        memcpy(&hv, &cvf, 4);
        const uint32_t su = (hu & ~0xFFu) | (rb >> 24), sv = (hv & ~0xFFu) | ((rb >> 16) & 0xFFu);
        float us, vs, rrd;
        memcpy(&us, &su, 4);
        memcpy(&vs, &sv, 4);
        const uint32_t rbits = ((su & 0xFFu) << 24) | ((sv & 0xFFu) << 16);
        memcpy(&rrd, &rbits, 4);
        /* the lane */
        const float up = fmaf(o[2], e[2], fmaf(o[1], e[1], o[0] * e[0]));
        const float vp = fmaf(o[2], e[5], fmaf(o[1], e[4], o[0] * e[3]));
        const float du = up - us, dv = vp - vs;
        const int pass = !(fmaf(dv, dv, du * du) > rrd);
        const int exact = !(h < 0.0f);
        out[0] += (uint64_t)(exact && !pass);
        out[1] += (uint64_t)pass;
        out[2] += (uint64_t)exact;
    }
}

/* Test-only: the product's light-plane shadow screen (rt_kernels.hip walk<>,
 * shd_screen_kernel; rt_capi.cpp do_render makes the basis) against the
 * exact discriminant of isect, for m (origin, sphere) pairs with the
 * frame's shadow direction L.  The basis {e1, e2} is made from L as the host
 * makes it (f64, rounded to f32); slack_m scales the 2D slack delta =
 * slack_m u (M + 1e-4) and grow (0 or 4) the radius factors of the record.
 * out[0] = pairs the exact test accepts and the screen rejects (must be 0),
 * out[1] = pairs the screen passes, out[2] = pairs the exact test accepts. */
void orc_shd_screen_check(const float* origins, const float L[3], const float* sp,
                          const uint32_t* idx, uint32_t m, double big_m, double slack_m,
                          double grow, uint64_t out[3]) {
    const double u = 1.0 / 16777216.0;
    double l[3] = {L[0], L[1], L[2]};
    const double ln = sqrt(l[0] * l[0] + l[1] * l[1] + l[2] * l[2]);
    for (int i = 0; i < 3; ++i) l[i] /= ln;
    int kmin = 0;
    for (int i = 1; i < 3; ++i)
        if (fabs(l[i]) < fabs(l[kmin])) kmin = i;
    double e1[3] = {0.0, 0.0, 0.0};
    e1[kmin] = 1.0;
    const double al = l[kmin];
    for (int i = 0; i < 3; ++i) e1[i] -= al * l[i];
    const double n1 = sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]);
    for (int i = 0; i < 3; ++i) e1[i] /= n1;
    const double e2[3] = {l[1] * e1[2] - l[2] * e1[1], l[2] * e1[0] - l[0] * e1[2],
                          l[0] * e1[1] - l[1] * e1[0]};
    float e[6];
    for (int i = 0; i < 3; ++i) {
        e[i] = (float)e1[i];
        e[3 + i] = (float)e2[i];
    }
    const double delta = slack_m * u * (big_m + 1e-4);
    out[0] = out[1] = out[2] = 0;
    for (uint32_t k = 0; k < m; ++k) {
        const float* o = origins + 3u * k;
        const float* s = sp + 4u * idx[k];
        /* isect's discriminant (rt_kernels.hip isect_h), direction L */
        const float ocx = o[0] - s[0], ocy = o[1] - s[1], ocz = o[2] - s[2];
        const float b = fmaf(ocz, L[2], fmaf(ocy, L[1], ocx * L[0]));
        const float qx = fmaf(-b, L[0], ocx);
        const float qy = fmaf(-b, L[1], ocy);
        const float qz = fmaf(-b, L[2], ocz);
        const float qq = fmaf(qz, qz, fmaf(qy, qy, qx * qx));
        const float h = fmaf(s[3], s[3], -qq);
        /* the record (f64, rounded) and the lane's screen (f32, as the kernel) */
        const double cu = (double)s[0] * e[0] + (double)s[1] * e[1] + (double)s[2] * e[2];
        const double cv = (double)s[0] * e[3] + (double)s[1] * e[4] + (double)s[2] * e[5];
        const double rg = (double)s[3] * (1.0 + grow * u) + delta;
        const double rr = rg * rg * (1.0 + grow * u);
        float rrf = (float)rr;
        if ((double)rrf < rr) rrf = nextafterf(rrf, INFINITY); /* toward +inf */
        const float up = fmaf(o[2], e[2], fmaf(o[1], e[1], o[0] * e[0]));
        const float vp = fmaf(o[2], e[5], fmaf(o[1], e[4], o[0] * e[3]));
        const float du = up - (float)cu, dv = vp - (float)cv;
        const int pass = !(fmaf(dv, dv, du * du) > rrf);
        const int exact = !(h < 0.0f);
        out[0] += (uint64_t)(exact && !pass);
        out[1] += (uint64_t)pass;
        out[2] += (uint64_t)exact;
    }
}

/* ---- octree walk (DESIGN.md "Octree walk") --------------------------------- */

typedef struct {
    float og[3];   /* origin in (mirrored) grid units */
    float inv[3];  /* 1 / (|d| * scale), |d| clamped to >= 1e-20 */
    float nog[3];  /* -(og * inv) */
    uint32_t mask; /* bit i: axis i mirrored (d_i < 0) */
} walk_t;

/* t of the grid plane at (mirrored) integer coordinate k: one FMA, monotone in k */
static inline float plane(const walk_t* w, int i, uint32_t k) {
    return fmaf((float)k, w->inv[i], w->nog[i]);
}

static int walk(const orc_scene* s, const float o[3], const float d[3], float tmin, float tmax,
                int any_hit, float* t_out, uint32_t* idx_out, uint64_t* nodes, uint64_t* prims) {
    walk_t w;
    w.mask = 0;
    const uint32_t G = 1u << s->max_depth;
    for (int i = 0; i < 3; ++i) {
        const float g = (o[i] - s->rmin[i]) * s->scale[i];
        const int neg = d[i] < 0.0f;
        float a = fabsf(d[i]);
        if (a < 1e-20f) a = 1e-20f;
        w.og[i] = neg ? s->G - g : g;
        w.inv[i] = 1.0f / (a * s->scale[i]);
        w.nog[i] = -(w.og[i] * w.inv[i]);
        w.mask |= (uint32_t)neg << i;
    }
    float t0 = plane(&w, 0, 0), t1 = plane(&w, 0, G);
    for (int i = 1; i < 3; ++i) {
        const float a0 = plane(&w, i, 0), a1 = plane(&w, i, G);
        if (a0 > t0) t0 = a0;
        if (a1 < t1) t1 = a1;
    }
    if (t0 < tmin) t0 = tmin;
    if (t1 > tmax) t1 = tmax;
    if (!(t0 < t1)) return 0;

    float best_t = tmax;
    uint32_t best = 0xFFFFFFFFu;
    const onode* N = s->nodes;
    *nodes += 1; /* root record */
    if (N[0].leaf) {
        for (uint32_t j = 0; j < N[0].cnt; ++j) {
            const uint32_t idx = s->prims[N[0].off + j];
            float t;
            *prims += 1;
            if (isect(o, d, s->sp + 4u * idx, tmin, tmax, &t)) {
                if (any_hit) {
                    *t_out = t;
                    *idx_out = idx;
                    return 1;
                }
                if (t < best_t || (t == best_t && idx < best)) {
                    best_t = t;
                    best = idx;
                }
            }
        }
    } else {
        uint32_t stack[17];
        uint32_t depth = 0, c[3] = {0, 0, 0};
        uint32_t node = 0;
        stack[0] = 0;
        float t = t0;
        for (uint32_t it = 0, cap = 8u * G + 64u; it < cap; ++it) { /* same cap as the kernel */
            const uint32_t half = G >> (depth + 1);
            uint32_t bits = 0;
            for (int i = 0; i < 3; ++i)
                if (plane(&w, i, (2u * c[i] + 1u) * half) <= t) bits |= 1u << i;
            const uint32_t child = bits ^ w.mask;
            for (int i = 0; i < 3; ++i) c[i] = 2u * c[i] + ((bits >> i) & 1u);
            depth += 1;
            const int32_t ch = N[node].child[child];
            if (ch >= 0) {
                *nodes += 1;
                if (!N[ch].leaf) {
                    node = (uint32_t)ch;
                    stack[depth] = node;
                    continue;
                }
                for (uint32_t j = 0; j < N[ch].cnt; ++j) {
                    const uint32_t idx = s->prims[N[ch].off + j];
                    float th;
                    *prims += 1;
                    if (isect(o, d, s->sp + 4u * idx, tmin, tmax, &th)) {
                        if (any_hit) {
                            *t_out = th;
                            *idx_out = idx;
                            return 1;
                        }
                        if (th < best_t || (th == best_t && idx < best)) {
                            best_t = th;
                            best = idx;
                        }
                    }
                }
            }
            /* leave the leaf / empty cell at `depth`, coords c */
            const uint32_t size = G >> depth;
            float e[3];
            for (int i = 0; i < 3; ++i) e[i] = plane(&w, i, (c[i] + 1u) * size);
            float texit = e[0] < e[1] ? e[0] : e[1];
            texit = texit < e[2] ? texit : e[2];
            if (best_t < texit) break;
            if (texit >= t1) break;
            uint32_t diff = 0, out = 0;
            for (int i = 0; i < 3; ++i) {
                if (e[i] == texit) {
                    diff |= c[i] ^ (c[i] + 1u);
                    c[i] += 1u;
                    if (c[i] >= (1u << depth)) out = 1;
                }
            }
            if (out) break;
            const uint32_t m = 32u - (uint32_t)__builtin_clz(diff);
            depth -= m;
            for (int i = 0; i < 3; ++i) c[i] >>= m;
            node = stack[depth];
            t = texit;
        }
    }
    if (best != 0xFFFFFFFFu) {
        *t_out = best_t;
        *idx_out = best;
        return 1;
    }
    return 0;
}

int orc_trace(const orc_scene* s, const float o[3], const float d[3], float tmin, float tmax,
              int any_hit, float* t_out, uint32_t* idx_out, uint64_t counters[4]) {
    uint64_t nodes = 0, prims = 0;
    const int h = walk(s, o, d, tmin, tmax, any_hit, t_out, idx_out, &nodes, &prims);
    if (counters) {
        counters[2] += nodes;
        counters[3] += prims;
    }
    return h;
}

/* Brute force over every sphere (cross-check of the walk's conservativeness). */
int orc_trace_brute(const orc_scene* s, const float o[3], const float d[3], float tmin,
                    float tmax, int any_hit, float* t_out, uint32_t* idx_out) {
    float best_t = tmax;
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t i = 0; i < s->n; ++i) {
        float t;
        if (isect(o, d, s->sp + 4u * i, tmin, tmax, &t)) {
            if (any_hit) {
                *t_out = t;
                *idx_out = i;
                return 1;
            }
            if (t < best_t || (t == best_t && i < best)) {
                best_t = t;
                best = i;
            }
        }
    }
    if (best == 0xFFFFFFFFu) return 0;
    *t_out = best_t;
    *idx_out = best;
    return 1;
}

/* ========================================================================== */
/* scene render (DESIGN.md "Scene mode")                                      */
/* ========================================================================== */

#define SHADOW_EPS 1e-5f

/* Pairwise sum of n (a power of two) values: T(lo, n) = T(lo, n/2) + T(lo+n/2, n/2).
 * This is exactly what a shfl_xor butterfly over n lanes produces (each step
 * adds the same two partial sums in every lane; float + is commutative). */
static float tree_sum(const float* v, uint32_t n) {
    if (n == 1) return v[0];
    const uint32_t h = n / 2;
    return tree_sum(v, h) + tree_sum(v + h, h);
}

void orc_render_scene(const orc_scene* s, uint32_t W, uint32_t H, const float pose[16],
                      const float K[9], uint32_t spp, uint32_t seed, uint32_t flags,
                      const float light_dir[3], float ambient, uint32_t x0, uint32_t y0,
                      uint32_t x1, uint32_t y1, uint32_t row_step, uint32_t row_phase,
                      uint8_t* out8, float* out32, uint64_t counters[4], int n_threads) {
    orc_render_scene_frame(s, W, H, pose, K, spp, seed, flags, light_dir, ambient, x0, y0, x1, y1,
                           row_step, row_phase, 0, NULL, out8, out32, counters, n_threads);
}

void orc_render_scene_frame(const orc_scene* s, uint32_t W, uint32_t H, const float pose[16],
                            const float K[9], uint32_t spp, uint32_t seed, uint32_t flags,
                            const float light_dir[3], float ambient, uint32_t x0, uint32_t y0,
                            uint32_t x1, uint32_t y1, uint32_t row_step, uint32_t row_phase,
                            uint32_t frame, float* accum, uint8_t* out8, float* out32,
                            uint64_t counters[4], int n_threads) {
    const float origin[3] = {pose[12], pose[13], pose[14]};
    const int jitter = (flags & 1u) != 0;
    const int shadows = (flags & 8u) == 0;
    /* L = -normalize(light_dir): direction toward the light */
    const float ll = sqrtf(light_dir[0] * light_dir[0] + light_dir[1] * light_dir[1] +
                           light_dir[2] * light_dir[2]);
    const float L[3] = {-(light_dir[0] / ll), -(light_dir[1] / ll), -(light_dir[2] / ll)};
    /* progressive frame k (accum != NULL): samples [k*spp, (k+1)*spp), added
     * onto the stored sums; the image is the mean over (k+1)*spp samples */
    const uint32_t s_base = accum ? frame * spp : 0u;
    const float inv_spp = 1.0f / (float)(accum ? (frame + 1u) * spp : spp);
    const float miss_r = 200.0f / 255.0f;
    const uint32_t seedmix = mix32(seed ^ 0x9E3779B9u);
    if (x1 > W) x1 = W;
    if (y1 > H) y1 = H;
    if (row_step == 0) row_step = 1;
    uint64_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#ifdef _OPENMP
    if (n_threads > 0) omp_set_num_threads(n_threads);
#else
    (void)n_threads;
#endif
    const long ny = (long)y1 - (long)y0;
#pragma omp parallel for schedule(dynamic, 1) reduction(+ : c0, c1, c2, c3)
    for (long yy = 0; yy < (ny > 0 ? ny : 0); ++yy) {
        const uint32_t y = y0 + (uint32_t)yy;
        if (y % row_step != row_phase % row_step) continue;
        for (uint32_t x = x0; x < x1; ++x) {
            const uint32_t pid = y * W + x;
            const uint32_t hp = mix32(seedmix ^ pid);
            /* Per-pixel sum (DESIGN.md "Accumulate"): samples go in rounds of
             * spw = min(spp, 64); each round is pairwise-summed over g =
             * pow2ceil(spw) slots (missing samples are 0) and the round sums
             * are added in order: acc = T0, acc = acc + T1, ... */
            const uint32_t spw = spp >= 64u ? 64u : spp;
            uint32_t g = 1;
            while (g < spw) g *= 2;
            float rbuf[3][64];
            float ar = 0.0f, ag = 0.0f, ab = 0.0f;
            for (uint32_t sidx = 0; sidx < spp; ++sidx) {
                float u = (float)x, v = (float)y;
                const uint32_t sg = s_base + sidx;
                if (jitter) {
                    u = u + u01(mix32(hp ^ (sg << 1)));
                    v = v + u01(mix32(hp ^ ((sg << 1) | 1u)));
                }
                float d[3];
                orc_get_ray(pose, K, u, v, d);
                c0 += 1;
                float t;
                uint32_t idx;
                uint64_t nn = 0, pp = 0;
                float cr, cg, cb;
                if (!walk(s, origin, d, 0.0f, INFINITY, 0, &t, &idx, &nn, &pp)) {
                    cr = miss_r;
                    cg = sat(d[1]);
                    cb = sat(d[2]);
                } else {
                    const float* sp = s->sp + 4u * idx;
                    const float p[3] = {origin[0] + t * d[0], origin[1] + t * d[1],
                                        origin[2] + t * d[2]};
                    const float ir = 1.0f / sp[3];
                    const float n[3] = {(p[0] - sp[0]) * ir, (p[1] - sp[1]) * ir,
                                        (p[2] - sp[2]) * ir};
                    const float ndl = n[0] * L[0] + n[1] * L[1] + n[2] * L[2];
                    float lam = ndl > 0.0f ? ndl : 0.0f;
                    if (ndl > 0.0f && shadows) {
                        const float so[3] = {p[0] + n[0] * SHADOW_EPS, p[1] + n[1] * SHADOW_EPS,
                                             p[2] + n[2] * SHADOW_EPS};
                        float ts;
                        uint32_t is;
                        c1 += 1;
                        if (walk(s, so, L, 0.0f, INFINITY, 1, &ts, &is, &nn, &pp)) lam = 0.0f;
                    }
                    const float f = ambient + (1.0f - ambient) * lam;
                    const uint32_t a = s->albedo[idx];
                    cr = (float)(a & 0xFFu) * (1.0f / 255.0f) * f;
                    cg = (float)((a >> 8) & 0xFFu) * (1.0f / 255.0f) * f;
                    cb = (float)((a >> 16) & 0xFFu) * (1.0f / 255.0f) * f;
                }
                c2 += nn;
                c3 += pp;
                const uint32_t slot = sidx % spw;
                if (slot == 0)
                    for (uint32_t q = 0; q < g; ++q) rbuf[0][q] = rbuf[1][q] = rbuf[2][q] = 0.0f;
                rbuf[0][slot] = cr;
                rbuf[1][slot] = cg;
                rbuf[2][slot] = cb;
                if (slot == spw - 1 || sidx == spp - 1) {
                    const float tr = tree_sum(rbuf[0], g), tg = tree_sum(rbuf[1], g),
                                tb = tree_sum(rbuf[2], g);
                    if (sidx < spw && !(accum && frame)) {
                        ar = tr;
                        ag = tg;
                        ab = tb;
                    } else if (sidx < spw) { /* progressive: onto the stored sum */
                        const float* pa = accum + 4u * (size_t)pid;
                        ar = pa[0] + tr;
                        ag = pa[1] + tg;
                        ab = pa[2] + tb;
                    } else {
                        ar = ar + tr;
                        ag = ag + tg;
                        ab = ab + tb;
                    }
                }
            }
            if (accum) {
                float* pa = accum + 4u * (size_t)pid;
                pa[0] = ar;
                pa[1] = ag;
                pa[2] = ab;
                pa[3] = 0.0f;
            }
            const float mr = ar * inv_spp, mg = ag * inv_spp, mb = ab * inv_spp;
            uint8_t* px = out8 + 4u * (size_t)pid;
            px[0] = (uint8_t)(sat(mr) * 255.0f);
            px[1] = (uint8_t)(sat(mg) * 255.0f);
            px[2] = (uint8_t)(sat(mb) * 255.0f);
            px[3] = 255;
            if (out32) {
                float* pf = out32 + 4u * (size_t)pid;
                pf[0] = mr;
                pf[1] = mg;
                pf[2] = mb;
                pf[3] = 1.0f;
            }
        }
    }
    if (counters) {
        counters[0] += c0;
        counters[1] += c1;
        counters[2] += c2;
        counters[3] += c3;
    }
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
