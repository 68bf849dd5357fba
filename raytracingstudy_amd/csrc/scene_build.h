// scene_build.h — host-side synthetic scene generator and octree builder.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace rtamd {

struct HostNode {  // mirrors the device uint2 record
    uint32_t x, y;
};

struct BuiltOctree {
    std::vector<HostNode> nodes;     // nodes[0] = root
    std::vector<float> prim_sp;      // 4 floats per leaf reference
    std::vector<uint32_t> prim_idx;  // sphere index per leaf reference
    float rmin[3], rmax[3];          // effective root box (see build_octree)
    bool root_is_leaf = false;
    uint32_t n_leaves = 0;
    uint32_t depth_reached = 0;
};

// SURVEY.md 8d D2 generator (splitmix64 -> PCG32).
void generate_spheres(uint32_t n, uint32_t seed, float* spheres, uint32_t* albedo);

// Octree over [rmin, rmax] grown (only where needed, by a 1e-6*extent margin)
// to enclose every sphere's AABB: split a cell while it holds more than
// leaf_cap spheres and depth < max_depth; sphere/cell overlap is the
// conservative double-precision test of DESIGN.md "Octree build".
void build_octree(const float* spheres, uint32_t n, const float rmin[3], const float rmax[3],
                  uint32_t max_depth, uint32_t leaf_cap, BuiltOctree& out);

uint32_t depth_for_resolution(const float rmin[3], const float rmax[3], float res);

uint32_t mix32(uint32_t x);

// Binary sphere list: a 32-byte little-endian header
// {"RTSPHERE", u32 version = 1, u32 n, u32 flags (bit 0: albedo present),
// u32 header bytes = 32, u64 0}, then n x {f32 cx, cy, cz, r}, then n x u32
// RGBA8 when flag bit 0 is set.
bool save_sphere_file(const char* path, const float* spheres, const uint32_t* albedo, uint32_t n,
                      std::string* err);
// spheres == nullptr: only *n_out.  Otherwise capacity >= n; albedo may be
// nullptr; missing colours read as 0.8 grey.
bool load_sphere_file(const char* path, float* spheres, uint32_t* albedo, uint32_t capacity,
                      uint32_t* n_out, std::string* err);

}  // namespace rtamd
