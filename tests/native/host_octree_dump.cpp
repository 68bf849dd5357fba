// Test harness: run the product's host octree builder (scene_build.cpp) on a
// sphere file and dump the tree, so tests/test_octree_build.py can compare it
// with the oracle's tree without a GPU.
//   host_octree_dump <spheres.rtsph> <minx miny minz maxx maxy maxz> <depth> <cap> <out_prefix>
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "../../raytracingstudy_amd/csrc/scene_build.h"

int main(int argc, char** argv) {
    if (argc != 11) {
        fprintf(stderr, "usage: %s file minx miny minz maxx maxy maxz depth cap out\n", argv[0]);
        return 2;
    }
    uint32_t n = 0;
    std::string err;
    if (!rtamd::load_sphere_file(argv[1], nullptr, nullptr, 0, &n, &err)) {
        fprintf(stderr, "%s\n", err.c_str());
        return 1;
    }
    std::vector<float> sp(4u * (n ? n : 1));
    if (!rtamd::load_sphere_file(argv[1], sp.data(), nullptr, n, &n, &err)) {
        fprintf(stderr, "%s\n", err.c_str());
        return 1;
    }
    const float mn[3] = {strtof(argv[2], 0), strtof(argv[3], 0), strtof(argv[4], 0)};
    const float mx[3] = {strtof(argv[5], 0), strtof(argv[6], 0), strtof(argv[7], 0)};
    rtamd::BuiltOctree t;
    rtamd::build_octree(sp.data(), n, mn, mx, (uint32_t)atoi(argv[8]), (uint32_t)atoi(argv[9]), t);
    const std::string out = argv[10];
    FILE* f = fopen((out + ".nodes").c_str(), "wb");
    fwrite(t.nodes.data(), sizeof(rtamd::HostNode), t.nodes.size(), f);
    fclose(f);
    f = fopen((out + ".prims").c_str(), "wb");
    fwrite(t.prim_idx.data(), 4, t.prim_idx.size(), f);
    fclose(f);
    f = fopen((out + ".sp").c_str(), "wb");
    fwrite(t.prim_sp.data(), 4, t.prim_sp.size(), f);
    fclose(f);
    printf("%zu %u %zu %u %d %.9g %.9g %.9g %.9g %.9g %.9g\n", t.nodes.size(), t.n_leaves,
           t.prim_idx.size(), t.depth_reached, t.root_is_leaf ? 1 : 0, t.rmin[0], t.rmin[1],
           t.rmin[2], t.rmax[0], t.rmax[1], t.rmax[2]);
    return 0;
}
