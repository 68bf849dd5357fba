// scene_build.cpp — host-side scene generator + breadth-first octree builder.
//
// The reference has no primitives and no octree structure: Octree holds only
// its bounds and `resolution` (include/octree.h:7-23, constructed with
// min 0, max 1.28, resolution 0.01 at src/renderer.cu:134-138) and traverse()
// is a stub.  This builder defines the structure the render kernel walks;
// the semantics are specified in DESIGN.md "Octree build".
#include <stdexcept>
#include "scene_build.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

namespace rtamd {

uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

namespace {

uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Pcg32 {
    uint64_t state, inc;
    uint32_t next() {
        const uint64_t old = state;
        state = old * 6364136223846793005ull + inc;
        const uint32_t xs = static_cast<uint32_t>(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = static_cast<uint32_t>(old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
    float unit() { return static_cast<float>(next() >> 8) * (1.0f / 16777216.0f); }
};

struct Cell {
    uint32_t depth;
    uint32_t c[3];
    uint32_t slot;               // index of this node's record in nodes[]
    std::vector<uint32_t> list;  // sphere indices, ascending
};

struct Geometry {
    double lo[3], ext[3];
    double margin;
    void bounds(uint32_t depth, const uint32_t c[3], double blo[3], double bhi[3]) const {
        const double cells = static_cast<double>(1u << depth);
        for (int i = 0; i < 3; ++i) {
            blo[i] = lo[i] + ext[i] * (static_cast<double>(c[i]) / cells);
            bhi[i] = lo[i] + ext[i] * (static_cast<double>(c[i] + 1u) / cells);
        }
    }
    bool overlaps(const float* sp, const double blo[3], const double bhi[3]) const {
        double d2 = 0.0;
        for (int i = 0; i < 3; ++i) {
            const double c = static_cast<double>(sp[i]);
            if (c < blo[i]) {
                const double e = blo[i] - c;
                d2 += e * e;
            } else if (c > bhi[i]) {
                const double e = c - bhi[i];
                d2 += e * e;
            }
        }
        const double r = static_cast<double>(sp[3]) + margin;
        return d2 <= r * r;
    }
};

}  // namespace

void generate_spheres(uint32_t n, uint32_t seed, float* sp, uint32_t* albedo) {
    uint64_t sm = seed;
    Pcg32 g;
    g.state = splitmix64(sm);
    g.inc = splitmix64(sm) | 1ull;
    const float rscale = n ? static_cast<float>(0.02 * cbrt(1000.0 / static_cast<double>(n))) : 0.0f;
    for (uint32_t i = 0; i < n; ++i) {
        const float cx = g.unit() * 1.28f;
        const float cy = g.unit() * 1.28f;
        const float cz = g.unit() * 1.28f;
        const float ru = g.unit();
        sp[4 * i + 0] = cx;
        sp[4 * i + 1] = cy;
        sp[4 * i + 2] = cz;
        sp[4 * i + 3] = rscale * (0.5f + 0.5f * ru);
        uint32_t a = 0xFF000000u;
        for (int c = 0; c < 3; ++c) {
            const float v = 0.2f + 0.8f * g.unit();
            a |= (static_cast<uint32_t>(v * 255.0f) & 0xFFu) << (8 * c);
        }
        if (albedo) albedo[i] = a;
    }
}

uint32_t depth_for_resolution(const float rmin[3], const float rmax[3], float res) {
    float ext = 0.0f;
    for (int i = 0; i < 3; ++i) ext = std::max(ext, rmax[i] - rmin[i]);
    if (!(res > 0.0f)) return 7;
    uint32_t d = 0;
    while (d < 16 && static_cast<double>(ext) / static_cast<double>(1u << d) >
                         static_cast<double>(res) * (1.0 + 1e-6))
        ++d;
    return d;
}

void build_octree(const float* spheres, uint32_t n, const float rmin[3], const float rmax[3],
                  uint32_t max_depth, uint32_t leaf_cap, BuiltOctree& out) {
    out = BuiltOctree();
    double um = 0.0;
    for (int i = 0; i < 3; ++i)
        um = std::max(um, static_cast<double>(rmax[i]) - static_cast<double>(rmin[i]));
    for (int i = 0; i < 3; ++i) {
        double lo = static_cast<double>(rmin[i]), hi = static_cast<double>(rmax[i]);
        for (uint32_t k = 0; k < n; ++k) {
            const double c = static_cast<double>(spheres[4 * k + i]);
            const double r = static_cast<double>(spheres[4 * k + 3]);
            lo = std::min(lo, c - r);
            hi = std::max(hi, c + r);
        }
        out.rmin[i] = lo < static_cast<double>(rmin[i]) ? static_cast<float>(lo - 1e-6 * um) : rmin[i];
        out.rmax[i] = hi > static_cast<double>(rmax[i]) ? static_cast<float>(hi + 1e-6 * um) : rmax[i];
    }
    Geometry geo;
    double m = 0.0;
    for (int i = 0; i < 3; ++i) {
        geo.lo[i] = static_cast<double>(out.rmin[i]);
        geo.ext[i] = static_cast<double>(out.rmax[i]) - static_cast<double>(out.rmin[i]);
        m = std::max(m, geo.ext[i]);
    }
    geo.margin = 1e-6 * m;

    Cell root;
    root.depth = 0;
    root.c[0] = root.c[1] = root.c[2] = 0;
    root.slot = 0;
    {
        double blo[3], bhi[3];
        geo.bounds(0, root.c, blo, bhi);
        for (uint32_t i = 0; i < n; ++i)
            if (geo.overlaps(spheres + 4u * i, blo, bhi)) root.list.push_back(i);
    }
    out.nodes.push_back({0, 0});

    auto is_leaf = [&](const Cell& c) {
        return c.list.size() <= leaf_cap || c.depth >= max_depth;
    };
    out.root_is_leaf = is_leaf(root);

    // Breadth-first: `level` holds the cells of one depth in slot order, so
    // every node's children are appended as one contiguous block.
    std::vector<Cell> level;
    level.push_back(std::move(root));
    std::vector<uint32_t> sub;
    while (!level.empty()) {
        std::vector<Cell> next;
        for (Cell& cell : level) {
            if (is_leaf(cell)) {
                // leaf offsets are 32-bit record fields (+ the kPrimPad tail)
                if (out.prim_idx.size() + cell.list.size() + 4u >= (size_t(1) << 32))
                    throw std::length_error("more than 2^32 - 5 leaf references");
                const uint32_t off = static_cast<uint32_t>(out.prim_idx.size());
                for (uint32_t idx : cell.list) {
                    out.prim_idx.push_back(idx);
                    out.prim_sp.insert(out.prim_sp.end(), spheres + 4u * idx, spheres + 4u * idx + 4);
                }
                out.nodes[cell.slot] = {off, static_cast<uint32_t>(cell.list.size())};
                out.n_leaves++;
                out.depth_reached = std::max(out.depth_reached, cell.depth);
                continue;
            }
            uint32_t valid = 0, leafm = 0;
            Cell kids[8];
            for (uint32_t ch = 0; ch < 8; ++ch) {
                Cell& k = kids[ch];
                k.depth = cell.depth + 1;
                k.c[0] = 2 * cell.c[0] + (ch & 1u);
                k.c[1] = 2 * cell.c[1] + ((ch >> 1) & 1u);
                k.c[2] = 2 * cell.c[2] + ((ch >> 2) & 1u);
                double blo[3], bhi[3];
                geo.bounds(k.depth, k.c, blo, bhi);
                for (uint32_t idx : cell.list)
                    if (geo.overlaps(spheres + 4u * idx, blo, bhi)) k.list.push_back(idx);
                if (k.list.empty()) continue;
                valid |= 1u << ch;
                if (is_leaf(k)) leafm |= 1u << ch;
            }
            if (out.nodes.size() + 8u >= (size_t(1) << 32))
                throw std::length_error("more than 2^32 - 9 node records");
            const uint32_t first = static_cast<uint32_t>(out.nodes.size());
            out.nodes[cell.slot] = {first, valid | (leafm << 8)};
            for (uint32_t ch = 0; ch < 8; ++ch) {
                if (!(valid & (1u << ch))) continue;
                kids[ch].slot = static_cast<uint32_t>(out.nodes.size());
                out.nodes.push_back({0, 0});
                next.push_back(std::move(kids[ch]));
            }
            std::vector<uint32_t>().swap(cell.list);
        }
        level.swap(next);
    }
}

namespace {

constexpr char kSphereMagic[8] = {'R', 'T', 'S', 'P', 'H', 'E', 'R', 'E'};
constexpr uint32_t kSphereVersion = 1, kSphereHeader = 32;

void put32(unsigned char* p, uint32_t v) {
    for (int i = 0; i < 4; ++i) p[i] = static_cast<unsigned char>(v >> (8 * i));
}
uint32_t get32(const unsigned char* p) {
    return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}

struct File {
    FILE* f;
    explicit File(FILE* x) : f(x) {}
    ~File() {
        if (f) fclose(f);
    }
};

}  // namespace

bool save_sphere_file(const char* path, const float* spheres, const uint32_t* albedo, uint32_t n,
                      std::string* err) {
    File f(fopen(path, "wb"));
    if (!f.f) {
        *err = std::string("cannot open ") + path + " for writing";
        return false;
    }
    unsigned char h[kSphereHeader] = {0};
    memcpy(h, kSphereMagic, 8);
    put32(h + 8, kSphereVersion);
    put32(h + 12, n);
    put32(h + 16, albedo ? 1u : 0u);
    put32(h + 20, kSphereHeader);
    bool ok = fwrite(h, 1, sizeof(h), f.f) == sizeof(h);
    // payload little-endian: the host (x86-64) order, written as is
    if (ok && n) ok = fwrite(spheres, sizeof(float) * 4, n, f.f) == n;
    if (ok && n && albedo) ok = fwrite(albedo, sizeof(uint32_t), n, f.f) == n;
    if (ok) ok = fflush(f.f) == 0;
    if (!ok) *err = std::string("write error on ") + path;
    return ok;
}

bool load_sphere_file(const char* path, float* spheres, uint32_t* albedo, uint32_t capacity,
                      uint32_t* n_out, std::string* err) {
    File f(fopen(path, "rb"));
    if (!f.f) {
        *err = std::string("cannot open ") + path;
        return false;
    }
    unsigned char h[kSphereHeader];
    if (fread(h, 1, sizeof(h), f.f) != sizeof(h) || memcmp(h, kSphereMagic, 8) != 0) {
        *err = std::string(path) + ": not a sphere file (bad magic)";
        return false;
    }
    const uint32_t ver = get32(h + 8), n = get32(h + 12), flags = get32(h + 16),
                   hb = get32(h + 20);
    if (ver != kSphereVersion || hb != kSphereHeader || (flags & ~1u)) {
        *err = std::string(path) + ": unsupported sphere file version/header";
        return false;
    }
    const bool has_albedo = flags & 1u;
    if (fseek(f.f, 0, SEEK_END) != 0) {
        *err = std::string(path) + ": cannot seek";
        return false;
    }
    const long size = ftell(f.f);
    const uint64_t want = kSphereHeader + uint64_t(n) * 16u + (has_albedo ? uint64_t(n) * 4u : 0u);
    if (size < 0 || uint64_t(size) != want) {
        *err = std::string(path) + ": file size does not match its sphere count";
        return false;
    }
    *n_out = n;
    if (!spheres) return true;
    if (capacity < n) {
        *err = std::string(path) + ": capacity smaller than the sphere count";
        return false;
    }
    fseek(f.f, kSphereHeader, SEEK_SET);
    if (n && fread(spheres, sizeof(float) * 4, n, f.f) != n) {
        *err = std::string(path) + ": short read";
        return false;
    }
    if (albedo) {
        if (has_albedo) {
            if (n && fread(albedo, sizeof(uint32_t), n, f.f) != n) {
                *err = std::string(path) + ": short read";
                return false;
            }
        } else {
            for (uint32_t i = 0; i < n; ++i) albedo[i] = 0xFFCCCCCCu;
        }
    }
    return true;
}

}  // namespace rtamd
