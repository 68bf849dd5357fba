// rt_renderer.hpp — header-only C++ host surface with the reference's
// KernelRenderer method names (include/renderer.cuh:25-50), forwarding to the
// C-ABI in rt.h.  A maintainer swaps `#include "renderer.cuh"` for this header
// in Displayer (src/window/displayer.cpp, include/window/displayer.h) and
// passes glm::value_ptr(...) where the reference passed glm matrices by value.
//
// Differences from the reference, all additive:
//   * every method reports failure (throws rtamd::Error with the library's
//     message) instead of returning void silently (src/renderer.cu:143-153);
//   * render() takes the device pointer the GL PBO maps to (the caller keeps
//     hipGraphicsMapResources / hipGraphicsUnmapResources, exactly where the
//     reference calls cudaGraphicsMapResources at src/renderer.cu:145-151),
//     or nullptr for the renderer's own framebuffer;
//   * setOctree (declared but never defined in the reference,
//     include/renderer.cuh:35) is implemented, and setScene adds spheres.
#pragma once

#include <stdexcept>
#include <string>
#include <vector>

#include "rt.h"

namespace rtamd {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& msg) : std::runtime_error(msg), code(code) {}
    int code;
};

inline void check(int code, const rt_renderer* r = nullptr) {
    if (code != RT_OK) throw Error(code, rt_last_error(r));
}

class KernelRenderer {
public:
    // Reference: KernelRenderer(cudaGraphicsResource_t, int width, int height)
    // (src/renderer.cu:124-141).  The graphics resource stays with the caller.
    KernelRenderer(int width, int height, uint32_t mode = RT_MODE_COMPAT, uint32_t spp = 1,
                   int device = -1) {
        rt_config cfg;
        rt_config_default(&cfg);
        cfg.width = static_cast<uint32_t>(width);
        cfg.height = static_cast<uint32_t>(height);
        cfg.mode = mode;
        cfg.spp = spp;
        cfg.device = device;
        check(rt_create(&cfg, &r_));
    }
    // The reference's exact constructor shape (src/renderer.cu:124-141): the
    // PBO resource (registered with hipGraphicsGLRegisterBuffer) is bound, so
    // render() maps, renders into and unmaps it.
    KernelRenderer(void* graphics_resource, int width, int height, uint32_t mode = RT_MODE_COMPAT,
                   uint32_t spp = 1)
        : KernelRenderer(width, height, mode, spp) {
        setGraphicsResource(graphics_resource);
    }
    explicit KernelRenderer(const rt_config& cfg) { check(rt_create(&cfg, &r_)); }
    // One process, several GPUs (rt_create_multi): every render()
    // draws the frame across `devices` (tiles round-robin, slabs to devices[0]
    // over RCCL or peer copies, one unpack); every other method is unchanged.
    // The Displayer (src/window/displayer.cpp:28) only swaps this constructor in.
    KernelRenderer(const rt_config& cfg, const std::vector<int>& devices,
                   uint32_t transport = RT_TRANSPORT_AUTO) {
        check(rt_create_multi(&cfg, devices.data(), static_cast<uint32_t>(devices.size()), transport,
                              &r_));
    }
    rt_multi_info multiInfo() const {
        rt_multi_info i;
        check(rt_get_multi_info(r_, &i), r_);
        return i;
    }
    ~KernelRenderer() { rt_destroy(r_); }
    KernelRenderer(const KernelRenderer&) = delete;
    KernelRenderer& operator=(const KernelRenderer&) = delete;

    // render() (src/renderer.cu:143-153): dev_rgba8 = mapped PBO pointer.
    void render(void* dev_rgba8 = nullptr, void* stream = nullptr, rt_stats* stats = nullptr) {
        check(rt_render(r_, dev_rgba8, stream, stats), r_);
    }
    // the reference assigns renderer->cudaResource after re-registering the
    // resized PBO (src/window/displayer.cpp:61-70)
    void setGraphicsResource(void* graphics_resource) {
        check(rt_bind_graphics_resource(r_, graphics_resource), r_);
    }
    // any toolkit's display buffer: render() maps, fills and unmaps it per
    // frame through `ops` (rt_bind_display; nullptr unbinds)
    void setDisplay(const rt_display_ops* ops, void* user) { check(rt_bind_display(r_, ops, user), r_); }
    // resize(int, int) (src/renderer.cu:155-187)
    void resize(int width, int height) {
        check(rt_resize(r_, static_cast<uint32_t>(width), static_cast<uint32_t>(height)), r_);
    }
    // setPosition(glm::mat4) (src/renderer.cu:111-113): pass glm::value_ptr(pose)
    void setPosition(const float* pose_colmajor16) { check(rt_set_pose(r_, pose_colmajor16), r_); }
    // setIntrinsic(glm::mat3) (src/renderer.cu:115-117): pass glm::value_ptr(K)
    void setIntrinsic(const float* K_colmajor9) { check(rt_set_intrinsic(r_, K_colmajor9), r_); }
    // setOctree(glm::vec3 min, glm::vec3 max, float resolution) (include/renderer.cuh:35)
    void setOctree(const float* min3, const float* max3, float resolution) {
        check(rt_set_octree(r_, min3, max3, resolution), r_);
    }
    // new: spheres (cx, cy, cz, r) x n, optional RGBA8 albedo
    void setScene(const std::vector<float>& spheres, const std::vector<uint32_t>& albedo = {},
                  const rt_octree_params* oct = nullptr) {
        const uint32_t n = static_cast<uint32_t>(spheres.size() / 4);
        check(rt_set_scene(r_, spheres.data(), albedo.empty() ? nullptr : albedo.data(), n, oct),
              r_);
    }
    // new: sphere list already in device memory (built into an octree on the GPU)
    void setSceneDevice(const void* dev_spheres, uint32_t n, const void* dev_albedo = nullptr,
                        const rt_octree_params* oct = nullptr, void* stream = nullptr) {
        check(rt_set_scene_device(r_, dev_spheres, dev_albedo, n, oct, stream), r_);
    }
    // new: binary sphere file (rt_save_spheres format)
    void setSceneFile(const std::string& path, const rt_octree_params* oct = nullptr) {
        std::vector<float> sp;
        std::vector<uint32_t> al;
        loadSpheres(path, sp, al);
        setScene(sp, al, oct);
    }
    static void loadSpheres(const std::string& path, std::vector<float>& spheres,
                            std::vector<uint32_t>& albedo) {
        uint32_t n = 0;
        check(rt_load_spheres(path.c_str(), nullptr, nullptr, 0, &n));
        spheres.resize(4 * size_t(n));
        albedo.resize(n);
        check(rt_load_spheres(path.c_str(), spheres.data(), albedo.data(), n, &n));
    }
    static void saveSpheres(const std::string& path, const std::vector<float>& spheres,
                            const std::vector<uint32_t>& albedo = {}) {
        check(rt_save_spheres(path.c_str(), spheres.data(), albedo.empty() ? nullptr : albedo.data(),
                              static_cast<uint32_t>(spheres.size() / 4)));
    }
    // multi-GPU: render only the listed 64x64 tiles into a packed device slab
    // (rt_render_tiles), and scatter packed slabs into a frame (rt_unpack_tiles)
    void renderTiles(const std::vector<uint32_t>& ids, uint32_t tile_size, void* dev_packed,
                     void* stream = nullptr, rt_stats* stats = nullptr) {
        check(rt_render_tiles(r_, ids.data(), static_cast<uint32_t>(ids.size()), tile_size,
                              dev_packed, stream, stats),
              r_);
    }
    void unpackTiles(const void* dev_packed, const std::vector<uint32_t>& ids, uint32_t tile_size,
                     void* dev_rgba8 = nullptr, void* stream = nullptr) {
        check(rt_unpack_tiles(r_, dev_packed, ids.data(), static_cast<uint32_t>(ids.size()),
                              tile_size, dev_rgba8, stream),
              r_);
    }
    rt_scene_info sceneInfo() const {
        rt_scene_info i;
        check(rt_get_scene_info(r_, &i), r_);
        return i;
    }
    void readback(uint8_t* host_rgba8, float* host_rgba32f = nullptr) {
        check(rt_readback(r_, host_rgba8, host_rgba32f), r_);
    }
    void synchronize() { check(rt_synchronize(r_), r_); }
    rt_renderer* handle() { return r_; }

private:
    rt_renderer* r_ = nullptr;
};

}  // namespace rtamd
