// rt_cli — headless native driver over the C++ host surface (rt_renderer.hpp).
//
// Plays the reference's main.cpp / Window / Displayer loop without a window
// (main.cpp:4-13, src/window/window.cpp:98-108): builds a renderer, sets the
// Displayer's pose each frame, renders, and optionally writes a PPM.  Used by
// tests/test_native_cli.py and for rocprof runs without Python.
//
//   rt_cli [--config c1|c2|c3|c4|c5] [--width W --height H --spp S --spheres N
//           --depth D] [--frames F] [--out image.ppm] [--scene in.rtsph]
//          [--save-scene out.rtsph] [--host-build] [--gpus N [--same-device]]
//          [--progressive] [--panel] [--walk]
//
// --panel prints the stats panel (rt_camera.hpp StatsPanel: the reference's
// ImGui window numbers plus Mrays/s, spp, GPUs) after every frame; --walk
// moves the camera through the Displayer's controller (W held every frame);
// --progressive accumulates samples while the camera stays put.
//
// --gpus N: one process drives N devices: renderer k renders
// the 64x64 tiles t = k, k+N, ... into a packed slab on device k; the slabs
// are copied peer-to-peer (xGMI) to device 0 and unpacked there into the
// frame.  --same-device puts all N renderers on device 0 (a logic rehearsal
// on one GPU).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include <memory>

#include "../../include/rt_camera.hpp"
#include "../../include/rt_renderer.hpp"

namespace {

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) throw rtamd::Error(RT_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

int write_ppm(const std::string& out, const std::vector<uint8_t>& img, int W, int H) {
    FILE* f = fopen(out.c_str(), "wb");
    if (!f) {
        fprintf(stderr, "cannot write %s\n", out.c_str());
        return 1;
    }
    fprintf(f, "P6\n%d %d\n255\n", W, H);
    for (size_t i = 0; i < (size_t)W * H; ++i) fwrite(&img[4 * i], 1, 3, f);
    fclose(f);
    return 0;
}

// One process, N devices: renderer 0 (already set up) plus N-1 more with the
// same scene; tiles interleaved over renderers; peer copies to device 0.
int run_multi(rtamd::KernelRenderer& r0, const rt_config& rc, const float pose[16], int gpus,
              bool same_device, int frames, const std::string& out, int W, int H, int spp,
              int depth, long n, const std::string& scene_in) {
    const int ndev = rt_device_count();
    if (ndev < 1) throw rtamd::Error(RT_E_HIP, "no HIP device");
    if (!same_device && ndev < gpus) throw rtamd::Error(RT_E_INVALID, "fewer devices than --gpus");
    const uint32_t ts = 64, tx = (W + ts - 1) / ts, ty = (H + ts - 1) / ts, T = tx * ty;
    std::vector<float> sp;
    std::vector<uint32_t> al;
    if (!scene_in.empty()) {
        rtamd::KernelRenderer::loadSpheres(scene_in, sp, al);
    } else {
        sp.resize(4 * (size_t)n);
        al.resize((size_t)n);
        rtamd::check(rt_generate_spheres((uint32_t)n, 0x2545F491u, sp.data(), al.data()));
    }
    rt_octree_params p;
    rt_octree_params_default(&p);
    p.max_depth = (uint32_t)depth;
    std::vector<std::unique_ptr<rtamd::KernelRenderer>> more;
    std::vector<rtamd::KernelRenderer*> rs{&r0};
    std::vector<int> dev{0};  // renderer 0 runs on the current device (0)
    for (int k = 1; k < gpus; ++k) {
        rt_config c = rc;
        c.device = same_device ? 0 : k;
        more.emplace_back(new rtamd::KernelRenderer(c));
        more.back()->resize(W, H);
        more.back()->setPosition(pose);
        more.back()->setScene(sp, al, &p);
        rs.push_back(more.back().get());
        dev.push_back(c.device);
    }
    std::vector<std::vector<uint32_t>> ids(gpus);
    for (uint32_t t = 0; t < T; ++t) ids[t % gpus].push_back(t);
    const size_t slab_bytes = ids[0].size() * ts * ts * 4;
    std::vector<void*> slab(gpus, nullptr), on0(gpus, nullptr);
    for (int k = 0; k < gpus; ++k) {
        hip_check(hipSetDevice(dev[k]), "hipSetDevice");
        hip_check(hipMalloc(&slab[k], slab_bytes), "hipMalloc slab");
        if (k && dev[k] != dev[0]) {
            hip_check(hipSetDevice(dev[0]), "hipSetDevice");
            hip_check(hipMalloc(&on0[k], slab_bytes), "hipMalloc gather");
            int can = 0;
            hip_check(hipDeviceCanAccessPeer(&can, dev[0], dev[k]), "hipDeviceCanAccessPeer");
            if (can) (void)hipDeviceEnablePeerAccess(dev[k], 0);
        } else {
            on0[k] = slab[k];
        }
    }
    double best = 1e30, best_kernel = 0;
    uint64_t rays = 0;
    for (int f = 0; f < frames; ++f) {
        for (auto* r : rs) r->setPosition(pose);
        auto t0 = std::chrono::steady_clock::now();
        std::vector<rt_stats> st(gpus);
        for (int k = 0; k < gpus; ++k) rs[k]->renderTiles(ids[k], ts, slab[k], nullptr, nullptr);
        for (int k = 0; k < gpus; ++k) rs[k]->synchronize();
        for (int k = 1; k < gpus; ++k)
            if (on0[k] != slab[k])
                hip_check(hipMemcpyPeer(on0[k], dev[0], slab[k], dev[k], ids[k].size() * ts * ts * 4),
                          "hipMemcpyPeer");
        for (int k = 0; k < gpus; ++k) rs[0]->unpackTiles(on0[k], ids[k], ts);
        rs[0]->synchronize();
        auto t1 = std::chrono::steady_clock::now();
        best = std::min(best, std::chrono::duration<double, std::milli>(t1 - t0).count());
        if (f == frames - 1) {  // a counted frame: per-renderer kernel time and rays
            double mx = 0;
            rays = 0;
            for (int k = 0; k < gpus; ++k) {
                rs[k]->renderTiles(ids[k], ts, slab[k], nullptr, &st[k]);
                mx = std::max(mx, (double)st[k].ms);
                rays += st[k].primary_rays + st[k].shadow_rays;
            }
            best_kernel = mx;
        }
    }
    printf("%d renderers on %s: %dx%d spp %d: frame %.3f ms (tiles + peer gather + unpack), "
           "slowest renderer kernel %.3f ms, %llu rays, %.1f Mrays/s\n",
           gpus, same_device ? "device 0" : "devices 0..N-1", W, H, spp, best, best_kernel,
           (unsigned long long)rays, rays / (best * 1e3));
    int rc_out = 0;
    if (!out.empty()) {
        std::vector<uint8_t> img((size_t)W * H * 4);
        rs[0]->readback(img.data());
        rc_out = write_ppm(out, img, W, H);
    }
    for (int k = 0; k < gpus; ++k) {
        (void)hipSetDevice(dev[k]);
        (void)hipFree(slab[k]);
        if (on0[k] != slab[k]) {
            (void)hipSetDevice(dev[0]);
            (void)hipFree(on0[k]);
        }
    }
    return rc_out;
}

int main(int argc, char** argv) {
    std::string cfg = "c2", out, scene_in, scene_out;
    bool host_build = false, same_device = false, progressive = false, panel = false,
         walk = false;
    int gpus = 1;
    int W = 0, H = 0, spp = 0, frames = 3;
    long n = -1;
    int depth = 0;
    for (int i = 1; i < argc; ++i) {
        auto next = [&](const char* what) -> const char* {
            if (i + 1 >= argc) {
                fprintf(stderr, "missing value for %s\n", what);
                exit(2);
            }
            return argv[++i];
        };
        if (!strcmp(argv[i], "--config")) cfg = next("--config");
        else if (!strcmp(argv[i], "--width")) W = atoi(next("--width"));
        else if (!strcmp(argv[i], "--height")) H = atoi(next("--height"));
        else if (!strcmp(argv[i], "--spp")) spp = atoi(next("--spp"));
        else if (!strcmp(argv[i], "--spheres")) n = atol(next("--spheres"));
        else if (!strcmp(argv[i], "--depth")) depth = atoi(next("--depth"));
        else if (!strcmp(argv[i], "--frames")) frames = atoi(next("--frames"));
        else if (!strcmp(argv[i], "--out")) out = next("--out");
        else if (!strcmp(argv[i], "--scene")) scene_in = next("--scene");
        else if (!strcmp(argv[i], "--save-scene")) scene_out = next("--save-scene");
        else if (!strcmp(argv[i], "--host-build")) host_build = true;
        else if (!strcmp(argv[i], "--gpus")) gpus = atoi(next("--gpus"));
        else if (!strcmp(argv[i], "--same-device")) same_device = true;
        else if (!strcmp(argv[i], "--progressive")) progressive = true;
        else if (!strcmp(argv[i], "--panel")) panel = true;
        else if (!strcmp(argv[i], "--walk")) walk = true;
        else {
            fprintf(stderr, "unknown argument %s\n", argv[i]);
            return 2;
        }
    }
    struct C { const char* name; int w, h, spp; long n; int depth; uint32_t mode; };
    const C table[] = {{"c1", 256, 256, 1, 0, 7, RT_MODE_COMPAT},
                       {"c2", 1920, 1080, 1, 1000, 7, RT_MODE_SCENE},
                       {"c3", 1920, 1080, 64, 100000, 7, RT_MODE_SCENE},
                       {"c4", 3840, 2160, 64, 100000, 7, RT_MODE_SCENE},
                       {"c5", 1920, 1080, 256, 1000000, 12, RT_MODE_SCENE}};
    const C* c = nullptr;
    for (const C& e : table)
        if (cfg == e.name) c = &e;
    if (!c) {
        fprintf(stderr, "unknown config %s\n", cfg.c_str());
        return 2;
    }
    W = W ? W : c->w;
    H = H ? H : c->h;
    spp = spp ? spp : c->spp;
    n = n >= 0 ? n : c->n;
    depth = depth ? depth : c->depth;
    try {
        rt_config rc;
        rt_config_default(&rc);
        rc.width = W;
        rc.height = H;
        rc.spp = spp;
        rc.mode = c->mode;
        if (host_build) rc.flags |= RT_FLAG_HOST_BUILD;
        if (progressive) rc.flags |= RT_FLAG_PROGRESSIVE;
        rtamd::KernelRenderer r(rc);
        r.resize(W, H);
        // Displayer default orientation (include/window/displayer.h:47-52):
        // rot = diag(1,-1,-1); compat at (0,0,3), scene at (0.64,0.64,2.2)
        const bool scene = c->mode == RT_MODE_SCENE;
        const float pose[16] = {1, 0, 0, 0, 0, -1, 0, 0, 0, 0, -1, 0,
                                scene ? 0.64f : 0.f, scene ? 0.64f : 0.f, scene ? 2.2f : 3.f, 1};
        if (scene) {
            std::vector<float> sp;
            std::vector<uint32_t> al;
            if (!scene_in.empty()) {
                rtamd::KernelRenderer::loadSpheres(scene_in, sp, al);
            } else {
                sp.resize(4 * (size_t)n);
                al.resize((size_t)n);
                rtamd::check(rt_generate_spheres((uint32_t)n, 0x2545F491u, sp.data(), al.data()));
            }
            if (!scene_out.empty()) rtamd::KernelRenderer::saveSpheres(scene_out, sp, al);
            rt_octree_params p;
            rt_octree_params_default(&p);
            p.max_depth = (uint32_t)depth;
            r.setScene(sp, al, &p);
            const rt_scene_info si = r.sceneInfo();
            printf("scene: %u spheres, %u nodes, %u leaves, %u refs, depth %u/%u, %s build %.2f ms\n",
                   si.n_spheres, si.n_nodes, si.n_leaves, si.n_prim_refs, si.depth_reached,
                   si.max_depth, si.builder == RT_BUILDER_HOST ? "host" : "device", si.build_ms);
        }
        if (gpus > 1) {
            if (!scene) throw rtamd::Error(RT_E_INVALID, "--gpus needs a scene config");
            return run_multi(r, rc, pose, gpus, same_device, frames, out, W, H, spp, depth, n,
                             scene_in);
        }
        rt_stats st{};
        double best = 1e30;
        // the Displayer's controller, starting at this config's camera position
        rtamd::CameraController cam;
        for (int i = 0; i < 3; ++i) cam.pos[i] = pose[12 + i];
        rtamd::StatsPanel stats_panel;
        for (int f = 0; f < frames; ++f) {
            auto t0 = std::chrono::steady_clock::now();
            if (walk) {
                rtamd::Keys k;
                k.w = true;
                cam.processInput(k, r);  // like Displayer::processInput, every frame
            } else {
                r.setPosition(pose);
            }
            r.render(nullptr, nullptr, &st);
            auto t1 = std::chrono::steady_clock::now();
            const double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
            best = std::min(best, ms);
            if (panel) {
                stats_panel.update(ms, st, 1);
                printf("-- frame %d --\n%s", f, stats_panel.text().c_str());
            }
        }
        const double rays = (double)st.primary_rays + (double)st.shadow_rays;
        printf("%s %dx%d spp %d: kernel %.3f ms, wall %.3f ms, %.0f rays (%llu primary + %llu shadow), "
               "%.1f Mrays/s\n",
               c->name, W, H, spp, st.ms, best, rays, (unsigned long long)st.primary_rays,
               (unsigned long long)st.shadow_rays, rays / (st.ms * 1e3));
        if (!out.empty()) {
            std::vector<uint8_t> img((size_t)W * H * 4);
            r.readback(img.data());
            FILE* f = fopen(out.c_str(), "wb");
            if (!f) {
                fprintf(stderr, "cannot write %s\n", out.c_str());
                return 1;
            }
            fprintf(f, "P6\n%d %d\n255\n", W, H);
            for (size_t i = 0; i < (size_t)W * H; ++i) fwrite(&img[4 * i], 1, 3, f);
            fclose(f);
        }
    } catch (const rtamd::Error& e) {
        fprintf(stderr, "rt_cli: %s (code %d)\n", e.what(), e.code);
        return 1;
    }
    return 0;
}
