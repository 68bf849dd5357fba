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
//          [--progressive] [--panel] [--walk] [--test-poison]
//
// --panel prints the stats panel (rt_camera.hpp StatsPanel: the reference's
// ImGui window numbers plus Mrays/s, spp, GPUs) after every frame; --walk
// moves the camera through the Displayer's controller (W held every frame);
// --progressive accumulates samples while the camera stays put.
//
// --gpus N: one process drives N devices through the C-ABI's
// multi-device handle (rt_create_multi): device k renders the 64x64 tiles
// t = k, k+N, ... into a packed slab, the slabs go to device 0 over RCCL and
// are unpacked there into the frame, two frames in flight.  --same-device puts
// all N renderers on device 0 (a rehearsal of the plan on one GPU; peer-copy
// transport, since RCCL refuses a device twice).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>


#include "../../include/rt_camera.hpp"
#include "../../include/rt_renderer.hpp"

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

// One process, N devices: the C-ABI's multi-device handle
// (rt_create_multi) renders every frame across the devices: tiles
// round-robin, each device's slab to device 0 over RCCL (grouped ncclSend /
// ncclRecv on per-device comm streams; peer copies for a --same-device
// rehearsal), one unpack, two frames in flight.
int run_multi(const rt_config& rc, const float pose[16], int gpus, bool same_device, int frames,
              const std::string& out, int W, int H, int spp, int depth, long n,
              const std::string& scene_in) {
    const int ndev = rt_device_count();
    if (ndev < 1) throw rtamd::Error(RT_E_HIP, "no HIP device");
    if (!same_device && ndev < gpus) throw rtamd::Error(RT_E_INVALID, "fewer devices than --gpus");
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
    std::vector<int> devs(gpus);
    for (int k = 0; k < gpus; ++k) devs[k] = same_device ? 0 : k;
    rtamd::KernelRenderer r(rc, devs);
    r.resize(W, H);
    r.setPosition(pose);
    r.setScene(sp, al, &p);
    const rt_multi_info mi = r.multiInfo();
    rt_stats st{};
    r.render(nullptr, nullptr, &st);  // counted frame (devices one after another)
    const uint64_t rays = st.primary_rays + st.shadow_rays;
    r.synchronize();
    // timed: frames back to back, two in flight, one wait at the end
    const int timed = frames > 0 ? frames : 1;
    auto t0 = std::chrono::steady_clock::now();
    for (int f = 0; f < timed; ++f) {
        r.setPosition(pose);  // the Displayer sets the pose every frame
        r.render();
    }
    r.synchronize();
    const double ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / timed;
    printf("%d devices (%s, transport %s): %dx%d spp %d: %.3f ms/frame over %d frames "
           "(tiles + %s gather + unpack, 2 in flight), %llu rays, %.1f Mrays/s\n",
           gpus, same_device ? "all on device 0" : "devices 0..N-1",
           mi.transport == RT_TRANSPORT_RCCL ? "rccl" : "peer", W, H, spp, ms, timed,
           mi.transport == RT_TRANSPORT_RCCL ? "RCCL" : "peer-copy", (unsigned long long)rays,
           rays / (ms * 1e3));
    if (!out.empty()) {
        std::vector<uint8_t> img((size_t)W * H * 4);
        r.readback(img.data());
        return write_ppm(out, img, W, H);
    }
    return 0;
}

int main(int argc, char** argv) {
    std::string cfg = "c2", out, scene_in, scene_out;
    bool host_build = false, same_device = false, progressive = false, panel = false,
         walk = false, poison = false;
    int gpus = 1;
    bool multi = false;  // --gpus given (even 1: a 1-device RCCL communicator)
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
        else if (!strcmp(argv[i], "--gpus")) gpus = atoi(next("--gpus")), multi = true;
        else if (!strcmp(argv[i], "--same-device")) same_device = true;
        else if (!strcmp(argv[i], "--progressive")) progressive = true;
        else if (!strcmp(argv[i], "--panel")) panel = true;
        else if (!strcmp(argv[i], "--walk")) walk = true;
        else if (!strcmp(argv[i], "--test-poison")) poison = true;  // RT_FLAG_TEST_POISON (tests)
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
        if (poison) rc.flags |= RT_FLAG_TEST_POISON;
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
        if (multi) {
            if (gpus < 1 || gpus > RT_MAX_DEVICES) throw rtamd::Error(RT_E_INVALID, "--gpus must be 1..16");
            if (!scene) throw rtamd::Error(RT_E_INVALID, "--gpus needs a scene config");
            return run_multi(rc, pose, gpus, same_device, frames, out, W, H, spp, depth, n,
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
