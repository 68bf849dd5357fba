// rt_cli — headless native driver over the C++ host surface (rt_renderer.hpp).
//
// Plays the reference's main.cpp / Window / Displayer loop without a window
// (main.cpp:4-13, src/window/window.cpp:98-108): builds a renderer, sets the
// Displayer's pose each frame, renders, and optionally writes a PPM.  Used by
// tests/test_native_cli.py and for rocprof runs without Python.
//
//   rt_cli [--config c1|c2|c3|c5] [--width W --height H --spp S --spheres N
//           --depth D] [--frames F] [--out image.ppm] [--scene in.rtsph]
//          [--save-scene out.rtsph] [--host-build]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "../../include/rt_renderer.hpp"

int main(int argc, char** argv) {
    std::string cfg = "c2", out, scene_in, scene_out;
    bool host_build = false;
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
        rt_stats st{};
        double best = 1e30;
        for (int f = 0; f < frames; ++f) {
            r.setPosition(pose);  // every frame, like Displayer::processInput
            auto t0 = std::chrono::steady_clock::now();
            r.render(nullptr, nullptr, &st);
            auto t1 = std::chrono::steady_clock::now();
            best = std::min(best, std::chrono::duration<double, std::milli>(t1 - t0).count());
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
