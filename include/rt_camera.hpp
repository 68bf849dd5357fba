// rt_camera.hpp — the Displayer's camera controls and stats panel over the
// C-ABI, without glm, GLFW or ImGui.
//
// CameraController is the reference's input state machine
// (include/window/displayer.h:20-83): WASD moves along the current front/right
// axes, space / shift+space along the camera up axis (0.01 per frame),
// right-drag turns yaw/pitch (0.3 degrees per pixel; yaw wraps to [0, 360],
// pitch clamps to +-89), and every frame the pose
//     front = rotate(yaw, Y) * rotate(pitch, X) * (0, 0, -1)
//     pose  = inverse(lookAt(pos, pos + front, up)) * diag(1, -1, -1, 1)
// is pushed through rt_set_pose (KernelRenderer::setPosition).  The window
// toolkit only has to report key states and mouse events.
//
// StatsPanel holds what the reference's ImGui window shows
// (src/window/window.cpp:137-150, 163-169: elapsed time, FPS, frames), plus
// the renderer's own numbers: Mrays/s, samples per pixel in the image, GPUs.
// A window with ImGui draws text(); a headless driver prints it.
#pragma once
#include <math.h>
#include <stdint.h>
#include <stdio.h>

#include <string>

#include "rt_renderer.hpp"

namespace rtamd {

struct Keys {
    bool w = false, a = false, s = false, d = false, space = false, shift = false;
};

class CameraController {
public:
    static constexpr float kMoveSpeed = 0.01f;  // displayer.h:22
    static constexpr float kTurnSpeed = 0.3f;   // displayer.h:71

    float pos[3] = {0.0f, 0.0f, 3.0f};    // displayer.h:89-94 defaults
    float front[3] = {0.0f, 0.0f, -1.0f};
    float up[3] = {0.0f, 1.0f, 0.0f};
    float yaw = 0.0f, pitch = 0.0f;
    bool control = false;
    float prev_mouse[2] = {0.0f, 0.0f};

    // processInput (displayer.h:20-55): move, then refresh front and the pose.
    void processInput(const Keys& k, float pose_out[16]) {
        if (k.w) axpy(kMoveSpeed, front);
        if (k.s) axpy(-kMoveSpeed, front);
        float nf[3] = {-front[0], -front[1], -front[2]}, right[3], cup[3];
        cross(up, nf, right);
        normalize(right);
        if (k.d) axpy(kMoveSpeed, right);
        if (k.a) axpy(-kMoveSpeed, right);
        cross(nf, right, cup);
        normalize(cup);
        if (k.space) axpy(k.shift ? -kMoveSpeed : kMoveSpeed, cup);
        const float ry = yaw * 0.017453292519943295f, rp = pitch * 0.017453292519943295f;
        // rotate(pitch, X) * (0,0,-1) = (0, sin p, -cos p); then rotate(yaw, Y)
        const float fy = sinf(rp), fz = -cosf(rp);
        front[0] = sinf(ry) * fz;
        front[1] = fy;
        front[2] = cosf(ry) * fz;
        pose(pose_out);
    }
    void processInput(const Keys& k, KernelRenderer& r) {
        float p[16];
        processInput(k, p);
        r.setPosition(p);
    }
    // mouseButton (displayer.h:57-67): the right button starts / ends turning
    void mouseButton(bool right_button, bool press, double x, double y) {
        if (!right_button) return;
        if (press) {
            prev_mouse[0] = static_cast<float>(x);
            prev_mouse[1] = static_cast<float>(y);
            control = true;
        } else {
            control = false;
        }
    }
    // mouseMove (displayer.h:69-83)
    void mouseMove(double x, double y) {
        if (!control) return;
        const float px = static_cast<float>(x), py = static_cast<float>(y);
        yaw -= (px - prev_mouse[0]) * kTurnSpeed;
        pitch -= (py - prev_mouse[1]) * kTurnSpeed;
        if (yaw < 0.0f) yaw += 360.0f;
        if (yaw > 360.0f) yaw -= 360.0f;
        if (pitch > 89.0f) pitch = 89.0f;
        if (pitch < -89.0f) pitch = -89.0f;
        prev_mouse[0] = px;
        prev_mouse[1] = py;
    }
    // inverse(lookAt(pos, pos + front, up)) * diag(1,-1,-1,1), column-major [c*4+r]
    void pose(float m[16]) const {
        float f[3] = {front[0], front[1], front[2]}, s[3], u[3];
        normalize(f);
        cross(f, up, s);
        normalize(s);
        cross(s, f, u);
        for (int i = 0; i < 3; ++i) {
            m[0 * 4 + i] = s[i];
            m[1 * 4 + i] = -u[i];
            m[2 * 4 + i] = f[i];
            m[3 * 4 + i] = pos[i];
        }
        m[3] = m[7] = m[11] = 0.0f;
        m[15] = 1.0f;
    }

private:
    void axpy(float a, const float v[3]) {
        for (int i = 0; i < 3; ++i) pos[i] += a * v[i];
    }
    static void cross(const float a[3], const float b[3], float o[3]) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    }
    static void normalize(float v[3]) {
        const float l = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        for (int i = 0; i < 3; ++i) v[i] /= l;
    }
};

class StatsPanel {
public:
    double elapsed_s = 0.0;   // time since the first frame (window.cpp:165)
    double fps = 0.0;         // 1 / last frame time (window.cpp:166-168)
    uint64_t frames = 0;      // window.cpp:106
    double mrays_s = 0.0;     // rays of the last frame / its device time
    uint32_t spp = 0;         // samples per pixel in the image (progressive: accumulated)
    int gpus = 1;

    // one call per frame: wall time of the frame and the renderer's stats
    void update(double frame_ms, const rt_stats& st, int n_gpus = 1) {
        elapsed_s += frame_ms * 1e-3;
        fps = frame_ms > 0.0 ? 1e3 / frame_ms : 0.0;
        ++frames;
        const double rays = static_cast<double>(st.primary_rays + st.shadow_rays);
        mrays_s = st.ms > 0.0f ? rays / (st.ms * 1e3) : 0.0;
        spp = st.samples_per_pixel;
        gpus = n_gpus;
    }
    std::string text() const {
        char b[256];
        snprintf(b, sizeof(b),
                 "Elapsed Time %f\nFPS %f\nframes %llu\nMrays/s %.1f\nspp %u\nGPUs %d\n",
                 elapsed_s, fps, static_cast<unsigned long long>(frames), mrays_s, spp, gpus);
        return b;
    }
};

}  // namespace rtamd
