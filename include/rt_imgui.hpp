// rt_imgui.hpp — the Displayer's ImGui panel over the C-ABI.
//
// The reference draws one ImGui window per frame, "ui window"
// (src/window/window.cpp:137-150): elapsed time, FPS and frame count, and three
// drag widgets that edit the Displayer's camera in place (position step 0.01,
// yaw step 0.5, pitch step 0.5 clamped to +-89).  Its frame order
// (window.cpp:98-106) is processInput -> display -> panel, so an edit made in
// frame k reaches the renderer through the pose that processInput pushes in
// frame k+1 (include/window/displayer.h:42-53, rt_set_pose here).
//
// drawStatsPanel() is that window over rtamd::StatsPanel and
// rtamd::CameraController, with the renderer's own numbers added (Mrays/s,
// samples per pixel in the image, GPUs).  It needs the application's ImGui
// (the reference vendors imgui/ and builds it with its GL/GLFW backends);
// include imgui.h before this header or let it be found on the include path.
#pragma once
#include "imgui.h"
#include "rt_camera.hpp"

namespace rtamd {

// Screen rectangles {x0, y0, x1, y1} of the panel's edit widgets in the frame
// just drawn, for input automation (tests, scripted camera paths).
struct PanelItems {
    float pos[4] = {0, 0, 0, 0};
    float yaw[4] = {0, 0, 0, 0};
    float pitch[4] = {0, 0, 0, 0};
};

// One frame of the panel; returns true when an edit changed the camera.
inline bool drawStatsPanel(const StatsPanel& p, CameraController& cam,
                           PanelItems* items = nullptr, const char* title = "ui window") {
    auto rect = [](float r[4]) {
        const ImVec2 a = ImGui::GetItemRectMin(), b = ImGui::GetItemRectMax();
        r[0] = a.x;
        r[1] = a.y;
        r[2] = b.x;
        r[3] = b.y;
    };
    bool changed = false;
    if (ImGui::Begin(title)) {
        // window.cpp:140-142 (elapsedTime and FPS are doubles, n_frames an int)
        ImGui::Text("Elapsed Time %f", p.elapsed_s);
        ImGui::Text("FPS %f", p.fps);
        ImGui::Text("frames %d", static_cast<int>(p.frames));
        // the renderer's numbers (rt_stats)
        ImGui::Text("Mrays/s %.1f", p.mrays_s);
        ImGui::Text("spp %u", p.spp);
        ImGui::Text("GPUs %d", p.gpus);
        // window.cpp:143-145: live camera edits
        changed |= ImGui::DragFloat3("camera pos", cam.pos, 0.01f);
        if (items) rect(items->pos);
        changed |= ImGui::DragFloat("camera yaw", &cam.yaw, 0.5f);
        if (items) rect(items->yaw);
        changed |= ImGui::DragFloat("camera pitch", &cam.pitch, 0.5f, -89.0f, 89.0f);
        if (items) rect(items->pitch);
    }
    ImGui::End();
    return changed;
}

}  // namespace rtamd
