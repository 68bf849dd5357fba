// Headless frames of the Displayer loop with the ImGui panel (include/rt_imgui.hpp),
// built by tests/test_imgui_panel.py against the reference's own ImGui core
// (/root/reference/imgui: imgui.cpp, imgui_draw.cpp, imgui_widgets.cpp,
// imgui_tables.cpp; no GL/GLFW backend).  Test infrastructure.
//
// The C-ABI entry points KernelRenderer reaches are defined here as a
// recording stub (no GPU in the test container): every rt_set_pose call is
// logged, so the test sees exactly what the panel's edits push to the renderer.
//
// Each frame follows src/window/window.cpp:98-106: time update, NewFrame,
// processInput (pose -> rt_set_pose), display (rt_render), the panel, Render.
// Mouse input is injected through io.AddMouse*Event to drag the yaw, pitch and
// position widgets.  Output: one JSON object on stdout.
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "imgui.h"
#include "rt_imgui.hpp"

// ---- recording C-ABI stub -------------------------------------------------------
struct rt_renderer {
    int renders = 0;
};
static std::vector<std::vector<float>> g_poses;
static int g_renders = 0;
static std::string g_clipboard;
extern "C" {
void rt_config_default(rt_config* c) { memset(c, 0, sizeof(*c)); }
int rt_create(const rt_config*, rt_renderer** out) {
    *out = new rt_renderer();
    return RT_OK;
}
int rt_destroy(rt_renderer* r) {
    delete r;
    return RT_OK;
}
int rt_set_pose(rt_renderer*, const float* m) {
    g_poses.emplace_back(m, m + 16);
    return RT_OK;
}
int rt_render(rt_renderer* r, void*, void*, rt_stats*) {
    ++r->renders;
    ++g_renders;
    return RT_OK;
}
const char* rt_last_error(const rt_renderer*) { return ""; }
}

// ---- frames -----------------------------------------------------------------------
namespace {

struct Loop {
    rtamd::KernelRenderer renderer{320, 240, RT_MODE_SCENE, 64};
    rtamd::CameraController cam;
    rtamd::StatsPanel panel;
    rtamd::PanelItems items;
    std::string log;
    int edits = 0;

    void frame(bool capture_text) {
        rt_stats st{};
        st.primary_rays = 320ull * 240 * 64;
        st.shadow_rays = 1000000;
        st.samples_per_pixel = 64;
        st.ms = 2.0f;
        panel.update(16.0, st, 8);  // Window::timeUpdate
        ImGuiIO& io = ImGui::GetIO();
        io.DeltaTime = 1.0f / 60.0f;
        ImGui::NewFrame();
        cam.processInput(rtamd::Keys{}, renderer);  // displayer->processInput
        renderer.render();                          // displayer->display
        // text capture: ImGui's logging, started inside the panel's window, is
        // finished by the panel's own End() and handed to the clipboard hook
        if (capture_text) {
            ImGui::Begin("ui window");
            ImGui::LogToClipboard();
        }
        edits += rtamd::drawStatsPanel(panel, cam, &items) ? 1 : 0;  // renderImGui
        if (capture_text) {
            ImGui::End();
            log = g_clipboard;
        }
        ImGui::Render();
    }
};

void json_str(const std::string& s) {
    putchar('"');
    for (char c : s) {
        if (c == '"' || c == '\\') printf("\\%c", c);
        else if (c == '\n') printf("\\n");
        else if (static_cast<unsigned char>(c) < 0x20) printf("\\u%04x", c);
        else putchar(c);
    }
    putchar('"');
}

void json_floats(const float* v, int n) {
    putchar('[');
    for (int i = 0; i < n; ++i) printf("%s%.9g", i ? ", " : "", v[i]);
    putchar(']');
}

// drag from (x, y) by (dx, dy): hover, press, move, release (one event a frame,
// as ImGui's trickled input queue delivers them)
void drag(Loop& L, float x, float y, float dx, float dy) {
    ImGuiIO& io = ImGui::GetIO();
    io.AddMousePosEvent(x, y);
    L.frame(false);
    io.AddMouseButtonEvent(0, true);
    L.frame(false);
    io.AddMousePosEvent(x + dx, y + dy);
    L.frame(false);
    io.AddMouseButtonEvent(0, false);
    L.frame(false);
    io.AddMousePosEvent(-FLT_MAX, -FLT_MAX);
    L.frame(false);
}

}  // namespace

int main() {
    IMGUI_CHECKVERSION();
    ImGui::CreateContext();
    ImGuiIO& io = ImGui::GetIO();
    io.IniFilename = nullptr;
    io.SetClipboardTextFn = [](void*, const char* t) { g_clipboard = t; };
    io.DisplaySize = ImVec2(1280.0f, 720.0f);
    unsigned char* px = nullptr;
    int tw = 0, th = 0;
    io.Fonts->GetTexDataAsRGBA32(&px, &tw, &th);  // what the GL backend uploads

    Loop L;
    for (int i = 0; i < 3; ++i) L.frame(false);  // window placement and auto-fit settle
    L.frame(true);
    const std::string text0 = L.log;
    const size_t poses_before = g_poses.size();

    // yaw: +40 px at 0.5 per px
    const rtamd::PanelItems it = L.items;
    drag(L, it.yaw[0] + 6.0f, 0.5f * (it.yaw[1] + it.yaw[3]), 40.0f, 0.0f);
    const float yaw_after = L.cam.yaw;
    const std::vector<float> pose_yaw = g_poses.back();
    // pitch: +400 px at 0.5 per px, clamped to 89
    drag(L, L.items.pitch[0] + 6.0f, 0.5f * (L.items.pitch[1] + L.items.pitch[3]), 400.0f, 0.0f);
    const float pitch_after = L.cam.pitch;
    const std::vector<float> pose_pitch = g_poses.back();
    // position x (the first of DragFloat3's three fields): -50 px at 0.01 per px
    drag(L, L.items.pos[0] + 6.0f, 0.5f * (L.items.pos[1] + L.items.pos[3]), -50.0f, 0.0f);
    const std::vector<float> pose_pos = g_poses.back();
    L.frame(true);
    const std::string text1 = L.log;

    printf("{\"imgui\": ");
    json_str(IMGUI_VERSION);
    printf(", \"font_atlas\": [%d, %d], \"text0\": ", tw, th);
    json_str(text0);
    printf(", \"text1\": ");
    json_str(text1);
    printf(", \"yaw\": %.9g, \"pitch\": %.9g, \"pos\": ", yaw_after, pitch_after);
    json_floats(L.cam.pos, 3);
    printf(", \"pose_after_yaw\": ");
    json_floats(pose_yaw.data(), 16);
    printf(", \"pose_after_pitch\": ");
    json_floats(pose_pitch.data(), 16);
    printf(", \"pose_after_pos\": ");
    json_floats(pose_pos.data(), 16);
    printf(", \"set_pose_calls\": %zu, \"set_pose_calls_before_edits\": %zu, \"renders\": %d, "
           "\"edits\": %d, \"frames\": %d, \"yaw_rect\": ",
           g_poses.size(), poses_before, g_renders, L.edits, static_cast<int>(L.panel.frames));
    json_floats(it.yaw, 4);
    printf("}\n");
    ImGui::DestroyContext();
    return 0;
}
