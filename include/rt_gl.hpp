// rt_gl.hpp — GL pixel-buffer interop for the C++ host surface.
//
// The reference's Displayer creates a GL_PIXEL_UNPACK_BUFFER of W*H*4 bytes and
// registers it with CUDA (src/window/displayer.cpp:13-17), re-registering it
// after a resize (:61-70).  rtamd::GlPbo is that registration on ROCm
// (hipGraphicsGLRegisterBuffer), RAII-owned; hand `resource()` to
// KernelRenderer (ctor or setGraphicsResource) and every render() maps,
// fills and unmaps the PBO, which the Displayer then draws with
// glTexSubImage2D (:53).  Needs a current GL context on the calling thread.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_gl_interop.h>

#include "rt_renderer.hpp"

namespace rtamd {

class GlPbo {
public:
    GlPbo() = default;
    explicit GlPbo(unsigned int gl_buffer) { reset(gl_buffer); }
    ~GlPbo() { release(); }
    GlPbo(const GlPbo&) = delete;
    GlPbo& operator=(const GlPbo&) = delete;

    // (Re-)register a GL buffer object; the previous registration is dropped.
    void reset(unsigned int gl_buffer) {
        release();
        hipError_t e = hipGraphicsGLRegisterBuffer(&res_, gl_buffer,
                                                   hipGraphicsRegisterFlagsWriteDiscard);
        if (e != hipSuccess) {
            res_ = nullptr;
            throw Error(RT_E_HIP, std::string("hipGraphicsGLRegisterBuffer: ") + hipGetErrorString(e));
        }
    }
    void release() {
        if (res_) (void)hipGraphicsUnregisterResource(res_);
        res_ = nullptr;
    }
    void* resource() const { return res_; }

private:
    hipGraphicsResource_t res_ = nullptr;
};

}  // namespace rtamd
