// Compile check of the GL interop host surface (include/rt_gl.hpp): what the
// reference's Displayer does with its PBO (src/window/displayer.cpp:13-17,
// 51-53, 61-70), written against this repo's headers.  Built, not run: it
// needs a GL context.
#include <GL/gl.h>

#include "rt_gl.hpp"

void display_frame(unsigned int pbo, int w, int h, const float* pose) {
    rtamd::GlPbo reg(pbo);                                   // cudaGraphicsGLRegisterBuffer
    rtamd::KernelRenderer r(reg.resource(), w, h, RT_MODE_SCENE, 64);
    r.setPosition(pose);                                     // Displayer::processInput
    r.render();                                              // map -> render -> unmap
    reg.reset(pbo);                                          // after a window resize
    r.setGraphicsResource(reg.resource());                   // renderer->cudaResource = ...
    r.resize(w, h);
    r.render();
}
