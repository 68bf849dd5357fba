// Test harness: drive rtamd::CameraController (include/rt_camera.hpp) with a
// scripted input sequence and print every pose, for tests/test_controls.py to
// compare with the Python mirror.  Input lines on stdin:
//   k <w> <a> <s> <d> <space> <shift>     one processInput frame
//   b <right> <press> <x> <y>             mouseButton
//   m <x> <y>                             mouseMove
#include <stdio.h>

#include "rt_camera.hpp"

int main() {
    rtamd::CameraController c;
    char op;
    while (scanf(" %c", &op) == 1) {
        if (op == 'k') {
            int w, a, s, d, sp, sh;
            if (scanf("%d %d %d %d %d %d", &w, &a, &s, &d, &sp, &sh) != 6) return 2;
            rtamd::Keys k;
            k.w = w; k.a = a; k.s = s; k.d = d; k.space = sp; k.shift = sh;
            float p[16];
            c.processInput(k, p);
            for (int i = 0; i < 16; ++i) printf("%.9g%c", p[i], i == 15 ? '\n' : ' ');
        } else if (op == 'b') {
            int right, press;
            double x, y;
            if (scanf("%d %d %lf %lf", &right, &press, &x, &y) != 4) return 2;
            c.mouseButton(right, press, x, y);
        } else if (op == 'm') {
            double x, y;
            if (scanf("%lf %lf", &x, &y) != 2) return 2;
            c.mouseMove(x, y);
        }
    }
    return 0;
}
