// Throughput of v_permlane32_swap against plain VALU (diagnostic for
// DESIGN.md 5.1 "Half-wave loads"): every lane runs N steps of 4 independent
// chains; a step is either 4 swaps (+ the copies the builtin needs) or 4 adds.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int kMode>
__global__ void __launch_bounds__(256) bench(unsigned* out, int n) {
    unsigned a = threadIdx.x, b = a * 3u + 1u, c = a * 5u + 2u, d = a * 7u + 3u;
    for (int i = 0; i < n; ++i) {
        if (kMode == 1) {
            auto ra = __builtin_amdgcn_permlane32_swap(a, a, false, false);
            auto rb = __builtin_amdgcn_permlane32_swap(b, b, false, false);
            auto rc = __builtin_amdgcn_permlane32_swap(c, c, false, false);
            auto rd = __builtin_amdgcn_permlane32_swap(d, d, false, false);
            a = ra[0] + ra[1]; b = rb[0] + rb[1]; c = rc[0] + rc[1]; d = rd[0] + rd[1];
        } else {
            a = a + (a >> 1) + 1u; b = b + (b >> 1) + 1u; c = c + (c >> 1) + 1u; d = d + (d >> 1) + 1u;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d;
}

int main() {
    unsigned* out;
    hipMalloc(&out, 256u * 2048u * 4u);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int n = 4096;
    for (int rep = 0; rep < 2; ++rep) {
        for (int mode = 0; mode < 2; ++mode) {
            hipEventRecord(e0);
            if (mode) hipLaunchKernelGGL(bench<1>, dim3(2048), dim3(256), 0, 0, out, n);
            else hipLaunchKernelGGL(bench<0>, dim3(2048), dim3(256), 0, 0, out, n);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            // 2048 blocks x 4 waves x n steps x (4 swaps or 8 VALU)
            const double waves_steps = 2048.0 * 4.0 * n;
            printf("%s: %.3f ms, %.2f ns per wave-step over the GPU\n",
                   mode ? "permlane32_swap x4 (+4 add)" : "8 VALU (add,shift) x4", ms,
                   ms * 1e6 / waves_steps);
        }
    }
    hipFree(out);
    return 0;
}
