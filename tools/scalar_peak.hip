// Microbenchmark: scalar-pipeline issue rate of one MI355X CU (SALU
// arithmetic and not-taken branches), to price the scalar roof of
// scene_kernel (bench.py roofline "scalar_issue").  Register-only
// instructions, no memory traffic.  Every CU runs 32 waves; each wave issues
// ITER x 64 independent s_add_u32 (or s_cbranch_scc1 not taken).
//   hipcc --offload-arch=gfx950 -O3 -o tools/scalar_peak tools/scalar_peak.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITER 4096

__global__ void __launch_bounds__(256) salu_kernel(unsigned* out, unsigned seed) {
    const long long t0 = clock64();
    unsigned a = seed, b = seed + 1, c = seed + 2, d = seed + 3;
    unsigned e = seed + 4, f = seed + 5, g = seed + 6, h = seed + 7;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            asm volatile(
                "s_add_u32 %0, %0, 1\n s_add_u32 %1, %1, 1\n s_add_u32 %2, %2, 1\n"
                "s_add_u32 %3, %3, 1\n s_add_u32 %4, %4, 1\n s_add_u32 %5, %5, 1\n"
                "s_add_u32 %6, %6, 1\n s_add_u32 %7, %7, 1\n"
                : "+s"(a), "+s"(b), "+s"(c), "+s"(d), "+s"(e), "+s"(f), "+s"(g), "+s"(h)
                :
                : "scc");
        }
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) out[blockIdx.x] = (unsigned)(t1 - t0) + ((a ^ b ^ c ^ d ^ e ^ f ^ g ^ h) == 0x12345u);
}

__global__ void __launch_bounds__(256) branch_kernel(unsigned* out, unsigned seed) {
    const long long t0 = clock64();
    unsigned a = seed;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            // scc = 0 after s_cmp_eq (a never equals 0xFFFFFFFF here): not taken
            asm volatile(
                "s_cmp_eq_u32 %0, -1\n"
                "s_cbranch_scc1 1f\n s_cbranch_scc1 1f\n s_cbranch_scc1 1f\n s_cbranch_scc1 1f\n"
                "s_cbranch_scc1 1f\n s_cbranch_scc1 1f\n s_cbranch_scc1 1f\n"
                "1:\n"
                : "+s"(a)
                :
                : "scc");
        }
        a += 1;
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) out[blockIdx.x] = (unsigned)(t1 - t0) + (a == 0x12345u);
}

__global__ void __launch_bounds__(256) valu_kernel(unsigned* out, unsigned seed_u) {
    const long long t0 = clock64();
    const float seed = (float)seed_u;
    float a = seed + threadIdx.x, b = a + 1, c = a + 2, d = a + 3;
    float e = a + 4, f = a + 5, g = a + 6, h = a + 7;
    for (int i = 0; i < ITER; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            asm volatile(
                "v_fma_f32 %0, %0, %0, 1.0\n v_fma_f32 %1, %1, %1, 1.0\n v_fma_f32 %2, %2, %2, 1.0\n"
                "v_fma_f32 %3, %3, %3, 1.0\n v_fma_f32 %4, %4, %4, 1.0\n v_fma_f32 %5, %5, %5, 1.0\n"
                "v_fma_f32 %6, %6, %6, 1.0\n v_fma_f32 %7, %7, %7, 1.0\n"
                : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g), "+v"(h));
        }
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) out[blockIdx.x] = (unsigned)(t1 - t0) + ((a + b + c + d + e + f + g + h) == 1234.5f);
}

static unsigned* g_host;
static double g_cycles;
template <typename K, typename T>
static float run(K k, T* buf, int blocks) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, (T)1);  // warm-up
    hipEventRecord(e0);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, buf, (T)1);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) printf("launch error: %s\n", hipGetErrorString(err));
    hipMemcpy(g_host, buf, blocks * 4, hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < blocks; ++i) s += g_host[i];
    g_cycles = s / blocks;  // shader cycles of one workgroup (all 32 waves of a CU run together)
    return ms;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const int blocks = cus * 8;  // 8 x 4 waves = 32 waves per CU
    const double clk = p.clockRate * 1e3;  // Hz (max engine clock)
    void* buf;
    hipMalloc(&buf, blocks * 4);
    g_host = new unsigned[blocks];
    const double waves = blocks * 4.0, per_wave = double(ITER) * 64;
    // per CU: 32 waves; rates per shader cycle from each workgroup's own
    // s_memtime span (the 8 workgroups of a CU run concurrently)
    float ms = run(salu_kernel, (unsigned*)buf, blocks);
    const double salu_cyc = g_cycles, salu_ms = ms;
    ms = run(branch_kernel, (unsigned*)buf, blocks);
    const double br_cyc = g_cycles, br_ms = ms;
    ms = run(valu_kernel, (unsigned*)buf, blocks);
    const double va_cyc = g_cycles, va_ms = ms;
    const double per_cu_waves = 32.0;
    printf("{\"cus\": %d, \"max_clock_ghz\": %.3f, "
           "\"salu\": {\"ms\": %.3f, \"wg_cycles\": %.0f, \"per_cu_cycle\": %.3f, \"clock_ghz\": %.3f}, "
           "\"scalar_cmp_branch\": {\"ms\": %.3f, \"wg_cycles\": %.0f, \"per_cu_cycle\": %.3f}, "
           "\"valu\": {\"ms\": %.3f, \"wg_cycles\": %.0f, \"per_simd_cycle\": %.3f}}\n",
           cus, clk / 1e9, salu_ms, salu_cyc, per_cu_waves * per_wave / salu_cyc,
           salu_cyc / (salu_ms * 1e6), br_ms, br_cyc, per_cu_waves * ITER * 64.0 / br_cyc,
           va_ms, va_cyc, per_cu_waves * per_wave / 4.0 / va_cyc);
    hipFree(buf);
    return 0;
}
