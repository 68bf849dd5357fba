// Vector-memory cost per load instruction on gfx950, L1-resident data
// (diagnostic for DESIGN.md 5.1 "What the cost is per" and VERDICT r03 item
// 2): every wave issues N independent loads of W dwords per lane from a 4 KB
// table, in one of four lane patterns:
//   0 uniform : all 64 lanes read the same address (one pixel's samples
//               reading one sphere: the scene kernel's sphere loads)
//   1 strided : lane l reads W dwords at l*W (fully coalesced, 64*W*4 bytes)
//   2 one-lane: only lane 0 is active
//   3 quads   : 4 distinct addresses, 16 lanes each
// plus scalar loads (s_load_dwordx4 / x8) of a uniform address.  Prints ns and
// CU-cycles (at the measured clock) per wave-instruction with 8 waves/SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o vmem_cost vmem_cost.hip && ./vmem_cost
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kTableDw = 1024;  // 4 KB

__device__ __forceinline__ uint32_t vzero() {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));  // an opaque VGPR zero: forces vector addressing
    return z;
}

template <int W, int kPat>
__global__ void __launch_bounds__(256) vload(const uint32_t* __restrict__ t, uint32_t* out, int n,
                                             long long* clk) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t z = vzero();
    uint32_t acc = 0;
    long long c0 = 0;
    if (threadIdx.x == 0 && blockIdx.x == 0) c0 = wall_clock64();
    uint32_t lo = 0;
    if (kPat == 1) lo = lane * W;
    if (kPat == 3) lo = (lane >> 4) * 64u;
#pragma unroll 4
    for (int i = 0; i < n; ++i) {
        // table row: pseudo-random 16-dword-aligned row, the same for every lane
        const uint32_t row = ((static_cast<uint32_t>(i) * 37u) & 15u) * 64u;
        const uint32_t off = (kPat == 1 ? ((row + lo) & (kTableDw - 1)) : (row + lo)) + z;
        if (kPat == 2 && lane != 0) continue;
        if (W == 1) {
            acc ^= t[off];
        } else if (W == 2) {
            const uint2 v = *reinterpret_cast<const uint2*>(t + (off & ~1u));
            acc ^= v.x + v.y;
        } else if (W == 3) {
            const uint3 v = *reinterpret_cast<const uint3*>(t + (off & ~3u));
            acc ^= v.x + v.y + v.z;
        } else {
            const uint4 v = *reinterpret_cast<const uint4*>(t + (off & ~3u));
            acc ^= v.x + v.y + v.z + v.w;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = wall_clock64() - c0;
}

// scalar loads of a uniform address (s_load_dwordx4 / x8)
template <int W>
__global__ void __launch_bounds__(256) sload(const uint32_t* __restrict__ t, uint32_t* out, int n) {
    uint32_t acc = 0;
    for (int i = 0; i < n; ++i) {
        const uint32_t row = __builtin_amdgcn_readfirstlane(((static_cast<uint32_t>(i) * 37u) & 15u) * 64u);
        if (W == 4) {
            const uint4 v = *reinterpret_cast<const uint4*>(t + row);
            acc ^= v.x + v.y + v.z + v.w;
        } else {
            const uint4 v = *reinterpret_cast<const uint4*>(t + row);
            const uint4 u = *reinterpret_cast<const uint4*>(t + row + 4);
            acc ^= v.x + v.y + v.z + v.w + u.x + u.y + u.z + u.w;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc + threadIdx.x;
}

// VALU reference: 4 dependent-free adds per iteration
__global__ void __launch_bounds__(256) valu(uint32_t* out, int n) {
    uint32_t a = threadIdx.x, b = a * 3u, c = a * 5u, d = a * 7u;
    for (int i = 0; i < n; ++i) {
        a = a * 3u + 1u; b = b * 3u + 1u; c = c * 3u + 1u; d = d * 3u + 1u;
    }
    out[blockIdx.x * 256 + threadIdx.x] = a ^ b ^ c ^ d;
}

template <typename F>
static float timed(F f) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    f();  // warm-up
    hipEventRecord(e0);
    f();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    return ms;
}

int main() {
    int cus = 256;
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, 0) == hipSuccess) cus = p.multiProcessorCount;
    const int wg_per_cu = 8;  // 8 waves per SIMD
    const int blocks = cus * wg_per_cu;
    const int n = 8192;
    uint32_t *t, *out;
    long long* clk;
    hipMalloc(&t, kTableDw * 4 + 64);
    hipMemset(t, 1, kTableDw * 4 + 64);
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipMalloc(&clk, 8);
    const double waves_per_cu = wg_per_cu * 4.0;
    // clock: a VALU loop of known cost (4 independent v_mad_u32_u24 / v_mul_lo
    // chains; reported, not assumed)
    const float vms = timed([&] { hipLaunchKernelGGL(valu, dim3(blocks), dim3(256), 0, 0, out, n); });
    printf("{\"cus\": %d, \"waves_per_cu\": %.0f, \"n\": %d, \"valu_loop_ns_per_iter_per_wave\": %.4f}\n",
           cus, waves_per_cu, n, vms * 1e6 / (waves_per_cu * n));
    const char* pats[4] = {"uniform", "strided", "one_lane", "quads"};
#define RUN(W, P)                                                                                \
    {                                                                                            \
        const float ms = timed([&] {                                                             \
            hipLaunchKernelGGL((vload<W, P>), dim3(blocks), dim3(256), 0, 0, t, out, n, clk);    \
        });                                                                                      \
        const double ns = ms * 1e6 / (waves_per_cu * n);                                         \
        printf("{\"load\": \"global_dword%s\", \"pattern\": \"%s\", \"ns_per_wave_inst_per_cu\": %.4f, " \
               "\"cu_cycles_at_2.4GHz\": %.2f}\n",                                               \
               W == 1 ? "" : W == 2 ? "x2" : W == 3 ? "x3" : "x4", pats[P], ns, ns * 2.4);       \
    }
    for (int rep = 0; rep < 2; ++rep) {
        RUN(1, 0) RUN(2, 0) RUN(3, 0) RUN(4, 0)
        RUN(1, 1) RUN(2, 1) RUN(3, 1) RUN(4, 1)
        RUN(1, 2) RUN(2, 2) RUN(3, 2) RUN(4, 2)
        RUN(1, 3) RUN(2, 3) RUN(3, 3) RUN(4, 3)
        for (int w = 4; w <= 8; w += 4) {
            const float ms = timed([&] {
                if (w == 4) hipLaunchKernelGGL(sload<4>, dim3(blocks), dim3(256), 0, 0, t, out, n);
                else hipLaunchKernelGGL(sload<8>, dim3(blocks), dim3(256), 0, 0, t, out, n);
            });
            const double ns = ms * 1e6 / (waves_per_cu * n);
            printf("{\"load\": \"s_load_dwordx%d\", \"pattern\": \"uniform\", \"ns_per_wave_inst_per_cu\": %.4f, "
                   "\"cu_cycles_at_2.4GHz\": %.2f}\n", w, ns, ns * 2.4);
        }
    }
    hipFree(t);
    hipFree(out);
    hipFree(clk);
    return 0;
}
