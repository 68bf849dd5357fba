// LDS read cost per wave instruction on gfx950, next to the texture path
// (DESIGN.md 5.1 "LDS leaf staging"): every wave issues N independent reads
// of W dwords per lane from a 4 KB LDS table, all 64 lanes at one address
// (the broadcast a staged leaf's chunk reads) or lane-strided; then a loop
// that issues one uniform global dwordx4 (L1-resident) AND one uniform
// ds_read_b128 per iteration, against each alone: whether the two paths
// overlap (time ~ max) or share a resource (time ~ sum).  8 waves per SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o lds_cost lds_cost.hip && ./lds_cost
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kTableDw = 1024;  // 4 KB

__device__ __forceinline__ uint32_t vzero() {
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}

// kPat 0: every lane the same address; 1: lane l at l * W dwords
template <int W, int kPat>
__global__ void __launch_bounds__(256) lds_load(uint32_t* out, int n) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[kTableDw + 64];
    for (int i = threadIdx.x; i < kTableDw + 64; i += 256) tab[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t z = vzero();
    const uint32_t lo = kPat == 1 ? lane * W : 0u;
    uint32_t acc = 0;
#pragma unroll 4
    for (int i = 0; i < n; ++i) {
        const uint32_t row = ((static_cast<uint32_t>(i) * 37u) & 15u) * 64u;
        const uint32_t off = ((row + lo) & (kTableDw - 1)) + z;
        if (W == 1) {
            acc ^= tab[off];
        } else if (W == 2) {
            const uint2 v = *reinterpret_cast<const uint2*>(tab + (off & ~1u));
            acc ^= v.x + v.y;
        } else {
            const uint4 v = *reinterpret_cast<const uint4*>(tab + (off & ~3u));
            acc ^= v.x + v.y + v.z + v.w;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// kWhich bit 0: a uniform global dwordx4 per iteration; bit 1: a uniform ds_read_b128
template <int kWhich>
__global__ void __launch_bounds__(256) mixed(const uint32_t* __restrict__ t, uint32_t* out, int n) {
    __shared__ __attribute__((aligned(16))) uint32_t tab[kTableDw + 64];
    for (int i = threadIdx.x; i < kTableDw + 64; i += 256) tab[i] = i * 2654435761u;
    __syncthreads();
    const uint32_t z = vzero();
    uint32_t acc = 0;
#pragma unroll 4
    for (int i = 0; i < n; ++i) {
        const uint32_t row = ((static_cast<uint32_t>(i) * 37u) & 15u) * 64u + z;
        if (kWhich & 1) {
            const uint4 v = *reinterpret_cast<const uint4*>(t + row);
            acc ^= v.x + v.y + v.z + v.w;
        }
        if (kWhich & 2) {
            const uint4 v = *reinterpret_cast<const uint4*>(tab + ((row + 4u) & (kTableDw - 1)));
            acc ^= v.x + v.y + v.z + v.w;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
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
    const int wg_per_cu = 8;
    const int blocks = cus * wg_per_cu;
    const int n = 8192;
    uint32_t *t, *out;
    hipMalloc(&t, kTableDw * 4 + 64);
    hipMemset(t, 1, kTableDw * 4 + 64);
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    const double waves_per_cu = wg_per_cu * 4.0;
    printf("{\"cus\": %d, \"waves_per_cu\": %.0f, \"n\": %d}\n", cus, waves_per_cu, n);
    const char* pats[2] = {"uniform", "strided"};
#define RUN(W, P)                                                                                 \
    {                                                                                             \
        const float ms = timed([&] { hipLaunchKernelGGL((lds_load<W, P>), dim3(blocks), dim3(256), 0, 0, out, n); }); \
        const double ns = ms * 1e6 / (waves_per_cu * n);                                          \
        printf("{\"load\": \"ds_read_b%d\", \"pattern\": \"%s\", \"ns_per_wave_inst_per_cu\": %.4f, " \
               "\"cu_cycles_at_2.4GHz\": %.2f}\n", 32 * W, pats[P], ns, ns * 2.4);                \
    }
#define MIX(K, NAME)                                                                              \
    {                                                                                             \
        const float ms = timed([&] { hipLaunchKernelGGL((mixed<K>), dim3(blocks), dim3(256), 0, 0, t, out, n); }); \
        const double ns = ms * 1e6 / (waves_per_cu * n);                                          \
        printf("{\"loop\": \"%s\", \"ns_per_iter_per_cu\": %.4f, \"cu_cycles_at_2.4GHz\": %.2f}\n", \
               NAME, ns, ns * 2.4);                                                               \
    }
    for (int rep = 0; rep < 2; ++rep) {
        RUN(1, 0) RUN(2, 0) RUN(4, 0)
        RUN(1, 1) RUN(2, 1) RUN(4, 1)
        MIX(1, "global_dwordx4 uniform") MIX(2, "ds_read_b128 uniform")
        MIX(3, "both per iteration")
    }
    hipFree(t);
    hipFree(out);
    return 0;
}
