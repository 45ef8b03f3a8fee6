// Probe: float-atomic throughput on gfx950 for the item-row pattern of the SGD kernels (rows of
// 512 B, two 64-lane instructions per row update, rows drawn pseudo-randomly from a table of
// ML-1M's 3,706 items), by scope and by table placement:
//   agent  : __hip_atomic_fetch_add(relaxed, agent scope), one shared table
//   wg     : the same with workgroup scope (what another workgroup sees is not promised: the
//            probe checks the sum of every element against the expected total)
//   buf0   : raw buffer atomic, cache policy 0 (the kernels' form)
//   xcd    : buf0 into one table copy per XCD (row + xcc_id * table), summed afterwards
//   hipcc --offload-arch=gfx950 -O3 tools/probe_atomics.hip -o /tmp/pa && /tmp/pa
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

constexpr int kRowF = 128;  // floats per row (512 B)

__device__ __forceinline__ int xcc_id() {
    return (int)(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 0xF);
}

template <int MODE>
__global__ __launch_bounds__(256) void hammer(float *tab, int n_rows, int iters, uint32_t seed, int skew)
{
    const int lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    uint32_t s = seed ^ (wave * 2654435761u);
    float *base = tab;
    if (MODE == 3) base = tab + (size_t)xcc_id() * n_rows * kRowF;
    const uint32_t bytes = (uint32_t)n_rows * kRowF * 4;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
    for (int it = 0; it < iters; ++it) {
        s = s * 1664525u + 1013904223u;
        uint32_t row = (s >> 8) % (uint32_t)n_rows;
        if (skew) {  // popularity ~ power law: row = n * x^3, x uniform in [0, 1)
            const float x = (float)(s >> 8) * (1.0f / 16777216.0f);
            row = (uint32_t)((float)n_rows * x * x * x);
        }
        row = __builtin_amdgcn_readfirstlane(row);
        for (int h = 0; h < 2; ++h) {
            const int c = lane + 64 * h;
            if (MODE == 0)
                __hip_atomic_fetch_add(base + (size_t)row * kRowF + c, 1.0f, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            else if (MODE == 1)
                __hip_atomic_fetch_add(base + (size_t)row * kRowF + c, 1.0f, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            else
                __builtin_amdgcn_raw_ptr_buffer_atomic_fadd_f32(1.0f, r, (uint32_t)c * 4,
                                                                row * kRowF * 4, 0);
        }
    }
}

int main(int argc, char **argv)
{
    const int skew = argc > 1 ? atoi(argv[1]) : 0;
    printf("row distribution: %s\n", skew ? "skewed (n x^3)" : "uniform");
    const int n_rows = 3706, blocks = 256 * 4, iters = 2000;  // 4 blocks (16 waves) per CU
    float *tab;
    const size_t tab_f = (size_t)n_rows * kRowF;
    hipMalloc(&tab, 8 * tab_f * sizeof(float));
    float *h = (float *)malloc(8 * tab_f * sizeof(float));
    const char *names[] = {"agent", "wg", "buf0", "xcd"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(tab, 0, 8 * tab_f * sizeof(float));
            hipEvent_t a, b;
            hipEventCreate(&a); hipEventCreate(&b);
            hipEventRecord(a, 0);
            switch (mode) {
                case 0: hipLaunchKernelGGL(hammer<0>, dim3(blocks), dim3(256), 0, 0, tab, n_rows, iters, 7u, skew); break;
                case 1: hipLaunchKernelGGL(hammer<1>, dim3(blocks), dim3(256), 0, 0, tab, n_rows, iters, 7u, skew); break;
                case 2: hipLaunchKernelGGL(hammer<2>, dim3(blocks), dim3(256), 0, 0, tab, n_rows, iters, 7u, skew); break;
                default: hipLaunchKernelGGL(hammer<3>, dim3(blocks), dim3(256), 0, 0, tab, n_rows, iters, 7u, skew); break;
            }
            hipEventRecord(b, 0);
            if (hipEventSynchronize(b) != hipSuccess) { printf("kernel failed\n"); return 1; }
            float ms;
            hipEventElapsedTime(&ms, a, b);
            hipMemcpy(h, tab, 8 * tab_f * sizeof(float), hipMemcpyDeviceToHost);
            double total = 0;
            for (size_t x = 0; x < 8 * tab_f; ++x) total += h[x];
            const double expect = (double)blocks * 4 * iters * 128;
            const double gbs = (double)blocks * 4 * iters * 512 / (ms * 1e-3) / 1e9;
            printf("%-6s rep %d: %8.3f ms  %8.1f GB/s of added bytes  sum %s (%.0f / %.0f)\n",
                   names[mode], rep, ms, gbs, total == expect ? "exact" : "LOST UPDATES", total,
                   expect);
        }
    }
    return 0;
}
