// Probe of the gfx950 buffer range check (raw buffer, stride 0): which (voffset, soffset) pairs
// read the record's memory and which return 0.  An 8 GiB allocation with the descriptor base in
// its middle keeps every probed byte address mapped, whatever the check does.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_buffer_range.hip -o /tmp/probe && /tmp/probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void probe(const float *base, uint32_t num_records, const uint32_t *vo, const uint32_t *so,
                      float *out, int n)
{
    const int i = threadIdx.x;
    if (i >= n) return;
    const uint64_t a = (uint64_t)base;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        (void *)a, 0, (int)num_records, 0x00020000);
    // soffset must be wave-uniform: one probe per loop trip, every lane the same pair
    for (int k = 0; k < n; ++k) {
        const uint32_t s = __builtin_amdgcn_readfirstlane(so[k]);
        const uint32_t v = vo[k];
        const float x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, v, s, 0));
        if (i == 0) out[k] = x;
    }
}

int main(int argc, char **argv)
{
    const size_t total = 8ull << 30, mid = 7ull << 29;  // 8 GiB, base at 3.5 GiB
    char *buf;
    if (hipMalloc(&buf, total) != hipSuccess) { printf("alloc failed\n"); return 1; }
    hipMemset(buf, 0x3f, total);  // every float reads 0.747 (0x3f3f3f3f)
    const float *base = (const float *)(buf + mid);
    const uint32_t N = argc > 1 ? (uint32_t)strtoul(argv[1], 0, 0) : 1u << 20;  // num_records
    printf("num_records = 0x%x\n", N);
    struct { uint32_t v, s; const char *what; } cases[] = {
        {0x80000010u, 0x10000000u, "v=2^31+16 s=2^28"},
        {0x80000000u, 0x80000000u, "v=2^31 s=2^31 (sum wraps to 0)"},
        {0x90000000u, 0x70000010u, "v=0x90000000 s=0x70000010 (sum 2^32+16)"},
        {N - 4, 0, "v=N-4"},
        {N - 0x1000u, 0xFF0u, "v=N-4096 s=4080 (sum N-16)"},
        {0, 0, "v=0 s=0 (in range)"},
        {N - 4, 0, "v=N-4 s=0 (last dword)"},
        {N, 0, "v=N s=0"},
        {0, N, "v=0 s=N  (soffset alone past N)"},
        {N / 2, N / 2, "v=N/2 s=N/2 (sum = N)"},
        {N / 2, N / 2 - 4, "v=N/2 s=N/2-4 (sum = N-4)"},
        {0x40000000u, 0, "v=2^30"},
        {0x7FFFFFF0u, 0, "v=2^31-16"},
        {0x80000010u, 0, "v=2^31+16"},
        {0xC0000000u, 0, "v=3*2^30"},
        {0xFFFFFFF0u, 0, "v=2^32-16"},
        {0, 0x40000000u, "s=2^30"},
        {0, 0x80000010u, "s=2^31+16"},
        {0x40000000u, 0x40000010u, "v=2^30 s=2^30+16 (sum 2^31+16)"},
        {0x7FFFFFF0u, 0x20u, "v=2^31-16 s=32 (sum 2^31+16)"},
    };
    const int n = sizeof(cases) / sizeof(cases[0]);
    uint32_t hv[64], hs[64];
    for (int k = 0; k < n; ++k) { hv[k] = cases[k].v; hs[k] = cases[k].s; }
    uint32_t *dv, *ds;
    float *dout;
    hipMalloc(&dv, sizeof(hv)); hipMalloc(&ds, sizeof(hs)); hipMalloc(&dout, 64 * sizeof(float));
    hipMemcpy(dv, hv, sizeof(hv), hipMemcpyHostToDevice);
    hipMemcpy(ds, hs, sizeof(hs), hipMemcpyHostToDevice);
    hipMemset(dout, 0xff, 64 * sizeof(float));
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, base, N, dv, ds, dout, n);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    float ho[64];
    hipMemcpy(ho, dout, sizeof(ho), hipMemcpyDeviceToHost);
    for (int k = 0; k < n; ++k)
        printf("%-40s -> %s (%g)\n", cases[k].what, ho[k] == 0.0f ? "DROPPED" : "READ", ho[k]);
    return 0;
}
