// Probe (timing only, not part of the product): the shader clock seen by one wave, from the
// cycle counter (s_memtime) against the constant 100 MHz real-time counter (s_memrealtime),
// over a dependent fp64 FMA chain.  out[0] = shader cycles, out[1] = 100 MHz ticks, out[2] = sum.
#include <hip/hip_runtime.h>
#include <cstdint>

__global__ void clock_probe_kernel(long long *out, int iters)
{
    if (threadIdx.x >= 64) return;
    double x = 1.0 + threadIdx.x * 1e-9, y = 0.999999;
    const long long c0 = clock64(), w0 = wall_clock64();
    for (int i = 0; i < iters; ++i) {
        x = __fma_rn(x, y, 1e-9);
        x = __fma_rn(x, y, 1e-9);
        x = __fma_rn(x, y, 1e-9);
        x = __fma_rn(x, y, 1e-9);
    }
    const long long c1 = clock64(), w1 = wall_clock64();
    if (threadIdx.x == 0) {
        out[0] = c1 - c0;
        out[1] = w1 - w0;
        out[2] = (long long)(x * 1e6);
    }
}

extern "C" int clock_probe(long long *out, int iters, void *stream)
{
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out, iters);
    return (int)hipGetLastError();
}
