// Tools only: a long-running, small kernel standing in for an RCCL transfer kernel (a few workgroups that stay
// resident for a given time (100 MHz realtime ticks)), to measure whether it overlaps the row-block render on another stream
// (tools/overlap_probe.py). Built by tools/overlap_probe.py into tools/libspin.so.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void spin_kernel(long long cycles, float* sink)
{
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    float acc = (float)threadIdx.x;
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < cycles) acc = acc * 1.0000001f + 1.0f;
    if (acc == -1.0f) sink[threadIdx.x] = acc; /* never true; keeps the loop */
}

extern "C" int spin_launch(void* stream, int blocks, long long cycles, float* sink)
{
    hipLaunchKernelGGL(spin_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, cycles, sink);
    return (int)hipGetLastError();
}

extern "C" int masked_stream_create(void** out, uint32_t words, const uint32_t* mask)
{
    hipStream_t s = nullptr;
    const hipError_t e = hipExtStreamCreateWithCUMask(&s, words, mask);
    *out = (void*)s;
    return (int)e;
}
