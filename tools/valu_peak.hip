// valu_peak.hip — measured VALU issue ceiling of the MI355X, for the roofline's `peak` (bench.py).
//
// Every SIMD runs W waves of 64 lanes; each wave runs K independent FMA chains (no dependency stall once K >= 4) for
// N iterations. wave-instructions / s over the whole chip, against 1024 SIMDs x clock, gives the cycles one wave64
// VALU instruction occupies a SIMD -- scalar v_fma_f32 and packed v_pk_fma_f32 -- and how many waves per SIMD it
// takes to reach it. Build: hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize tools/valu_peak.hip -o tools/valu_peak
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float v2f __attribute__((ext_vector_type(2)));

template <int K, bool PACKED>
__global__ __launch_bounds__(64) void fma_chains(float* out, int iters, float a, float b)
{
    float x[K];
    v2f y[K];
#pragma unroll
    for (int k = 0; k < K; k++) {
        x[k] = threadIdx.x * 1e-3f + k;
        y[k] = (v2f){x[k], x[k] + 0.5f};
    }
    const v2f a2 = {a, a}, b2 = {b, b};
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < K; k++) {
            if (PACKED)
                y[k] = __builtin_elementwise_fma(y[k], a2, b2);
            else
                x[k] = __builtin_fmaf(x[k], a, b);
        }
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < K; k++) s += PACKED ? (y[k].x + y[k].y) : x[k];
    if (s == 12345.0f) out[threadIdx.x] = s;
}

template <int K, bool PACKED>
static void run(int cus, int waves_per_simd, int iters, float* out)
{
    const int blocks = cus * 4 * waves_per_simd;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL((fma_chains<K, PACKED>), dim3(blocks), dim3(64), 0, 0, out, iters, 0.999f, 0.001f);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL((fma_chains<K, PACKED>), dim3(blocks), dim3(64), 0, 0, out, iters, 0.999f, 0.001f);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double winstr = (double)blocks * iters * K;            // wave64 VALU instructions in the loop
    const double rate = winstr / (best * 1e-3);                  // wave-instructions per second
    printf("{\"packed\": %d, \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"gwave_instr_per_s\": %.1f, "
           "\"cycles_per_wave_instr_at_2.4GHz\": %.3f}\n",
           PACKED ? 1 : 0, K, waves_per_simd, best, rate / 1e9, (double)cus * 4 * 2.4e9 / rate);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main()
{
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    float* out = nullptr;
    (void)hipMalloc(&out, 4096);
    const int iters = 20000;
    for (int w : {1, 2, 4, 8}) {
        run<8, false>(cus, w, iters, out);
        run<8, true>(cus, w, iters, out);
    }
    run<2, false>(cus, 4, iters, out);   // dependent chains: latency-bound
    (void)hipFree(out);
    return 0;
}
