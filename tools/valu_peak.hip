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

/* One VALU instruction of kind OP on chain register x (inline asm, so the compiler neither folds nor reorders the
 * chains): 1 v_max_f32, 2 v_add_u32, 3 v_xor_b32. Different instruction kinds draw different power, and the clock the
 * chip holds under load -- so the issue rate it sustains -- depends on the mix. */
template <int OP>
__device__ __forceinline__ void op_asm(float& x, float a)
{
    if (OP == 1) asm volatile("v_max_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    if (OP == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(a));
    if (OP == 3) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(a));
    if (OP == 4) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    if (OP == 5) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(a));
    if (OP == 6) asm volatile("v_rcp_f32 %0, %0" : "+v"(x));
    if (OP == 7) asm volatile("v_mov_b32 %0, %1" : "+v"(x) : "v"(a));
    if (OP == 8) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(a) : "vcc");
    if (OP == 9) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(x));
    if (OP == 10) asm volatile("v_min3_f32 %0, %0, %1, %0" : "+v"(x) : "v"(a));
}
/* Kinds that need a second register class: a select on an SGPR mask, a compare into an SGPR pair, packed FP32. */
template <int OP>
__device__ __forceinline__ void op2_asm(float& x, v2f& y, float a, v2f a2, unsigned long long m)
{
    if (OP == 11) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "s"(m));
    if (OP == 12) {
        unsigned long long c;
        asm volatile("v_cmp_gt_f32_e64 %0, %1, %2" : "=s"(c) : "v"(x), "v"(a));
        asm volatile("; %0" ::"s"(c));
    }
    if (OP == 13) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(y) : "v"(a2));
    if (OP == 14) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(y) : "v"(a2));
}

template <int K, int OP>
__global__ __launch_bounds__(64) void op2_chains(float* out, int iters, float a)
{
    float x[K];
    v2f y[K];
    const v2f a2 = {a, a};
    const unsigned long long m = __ballot(threadIdx.x & 1);
#pragma unroll
    for (int k = 0; k < K; k++) {
        x[k] = threadIdx.x * 1e-3f + k;
        y[k] = (v2f){x[k], x[k] + 0.5f};
    }
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < K; k++) op2_asm<OP>(x[k], y[k], a, a2, m);
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < K; k++) s += x[k] + y[k].x + y[k].y;
    if (s == 12345.0f) out[threadIdx.x] = s;
}

template <int K, int OP>
__global__ __launch_bounds__(64) void op_chains(float* out, int iters, float a)
{
    float x[K];
#pragma unroll
    for (int k = 0; k < K; k++) x[k] = threadIdx.x * 1e-3f + k;
    for (int i = 0; i < iters; i++) {
#pragma unroll
        for (int k = 0; k < K; k++) op_asm<OP>(x[k], a);
    }
    float s = 0.0f;
#pragma unroll
    for (int k = 0; k < K; k++) s += x[k];
    if (s == 12345.0f) out[threadIdx.x] = s;
}

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

template <int K, int OP>
static void run_op(int cus, int waves_per_simd, int iters, float* out)
{
    const int blocks = cus * 4 * waves_per_simd;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    auto kern = OP <= 10 ? op_chains<K, (OP <= 10 ? OP : 1)> : op2_chains<K, (OP > 10 ? OP : 11)>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, iters, 0.999f);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        (void)hipEventRecord(e0, 0);
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, out, iters, 0.999f);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const double winstr = (double)blocks * iters * K;
    const double rate = winstr / (best * 1e-3);
    static const char* names[] = {"v_fma_f32",     "v_max_f32",        "v_add_u32",    "v_xor_b32",
                                  "v_mul_f32",     "v_add_f32",        "v_rcp_f32",    "v_mov_b32",
                                  "v_cndmask_b32 (vcc clobbered)",     "v_lshlrev_b32", "v_min3_f32",
                                  "v_cndmask_b32_e64 (sgpr mask)",     "v_cmp_gt_f32_e64", "v_pk_mul_f32",
                                  "v_pk_add_f32"};
    printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.4f, \"gwave_instr_per_s\": %.1f, "
           "\"cycles_per_wave_instr_at_2.4GHz\": %.3f}\n",
           names[OP], K, waves_per_simd, best, rate / 1e9, (double)cus * 4 * 2.4e9 / rate);
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
    for (int w : {4, 8}) {
        run_op<8, 1>(cus, w, iters, out);
        run_op<8, 2>(cus, w, iters, out);
        run_op<8, 3>(cus, w, iters, out);
    }
    /* the instruction classes of the mix-weighted ceiling (bench.py roofline), 8 waves/SIMD */
    run_op<8, 4>(cus, 8, iters, out);
    run_op<8, 5>(cus, 8, iters, out);
    run_op<8, 6>(cus, 8, iters, out);
    run_op<8, 7>(cus, 8, iters, out);
    run_op<8, 8>(cus, 8, iters, out);
    run_op<8, 9>(cus, 8, iters, out);
    for (int w : {4, 8}) {
        run_op<8, 5>(cus, w == 4 ? 4 : 8, iters, out);
        run_op<8, 10>(cus, w, iters, out);
        run_op<8, 11>(cus, w, iters, out);
        run_op<8, 12>(cus, w, iters, out);
        run_op<8, 13>(cus, w, iters, out);
        run_op<8, 14>(cus, w, iters, out);
    }
    (void)hipFree(out);
    return 0;
}
