// Exhaustive: is v_sqrt_f32 (__builtin_amdgcn_sqrtf) equal to IEEE sqrtf for every positive normal binary32?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void check(unsigned long long* mism, unsigned long long* first)
{
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < (1ull << 31); k += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t bits = (uint32_t)k;              /* all non-negative patterns */
        const float x = __uint_as_float(bits);
        if (!(x >= 0x1p-126f && x < __builtin_inff())) continue;
        const float ref = sqrtf(x);
        const float y = __builtin_amdgcn_sqrtf(x);
        if (__float_as_uint(y) != __float_as_uint(ref)) { atomicAdd(mism, 1ull); atomicMin(first, (unsigned long long)bits); }
    }
}
int main()
{
    unsigned long long *m, *f, z = 0, ff = ~0ull, c = 0, fb = 0;
    (void)hipMalloc(&m, 8); (void)hipMalloc(&f, 8);
    (void)hipMemcpy(m, &z, 8, hipMemcpyHostToDevice); (void)hipMemcpy(f, &ff, 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, m, f);
    (void)hipMemcpy(&c, m, 8, hipMemcpyDeviceToHost); (void)hipMemcpy(&fb, f, 8, hipMemcpyDeviceToHost);
    printf("v_sqrt_f32 mismatches vs IEEE sqrtf: %llu (first 0x%08llx)\n", c, c ? fb : 0ull);
    return 0;
}
