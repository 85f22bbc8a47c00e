/*
 * pt_composite.hip — the display step after the path (composite.comp:3-54): gamma 1/2.2 and
 * the PBR Neutral tonemap over the float4 accumulation image, written as rgba32f (what composite.comp stores) or
 * as RGBA8 UNORM for display (4x fewer bytes to read back or gather).
 *
 * Bound: HBM streaming, 16 B read + 16 B (or 4 B) written per pixel; ~70 binary32 ops + 3 log/exp pairs per
 * pixel, far below the VALU roofline at 16-32 B/px. Grid-stride, 4 pixels of 16 B per thread in flight.
 */
#include <hip/hip_runtime.h>

#include "pt_kernels.h"
#include "wcpt_composite.h"

namespace wcpt {
namespace dev {

template <bool RGBA8>
__global__ __launch_bounds__(256) void composite_kernel(const float4* __restrict__ img, uint64_t n, float4* __restrict__ out32,
                                                        uchar4* __restrict__ out8)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256u) {
        const float4 v = img[i];
        const float in[4] = {v.x, v.y, v.z, v.w};
        float o[4];
        wcpt_composite_texel(in, o);
        if (RGBA8)
            out8[i] = make_uchar4(wcpt_unorm8(o[0]), wcpt_unorm8(o[1]), wcpt_unorm8(o[2]), 255);
        else
            out32[i] = make_float4(o[0], o[1], o[2], o[3]);
    }
}

} // namespace dev

hipError_t launch_composite(const float4* img, uint64_t pixels, void* dst, bool rgba8, int cus, hipStream_t stream)
{
    if (pixels == 0) return hipSuccess;
    uint64_t blocks = (pixels + 255u) / 256u;
    const uint64_t cap = (uint64_t)(cus > 0 ? cus : 256) * 8u;
    if (blocks > cap) blocks = cap;
    if (rgba8)
        hipLaunchKernelGGL(dev::composite_kernel<true>, dim3((uint32_t)blocks), dim3(256), 0, stream, img, pixels, nullptr,
                           static_cast<uchar4*>(dst));
    else
        hipLaunchKernelGGL(dev::composite_kernel<false>, dim3((uint32_t)blocks), dim3(256), 0, stream, img, pixels,
                           static_cast<float4*>(dst), nullptr);
    return hipGetLastError();
}

} // namespace wcpt
