/* pt_kernels.h — launch interface between the C-ABI runtime and the HIP kernels. */
#ifndef WCPT_PT_KERNELS_H
#define WCPT_PT_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wcpt.h"

namespace wcpt {

/* Traversal stack entries per lane. The reference declares 32 (pathTracer.comp:151), which a depth-32
 * midpoint BVH can overflow; our far-child stack needs at most tree depth entries. Deeper trees set the
 * WCPT_ERROR_STACK_OVERFLOW status instead of writing out of bounds. */
constexpr int kStackDepth = 48;

struct LaunchArgs {
    wcpt_scene_data sd;
    const wcpt_material* materials;
    const wcpt_sphere* spheres;
    const wcpt_draw_command* draws;
    float4* image;
    uint32_t W, H, y0, rows;
    uint32_t* status;
    unsigned long long* counters;
};

hipError_t launch_megakernel(const LaunchArgs& a, bool count, hipStream_t stream);
hipError_t launch_selftest(int fn, const uint32_t* in, const uint32_t* in2, uint32_t* out, uint32_t n,
                           hipStream_t stream);

} // namespace wcpt

#endif
