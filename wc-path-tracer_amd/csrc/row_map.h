/* row_map.h — which frame row each local row of a context is (row blocks, or interleaved row stripes).
 *
 * A context renders `rows` local rows; local row ly is frame row y0 + ly + (ly >> shift) * gap. A contiguous row block
 * [y0, y0 + rows) (wcpt_set_row_range) has shift 31 and gap 0 (ly < 2^31, so ly >> 31 = 0). Interleaved stripes of
 * 2^shift rows every `period` rows (wcpt_set_row_stripes: rank r of n takes stripes r, r + n, r + 2n, ...) have
 * y0 = first stripe's row and gap = period - 2^shift. Shared by the kernels (pt_device.h) and the host runtime. */
#ifndef WCPT_ROW_MAP_H
#define WCPT_ROW_MAP_H

#include <stdint.h>

namespace wcpt {

struct RowMap {
    uint32_t y0, shift, gap;
};
constexpr uint32_t kContiguousShift = 31;

#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
__host__ __device__
#endif
inline uint32_t frame_row(const RowMap& m, uint32_t ly)
{
    return m.y0 + ly + (ly >> m.shift) * m.gap;
}

/* the same in 64 bits, for host-side bounds checks that must not wrap */
inline uint64_t frame_row64(const RowMap& m, uint32_t ly)
{
    return (uint64_t)m.y0 + ly + (uint64_t)(ly >> m.shift) * m.gap;
}

} // namespace wcpt

#endif
