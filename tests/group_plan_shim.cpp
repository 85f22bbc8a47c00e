// Test shim (CPU): exposes the product's frame plan (wc-path-tracer_amd/csrc/group_plan.h, what wcpt_group_render
// executes) to tests/test_group_plan.py over ctypes. Built by the test with g++; no HIP involved.
#include <cstdint>
#include <vector>

#include "../wc-path-tracer_amd/csrc/group_plan.h"

extern "C" int plan_frames(int nranks, int root, int overlap, int transport, int nlocal, const int32_t* local_ranks,
                           const int32_t* presenting, int frames, int32_t* out, int cap)
{
    std::vector<wcpt::plan::RankState> local(nlocal);
    for (int i = 0; i < nlocal; i++) local[i] = {local_ranks[i], {false, false}};
    std::vector<wcpt::plan::Step> steps;
    int n = 0;
    for (int f = 0; f < frames; f++) {
        const bool exchange = presenting[f] != 0 && nranks > 1;
        wcpt::plan::frame_steps(nranks, root, overlap != 0, exchange, transport, (uint64_t)f, local, steps);
        for (const wcpt::plan::Step& s : steps) {
            if (n >= cap) return -1;
            int32_t* o = out + 6 * n++;
            o[0] = f;
            o[1] = s.op;
            o[2] = s.rank;
            o[3] = s.buffer;
            o[4] = s.peer;
            o[5] = s.stream;
        }
    }
    return n;
}
