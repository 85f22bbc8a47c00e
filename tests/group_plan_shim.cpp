// Test shim (CPU): exposes the product's frame plan (wc-path-tracer_amd/csrc/group_plan.h, what wcpt_group_render
// executes) to tests/test_group_plan.py over ctypes. Built by the test with g++; no HIP involved.
#include <cstdint>
#include <vector>

#include "../wc-path-tracer_amd/csrc/group_plan.h"

extern "C" int plan_frames(int nranks, int root, int overlap, int transport, int nlocal, const int32_t* local_ranks,
                           const int32_t* presenting, int frames, int32_t* out, int cap, int stripes)
{
    std::vector<wcpt::plan::RankState> local(nlocal);
    for (int i = 0; i < nlocal; i++) local[i] = {local_ranks[i], {false, false}};
    std::vector<wcpt::plan::Step> steps;
    int n = 0;
    for (int f = 0; f < frames; f++) {
        const bool exchange = presenting[f] != 0 && nranks > 1;
        wcpt::plan::frame_steps(nranks, root, overlap != 0, exchange, transport, (uint64_t)f, local, steps, stripes != 0);
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

// The bounded wait of wcpt_group_sync (wc-path-tracer_amd/csrc/group_wait.h) against a stand-in stream and clock: the
// stream drains after `ready_after` polls (< 0: never), the transport reports an asynchronous error from poll
// `error_after` on (< 0: never), and a poll fails at `fail_at` (< 0: never). Each poll advances the clock by
// ms_per_poll, each nap by its length. Returns the wait's result; *elapsed_ms / *polls / *naps say how it got there.
#include "../wc-path-tracer_amd/csrc/group_wait.h"

extern "C" int wait_sim(int ready_after, int error_after, int fail_at, double timeout_ms, double ms_per_poll,
                        double* elapsed_ms, int* polls, int* naps)
{
    double clock = 1000.0;
    int n = 0, k = 0;
    const double t0 = clock;
    const wcpt::gwait::Result r = wcpt::gwait::wait_for(
        [&]() {
            const int i = n++;
            clock += ms_per_poll;
            if (fail_at >= 0 && i >= fail_at) return (int)wcpt::gwait::kPollError;
            return ready_after >= 0 && i >= ready_after ? (int)wcpt::gwait::kReady : (int)wcpt::gwait::kBusy;
        },
        [&]() { return error_after >= 0 && n > error_after; }, t0, timeout_ms, [&]() { return clock; },
        [&](double us) {
            k++;
            clock += us / 1000.0;
        });
    *elapsed_ms = clock - t0;
    *polls = n;
    *naps = k;
    return (int)r;
}

// The same wait against a stream that drains at a given time (drain_ms after the call): how late the wait returns.
extern "C" int wait_sim_time(double drain_ms, double timeout_ms, double ms_per_poll, double* elapsed_ms, int* polls,
                             int* naps)
{
    double clock = 1000.0;
    int n = 0, k = 0;
    const double t0 = clock;
    const wcpt::gwait::Result r = wcpt::gwait::wait_for(
        [&]() {
            n++;
            clock += ms_per_poll;
            return clock - t0 >= drain_ms ? (int)wcpt::gwait::kReady : (int)wcpt::gwait::kBusy;
        },
        [&]() { return false; }, t0, timeout_ms, [&]() { return clock; },
        [&](double us) {
            k++;
            clock += us / 1000.0;
        });
    *elapsed_ms = clock - t0;
    *polls = n;
    *naps = k;
    return (int)r;
}
