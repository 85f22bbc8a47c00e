/*
 * group_wait.h — the bounded wait of wcpt_group_sync / wcpt_group_destroy (include/wcpt.h WCPT_GROUP_OPTION_TIMEOUT_MS).
 *
 * A frame's exchange is a matched send/receive between processes: when a peer dies, or skips its part of a frame, the
 * other ranks' transfers never complete, and neither does anything queued behind them on the device. A blocking
 * hipStreamSynchronize would then never return, and the RCCL asynchronous-error check after it would never run -- a
 * Jai host calling wcpt_group_sync would hang forever instead of getting an error back (every entry
 * point returns an int; PathTracingRenderer.jai:302-305 logs and continues). So the group polls instead: the stream
 * (hipStreamQuery), then the communicator's asynchronous error (ncclCommGetAsyncError), then the deadline; the caller
 * aborts the communicator (ncclCommAbort) on a transport error or a timeout and returns WCPT_ERROR_DEVICE_LOST.
 *
 * Plain C++ with the device and clock calls passed in, so tests/test_group_plan.py runs the same loop on the CPU
 * against stand-in streams (tests/group_plan_shim.cpp).
 */
#pragma once

#include <cstdint>

namespace wcpt {
namespace gwait {

enum Poll : int { kReady = 0, kBusy = 1, kPollError = -1 };
enum Result : int { kDone = 0, kFailed = 1, kTransportError = 2, kTimedOut = 3 };

/* Spin this long after the call before the first sleep (a drained or nearly drained stream returns at once), then
 * sleep between polls for kNapFraction of the time waited so far, within [kNapMinUs, kNapMaxUs]: a wait returns at
 * most that fraction late. (Round 6 first doubled the nap up to 1 ms: a 7-ms wait for 20 frames then overslept by up
 * to a millisecond, +10 % on a 20-frame bench window, profiles/r06_short_window_s20.log.) */
constexpr double kSpinMs = 0.05;
constexpr double kNapMinUs = 10.0;
constexpr double kNapMaxUs = 1000.0;
constexpr double kNapFraction = 0.005;

/* Wait until poll() returns kReady. Between polls: transport_error() (true once the transport has reported an
 * asynchronous error) and the deadline `t0_ms + timeout_ms` of now_ms()'s clock (timeout_ms <= 0: no deadline, so only
 * a transport error or a failed poll ends a wait that never completes). t0_ms is the start of the whole operation, so
 * several waits in a row share one deadline. sleep_us(us) naps between polls. */
template <class PollF, class ErrF, class NowF, class SleepF>
Result wait_for(PollF poll, ErrF transport_error, double t0_ms, double timeout_ms, NowF now_ms, SleepF sleep_us)
{
    double nap;
    for (;;) {
        const int p = poll();
        if (p == kReady) return kDone;
        if (p != kBusy) return kFailed;
        if (transport_error()) return kTransportError;
        const double t = now_ms();
        if (timeout_ms > 0.0 && t - t0_ms >= timeout_ms) return kTimedOut;
        if (t - t0_ms < kSpinMs) continue;
        nap = (t - t0_ms) * 1000.0 * kNapFraction;
        sleep_us(nap < kNapMinUs ? kNapMinUs : (nap > kNapMaxUs ? kNapMaxUs : nap));
    }
}

} // namespace gwait
} // namespace wcpt
