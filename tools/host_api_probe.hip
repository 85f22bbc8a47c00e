/*
 * host_api_probe.hip — host cost of the HIP calls one group frame issues per rank (wcpt_group.hip), on this box:
 * hipEventRecord, hipStreamWaitEvent, a small kernel launch, hipMemcpyPeerAsync / hipMemcpyAsync of a small block,
 * hipSetDevice, hipEventQuery. Each call is timed over many repetitions with the device kept busy-free (tiny work),
 * from 1 thread and from T threads at once (each on its own stream of device 0), so the numbers say how a per-rank
 * cost adds up when ranks issue from one thread, and whether issuing from several threads overlaps on one device.
 *
 *   hipcc --offload-arch=gfx950 -O2 -o tools/host_api_probe tools/host_api_probe.hip -lpthread
 *   tools/host_api_probe [reps]
 */
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

struct Args256 {
    unsigned char b[256];
};

__global__ void tiny(Args256 a, float* out)
{
    if (threadIdx.x == 0 && blockIdx.x == 0 && out) out[0] = (float)a.b[threadIdx.x];
}

using Clock = std::chrono::steady_clock;

struct Probe {
    hipStream_t s = nullptr, c = nullptr;
    hipEvent_t e = nullptr;
    void* a = nullptr;
    void* b = nullptr;
    float* o = nullptr;
};

enum Op { kRecord, kWait, kLaunch, kCopy, kPeer, kSetDev, kQuery, kNumOps };
const char* kNames[kNumOps] = {"hipEventRecord", "hipStreamWaitEvent", "kernel launch (256 B args)",
                               "hipMemcpyAsync D2D 4 KiB", "hipMemcpyPeerAsync 4 KiB (same device)", "hipSetDevice",
                               "hipEventQuery"};

void setup(Probe& p)
{
    CHECK(hipSetDevice(0));
    CHECK(hipStreamCreateWithFlags(&p.s, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&p.c, hipStreamNonBlocking));
    CHECK(hipEventCreateWithFlags(&p.e, hipEventDisableTiming));
    CHECK(hipMalloc(&p.a, 4096));
    CHECK(hipMalloc(&p.b, 4096));
    CHECK(hipMalloc(&p.o, 64));
}

/* microseconds per call of `op`, issued `reps` times on the probe's streams (drained every 64 calls so queues stay
 * short, the drain not timed) */
double run_op(Probe& p, int op, int reps)
{
    Args256 args{};
    double total = 0;
    for (int base = 0; base < reps; base += 64) {
        const auto t0 = Clock::now();
        for (int i = 0; i < 64; i++) {
            switch (op) {
            case kRecord: CHECK(hipEventRecord(p.e, p.s)); break;
            case kWait: CHECK(hipStreamWaitEvent(p.c, p.e, 0)); break;
            case kLaunch: tiny<<<1, 64, 0, p.s>>>(args, p.o); break;
            case kCopy: CHECK(hipMemcpyAsync(p.b, p.a, 4096, hipMemcpyDeviceToDevice, p.s)); break;
            case kPeer: CHECK(hipMemcpyPeerAsync(p.b, 0, p.a, 0, 4096, p.s)); break;
            case kSetDev: CHECK(hipSetDevice(0)); break;
            case kQuery: (void)hipEventQuery(p.e); break;
            }
        }
        total += std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
        CHECK(hipStreamSynchronize(p.s));
        CHECK(hipStreamSynchronize(p.c));
    }
    return total / reps;
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 4096;
    const int max_threads = 8;
    std::vector<Probe> probes(max_threads);
    for (auto& p : probes) setup(p);
    CHECK(hipEventRecord(probes[0].e, probes[0].s));
    for (int op = 0; op < kNumOps; op++) (void)run_op(probes[0], op, 256); /* warm-up */
    std::printf("{\"reps\": %d, \"ops\": {\n", reps);
    for (int op = 0; op < kNumOps; op++) {
        std::printf("  \"%s\": {", kNames[op]);
        for (int t : {1, 2, 4, 8}) {
            std::vector<double> us(t, 0.0);
            std::atomic<int> ready{0};
            std::atomic<bool> go{false};
            std::vector<std::thread> th;
            const auto t0 = Clock::now();
            for (int k = 0; k < t; k++)
                th.emplace_back([&, k] {
                    CHECK(hipSetDevice(0));
                    ready++;
                    while (!go.load()) {
                    }
                    us[k] = run_op(probes[k], op, reps);
                });
            while (ready.load() < t) {
            }
            go = true;
            for (auto& x : th) x.join();
            const double wall = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
            double mx = 0;
            for (double v : us) mx = v > mx ? v : mx;
            /* per call on one thread; with t threads: the slowest thread's per-call time, and the wall time per
             * "round" of t calls (one call per thread), i.e. what a t-rank frame would cost issued in parallel */
            std::printf("\"t%d\": {\"per_call_us\": %.2f, \"round_wall_us\": %.2f}%s", t, mx, wall / reps,
                        t == 8 ? "" : ", ");
        }
        std::printf("}%s\n", op + 1 == kNumOps ? "" : ",");
        std::fflush(stdout);
    }
    std::printf("}}\n");
    for (auto& p : probes) {
        CHECK(hipStreamSynchronize(p.s));
        CHECK(hipStreamSynchronize(p.c));
    }
    return 0;
}
