/*
 * wcpt_group.hip — one frame on several devices (include/wcpt.h wcpt_group_*).
 *
 * The reference renders every frame on one device from one thread (src/main.jai:185-194 -> Render,
 * src/PathTracingRenderer.jai:399-457). Every pixel is independent -- its seed depends only on the global (x, y,
 * frame) (pathTracer.comp:304) and the accumulation is per pixel (:314-323) -- so the frame partitions into row
 * blocks: rank r of N renders rows [r*H/N, (r+1)*H/N) on its own device, keeps only that block of the accumulation
 * image, and the union is bit-identical to a one-device render. The one exchange is presenting a frame: the blocks
 * go to the root device. That is a gather of unequal blocks (H/N need not be an integer).
 *
 * Two ways to hold the ranks:
 *  - one process, one thread, all devices (wcpt_group_create[_ex]): the shape of the reference's host. RCCL transport:
 *    ncclCommInitAll (rccl.h:236), one communicator per device, every frame's sends and receives inside one
 *    ncclGroupStart/ncclGroupEnd (rccl.h:700,722); xGMI carries the 7 incoming blocks of an 8-GPU node over 7 links
 *    at once. COPY transport: each rank pushes its block into the root's frame with hipMemcpyPeerAsync on its own
 *    device's copy path; a device may be listed more than once (an N-rank rehearsal on fewer devices).
 *  - one process per device (wcpt_group_create_rank): ncclCommInitRank with an id the host distributes; each process
 *    holds its own rank and the gather is the same send/receive pattern.
 *
 * Overlap (WCPT_GROUP_OPTION_OVERLAP, default on). Each local rank has a render stream (its context's) and a
 * communication stream. Frame k on a sending rank: the render writes the block into payload buffer k % 2
 * (wcpt_set_gather_output: no copy pass), an event marks the render's end, the communication stream waits for it and
 * sends, and an event marks the send's end; the render of frame k + 2, which rewrites that buffer, waits for that
 * event on the device (hipStreamWaitEvent), so the host never blocks. The root renders its block straight into the
 * presented frame and receives the others' rows on its communication stream, so its next render does not wait for the
 * slowest rank's transfer. A payload buffer that must grow (a resize, a wider format) is replaced by a new hipMalloc
 * buffer and the old one is retired: queued transfers may still read it, so it is freed at the next point where the
 * group waits for all its work anyway (wcpt_group_sync, wcpt_group_destroy) -- a resize never synchronises the device
 * (hipFree would). Plain device allocations, not the stream-ordered pool: they are what RCCL's transports expect of a
 * user buffer.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/wcpt.h"
#include "group_plan.h"
#include "group_wait.h"
#include "pt_kernels.h"

static_assert(sizeof(ncclUniqueId) == WCPT_GROUP_UNIQUE_ID_BYTES, "WCPT_GROUP_UNIQUE_ID_BYTES");

namespace {

constexpr int kPayloadBuffers = wcpt::plan::kPayloadBuffers;
namespace plan = wcpt::plan;
namespace gwait = wcpt::gwait;
/* The default bound on one wcpt_group_sync of a group of several ranks. An editor loop syncs every frame (main.jai:73-95);
 * bench.py syncs after at most a few hundred frames (c4 at 8 ranks: ~45 ms each). */
constexpr int kDefaultTimeoutMs = 60000;

/* One rank driven by this process. */
struct LocalRank {
    int rank = 0;
    int device = 0;
    wcpt_context* ctx = nullptr;
    ncclComm_t comm = nullptr;
    hipStream_t comm_stream = nullptr;
    void* payload[kPayloadBuffers] = {};
    uint64_t payload_cap[kPayloadBuffers] = {};
    hipEvent_t ready[kPayloadBuffers] = {};  /* the render that wrote payload[b] has finished */
    hipEvent_t sent[kPayloadBuffers] = {};   /* the transfer that read payload[b] has finished */
    /* with the frame overlap, `ready` covers the context's stream and these its pipe streams (created on first use) */
    hipEvent_t ready_pipe[kPayloadBuffers][wcpt::kMaxFrameStreams - 1] = {};
    int ready_n[kPayloadBuffers] = {};
    bool sent_pending[kPayloadBuffers] = {};
    std::vector<void*> retired;              /* replaced payload buffers, freed at the next group-wide wait */
    void* stage = nullptr;                   /* root, RCCL with row stripes: every sender's block back to back */
    uint64_t stage_cap = 0;
};

#if WCPT_GROUP_TIMERS
/* tools-only build (tools/host_group_probe.py --timers): host nanoseconds per plan step kind, printed at destroy */
struct StepTimers {
    double ns[16] = {};
    uint64_t n[16] = {};
};
StepTimers g_timers;
thread_local bool t_worker = false; /* the issue threads' steps are not timed (g_timers is the caller thread's) */
struct StepTimer {
    int k;
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    explicit StepTimer(int kind) : k(kind) {}
    ~StepTimer()
    {
        if (t_worker) return;
        g_timers.ns[k] += std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
        g_timers.n[k]++;
    }
};
#define STEP_TIMER(kind) StepTimer step_timer_(kind)
#else
#define STEP_TIMER(kind) (void)0
#endif

/* A host thread that issues one local rank's share of every frame (WCPT_GROUP_OPTION_THREADS). It spins for a while
 * after a frame (the next one usually follows within microseconds) and then sleeps on a condition variable. */
struct Worker {
    std::thread th;
    std::atomic<uint64_t> go{0};         /* sequence number of the frame to issue */
    std::atomic<bool> sleeping{false};
    std::mutex m;
    std::condition_variable cv;
    size_t local = 0;                    /* index of its rank in wcpt_group::local */
    int rc = 0;
};

} // namespace

struct wcpt_group {
    int nranks = 0;
    int root = 0;
    int transport = WCPT_GROUP_TRANSPORT_RCCL;
    bool overlap = true;
    bool broken = false;
    std::vector<LocalRank> local;       /* this process's ranks, in rank order */
    int root_local = -1;                /* index of the root in `local`, or -1 */
    uint32_t width = 0, height = 0;
    int format = 0;                     /* WCPT_PAYLOAD_* of the presented frame; 0 = not presenting */
    uint64_t dst = 0, dst_bytes = 0;    /* the presented frame on the root device (root's process only) */
    uint64_t frames = 0;
    std::vector<wcpt::plan::RankState> plan_state; /* scratch of wcpt_group_render (no per-frame allocation) */
    std::vector<wcpt::plan::Step> steps;
    /* WCPT_GROUP_OPTION_THREADS: 0 (default) off, 1 on, -1 on when this process's ranks span more than one device
     * (COPY, DIRECT). Off by default: the threaded issue has run only with every rank on one device. */
    int threads = 0;
    /* WCPT_GROUP_OPTION_TIMEOUT_MS: -1 (default) = kDefaultTimeoutMs in a group of several ranks, none in a group of
     * one; 0 = wait forever */
    int timeout_ms = -1;
    /* WCPT_GROUP_OPTION_ROW_STRIPE: rows per interleaved stripe, 0 = contiguous row blocks */
    uint32_t stripe = 0;
    std::vector<std::unique_ptr<Worker>> workers; /* local ranks 1..n-1 (the caller's thread issues local rank 0) */
    std::atomic<bool> stopping{false};
    std::atomic<uint32_t> done{0};
    uint64_t seq = 0;
    /* the frame the workers issue (valid while wcpt_group_render waits for them) */
    const wcpt_scene_data* job_scene = nullptr;
    const uint64_t* job_m = nullptr;
    const uint64_t* job_s = nullptr;
    const uint64_t* job_d = nullptr;
    bool job_exchange = false;
};

namespace {

int group_error(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    return wcpt::context_error(nullptr, code, buf);
}

int hip_fail(hipError_t e, const char* what)
{
    (void)hipGetLastError();
    return group_error(e == hipErrorOutOfMemory ? WCPT_ERROR_OUT_OF_DEVICE_MEMORY : WCPT_ERROR_DEVICE_LOST, "%s: %s",
                       what, hipGetErrorString(e));
}

#define GHIP(expr, what)                          \
    do {                                          \
        hipError_t _e = (expr);                   \
        if (_e != hipSuccess) return hip_fail(_e, (what)); \
    } while (0)

int nccl_fail(ncclResult_t e, const char* what)
{
    return group_error(WCPT_ERROR_DEVICE_LOST, "%s: %s", what, ncclGetErrorString(e));
}

uint64_t pixel_bytes(int format) { return format == WCPT_PAYLOAD_DISPLAY_RGBA8 ? 4u : 4ull * (uint64_t)format; }

bool valid_format(int f)
{
    return f == WCPT_PAYLOAD_RGB32F || f == WCPT_PAYLOAD_RGBA32F || f == WCPT_PAYLOAD_DISPLAY_RGBA8;
}

/* rank's rows: a contiguous block, or its first stripe's row and its row count (WCPT_GROUP_OPTION_ROW_STRIPE) */
void block_of(const wcpt_group* g, int rank, uint32_t& y0, uint32_t& rows)
{
    (void)wcpt_row_stripes(g->height, (uint32_t)g->nranks, (uint32_t)rank, g->stripe, &y0, &rows);
}

/* Where rank's `rows` rows sit in the frame relative to its first (row_map.h): stripes of g->stripe rows every
 * nranks * stripe rows. Rank `rank`'s rows, back to back at `src` (px bytes per pixel), to their rows of `frame`:
 * one 2D copy of its whole stripes (pitch nranks * stripe rows in the frame, stripe rows at the source) and one copy
 * of its short last stripe, if it holds one. hipMemcpyDefault: the source may be another device's memory (COPY). */
hipError_t copy_stripes(const wcpt_group* g, int rank, void* frame, const void* src, uint64_t px, hipStream_t s)
{
    uint32_t y0 = 0, rows = 0;
    block_of(g, rank, y0, rows);
    const uint64_t row = (uint64_t)g->width * px;
    const uint64_t S = g->stripe, P = S * (uint64_t)g->nranks;
    const uint64_t full = rows / S, tail = rows % S;
    char* dst = static_cast<char*>(frame) + (uint64_t)y0 * row;
    hipError_t e = hipSuccess;
    if (full) e = hipMemcpy2DAsync(dst, P * row, src, S * row, S * row, full, hipMemcpyDefault, s);
    if (e == hipSuccess && tail)
        e = hipMemcpyAsync(dst + full * P * row, static_cast<const char*>(src) + full * S * row, tail * row,
                           hipMemcpyDefault, s);
    return e;
}

bool presenting(const wcpt_group* g) { return g->format != 0 && g->width != 0; }

/* Retire a payload buffer: queued renders and transfers may still touch it, so it is freed at the next group-wide wait
 * (free_retired). */
void release_payload(LocalRank& lr, int b)
{
    if (lr.payload[b]) lr.retired.push_back(lr.payload[b]);
    lr.payload[b] = nullptr;
    lr.payload_cap[b] = 0;
    lr.sent_pending[b] = false;
}

/* Free a rank's retired payloads; its render and communication streams have drained. */
void free_retired(LocalRank& lr)
{
    if (lr.retired.empty()) return;
    (void)hipSetDevice(lr.device);
    for (void* p : lr.retired) (void)hipFree(p);
    lr.retired.clear();
}

/* Size every sending rank's payload buffers for the current frame and format (replaced ones are retired: no device sync) and
 * point the root's render at its block of the presented frame. Called after a screen or output change. */
int attach_payloads(wcpt_group* g)
{
    for (LocalRank& lr : g->local) {
        int rc = wcpt_set_option(lr.ctx, WCPT_OPTION_GATHER_FRAME_ROWS, 0);
        if (rc) return rc;
        if (!presenting(g)) {
            rc = wcpt_set_gather_output(lr.ctx, 0, 0, 0);
            if (rc) return rc;
            continue;
        }
        uint32_t y0 = 0, rows = 0;
        block_of(g, lr.rank, y0, rows);
        const uint64_t bytes = (uint64_t)g->width * rows * pixel_bytes(g->format);
        if (lr.rank == g->root || g->transport == WCPT_GROUP_TRANSPORT_DIRECT) {
            /* the root renders into its rows of the frame; with the DIRECT transport every rank does, over xGMI */
            if (g->stripe) {
                /* interleaved stripes: the output is the whole frame, addressed by frame row */
                rc = wcpt_set_option(lr.ctx, WCPT_OPTION_GATHER_FRAME_ROWS, 1);
                if (!rc) rc = wcpt_set_gather_output(lr.ctx, g->dst, g->dst_bytes, (uint32_t)g->format);
            } else {
                rc = wcpt_set_gather_output(lr.ctx, g->dst + (uint64_t)g->width * y0 * pixel_bytes(g->format), bytes,
                                            (uint32_t)g->format);
            }
            if (rc) return rc;
            if (lr.rank == g->root && g->stripe && g->transport == WCPT_GROUP_TRANSPORT_RCCL && g->nranks > 1) {
                /* the senders' blocks arrive back to back in the staging buffer, then go to their rows (kScatter) */
                const uint64_t need = (uint64_t)g->width * (g->height - rows) * pixel_bytes(g->format);
                if (lr.stage_cap < need) {
                    GHIP(hipSetDevice(lr.device), "hipSetDevice");
                    if (lr.stage) lr.retired.push_back(lr.stage);
                    lr.stage = nullptr;
                    lr.stage_cap = 0;
                    const hipError_t e = hipMalloc(&lr.stage, need);
                    if (e != hipSuccess) {
                        lr.stage = nullptr;
                        (void)hipGetLastError();
                        return group_error(WCPT_ERROR_OUT_OF_DEVICE_MEMORY, "hipMalloc(staging of the root, %llu bytes): %s",
                                           (unsigned long long)need, hipGetErrorString(e));
                    }
                    lr.stage_cap = need;
                }
            }
            continue;
        }
        GHIP(hipSetDevice(lr.device), "hipSetDevice");
        for (int b = 0; b < kPayloadBuffers; b++) {
            if (lr.payload_cap[b] >= bytes) continue;
            release_payload(lr, b);
            const hipError_t e = hipMalloc(&lr.payload[b], bytes);
            if (e != hipSuccess) {
                lr.payload[b] = nullptr;
                (void)hipGetLastError();
                return group_error(WCPT_ERROR_OUT_OF_DEVICE_MEMORY, "hipMalloc(payload of rank %d, %llu bytes): %s",
                                   lr.rank, (unsigned long long)bytes, hipGetErrorString(e));
            }
            lr.payload_cap[b] = bytes;
        }
        /* the next render picks its buffer; park the output on buffer 0 meanwhile */
        rc = wcpt_set_gather_output(lr.ctx, reinterpret_cast<uint64_t>(lr.payload[0]), bytes, (uint32_t)g->format);
        if (rc) return rc;
    }
    return WCPT_SUCCESS;
}

/* Set up everything a local rank needs beyond its context (created by the caller). A group of one has no exchange and
 * gets no communication stream: its device keeps exactly the context's streams (the wavefront pipelines' streams sit
 * close to the device's hardware-queue limit). */
int init_local(LocalRank& lr, int nranks)
{
    GHIP(hipSetDevice(lr.device), "hipSetDevice");
    if (nranks > 1)
        GHIP(hipStreamCreateWithFlags(&lr.comm_stream, hipStreamNonBlocking), "hipStreamCreate(communication)");
    for (int b = 0; b < kPayloadBuffers; b++) {
        GHIP(hipEventCreateWithFlags(&lr.ready[b], hipEventDisableTiming), "hipEventCreate");
        GHIP(hipEventCreateWithFlags(&lr.sent[b], hipEventDisableTiming), "hipEventCreate");
    }
    return WCPT_SUCCESS;
}

/* A transport failure inside a posted exchange: the communicators may hold half-matched operations, so abort them
 * (their kernels are torn down) and refuse further frames. */
int break_group(wcpt_group* g, int rc)
{
    g->broken = true;
    for (LocalRank& lr : g->local)
        if (lr.comm) {
            (void)ncclCommAbort(lr.comm);
            lr.comm = nullptr;
        }
    return rc;
}

/* An error that only this process can have seen (a device failure, a check on the root's own destination) in a group
 * whose other ranks live in other processes: those processes go on and post their part of the next frame's exchange,
 * which this one no longer matches, so the group is broken here (its communicator aborted) rather than left to hang.
 * In a one-process group every rank sees the same error and the group stays usable. */
int split_refusal(wcpt_group* g, int rc)
{
    return (int)g->local.size() < g->nranks ? break_group(g, rc) : rc;
}

int alloc_group(int nranks, int root, int transport, wcpt_group** out)
{
    wcpt_group* g = new (std::nothrow) wcpt_group();
    if (!g) return group_error(WCPT_ERROR_OUT_OF_HOST_MEMORY, "out of host memory");
    g->nranks = nranks;
    g->root = root;
    g->transport = transport;
    *out = g;
    return WCPT_SUCCESS;
}

int device_count()
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return count;
}

} // namespace

namespace {

/* Issue the planned steps of rank `only` (-1: of every local rank, in plan order) for the frame in g->steps. Every
 * error it returns must break the group (issue_frame does, once every issuing thread has finished). Issued from the caller's thread, or from a rank's worker thread: a rank's steps
 * touch only that rank's context, streams, events and communicator (and, COPY transport, the root's frame through the
 * sender's own device), so ranks issue independently; device-side order between them is the events'. */
int run_steps(wcpt_group* g, int only, const wcpt_scene_data* scene, const uint64_t* materials, const uint64_t* spheres,
              const uint64_t* draw_commands, bool exchange)
{
    const size_t nl = g->local.size();
    const uint64_t px = exchange ? pixel_bytes(g->format) : 0;
    auto local_index = [&](int rank) -> size_t {
        for (size_t i = 0; i < nl; i++)
            if (g->local[i].rank == rank) return i;
        return 0; /* the plan names local ranks only */
    };
    auto stream_of = [&](LocalRank& lr, int s) {
        return s == plan::kCommStream ? lr.comm_stream : wcpt::context_stream(lr.ctx);
    };
    auto block_bytes = [&](int rank) {
        uint32_t y0 = 0, rows = 0;
        block_of(g, rank, y0, rows);
        return (uint64_t)g->width * rows * px;
    };
    auto frame_rows = [&](int rank) {
        uint32_t y0 = 0, rows = 0;
        block_of(g, rank, y0, rows);
        return reinterpret_cast<void*>(g->dst + (uint64_t)g->width * y0 * px);
    };
    /* row stripes, RCCL: where rank `peer`'s block lands in the root's staging buffer (the senders' blocks in rank
     * order, back to back) */
    auto stage_of = [&](const LocalRank& rt, int peer) {
        uint64_t off = 0;
        for (int r = 0; r < peer; r++)
            if (r != g->root) off += block_bytes(r);
        return static_cast<void*>(static_cast<char*>(rt.stage) + off);
    };
    /* 2-5 may fail only on a device or transport error. Once the plan has started, ranks (and, in a group of several
     * processes, the peers posting their part of this frame's exchange) are out of step, so any failure breaks the
     * group -- the same rule for a failing hipEventRecord / hipStreamWaitEvent / copy as for a failing render. */
#define PHIP(expr, what)                                     \
    do {                                                     \
        hipError_t _e = (expr);                              \
        if (_e != hipSuccess) return hip_fail(_e, (what));   \
    } while (0)
    bool in_group = false; /* inside ncclGroupStart: every transfer argument was fixed above, so a failure below is
                            * the transport's, and a half-posted exchange is aborted rather than launched */
    ncclResult_t xfer_err = ncclSuccess;
    const char* xfer_what = "";
    for (const plan::Step& st : g->steps) {
        if (only >= 0 && st.rank != only) continue;
        const size_t i = local_index(st.rank);
        LocalRank& lr = g->local[i];
        STEP_TIMER(st.op & 7);
        if (in_group && st.op != plan::kSend && st.op != plan::kRecv) {
            in_group = false;
            const ncclResult_t e = ncclGroupEnd();
            if (xfer_err != ncclSuccess) return nccl_fail(xfer_err, xfer_what);
            if (e != ncclSuccess) return nccl_fail(e, "ncclGroupEnd");
        }
        switch (st.op) {
        case plan::kWaitSent: {
            /* every stream the next frame may render on waits for the payload's previous transfer: the context's
             * stream and, while the frame overlap holds frames on them, its pipe streams (no join) */
            PHIP(hipSetDevice(lr.device), "hipSetDevice");
            hipStream_t fs[wcpt::kMaxFrameStreams];
            const int n = wcpt::context_frame_streams(lr.ctx, fs, wcpt::kMaxFrameStreams);
            for (int k = 0; k < n; k++)
                PHIP(hipStreamWaitEvent(fs[k], lr.sent[st.buffer], 0), "hipStreamWaitEvent(sent)");
            break;
        }
        case plan::kSetOutput: {
            const uint64_t bytes = block_bytes(lr.rank);
            if (!lr.payload[st.buffer] || lr.payload_cap[st.buffer] < bytes)
                return group_error(WCPT_ERROR_INVALID_ARGUMENT, "rank %d: payload missing (set the output again)",
                                   lr.rank);
            const int rc = wcpt_set_gather_output(lr.ctx, reinterpret_cast<uint64_t>(lr.payload[st.buffer]), bytes,
                                                  (uint32_t)g->format);
            if (rc) return rc;
            break;
        }
        case plan::kRender: {
            /* validated: a failure now is a device/launch failure, and the ranks are out of step */
            const int rc = wcpt_render(lr.ctx, scene, materials[i], spheres[i], draw_commands[i]);
            if (rc) return rc;
            break;
        }
        case plan::kRecordReady: {
            /* the frame is complete when the context's stream and every pipe stream holding part of it are: one event
             * on each (in line transfers run on the render stream, whose frames are joined: one stream) */
            PHIP(hipSetDevice(lr.device), "hipSetDevice");
            hipStream_t fs[wcpt::kMaxFrameStreams];
            const int n = g->overlap ? wcpt::context_frame_streams(lr.ctx, fs, wcpt::kMaxFrameStreams) : 0;
            PHIP(hipEventRecord(lr.ready[st.buffer], n ? fs[0] : stream_of(lr, st.stream)), "hipEventRecord(ready)");
            for (int k = 1; k < n; k++) {
                hipEvent_t& ev = lr.ready_pipe[st.buffer][k - 1];
                if (!ev) PHIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate(ready)");
                PHIP(hipEventRecord(ev, fs[k]), "hipEventRecord(ready)");
            }
            lr.ready_n[st.buffer] = n > 1 ? n : 1;
            break;
        }
        case plan::kCommWaitReady:
            PHIP(hipSetDevice(lr.device), "hipSetDevice");
            PHIP(hipStreamWaitEvent(stream_of(lr, st.stream), lr.ready[st.buffer], 0), "hipStreamWaitEvent(ready)");
            for (int k = 1; k < lr.ready_n[st.buffer]; k++)
                PHIP(hipStreamWaitEvent(stream_of(lr, st.stream), lr.ready_pipe[st.buffer][k - 1], 0),
                     "hipStreamWaitEvent(ready)");
            break;
        case plan::kSend:
            if (g->transport == WCPT_GROUP_TRANSPORT_COPY) {
                const LocalRank& rt = g->local[g->root_local]; /* the COPY transport is single-process */
                PHIP(hipSetDevice(lr.device), "hipSetDevice");
                if (g->stripe) {
                    PHIP(copy_stripes(g, lr.rank, reinterpret_cast<void*>(g->dst), lr.payload[st.buffer], px,
                                      stream_of(lr, st.stream)), "hipMemcpy2DAsync(stripes)");
                    break;
                }
                PHIP(hipMemcpyPeerAsync(frame_rows(lr.rank), rt.device, lr.payload[st.buffer], lr.device,
                                        block_bytes(lr.rank), stream_of(lr, st.stream)),
                     "hipMemcpyPeerAsync(block)");
                break;
            }
            /* fall through */
        case plan::kRecv:
            if (!in_group) {
                const ncclResult_t e = ncclGroupStart();
                if (e != ncclSuccess) return nccl_fail(e, "ncclGroupStart");
                in_group = true;
            }
            if (xfer_err != ncclSuccess) break; /* skip the rest; the group is ended and aborted below */
            if (st.op == plan::kSend) {
                xfer_err = ncclSend(lr.payload[st.buffer], block_bytes(lr.rank), ncclUint8, st.peer, lr.comm,
                                    stream_of(lr, st.stream));
                xfer_what = "ncclSend";
            } else {
                xfer_err = ncclRecv(g->stripe ? stage_of(lr, st.peer) : frame_rows(st.peer), block_bytes(st.peer),
                                    ncclUint8, st.peer, lr.comm, stream_of(lr, st.stream));
                xfer_what = "ncclRecv";
            }
            break;
        case plan::kScatter:
            PHIP(hipSetDevice(lr.device), "hipSetDevice");
            PHIP(copy_stripes(g, st.peer, reinterpret_cast<void*>(g->dst), stage_of(lr, st.peer), px,
                              stream_of(lr, st.stream)), "hipMemcpy2DAsync(received stripes)");
            break;
        case plan::kRecordSent:
            PHIP(hipSetDevice(lr.device), "hipSetDevice");
            PHIP(hipEventRecord(lr.sent[st.buffer], stream_of(lr, st.stream)), "hipEventRecord(sent)");
            lr.sent_pending[st.buffer] = true;
            break;
        default:
            return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group plan step %d", st.op);
        }
    }
    if (in_group) { /* a process holding only the root: its receives end the plan */
        const ncclResult_t e = ncclGroupEnd();
        if (xfer_err != ncclSuccess) return nccl_fail(xfer_err, xfer_what);
        if (e != ncclSuccess) return nccl_fail(e, "ncclGroupEnd");
    }
    return WCPT_SUCCESS;
#undef PHIP
}

/* The worker's loop: wait for a frame (spin ~kSpinUs, then sleep), issue its rank's steps, report. */
constexpr double kSpinUs = 200.0;

void worker_main(wcpt_group* g, Worker* w)
{
#if WCPT_GROUP_TIMERS
    t_worker = true;
#endif
    uint64_t seen = 0;
    for (;;) {
        const auto t0 = std::chrono::steady_clock::now();
        uint32_t spins = 0;
        while (w->go.load(std::memory_order_seq_cst) == seen && !g->stopping.load(std::memory_order_relaxed)) {
            __builtin_ia32_pause();
            if ((++spins & 255u) == 0 &&
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > kSpinUs) {
                std::unique_lock<std::mutex> lk(w->m);
                w->sleeping.store(true, std::memory_order_seq_cst);
                w->cv.wait(lk, [&] {
                    return w->go.load(std::memory_order_seq_cst) != seen || g->stopping.load(std::memory_order_seq_cst);
                });
                w->sleeping.store(false, std::memory_order_relaxed);
            }
        }
        if (g->stopping.load(std::memory_order_acquire)) return;
        seen = w->go.load(std::memory_order_acquire);
        w->rc = run_steps(g, g->local[w->local].rank, g->job_scene, g->job_m, g->job_s, g->job_d, g->job_exchange);
        g->done.fetch_add(1, std::memory_order_release);
    }
}

void stop_workers(wcpt_group* g)
{
    if (g->workers.empty()) return;
    g->stopping.store(true, std::memory_order_seq_cst);
    for (auto& w : g->workers) {
        std::lock_guard<std::mutex> lk(w->m);
        w->cv.notify_one();
    }
    for (auto& w : g->workers)
        if (w->th.joinable()) w->th.join();
    g->workers.clear();
    g->stopping.store(false);
}

bool use_threads(const wcpt_group* g)
{
    if (g->local.size() < 2 || g->threads == 0) return false;
    if (g->threads == 1) return true;
    /* auto: COPY / DIRECT groups over several devices. A one-process RCCL group keeps the single-thread form (every
     * frame's sends and receives in one ncclGroupStart/End, rccl.h:700,722) unless threads are asked for: its
     * thread-per-device form is RCCL's other supported pattern, but no multi-GPU box here has run it. */
    if (g->transport == WCPT_GROUP_TRANSPORT_RCCL) return false;
    for (const LocalRank& lr : g->local)
        if (lr.device != g->local[0].device) return true;
    return false;
}

/* Issue the planned frame: from the caller's thread alone, or with every local rank but the first issued by its own
 * worker thread at the same time (the caller issues the first and waits until every worker has issued its share, so
 * the call returns with the whole frame enqueued, as in the one-thread mode; nothing waits for the device). */
int issue_frame(wcpt_group* g, const wcpt_scene_data* scene, const uint64_t* materials, const uint64_t* spheres,
                const uint64_t* draw_commands, bool exchange)
{
    const size_t nl = g->local.size();
    if (!use_threads(g)) {
        const int rc = run_steps(g, -1, scene, materials, spheres, draw_commands, exchange);
        if (rc) return break_group(g, rc);
        g->frames++;
        return WCPT_SUCCESS;
    }
    if (g->workers.size() != nl - 1) {
        stop_workers(g);
        try {
            for (size_t i = 1; i < nl; i++) {
                g->workers.emplace_back(new Worker());
                Worker* w = g->workers.back().get();
                w->local = i;
                w->th = std::thread(worker_main, g, w);
            }
        } catch (...) {
            stop_workers(g);
            return group_error(WCPT_ERROR_OUT_OF_HOST_MEMORY, "could not start the group's issue threads");
        }
    }
    g->job_scene = scene;
    g->job_m = materials;
    g->job_s = spheres;
    g->job_d = draw_commands;
    g->job_exchange = exchange;
    g->done.store(0, std::memory_order_relaxed);
    const uint64_t seq = ++g->seq;
    for (auto& w : g->workers) {
        w->go.store(seq, std::memory_order_seq_cst);
        if (w->sleeping.load(std::memory_order_seq_cst)) {
            std::lock_guard<std::mutex> lk(w->m);
            w->cv.notify_one();
        }
    }
    int rc = run_steps(g, g->local[0].rank, scene, materials, spheres, draw_commands, exchange);
    const uint32_t want = (uint32_t)g->workers.size();
    for (uint32_t spins = 0; g->done.load(std::memory_order_acquire) != want; spins++) {
        if (spins < 4096u)
            __builtin_ia32_pause();
        else
            std::this_thread::yield();
    }
    for (auto& w : g->workers)
        if (!rc && w->rc) rc = w->rc;
    if (rc) return break_group(g, rc);
    g->frames++;
    return WCPT_SUCCESS;
}

double now_ms()
{
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

double timeout_of(const wcpt_group* g)
{
    if (g->timeout_ms >= 0) return (double)g->timeout_ms;
    return g->nranks > 1 ? (double)kDefaultTimeoutMs : 0.0;
}

/* Wait, bounded (group_wait.h), until local rank lr's render stream and communication stream have drained. Returns
 * WCPT_SUCCESS; a failed poll (hip_fail); or, on an RCCL asynchronous error or the deadline t0 + the group's timeout,
 * WCPT_ERROR_DEVICE_LOST with the communicators aborted (break_group): the frame's exchange cannot complete, since a
 * peer failed or did not post its part. */
int wait_rank(wcpt_group* g, LocalRank& lr, double t0)
{
    const hipStream_t streams[2] = {wcpt::context_stream(lr.ctx), lr.comm_stream};
    const char* names[2] = {"render", "communication"};
    for (int k = 0; k < 2; k++) {
        if (!streams[k]) continue;
        if (hipSetDevice(lr.device) != hipSuccess) return hip_fail(hipGetLastError(), "hipSetDevice");
        hipError_t failed = hipSuccess;
        ncclResult_t async = ncclSuccess;
        const gwait::Result r = gwait::wait_for(
            [&]() {
                const hipError_t e = hipStreamQuery(streams[k]);
                if (e == hipSuccess) return (int)gwait::kReady;
                if (e == hipErrorNotReady) return (int)gwait::kBusy;
                failed = e;
                return (int)gwait::kPollError;
            },
            [&]() {
                if (!lr.comm) return false;
                ncclResult_t a = ncclSuccess;
                if (ncclCommGetAsyncError(lr.comm, &a) != ncclSuccess) return false;
                if (a == ncclSuccess || a == ncclInProgress) return false;
                async = a;
                return true;
            },
            t0, timeout_of(g), now_ms,
            [](double us) { std::this_thread::sleep_for(std::chrono::duration<double, std::micro>(us)); });
        switch (r) {
        case gwait::kDone:
            break;
        case gwait::kFailed:
            (void)hipGetLastError();
            return hip_fail(failed, names[k][0] == 'r' ? "hipStreamQuery(render)" : "hipStreamQuery(communication)");
        case gwait::kTransportError:
            return break_group(g, group_error(WCPT_ERROR_DEVICE_LOST, "rank %d: RCCL asynchronous error on the %s "
                                              "stream: %s (communicators aborted)", lr.rank, names[k],
                                              ncclGetErrorString(async)));
        case gwait::kTimedOut:
            return break_group(g, group_error(WCPT_ERROR_DEVICE_LOST, "rank %d: the %s stream did not drain within "
                                              "%.0f ms (WCPT_GROUP_OPTION_TIMEOUT_MS): a peer failed or did not post "
                                              "its part of a frame's exchange (communicators aborted)", lr.rank,
                                              names[k], timeout_of(g)));
        }
    }
    return WCPT_SUCCESS;
}

/* After the communicators were aborted: give the streams a bounded time to drain (RCCL's aborted kernels exit), so
 * that destroying the group does not block on them. */
void drain_after_abort(wcpt_group* g)
{
    const double t0 = now_ms();
    const int saved = g->timeout_ms;
    const double bound = timeout_of(g);
    g->timeout_ms = bound > 0.0 && bound < 10000.0 ? (int)bound : 10000;
    for (LocalRank& lr : g->local) (void)wait_rank(g, lr, t0);
    g->timeout_ms = saved;
    (void)hipGetLastError();
}

} // namespace

extern "C" {

int wcpt_group_create_ex(const int* devices, int n, int root, int transport, wcpt_group** out)
{
    if (!out) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (!devices || n < 1) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group of %d devices", n);
    if (root < 0 || root >= n) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "root %d outside [0,%d)", root, n);
    if (transport != WCPT_GROUP_TRANSPORT_RCCL && transport != WCPT_GROUP_TRANSPORT_COPY &&
        transport != WCPT_GROUP_TRANSPORT_DIRECT)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group transport %d", transport);
    const int count = device_count();
    if (count == 0) return group_error(WCPT_ERROR_INITIALIZATION_FAILED, "no HIP device available");
    for (int r = 0; r < n; r++) {
        if (devices[r] < 0 || devices[r] >= count)
            return group_error(WCPT_ERROR_INVALID_ARGUMENT, "device %d out of range [0,%d)", devices[r], count);
        for (int q = 0; q < r && transport == WCPT_GROUP_TRANSPORT_RCCL; q++)
            if (devices[q] == devices[r])
                return group_error(WCPT_ERROR_INVALID_ARGUMENT,
                                   "device %d listed twice (RCCL: one rank per device; WCPT_GROUP_TRANSPORT_COPY allows it)",
                                   devices[r]);
    }
    wcpt_group* g = nullptr;
    int rc = alloc_group(n, root, transport, &g);
    if (rc) return rc;
    g->local.resize(n);
    g->root_local = root;
    for (int r = 0; r < n; r++) {
        LocalRank& lr = g->local[r];
        lr.rank = r;
        lr.device = devices[r];
        rc = wcpt_create(devices[r], &lr.ctx);
        if (!rc) rc = init_local(lr, n);
        if (rc) {
            wcpt_group_destroy(g);
            return rc;
        }
    }
    if (n > 1 && transport == WCPT_GROUP_TRANSPORT_RCCL) {
        std::vector<ncclComm_t> comms(n, nullptr);
        const ncclResult_t e = ncclCommInitAll(comms.data(), n, devices);
        if (e != ncclSuccess) {
            wcpt_group_destroy(g);
            return nccl_fail(e, "ncclCommInitAll");
        }
        for (int r = 0; r < n; r++) g->local[r].comm = comms[r];
    }
    if (n > 1 && (transport == WCPT_GROUP_TRANSPORT_COPY || transport == WCPT_GROUP_TRANSPORT_DIRECT)) {
        /* each sender writes into the root's frame: give its device access to the root's memory (xGMI peer access
         * where the pair supports it; otherwise, COPY only, hipMemcpyPeerAsync stages the copy) */
        for (int r = 0; r < n; r++) {
            if (r == root || devices[r] == devices[root]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, devices[r], devices[root]) == hipSuccess && can) {
                (void)hipSetDevice(devices[r]);
                const hipError_t e = hipDeviceEnablePeerAccess(devices[root], 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
                    wcpt_group_destroy(g);
                    return hip_fail(e, "hipDeviceEnablePeerAccess");
                }
            } else if (transport == WCPT_GROUP_TRANSPORT_DIRECT) {
                (void)hipGetLastError();
                wcpt_group_destroy(g);
                return group_error(WCPT_ERROR_INITIALIZATION_FAILED,
                                   "DIRECT transport: device %d cannot access the root's device %d (no peer access)",
                                   devices[r], devices[root]);
            }
            (void)hipGetLastError();
        }
    }
    *out = g;
    return WCPT_SUCCESS;
}

int wcpt_group_create(const int* devices, int n, int root, wcpt_group** out)
{
    return wcpt_group_create_ex(devices, n, root, WCPT_GROUP_TRANSPORT_RCCL, out);
}

int wcpt_group_unique_id(uint8_t* id)
{
    if (!id) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "null id");
    ncclUniqueId u;
    const ncclResult_t e = ncclGetUniqueId(&u);
    if (e != ncclSuccess) return nccl_fail(e, "ncclGetUniqueId");
    std::memcpy(id, &u, sizeof(u));
    return WCPT_SUCCESS;
}

int wcpt_group_create_rank(int device, int nranks, int rank, int root, const uint8_t* id, wcpt_group** out)
{
    if (!out) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (nranks < 1 || rank < 0 || rank >= nranks)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "rank %d of %d", rank, nranks);
    if (root < 0 || root >= nranks) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "root %d outside [0,%d)", root, nranks);
    if (nranks > 1 && !id) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "null unique id");
    const int count = device_count();
    if (count == 0) return group_error(WCPT_ERROR_INITIALIZATION_FAILED, "no HIP device available");
    if (device < 0 || device >= count)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "device %d out of range [0,%d)", device, count);
    wcpt_group* g = nullptr;
    int rc = alloc_group(nranks, root, WCPT_GROUP_TRANSPORT_RCCL, &g);
    if (rc) return rc;
    g->local.resize(1);
    g->root_local = rank == root ? 0 : -1;
    LocalRank& lr = g->local[0];
    lr.rank = rank;
    lr.device = device;
    rc = wcpt_create(device, &lr.ctx);
    if (!rc) rc = init_local(lr, nranks);
    if (rc) {
        wcpt_group_destroy(g);
        return rc;
    }
    if (nranks > 1) {
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof(u));
        (void)hipSetDevice(device);
        const ncclResult_t e = ncclCommInitRank(&lr.comm, nranks, u, rank);
        if (e != ncclSuccess) {
            lr.comm = nullptr;
            wcpt_group_destroy(g);
            return nccl_fail(e, "ncclCommInitRank");
        }
    }
    *out = g;
    return WCPT_SUCCESS;
}

int wcpt_group_destroy(wcpt_group* g)
{
    if (!g) return WCPT_SUCCESS;
    stop_workers(g);
#if WCPT_GROUP_TIMERS
    {
        static const char* names[10] = {"wait_sent", "set_output", "render", "record_ready", "comm_wait_ready",
                                        "send", "recv", "record_sent", "validate", ""};
        std::fprintf(stderr, "group_timers ranks=%d frames=%llu", g->nranks, (unsigned long long)g->frames);
        for (int k = 0; k < 9; k++)
            if (g_timers.n[k])
                std::fprintf(stderr, " %s=%.2fus/frame(%.2fus/call)", names[k],
                             g_timers.ns[k] / 1e3 / (g->frames ? g->frames : 1), g_timers.ns[k] / 1e3 / g_timers.n[k]);
        std::fprintf(stderr, "\n");
        g_timers = StepTimers();
    }
#endif
    {
        /* bounded, as in wcpt_group_sync: a peer that died leaves this process's transfers unmatched; abort them
         * (ncclCommAbort) rather than block here, then let the aborted work drain */
        const double t0 = now_ms();
        bool ok = true;
        for (LocalRank& lr : g->local)
            if (lr.ctx && wait_rank(g, lr, t0) != WCPT_SUCCESS) ok = false;
        if (!ok || g->broken) drain_after_abort(g);
    }
    for (LocalRank& lr : g->local) {
        if (lr.ctx) (void)wcpt_sync(lr.ctx);
        if (lr.comm_stream) {
            (void)hipSetDevice(lr.device);
            (void)hipStreamSynchronize(lr.comm_stream);
        }
    }
    for (LocalRank& lr : g->local)
        if (lr.comm) (void)ncclCommDestroy(lr.comm);
    for (LocalRank& lr : g->local) {
        (void)hipSetDevice(lr.device);
        for (int b = 0; b < kPayloadBuffers; b++) {
            if (lr.payload[b]) (void)hipFree(lr.payload[b]);
            if (lr.ready[b]) (void)hipEventDestroy(lr.ready[b]);
            if (lr.sent[b]) (void)hipEventDestroy(lr.sent[b]);
            for (hipEvent_t ev : lr.ready_pipe[b])
                if (ev) (void)hipEventDestroy(ev);
        }
        if (lr.stage) (void)hipFree(lr.stage);
        free_retired(lr);
        if (lr.comm_stream) {
            (void)hipStreamSynchronize(lr.comm_stream);
            (void)hipStreamDestroy(lr.comm_stream);
        }
        if (lr.ctx) wcpt_destroy(lr.ctx);
    }
    (void)hipGetLastError();
    delete g;
    return WCPT_SUCCESS;
}

wcpt_context* wcpt_group_context(wcpt_group* g, int rank)
{
    if (!g) return nullptr;
    for (LocalRank& lr : g->local)
        if (lr.rank == rank) return lr.ctx;
    return nullptr;
}

int wcpt_row_block(uint32_t height, uint32_t n, uint32_t rank, uint32_t* y0, uint32_t* rows)
{
    if (!y0 || !rows || n == 0 || rank >= n) return WCPT_ERROR_INVALID_ARGUMENT;
    const uint32_t a = (uint32_t)((uint64_t)rank * height / n);
    const uint32_t b = (uint32_t)((uint64_t)(rank + 1) * height / n);
    *y0 = a;
    *rows = b - a;
    return WCPT_SUCCESS;
}

int wcpt_row_stripes(uint32_t height, uint32_t n, uint32_t rank, uint32_t stripe, uint32_t* y_first, uint32_t* rows)
{
    if (stripe == 0) return wcpt_row_block(height, n, rank, y_first, rows);
    if (!y_first || !rows || n == 0 || rank >= n || (stripe & (stripe - 1u))) return WCPT_ERROR_INVALID_ARGUMENT;
    /* stripes s = rank, rank + n, ... below T = ceil(height / stripe); only the frame's last stripe can be short */
    const uint64_t T = ((uint64_t)height + stripe - 1u) / stripe;
    const uint64_t count = T > rank ? (T - 1u - rank) / n + 1u : 0u;
    uint64_t r = count * stripe;
    if (count && (T - 1u - rank) % n == 0 && height % stripe) r -= stripe - height % stripe; /* it holds the short one */
    *y_first = rank * stripe;
    *rows = (uint32_t)r;
    return WCPT_SUCCESS;
}

int wcpt_group_set_option(wcpt_group* g, int option, int value)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (option == WCPT_GROUP_OPTION_ROW_STRIPE) {
        if (value < 0 || value > 32768 || (value & (value - 1)))
            return group_error(WCPT_ERROR_INVALID_ARGUMENT, "row stripe %d (0, or a power of two up to 32768)", value);
        if (g->broken) return group_error(WCPT_ERROR_DEVICE_LOST, "group aborted after a transport failure");
        const int rc = wcpt_group_sync(g); /* queued frames keep the split they were issued with */
        if (rc) return rc;
        const uint32_t old = g->stripe;
        g->stripe = (uint32_t)value;
        if (g->width && old != g->stripe) {
            const int rc2 = wcpt_group_create_screen(g, g->width, g->height); /* lay the frame out again */
            if (rc2) {
                if (!g->broken) g->stripe = old;
                return rc2;
            }
        }
        return WCPT_SUCCESS;
    }
    if (option == WCPT_GROUP_OPTION_TIMEOUT_MS) {
        if (value < 0) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group timeout %d ms (>= 0; 0 = none)", value);
        g->timeout_ms = value;
        return WCPT_SUCCESS;
    }
    if (option == WCPT_GROUP_OPTION_THREADS) {
        if (value < -1 || value > 1) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group threads %d (-1, 0, 1)", value);
        g->threads = value;
        if (!use_threads(g)) stop_workers(g);
        return WCPT_SUCCESS;
    }
    if (option != WCPT_GROUP_OPTION_OVERLAP) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "unknown group option %d", option);
    const int rc = wcpt_group_sync(g); /* the streams' queued work follows the mode it was queued with */
    if (rc) return rc;
    g->overlap = value != 0;
    return WCPT_SUCCESS;
}

int wcpt_group_info_get(wcpt_group* g, wcpt_group_info* out)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (!out) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "null info");
    std::memset(out, 0, sizeof(*out));
    out->nranks = g->nranks;
    if (!g->local.empty() && g->local[0].comm) {
        int c = 0;
        const ncclResult_t e = ncclCommCount(g->local[0].comm, &c);
        if (e != ncclSuccess) return nccl_fail(e, "ncclCommCount");
        out->nranks = c;
    }
    out->local_ranks = (int32_t)g->local.size();
    out->first_local_rank = g->local.empty() ? -1 : g->local[0].rank;
    out->root = g->root;
    out->transport = g->transport;
    out->overlap = g->overlap ? 1 : 0;
    std::vector<int> seen;
    for (const LocalRank& lr : g->local) {
        bool dup = false;
        for (int d : seen) dup |= d == lr.device;
        if (!dup) seen.push_back(lr.device);
    }
    out->distinct_devices = (int32_t)seen.size();
    out->broken = g->broken ? 1 : 0;
    out->frames = g->frames;
    out->issue_threads = (int32_t)g->workers.size();
    return WCPT_SUCCESS;
}

int wcpt_group_create_screen(wcpt_group* g, uint32_t width, uint32_t height)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (g->broken) return group_error(WCPT_ERROR_DEVICE_LOST, "group aborted after a transport failure");
    if (width == 0 || height < (uint32_t)g->nranks) /* the same decision in every process */
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "%ux%u frame for %d row blocks", width, height, g->nranks);
    if (g->stripe && ((uint64_t)height + g->stripe - 1u) / g->stripe < (uint64_t)g->nranks)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "%ux%u frame: fewer stripes of %u rows than %d ranks", width,
                           height, g->stripe, g->nranks);
    const uint32_t old_w = g->width, old_h = g->height;
    g->width = width;
    g->height = height;
    for (LocalRank& lr : g->local) {
        /* the row-block split of SURVEY.md §8(e) (wcpt_row_block): blocks differ by at most one row; frame size and
         * block are set in one step, so no rank ever allocates more than its block (zeroed: CreateScreen) */
        uint32_t y0 = 0, rows = 0;
        block_of(g, lr.rank, y0, rows);
        const int rc = wcpt::set_frame_block(lr.ctx, width, height, y0, rows, g->stripe,
                                             g->stripe * (uint32_t)g->nranks);
        if (rc) {
            g->width = old_w;
            g->height = old_h;
            /* a device failure here is this process's alone: its ranks keep the old frame while the other processes'
             * take the new one, so the group cannot stay in step */
            return split_refusal(g, rc);
        }
    }
    /* every process knows the output's size (wcpt_group_set_output reads `bytes` everywhere), so this refusal is the
     * same in all of them and leaves the group usable */
    if (g->format && (uint64_t)width * height * pixel_bytes(g->format) > g->dst_bytes) {
        g->format = 0; /* the output no longer holds the frame: stop presenting until a new one is set */
        g->dst = g->dst_bytes = 0;
        const int rc = attach_payloads(g);
        if (rc) return split_refusal(g, rc);
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group output too small for %ux%u: set a new one", width, height);
    }
    const int rc = attach_payloads(g);
    return rc ? split_refusal(g, rc) : WCPT_SUCCESS;
}

int wcpt_group_set_output(wcpt_group* g, int format, uint64_t dst, uint64_t bytes)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (g->broken) return group_error(WCPT_ERROR_DEVICE_LOST, "group aborted after a transport failure");
    const bool holds_root = g->root_local >= 0;
    /* Decisions on (format, bytes) and the frame size, which every process of a wcpt_group_create_rank group is given
     * alike, are made alike everywhere and leave the group usable. Decisions only the root's process can make (its
     * `dst`) are collective failures there: the other processes would post their part of the next exchange. */
    const bool multi = (int)g->local.size() < g->nranks;
    if (format == 0 || (holds_root && dst == 0)) {
        g->format = 0;
        g->dst = g->dst_bytes = 0;
        const int rc = attach_payloads(g);
        if (rc) return split_refusal(g, rc);
        /* one process: a null destination turns presenting off. Several processes: only format 0 does so everywhere;
         * the others cannot see the root's destination and would go on sending */
        if (format != 0 && multi)
            return break_group(g, group_error(WCPT_ERROR_INVALID_ARGUMENT,
                                              "group output: null destination with format %d; turn presenting off "
                                              "with format 0 in every process", format));
        return WCPT_SUCCESS;
    }
    if (!valid_format(format)) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "output format %d (3, 4 or 8)", format);
    if (g->width && (uint64_t)g->width * g->height * pixel_bytes(format) > bytes)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group output of %llu bytes < %ux%u x %llu",
                           (unsigned long long)bytes, g->width, g->height, (unsigned long long)pixel_bytes(format));
    if (holds_root && ((dst & 3u) || (format == WCPT_PAYLOAD_RGBA32F && (dst & 15u))))
        return split_refusal(g, group_error(WCPT_ERROR_INVALID_ARGUMENT, "misaligned group output"));
    g->format = format;
    g->dst = holds_root ? dst : 0;
    g->dst_bytes = bytes;
    const int rc = attach_payloads(g);
    return rc ? split_refusal(g, rc) : WCPT_SUCCESS;
}

int wcpt_group_render(wcpt_group* g, const wcpt_scene_data* scene, const uint64_t* materials, const uint64_t* spheres,
                      const uint64_t* draw_commands)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (g->broken) return group_error(WCPT_ERROR_DEVICE_LOST, "group aborted after a transport failure");
    if (!scene || !materials || !spheres || !draw_commands)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "wcpt_group_render: null argument");
    if (!g->width) return group_error(WCPT_ERROR_NO_SCREEN, "wcpt_group_render: no screen (wcpt_group_create_screen)");
    const size_t nl = g->local.size();
    const bool exchange = presenting(g) && g->nranks > 1;
    /* 0. the senders' payload buffers (attach_payloads sized them; a failed attach leaves one missing): a refusal
     * before any device work, so a one-process group stays usable (split_refusal), instead of the plan's
     * set-output step failing after other ranks' steps were issued */
    if (exchange && g->transport != WCPT_GROUP_TRANSPORT_DIRECT) {
        for (const LocalRank& lr : g->local) {
            if (lr.rank == g->root) continue;
            uint32_t y0 = 0, rows = 0;
            block_of(g, lr.rank, y0, rows);
            const uint64_t bytes = (uint64_t)g->width * rows * pixel_bytes(g->format);
            for (int b = 0; b < kPayloadBuffers; b++)
                if (!lr.payload[b] || lr.payload_cap[b] < bytes)
                    return split_refusal(g, group_error(WCPT_ERROR_INVALID_ARGUMENT, "rank %d: payload missing (set "
                                                        "the output again)", lr.rank));
        }
    }
    /* 1. every rank's arguments first: an argument error leaves every accumulation image as it was. In a group whose
     * other ranks live in other processes, those processes still post their part of this frame's exchange; this one
     * cannot, so its communicator is aborted (the exchange fails there instead of waiting for a send that never
     * comes) and the group is unusable -- the collective contract of wcpt_group_create_rank. */
    {
        STEP_TIMER(8);
        for (size_t i = 0; i < nl; i++) {
            const int rc = wcpt::render_validate(g->local[i].ctx, scene, materials[i], spheres[i], draw_commands[i]);
            if (rc) {
                for (size_t j = 0; j < i; j++) wcpt::render_abandon(g->local[j].ctx);
                return (exchange && (int)nl < g->nranks) ? break_group(g, rc) : rc;
            }
        }
    }
    /* 2-5. the frame's device operations in the order of group_plan.h (tests/test_group_plan.py checks that order on
     * a simulated device): payload reuse behind the previous transfer, renders, ready events, transfers, sent events */
    g->plan_state.resize(nl);
    for (size_t i = 0; i < nl; i++) {
        /* transfers in line with the renders (GROUP_OPTION_OVERLAP 0) run on the render stream, which joins the
         * context's frames every frame: no frame overlap there. With the communication streams a sender fences each
         * frame on every stream that holds part of it (kRecordReady) and its pipes run on */
        wcpt::set_overlap_suppressed(g->local[i].ctx, exchange && g->transport != WCPT_GROUP_TRANSPORT_DIRECT &&
                                                          !g->overlap);
        g->plan_state[i].rank = g->local[i].rank;
        for (int k = 0; k < kPayloadBuffers; k++) g->plan_state[i].sent_pending[k] = g->local[i].sent_pending[k];
    }
    plan::frame_steps(g->nranks, g->root, g->overlap, exchange, g->transport, g->frames, g->plan_state, g->steps,
                      g->stripe != 0);
    return issue_frame(g, scene, materials, spheres, draw_commands, exchange);
}

int wcpt_group_sync(wcpt_group* g)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    /* bounded: poll every local rank's streams (group_wait.h) instead of blocking in hipStreamSynchronize, so a peer
     * that failed or skipped a frame ends in WCPT_ERROR_DEVICE_LOST after the group's timeout, not in a hang */
    const double t0 = now_ms();
    int first = WCPT_SUCCESS;
    for (LocalRank& lr : g->local) {
        int rc = wait_rank(g, lr, t0);
        if (!rc) rc = wcpt_sync(lr.ctx); /* drained: returns at once, with the render status (stack overflow) */
        if (!rc) free_retired(lr);
        if (!rc && lr.comm) {
            ncclResult_t async = ncclSuccess;
            if (ncclCommGetAsyncError(lr.comm, &async) == ncclSuccess && async != ncclSuccess &&
                async != ncclInProgress)
                rc = break_group(g, nccl_fail(async, "RCCL asynchronous error"));
        }
        if (rc && !first) first = rc;
    }
    if (first && g->broken) drain_after_abort(g);
    if (!first && g->broken) first = group_error(WCPT_ERROR_DEVICE_LOST, "group aborted after a transport failure");
    return first;
}

} /* extern "C" */
