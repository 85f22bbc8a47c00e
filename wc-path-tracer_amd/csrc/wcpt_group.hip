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
#include <cstring>
#include <new>
#include <vector>

#include "../../include/wcpt.h"
#include "group_plan.h"
#include "pt_kernels.h"

static_assert(sizeof(ncclUniqueId) == WCPT_GROUP_UNIQUE_ID_BYTES, "WCPT_GROUP_UNIQUE_ID_BYTES");

namespace {

constexpr int kPayloadBuffers = wcpt::plan::kPayloadBuffers;
namespace plan = wcpt::plan;

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
    bool sent_pending[kPayloadBuffers] = {};
    std::vector<void*> retired;              /* replaced payload buffers, freed at the next group-wide wait */
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

void block_of(const wcpt_group* g, int rank, uint32_t& y0, uint32_t& rows)
{
    (void)wcpt_row_block(g->height, (uint32_t)g->nranks, (uint32_t)rank, &y0, &rows);
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
        if (!presenting(g)) {
            const int rc = wcpt_set_gather_output(lr.ctx, 0, 0, 0);
            if (rc) return rc;
            continue;
        }
        uint32_t y0 = 0, rows = 0;
        block_of(g, lr.rank, y0, rows);
        const uint64_t bytes = (uint64_t)g->width * rows * pixel_bytes(g->format);
        if (lr.rank == g->root) {
            const int rc = wcpt_set_gather_output(lr.ctx, g->dst + (uint64_t)g->width * y0 * pixel_bytes(g->format),
                                                  bytes, (uint32_t)g->format);
            if (rc) return rc;
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
        const int rc = wcpt_set_gather_output(lr.ctx, reinterpret_cast<uint64_t>(lr.payload[0]), bytes,
                                              (uint32_t)g->format);
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

extern "C" {

int wcpt_group_create_ex(const int* devices, int n, int root, int transport, wcpt_group** out)
{
    if (!out) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (!devices || n < 1) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group of %d devices", n);
    if (root < 0 || root >= n) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "root %d outside [0,%d)", root, n);
    if (transport != WCPT_GROUP_TRANSPORT_RCCL && transport != WCPT_GROUP_TRANSPORT_COPY)
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
    if (n > 1 && transport == WCPT_GROUP_TRANSPORT_COPY) {
        /* each sender writes into the root's frame: give its device access to the root's memory (xGMI peer access
         * where the pair supports it; otherwise hipMemcpyPeerAsync stages the copy) */
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
        }
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

int wcpt_group_set_option(wcpt_group* g, int option, int value)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
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
    return WCPT_SUCCESS;
}

int wcpt_group_create_screen(wcpt_group* g, uint32_t width, uint32_t height)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (g->broken) return group_error(WCPT_ERROR_DEVICE_LOST, "group aborted after a transport failure");
    if (width == 0 || height < (uint32_t)g->nranks)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "%ux%u frame for %d row blocks", width, height, g->nranks);
    const uint32_t old_w = g->width, old_h = g->height;
    g->width = width;
    g->height = height;
    for (LocalRank& lr : g->local) {
        /* the row-block split of SURVEY.md §8(e) (wcpt_row_block): blocks differ by at most one row; frame size and
         * block are set in one step, so no rank ever allocates more than its block (zeroed: CreateScreen) */
        uint32_t y0 = 0, rows = 0;
        block_of(g, lr.rank, y0, rows);
        const int rc = wcpt::set_frame_block(lr.ctx, width, height, y0, rows);
        if (rc) {
            g->width = old_w;
            g->height = old_h;
            return rc;
        }
    }
    if (g->format && g->root_local >= 0 && (uint64_t)width * height * pixel_bytes(g->format) > g->dst_bytes) {
        g->format = 0; /* the output no longer holds the frame: stop presenting until a new one is set */
        g->dst = g->dst_bytes = 0;
        const int rc = attach_payloads(g);
        if (rc) return rc;
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group output too small for %ux%u: set a new one", width, height);
    }
    return attach_payloads(g);
}

int wcpt_group_set_output(wcpt_group* g, int format, uint64_t dst, uint64_t bytes)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (g->broken) return group_error(WCPT_ERROR_DEVICE_LOST, "group aborted after a transport failure");
    const bool holds_root = g->root_local >= 0;
    if ((holds_root && dst == 0) || format == 0) {
        g->format = 0;
        g->dst = g->dst_bytes = 0;
        return attach_payloads(g);
    }
    if (!valid_format(format)) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "output format %d (3, 4 or 8)", format);
    if (holds_root) {
        if ((dst & 3u) || (format == WCPT_PAYLOAD_RGBA32F && (dst & 15u)))
            return group_error(WCPT_ERROR_INVALID_ARGUMENT, "misaligned group output");
        if (g->width && (uint64_t)g->width * g->height * pixel_bytes(format) > bytes)
            return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group output of %llu bytes < %ux%u x %llu",
                               (unsigned long long)bytes, g->width, g->height, (unsigned long long)pixel_bytes(format));
    }
    g->format = format;
    g->dst = holds_root ? dst : 0;
    g->dst_bytes = holds_root ? bytes : 0;
    return attach_payloads(g);
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
    /* 1. every rank's arguments first: an argument error leaves every accumulation image as it was. In a group whose
     * other ranks live in other processes, those processes still post their part of this frame's exchange; this one
     * cannot, so its communicator is aborted (the exchange fails there instead of waiting for a send that never
     * comes) and the group is unusable -- the collective contract of wcpt_group_create_rank. */
    for (size_t i = 0; i < nl; i++) {
        const int rc = wcpt::render_validate(g->local[i].ctx, scene, materials[i], spheres[i], draw_commands[i]);
        if (rc) return (exchange && (int)nl < g->nranks) ? break_group(g, rc) : rc;
    }
    /* 2-5. the frame's device operations in the order of group_plan.h (tests/test_group_plan.py checks that order on
     * a simulated device): payload reuse behind the previous transfer, renders, ready events, transfers, sent events */
    g->plan_state.resize(nl);
    for (size_t i = 0; i < nl; i++) {
        g->plan_state[i].rank = g->local[i].rank;
        for (int k = 0; k < kPayloadBuffers; k++) g->plan_state[i].sent_pending[k] = g->local[i].sent_pending[k];
    }
    plan::frame_steps(g->nranks, g->root, g->overlap, exchange, g->transport == WCPT_GROUP_TRANSPORT_COPY, g->frames,
                      g->plan_state, g->steps);
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
    bool in_group = false; /* inside ncclGroupStart: every transfer argument was fixed above, so a failure below is
                            * the transport's, and a half-posted exchange is aborted rather than launched */
    ncclResult_t xfer_err = ncclSuccess;
    const char* xfer_what = "";
    size_t renders = 0;
    for (const plan::Step& st : g->steps) {
        const size_t i = local_index(st.rank);
        LocalRank& lr = g->local[i];
        if (in_group && st.op != plan::kSend && st.op != plan::kRecv) {
            in_group = false;
            const ncclResult_t e = ncclGroupEnd();
            if (xfer_err != ncclSuccess) return break_group(g, nccl_fail(xfer_err, xfer_what));
            if (e != ncclSuccess) return break_group(g, nccl_fail(e, "ncclGroupEnd"));
        }
        switch (st.op) {
        case plan::kWaitSent:
            GHIP(hipSetDevice(lr.device), "hipSetDevice");
            GHIP(hipStreamWaitEvent(stream_of(lr, st.stream), lr.sent[st.buffer], 0), "hipStreamWaitEvent(sent)");
            break;
        case plan::kSetOutput: {
            const uint64_t bytes = block_bytes(lr.rank);
            if (!lr.payload[st.buffer] || lr.payload_cap[st.buffer] < bytes)
                return group_error(WCPT_ERROR_INVALID_ARGUMENT, "rank %d: payload missing (set the output again)", lr.rank);
            const int rc = wcpt_set_gather_output(lr.ctx, reinterpret_cast<uint64_t>(lr.payload[st.buffer]), bytes,
                                                  (uint32_t)g->format);
            if (rc) return rc;
            break;
        }
        case plan::kRender: {
            /* validated: a failure now is a device/launch failure, and the ranks are out of step */
            const int rc = wcpt_render(lr.ctx, scene, materials[i], spheres[i], draw_commands[i]);
            if (rc) {
                g->broken = true;
                return rc;
            }
            if (++renders == nl) g->frames++;
            break;
        }
        case plan::kRecordReady:
            GHIP(hipSetDevice(lr.device), "hipSetDevice");
            GHIP(hipEventRecord(lr.ready[st.buffer], stream_of(lr, st.stream)), "hipEventRecord(ready)");
            break;
        case plan::kCommWaitReady:
            GHIP(hipSetDevice(lr.device), "hipSetDevice");
            GHIP(hipStreamWaitEvent(stream_of(lr, st.stream), lr.ready[st.buffer], 0), "hipStreamWaitEvent(ready)");
            break;
        case plan::kSend:
            if (g->transport == WCPT_GROUP_TRANSPORT_COPY) {
                const LocalRank& rt = g->local[g->root_local]; /* the COPY transport is single-process */
                GHIP(hipSetDevice(lr.device), "hipSetDevice");
                GHIP(hipMemcpyPeerAsync(frame_rows(lr.rank), rt.device, lr.payload[st.buffer], lr.device,
                                        block_bytes(lr.rank), stream_of(lr, st.stream)),
                     "hipMemcpyPeerAsync(block)");
                break;
            }
            /* fall through */
        case plan::kRecv:
            if (!in_group) {
                const ncclResult_t e = ncclGroupStart();
                if (e != ncclSuccess) return break_group(g, nccl_fail(e, "ncclGroupStart"));
                in_group = true;
            }
            if (xfer_err != ncclSuccess) break; /* skip the rest; the group is ended and aborted below */
            if (st.op == plan::kSend) {
                xfer_err = ncclSend(lr.payload[st.buffer], block_bytes(lr.rank), ncclUint8, st.peer, lr.comm,
                                    stream_of(lr, st.stream));
                xfer_what = "ncclSend";
            } else {
                xfer_err = ncclRecv(frame_rows(st.peer), block_bytes(st.peer), ncclUint8, st.peer, lr.comm,
                                    stream_of(lr, st.stream));
                xfer_what = "ncclRecv";
            }
            break;
        case plan::kRecordSent:
            GHIP(hipSetDevice(lr.device), "hipSetDevice");
            GHIP(hipEventRecord(lr.sent[st.buffer], stream_of(lr, st.stream)), "hipEventRecord(sent)");
            lr.sent_pending[st.buffer] = true;
            break;
        default:
            return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group plan step %d", st.op);
        }
    }
    if (in_group) { /* a process holding only the root: its receives end the plan */
        const ncclResult_t e = ncclGroupEnd();
        if (xfer_err != ncclSuccess) return break_group(g, nccl_fail(xfer_err, xfer_what));
        if (e != ncclSuccess) return break_group(g, nccl_fail(e, "ncclGroupEnd"));
    }
    return WCPT_SUCCESS;
}

int wcpt_group_sync(wcpt_group* g)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    int first = WCPT_SUCCESS;
    for (LocalRank& lr : g->local) {
        int rc = wcpt_sync(lr.ctx);
        if (!rc && lr.comm_stream) {
            (void)hipSetDevice(lr.device);
            const hipError_t e = hipStreamSynchronize(lr.comm_stream);
            if (e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize(communication)");
        }
        if (!rc) free_retired(lr);
        if (!rc && lr.comm) {
            ncclResult_t async = ncclSuccess;
            if (ncclCommGetAsyncError(lr.comm, &async) == ncclSuccess && async != ncclSuccess)
                rc = break_group(g, nccl_fail(async, "RCCL asynchronous error"));
        }
        if (rc && !first) first = rc;
    }
    if (!first && g->broken) first = group_error(WCPT_ERROR_DEVICE_LOST, "group aborted after a transport failure");
    return first;
}

} /* extern "C" */
