/*
 * wcpt_group.hip — one frame on several devices from one host thread (include/wcpt.h wcpt_group_*).
 *
 * The reference renders every frame on one device from one thread (src/main.jai:185-194 -> Render,
 * src/PathTracingRenderer.jai:399-457). Every pixel is independent -- its seed depends only on the global (x, y,
 * frame) (pathTracer.comp:304) and the accumulation is per pixel (:314-323) -- so the frame partitions into row
 * blocks: rank r of N renders rows [r*H/N, (r+1)*H/N) on its own device, keeps only that block of the accumulation
 * image, and the union is bit-identical to a one-device render. The one exchange is presenting a frame: the blocks
 * go to the root device. That is a gather of unequal blocks (H/N need not be an integer), issued as grouped
 * point-to-point ncclSend / ncclRecv on the ranks' render streams (rccl.h:700,722), so each transfer follows its
 * rank's render in stream order and xGMI carries the 7 incoming blocks of an 8-GPU node over 7 links at once.
 * The communicator is ncclCommInitAll (rccl.h:236): one process, one communicator per device, which is how a
 * single-threaded host like the reference's drives RCCL (every call on several communicators inside one
 * ncclGroupStart/ncclGroupEnd).
 *
 * The payload is written by the render itself (wcpt_set_gather_output): the root renders its block straight into the
 * presented frame, the other ranks into a group-owned payload buffer on their device that the send reads.
 */
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdarg>
#include <cstdio>
#include <vector>

#include "../../include/wcpt.h"
#include "pt_kernels.h"

struct wcpt_group {
    int n = 0;
    int root = 0;
    std::vector<int> devices;
    std::vector<wcpt_context*> ctx;
    std::vector<ncclComm_t> comm;      /* n > 1 only */
    uint32_t width = 0, height = 0;
    std::vector<uint32_t> y0, rows;    /* row block of each rank */
    int format = 0;                    /* WCPT_PAYLOAD_* of the presented frame; 0 = not presenting */
    uint64_t dst = 0, dst_bytes = 0;   /* the presented frame on the root device */
    std::vector<void*> payload;        /* rank r != root: its block's payload on its device */
    std::vector<uint64_t> payload_cap;
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

uint64_t pixel_bytes(int format) { return format == WCPT_PAYLOAD_DISPLAY_RGBA8 ? 4u : 4ull * (uint64_t)format; }

bool valid_format(int f)
{
    return f == WCPT_PAYLOAD_RGB32F || f == WCPT_PAYLOAD_RGBA32F || f == WCPT_PAYLOAD_DISPLAY_RGBA8;
}

/* Point every rank's render at its payload: the root's block of the presented frame, or the rank's own buffer
 * (grown on demand). format == 0 turns the payloads off. */
int attach_payloads(wcpt_group* g)
{
    for (int r = 0; r < g->n; r++) {
        if (!g->format || !g->width) {
            const int rc = wcpt_set_gather_output(g->ctx[r], 0, 0, 0);
            if (rc) return rc;
            continue;
        }
        const uint64_t bytes = (uint64_t)g->width * g->rows[r] * pixel_bytes(g->format);
        uint64_t addr = 0;
        if (r == g->root) {
            addr = g->dst + (uint64_t)g->width * g->y0[r] * pixel_bytes(g->format);
        } else {
            if (g->payload_cap[r] < bytes) {
                if (hipSetDevice(g->devices[r]) != hipSuccess) return group_error(WCPT_ERROR_DEVICE_LOST, "hipSetDevice");
                if (g->payload[r]) {
                    (void)hipDeviceSynchronize(); /* the previous payload may still be read by a send */
                    (void)hipFree(g->payload[r]);
                }
                g->payload[r] = nullptr;
                g->payload_cap[r] = 0;
                if (hipMalloc(&g->payload[r], bytes) != hipSuccess)
                    return group_error(WCPT_ERROR_OUT_OF_DEVICE_MEMORY, "hipMalloc(payload of rank %d, %llu bytes)", r,
                                       (unsigned long long)bytes);
                g->payload_cap[r] = bytes;
            }
            addr = reinterpret_cast<uint64_t>(g->payload[r]);
        }
        const int rc = wcpt_set_gather_output(g->ctx[r], addr, bytes, (uint32_t)g->format);
        if (rc) return rc;
    }
    return WCPT_SUCCESS;
}

int nccl_fail(ncclResult_t e, const char* what)
{
    return group_error(WCPT_ERROR_DEVICE_LOST, "%s: %s", what, ncclGetErrorString(e));
}

} // namespace

extern "C" {

int wcpt_group_create(const int* devices, int n, int root, wcpt_group** out)
{
    if (!out) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "null out");
    *out = nullptr;
    if (!devices || n < 1) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group of %d devices", n);
    if (root < 0 || root >= n) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "root %d outside [0,%d)", root, n);
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) {
        (void)hipGetLastError();
        return group_error(WCPT_ERROR_INITIALIZATION_FAILED, "no HIP device available");
    }
    for (int r = 0; r < n; r++) {
        if (devices[r] < 0 || devices[r] >= count)
            return group_error(WCPT_ERROR_INVALID_ARGUMENT, "device %d out of range [0,%d)", devices[r], count);
        for (int q = 0; q < r; q++)
            if (devices[q] == devices[r])
                return group_error(WCPT_ERROR_INVALID_ARGUMENT, "device %d listed twice (one rank per device)", devices[r]);
    }
    wcpt_group* g = new (std::nothrow) wcpt_group();
    if (!g) return group_error(WCPT_ERROR_OUT_OF_HOST_MEMORY, "out of host memory");
    g->n = n;
    g->root = root;
    g->devices.assign(devices, devices + n);
    g->ctx.assign(n, nullptr);
    g->y0.assign(n, 0);
    g->rows.assign(n, 0);
    g->payload.assign(n, nullptr);
    g->payload_cap.assign(n, 0);
    for (int r = 0; r < n; r++) {
        const int rc = wcpt_create(devices[r], &g->ctx[r]);
        if (rc) {
            wcpt_group_destroy(g);
            return rc;
        }
    }
    if (n > 1) {
        g->comm.assign(n, nullptr);
        const ncclResult_t e = ncclCommInitAll(g->comm.data(), n, devices);
        if (e != ncclSuccess) {
            g->comm.clear();
            wcpt_group_destroy(g);
            return nccl_fail(e, "ncclCommInitAll");
        }
    }
    *out = g;
    return WCPT_SUCCESS;
}

int wcpt_group_destroy(wcpt_group* g)
{
    if (!g) return WCPT_SUCCESS;
    for (int r = 0; r < g->n; r++)
        if (g->ctx[r]) (void)wcpt_sync(g->ctx[r]);
    for (ncclComm_t c : g->comm)
        if (c) (void)ncclCommDestroy(c);
    for (int r = 0; r < g->n; r++) {
        if (g->payload[r]) {
            (void)hipSetDevice(g->devices[r]);
            (void)hipFree(g->payload[r]);
        }
        if (g->ctx[r]) wcpt_destroy(g->ctx[r]);
    }
    delete g;
    return WCPT_SUCCESS;
}

wcpt_context* wcpt_group_context(wcpt_group* g, int rank)
{
    if (!g || rank < 0 || rank >= g->n) return nullptr;
    return g->ctx[rank];
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

int wcpt_group_create_screen(wcpt_group* g, uint32_t width, uint32_t height)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (width == 0 || height < (uint32_t)g->n)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "%ux%u frame for %d row blocks", width, height, g->n);
    for (int r = 0; r < g->n; r++) {
        /* the row-block split of SURVEY.md §8(e) (wcpt_row_block): blocks differ by at most one row */
        uint32_t y0 = 0, rows = 0;
        (void)wcpt_row_block(height, (uint32_t)g->n, (uint32_t)r, &y0, &rows);
        const uint32_t y1 = y0 + rows;
        /* a resized frame first keeps the previous block (clipped to the new height), so no rank ever allocates the
         * whole frame; a fresh context takes its block before its first screen */
        int rc = g->width ? wcpt_create_screen(g->ctx[r], width, height) : WCPT_SUCCESS;
        if (!rc) rc = wcpt_set_row_range(g->ctx[r], y0, y1 - y0);
        if (!rc) rc = wcpt_create_screen(g->ctx[r], width, height); /* zeroes the block (CreateScreen) */
        if (rc) return rc;
        g->y0[r] = y0;
        g->rows[r] = y1 - y0;
    }
    g->width = width;
    g->height = height;
    if (g->format && (uint64_t)width * height * pixel_bytes(g->format) > g->dst_bytes) {
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
    if (dst == 0) {
        g->format = 0;
        g->dst = g->dst_bytes = 0;
        return attach_payloads(g);
    }
    if (!valid_format(format)) return group_error(WCPT_ERROR_INVALID_ARGUMENT, "output format %d (3, 4 or 8)", format);
    if ((dst & 3u) || (format == WCPT_PAYLOAD_RGBA32F && (dst & 15u)))
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "misaligned group output");
    if (g->width && (uint64_t)g->width * g->height * pixel_bytes(format) > bytes)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "group output of %llu bytes < %ux%u x %llu",
                           (unsigned long long)bytes, g->width, g->height, (unsigned long long)pixel_bytes(format));
    g->format = format;
    g->dst = dst;
    g->dst_bytes = bytes;
    return attach_payloads(g);
}

int wcpt_group_render(wcpt_group* g, const wcpt_scene_data* scene, const uint64_t* materials, const uint64_t* spheres,
                      const uint64_t* draw_commands)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    if (!scene || !materials || !spheres || !draw_commands)
        return group_error(WCPT_ERROR_INVALID_ARGUMENT, "wcpt_group_render: null argument");
    if (!g->width) return group_error(WCPT_ERROR_NO_SCREEN, "wcpt_group_render: no screen (wcpt_group_create_screen)");
    for (int r = 0; r < g->n; r++) {
        const int rc = wcpt_render(g->ctx[r], scene, materials[r], spheres[r], draw_commands[r]);
        if (rc) return rc;
    }
    if (!g->format || g->n == 1) return WCPT_SUCCESS; /* the root rendered its block into the output already */
    const uint64_t px = pixel_bytes(g->format);
    ncclResult_t e = ncclGroupStart();
    if (e != ncclSuccess) return nccl_fail(e, "ncclGroupStart");
    ncclResult_t first = ncclSuccess;
    for (int r = 0; r < g->n && first == ncclSuccess; r++) {
        if (r == g->root) continue;
        const uint64_t bytes = (uint64_t)g->width * g->rows[r] * px;
        void* at = reinterpret_cast<void*>(g->dst + (uint64_t)g->width * g->y0[r] * px);
        first = ncclSend(g->payload[r], bytes, ncclUint8, g->root, g->comm[r], wcpt::context_stream(g->ctx[r]));
        if (first == ncclSuccess)
            first = ncclRecv(at, bytes, ncclUint8, r, g->comm[g->root], wcpt::context_stream(g->ctx[g->root]));
    }
    e = ncclGroupEnd();
    if (first != ncclSuccess) return nccl_fail(first, "ncclSend/ncclRecv");
    if (e != ncclSuccess) return nccl_fail(e, "ncclGroupEnd");
    return WCPT_SUCCESS;
}

int wcpt_group_sync(wcpt_group* g)
{
    if (!g) return group_error(WCPT_ERROR_INVALID_HANDLE, "null group");
    int first = WCPT_SUCCESS;
    for (int r = 0; r < g->n; r++) {
        const int rc = wcpt_sync(g->ctx[r]);
        if (rc && !first) first = rc;
    }
    return first;
}

} /* extern "C" */
