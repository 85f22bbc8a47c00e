/*
 * wcpt_runtime.hip — C-ABI runtime: device context, device buffers, output image, dispatch, timing.
 *
 * Replaces the Vulkan plumbing of the reference's renderer host (src/PathTracingRenderer.jai,
 * src/BufferManager.jai, modules/VKUtils/{Buffer,Synchronization}.jai); see include/wcpt.h for the
 * line-by-line mapping. HIP device memory replaces VMA GPU-only buffers; a device pointer IS the buffer
 * device address (VK_KHR_buffer_device_address, pathTracer.comp:74-95).
 */
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/wcpt.h"
#include "pt_kernels.h"

namespace {

constexpr int kNumCounters = 16; /* wcpt_counters: 8 reference counters + 6 diagnostics + 2 reference-stack fields */
std::mutex g_err_mutex;
std::string g_last_error;

/* Device buffers are handed out at base address = 32 (mod 64) (a 64-byte-aligned allocation + 32). A BVH
 * node is 32 bytes and the two children of an interior node sit at indices (2k+1, 2k+2) (the builder appends
 * them as a pair after the root, PathTracingRenderer.jai:196-202), so with this base every child pair the
 * traversal fetches together occupies exactly one 64-byte cache line instead of straddling two. Scattered
 * line visits are what bounds traversal (tools/gather_bench.hip). 32-byte alignment is enough for every
 * other buffer type (largest access: 16 bytes). */
constexpr uint64_t kBufferSkew = 32;

struct Buffer {
    void* raw = nullptr;   /* hipMalloc result */
    void* ptr = nullptr;   /* raw + kBufferSkew: the device address handed out */
    uint64_t bytes = 0;
    uint64_t generation = 0;      /* context-wide counter value of the last alloc / upload / grow */
    std::vector<uint8_t> shadow;  /* host copy of the uploaded contents (buffers <= kShadowMax bytes) */
    std::vector<uint8_t> known;   /* per kShadowChunk bytes: 1 when `shadow` holds what wcpt_buffer_upload wrote */
};

/* Small buffers (draw commands, materials, spheres) keep a host copy of what was uploaded, so that the render
 * call can read the draw commands without a device round trip. */
constexpr uint64_t kShadowMax = 1ull << 20;
/* Granularity of the host copy's validity map. hipMalloc contents are undefined, so a byte range of the host copy is
 * trusted only where wcpt_buffer_upload wrote it; any other range is read from the device. */
constexpr uint64_t kShadowChunk = 32;

/* Mark the chunks of [offset, end) that the upload covers entirely as known (partially covered chunks keep their
 * state: the host copy is updated byte-exactly either way). */
void shadow_mark(Buffer& b, uint64_t offset, uint64_t end)
{
    if (b.known.empty()) return;
    const uint64_t c0 = (offset + kShadowChunk - 1) / kShadowChunk, c1 = end / kShadowChunk;
    for (uint64_t c = c0; c < c1 && c < b.known.size(); c++) b.known[c] = 1;
}

/* True when the host copy holds every byte of [offset, offset + bytes). */
bool shadow_known(const Buffer& b, uint64_t offset, uint64_t bytes)
{
    if (b.shadow.size() != b.bytes || bytes == 0 || offset + bytes > b.bytes) return false;
    for (uint64_t c = offset / kShadowChunk; c < (offset + bytes + kShadowChunk - 1) / kShadowChunk; c++)
        if (c >= b.known.size() || !b.known[c]) return false;
    return true;
}

/* Derived triangle records of one draw command (pt_device.h): rebuilt when the draw's vertex/index buffers,
 * their generations or its index count change (or on every render with WCPT_OPTION_TRIANGLE_CACHE = 0). */
constexpr uint64_t kUnknownGeneration = ~0ull;
struct TriRecords {
    uint64_t vb = 0, ib = 0, gen_vb = kUnknownGeneration, gen_ib = kUnknownGeneration;
    uint32_t ntri = 0;
    bool valid = false;
    void* mem = nullptr;    /* single records, then pair records */
    uint64_t cap = 0;
    uint64_t pair_offset = 0;
    uint64_t build_id = 0;  /* incremented on every rebuild of the records */
    /* whether every node of the draw's BVH (address bvh, `bvh_nodes` nodes, buffer generation gen_bvh) has
     * triangleCount < 255 (pt_device.h kTriFlagSmallLeaves) */
    uint64_t bvh = 0, gen_bvh = kUnknownGeneration;
    uint64_t bvh_nodes = 0;
    uint32_t bvh_ntri = 0;
    uint32_t leaf_flags = 0;   /* launch_scan_leaf_counts */
    bool leaves_valid = false;
    /* primary-ray pair records (pt_device.h TriPairP) for the camera position `porigin` (bit patterns), derived from
     * the pair records of build `pbuild` */
    void* pmem = nullptr;   /* two copies of pcap bytes: the context stream's, then the overlap's pipe 1's (pmem1) */
    uint64_t pcap = 0;
    bool pvalid = false;
    uint32_t porigin[3] = {0, 0, 0};
    uint64_t pbuild = 0;
    /* pipe 1's copy (frame overlap): rebuilt on pipe 1's stream only, so neither copy is ever written while the other
     * stream's frames read it (prep_pipe1) */
    bool pvalid1 = false;
    uint32_t porigin1[3] = {0, 0, 0};
    uint64_t pbuild1 = 0;
    void* pmem1() const { return pmem ? static_cast<char*>(pmem) + pcap : nullptr; }
};

/* Pair records (packed two-triangle tests) pay off when leaves are fat: mean triangles per leaf >= this,
 * estimated as triangles / leaves with leaves = (nodes + 1) / 2 from the BVH buffer's size. Measured: the
 * Cornell box (17 per leaf) gains, the atrium (~2 per leaf) loses. */
constexpr double kPairMinTrianglesPerLeaf = 4.0;
/* Largest triangle count of a draw whose pair records are used: 40 B per triangle must stay addressable with 32-bit
 * byte offsets (2^26 triangles = 2.5 GiB of pair records); larger draws use single records. */
constexpr uint64_t kPairMaxTriangles = 1ull << 26;
/* Primary-ray pair records for the megakernel (pt_device.h WCPT_PRIMARY_PAIRS) */
constexpr bool kPrimaryPairs = WCPT_PRIMARY_PAIRS != 0;

/* Bytes per pixel of a gather payload format (wcpt.h WCPT_PAYLOAD_*) */
uint64_t payload_pixel_bytes(uint32_t format) { return format == WCPT_PAYLOAD_DISPLAY_RGBA8 ? 4u : 4ull * format; }

hipError_t skewed_alloc(Buffer& b, uint64_t bytes)
{
    b.raw = nullptr;
    b.ptr = nullptr;
    b.bytes = bytes;
    if (!bytes) return hipSuccess;
    hipError_t e = hipMalloc(&b.raw, bytes + 2 * kBufferSkew);
    if (e != hipSuccess) return e;
    b.ptr = static_cast<char*>(b.raw) + kBufferSkew;
    return hipSuccess;
}

} // namespace

struct wcpt_context {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::unordered_map<uint64_t, Buffer> buffers;
    uint64_t next_handle = 1;
    float4* image = nullptr;           /* the image kernels write: own_image or an external buffer */
    float4* own_image = nullptr;
    uint64_t image_bytes_cap = 0;
    uint64_t external_bytes = 0;       /* != 0 while an external image is attached */
    float* wire = nullptr;             /* wcpt_set_gather_output */
    uint64_t wire_bytes = 0;
    uint32_t wire_ch = 3;
    uint32_t width = 0, height = 0, y0 = 0, rows = 0; /* rows == height when not sharded */
    uint32_t stripe = 0, period = 0;   /* wcpt_set_row_stripes (0: a contiguous block [y0, y0 + rows)) */
    bool sharded = false;
    int gather_frame_rows = 0;         /* WCPT_OPTION_GATHER_FRAME_ROWS */
    uint32_t* d_status = nullptr;
    unsigned long long* d_counters = nullptr;
    wcpt::WfPipes wf;                  /* path state + streams of the wavefront pipelines (allocated on first use) */
    wcpt::MkState mk;                  /* megakernel launch state (CU count, cost-ordered tiles) */
    uint32_t* d_scratch = nullptr;
    uint32_t* d_scan = nullptr;        /* leaf-count scan flag (prepare_tri_records) */
    uint64_t scratch_bytes = 0;
    int kernel = WCPT_KERNEL_MEGAKERNEL;
    int kernel_run = WCPT_KERNEL_MEGAKERNEL; /* the variant the current/last render runs (WCPT_KERNEL_AUTO resolved) */
    int stack_kind = 1;                /* WCPT_OPTION_STACK: 0 scratch, 1 LDS + spill (default; c2 -2%, 135-row blocks -8%) */
    int diagnostics = 0;               /* WCPT_OPTION_DIAGNOSTICS */
    int sort_rays = 0;                 /* WCPT_OPTION_SORT_RAYS (wavefront only; measured a net loss on c3) */
    int wf_stack = 10;                 /* WCPT_OPTION_WF_STACK: LDS stack entries of the wavefront trace kernel */
    int tri_cache = 1;                 /* WCPT_OPTION_TRIANGLE_CACHE */
    int packed_refs = 1;               /* WCPT_OPTION_PACKED_REFS */
    int wf_fetch = -1;                 /* WCPT_OPTION_WF_FETCH */
    int wf_persist = -1;               /* WCPT_OPTION_WF_PERSIST */
    int wf_refill = 20;                /* WCPT_OPTION_WF_REFILL (round 5 with the deferred hit stores, c4: 8 / 12 / 16 / 20 / 24 / 32 -> 203.5 / 199.6 / 198.9 / 198.0 / 198.6 / 201.4 ms; c3 flat; profiles/r05_fetch_once_ab.log) */
    /* the path-persistent trace's threshold while the option is unset (round 6, c3 8-way slowest share over 3 rounds,
     * refill 8 / 12 / 16 / 20: 8-row stripes 1.265 / 1.250 / 1.249 / 1.262 ms, row blocks 1.314 / 1.280 / 1.293 / 1.287
     * ms; profiles/r06_persist_refill_sweep_c3.log) */
    int wf_refill_persist = 12;
#ifndef WCPT_WF_PIPES_DEFAULT
#define WCPT_WF_PIPES_DEFAULT 0
#endif
    int wf_pipes = WCPT_WF_PIPES_DEFAULT; /* WCPT_OPTION_WF_PIPES (0 = by queue length, pt_wavefront.hip launch_wavefront) */
    int pair_records = -1;             /* WCPT_OPTION_PAIR_RECORDS: -1 auto, 0 singles, 1 pairs (megakernel) */
    int mk_tile_order = 2;             /* WCPT_OPTION_MK_TILE_ORDER: auto */
    int frame_overlap = 1;             /* WCPT_OPTION_FRAME_OVERLAP: auto */
    bool overlap_suppressed = false;   /* set by a group (wcpt::set_overlap_suppressed) */
    bool prep_missed = false;          /* the last render's preparation missed its cache (prepare_tri_records) */
    uint64_t generation = 0;           /* bumped by every buffer alloc / upload / free and every option change */
    /* Frame preparation of the last render (prepare_tri_records) and the last validation (render_validate), reused
     * while nothing they read can have changed: the same draw-command address and count, no buffer allocated,
     * uploaded or freed and no option changed since (ctx->generation), the draw commands read from the host copy of
     * wcpt_buffer_upload (never from the device, which the application may write behind the runtime), and for the
     * primary-ray records the same camera position. An unchanged frame -- progressive accumulation, a group's every
     * rank every frame -- then does no draw-command copy, lookup, allocation or table compare. */
    struct PrepCache {
        bool valid = false;
        uint64_t gen = 0, draws = 0;
        uint32_t n = 0;
        uint32_t origin[3] = {0, 0, 0};
        bool pair_records = false, wf_fast = false;
        int kernel_run = WCPT_KERNEL_MEGAKERNEL;
    } prep;
    struct ValidCache {
        bool valid = false;
        uint64_t gen = 0, draws = 0;
        uint32_t n = 0;
    } validated;
    /* draw commands render_validate had to read from the device, handed to the render that follows it (one read, one
     * host-blocking sync per frame instead of two) */
    std::vector<wcpt_draw_command> handoff;
    uint64_t handoff_draws = 0;
    bool handoff_valid = false;
    std::vector<TriRecords> tri;       /* per draw command index */
    std::vector<uint64_t> tri_table;   /* host image of d_tri_table: {address, ntri} per draw */
    uint64_t* d_tri_table = nullptr;   /* two tables of tri_table_cap draws: the context stream's, then pipe 1's, whose
                                        * word 4 points at the pipe-1 copy of the primary-ray records */
    uint32_t tri_table_cap = 0;        /* draws d_tri_table can hold */
    bool prim_records = false;         /* the last preparation derived primary-ray records (table word 4) */
    std::string last_error;
    bool profiling = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
    size_t events_used = 0;
    int profile_region = 0;     /* WCPT_OPTION_PROFILE_REGION */
    uint32_t region_renders = 0; /* renders since wcpt_profile_begin (region timing) */
};

namespace {

int set_error(wcpt_context* ctx, int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (ctx) ctx->last_error = buf;
    std::lock_guard<std::mutex> lk(g_err_mutex);
    g_last_error = buf;
    return code;
}

int hip_fail(wcpt_context* ctx, hipError_t e, const char* what)
{
    const int code = (e == hipErrorOutOfMemory) ? WCPT_ERROR_OUT_OF_DEVICE_MEMORY : WCPT_ERROR_DEVICE_LOST;
    return set_error(ctx, code, "%s: %s", what, hipGetErrorString(e));
}

#define HIP_TRY(ctx, expr, what)                                  \
    do {                                                          \
        hipError_t _e = (expr);                                   \
        if (_e != hipSuccess) return hip_fail((ctx), _e, (what)); \
    } while (0)

/* the context's device current, without touching its stream (render_common: a render may continue the overlap) */
int bind_device(wcpt_context* ctx)
{
    if (!ctx) return set_error(nullptr, WCPT_ERROR_INVALID_HANDLE, "null context");
    HIP_TRY(ctx, hipSetDevice(ctx->device), "hipSetDevice");
    return WCPT_SUCCESS;
}

/* Frames the frame-overlap pipes hold (MkState::pending) are joined into the context's stream before anything else
 * is queued there or waited for: every entry point but a render binds through here, and so does the group's access
 * to the stream (context_stream), so stream order is as if each render had run on the stream itself. */
int join_pending(wcpt_context* ctx)
{
    if (ctx->mk.pending) HIP_TRY(ctx, wcpt::mk_join(ctx->mk, ctx->stream), "frame overlap join");
    if (ctx->wf.pending) HIP_TRY(ctx, wcpt::wf_join(ctx->wf, ctx->stream), "frame overlap join (wavefront)");
    return WCPT_SUCCESS;
}

int bind(wcpt_context* ctx)
{
    const int rc = bind_device(ctx);
    return rc ? rc : join_pending(ctx);
}

Buffer* find_buffer(wcpt_context* ctx, wcpt_buffer h)
{
    auto it = ctx->buffers.find(h);
    return it == ctx->buffers.end() ? nullptr : &it->second;
}

int ensure_scratch(wcpt_context* ctx, uint64_t bytes)
{
    if (ctx->scratch_bytes >= bytes) return WCPT_SUCCESS;
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    ctx->d_scratch = nullptr;
    ctx->scratch_bytes = 0;
    HIP_TRY(ctx, hipMalloc(&ctx->d_scratch, bytes), "hipMalloc(selftest scratch)");
    ctx->scratch_bytes = bytes;
    return WCPT_SUCCESS;
}

int alloc_image(wcpt_context* ctx, uint32_t w, uint32_t h, uint32_t y0, uint32_t rows)
{
    const uint64_t bytes = (uint64_t)w * rows * 16ull;
    if (ctx->external_bytes) {
        if (bytes > ctx->external_bytes)
            return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "external image of %llu bytes < %llu needed",
                             (unsigned long long)ctx->external_bytes, (unsigned long long)bytes);
    } else if (bytes > ctx->image_bytes_cap) {
        if (ctx->own_image) (void)hipFree(ctx->own_image);
        ctx->own_image = nullptr;
        ctx->image = nullptr;
        ctx->image_bytes_cap = 0;
        HIP_TRY(ctx, hipMalloc(&ctx->own_image, bytes), "hipMalloc(image)");
        ctx->image_bytes_cap = bytes;
        ctx->image = ctx->own_image;
    }
    ctx->width = w;
    ctx->height = h;
    ctx->y0 = y0;
    ctx->rows = rows;
    return WCPT_SUCCESS;
}

/* The context's row map (row_map.h): frame row of each local row. */
wcpt::RowMap row_map(const wcpt_context* ctx)
{
    if (!ctx->stripe) return {ctx->y0, wcpt::kContiguousShift, 0u};
    return {ctx->y0, (uint32_t)__builtin_ctz(ctx->stripe), ctx->period - ctx->stripe};
}

/* The frame row of the context's last local row (its rows must be > 0). */
uint64_t last_frame_row(const wcpt_context* ctx) { return wcpt::frame_row64(row_map(ctx), ctx->rows - 1u); }

/* The buffer whose [ptr, ptr + bytes) contains device address `addr`, or null. */
Buffer* buffer_at(wcpt_context* ctx, uint64_t addr, uint64_t& offset)
{
    for (auto& kv : ctx->buffers) {
        const uint64_t base = reinterpret_cast<uint64_t>(kv.second.ptr);
        if (kv.second.ptr && addr >= base && addr < base + kv.second.bytes) {
            offset = addr - base;
            return &kv.second;
        }
    }
    return nullptr;
}

/* Frame overlap, pipe 1 (pt_kernels.hip launch_megakernel): before its launch, on its own stream, the pipe-1 copy of
 * each draw's primary-ray records is derived again when it is not of the frame's camera position and records build.
 * Only pipe 1's stream ever writes that copy and the context's stream the other, so a moving camera needs no join. */
hipError_t prep_pipe1(void* user, hipStream_t stream)
{
    wcpt_context* ctx = static_cast<wcpt_context*>(user);
    for (TriRecords& t : ctx->tri) {
        if (!t.pvalid || t.ntri == 0) continue;
        if (t.pvalid1 && t.pbuild1 == t.pbuild && std::memcmp(t.porigin1, t.porigin, sizeof(t.porigin)) == 0) continue;
        float o[3];
        std::memcpy(o, t.porigin, sizeof(o));
        const uint64_t npairs = ((uint64_t)t.ntri + 1u) / 2u;
        const hipError_t e = wcpt::launch_build_primary_pairs(static_cast<const char*>(t.mem) + t.pair_offset,
                                                              (uint32_t)npairs, o[0], o[1], o[2], t.pmem1(), stream);
        if (e != hipSuccess) return e;
        t.pvalid1 = true;
        t.pbuild1 = t.pbuild;
        std::memcpy(t.porigin1, t.porigin, sizeof(t.porigin));
    }
    return hipSuccess;
}

void set_pipe1_records(wcpt_context* ctx, uint32_t n, wcpt::LaunchArgs& a)
{
    a.tri_records_pipe1 = nullptr;
    a.pipe1_prepare = nullptr;
    a.pipe1_user = nullptr;
    if (!ctx->prim_records || n == 0) return; /* no primary-ray records: both pipes read the one table */
    a.tri_records_pipe1 = ctx->d_tri_table + 5ull * ctx->tri_table_cap;
    a.pipe1_prepare = prep_pipe1;
    a.pipe1_user = ctx;
}

/* Derive (or reuse) the triangle records of every draw command and point a.tri_records at the table. The draw
 * commands are read from the host copy of their buffer when every byte of them was written through
 * wcpt_buffer_upload and the triangle cache is on; otherwise from the device (a synchronous copy of 32 B per draw),
 * so that draw commands written by other means (hipMemcpy, the application's own kernels) are honoured with
 * WCPT_OPTION_TRIANGLE_CACHE = 0. */
int prepare_tri_records(wcpt_context* ctx, const wcpt_scene_data& sd, uint64_t draws, wcpt::LaunchArgs& a)
{
    const uint32_t n = sd.drawCommandCount;
    a.tri_records = nullptr;
    a.wf_fast = false;
    if (n == 0) {
        /* WCPT_KERNEL_AUTO with no draws: the megakernel (the rule below); an explicit choice stands */
        ctx->kernel_run = ctx->kernel != WCPT_KERNEL_AUTO ? ctx->kernel : WCPT_KERNEL_MEGAKERNEL;
        return WCPT_SUCCESS;
    }
    const bool handoff = ctx->handoff_valid && ctx->handoff_draws == draws && ctx->handoff.size() == n;
    ctx->handoff_valid = false;
    wcpt_context::PrepCache& pc = ctx->prep;
    if (!handoff && pc.valid && pc.gen == ctx->generation && pc.draws == draws && pc.n == n &&
        std::memcmp(pc.origin, sd.position, sizeof(pc.origin)) == 0) {
        a.pair_records = pc.pair_records;
        a.wf_fast = pc.wf_fast;
        ctx->kernel_run = pc.kernel_run;
        a.tri_records = ctx->d_tri_table;
        set_pipe1_records(ctx, n, a);
        ctx->prep_missed = false;
        return WCPT_SUCCESS;
    }
    /* Only the camera moved (an editor drag, bench.py --camera orbit): the primary-ray records are derived again for
     * the new position -- the context stream's copy here, behind that stream's frames; pipe 1's copy on its own stream
     * before its launch (prep_pipe1) -- and nothing else changes, so the frame overlap goes on. */
    if (!handoff && pc.valid && pc.gen == ctx->generation && pc.draws == draws && pc.n == n) {
        uint32_t origin[3];
        std::memcpy(origin, sd.position, sizeof(origin));
        if (ctx->prim_records) {
            for (uint32_t d = 0; d < n; d++) {
                TriRecords& t = ctx->tri[d];
                if (!t.pvalid || t.ntri == 0) continue;
                const uint64_t npairs = ((uint64_t)t.ntri + 1u) / 2u;
                HIP_TRY(ctx, wcpt::launch_build_primary_pairs(static_cast<const char*>(t.mem) + t.pair_offset,
                                                              (uint32_t)npairs, sd.position[0], sd.position[1],
                                                              sd.position[2], t.pmem, ctx->stream),
                        "build_primary_pairs");
                std::memcpy(t.porigin, origin, sizeof(origin));
            }
        }
        std::memcpy(pc.origin, origin, sizeof(pc.origin));
        a.pair_records = pc.pair_records;
        a.wf_fast = pc.wf_fast;
        ctx->kernel_run = pc.kernel_run;
        a.tri_records = ctx->d_tri_table;
        set_pipe1_records(ctx, n, a);
        ctx->prep_missed = false;
        return WCPT_SUCCESS;
    }
    pc.valid = false;
    /* the preparation below may rebuild records that pending frames read, and queues its work on the stream; the
     * frame that follows runs on the stream itself (render_common): a camera that moves every frame rebuilds the
     * primary-ray records every frame, and a fork and a join per frame would cost more than the overlap returns */
    ctx->prep_missed = true;
    int jrc = join_pending(ctx);
    if (jrc) return jrc;
    const uint64_t dbytes = (uint64_t)n * sizeof(wcpt_draw_command);
    uint64_t off = 0;
    Buffer* db = buffer_at(ctx, draws, off);
    const bool from_host = ctx->tri_cache && db && shadow_known(*db, off, dbytes);
    std::vector<wcpt_draw_command> dc;
    if (handoff) {
        dc.swap(ctx->handoff);
    } else {
        dc.resize(n);
        if (from_host) {
            std::memcpy(dc.data(), db->shadow.data() + off, dbytes);
        } else {
            HIP_TRY(ctx, hipMemcpyAsync(dc.data(), reinterpret_cast<const void*>(draws), dbytes, hipMemcpyDeviceToHost,
                                        ctx->stream), "hipMemcpyAsync(draw commands)");
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize(draw commands)");
        }
    }
    if (ctx->tri.size() < n) ctx->tri.resize(n);
    constexpr uint64_t W = 5; /* table words per draw (pt_device.h kTriTableWords) */
    bool table_dirty = ctx->tri_table.size() < W * n;
    if (table_dirty) ctx->tri_table.resize(W * n, 0);
    uint64_t tris_all = 0, leaves_all = 0, tris_max = 0;
    for (uint32_t d = 0; d < n; d++) {
        TriRecords& t = ctx->tri[d];
        const uint64_t vb = dc[d].vertexBuffer, ib = dc[d].indexBuffer;
        uint64_t ov = 0, oi = 0, o = 0;
        Buffer* bv = buffer_at(ctx, vb, ov);
        Buffer* bi = buffer_at(ctx, ib, oi);
        const uint64_t gv = bv ? bv->generation : kUnknownGeneration;
        const uint64_t gi = bi ? bi->generation : kUnknownGeneration;
        const uint32_t ntri = dc[d].indexCount / 3u;
        /* The records are built from indices [0, indexCount) of the draw: an index buffer known to the context must
         * hold them (the reference's kernel never reads indexCount, but the record build does). Vertex indices are
         * checked against the vertex buffer's size on the device (an out-of-range index gives a triangle that is
         * never hit, instead of a read past the buffer). */
        if (bi && (uint64_t)ntri * 12ull > bi->bytes - oi)
            return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT,
                             "draw command %u: indexCount %u exceeds its index buffer (%llu bytes from offset %llu)", d,
                             dc[d].indexCount, (unsigned long long)(bi->bytes - oi), (unsigned long long)oi);
        const uint32_t nvert = bv ? (uint32_t)std::min<uint64_t>((bv->bytes - ov) / 12ull, 0xFFFFFFFFull) : 0xFFFFFFFFu;
        const bool reuse = ctx->tri_cache && t.valid && t.vb == vb && t.ib == ib && t.ntri == ntri && t.gen_vb == gv &&
                           t.gen_ib == gi && gv != kUnknownGeneration && gi != kUnknownGeneration;
        if (!reuse) {
            const uint64_t singles = ((uint64_t)ntri * wcpt::kSingleRecordBytes + 255u) & ~255ull;
            const uint64_t bytes = singles + ((uint64_t)ntri / 2u + 1u) * wcpt::kPairRecordBytes;
            if (t.cap < bytes) {
                if (t.mem) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
                if (t.mem) (void)hipFree(t.mem);
                t.mem = nullptr;
                t.cap = 0;
                HIP_TRY(ctx, hipMalloc(&t.mem, bytes), "hipMalloc(triangle records)");
                t.cap = bytes;
            }
            if (ntri && (vb == 0 || ib == 0))
                return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "draw command %u: null vertex/index buffer", d);
            t.pair_offset = singles;
            HIP_TRY(ctx, wcpt::launch_build_tri_records(reinterpret_cast<const uint32_t*>(ib),
                                                        reinterpret_cast<const float*>(vb), ntri, nvert, t.mem,
                                                        static_cast<char*>(t.mem) + singles, ctx->stream),
                    "build_tri_records");
            t.vb = vb;
            t.ib = ib;
            t.gen_vb = gv;
            t.gen_ib = gi;
            t.ntri = ntri;
            t.valid = true;
            t.build_id++;
        }
        const uint64_t addr = reinterpret_cast<uint64_t>(t.mem);
        /* stack entries may carry the child's (left, count) when every node index and index position fits in 24
         * bits (pt_device.h node_ref); unknown BVH size -> node-index entries */
        Buffer* bb = buffer_at(ctx, dc[d].bvhBuffer, o);
        const uint64_t nodes = bb ? (bb->bytes - o) / sizeof(wcpt_node) : ~0ull;
        uint64_t flags = (ctx->packed_refs && nodes < (1ull << 24) && dc[d].indexCount < (1u << 24)) ? 1u : 0u;
        if (dc[d].indexCount < (1u << 24)) flags |= 2u; /* pt_device.h kTriFlagIndex24 */
        /* pt_device.h kTriFlagSmallLeaves / kTriFlagLeafRecords: scanned on the device once per BVH buffer generation,
         * which only the triangle cache tracks; with the cache off the BVH may change behind the runtime on any frame,
         * and a scan per render would block the host, so the fast leaf layout is simply not used */
        if ((flags & 1u) && ctx->tri_cache) {
            const uint64_t gb = bb->generation;
            if (!(t.leaves_valid && t.bvh == dc[d].bvhBuffer && t.gen_bvh == gb && t.bvh_nodes == nodes &&
                  t.bvh_ntri == ntri)) {
                if (!ctx->d_scan) HIP_TRY(ctx, hipMalloc(&ctx->d_scan, sizeof(uint32_t)), "hipMalloc(leaf scan flag)");
                HIP_TRY(ctx, wcpt::launch_scan_leaf_counts(reinterpret_cast<const void*>(dc[d].bvhBuffer), (uint32_t)nodes,
                                                           ntri, ctx->d_scan, ctx->stream), "scan_leaf_counts");
                uint32_t lf = 3;
                HIP_TRY(ctx, hipMemcpyAsync(&lf, ctx->d_scan, sizeof(lf), hipMemcpyDeviceToHost, ctx->stream),
                        "hipMemcpyAsync(leaf scan flag)");
                HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize(leaf scan flag)");
                t.bvh = dc[d].bvhBuffer;
                t.gen_bvh = gb;
                t.bvh_nodes = nodes;
                t.bvh_ntri = ntri;
                t.leaf_flags = lf;
                t.leaves_valid = true;
            }
            if (!(t.leaf_flags & 1u)) flags |= 4u; /* pt_device.h kTriFlagSmallLeaves */
            if (!(t.leaf_flags & 2u)) flags |= 8u; /* pt_device.h kTriFlagLeafRecords */
        }
        flags |= (uint64_t)nvert << 32;                 /* pt_device.h draw_vertex_count: bounds the index path */
        /* word 2: ntri, and in its high half the BVH node count when packed refs apply (the buffer-resource node loads
         * of pt_device.h load_pair_rsrc cover exactly those nodes) */
        const uint64_t word2 = (uint64_t)ntri | ((flags & 1u) ? (nodes << 32) : 0ull);
        const uint64_t entry[W] = {addr, addr + t.pair_offset, word2, flags, ctx->tri_table[W * d + 4]};
        for (uint64_t w = 0; w < W; w++) {
            if (ctx->tri_table[W * d + w] != entry[w]) {
                ctx->tri_table[W * d + w] = entry[w];
                table_dirty = true;
            }
        }
        tris_all += ntri;
        tris_max = std::max<uint64_t>(tris_max, ntri);
        leaves_all += bb ? (bb->bytes / sizeof(wcpt_node) + 1u) / 2u : ntri; /* unknown BVH: assume thin leaves */
    }
    /* the wavefront trace's one-draw fast layout: packed stack refs, 24-bit record offsets, buffer-resource node loads */
    a.wf_fast = n == 1 && (ctx->tri_table[3] & 15u) == 15u && (ctx->tri_table[2] >> 32) > 0;
    /* pair leaves address a draw's pair records with 32-bit byte offsets (pt_device.h load_pair_at) */
    a.pair_records = tris_max <= kPairMaxTriangles &&
                     (ctx->pair_records == 1 ||
                      (ctx->pair_records < 0 && leaves_all > 0 && (double)tris_all >= kPairMinTrianglesPerLeaf * leaves_all));
    /* WCPT_KERNEL_AUTO: the megakernel where leaves hold several triangles (its pair loops and scalar-cache leaves pay),
     * the wavefront kernel on thin leaves (Cornell 0.37 / mushroom 1.22 ms megakernel against 2.0 ms wavefront on the
     * mushroom; the atrium 4.8 ms wavefront against 9.8 ms megakernel) */
    ctx->kernel_run = ctx->kernel != WCPT_KERNEL_AUTO ? ctx->kernel
                                                      : (a.pair_records || n == 0 ? WCPT_KERNEL_MEGAKERNEL : WCPT_KERNEL_WAVEFRONT);
    /* primary-ray pair records (megakernel with pair records): derived once per camera position and records build */
    const bool want_primary = kPrimaryPairs && a.pair_records && ctx->kernel_run == WCPT_KERNEL_MEGAKERNEL;
    uint32_t origin[3];
    std::memcpy(origin, sd.position, sizeof(origin));
    for (uint32_t d = 0; d < n; d++) {
        TriRecords& t = ctx->tri[d];
        uint64_t paddr = 0;
        if (want_primary && t.ntri > 0) {
            const uint64_t npairs = ((uint64_t)t.ntri + 1u) / 2u; /* the pair records build_tri_records writes */
            const uint64_t bytes = npairs * wcpt::kPrimPairRecordBytes;
            const bool fresh = t.pvalid && t.pbuild == t.build_id && std::memcmp(t.porigin, origin, sizeof(origin)) == 0;
            if (!fresh) {
                if (t.pcap < bytes) {
                    if (t.pmem) {
                        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
                        (void)hipFree(t.pmem);
                    }
                    t.pmem = nullptr;
                    t.pcap = 0;
                    t.pvalid = false;
                    t.pvalid1 = false;
                    HIP_TRY(ctx, hipMalloc(&t.pmem, 2 * bytes), "hipMalloc(primary-ray pair records)");
                    t.pcap = bytes;
                }
                HIP_TRY(ctx, wcpt::launch_build_primary_pairs(static_cast<const char*>(t.mem) + t.pair_offset,
                                                              (uint32_t)npairs, sd.position[0], sd.position[1],
                                                              sd.position[2], t.pmem, ctx->stream),
                        "build_primary_pairs");
                t.pvalid = true;
                t.pbuild = t.build_id;
                std::memcpy(t.porigin, origin, sizeof(origin));
            }
            paddr = reinterpret_cast<uint64_t>(t.pmem);
        }
        if (ctx->tri_table[W * d + 4] != paddr) {
            ctx->tri_table[W * d + 4] = paddr;
            table_dirty = true;
        }
    }
    if (ctx->tri_table_cap < n) {
        if (ctx->d_tri_table) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
            (void)hipFree(ctx->d_tri_table);
        }
        ctx->d_tri_table = nullptr;
        ctx->tri_table_cap = 0;
        HIP_TRY(ctx, hipMalloc(&ctx->d_tri_table, 2 * W * n * sizeof(uint64_t)), "hipMalloc(triangle record table)");
        ctx->tri_table_cap = n;
        table_dirty = true;
    }
    if (table_dirty) {
        /* both tables: the second differs only in word 4, pipe 1's copy of the primary-ray records */
        std::vector<uint64_t> both(2 * W * ctx->tri_table_cap, 0);
        std::copy(ctx->tri_table.begin(), ctx->tri_table.begin() + W * n, both.begin());
        std::copy(ctx->tri_table.begin(), ctx->tri_table.begin() + W * n, both.begin() + W * ctx->tri_table_cap);
        for (uint32_t d = 0; d < n; d++)
            if (ctx->tri_table[W * d + 4])
                both[W * ctx->tri_table_cap + W * d + 4] = reinterpret_cast<uint64_t>(ctx->tri[d].pmem1());
        HIP_TRY(ctx, hipMemcpyAsync(ctx->d_tri_table, both.data(), both.size() * sizeof(uint64_t),
                                    hipMemcpyHostToDevice, ctx->stream), "hipMemcpyAsync(triangle record table)");
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize(triangle record table)");
    }
    ctx->prim_records = want_primary;
    a.tri_records = ctx->d_tri_table;
    set_pipe1_records(ctx, n, a);
    if (from_host && !handoff) {
        pc.valid = true;
        pc.gen = ctx->generation;
        pc.draws = draws;
        pc.n = n;
        std::memcpy(pc.origin, sd.position, sizeof(pc.origin));
        pc.pair_records = a.pair_records;
        pc.wf_fast = a.wf_fast;
        pc.kernel_run = ctx->kernel_run;
    }
    return WCPT_SUCCESS;
}

/* The argument checks of wcpt_render that need no device work (render_common, wcpt::render_validate). */
int check_render_args(wcpt_context* ctx, const wcpt_scene_data* scene, uint64_t materials, uint64_t spheres,
                      uint64_t draws, int mode)
{
    if (!scene) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "wcpt_render: null SceneData");
    if (!ctx->image || ctx->width == 0 || ctx->rows == 0)
        return set_error(ctx, WCPT_ERROR_NO_SCREEN, "wcpt_render: no output image (call wcpt_create_screen)");
    if (scene->sphereCount > 0 && spheres == 0)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "wcpt_render: sphereCount > 0 with a null sphere buffer");
    if (scene->drawCommandCount > 0 && draws == 0)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "wcpt_render: drawCommandCount > 0 with null draw commands");
    if (materials == 0 && (scene->sphereCount > 0 || scene->drawCommandCount > 0))
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "wcpt_render: null material buffer");
    /* the output's rows: the context's rows back to back, or (WCPT_OPTION_GATHER_FRAME_ROWS) frame rows up to its last */
    const uint64_t wire_rows = ctx->gather_frame_rows ? last_frame_row(ctx) + 1u : ctx->rows;
    if (ctx->wire && mode == wcpt::kModeRender &&
        (uint64_t)ctx->width * wire_rows * payload_pixel_bytes(ctx->wire_ch) > ctx->wire_bytes)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "gather output of %llu bytes too small for %ux%llu x %u B",
                         (unsigned long long)ctx->wire_bytes, ctx->width, (unsigned long long)wire_rows,
                         (unsigned)payload_pixel_bytes(ctx->wire_ch));
    return WCPT_SUCCESS;
}

int render_common(wcpt_context* ctx, const wcpt_scene_data* scene, uint64_t materials, uint64_t spheres,
                  uint64_t draws, int mode)
{
    int rc = bind_device(ctx);
    if (rc) return rc;
    /* frame overlap (WCPT_OPTION_FRAME_OVERLAP, pt_kernels.hip launch_megakernel): renders only, on the context's own
     * stream (work the application queues on a stream of its own could not be ordered behind the pipes), and not
     * under per-render timing events (they bracket each frame on the stream) */
    int overlap = (mode == wcpt::kModeRender && ctx->stream == ctx->own_stream && !ctx->overlap_suppressed &&
                   !(ctx->profiling && !ctx->profile_region)) ? ctx->frame_overlap : 0;
    if (!overlap) {
        rc = join_pending(ctx);
        if (rc) return rc;
    }
    rc = check_render_args(ctx, scene, materials, spheres, draws, mode);
    if (rc) return rc;
    wcpt::LaunchArgs a;
    a.sd = *scene;
    a.materials = reinterpret_cast<const wcpt_material*>(materials);
    a.spheres = reinterpret_cast<const wcpt_sphere*>(spheres);
    a.draws = reinterpret_cast<const wcpt_draw_command*>(draws);
    a.image = ctx->image;
    a.wire = nullptr;
    a.wire_ch = ctx->wire_ch;
    if (ctx->wire && mode == wcpt::kModeRender) a.wire = ctx->wire;
    a.W = ctx->width;
    a.H = ctx->height;
    a.y0 = ctx->y0;
    a.rows = ctx->rows;
    {
        const wcpt::RowMap m = row_map(ctx);
        a.row_shift = m.shift;
        a.row_gap = m.gap;
        a.wire_rows = ctx->gather_frame_rows ? m : wcpt::RowMap{0u, wcpt::kContiguousShift, 0u};
    }
    a.status = ctx->d_status;
    a.counters = ctx->d_counters;
    a.tri_records = nullptr;
    a.pair_records = false;
    a.wf_fast = false;
    a.wf_refill = (uint32_t)ctx->wf_refill;
    a.wf_refill_persist = (uint32_t)ctx->wf_refill_persist;
    a.wf_fetch = ctx->wf_fetch;
    a.wf_persist = ctx->wf_persist;
    a.mk_tile_order = (uint32_t)ctx->mk_tile_order;
    hipEvent_t e0 = nullptr, e1 = nullptr;
/* Profiling events time the launches only: no system-scope fence when they are recorded (hip_runtime_api.h,
 * hipEventDisableSystemFence), so the timed frames pay no cache writeback between launches (c2 0.538 -> 0.534
 * ms/frame against hipEventReleaseToDevice and hipEventDefault, which measured alike). */
#ifndef WCPT_PROFILE_EVENT_FLAGS
#define WCPT_PROFILE_EVENT_FLAGS hipEventDisableSystemFence
#endif
    if (ctx->profiling && mode == wcpt::kModeRender && ctx->profile_region) {
        /* region timing: one event before the first render; wcpt_profile_end records the closing one */
        if (ctx->events.empty()) {
            hipEvent_t b, c;
            HIP_TRY(ctx, hipEventCreateWithFlags(&b, WCPT_PROFILE_EVENT_FLAGS), "hipEventCreate");
            HIP_TRY(ctx, hipEventCreateWithFlags(&c, WCPT_PROFILE_EVENT_FLAGS), "hipEventCreate");
            ctx->events.emplace_back(b, c);
        }
        if (ctx->region_renders++ == 0) {
            HIP_TRY(ctx, hipEventRecord(ctx->events[0].first, ctx->stream), "hipEventRecord");
            ctx->events_used = 1;
        }
    } else if (ctx->profiling && mode == wcpt::kModeRender) {
        if (ctx->events_used == ctx->events.size()) {
            hipEvent_t b, c;
            HIP_TRY(ctx, hipEventCreateWithFlags(&b, WCPT_PROFILE_EVENT_FLAGS), "hipEventCreate");
            HIP_TRY(ctx, hipEventCreateWithFlags(&c, WCPT_PROFILE_EVENT_FLAGS), "hipEventCreate");
            ctx->events.emplace_back(b, c);
        }
        e0 = ctx->events[ctx->events_used].first;
        e1 = ctx->events[ctx->events_used].second;
        ctx->events_used++;
        HIP_TRY(ctx, hipEventRecord(e0, ctx->stream), "hipEventRecord");
    }
    ctx->prep_missed = false;
    rc = prepare_tri_records(ctx, *scene, draws, a);
    if (rc) return rc;
    if (ctx->prep_missed) overlap = 0;
    /* the other kernel's pending frames (the same image) first */
    if (ctx->kernel_run != WCPT_KERNEL_MEGAKERNEL && ctx->mk.pending)
        HIP_TRY(ctx, wcpt::mk_join(ctx->mk, ctx->stream), "frame overlap join");
    if (ctx->kernel_run != WCPT_KERNEL_WAVEFRONT && ctx->wf.pending)
        HIP_TRY(ctx, wcpt::wf_join(ctx->wf, ctx->stream), "frame overlap join (wavefront)");
#if WCPT_MK_TIMERS
    /* tools-only build: the render's megakernel adds its phase timers to the counters (wcpt_read_diagnostics) */
    rc = join_pending(ctx);
    if (rc) return rc;
    if (mode == wcpt::kModeRender && ctx->kernel_run == WCPT_KERNEL_MEGAKERNEL)
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_counters, 0, kNumCounters * sizeof(unsigned long long), ctx->stream),
                "hipMemsetAsync(timers)");
#endif
    hipError_t e = hipSuccess;
    switch (ctx->kernel_run) {
    case WCPT_KERNEL_MEGAKERNEL: e = wcpt::launch_megakernel(a, mode, ctx->stack_kind, ctx->mk, ctx->stream, overlap); break;
    case WCPT_KERNEL_WAVEFRONT:
        e = wcpt::launch_wavefront(a, mode, ctx->wf, ctx->wf_pipes, ctx->sort_rays != 0, ctx->wf_stack, ctx->stream, overlap);
        break;
    default: return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "kernel variant %d not available", ctx->kernel_run);
    }
    if (e != hipSuccess) return hip_fail(ctx, e, "kernel launch");
    if (e1) HIP_TRY(ctx, hipEventRecord(e1, ctx->stream), "hipEventRecord");
    return WCPT_SUCCESS;
}

int read_status(wcpt_context* ctx)
{
    uint32_t st = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&st, ctx->d_status, 4, hipMemcpyDeviceToHost, ctx->stream), "hipMemcpyAsync(status)");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    if (st) {
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_status, 0, 4, ctx->stream), "hipMemsetAsync(status)");
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
        return set_error(ctx, WCPT_ERROR_STACK_OVERFLOW,
                         "BVH traversal stack overflow (tree deeper than %d levels); image is incomplete",
                         wcpt::kStackDepth);
    }
    return WCPT_SUCCESS;
}

} // namespace

/* Internal hooks for the multi-device group (wcpt_group.hip): a context's current stream, and error reporting
 * through the same last-error strings as the C entry points. */
namespace wcpt {
hipStream_t context_stream(wcpt_context* ctx)
{
    if (!ctx) return nullptr;
    /* the group queues waits, copies and events here: pending overlap frames first (a failed join surfaces at the
     * group's next stream operation or sync) */
    (void)join_pending(ctx);
    return ctx->stream;
}
int context_device(wcpt_context* ctx) { return ctx ? ctx->device : -1; }
int context_error(wcpt_context* ctx, int code, const char* msg) { return set_error(ctx, code, "%s", msg); }
/* A validated frame that will not be rendered (another rank's validation failed): drop its hand-off. */
void render_abandon(wcpt_context* ctx)
{
    if (ctx) ctx->handoff_valid = false;
}

/* Every check wcpt_render would make before it launches anything, with no launch: the argument checks and, per draw
 * command, the index-count bound of the record build (prepare_tri_records). A group validates all its ranks first, so
 * that an argument error cannot leave some ranks a frame ahead of the others. */
void set_overlap_suppressed(wcpt_context* ctx, bool on)
{
    if (ctx) ctx->overlap_suppressed = on;
}

int context_frame_streams(wcpt_context* ctx, hipStream_t* out, int cap)
{
    if (!ctx || cap < 1) return 0;
    int n = 0;
    out[n++] = ctx->stream;
    if (ctx->mk.pending)
        for (uint32_t p = 1; p < wcpt::kMkPipes && n < cap; p++) out[n++] = ctx->mk.pipe[p];
    if (ctx->wf.pending)
        for (uint32_t j = 1; j < ctx->wf.pending_pipes && n < cap; j++) out[n++] = ctx->wf.aux[j];
    return n;
}

int render_validate(wcpt_context* ctx, const wcpt_scene_data* scene, uint64_t materials, uint64_t spheres,
                    uint64_t draws)
{
    int rc = bind_device(ctx); /* a validation that reads nothing from the device leaves pending frames running */
    if (rc) return rc;
    rc = check_render_args(ctx, scene, materials, spheres, draws, kModeRender);
    if (rc) return rc;
    const uint32_t n = scene->drawCommandCount;
    ctx->handoff_valid = false;
    if (n == 0) return WCPT_SUCCESS;
    wcpt_context::ValidCache& vc = ctx->validated;
    if (vc.valid && vc.gen == ctx->generation && vc.draws == draws && vc.n == n) return WCPT_SUCCESS;
    vc.valid = false;
    const uint64_t dbytes = (uint64_t)n * sizeof(wcpt_draw_command);
    uint64_t off = 0;
    Buffer* db = buffer_at(ctx, draws, off);
    const bool from_host = ctx->tri_cache && db && shadow_known(*db, off, dbytes);
    std::vector<wcpt_draw_command>& dc = ctx->handoff;
    dc.resize(n);
    if (from_host) {
        std::memcpy(dc.data(), db->shadow.data() + off, dbytes);
    } else {
        /* read from the device (the application may write draw commands behind the runtime); the render that follows
         * takes these (prepare_tri_records), so a frame reads them once */
        rc = join_pending(ctx);
        if (rc) return rc;
        HIP_TRY(ctx, hipMemcpyAsync(dc.data(), reinterpret_cast<const void*>(draws), dbytes, hipMemcpyDeviceToHost,
                                    ctx->stream), "hipMemcpyAsync(draw commands)");
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize(draw commands)");
    }
    for (uint32_t d = 0; d < n; d++) {
        const uint32_t ntri = dc[d].indexCount / 3u;
        uint64_t oi = 0;
        Buffer* bi = buffer_at(ctx, dc[d].indexBuffer, oi);
        if (bi && (uint64_t)ntri * 12ull > bi->bytes - oi)
            return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT,
                             "draw command %u: indexCount %u exceeds its index buffer (%llu bytes from offset %llu)", d,
                             dc[d].indexCount, (unsigned long long)(bi->bytes - oi), (unsigned long long)oi);
        if (ntri && (dc[d].vertexBuffer == 0 || dc[d].indexBuffer == 0))
            return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "draw command %u: null vertex/index buffer", d);
    }
    if (from_host) {
        vc.valid = true;
        vc.gen = ctx->generation;
        vc.draws = draws;
        vc.n = n;
    } else {
        ctx->handoff_draws = draws;
        ctx->handoff_valid = true;
    }
    return WCPT_SUCCESS;
}

/* CreateScreen of one row block in one step: the frame's size and the context's block [y0, y0 + rows) are set
 * together, so only the block is allocated (and zeroed), whatever the previous frame's size was. */
int set_frame_block(wcpt_context* ctx, uint32_t width, uint32_t height, uint32_t y0, uint32_t rows, uint32_t stripe,
                    uint32_t period)
{
    int rc = bind(ctx);
    if (rc) return rc;
    if (stripe && (stripe & (stripe - 1u) || stripe > 32768u || period < stripe))
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "row stripes of %u rows every %u rows", stripe, period);
    const uint64_t last = rows == 0 ? 0 : frame_row64(wcpt::RowMap{y0, stripe ? (uint32_t)__builtin_ctz(stripe) : kContiguousShift,
                                                                 stripe ? period - stripe : 0u}, rows - 1u);
    if (width == 0 || rows == 0 || last >= height)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "%u rows from row %u (stripes %u / %u) in a %ux%u frame", rows,
                         y0, stripe, period, width, height);
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    ctx->sharded = true;
    ctx->stripe = stripe;
    ctx->period = stripe ? period : 0u;
    rc = alloc_image(ctx, width, height, y0, rows);
    if (rc) return rc;
    if (!ctx->external_bytes) {
        HIP_TRY(ctx, hipMemsetAsync(ctx->image, 0, (uint64_t)width * rows * 16ull, ctx->stream), "hipMemsetAsync(image)");
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    }
    return WCPT_SUCCESS;
}
} // namespace wcpt

extern "C" {

int wcpt_abi_version(void) { return WCPT_ABI_VERSION; }

#ifndef WCPT_BUILD_ID
#define WCPT_BUILD_ID "unknown"
#endif
const char* wcpt_build_id(void) { return WCPT_BUILD_ID; }

int wcpt_runtime_version(int* version)
{
    if (!version) return set_error(nullptr, WCPT_ERROR_INVALID_ARGUMENT, "null version");
    hipError_t e = hipRuntimeGetVersion(version);
    if (e != hipSuccess) return hip_fail(nullptr, e, "hipRuntimeGetVersion");
    return WCPT_SUCCESS;
}

const char* wcpt_last_error(const wcpt_context* ctx)
{
    if (ctx) return ctx->last_error.c_str();
    std::lock_guard<std::mutex> lk(g_err_mutex);
    return g_last_error.c_str();
}

int wcpt_device_count(int* count)
{
    if (!count) return set_error(nullptr, WCPT_ERROR_INVALID_ARGUMENT, "null count");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        (void)hipGetLastError();
        return WCPT_SUCCESS; /* no device is not an error for the query */
    }
    *count = n;
    return WCPT_SUCCESS;
}

int wcpt_device_pci_bus_id(int device, char* out, int len)
{
    if (!out || len < 13) return set_error(nullptr, WCPT_ERROR_INVALID_ARGUMENT, "pci bus id buffer of %d bytes", len);
    const hipError_t e = hipDeviceGetPCIBusId(out, len, device);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        out[0] = 0;
        return set_error(nullptr, WCPT_ERROR_INVALID_ARGUMENT, "hipDeviceGetPCIBusId(%d): %s", device, hipGetErrorString(e));
    }
    return WCPT_SUCCESS;
}

int wcpt_create(int device, wcpt_context** out_ctx)
{
    if (!out_ctx) return set_error(nullptr, WCPT_ERROR_INVALID_ARGUMENT, "null out_ctx");
    *out_ctx = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return set_error(nullptr, WCPT_ERROR_INITIALIZATION_FAILED, "no HIP device available");
    }
    if (device < 0 || device >= n)
        return set_error(nullptr, WCPT_ERROR_INVALID_ARGUMENT, "device %d out of range [0,%d)", device, n);
    wcpt_context* ctx = new (std::nothrow) wcpt_context();
    if (!ctx) return set_error(nullptr, WCPT_ERROR_OUT_OF_HOST_MEMORY, "out of host memory");
    ctx->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&ctx->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&ctx->d_status, 4);
    if (e == hipSuccess) e = hipMalloc(&ctx->d_counters, kNumCounters * sizeof(unsigned long long));
    if (e == hipSuccess) e = hipMemset(ctx->d_status, 0, 4);
    if (e != hipSuccess) {
        int rc = hip_fail(nullptr, e, "wcpt_create");
        wcpt_destroy(ctx);
        return rc;
    }
    ctx->stream = ctx->own_stream;
    *out_ctx = ctx;
    return WCPT_SUCCESS;
}

int wcpt_destroy(wcpt_context* ctx)
{
    if (!ctx) return WCPT_SUCCESS;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)join_pending(ctx);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (auto& kv : ctx->buffers)
        if (kv.second.raw) (void)hipFree(kv.second.raw);
    if (ctx->own_image) (void)hipFree(ctx->own_image);
    if (ctx->d_status) (void)hipFree(ctx->d_status);
    if (ctx->d_counters) (void)hipFree(ctx->d_counters);
    wcpt::wf_release(ctx->wf);
    wcpt::mk_release(ctx->mk);
    for (auto& t : ctx->tri) {
        if (t.mem) (void)hipFree(t.mem);
        if (t.pmem) (void)hipFree(t.pmem);
    }
    if (ctx->d_tri_table) (void)hipFree(ctx->d_tri_table);
    if (ctx->d_scratch) (void)hipFree(ctx->d_scratch);
    if (ctx->d_scan) (void)hipFree(ctx->d_scan);
    for (auto& p : ctx->events) {
        (void)hipEventDestroy(p.first);
        (void)hipEventDestroy(p.second);
    }
    if (ctx->own_stream) (void)hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return WCPT_SUCCESS;
}

int wcpt_set_stream(wcpt_context* ctx, void* hip_stream)
{
    int rc = bind(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    ctx->stream = hip_stream ? reinterpret_cast<hipStream_t>(hip_stream) : ctx->own_stream;
    return WCPT_SUCCESS;
}

int wcpt_set_kernel(wcpt_context* ctx, int variant)
{
    if (!ctx) return set_error(nullptr, WCPT_ERROR_INVALID_HANDLE, "null context");
    if (variant != WCPT_KERNEL_MEGAKERNEL && variant != WCPT_KERNEL_WAVEFRONT && variant != WCPT_KERNEL_AUTO)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "kernel variant %d not available", variant);
    if (ctx->kernel != variant) ctx->generation++; /* the cached frame preparation resolved the variant */
    ctx->kernel = variant;
    return WCPT_SUCCESS;
}

int wcpt_last_kernel(wcpt_context* ctx, int* variant)
{
    if (!ctx) return set_error(nullptr, WCPT_ERROR_INVALID_HANDLE, "null context");
    if (!variant) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "null variant");
    *variant = ctx->kernel_run;
    return WCPT_SUCCESS;
}

int wcpt_set_option(wcpt_context* ctx, int option, int value)
{
    if (!ctx) return set_error(nullptr, WCPT_ERROR_INVALID_HANDLE, "null context");
    /* The options that prepare_tri_records / render_validate read (record formats, stack-entry layout, the cache
     * itself) invalidate their cached frame preparation once accepted: ctx->generation++ there only, so a host that
     * sets the other options every frame keeps the cache. */
    switch (option) {
    case WCPT_OPTION_SORT_RAYS:
        ctx->sort_rays = value ? 1 : 0;
        return WCPT_SUCCESS;
    case WCPT_OPTION_WF_REFILL:
        if (value < 1 || value > 64) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "refill threshold %d", value);
        ctx->wf_refill = value;
        ctx->wf_refill_persist = value; /* an explicit value governs both traces */
        return WCPT_SUCCESS;
    case WCPT_OPTION_WF_PIPES:
        if (value < 0 || value > wcpt::kWfMaxPipes) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "pipelines %d", value);
        ctx->wf_pipes = value;
        return WCPT_SUCCESS;
    case WCPT_OPTION_MK_TILE_ORDER:
        if (value < 0 || value > 6) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "tile order %d", value);
        ctx->mk_tile_order = value;
        return WCPT_SUCCESS;
    case WCPT_OPTION_FRAME_OVERLAP:
        if (value < 0 || value > 2) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "frame overlap %d", value);
        ctx->frame_overlap = value;
        return WCPT_SUCCESS;
    case WCPT_OPTION_PACKED_REFS:
        ctx->packed_refs = value ? 1 : 0;
        ctx->generation++;
        return WCPT_SUCCESS;
    case WCPT_OPTION_PAIR_RECORDS:
        if (value < -1 || value > 1) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "pair records %d", value);
        ctx->pair_records = value;
        ctx->generation++;
        return WCPT_SUCCESS;
    case WCPT_OPTION_TRIANGLE_CACHE:
        ctx->tri_cache = value ? 1 : 0;
        ctx->generation++;
        return WCPT_SUCCESS;
    case WCPT_OPTION_WF_STACK:
        if (value != 10 && value != 16 && value != 24)
            return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "wavefront LDS stack %d (10, 16 or 24)", value);
        ctx->wf_stack = value;
        return WCPT_SUCCESS;
    case WCPT_OPTION_DIAGNOSTICS:
        ctx->diagnostics = value ? 1 : 0;
        return WCPT_SUCCESS;
    case WCPT_OPTION_WF_PERSIST:
        if (value < -1 || value > 1) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "wavefront persist %d", value);
        ctx->wf_persist = value;
        return WCPT_SUCCESS;
    case WCPT_OPTION_WF_FETCH:
        if (value < -1 || value > 1) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "wavefront fetch rounds %d", value);
        ctx->wf_fetch = value;
        return WCPT_SUCCESS;
    case WCPT_OPTION_PROFILE_REGION:
        if (ctx->profiling) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "profile region: set outside profiling");
        ctx->profile_region = value ? 1 : 0;
        return WCPT_SUCCESS;
    case WCPT_OPTION_STACK:
        if (value < 0 || value > 1) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "stack kind %d", value);
        ctx->stack_kind = value;
        return WCPT_SUCCESS;
    case WCPT_OPTION_GATHER_FRAME_ROWS:
        if (value < 0 || value > 1) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "gather frame rows %d", value);
        ctx->gather_frame_rows = value;
        return WCPT_SUCCESS;
    default: return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "unknown option %d", option);
    }
}

/* ---- buffers ------------------------------------------------------------------------------------ */
int wcpt_buffer_alloc(wcpt_context* ctx, uint64_t bytes, wcpt_buffer* out)
{
    int rc = bind(ctx);
    if (rc) return rc;
    if (!out) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "null out handle");
    Buffer b;
    HIP_TRY(ctx, skewed_alloc(b, bytes), "hipMalloc(buffer)");
    b.generation = ++ctx->generation;
    if (bytes <= kShadowMax) b.shadow.assign(bytes, 0); /* hipMalloc contents are undefined; see upload */
    if (bytes <= kShadowMax) b.known.assign((bytes + kShadowChunk - 1) / kShadowChunk, 0);
    const uint64_t h = ctx->next_handle++;
    ctx->buffers[h] = b;
    *out = h;
    return WCPT_SUCCESS;
}

int wcpt_buffer_upload(wcpt_context* ctx, wcpt_buffer buf, const void* src, uint64_t bytes, uint64_t offset)
{
    int rc = bind(ctx);
    if (rc) return rc;
    Buffer* b = find_buffer(ctx, buf);
    if (!b) return set_error(ctx, WCPT_ERROR_INVALID_HANDLE, "unknown buffer handle %llu", (unsigned long long)buf);
    if (bytes && !src) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "null upload source");
    uint64_t end = 0;
    if (__builtin_add_overflow(offset, bytes, &end) || end > (1ull << 48))
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "upload range offset %llu + %llu bytes overflows",
                         (unsigned long long)offset, (unsigned long long)bytes);
    if (end > b->bytes) {
        /* grow, keeping the old contents (BufferManager.jai:53-54 reallocates on growth) */
        Buffer nb;
        HIP_TRY(ctx, skewed_alloc(nb, end), "hipMalloc(buffer grow)");
        if (b->ptr && b->bytes) {
            hipError_t e = hipMemcpyAsync(nb.ptr, b->ptr, b->bytes, hipMemcpyDeviceToDevice, ctx->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
            if (e != hipSuccess) {
                (void)hipFree(nb.raw);
                return hip_fail(ctx, e, "buffer grow copy");
            }
        }
        if (b->raw) (void)hipFree(b->raw);
        nb.shadow = std::move(b->shadow);
        nb.known = std::move(b->known);
        *b = std::move(nb);
        if (b->bytes <= kShadowMax) {
            b->shadow.resize(b->bytes, 0);
            b->known.resize((b->bytes + kShadowChunk - 1) / kShadowChunk, 0); /* the grown tail is undefined */
        } else {
            b->shadow.clear();
            b->known.clear();
        }
    }
    if (bytes) {
        HIP_TRY(ctx, hipMemcpyAsync(static_cast<char*>(b->ptr) + offset, src, bytes, hipMemcpyHostToDevice, ctx->stream),
                "hipMemcpyAsync(upload)");
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize(upload)"); /* blocking, like :98-112 */
        if (b->shadow.size() == b->bytes && b->bytes) {
            std::memcpy(b->shadow.data() + offset, src, bytes);
            shadow_mark(*b, offset, end);
        }
    }
    b->generation = ++ctx->generation;
    return WCPT_SUCCESS;
}

int wcpt_buffer_download(wcpt_context* ctx, wcpt_buffer buf, void* dst, uint64_t bytes, uint64_t offset)
{
    int rc = bind(ctx);
    if (rc) return rc;
    Buffer* b = find_buffer(ctx, buf);
    if (!b) return set_error(ctx, WCPT_ERROR_INVALID_HANDLE, "unknown buffer handle %llu", (unsigned long long)buf);
    if (bytes > b->bytes || offset > b->bytes - bytes)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "download out of range");
    if (bytes && !dst) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "null download destination");
    if (bytes) {
        HIP_TRY(ctx, hipMemcpyAsync(dst, static_cast<char*>(b->ptr) + offset, bytes, hipMemcpyDeviceToHost, ctx->stream),
                "hipMemcpyAsync(download)");
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize(download)");
    }
    return WCPT_SUCCESS;
}

int wcpt_buffer_size(wcpt_context* ctx, wcpt_buffer buf, uint64_t* out_bytes)
{
    if (!ctx) return set_error(nullptr, WCPT_ERROR_INVALID_HANDLE, "null context");
    Buffer* b = find_buffer(ctx, buf);
    if (!b) return set_error(ctx, WCPT_ERROR_INVALID_HANDLE, "unknown buffer handle");
    if (!out_bytes) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "null out_bytes");
    *out_bytes = b->bytes;
    return WCPT_SUCCESS;
}

uint64_t wcpt_buffer_device_address(wcpt_context* ctx, wcpt_buffer buf)
{
    if (!ctx) return 0;
    Buffer* b = find_buffer(ctx, buf);
    if (!b) {
        set_error(ctx, WCPT_ERROR_INVALID_HANDLE, "unknown buffer handle");
        return 0;
    }
    return reinterpret_cast<uint64_t>(b->ptr);
}

int wcpt_buffer_free(wcpt_context* ctx, wcpt_buffer buf)
{
    int rc = bind(ctx);
    if (rc) return rc;
    auto it = ctx->buffers.find(buf);
    if (it == ctx->buffers.end()) return set_error(ctx, WCPT_ERROR_INVALID_HANDLE, "unknown buffer handle");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize(free)");
    if (it->second.raw) HIP_TRY(ctx, hipFree(it->second.raw), "hipFree");
    ctx->buffers.erase(it);
    ctx->generation++;
    return WCPT_SUCCESS;
}

/* ---- image -------------------------------------------------------------------------------------- */
int wcpt_create_screen(wcpt_context* ctx, uint32_t width, uint32_t height)
{
    int rc = bind(ctx);
    if (rc) return rc;
    if (width == 0 || height == 0) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "zero-sized screen");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    uint32_t y0 = 0, rows = height;
    if (ctx->sharded && ctx->stripe) {
        /* interleaved stripes: kept while every row still lies in the new frame, else the full frame */
        if (ctx->rows && last_frame_row(ctx) < height) {
            y0 = ctx->y0;
            rows = ctx->rows;
        } else {
            ctx->sharded = false;
            ctx->stripe = ctx->period = 0;
        }
    } else if (ctx->sharded && ctx->y0 < height) {
        y0 = ctx->y0;
        rows = (ctx->y0 + ctx->rows <= height) ? ctx->rows : height - ctx->y0;
    } else {
        ctx->sharded = false;
    }
    rc = alloc_image(ctx, width, height, y0, rows);
    if (rc) return rc;
    /* The reference's storage image starts undefined (PathTracingRenderer.jai:345-385) and its editor's first
     * frame already blends with it (renderedFramesCount 1, editor.jai:149-152): define it as zero. */
    if (!ctx->external_bytes) {
        HIP_TRY(ctx, hipMemsetAsync(ctx->image, 0, (uint64_t)width * rows * 16ull, ctx->stream), "hipMemsetAsync(image)");
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    }
    return WCPT_SUCCESS;
}

int wcpt_resize(wcpt_context* ctx, uint32_t width, uint32_t height)
{
    return wcpt_create_screen(ctx, width, height); /* Resize = DestroyScreen + CreateScreen (:393-397) */
}

int wcpt_set_row_range(wcpt_context* ctx, uint32_t y0, uint32_t rows)
{
    int rc = bind(ctx);
    if (rc) return rc;
    if (rows == 0) {
        ctx->sharded = false;
        ctx->stripe = ctx->period = 0;
        if (ctx->height) return alloc_image(ctx, ctx->width, ctx->height, 0, ctx->height);
        return WCPT_SUCCESS;
    }
    if (ctx->height && (uint64_t)y0 + rows > ctx->height)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "row range [%u,%u) outside frame height %u", y0, y0 + rows,
                         ctx->height);
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    ctx->sharded = true;
    ctx->stripe = ctx->period = 0;
    ctx->y0 = y0;
    ctx->rows = rows;
    if (ctx->height) return alloc_image(ctx, ctx->width, ctx->height, y0, rows);
    return WCPT_SUCCESS;
}

int wcpt_set_row_stripes(wcpt_context* ctx, uint32_t y_first, uint32_t rows, uint32_t stripe, uint32_t period)
{
    if (stripe == 0) return wcpt_set_row_range(ctx, y_first, rows);
    int rc = bind(ctx);
    if (rc) return rc;
    if (rows == 0 || stripe & (stripe - 1u) || stripe > 32768u || period < stripe)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "%u rows in stripes of %u rows every %u rows", rows, stripe,
                         period);
    const uint64_t last = wcpt::frame_row64(wcpt::RowMap{y_first, (uint32_t)__builtin_ctz(stripe), period - stripe}, rows - 1u);
    if (ctx->height && last >= ctx->height)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "row stripes reach row %llu of a frame of height %u",
                         (unsigned long long)last, ctx->height);
    if (last > 0xFFFFFFFFull)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "row stripes past row 2^32");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    ctx->sharded = true;
    ctx->stripe = stripe;
    ctx->period = period;
    ctx->y0 = y_first;
    ctx->rows = rows;
    if (ctx->height) return alloc_image(ctx, ctx->width, ctx->height, y_first, rows);
    return WCPT_SUCCESS;
}

uint64_t wcpt_image_device_ptr(wcpt_context* ctx) { return ctx ? reinterpret_cast<uint64_t>(ctx->image) : 0; }

int wcpt_set_external_image(wcpt_context* ctx, uint64_t device_ptr, uint64_t bytes)
{
    int rc = bind(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    if (device_ptr == 0) {
        ctx->external_bytes = 0;
        ctx->image = ctx->own_image;
        if (ctx->width && ctx->rows) return alloc_image(ctx, ctx->width, ctx->height, ctx->y0, ctx->rows);
        return WCPT_SUCCESS;
    }
    if (bytes == 0) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "external image of 0 bytes");
    if (ctx->width && (uint64_t)ctx->width * ctx->rows * 16ull > bytes)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "external image too small for %ux%u", ctx->width, ctx->rows);
    ctx->external_bytes = bytes;
    ctx->image = reinterpret_cast<float4*>(device_ptr);
    return WCPT_SUCCESS;
}

int wcpt_set_gather_output(wcpt_context* ctx, uint64_t device_ptr, uint64_t bytes, uint32_t channels)
{
    if (!ctx) return set_error(nullptr, WCPT_ERROR_INVALID_HANDLE, "null context");
    if (device_ptr == 0) {
        ctx->wire = nullptr;
        ctx->wire_bytes = 0;
        return WCPT_SUCCESS;
    }
    if (channels != WCPT_PAYLOAD_RGB32F && channels != WCPT_PAYLOAD_RGBA32F && channels != WCPT_PAYLOAD_DISPLAY_RGBA8)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "gather output format %u (3, 4 or 8)", channels);
    if (bytes == 0 || (device_ptr & 3u))
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "gather output: %llu bytes at a misaligned or empty buffer",
                         (unsigned long long)bytes);
    if (channels == WCPT_PAYLOAD_RGBA32F && (device_ptr & 15u))
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "gather output: RGBA needs 16-byte alignment");
    ctx->wire = reinterpret_cast<float*>(device_ptr);
    ctx->wire_bytes = bytes;
    ctx->wire_ch = channels;
    return WCPT_SUCCESS;
}

int wcpt_readback(wcpt_context* ctx, float* dst, uint64_t bytes)
{
    int rc = bind(ctx);
    if (rc) return rc;
    const uint64_t have = (uint64_t)ctx->width * ctx->rows * 16ull;
    if (!ctx->image) return set_error(ctx, WCPT_ERROR_NO_SCREEN, "no output image");
    if (!dst || bytes > have) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "readback of %llu bytes, image holds %llu",
                                               (unsigned long long)bytes, (unsigned long long)have);
    HIP_TRY(ctx, hipMemcpyAsync(dst, ctx->image, bytes, hipMemcpyDeviceToHost, ctx->stream), "hipMemcpyAsync(readback)");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize(readback)");
    return read_status(ctx);
}

int wcpt_composite(wcpt_context* ctx, uint64_t dst, int format)
{
    int rc = bind(ctx);
    if (rc) return rc;
    if (!ctx->image) return set_error(ctx, WCPT_ERROR_NO_SCREEN, "no output image");
    if (format != WCPT_COMPOSITE_RGBA32F && format != WCPT_COMPOSITE_RGBA8)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "composite format %d", format);
    if (!dst) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "null composite destination");
    const uint64_t pixels = (uint64_t)ctx->width * ctx->rows;
    const uint64_t need = pixels * (format == WCPT_COMPOSITE_RGBA8 ? 4ull : 16ull);
    uint64_t off = 0;
    Buffer* b = buffer_at(ctx, dst, off);
    if (b && off + need > b->bytes)
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "composite destination holds %llu bytes, %llu needed",
                         (unsigned long long)(b->bytes - off), (unsigned long long)need);
    int dev = 0, cus = 0;
    HIP_TRY(ctx, hipGetDevice(&dev), "hipGetDevice");
    HIP_TRY(ctx, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
    HIP_TRY(ctx, wcpt::launch_composite(ctx->image, pixels, reinterpret_cast<void*>(dst), format == WCPT_COMPOSITE_RGBA8,
                                        cus, ctx->stream), "composite launch");
    return WCPT_SUCCESS;
}

int wcpt_image_upload(wcpt_context* ctx, const float* src, uint64_t bytes)
{
    int rc = bind(ctx);
    if (rc) return rc;
    const uint64_t have = (uint64_t)ctx->width * ctx->rows * 16ull;
    if (!ctx->image) return set_error(ctx, WCPT_ERROR_NO_SCREEN, "no output image");
    if (!src || bytes > have) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "image upload size");
    HIP_TRY(ctx, hipMemcpyAsync(ctx->image, src, bytes, hipMemcpyHostToDevice, ctx->stream), "hipMemcpyAsync(image)");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    return WCPT_SUCCESS;
}

/* ---- dispatch ------------------------------------------------------------------------------------ */
int wcpt_render(wcpt_context* ctx, const wcpt_scene_data* scene, uint64_t materials, uint64_t spheres,
                uint64_t draw_commands)
{
    return render_common(ctx, scene, materials, spheres, draw_commands, wcpt::kModeRender);
}

int wcpt_sync(wcpt_context* ctx)
{
    int rc = bind(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    return read_status(ctx);
}

int wcpt_render_counters(wcpt_context* ctx, const wcpt_scene_data* scene, uint64_t materials, uint64_t spheres,
                         uint64_t draw_commands, wcpt_counters* out)
{
    int rc = bind(ctx);
    if (rc) return rc;
    if (!out) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "null counters");
    HIP_TRY(ctx, hipMemsetAsync(ctx->d_counters, 0, kNumCounters * sizeof(unsigned long long), ctx->stream), "hipMemsetAsync");
    rc = render_common(ctx, scene, materials, spheres, draw_commands,
                       ctx->diagnostics ? wcpt::kModeDiag : wcpt::kModeCount);
    if (rc) return rc;
    unsigned long long h[kNumCounters];
    HIP_TRY(ctx, hipMemcpyAsync(h, ctx->d_counters, sizeof(h), hipMemcpyDeviceToHost, ctx->stream), "hipMemcpyAsync");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    out->pixels = h[0];
    out->segments = h[1];
    out->sphere_tests = h[2];
    out->node_pops = h[3];
    out->interior_visits = h[4];
    out->triangle_tests = h[5];
    out->hits = h[6];
    out->draw_fetches = h[7];
    out->wave_interior_steps = h[8];
    out->lane_interior_steps = h[9];
    out->wave_triangle_steps = h[10];
    out->lane_triangle_steps = h[11];
    out->wave_segment_steps = h[12];
    out->lane_segment_steps = h[13];
    out->ref_stack_overflow_segments = h[14];
    out->ref_stack_max = h[15] == 0xFFFFFFFFull ? UINT64_MAX : h[15];
    return read_status(ctx);
}

int wcpt_read_diagnostics(wcpt_context* ctx, uint64_t* out, uint32_t n)
{
    int rc = bind(ctx);
    if (rc) return rc;
    if (!out || n > 8) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "wcpt_read_diagnostics: bad output");
    memset(out, 0, sizeof(uint64_t) * n);
#if WCPT_MK_TIMERS
    if (ctx->kernel_run == WCPT_KERNEL_MEGAKERNEL && n) { /* megakernel phase timers of the last render */
        HIP_TRY(ctx, hipMemcpyAsync(out, ctx->d_counters, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, ctx->stream),
                "hipMemcpyAsync(timers)");
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
        return WCPT_SUCCESS;
    }
#endif
    if (!ctx->wf.pipe[0].diag || n == 0) return WCPT_SUCCESS;
    HIP_TRY(ctx, hipMemcpyAsync(out, ctx->wf.pipe[0].diag, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, ctx->stream),
            "hipMemcpyAsync(diag)");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    return WCPT_SUCCESS;
}

/* ---- timing --------------------------------------------------------------------------------------- */
int wcpt_profile_begin(wcpt_context* ctx)
{
    int rc = bind(ctx);
    if (rc) return rc;
    ctx->profiling = true;
    ctx->events_used = 0;
    ctx->region_renders = 0;
    return WCPT_SUCCESS;
}

int wcpt_profile_end(wcpt_context* ctx, double* kernel_ms_total, uint32_t* launches)
{
    int rc = bind(ctx);
    if (rc) return rc;
    const bool region = ctx->profile_region && ctx->region_renders > 0;
    if (region) HIP_TRY(ctx, hipEventRecord(ctx->events[0].second, ctx->stream), "hipEventRecord");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    double total = 0.0;
    for (size_t i = 0; i < ctx->events_used; i++) {
        float ms = 0.0f;
        HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->events[i].first, ctx->events[i].second), "hipEventElapsedTime");
        total += ms;
    }
    if (kernel_ms_total) *kernel_ms_total = total;
    if (launches) *launches = region ? ctx->region_renders : (uint32_t)ctx->events_used;
    ctx->profiling = false;
    ctx->events_used = 0;
    ctx->region_renders = 0;
    return WCPT_SUCCESS;
}

/* ---- self-test -------------------------------------------------------------------------------------- */
int wcpt_selftest_device(wcpt_context* ctx, int fn, const uint32_t* in, const uint32_t* in2, uint32_t* out, uint32_t n)
{
    int rc = bind(ctx);
    if (rc) return rc;
    if (!in || !out || ((fn == 6 || fn == 14 || fn == 16 || fn == 17) && !in2))
        return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "null selftest arrays");
    if (fn < 0 || fn > 17) return set_error(ctx, WCPT_ERROR_INVALID_ARGUMENT, "unknown selftest fn %d", fn);
    const uint64_t outw = (fn == 1) ? 4ull * n : (fn == 7 ? 3ull * n : (uint64_t)n);
    rc = ensure_scratch(ctx, (2ull * n + outw) * 4ull + 16);
    if (rc) return rc;
    uint32_t* d_in = ctx->d_scratch;
    uint32_t* d_in2 = d_in + n;
    uint32_t* d_out = d_in2 + n;
    HIP_TRY(ctx, hipMemcpyAsync(d_in, in, 4ull * n, hipMemcpyHostToDevice, ctx->stream), "selftest upload");
    if (in2) HIP_TRY(ctx, hipMemcpyAsync(d_in2, in2, 4ull * n, hipMemcpyHostToDevice, ctx->stream), "selftest upload");
    HIP_TRY(ctx, wcpt::launch_selftest(fn, d_in, d_in2, d_out, n, ctx->stream), "selftest launch");
    HIP_TRY(ctx, hipMemcpyAsync(out, d_out, 4ull * outw, hipMemcpyDeviceToHost, ctx->stream), "selftest download");
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream), "hipStreamSynchronize");
    return WCPT_SUCCESS;
}

} /* extern "C" */
