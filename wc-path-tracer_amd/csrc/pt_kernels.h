/* pt_kernels.h — launch interface between the C-ABI runtime and the HIP kernels. */
#ifndef WCPT_PT_KERNELS_H
#define WCPT_PT_KERNELS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wcpt.h"
#include "row_map.h"

namespace wcpt {

/* Traversal stack entries per lane. The reference declares 32 (pathTracer.comp:151), which a depth-32
 * midpoint BVH can overflow; our far-child stack needs at most (tree depth - 1) entries. Deeper trees set
 * the WCPT_ERROR_STACK_OVERFLOW status instead of writing out of bounds. */
constexpr int kPrivateStack = 48;          /* stack kind 0: all entries in scratch                         */
#ifndef WCPT_MK_LDS_STACK
#define WCPT_MK_LDS_STACK 16
#endif
constexpr int kLdsStack = WCPT_MK_LDS_STACK; /* stack kind 1: entries in LDS (16 x 8 B x 64 lanes = 8 KiB/wave) */
constexpr int kSpillStack = 48 - kLdsStack;  /*               + entries 16..47 spilled to scratch              */
constexpr int kStackDepth = kLdsStack + kSpillStack;

struct LaunchArgs {
    wcpt_scene_data sd;
    const wcpt_material* materials;
    const wcpt_sphere* spheres;
    const wcpt_draw_command* draws;
    const uint64_t* tri_records; /* device table [drawCommandCount] of {singles, pairs, triangle count, -} */
    bool pair_records;           /* megakernel: leaf tests on pair records (fat leaves) instead of singles */
    uint32_t wf_refill;          /* wavefront trace: idle lanes that trigger a ray fetch (1..64) */
    uint32_t wf_refill_persist;  /* the path-persistent trace's refill and shading-batch threshold (1..64) */
    int wf_fetch;                /* wavefront trace fetch rounds per iteration: -1 auto, 0 two, 1 one (WCPT_OPTION_WF_FETCH) */
    int wf_persist;              /* path-persistent trace: -1 auto, 0 off, 1 wherever eligible (WCPT_OPTION_WF_PERSIST) */
    bool wf_fast;                /* wavefront trace: draw 0 has packed stack refs, 24-bit record offsets, leaves of < 255
                                    index positions on derived records (kTriFlagSmallLeaves, kTriFlagLeafRecords) and a known
                                    node count (table flags 1|2|4|8, word 2 high half > 0) */
    uint32_t mk_tile_order;      /* static megakernel: 0 XCD-banded, 1 scattered, 2 auto, 3-6 striped bands (WCPT_OPTION_MK_TILE_ORDER) */
    float4* image;
    float* wire;                 /* gather payload (wcpt_set_gather_output) or null */
    uint32_t wire_ch;            /* its format (wcpt.h WCPT_PAYLOAD_*): 3 = RGB32F (12 B/px), 4 = RGBA32F (16 B/px), 8 = display RGBA8 (4 B/px) */
    uint32_t W, H, y0, rows;
    /* frame row of local row ly: y0 + ly + (ly >> row_shift) * row_gap (row_map.h; contiguous: 31, 0) */
    uint32_t row_shift = kContiguousShift, row_gap = 0;
    RowMap wire_rows = {0, kContiguousShift, 0}; /* the gather output's row of local row ly (row_map.h) */
    uint32_t* status;
    unsigned long long* counters;
    /* frame overlap (launch_megakernel): pipe 1's record table (its own copy of the primary-ray records) or null for
     * tri_records, and the hook that brings that copy to the frame's camera on pipe 1's stream before its launch */
    const uint64_t* tri_records_pipe1 = nullptr;
    hipError_t (*pipe1_prepare)(void* user, hipStream_t stream) = nullptr;
    void* pipe1_user = nullptr;
};

/* Wavefront path state (pt_wavefront.hip): structure-of-arrays in one device allocation. */
/* Path state indexed by queue slot (structure of arrays): the kernels that produce a queue write it compacted,
 * in append order, so every consumer reads it with coalesced loads (no per-pixel gathers). */
struct PathSoA {
    float4* ray0;      /* (origin.xyz, direction.x)                                     */
    float4* ray1;      /* (direction.yz, bounce bits, sample bits)                      */
    float4* pre;       /* (invDirection.xyz, t of the sphere loop)                      */
    float4* light;     /* (totalLight.xyz, rng state bits)                              */
    float4* trans;     /* (transmittance.xyz, -)                                        */
    uint32_t* pre_prim;/* sphere loop's winner (kSpherePrim | i) or kNoPrim             */
    uint32_t* pix;     /* pixel index (ly * W + lx) of the path                         */
};
struct WfBuffers {
    PathSoA in;        /* queue being traced / shaded this iteration                    */
    PathSoA out;       /* queue shade appends the continuing paths to                   */
    float4* hit;       /* by input slot: (t, primitive bits, draw bits, -) of Intersect */
    float4* result;    /* by pixel: sum of sample radiance .xyz                          */
    float4* prim_hit;  /* by pixel: the primary segment's Intersect record (sample 0), reused by samples 1.. */
    const uint32_t* order; /* optional trace order of the input slots (ray sorting), or null */
    uint32_t* count_in;
    uint32_t* count_out;
    uint32_t* head;    /* trace kernel's dequeue position                               */
    unsigned long long* diag; /* DIAG builds: trace-loop phase timers (8 x u64)         */
    float* wire;       /* gather payload (LaunchArgs::wire) or null                     */
    uint32_t wire_ch;
    RowMap wire_rows;  /* LaunchArgs::wire_rows                                         */
};
/* One pipeline's path state, sized by the pipeline's own path count (its share of the 8x8 tiles), not the frame:
 * the slot arrays hold only the paths that pipeline can have live at once. The per-pixel sample sums are shared
 * by the pipelines (WfPipes::result; each pixel belongs to exactly one pipeline). */
struct WfState {
    void* mem = nullptr;
    uint32_t capacity = 0;         /* path slots of the arrays in `mem` (set once every allocation succeeded) */
    PathSoA soa[2] = {};
    float4* hit = nullptr;
    uint32_t* ctr = nullptr;
    unsigned long long* diag = nullptr;
    void* sort_mem = nullptr;      /* ray-sort scratch, allocated on the first sorted render */
    uint32_t sort_capacity = 0;
    uint32_t *sort_keys = nullptr, *sort_keys_alt = nullptr, *sort_iota = nullptr, *sort_order = nullptr;
    void* sort_temp = nullptr;
    size_t sort_temp_bytes = 0;
    int cus = 0;                   /* compute units of the context's device (0 = not yet queried)          */
    int trace_bpc[3][3][3] = {};   /* trace-kernel blocks per CU by (mode, geometry variant, LDS stack)      */
    int persist_bpc = 0;           /* the path-persistent trace's blocks per CU                             */
    /* queue counters: two sets of {count q0, count q1, trace head, -}; a frame uses set `parity` and its ray generation
     * zeroes the other set for the next frame (pt_wavefront.hip WCPT_WF_CTR_PARITY); `ctr_fresh` until the first zeroing */
    uint32_t parity = 0;
    bool ctr_fresh = true;
};

/* Concurrent wavefront pipelines (WCPT_OPTION_WF_PIPES): pipeline j of K owns the 8x8 tiles t with t % K == j and
 * runs its own init / trace / shade sequence on its own stream (pipeline 0 on the context's stream), so the tail of
 * one pipeline's trace (a few slow rays on an otherwise idle chip) overlaps the bulk of another's. Paths never
 * interact, so the image and the counters are those of one pipeline. */
constexpr int kWfMaxPipes = 4;
struct WfPipes {
    WfState pipe[kWfMaxPipes];
    float4* result = nullptr;            /* by pixel: sum of sample radiance .xyz (all pipelines) */
    uint64_t result_capacity = 0;        /* pixels; `result` holds 2 x this many float4: the sums, then prim_hit */
    hipStream_t aux[kWfMaxPipes] = {};   /* [1..K-1]: created on first use, on the context's device */
    hipEvent_t fork = nullptr;
    hipEvent_t join[kWfMaxPipes] = {};
    hipEvent_t ready[kWfMaxPipes] = {};  /* pipeline j's init has run (WCPT_WF_START_TOGETHER) */
    /* frame overlap (WCPT_OPTION_FRAME_OVERLAP): pipelines 1..pending_pipes-1 hold frames the context's stream has not
     * been joined to (wf_join), of a frame of pending_W x pending_rows */
    bool pending = false;
    uint32_t pending_pipes = 0, pending_W = 0, pending_rows = 0;
    bool pending_persist = false;
};
hipError_t wf_join(WfPipes& w, hipStream_t stream);

/* Megakernel launch state, per context. */
struct MkState {
    int cus = 0;               /* CU count of the context's device (0 = not yet queried) */
    /* Cost-ordered tiles (WCPT_OPTION_MK_TILE_ORDER 2): every render records each tile's time; after the first render
     * of a frame geometry and then every kResortEvery renders the tiles are sorted by it, longest first, and the
     * following renders take that order (pt_kernels.hip launch_megakernel). */
    void* mem = nullptr;       /* cost | sorted keys | iota | order, `cap` u32 each, then the sort's scratch */
    uint32_t cap = 0;
    uint32_t* cost = nullptr;
    uint32_t* keys = nullptr;
    uint32_t* iota = nullptr;
    uint32_t* order = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    uint32_t geom_w = 0, geom_rows = 0, geom_y0 = 0, geom_tiles = 0; /* geometry the costs and order belong to */
    uint32_t geom_shift = kContiguousShift, geom_gap = 0;            /* ... and its frame rows (row_map.h) */
    uint32_t renders = 0;      /* renders of that geometry */
    bool order_valid = false;
    /* Frame overlap (WCPT_OPTION_FRAME_OVERLAP, pt_kernels.hip launch_megakernel): a render splits the cost-ordered
     * tiles between two pipes (tile list `split`: the order's even positions, then its odd ones), pipe 0 on the
     * context's stream and pipe 1 on a stream of its own, and the next render's pipes continue without waiting for the
     * other pipe -- each pipe owns the same pixels in every frame, so per pixel the frames stay in order. `pending`: frames on the pipe streams that the
     * context's stream has not been joined to (mk_join; every entry point other than a render joins first). */
    uint32_t* split = nullptr; /* `cap` u32 after `order` */
    bool split_valid = false;
    bool pending = false;
    uint32_t pending_tiles = 0;
    hipStream_t pipe[2] = {};  /* [1]: pipe 1's stream (pipe 0 runs on the context's stream) */
    hipEvent_t fork = nullptr;
    hipEvent_t join[2] = {};
};
constexpr uint32_t kMkPipes = 2;
void mk_release(MkState& mk);
/* The context's stream continues after every frame the overlap pipes hold (no-op when none is pending). */
/* A group suppresses the overlap on a context whose frames it joins every frame anyway (a sender's ready event, the
 * root's in-line receives): there a fork and a join per frame would cost more than the tail they hide. */
void set_overlap_suppressed(wcpt_context* ctx, bool on);
/* The streams that hold the context's last frame and will run its next one: the context's stream, then the overlap
 * pipes' streams while frames are pending on them (at most kMaxFrameStreams). A group fences a frame's payload with an
 * event on each (and makes each wait for the payload's previous transfer) instead of joining the pipes every frame. */
constexpr int kMaxFrameStreams = 4;
int context_frame_streams(wcpt_context* ctx, hipStream_t* out, int cap);
hipError_t mk_join(MkState& mk, hipStream_t stream);

/* Launch modes: render the frame; count the reference algorithm's work (no image write); count + SIMD
 * diagnostics (ballot-based step counters, tools/diag.py). */
constexpr int kModeRender = 0, kModeCount = 1, kModeDiag = 2;

/* Derived triangle records (pt_device.h): triangle k = index positions 3k..3k+2 stored as (a, b - a, c - a);
 * singles: 48 B per triangle; pairs: 80 B per triangle pair (2j, 2j+1). */
constexpr uint32_t kSingleRecordBytes = 48, kPairRecordBytes = 80;
/* primary-ray pair records (pt_device.h TriPairP), built with launch_build_primary_pairs; WCPT_PRIMARY_PAIRS=0 turns
 * them off (the device then never finds a primary record address in the table) */
constexpr uint32_t kPrimPairRecordBytes = 112;
#ifndef WCPT_PRIMARY_PAIRS
#define WCPT_PRIMARY_PAIRS 1
#endif
/* vertex_count bounds the vertex indices read (0xFFFFFFFF: unknown); a triangle with an index past it gets a NaN
 * record, which no ray accepts. */
/* Primary-ray pair records (pt_device.h TriPairP) of `npairs` pair records for the camera origin (ox, oy, oz). */
hipError_t launch_build_primary_pairs(const void* pairs, uint32_t npairs, float ox, float oy, float oz, void* out,
                                      hipStream_t stream);
/* *flags (zeroed here): bit 0 when some leaf of the BVH has triangleCount >= 255 (pt_device.h kRefFetch), bit 1 when
 * some leaf's triangles are not all derived records of the draw's `triangles` (pt_device.h kTriFlagLeafRecords) */
hipError_t launch_scan_leaf_counts(const void* bvh, uint32_t nodes, uint32_t triangles, uint32_t* flags,
                                   hipStream_t stream);
hipError_t launch_build_tri_records(const uint32_t* indices, const float* vertices, uint32_t triangles,
                                    uint32_t vertex_count, void* singles, void* pairs, hipStream_t stream);
/* composite.comp (pt_composite.hip): gamma + PBR Neutral over `pixels` float4 texels into rgba32f or RGBA8 */
hipError_t launch_composite(const float4* img, uint64_t pixels, void* dst, bool rgba8, int cus, hipStream_t stream);
/* overlap: WCPT_OPTION_FRAME_OVERLAP as the runtime allows it for this render (0 off, 1 auto, 2 on whenever the tiles
 * are cost-ordered); with 0 a pending overlap is joined first and the frame runs on `stream` */
hipError_t launch_megakernel(const LaunchArgs& a, int mode, int stack_kind, MkState& mk, hipStream_t stream,
                             int overlap = 0);
/* sort_rays: sort the ray queue by (direction octant, origin Morton code) before each bounce's trace. */
/* lds_stack: LDS traversal-stack entries per lane of the trace kernel (10, 16 or 24; render mode only). */
/* pipes: concurrent pipelines (1..kWfMaxPipes; sorting and diagnostics use 1). */
hipError_t launch_wavefront(const LaunchArgs& a, int mode, WfPipes& w, int pipes, bool sort_rays, int lds_stack,
                            hipStream_t stream, int overlap = 0);
hipError_t wf_reserve(WfState& s, uint32_t paths);
hipError_t wf_reserve_sort(WfState& s, uint32_t paths);
void wf_release(WfState& s);
void wf_release(WfPipes& w);
hipError_t launch_selftest(int fn, const uint32_t* in, const uint32_t* in2, uint32_t* out, uint32_t n,
                           hipStream_t stream);

/* wcpt_runtime.hip internals used by the multi-device group (wcpt_group.hip) */
hipStream_t context_stream(wcpt_context* ctx);
int context_device(wcpt_context* ctx);
int context_error(wcpt_context* ctx, int code, const char* msg);
int render_validate(wcpt_context* ctx, const wcpt_scene_data* scene, uint64_t materials, uint64_t spheres,
                    uint64_t draws);
/* CreateScreen of one context's rows: a block [y0, y0 + rows), or (stripe > 0) interleaved stripes (row_map.h) */
int set_frame_block(wcpt_context* ctx, uint32_t width, uint32_t height, uint32_t y0, uint32_t rows, uint32_t stripe = 0,
                    uint32_t period = 0);
void render_abandon(wcpt_context* ctx);

} // namespace wcpt

#endif
