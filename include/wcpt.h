/*
 * wcpt.h — C-ABI drop-in boundary for the WC-Path-tracer compute path on MI355X (gfx950).
 *
 * This header is the only interface the reference's Jai host would see. It replaces the
 * Vulkan compute dispatch of `src/PathTracingRenderer.jai` (reference @ /root/reference):
 *
 *   reference (file:line)                                   replaced by
 *   -----------------------------------------------------   -----------------------------------------
 *   DBufferManager Allocate   src/BufferManager.jai:19-34    wcpt_buffer_alloc
 *   DBufferManager Update     src/BufferManager.jai:52-64    wcpt_buffer_upload   (grow-on-demand, :53-54)
 *   DBufferManager Free       src/BufferManager.jai:36-45    wcpt_buffer_free
 *   GetDeviceAddress          modules/VKUtils/Buffer.jai:101  wcpt_buffer_device_address
 *   CreateScreen              src/PathTracingRenderer.jai:345 wcpt_create_screen  (rgba32f image -> float4[H][W])
 *   Resize                    src/PathTracingRenderer.jai:393 wcpt_resize
 *   Render (push block + vkCmdDispatch)
 *                             src/PathTracingRenderer.jai:399-457  wcpt_render (SceneData by value + 3 BDAs)
 *   Submit / timeline wait    modules/VKUtils/Synchronization.jai:64-89, src/main.jai:73-95  wcpt_sync
 *   Deinit                    src/PathTracingRenderer.jai:473 wcpt_destroy
 *
 * Byte layouts of the POD types are the reference's GLSL `scalar` block layouts, which are identical to
 * the Jai structs (src/shaders/pathTracer.comp:10-95, src/PathTracingRenderer.jai:38-140).
 *
 * Errors: every entry point returns int (0 = success, negative = error; -1..-13 keep VkResult meaning).
 * Nothing aborts or exits. wcpt_last_error() gives a human-readable message.
 * Threading: one context per device; calls on one context are not thread-safe (the reference drives the
 * renderer from a single thread, src/main.jai:185-194).
 */
#ifndef WCPT_H
#define WCPT_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: wcpt_counters gained ref_stack_overflow_segments / ref_stack_max; the wcpt_group_* multi-device entry points.
 * 3: groups overlap each frame's gather with the next frame's render; wcpt_group_create_ex (transports),
 *    wcpt_group_unique_id / wcpt_group_create_rank (one process per device), wcpt_group_set_option, wcpt_group_info.
 * 4: WCPT_GROUP_OPTION_THREADS (each local rank's share of a frame issued from a host thread of its own);
 *    wcpt_group_info gained issue_threads; wcpt_group_set_output reads `bytes` in every process. Later additions that
 *    keep the layouts and calls (no version step): WCPT_GROUP_TRANSPORT_DIRECT, WCPT_OPTION_PROFILE_REGION,
 *    WCPT_OPTION_WF_FETCH, WCPT_OPTION_WF_PIPES 0 (automatic, now the default). */
#define WCPT_ABI_VERSION 4

/* ---- error codes (VkResult-compatible where a VkResult exists) ---------------------------------- */
#define WCPT_SUCCESS                      0
#define WCPT_ERROR_OUT_OF_HOST_MEMORY    (-1)
#define WCPT_ERROR_OUT_OF_DEVICE_MEMORY  (-2)
#define WCPT_ERROR_INITIALIZATION_FAILED (-3)
#define WCPT_ERROR_DEVICE_LOST           (-4)
#define WCPT_ERROR_UNKNOWN               (-13)
#define WCPT_ERROR_INVALID_ARGUMENT      (-1000)
#define WCPT_ERROR_INVALID_HANDLE        (-1001)
#define WCPT_ERROR_STACK_OVERFLOW        (-1002) /* BVH deeper than the traversal stack */
#define WCPT_ERROR_NO_SCREEN             (-1003) /* wcpt_render before wcpt_create_screen */
#define WCPT_ERROR_PARSE                 (-1004) /* OBJ text could not be parsed */

/* ---- material types (pathTracer.comp:30-33, PathTracingRenderer.jai:53-56) ---------------------- */
#define WCPT_MATERIAL_METAL      0u
#define WCPT_MATERIAL_DIELECTRIC 1u

/* ---- kernel variants ---------------------------------------------------------------------------- */
#define WCPT_KERNEL_MEGAKERNEL  0  /* one lane per pixel, exact reference semantics (default)          */
#define WCPT_KERNEL_WAVEFRONT   2  /* split ray-gen / traverse / shade queues (same semantics)         */
/* Chosen per render from the scene: the megakernel where the draws' leaves hold several triangles each (the pair-record
 * layout: Cornell-class and the reference's mushroom), the wavefront kernel for thin-leaf meshes (a Sponza-scale
 * midpoint BVH, ~2 triangles per leaf), the faster of the two on every bench scene. Same results either way. */
#define WCPT_KERNEL_AUTO        1

/* ---- tuning options (wcpt_set_option); none changes results ------------------------------------- */
#define WCPT_OPTION_STACK       1  /* megakernel traversal stack: 0 = scratch, 1 = LDS + spill (default) */
#define WCPT_OPTION_DIAGNOSTICS 2  /* 1: wcpt_render_counters also fills the SIMD-efficiency fields      */
#define WCPT_OPTION_SORT_RAYS   3  /* wavefront: sort bounce rays by (octant, origin Morton) (default 0) */
#define WCPT_OPTION_WF_STACK    4  /* wavefront: LDS traversal-stack entries per lane, 10 | 16 | 24 (default 10) */
/* Derived triangle records. wcpt_render derives per draw command one 48-byte record per triangle (a, b-a, c-a)
 * from the draw's index and vertex buffers; leaf tests read them instead of index + vertex gathers (same
 * arithmetic, same results). 1 (default): rebuilt only when a draw's buffers were re-uploaded through
 * wcpt_buffer_upload / re-allocated, or its buffers or index count changed; the draw commands themselves are read
 * from the context's host copy of what wcpt_buffer_upload wrote (bytes never uploaded are read from the device).
 * The same cache holds what the runtime learns about each draw's BVH buffer (whether every leaf is small and lies on
 * the derived records, which selects the wavefront's fast leaf layout); it is re-learned when the BVH buffer is
 * re-uploaded through wcpt_buffer_upload or re-allocated.
 * 0: the draw commands are read from the device, the records rebuilt on every render and the fast leaf layout is not
 * used (use this when the application writes draw-command, vertex, index or BVH buffers by other means, e.g. hipMemcpy
 * to a wcpt_buffer_device_address, a refit or its own kernels: with 1, such writes into uploaded ranges are not
 * seen). A BVH rewritten behind the cache can give a wrong image but never a read outside the derived records. */
#define WCPT_OPTION_TRIANGLE_CACHE 5
/* Megakernel leaf tests: -1 (default) choose by mean triangles per leaf; 0 single records; 1 pair records
 * (two triangles per lane with packed-FP32 arithmetic). Results are identical either way. */
#define WCPT_OPTION_PAIR_RECORDS 6
/* Traversal stack entries carry the deferred child's (left, count) (1, default, when the draw's BVH buffer is a
 * context buffer of < 2^24 nodes) so a pop needs no node fetch; 0: entries hold node indices. Same results. */
#define WCPT_OPTION_PACKED_REFS 7
/* Wavefront trace: a wave fetches new rays once this many of its 64 lanes are idle (1..64, default 20: fewer,
 * fuller fetch rounds; c3 9.0 -> 8.2 ms at 12 against 1; round 5, with the finished lanes' hit records stored at the
 * refill: c4 197.8-198.2 ms at 20 against 199.5 at 12 and 201.3 at 32, c3 unchanged within the spread). The
 * path-persistent trace (WCPT_OPTION_WF_PERSIST) reads it as its fetch and shading-batch threshold too, with its own
 * default of 12 while the option is unset (round 6: c3 8-way shares 1 % faster than at 20); a value set here governs
 * both. */
#define WCPT_OPTION_WF_REFILL 8
/* Megakernel tile order: 0 each XCD walks a contiguous band of 8x8 tiles; 1 scattered (tile b * m mod tiles), so the
 * tiles resident on a CU at once come from all over the frame; 3, 4, 5, 6 XCD bands striped by 1, 2, 4, 8 tile rows
 * (XCD x walks the stripes s = x mod 8, so every XCD sees every part of the frame while neighbouring tiles stay
 * together); 2 (default) cost-ordered: every render records each tile's time, and after the first render of a frame
 * geometry (width, rows, first row) and every 64 renders the tiles are sorted by it, longest first, for the renders
 * that follow (the launch's last round then holds the short tiles). Until the first sort: scattered when the launch
 * fits in about one round of resident waves, stripes of one tile row otherwise. Same results in every order. */
#define WCPT_OPTION_MK_TILE_ORDER 9
/* Wavefront: concurrent pipelines (1..4, or 0 = the default: on the path-persistent trace 1, or 2 under the frame
 * overlap; else 3 when the frame holds at most 8 paths per resident trace lane, else 2). Pipeline j renders the 8x8
 * tiles t with t % K == j on its own stream, so one pipeline's trace tail (a few slow rays) overlaps another's bulk.
 * Same results. */
#define WCPT_OPTION_WF_PIPES 10
/* Kernel timing (wcpt_profile_begin / wcpt_profile_end): 0 (default) one pair of HIP events around every render;
 * 1 two events for the whole profiled region, one before its first render and one recorded by wcpt_profile_end, so
 * kernel_ms_total spans the renders' launches and the gaps between them, and launches counts the renders. Each event
 * record is a packet on the stream: per-render pairs cost ~1.3 % of a 0.36-ms frame (c2: 0.3651-0.3660 against
 * 0.3607-0.3611 ms per frame without, profiles/r05_events_ab.log). Set it outside a profiled region. */
#define WCPT_OPTION_PROFILE_REGION 11
/* Wavefront trace: fetch rounds per traversal iteration. 1: the child pair of an interior lane and the triangle of a
 * leaf lane are fetched together (a lane that descends into a leaf tests it the next iteration); 0: the leaf fetch
 * follows the interior step, so a descent tests its first triangle in the same iteration; -1 (default): one round
 * when a pipeline's queue holds at most 8 rays per resident trace lane (fetch latency exposed), two otherwise
 * (issue-bound). Same results. */
#define WCPT_OPTION_WF_FETCH 12
/* Wavefront: the path-persistent trace, one launch per frame in which each lane runs its path's segments one after
 * another and shades between them, for one sample per pixel on one-draw scenes. -1 (default): where the frame has at
 * most 1.4 paths per resident lane of it (row blocks), 0 never, 1 whenever eligible. Same results. */
#define WCPT_OPTION_WF_PERSIST 13
/* The gather output (wcpt_set_gather_output) addressed by frame row: 1 = the pixel of frame row y goes to row y of
 * the output (a buffer of the whole frame, which several contexts can share, each writing only its own rows -- rows
 * blocks or interleaved stripes alike); 0 (default) = the context's rows back to back (row ly of its rows at row ly).
 * Added under ABI 4. */
#define WCPT_OPTION_GATHER_FRAME_ROWS 14
/* Frame overlap (megakernel, cost-ordered tiles): consecutive renders with no other call on the context between them
 * run as two pipes, each on a stream of its own and owning half the tiles (the same pixels in every frame), so one
 * pipe's next frame starts in the other's last round of waves instead of behind the whole frame. Every other entry
 * point (wcpt_sync, readback, composite, profile end, buffer calls, a group's exchange ...) first orders the context's
 * stream after both pipes, so what it sees or queues is as if each render had run on the stream; hence only on the
 * context's own stream (not after wcpt_set_stream) and not under per-render timing events. 1 (default): megakernel
 * launches from 1.5 rounds of resident waves up (a 1920x1080 frame or its 2- and 4-way row blocks, not an 8-way block),
 * wavefront frames of several pipelines; 0 off; 2 whenever the tiles are cost-ordered (worth it on a one-round launch
 * whose waves differ much in length: the reference's scene in an 8-way block 0.308 -> 0.260 ms, the Cornell box +0.9 %).
 * Same results. Added under ABI 4. */
#define WCPT_OPTION_FRAME_OVERLAP 15

/* ---- POD types with the reference byte layouts -------------------------------------------------- */

/* SceneData — pathTracer.comp:10-22 == PathTracingRenderer.jai:38-51. 164 bytes.
 * Matrices are column-major (GLSL mat4), as the Jai host uploads them after transpose()
 * (PathTracingRenderer.jai:28,33). */
typedef struct wcpt_scene_data {
    float    inverseProjection[16]; /*   0 */
    float    inverseView[16];       /*  64 */
    float    position[3];           /* 128 */
    uint32_t maxBounceCount;        /* 140  (Jai default 3) */
    uint32_t samples;               /* 144  (Jai default 1) */
    uint32_t sphereCount;           /* 148 */
    uint32_t drawCommandCount;      /* 152 */
    uint32_t renderedFramesCount;   /* 156 */
    uint32_t boxID;                 /* 160  (unused by the kernel) */
} wcpt_scene_data;

/* Material — pathTracer.comp:35-47 == PathTracingRenderer.jai:58-70. 60 bytes. */
typedef struct wcpt_material {
    uint32_t type;                  /*  0  WCPT_MATERIAL_* (Jai default METAL) */
    float    albedo[3];             /*  4 */
    float    emission[3];           /* 16 */
    float    emissionStrength;      /* 28  (Jai default 0) */
    float    metallic;              /* 32  (unused by the kernel) */
    float    roughness;             /* 36 */
    float    absorption[3];         /* 40 */
    float    absorptionStrength;    /* 52  (Jai default 1) */
    float    ior;                   /* 56  (Jai default 1) */
} wcpt_material;

/* Sphere — pathTracer.comp:60-64 == PathTracingRenderer.jai:86-90. 20 bytes. */
typedef struct wcpt_sphere {
    float    position[3];
    float    radius;
    uint32_t material;
} wcpt_sphere;

/* Node — pathTracer.comp:66-72 == PathTracingRenderer.jai:125-134. 32 bytes.
 * triangleCount counts INDICES (3 per triangle); 0 means interior, whose children are at
 * leftNodeOrTriangleIndex and leftNodeOrTriangleIndex+1. */
typedef struct wcpt_node {
    float    min[3];
    float    max[3];
    uint32_t leftNodeOrTriangleIndex;
    uint32_t triangleCount;
} wcpt_node;

/* DrawCommand — pathTracer.comp:82-87 == PathTracingRenderer.jai:135-140. The array stride is the Jai
 * size_of = 32 bytes (28 bytes of fields + 4 bytes tail padding). The three fields are device
 * addresses from wcpt_buffer_device_address(). The reference's kernel never reads indexCount; this runtime does:
 * it derives the triangle records from index positions [0, indexCount), so indexCount must not exceed the index
 * buffer (checked for context buffers: wcpt_render returns WCPT_ERROR_INVALID_ARGUMENT), and vertex indices past a
 * context vertex buffer give a triangle that is never hit. Write draw commands through wcpt_buffer_upload, or see
 * WCPT_OPTION_TRIANGLE_CACHE. */
typedef struct wcpt_draw_command {
    uint64_t vertexBuffer;          /* -> float[3] positions, stride 12 */
    uint64_t indexBuffer;           /* -> uint32 indices (BVH-permuted) */
    uint64_t bvhBuffer;             /* -> wcpt_node[] */
    uint32_t indexCount;
    uint32_t _pad;
} wcpt_draw_command;

/* Camera — PathTracingRenderer.jai:6-20 (the Jai Matrix4s are stored here already in the column-major
 * order the shader reads). */
typedef struct wcpt_camera {
    float position[3];
    float direction[3];
    float yaw;
    float pitch;
    float fov;                      /* vertical, degrees (Jai default 90) */
    float projection[16];
    float view[16];
    float inverseProjection[16];
    float inverseView[16];
} wcpt_camera;

/* Per-frame work counters of the reference algorithm; exact integers. */
typedef struct wcpt_counters {
    uint64_t pixels;          /* pixels rendered                                                   */
    uint64_t segments;        /* Intersect() calls = ray segments (the "rays" of Mray/s)          */
    uint64_t sphere_tests;    /* raySphereIntersect calls                                          */
    uint64_t node_pops;       /* BVH nodes popped from the stack (reference :158-159)              */
    uint64_t interior_visits; /* interior nodes whose two children were fetched (:183-184)        */
    uint64_t triangle_tests;  /* rayTriangleIntersect calls (:170)                                 */
    uint64_t hits;            /* segments that hit (material fetched, :251)                        */
    uint64_t draw_fetches;    /* DrawCommand fetches (:153)                                        */
    /* SIMD-efficiency diagnostics of this implementation (not reference work; 0 from the oracle):
     * per phase, wave-steps (a wave executed the step with >= 1 lane) and lane-steps (lanes that did).
     * lane/(64*wave) is the fraction of the 64 lanes doing useful work in that phase. */
    uint64_t wave_interior_steps, lane_interior_steps;
    uint64_t wave_triangle_steps, lane_triangle_steps;
    uint64_t wave_segment_steps, lane_segment_steps;
    /* The reference's traversal stack is `uint nodeStack[32]` (pathTracer.comp:151), pushed with the root (:155) and
     * both children of every interior node that survives its box test (:192-198). Counted exactly for the same frame
     * (ABI version 2): segments in which the reference writes nodeStack[32] or beyond -- undefined behaviour in the
     * reference, whose result for those rays has no reference meaning -- and the deepest stack the reference reaches
     * (entries after a push; UINT64_MAX if the tree was too deep to track, > 64 levels). This implementation's own
     * stack (48 entries, far children only) is unaffected by either. */
    uint64_t ref_stack_overflow_segments;
    uint64_t ref_stack_max;
} wcpt_counters;

/* Host mesh produced by the OBJ loader (ModelLoader.jai:60-141) or a scene generator. Memory is owned
 * by the library; release with wcpt_mesh_free. */
typedef struct wcpt_mesh {
    float*    positions;      /* vertex_count * 3 floats */
    uint32_t  vertex_count;
    uint32_t* indices;        /* index_count uint32 */
    uint32_t  index_count;
} wcpt_mesh;

/* Host scene (geometry + materials + spheres + camera). Owned by the library; wcpt_scene_free. */
typedef struct wcpt_scene {
    wcpt_mesh      mesh;
    wcpt_material* materials;
    uint32_t       material_count;
    wcpt_sphere*   spheres;
    uint32_t       sphere_count;
    wcpt_camera    camera;
} wcpt_scene;

typedef struct wcpt_context wcpt_context;
typedef uint64_t wcpt_buffer;      /* 0 is never a valid handle */

/* ---- library / context ---------------------------------------------------------------------------- */
int         wcpt_abi_version(void);
/* Identity of the sources and compile flags that decide this build's kernels and their launches (a short hash; the
 * multi-device group's exchange code and this header's comments are left out): measurements recorded against one
 * build (e.g. a counter profile) can tell whether they describe the kernels of the library that is loaded. */
const char* wcpt_build_id(void);
int         wcpt_device_count(int* count);
/* The PCI bus id of a device ("dddd:bb:dd.f", NUL-terminated in out[0..len)): identifies a GPU across processes that
 * see different device ordinals (e.g. a launcher that makes one device visible per process). */
int         wcpt_device_pci_bus_id(int device, char* out, int len);
int         wcpt_create(int device, wcpt_context** out_ctx);
int         wcpt_destroy(wcpt_context* ctx);                       /* Deinit, PathTracingRenderer.jai:473 */
const char* wcpt_last_error(const wcpt_context* ctx);              /* ctx may be NULL: last global error */
int         wcpt_set_stream(wcpt_context* ctx, void* hip_stream);  /* NULL: the context's own stream     */
int         wcpt_set_kernel(wcpt_context* ctx, int variant);       /* WCPT_KERNEL_*                       */
int         wcpt_last_kernel(wcpt_context* ctx, int* variant);     /* what the last render ran (AUTO resolved) */
int         wcpt_set_option(wcpt_context* ctx, int option, int value); /* WCPT_OPTION_*                   */

/* ---- device buffers (BufferManager.jai) ------------------------------------------------------------ */
int      wcpt_buffer_alloc(wcpt_context* ctx, uint64_t bytes, wcpt_buffer* out);
int      wcpt_buffer_upload(wcpt_context* ctx, wcpt_buffer buf, const void* src, uint64_t bytes,
                            uint64_t offset);  /* grows (reallocates) when offset+bytes > size, like :53-54 */
int      wcpt_buffer_download(wcpt_context* ctx, wcpt_buffer buf, void* dst, uint64_t bytes,
                              uint64_t offset);
int      wcpt_buffer_size(wcpt_context* ctx, wcpt_buffer buf, uint64_t* out_bytes);
uint64_t wcpt_buffer_device_address(wcpt_context* ctx, wcpt_buffer buf); /* 0 on error */
int      wcpt_buffer_free(wcpt_context* ctx, wcpt_buffer buf);

/* ---- output image (CreateScreen / Resize) --------------------------------------------------------- */
/* The context-owned image starts as zeros (the reference's is undefined; its editor blends frame 1 with it). */
int      wcpt_create_screen(wcpt_context* ctx, uint32_t width, uint32_t height);
int      wcpt_resize(wcpt_context* ctx, uint32_t width, uint32_t height);
/* Row-block shard: this context renders and stores only rows [y0, y0+rows) of the width x height
 * frame (global pixel indices and seeds unchanged). rows == 0 resets to the full frame. */
int      wcpt_set_row_range(wcpt_context* ctx, uint32_t y0, uint32_t rows);
/* Interleaved row stripes (SURVEY.md §8(e)'s fallback when static blocks cap the scaling): this context renders
 * `rows` rows of the frame -- stripes of `stripe` rows every `period` rows, the first starting at frame row y_first,
 * the last possibly short -- and stores them back to back ([rows][width]): local row ly is frame row
 * y_first + ly + (ly / stripe) * (period - stripe). Seeds and pixel indices stay global (pathTracer.comp:304), so the
 * rows are bit-identical to a whole-frame render's. `stripe` is a power of two (1..32768), period >= stripe;
 * stripe == 0 is wcpt_set_row_range(y_first, rows). wcpt_row_stripes gives rank r of n its (y_first, rows) for
 * period = n * stripe. Added under ABI 4. */
int      wcpt_set_row_stripes(wcpt_context* ctx, uint32_t y_first, uint32_t rows, uint32_t stripe, uint32_t period);
uint64_t wcpt_image_device_ptr(wcpt_context* ctx);                 /* float4[rows][width], pitch width*16 */
/* Render into caller-owned device memory (e.g. a torch tensor handed to RCCL, or imported interop memory)
 * instead of the context's own image. `bytes` must hold width*rows*16. device_ptr == 0 reverts to the
 * context-owned image. The caller keeps ownership. */
int      wcpt_set_external_image(wcpt_context* ctx, uint64_t device_ptr, uint64_t bytes);
/* Gather payload written by the render itself: every wcpt_render also stores each pixel it
 * finishes into caller-owned device memory at `device_ptr`, row-major [rows][width], in payload format `channels`:
 *   WCPT_PAYLOAD_RGB32F (3)  float RGB, the accumulation image's values (alpha is always 1.0, pathTracer.comp:323);
 *   WCPT_PAYLOAD_RGBA32F (4) float RGBA, the accumulation image's values (16-byte aligned);
 *   WCPT_PAYLOAD_DISPLAY_RGBA8 (8) the display step of composite.comp:36-53 (gamma 1/2.2 + PBR Neutral, UNORM8 as
 *     wcpt_composite's RGBA8) of the accumulated value, 4 B/px: a presented multi-device frame at a quarter of the
 *     float payload's bytes, with no separate composite pass.
 * A multi-GPU host points it at the buffer it hands to the collective, so no copy kernel sits between the render and
 * the gather. `bytes` must hold width*rows*(bytes per pixel) at render time. device_ptr == 0 turns it off. Takes
 * effect for the next render; no synchronisation. The caller keeps ownership. */
#define WCPT_PAYLOAD_RGB32F        3
#define WCPT_PAYLOAD_RGBA32F       4
#define WCPT_PAYLOAD_DISPLAY_RGBA8 8
int      wcpt_set_gather_output(wcpt_context* ctx, uint64_t device_ptr, uint64_t bytes, uint32_t channels);
int      wcpt_readback(wcpt_context* ctx, float* dst, uint64_t bytes);
int      wcpt_image_upload(wcpt_context* ctx, const float* src, uint64_t bytes); /* seed accumulation */

/* ---- display step after the path (composite.comp:3-54) ------------------------ */
/* Gamma 1/2.2 + PBR Neutral tonemap of the accumulation image (this context's rows) into caller-owned device
 * memory at `dst` (e.g. wcpt_buffer_device_address of a buffer of width*rows*16 or *4 bytes). Asynchronous on
 * the context's stream. RGBA32F is what composite.comp stores; RGBA8 (UNORM, round to nearest) is the display
 * format (4x fewer bytes for readback or a multi-GPU gather). */
#define WCPT_COMPOSITE_RGBA32F 0
#define WCPT_COMPOSITE_RGBA8   1
int      wcpt_composite(wcpt_context* ctx, uint64_t dst, int format);

/* ---- dispatch ---------------------------------------------------------------------------------------- */
/* The push block of pathTracer.comp:90-95 minus `sdp`: SceneData travels by value. Asynchronous on the
 * context's stream; the caller owns renderedFramesCount sequencing (PathTracingRenderer.jai:423). */
int      wcpt_render(wcpt_context* ctx, const wcpt_scene_data* scene, uint64_t materials,
                     uint64_t spheres, uint64_t draw_commands);
int      wcpt_sync(wcpt_context* ctx);
/* Same frame through the instrumented kernel: counts the reference algorithm's work.
 * Does not write the image. Synchronous. */
int      wcpt_render_counters(wcpt_context* ctx, const wcpt_scene_data* scene, uint64_t materials,
                              uint64_t spheres, uint64_t draw_commands, wcpt_counters* out);

/* Wavefront trace-loop phase timers of the last wcpt_render_counters call with WCPT_OPTION_DIAGNOSTICS set
 * (s_memtime cycles summed over waves): {fetch, leaf, interior, pop, epilogue, waves, iterations, -}. */
int      wcpt_read_diagnostics(wcpt_context* ctx, uint64_t* out, uint32_t n);

/* ---- one frame on several devices ------------------------------------------------------- */
/* The reference host is one process and one thread (main.jai:185-194) driving Render (PathTracingRenderer.jai:399).
 * A group keeps that shape for N devices: one context per device, rank r rendering rows [r*H/N, (r+1)*H/N) of the
 * frame with unchanged global pixel indices and seeds (so the frame equals a one-device render bit for bit), and one
 * exchange per presented frame: the row blocks go to the root device over xGMI (blocks may differ by a row).
 *   wcpt_group_create      one process, one thread, devices[0..n) distinct device ordinals, RCCL transport
 *                          (ncclCommInitAll, rccl.h:236; grouped ncclSend/ncclRecv, rccl.h:700,722). `root` is the
 *                          rank that receives the frame.
 *   wcpt_group_create_ex   the same with a transport: WCPT_GROUP_TRANSPORT_RCCL, WCPT_GROUP_TRANSPORT_COPY
 *                          (hipMemcpyPeerAsync of each block into the root's frame, on the sending device's copy
 *                          path; a device may then be listed more than once, so an N-rank group can be rehearsed on
 *                          fewer devices: every rank still has its own context, streams and payloads), or
 *                          WCPT_GROUP_TRANSPORT_DIRECT (each render writes its block into the root's frame itself).
 *                          Status: RCCL between n > 1 distinct GPUs over xGMI is UNVERIFIED on hardware here (the
 *                          development boxes have one GPU). The one-process-per-device form (below) has run with 2,
 *                          4 and 8 ranks on one GPU over RCCL's socket transport (bench.py --rccl-rehearsal, frame verified
 *                          bit-exact); the COPY and DIRECT transports run the same bookkeeping and are tested with 2-8
 *                          ranks on one GPU.
 *   wcpt_group_unique_id / wcpt_group_create_rank   one process per device (e.g. one process per GPU under
 *                          torchrun): the root's process makes the id (ncclGetUniqueId), the host hands its 128 bytes
 *                          to every process, and each process creates its rank (ncclCommInitRank). RCCL only. All
 *                          processes then make the same wcpt_group_* calls in the same order (collective).
 *   wcpt_group_context     rank r's context (NULL for a rank of another process): upload that device's copy of the
 *                          scene with wcpt_buffer_* and set kernels/options on it, as for a single context. Owned by
 *                          the group.
 *   wcpt_group_create_screen  CreateScreen/Resize for the whole frame (each rank allocates only its row block).
 *   wcpt_group_set_output  where the presented frame goes: device memory on the root device (e.g.
 *                          wcpt_buffer_device_address of a root-context buffer) of `bytes` >= width*height*(payload
 *                          bytes per pixel), row-major, in WCPT_PAYLOAD_* format; format 0 turns presenting off (the
 *                          ranks keep accumulating their blocks), and so does dst == 0 in a one-process group. Every
 *                          process passes the same `format` and `bytes` (a process that does not hold the root ignores
 *                          `dst`), so each makes the same decision on them and on later resizes. The root renders its
 *                          own block straight into the output; the other ranks' renders write their blocks into
 *                          group-owned payload buffers (no copy pass).
 *   wcpt_group_render      Render on every rank of this process (scene by value; materials/spheres/draw_commands are
 *                          arrays of one device address per local rank, in rank order), then, with an output set,
 *                          the gather of this frame. Asynchronous, like wcpt_render. Every rank's arguments are
 *                          checked before any rank renders, so an argument error leaves every rank's accumulation as
 *                          it was. With WCPT_GROUP_OPTION_OVERLAP (default 1) each rank's transfer runs on a
 *                          communication stream of its own, ordered after that rank's render by an event, while the
 *                          next frame renders into a second payload buffer; a render waits (on the device, not the
 *                          host) only for the transfer that last read the payload it rewrites. 0: transfers run on
 *                          the render streams, in line with the renders.
 *   wcpt_group_sync        waits for every local rank's renders and transfers (and reports a traversal-stack
 *                          overflow on any of them). The presented frame is complete after it. The wait is bounded
 *                          (WCPT_GROUP_OPTION_TIMEOUT_MS): a frame whose exchange cannot complete (a peer failed or
 *                          skipped it) ends in WCPT_ERROR_DEVICE_LOST, not in a hang.
 * Errors leave the group usable, except (a) any failure once a frame's device work has started to be issued (a render
 * launch, an event, a transfer: the ranks are then out of step), and (b), in a group created with
 * wcpt_group_create_rank, an error that the other processes cannot have seen -- any wcpt_group_render error while
 * presenting, a check of the root's own `dst` (alignment, a null dst with a nonzero format), a device failure in
 * wcpt_group_create_screen / wcpt_group_set_output -- since the other processes still post their part of the next
 * exchange. The group then aborts its communicators and every later call but wcpt_group_destroy returns
 * WCPT_ERROR_DEVICE_LOST; the other processes' exchange does not complete, and their wcpt_group_sync returns
 * WCPT_ERROR_DEVICE_LOST at its timeout (or earlier, on the transport's asynchronous error). Refusals made
 * alike in every process (frame size, format, `bytes`) leave the group usable.
 * wcpt_last_error(wcpt_group_context(g, r)) or wcpt_last_error(NULL) explains an error. */
/* The row-block split itself, for a host that runs one process per device (then wcpt_set_row_range with the
 * result): rank r of n renders rows [r*height/n, (r+1)*height/n). Host-only, no device needed. */
int           wcpt_row_block(uint32_t height, uint32_t n, uint32_t rank, uint32_t* y0, uint32_t* rows);
/* The interleaved split (wcpt_set_row_stripes with period = n * stripe): rank r of n takes the stripes r, r + n,
 * r + 2n, ... of `stripe` rows; *y_first = r * stripe, *rows = the rows it holds (0 when the frame has fewer than r + 1
 * stripes). stripe == 0 is wcpt_row_block. Host-only. Added under ABI 4. */
int           wcpt_row_stripes(uint32_t height, uint32_t n, uint32_t rank, uint32_t stripe, uint32_t* y_first,
                               uint32_t* rows);
typedef struct wcpt_group wcpt_group;
#define WCPT_GROUP_TRANSPORT_RCCL 0
#define WCPT_GROUP_TRANSPORT_COPY 1
/* One process (wcpt_group_create_ex): every sender's render writes its row block straight into the root's frame over
 * xGMI (peer access, enabled at creation; refused when a sender's device cannot access the root's), so presenting a
 * frame costs no transfer, event or copy: the host issues one launch per rank. A device may be listed more than once. */
#define WCPT_GROUP_TRANSPORT_DIRECT 2
#define WCPT_GROUP_UNIQUE_ID_BYTES 128   /* == sizeof(ncclUniqueId) (rccl.h NCCL_UNIQUE_ID_BYTES) */
#define WCPT_GROUP_OPTION_OVERLAP 1
/* How a one-process group issues a frame to its devices. 1: the caller's thread issues the first local rank's share
 * (validation, render launch, events, transfer) while a host thread per other local rank issues that rank's share at the
 * same time, and wcpt_group_render returns once every share is enqueued (the API stays single-threaded for the caller;
 * threads spin ~0.2 ms between frames, then sleep). 0 (default): the caller's thread issues every rank's share in turn.
 * -1: 1 when the group's ranks span more than one device and the transport is COPY or DIRECT, else 0 (an RCCL group
 * issues all its sends and receives inside one ncclGroupStart/End from one thread unless 1 is set). Same device work
 * either way. Off by default because the threaded issue has only run with every rank on one device. Host issue per
 * frame at 8 ranks (measured on one device): COPY 95-137 us in one thread, 28-40 us with threads; DIRECT
 * 27.5 us in one thread, 13.5 us with threads. */
#define WCPT_GROUP_OPTION_THREADS 2
/* Bound on one wcpt_group_sync (and on the drain in wcpt_group_destroy), in milliseconds; 0 = wait forever; default
 * 60000 in a group of several ranks (none in a group of one). The sync polls each local rank's render and
 * communication streams (hipStreamQuery) and the communicator's asynchronous error (ncclCommGetAsyncError) instead of
 * blocking: when a peer has failed or did not post its part of a frame's exchange, the transfers never complete, so on
 * an asynchronous error or at the deadline the group aborts its communicators (ncclCommAbort), lets the aborted work
 * drain, and returns WCPT_ERROR_DEVICE_LOST (the group is then broken: every later call but wcpt_group_destroy returns
 * WCPT_ERROR_DEVICE_LOST). Pick it above the longest run of frames the host queues between two syncs. Option 3 was
 * added under ABI 4. */
#define WCPT_GROUP_OPTION_TIMEOUT_MS 3
/* Rows per interleaved stripe of the group's split: 0 (default) = contiguous row blocks (wcpt_row_block); a power of
 * two = rank r renders the stripes r, r + n, r + 2n, ... of that many rows (wcpt_row_stripes), so every rank gets rows
 * from the whole frame and a scene whose cost sits in one region no longer loads one rank. Multiples of 8 keep the
 * kernels' 8x8 tiles inside a stripe. The presented frame is the same bits either way: the root renders its stripes
 * straight into their rows of the output, RCCL blocks arrive in a root-side staging buffer and are copied to their rows
 * on the root's communication stream (hipMemcpy2DAsync), COPY senders copy their stripes to their rows, and DIRECT
 * senders write their rows themselves. Every process sets the same value; takes effect at once (the screen is laid
 * out again and accumulation restarts). Added under ABI 4. */
#define WCPT_GROUP_OPTION_ROW_STRIPE 4
typedef struct wcpt_group_info {
    int32_t nranks;            /* ranks of the group; RCCL: ncclCommCount of this process's first communicator */
    int32_t local_ranks;       /* ranks driven by this process */
    int32_t first_local_rank;
    int32_t root;
    int32_t transport;         /* WCPT_GROUP_TRANSPORT_* */
    int32_t overlap;           /* WCPT_GROUP_OPTION_OVERLAP */
    int32_t distinct_devices;  /* distinct devices among this process's ranks */
    int32_t broken;            /* 1 after a transport failure aborted the communicators */
    uint64_t frames;           /* frames rendered (and, with an output set, gathered) */
    int32_t issue_threads;     /* host threads issuing frames beside the caller's (WCPT_GROUP_OPTION_THREADS) */
    int32_t _pad;
} wcpt_group_info;
int           wcpt_group_create(const int* devices, int n, int root, wcpt_group** out);
int           wcpt_group_create_ex(const int* devices, int n, int root, int transport, wcpt_group** out);
int           wcpt_group_unique_id(uint8_t* id /* WCPT_GROUP_UNIQUE_ID_BYTES */);
int           wcpt_group_create_rank(int device, int nranks, int rank, int root, const uint8_t* id, wcpt_group** out);
int           wcpt_group_destroy(wcpt_group* g);
wcpt_context* wcpt_group_context(wcpt_group* g, int rank);
int           wcpt_group_set_option(wcpt_group* g, int option, int value);
int           wcpt_group_info_get(wcpt_group* g, wcpt_group_info* out);
int           wcpt_group_create_screen(wcpt_group* g, uint32_t width, uint32_t height);
int           wcpt_group_set_output(wcpt_group* g, int format, uint64_t dst, uint64_t bytes);
int           wcpt_group_render(wcpt_group* g, const wcpt_scene_data* scene, const uint64_t* materials,
                                const uint64_t* spheres, const uint64_t* draw_commands);
int           wcpt_group_sync(wcpt_group* g);

/* HIP runtime version the library runs on (hipRuntimeGetVersion), e.g. 70226090 for ROCm 7.2. */
int      wcpt_runtime_version(int* version);

/* ---- kernel timing (HIP events on the context's stream) -------------------------------------------- */
int      wcpt_profile_begin(wcpt_context* ctx);
int      wcpt_profile_end(wcpt_context* ctx, double* kernel_ms_total, uint32_t* launches);

/* ---- host utilities (no GPU needed) ----------------------------------------------------------------- */
/* OBJ text -> unique (v,vt,vn) vertices + fan-triangulated indices (ModelLoader.jai:60-141). */
int      wcpt_obj_parse(const char* text, uint64_t length, wcpt_mesh* out);
int      wcpt_obj_load(const char* path, wcpt_mesh* out);
void     wcpt_mesh_free(wcpt_mesh* mesh);
/* Midpoint BVH (PathTracingRenderer.jai:147-217). Permutes `indices` in place. `nodes` must hold
 * max_nodes entries; 2*index_count/3 is always enough. */
int      wcpt_bvh_build(const float* positions, uint32_t vertex_count, uint32_t* indices,
                        uint32_t index_count, wcpt_node* nodes, uint32_t max_nodes, uint32_t* nodes_used);
/* Optional binned-SAH builder: same node format and conventions, a different tree (far
 * fewer nodes visited on large meshes). Images equal the midpoint tree's except where two triangles hit at exactly
 * the same t. Permutes `indices` into leaf order; 2*index_count/3 nodes always suffice. */
int      wcpt_bvh_build_sah(const float* positions, uint32_t vertex_count, uint32_t* indices,
                            uint32_t index_count, wcpt_node* nodes, uint32_t max_nodes, uint32_t* nodes_used);
/* Camera Update (PathTracingRenderer.jai:22-36): yaw/pitch/fov/position -> matrices. */
int      wcpt_camera_update(wcpt_camera* cam, float aspect_ratio);
/* Scene generators: "default" (reference Init scene, PathTracingRenderer.jai:322-339, without a mesh),
 * "cornell" (Cornell-class box), "atrium" (deterministic Sponza-scale procedural OBJ, ~260k tris). */
int      wcpt_scene_generate(const char* name, uint32_t seed, wcpt_scene* out);
void     wcpt_scene_free(wcpt_scene* scene);
/* Scene as OBJ text (so the atrium goes through the same loader path as ModelLoader.jai). The returned
 * string is owned by the library: release with wcpt_string_free. */
int      wcpt_mesh_to_obj(const wcpt_mesh* mesh, char** out_text, uint64_t* out_length);
void     wcpt_string_free(char* text);

/* ---- self-test entry points (used by the parity tests; GPU) ---------------------------------------- */
/* Evaluates device functions on n inputs: fn 0 = pcg_hash, 1 = rand stream (4 per input),
 * 2 = log, 3 = cos, 4 = exp, 5 = sqrt (the kernels' sqrt_exact), 6 = divide(in, in2), 7 = RandomDirection (3 per input),
 * 8 = exhaustive check of the fast reciprocal (out[i] = mismatches vs IEEE 1/x over the bit patterns
 * (in[i] << 16) | k, k < 2^16), 9 = the reciprocal used by the kernels, 10/11 = as 8 over every normal /
 * every input, 12 = as 8 for the kernels' reciprocals (rcp_exact, and its packed pair form on (x, ~x)),
 * 13 = how many inputs of the block fail the fast result's class check (take the general division),
 * 14 = the two triangle acceptance forms on (u, v) = (in, in2) with t = 1 (bit 0 compares, bit 1 minimum3),
 * 15 = as 8 for the kernels' square root (sqrt_exact) against the correctly rounded sqrtf,
 * 16 = the kernels' GLSL vector / scalar on one component: in * RN(1 / in2), 17 = as 8 for the integer form of the
 * triangle take (0 < t < rec.t as bits(t) - 1 < bits(rec.t) - 1) with rec.t = in2[i]. Host arrays of 32-bit words. */
int      wcpt_selftest_device(wcpt_context* ctx, int fn, const uint32_t* in, const uint32_t* in2,
                              uint32_t* out, uint32_t n);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* WCPT_H */
