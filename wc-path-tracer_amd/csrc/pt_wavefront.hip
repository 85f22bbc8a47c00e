/*
 * pt_wavefront.hip — wavefront variant of the path tracer (BASELINE.json config 5).
 *
 * The megakernel (pt_kernels.hip) runs one pixel per lane from ray generation to accumulation. On an
 * incoherent scene (the 262k-triangle atrium) its lanes mostly idle: per-ray traversal work is heavy-tailed,
 * and a wave runs as long as its longest ray (measured SIMD efficiency 16% on interior-node steps and 5% on
 * triangle steps, tools/diag.py). Here the same per-path operations are split into three kernels over a
 * queue of live paths:
 *
 *   wf_init   ray generation (pathTracer.comp:290-306): path state + primary ray, enqueue every pixel
 *   wf_trace  Intersect (:135-211) for every queued ray: persistent waves, a lane that finishes its ray
 *             takes the next one at once (dynamic fetch; one atomicAdd per 64 rays per wave), and a
 *             single-step traversal loop (one interior node OR one triangle per lane per iteration), so a
 *             lane in a 48-triangle leaf no longer stalls the other 63
 *   wf_shade  shading (:248-280) + sample loop (:309-312) + accumulation (:314-323); continuing paths are
 *             appended to the next queue (one atomicAdd per 256-thread block per round)
 *
 * The host runs trace+shade samples*(maxBounceCount+1) times (each iteration advances every live path by
 * exactly one segment). Each path executes exactly the megakernel's operation sequence (same traversal
 * order, same RNG stream), so the image is bit-identical; only the order in which paths are processed
 * changes. Path state lives in HBM as structure-of-arrays float4s (112 B/path + 4 B sphere-loop winner).
 *
 * Everything of Intersect that does not depend on the BVH runs where every lane is busy: the sphere loop
 * (:136-149) and 1/direction run in the kernel that creates the ray (wf_init / wf_shade) and travel with it
 * in `pre`; the winner's normal, facing and material (:145, :173, :204-208) are rebuilt in wf_shade from the
 * (t, primitive) record the trace kernel leaves. The divergent trace loop keeps only the BVH walk.
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "pt_device.h"
#include "pt_kernels.h"

namespace wcpt {
namespace dev {

/* Queue entries a wave claims per atomicAdd. */
#ifndef WCPT_TRACE_CHUNK
#define WCPT_TRACE_CHUNK 64
#endif
constexpr uint32_t kTraceChunk = WCPT_TRACE_CHUNK;
constexpr int kShadeBlock = 256;


__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ unsigned long long lanemask_lt() { return (1ull << lane_id()) - 1ull; }

/* The Intersect prologue of a new segment (:136-149, the sphere loop), run where the ray is created with every
 * lane busy; its result travels with the ray in `pre`. Counts the segment (one Intersect call per queued ray). */
template <bool COUNT>
__device__ __forceinline__ void segment_prologue(const Ray& r, const wcpt_scene_data& sd,
                                                 const wcpt_sphere* __restrict__ spheres, float& rt, uint32_t& prim,
                                                 Counters& cnt)
{
    rt = kInfinity;
    prim = kNoPrim;
    sphere_loop(r, sd.sphereCount, spheres, rt, prim);
    if (COUNT) {
        cnt.segments++;
        cnt.sphere_tests += sd.sphereCount;
    }
}

/* Write one queued path at `slot` of a slot-indexed state set. */
__device__ __forceinline__ void write_path(const PathSoA& o, uint32_t slot, const Ray& r, uint32_t bounce,
                                           uint32_t sample, float rt, uint32_t prim, f3 light, uint32_t seed, f3 trans,
                                           uint32_t pix)
{
    o.ray0[slot] = make_float4(r.origin.x, r.origin.y, r.origin.z, r.direction.x);
    o.ray1[slot] = make_float4(r.direction.y, r.direction.z, __uint_as_float(bounce), __uint_as_float(sample));
    o.pre[slot] = make_float4(r.invDirection.x, r.invDirection.y, r.invDirection.z, rt);
    o.light[slot] = make_float4(light.x, light.y, light.z, __uint_as_float(seed));
    o.trans[slot] = make_float4(trans.x, trans.y, trans.z, 0.0f);
    o.pre_prim[slot] = prim;
    o.pix[slot] = pix;
}

/* Block-aggregated append of `pred` lanes to a queue: one atomicAdd per block. All threads of the block must
 * call it (it contains __syncthreads). Returns the slot for predicated lanes. */
__device__ __forceinline__ uint32_t block_append(uint32_t* counter, bool pred, uint32_t* s_wave, uint32_t* s_base)
{
    const uint32_t wave = threadIdx.x >> 6;
    const unsigned long long m = __ballot(pred);
    if (lane_id() == 0) s_wave[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t total = 0;
        for (uint32_t w = 0; w < blockDim.x / 64u; w++) {
            const uint32_t c = s_wave[w];
            s_wave[w] = total;
            total += c;
        }
        *s_base = total ? atomicAdd(counter, total) : 0u;
    }
    __syncthreads();
    const uint32_t slot = *s_base + s_wave[wave] + (uint32_t)__popcll(m & lanemask_lt());
    __syncthreads();
    return slot;
}

#ifndef WCPT_WF_PUSH_CULL
#define WCPT_WF_PUSH_CULL 1
#endif
#ifndef WCPT_WF_ANYHIT_LAST
#define WCPT_WF_ANYHIT_LAST 1
#endif
#ifndef WCPT_WF_TAIL_WINDOW
#define WCPT_WF_TAIL_WINDOW 16 /* rays per wave of the grid: claims for idle lanes only in the queue's last window */
#endif
#ifndef WCPT_WF_POP_ONCE
#define WCPT_WF_POP_ONCE 1
#endif
#ifndef WCPT_WF_PRIMARY_REUSE
#define WCPT_WF_PRIMARY_REUSE 1 /* samples 1.. shade their primary segment from sample 0's record */
#endif
#ifndef WCPT_WF_SMALL_LEAVES
#define WCPT_WF_SMALL_LEAVES 1 /* the fast layout also requires kTriFlagSmallLeaves: packed stack entries need no fetch case */
#endif
#ifndef WCPT_WF_LEAF_RECORDS
#define WCPT_WF_LEAF_RECORDS 1 /* the fast layout also requires kTriFlagLeafRecords: leaf steps need no index path */
#endif
/* Path-persistent trace (PERSIST instances, launch_wavefront): one launch runs every segment of its paths. A lane whose
 * ray is done shades it in place (resolve_hit, path_shade, the next segment's sphere loop, or the pixel's store) and
 * goes on with the path's next segment, so no path waits for the slowest ray of its bounce; the wave shades once
 * `refill` of its lanes wait, or when none is tracing. Used where a pipeline's queue is short (row blocks), for one
 * sample per pixel. */
#ifndef WCPT_WF_CTR_PARITY
#define WCPT_WF_CTR_PARITY 1
#endif
#ifndef WCPT_WF_PERSIST_WAVES
#define WCPT_WF_PERSIST_WAVES 4
#endif
#ifndef WCPT_WF_PERSIST_GEO
#define WCPT_WF_PERSIST_GEO 3 /* the persistent trace's fetch rounds: 3 one per iteration, 2 two */
#endif
#ifndef WCPT_WF_GEO2_WAVES
#define WCPT_WF_GEO2_WAVES 8 /* occupancy floor of the fast-layout trace (waves per SIMD) */
#endif

/* ---- ray generation ------------------------------------------------------------------------------- */
template <bool COUNT>
__global__ __launch_bounds__(kShadeBlock) void wf_init(const wcpt_scene_data sd, const wcpt_sphere* __restrict__ spheres,
                                                       WfBuffers b, float4* __restrict__ image,
                                                       uint32_t W, uint32_t H, const RowMap rm, uint32_t rows,
                                                       uint32_t tilesX, uint32_t total, uint32_t pipe, uint32_t npipes,
                                                       unsigned long long* __restrict__ counters,
                                                       uint32_t* __restrict__ zero_next)
{
    /* the queue counters of the pipeline's next frame (the other counter set, unused by this frame): zeroed here, so a
     * frame needs no memset launch of its own (WCPT_WF_CTR_PARITY) */
    if (zero_next && blockIdx.x == 0 && threadIdx.x < 4u) zero_next[threadIdx.x] = 0u;
    __shared__ uint32_t s_wave[kShadeBlock / 64], s_base;
    Counters cnt = {};
    for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += gridDim.x * blockDim.x) {
        const uint32_t w = base + threadIdx.x;
        bool live = false;
        uint32_t p = 0, seed = 0, prim = kNoPrim;
        float rt = kInfinity;
        Ray ray;
        if (w < total) {
            const uint32_t t = (w >> 6) * npipes + pipe, q = w & 63u; /* 8x8 tiles (this pipeline's): coherent initial queue */
            const uint32_t lx = (t % tilesX) * 8u + (q & 7u);
            const uint32_t ly = (t / tilesX) * 8u + (q >> 3);
            if (lx < W && ly < rows) {
                p = ly * W + lx;
                const uint32_t y = frame_row(rm, ly); /* row block or interleaved stripes (row_map.h) */
                seed = pcg_hash(lx + y * W + sd.renderedFramesCount * 719393u); /* :304-305 */
                b.result[p] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (sd.samples > 0) {
                    PathState ps;
                    path_begin(ps, mk3(sd.position[0], sd.position[1], sd.position[2]),
                               primary_direction(sd, lx, y, W, H));
                    ray = ps.ray;
                    segment_prologue<COUNT>(ray, sd, spheres, rt, prim, cnt);
                    live = true;
                } else { /* samples == 0: result / 0 = NaN (:312), stored as the reference would */
                    const f3 r = mk3(0.0f, 0.0f, 0.0f) / (float)sd.samples;
                    if (!COUNT) store_pixel(image, b.wire, b.wire_ch, b.wire_rows, W, lx, ly, r);
                    if (COUNT) cnt.pixels++;
                }
            }
        }
        const uint32_t slot = block_append(b.count_in, live, s_wave, &s_base);
        if (live)
            write_path(b.in, slot, ray, 0u, 0u, rt, prim, mk3(0.0f, 0.0f, 0.0f), seed, mk3(1.0f, 1.0f, 1.0f), p);
    }
    flush_counters<COUNT>(cnt, counters);
}

/* ---- trace ------------------------------------------------------------------------------------------ */
/* Register budget: the trace loop carries only the ray (9), the closest hit as (t, primitive id) (2-3), a
 * 3-word node cursor and the stack pointer; the normal and material of the winning primitive are rebuilt
 * once per ray in the epilogue with the reference's expressions (:145, :173), which gives bit-identical
 * values. With the 10-entry LDS stack (5 KiB/wave) and __launch_bounds__(64, 8) the kernel runs 8 waves per
 * SIMD (32 per CU) to keep more dependent node fetches in flight. */
/* LDS per wave: the traversal stack, n entries per lane, 8 B each, lane-interleaved. n = 10 -> 5 KiB/wave,
 * 8 waves/SIMD; 16 -> 5 waves; 24 -> 3 waves. Deeper entries spill to scratch (measured on c3: 10 and 16
 * entries run within 1%, 24 is 13% slower -- the traversal is bound by node-fetch latency, not the spill). */
constexpr int wf_lds_per_wave(int n) { return n * 512; }
constexpr int wf_waves_per_simd(int n) { return (163840 / wf_lds_per_wave(n)) / 4 < 8 ? (163840 / wf_lds_per_wave(n)) / 4 : 8; }
enum : uint32_t { kModeInterior = 0, kModeLeaf = 1, kModePop = 2, kModeDone = 3, kModeShade = 4, kModeIdle = 5,
                  kModeIdlePend = 6 };
/* Deferred hit stores: a lane whose ray is done keeps its (t, primitive) record in registers (kModeIdlePend, an idle
 * lane) and the wave writes the records when it next refills, or at its exit. On gfx9 a store counts in vmcnt, and the
 * loop's in-order vmcnt waits (the pop's, the node fetch's) would otherwise wait for it on the next iteration.
 * Measured with the in-branch spill wait (pt_device.h WCPT_STACK_SPILL_WAIT), 2 alternating rounds
 * (profiles/r05_store_wait_ab.log): c3 4.708-4.714 against 4.848-4.856 ms (-2.9 %), c4 199.5 against 205.3 ms
 * (-2.8 %); alone c3 -2.0 %, c4 -2.7 %. */
#ifndef WCPT_WF_DEFER_HIT
#define WCPT_WF_DEFER_HIT 1
#endif

#ifndef WCPT_WF_TRACE_SHARE
#define WCPT_WF_TRACE_SHARE 1
#endif
#ifndef WCPT_WF_REC_OFF24
#define WCPT_WF_REC_OFF24 1
#endif
#ifndef WCPT_WF_PAIR_RSRC
#define WCPT_WF_PAIR_RSRC 1
#endif
#ifndef WCPT_WF_GEO_FAST
#define WCPT_WF_GEO_FAST 1
#endif
struct Geom {
    gtri_ptr tris;
    uint32_t ntri;
    uint32_t lim3; /* 3 * ntri (kTriFlagIndex24 draws) */
    bool packed;   /* stack entries carry (left, count): kTriFlagPackedRefs */
    bool idx24;    /* index positions < 2^24: kTriFlagIndex24 */
    gnode_ptr bvh;
    gu32_ptr indices;
    gf32_ptr vertices;
    uint32_t nodes;                /* BVH node count when the BVH is a known context buffer of < 2^24 nodes, else 0 */
    __amdgpu_buffer_rsrc_t rsrc;   /* buffer resource over those nodes (load_pair_rsrc) */
    __amdgpu_buffer_rsrc_t trsrc;  /* buffer resource over the ntri single records (load_tri_rsrc; kTriFlagIndex24 draws) */
};

__device__ __forceinline__ Geom load_geom(const wcpt_draw_command* __restrict__ draws,
                                          const uint64_t* __restrict__ tri_records, uint32_t d)
{
    Geom g;
    g.tris = (gtri_ptr)(uintptr_t)tri_records[kTriTableWords * d];      /* single records */
    g.ntri = (uint32_t)tri_records[kTriTableWords * d + 2u];
    g.packed = (tri_records[kTriTableWords * d + 3u] & kTriFlagPackedRefs) != 0u;
    g.idx24 = WCPT_WF_REC_OFF24 && (tri_records[kTriTableWords * d + 3u] & kTriFlagIndex24) != 0u;
    g.lim3 = 3u * g.ntri;
    g.bvh = as_nodes(draws[d].bvhBuffer);
    g.indices = as_u32(draws[d].indexBuffer);
    g.vertices = as_f32(draws[d].vertexBuffer);
    g.nodes = g.packed ? (uint32_t)(tri_records[kTriTableWords * d + 2u] >> 32) : 0u;
    g.rsrc = node_rsrc(g.bvh, g.nodes);
    g.trsrc = tri_rsrc(g.tris, g.idx24 ? g.ntri : 0u);
    return g;
}

/* DIAG builds only: per-wave cycle timers (s_memtime) of the trace loop's phases, summed over waves into
 * b.diag[0..4] = {fetch+loop, leaf, interior, pop, epilogue}, [5] = waves, [6] = loop iterations, [7] = the waves'
 * time after they found the queue empty (the launch's tail). The stamps
 * add their own cost; read the shares, not the totals (cdna_hip_programming.md §7, In-kernel stamps). */
constexpr int kDiagTimers = 8;
template <bool DIAG>
__device__ __forceinline__ void diag_mark(uint64_t* tim, uint64_t& tprev, int k)
{
    if (!DIAG) return;
    const uint64_t t = __builtin_amdgcn_s_memtime();
    tim[k] += t - tprev;
    tprev = t;
    if (k == 0) tim[6] += 1;
}

/* Node cursor: interior -> (a = left child index); leaf -> (a = current index position, b = end position,
 * r = byte offset of the current triangle's single record or kNoRecord; draws without kTriFlagIndex24 only). */
__device__ __forceinline__ void cursor_from(uint32_t left, uint32_t count, const Geom& g, uint32_t& a, uint32_t& b,
                                            uint32_t& r, uint32_t& mode)
{
    a = left;
    b = left + count;
    /* 24-bit draws find each triangle's record in the leaf step (tri_record_off24) */
    r = g.idx24 ? 0u : leaf_record_off(left, count, g.ntri);
    mode = count > 0 ? kModeLeaf : kModeInterior;
}

/* GEO: 0 any draws; 1 one draw command (the reference's case, kernel-uniform geometry in scalar registers); 2 one draw
 * whose table flags allow packed stack refs, 24-bit record offsets and buffer-resource node loads (the host checks
 * them), so the loop carries no branches for the other layouts; 3 the same with one fetch round per iteration
 * (wf_fetch_once). */
template <bool COUNT, bool DIAG, int GEO, int LDSN, bool PERSIST = false>
__global__ __launch_bounds__(64, PERSIST ? WCPT_WF_PERSIST_WAVES : (GEO >= 2 ? WCPT_WF_GEO2_WAVES : wf_waves_per_simd(LDSN)))
void wf_trace(const wcpt_scene_data sd, const wcpt_draw_command* __restrict__ draws,
              const uint64_t* __restrict__ tri_records, WfBuffers b, uint32_t* __restrict__ status,
              unsigned long long* __restrict__ counters, uint32_t refill, const wcpt_material* __restrict__ mats,
              const wcpt_sphere* __restrict__ spheres, float4* __restrict__ image, uint32_t W, uint32_t H)
{
    __shared__ uint64_t s_stack[LDSN * 64];
    if (blockIdx.x == 0 && threadIdx.x == 0) *b.count_out = 0; /* shade appends to it after this kernel */
    const uint32_t n = *b.count_in;
    const uint32_t lane = lane_id();
    uint64_t spill[kStackDepth - LDSN];
    LdsStack<LDSN, kStackDepth - LDSN> stk;
    stk.base = (lds_u64_ptr)(s_stack + lane);
    stk.spill = (priv_u64_ptr)spill;
    stk.sp = 0;
    Counters cnt = {};
    bool overflow = false;
    Geom g0 = {}, gl = g0;
    constexpr bool SINGLE = GEO >= 1;
    if (SINGLE) g0 = load_geom(draws, tri_records, 0); /* kernel-uniform: scalar registers */
    if (GEO >= 2) {
        g0.packed = true;
        g0.idx24 = true;
    }

    /* a lane without a ray is in kModeIdle (no separate `has` flag: its lane mask had to be carried through every
     * divergent block of the loop) */
    bool drained = false, tail_claims = false;
    /* this wave's claimed queue range [lo, hi) (wave-uniform). The first chunk is static (chunk blockIdx.x), so a
     * launch with fewer rays than resident waves costs no atomics for the waves without work: same-address
     * device-scope atomics serialise, and one per wave of the persistent grid cost ~0.28 ms per launch. Later
     * chunks come from the global head, which counts past the grid's static chunks. */
    const uint32_t static_end = gridDim.x * kTraceChunk;
    uint32_t lo = blockIdx.x * kTraceChunk, hi = min(lo + kTraceChunk, n);
    if (lo >= n) {
        lo = hi = 0;
        drained = true;
    }
    uint32_t p = 0, d = 0, prim = kNoPrim, primDraw = 0;
    uint32_t ca = 0, cb = 0, cr = 0, mode = kModeIdle;
    float rt = kInfinity;
    bool any = false; /* this ray is the last segment of its pixel's last sample (render build only) */
    RefStack rf;      /* the reference's stack index (counting builds, pt_device.h RefStack) */
    Ray ray;
    uint64_t tim[kDiagTimers] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tprev = DIAG ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t t_drain = 0; /* DIAG: when this wave found the queue empty (its tail starts) */

    /* Start draw command d, or the next one whose root survives the cull (:152-162); kModeDone past the last. */
    const uint32_t ndraw = SINGLE ? 1u : sd.drawCommandCount; /* SINGLE: the host launched it for one draw */
    auto start_draw = [&]() {
        for (; d < ndraw; d++) {
            if (!SINGLE) gl = load_geom(draws, tri_records, d);
            const Geom& g = SINGLE ? g0 : gl;
            if (COUNT) { cnt.draw_fetches++; cnt.node_pops++; }
            ref_root<COUNT>(rf, cnt);
            const NodeV root = load_node(g.bvh, 0);
            float c0, c1;
            node_box(ray, root, c0, c1);
            if (c0 > c1 || c1 < 0.0f || c0 > rt) continue;
            cursor_from(root.b.z, root.b.w, g, ca, cb, cr, mode);
            stk.reset();
            return;
        }
        mode = kModeDone;
    };

    for (;;) {
        /* dynamic fetch: idle lanes take the next queued rays, once at least `refill` lanes are idle (or none
         * has work left) */
        unsigned long long need = __ballot(mode >= kModeIdle);
        /* refill <= 64 (wcpt_set_option), so "every lane idle" is included in popcount >= refill; all 64 lanes stay in
         * the loop until the wave leaves it */
        if (!drained && (uint32_t)__popcll(need) >= refill) {
            if (WCPT_WF_DEFER_HIT && mode == kModeIdlePend) {
                b.hit[p] = make_float4(rt, __uint_as_float(prim), __uint_as_float(primDraw), 0.0f);
                mode = kModeIdle;
            }
            while (need) {
                if (lo == hi) {
                    uint32_t base = 0;
                    if (static_end >= n) { /* every chunk was static */
                        drained = true;
                        break;
                    }
                    /* near the end of the queue a wave claims only as many rays as it has idle lanes: a full chunk
                     * there is a reserve that one wave works through alone while the others have drained */
                    const uint32_t csz = tail_claims ? (uint32_t)__popcll(need) : kTraceChunk;
                    if (lane == 0) base = static_end + atomicAdd(b.head, csz);
                    base = __builtin_amdgcn_readfirstlane(base); /* wave-uniform: keeps lo/hi in SGPRs */
                    if (base >= n) {
                        drained = true;
                        break;
                    }
                    lo = base;
                    hi = min(base + csz, n);
                    tail_claims = WCPT_WF_TAIL_WINDOW > 0 && (uint64_t)hi + (uint64_t)gridDim.x * WCPT_WF_TAIL_WINDOW >= n;
                }
                const uint32_t avail = hi - lo;
                const uint32_t rank = (uint32_t)__popcll(need & lanemask_lt());
                const bool take = ((need >> lane) & 1ull) && rank < avail;
                if (take) {
                    p = b.order ? b.order[lo + rank] : lo + rank;   /* input slot: consecutive lanes, consecutive slots */
                    const float4 r0 = b.in.ray0[p];
#if WCPT_WF_ANYHIT_LAST
                    const float4 r1 = b.in.ray1[p];
                    /* path_shade's last-segment shortcut keeps only the material of this segment's hit, and every
                     * triangle carries material 0 (:175): whether some triangle is accepted below the sphere loop's
                     * rec.t is all that is read. Up to the first acceptance the traversal is the reference's, so the
                     * ray finishes there; its lane takes the next queued ray. */
                    any = !COUNT && WCPT_LAST_SEGMENT_SHORTCUT && __float_as_uint(r1.z) + 1u > sd.maxBounceCount &&
                          __float_as_uint(r1.w) + 1u == sd.samples;
#else
                    const float2 r1 = reinterpret_cast<const float2*>(b.in.ray1)[2u * p];
#endif
                    const float4 pr = b.in.pre[p];
                    ray.origin = mk3(r0.x, r0.y, r0.z);
                    ray.direction = mk3(r0.w, r1.x, r1.y);
                    ray.invDirection = mk3(pr.x, pr.y, pr.z);
                    rt = pr.w;                /* sphere loop (:136-149), run by the ray's creator */
                    prim = b.in.pre_prim[p];
                    if (COUNT) simd_step<DIAG>(cnt.wave_seg, cnt.lane_seg);
                    d = 0;
                    start_draw();
                }
                const uint32_t took = min(avail, (uint32_t)__popcll(need));
                lo += took;
                need &= ~__ballot(take);
            }
        }
        if (DIAG && drained && t_drain == 0) t_drain = __builtin_amdgcn_s_memtime();
        if (!__ballot(mode < kModeIdle)) break;
        diag_mark<DIAG>(tim, tprev, 0);
        {
            const Geom& g = SINGLE ? g0 : gl;
            /* one traversal step (:157-200) as sequential ifs in the order pop -> interior -> leaf: a lane that pops
             * an interior node fetches its children in the same iteration, and one that descends into a leaf tests
             * its first triangle in the same iteration (measured 1.4% faster than leaf -> interior -> pop). Each
             * lane still executes exactly the reference's sequence of steps. */
            if (mode == kModePop) {
#if WCPT_WF_POP_ONCE
                /* one stack entry per iteration: a culled entry (:162) leaves the lane in pop mode */
                if (stk.empty()) {
                    if (SINGLE) {
                        mode = kModeDone; /* the only draw is done */
                    } else {
                        d++;
                        start_draw();
                    }
                } else {
                    uint32_t ni;
                    float t0;
                    stk.pop(ni, t0);
                    ref_pop<COUNT>(rf);
                    if (!(t0 > rt)) {
                        const uint2 lc = (GEO >= 2 && WCPT_WF_SMALL_LEAVES) ? node_ref_lc_small(ni)
                                                                            : node_ref_lc(g.packed, g.bvh, ni);
                        cursor_from(lc.x, lc.y, g, ca, cb, cr, mode);
                    }
                }
#else
                bool found = false;
                while (!stk.empty()) {
                    uint32_t ni;
                    float t0;
                    stk.pop(ni, t0);
                    ref_pop<COUNT>(rf);
                    if (t0 > rt) continue;
                    const uint2 lc = node_ref_lc(g.packed, g.bvh, ni);
                    cursor_from(lc.x, lc.y, g, ca, cb, cr, mode);
                    found = true;
                    break;
                }
                if (!found) {
                    d++;
                    start_draw();
                }
#endif
            }
            /* the interior step on the fetched child pair (:164-200) */
            auto interior_step = [&](const NodeV& L, const NodeV& R) {
                float l0, l1, r0, r1;
                node_box(ray, L, l0, l1);
                node_box(ray, R, r0, r1);
                if (COUNT) {
                    cnt.interior_visits++;
                    cnt.node_pops += 2;
                    simd_step<DIAG>(cnt.wave_int, cnt.lane_int);
                }
                const float leftDist = (l0 > 0.0f) ? l0 : l1;
                const float rightDist = (r0 > 0.0f) ? r0 : r1;
                const bool passL = !(l0 > l1 || l1 < 0.0f);
                const bool passR = !(r0 > r1 || r1 < 0.0f);
                const bool leftFirst = leftDist < rightDist;
                const bool passNear = leftFirst ? passL : passR;
                const bool passFar = leftFirst ? passR : passL;
                /* A far child whose entry distance already exceeds rec.t would be culled at its pop (:162): rec.t
                 * only shrinks, so the render build does not push it (the counting build keeps the reference's
                 * pushes and pops). */
                const float farT0 = leftFirst ? r0 : l0;
                if (passFar && (COUNT || !WCPT_WF_PUSH_CULL || !(farT0 > rt))) {
                    const NodeV& F = leftFirst ? R : L;
                    const uint32_t fref = (GEO >= 2 && WCPT_WF_SMALL_LEAVES) ? node_ref_small(F.b.z, F.b.w)
                                                                            : node_ref(g.packed, leftFirst ? ca + 1 : ca, F.b.z, F.b.w);
                    if (!stk.push(fref, farT0))
                        overflow = true;
                }
                ref_interior<COUNT>(rf, passFar, cnt); /* the counting build pushes every passing far child */
                if (passNear && !((leftFirst ? l0 : r0) > rt)) {
                    const uint32_t nl = leftFirst ? L.b.z : R.b.z, nc = leftFirst ? L.b.w : R.b.w;
                    cursor_from(nl, nc, g, ca, cb, cr, mode);
                } else {
                    mode = kModePop;
                }
            };
            /* one triangle of the leaf (:174-190) */
            auto leaf_step = [&](const TriE& tr) {
                const float tt = rayTriangleE(ray, tr.a, tr.e1, tr.e2);
                if (COUNT) {
                    cnt.triangle_tests++;
                    simd_step<DIAG>(cnt.wave_tri, cnt.lane_tri);
                }
                const bool acc = tt != -1.0f && tt < rt;
                if (acc) {
                    rt = tt;
                    prim = ca;
                    primDraw = d;
                }
                ca += 3;
                if (!g.idx24) cr += (cr != kNoRecord) ? 48u : 0u;
                if (ca >= cb) mode = kModePop;
                if (acc && any) mode = kModeDone; /* any-hit segment: its answer is fixed */
            };
            auto index_tri = [&]() {
                return tri_from_indices(g.indices, g.vertices, ca, draw_vertex_count(tri_records, SINGLE ? 0u : d));
            };
            diag_mark<DIAG>(tim, tprev, 3); /* pop */
            if (GEO == 3 && WCPT_WF_PAIR_RSRC && WCPT_WF_LEAF_RECORDS) {
                /* one fetch round per iteration (GEO 3, wf_fetch_once): the child pair of an interior lane and the
                 * triangle of a leaf lane are both issued before either is waited for; a lane that descends into a leaf
                 * tests it next iteration */
                const bool fi = mode == kModeInterior, fl = mode == kModeLeaf;
                NodeV L, R;
                TriE tr;
                if (fi) load_pair_rsrc(g.rsrc, ca, L, R);
                if (fl) tr = load_tri_rsrc(g.trsrc, ca * 16u);
                if (fi) interior_step(L, R);
                diag_mark<DIAG>(tim, tprev, 2);
                if (fl) leaf_step(tr);
                diag_mark<DIAG>(tim, tprev, 1);
            } else {
            if (mode == kModeInterior) {
                NodeV L, R;
                if (WCPT_WF_PAIR_RSRC && (GEO >= 2 || g.nodes)) {
                    load_pair_rsrc(g.rsrc, ca, L, R);
                } else {
                    L = load_node(g.bvh, ca);
                    R = load_node(g.bvh, ca + 1);
                }
                interior_step(L, R);
            }
            diag_mark<DIAG>(tim, tprev, 2);
            if (mode == kModeLeaf) {
                /* one triangle per step, from the single records (pair records measured slower here: most
                 * atrium leaves hold 1-2 triangles, and the wider record costs fetch bytes and VGPRs) */
                if (GEO >= 2 && WCPT_WF_LEAF_RECORDS) {
                    /* every leaf triangle has its record (kTriFlagLeafRecords); the load goes through a buffer resource
                     * bounded by the draw's records, so a BVH rewritten behind the runtime's cache (wcpt.h
                     * WCPT_OPTION_TRIANGLE_CACHE) reads zeros -- a triangle no ray accepts -- instead of past them */
                    leaf_step(load_tri_rsrc(g.trsrc, ca * 16u));
                } else {
                    const uint32_t off = g.idx24 ? tri_record_off24(ca, g.lim3) : cr;
                    leaf_step(off != kNoRecord ? load_tri_at(g.tris, off) : index_tri());
                }
            }
            diag_mark<DIAG>(tim, tprev, 1);
            }
            if (mode == kModeDone) {
                /* Intersect result; wf_shade rebuilds the winner's normal and material (:204-208) */
                if (PERSIST) {
                    mode = kModeShade;
                } else if (WCPT_WF_DEFER_HIT) {
                    mode = kModeIdlePend;
                } else {
                    b.hit[p] = make_float4(rt, __uint_as_float(prim), __uint_as_float(primDraw), 0.0f);
                    mode = kModeIdle;
                }
                ref_segment_end<COUNT>(cnt);
            }
            diag_mark<DIAG>(tim, tprev, 4);
            if (PERSIST) {
                const unsigned long long sh = __ballot(mode == kModeShade);
                if (sh && ((uint32_t)__popcll(sh) >= refill || !__ballot(mode < kModeDone)) && mode == kModeShade) {
                    /* wf_shade's per-path step (:248-280, :309-323) for this lane's path at slot p, one sample */
                    const float4 r1 = b.in.ray1[p], li = b.in.light[p], tr = b.in.trans[p];
                    const uint32_t pix = b.in.pix[p];
                    PathState ps;
                    ps.ray = ray;
                    ps.totalLight = mk3(li.x, li.y, li.z);
                    ps.transmittance = mk3(tr.x, tr.y, tr.z);
                    ps.bounce = __float_as_uint(r1.z);
                    uint32_t sample = __float_as_uint(r1.w), seed = __float_as_uint(li.w);
                    const Hit h = resolve_hit(ps.ray, rt, prim, primDraw, spheres, draws, tri_records);
                    f3 L;
                    if (!path_shade(ps, h, seed, sd, mats, L, sample + 1u == sd.samples)) {
                        float rt0 = kInfinity;
                        uint32_t prim0 = kNoPrim;
                        segment_prologue<COUNT>(ps.ray, sd, spheres, rt0, prim0, cnt);
                        b.in.ray1[p] = make_float4(ps.ray.direction.y, ps.ray.direction.z, __uint_as_float(ps.bounce),
                                                   __uint_as_float(sample));
                        b.in.light[p] = make_float4(ps.totalLight.x, ps.totalLight.y, ps.totalLight.z, __uint_as_float(seed));
                        b.in.trans[p] = make_float4(ps.transmittance.x, ps.transmittance.y, ps.transmittance.z, 0.0f);
                        ray = ps.ray;
                        rt = rt0;
                        prim = prim0;
                        /* the queue-fetch path's guard (:392): any-hit only where that build option is on, and never
                         * in a counting pass (which walks the reference's full closest-hit traversal) */
                        any = !COUNT && WCPT_WF_ANYHIT_LAST && WCPT_LAST_SEGMENT_SHORTCUT &&
                              ps.bounce + 1u > sd.maxBounceCount && sample + 1u == sd.samples;
                        d = 0;
                        start_draw();
                    } else {
                        const float4 rs = b.result[pix];
                        f3 result = mk3(rs.x, rs.y, rs.z) + L;                  /* :310 */
                        result = result / (float)sd.samples;                      /* :312 (one sample) */
                        const uint32_t lx = pix % W, ly = pix / W;
                        float4* px = image + (size_t)ly * W + lx;
                        f3 acc;
                        if (sd.renderedFramesCount == 0) {
                            acc = result;
                        } else {
                            const float4 o = *px;
                            const float weight = 1.0f / (float)(sd.renderedFramesCount + 1u);
                            const float iw = 1.0f - weight;
                            acc = mk3(o.x * iw + result.x * weight, o.y * iw + result.y * weight,
                                      o.z * iw + result.z * weight);
                        }
                        store_pixel(image, b.wire, b.wire_ch, b.wire_rows, W, lx, ly, acc); /* :323 */
                        mode = kModeIdle;
                    }
                }
            }
        }
    }
    if (WCPT_WF_DEFER_HIT && mode == kModeIdlePend)
        b.hit[p] = make_float4(rt, __uint_as_float(prim), __uint_as_float(primDraw), 0.0f);
    if (overflow) atomicOr(status, 1u);
    flush_counters<COUNT>(cnt, counters);
    if (DIAG && lane == 0) {
        tim[5] += 1; /* waves */
        if (t_drain) tim[7] += __builtin_amdgcn_s_memtime() - t_drain; /* tail: queue empty, lanes finishing */
        for (int k = 0; k < kDiagTimers; k++) atomicAdd(&b.diag[k], (unsigned long long)tim[k]);
    }
}

/* ---- shade ------------------------------------------------------------------------------------------ */
#ifndef WCPT_SHADE_PREFETCH
#define WCPT_SHADE_PREFETCH 0 /* measured +0.8 % on c3, +0.7 % on c4: off */
#endif
/* One input queue slot of wf_shade: pixel, ray, light, transmittance and the trace's Intersect record. */
struct PathIn {
    uint32_t pix;
    float4 r0, r1, li, tr, hi;
};
__device__ __forceinline__ PathIn load_path_in(const WfBuffers& b, uint32_t w, uint32_t n)
{
    PathIn q = {};
    if (w < n) {
        q.pix = b.in.pix[w];
        q.r0 = b.in.ray0[w];
        q.r1 = b.in.ray1[w];
        q.li = b.in.light[w];
        q.tr = b.in.trans[w];
        q.hi = b.hit[w];
    }
    return q;
}
template <bool COUNT>
__global__ __launch_bounds__(kShadeBlock) void wf_shade(const wcpt_scene_data sd, const wcpt_material* __restrict__ mats,
                                                        const wcpt_sphere* __restrict__ spheres,
                                                        const wcpt_draw_command* __restrict__ draws,
                                                        const uint64_t* __restrict__ tri_records, WfBuffers b,
                                                        float4* __restrict__ image, uint32_t W,
                                                        uint32_t H, const RowMap rm, unsigned long long* __restrict__ counters)
{
    __shared__ uint32_t s_wave[kShadeBlock / 64], s_base;
    if (blockIdx.x == 0 && threadIdx.x == 0) *b.head = 0; /* the trace of this iteration has finished */
    const uint32_t n = *b.count_in;
    Counters cnt = {};
    const uint32_t stride = gridDim.x * blockDim.x;
#if WCPT_SHADE_PREFETCH
    /* The path state of the thread's next queue slot is loaded before the current one is shaded: the streams (path
     * state in queue order, coalesced) have one iteration of the grid-stride loop to arrive instead of stalling its
     * start, and the dependent gathers of the current path (normal, material) overlap them. */
    PathIn nxt = load_path_in(b, blockIdx.x * blockDim.x + threadIdx.x, n);
#endif
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += stride) {
        const uint32_t w = base + threadIdx.x;
        bool cont = false;
        uint32_t p = 0, sample = 0, seed = 0, prim0 = kNoPrim;
        float rt0 = kInfinity;
        PathState ps;
#if WCPT_SHADE_PREFETCH
        const PathIn cur = nxt;
        nxt = load_path_in(b, w + stride, n);
#else
        const PathIn cur = load_path_in(b, w, n);
#endif
        if (w < n) {
            p = cur.pix;                         /* slot w of the compacted input queue */
            const float4 r0 = cur.r0, r1 = cur.r1, li = cur.li, tr = cur.tr;
            const float4 hi = cur.hi;
            ps.ray.origin = mk3(r0.x, r0.y, r0.z);
            ps.ray.direction = mk3(r0.w, r1.x, r1.y);
            ps.totalLight = mk3(li.x, li.y, li.z);
            ps.transmittance = mk3(tr.x, tr.y, tr.z);
            ps.bounce = __float_as_uint(r1.z);
            sample = __float_as_uint(r1.w);
            seed = __float_as_uint(li.w);
            /* Every sample of a pixel starts with the same primary ray (:302, :309-310), so its Intersect record is
             * the same too: sample 0's is kept by pixel and later samples shade their primary segment from it
             * without tracing it again (render build only: the COUNT build traces every segment, as the reference
             * does, for the exact counters). */
            const bool reuse = !COUNT && WCPT_WF_PRIMARY_REUSE && sd.samples > 1u;
            if (reuse && ps.bounce == 0u && sample == 0u) b.prim_hit[p] = hi;
            float4 h4 = hi;
            f3 result = mk3(0.0f, 0.0f, 0.0f);
            bool summed = false; /* result holds b.result[p] + this call's finished samples */
            for (;;) {
                const Hit h = resolve_hit(ps.ray, h4.x, __float_as_uint(h4.y), __float_as_uint(h4.z), spheres, draws,
                                          tri_records);
                if (COUNT && h.hit) cnt.hits++;
                f3 L;
                if (!path_shade(ps, h, seed, sd, mats, L, sample + 1u == sd.samples)) {
                    cont = true;
                    break;
                }
                if (!summed) {
                    const float4 rs = b.result[p];
                    result = mk3(rs.x, rs.y, rs.z);
                    summed = true;
                }
                result = result + L;                                           /* :310 */
                sample++;
                const uint32_t lx = p % W, ly = p / W;
                if (sample < sd.samples) {                                  /* next sample, same primary ray */
                    path_begin(ps, mk3(sd.position[0], sd.position[1], sd.position[2]),
                               primary_direction(sd, lx, frame_row(rm, ly), W, H));
                    if (!reuse) {
                        cont = true;
                        break;
                    }
                    h4 = b.prim_hit[p];
                    continue;
                }
                result = result / (float)sd.samples;                       /* :312 */
                if (!COUNT) {
                    float4* px = image + (size_t)ly * W + lx;
                    f3 acc;
                    if (sd.renderedFramesCount == 0) {
                        acc = result;
                    } else {
                        const float4 o = *px;
                        const float weight = 1.0f / (float)(sd.renderedFramesCount + 1u);
                        const float iw = 1.0f - weight;
                        acc = mk3(o.x * iw + result.x * weight, o.y * iw + result.y * weight,
                                  o.z * iw + result.z * weight);
                    }
                    store_pixel(image, b.wire, b.wire_ch, b.wire_rows, W, lx, ly, acc); /* :323 */
                }
                if (COUNT) cnt.pixels++;
                break;
            }
            if (cont && summed) b.result[p] = make_float4(result.x, result.y, result.z, 0.0f);
            if (cont) segment_prologue<COUNT>(ps.ray, sd, spheres, rt0, prim0, cnt);
        }
        const uint32_t slot = block_append(b.count_out, cont, s_wave, &s_base);
        if (cont)
            write_path(b.out, slot, ps.ray, ps.bounce, sample, rt0, prim0, ps.totalLight, seed, ps.transmittance, p);
    }
    flush_counters<COUNT>(cnt, counters);
}

} // namespace dev

/* ---------------------------------------------------------------------------------------------------- */
/* CU count of the current device, cached per context (WfState) so that contexts on different devices each use
 * their own. */
static hipError_t cu_count(WfState& s, int& cus)
{
    if (s.cus == 0) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&s.cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
    }
    cus = s.cus;
    return hipSuccess;
}

hipError_t wf_reserve(WfState& s, uint32_t paths)
{
    if (paths <= s.capacity) return hipSuccess;
    if (s.mem) (void)hipFree(s.mem);
    s.mem = nullptr;
    s.capacity = 0;
    const size_t P = paths;
    /* two slot-indexed state sets (5 float4 + 2 u32 arrays each), the hit records by input slot, then the counters
     * and the diagnostics block */
    const size_t bytes = P * (2 * (5 * sizeof(float4) + 2 * sizeof(uint32_t)) + sizeof(float4)) + 256;
    char* m = nullptr;
    hipError_t e = hipMalloc(&m, bytes);
    if (e != hipSuccess) return e;
    s.mem = m;
    float4* f = reinterpret_cast<float4*>(m);
    for (int k = 0; k < 2; k++) {
        PathSoA& o = s.soa[k];
        o.ray0 = f;
        o.ray1 = f + P;
        o.pre = f + 2 * P;
        o.light = f + 3 * P;
        o.trans = f + 4 * P;
        f += 5 * P;
    }
    s.hit = f;
    uint32_t* u = reinterpret_cast<uint32_t*>(f + P);
    for (int k = 0; k < 2; k++) {
        s.soa[k].pre_prim = u;
        s.soa[k].pix = u + P;
        u += 2 * P;
    }
    s.ctr = u; /* two sets of [0] count q0, [1] count q1, [2] trace head, [3] - (WCPT_WF_CTR_PARITY) */
    s.diag = reinterpret_cast<unsigned long long*>(reinterpret_cast<uintptr_t>(s.ctr + 8 + 7) & ~uintptr_t(7));
    s.parity = 0;
    s.ctr_fresh = true;
    s.capacity = paths; /* only now: every array above exists */
    return hipSuccess;
}

/* Ray-sort scratch (WCPT_OPTION_SORT_RAYS): keys, alternate keys, slot ids, sorted order, radix-sort temporary
 * storage. Allocated on the first sorted render; capacity is set only once both steps succeeded. */
hipError_t wf_reserve_sort(WfState& s, uint32_t paths)
{
    if (paths <= s.sort_capacity) return hipSuccess;
    if (s.sort_mem) (void)hipFree(s.sort_mem);
    s.sort_mem = nullptr;
    s.sort_capacity = 0;
    const size_t P = paths;
    size_t temp = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, temp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                      (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)paths, 0, 32);
    if (e != hipSuccess) return e;
    char* q = nullptr;
    e = hipMalloc(&q, 4 * P * sizeof(uint32_t) + temp + 256);
    if (e != hipSuccess) return e;
    s.sort_mem = q;
    s.sort_keys = reinterpret_cast<uint32_t*>(q);
    s.sort_keys_alt = s.sort_keys + P;
    s.sort_iota = s.sort_keys_alt + P;
    s.sort_order = s.sort_iota + P;
    s.sort_temp = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(s.sort_order + P) + 255) & ~uintptr_t(255));
    s.sort_temp_bytes = temp;
    s.sort_capacity = paths;
    return hipSuccess;
}

/* Per-pixel sample sums shared by the pipelines (each pixel belongs to one pipeline). */
static hipError_t wf_reserve_result(WfPipes& w, uint64_t pixels)
{
    if (pixels <= w.result_capacity) return hipSuccess;
    if (w.result) (void)hipFree(w.result);
    w.result = nullptr;
    w.result_capacity = 0;
    hipError_t e = hipMalloc(&w.result, 2 * pixels * sizeof(float4)); /* the sums, then the primary records */
    if (e != hipSuccess) return e;
    w.result_capacity = pixels;
    return hipSuccess;
}

void wf_release(WfState& s)
{
    if (s.mem) (void)hipFree(s.mem);
    if (s.sort_mem) (void)hipFree(s.sort_mem);
    s = WfState{};
}

void wf_release(WfPipes& w)
{
    for (int j = 0; j < kWfMaxPipes; j++) {
        wf_release(w.pipe[j]);
        if (w.aux[j]) (void)hipStreamDestroy(w.aux[j]);
        if (w.join[j]) (void)hipEventDestroy(w.join[j]);
        if (w.ready[j]) (void)hipEventDestroy(w.ready[j]);
    }
    if (w.fork) (void)hipEventDestroy(w.fork);
    if (w.result) (void)hipFree(w.result);
    w = WfPipes{};
}

/* Ray sorting between bounces: key = direction octant (3 bits) | Morton code of the origin quantised to a
 * 512^3 grid over the first draw's root box (27 bits); queue slots at or past the live count get the sentinel
 * key 0xffffffff and sort to the end. Rays that start close together and head the same way then share a
 * wave, so their node fetches hit the same cache lines (tools/gather_bench.hip: coherent gathers reach ~7x
 * the scattered visit rate). The processing order of paths never affects their results. */
__device__ __forceinline__ uint32_t spread3(uint32_t v)
{
    v &= 0x1FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

__global__ __launch_bounds__(256) void wf_sort_keys(WfBuffers b, uint32_t P, const wcpt_draw_command* __restrict__ draws,
                                                    uint32_t* __restrict__ keys, uint32_t* __restrict__ iota)
{
    const uint32_t n = *b.count_in;
    const dev::gnode_ptr root = dev::as_nodes(draws[0].bvhBuffer);
    const float lo[3] = {root->min[0], root->min[1], root->min[2]};
    const float hi[3] = {root->max[0], root->max[1], root->max[2]};
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < P; i += gridDim.x * blockDim.x) {
        uint32_t key = 0xFFFFFFFFu;
        if (i < n) {
            const float4 r0 = b.in.ray0[i], r1 = b.in.ray1[i];
            const float o[3] = {r0.x, r0.y, r0.z};
            const uint32_t oct = (r0.w < 0.0f ? 4u : 0u) | (r1.x < 0.0f ? 2u : 0u) | (r1.y < 0.0f ? 1u : 0u);
            uint32_t m = 0;
            for (int a = 0; a < 3; a++) {
                const float ext = hi[a] - lo[a];
                float f = ext > 0.0f ? (o[a] - lo[a]) / ext : 0.0f;
                f = fminf(fmaxf(f, 0.0f), 1.0f);
                m |= spread3((uint32_t)(f * 511.0f)) << (2 - a);
            }
            key = (oct << 27) | m;
        }
        keys[i] = key;
        iota[i] = i;
    }
}

template <bool COUNT, bool DIAG, int GEO, int LDSN>
static void wf_iteration(const LaunchArgs& a, const WfBuffers& b, uint32_t trace_grid, uint32_t shade_grid,
                         hipStream_t stream)
{
    hipLaunchKernelGGL((dev::wf_trace<COUNT, DIAG, GEO, LDSN>), dim3(trace_grid), dim3(64), 0, stream, a.sd, a.draws,
                       a.tri_records, b, a.status, a.counters, a.wf_refill, a.materials, a.spheres, a.image, a.W, a.H);
    hipLaunchKernelGGL(dev::wf_shade<COUNT>, dim3(shade_grid), dim3(dev::kShadeBlock), 0, stream, a.sd, a.materials,
                       a.spheres, a.draws, a.tri_records, b, a.image, a.W, a.H, RowMap{a.y0, a.row_shift, a.row_gap}, a.counters);
}

template <bool COUNT, bool DIAG, int GEO, int LDSN>
static hipError_t trace_blocks_per_cu(int& bpc)
{
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, dev::wf_trace<COUNT, DIAG, GEO, LDSN>, 64, 0);
}

/* One (mode, single-draw, LDS depth) instantiation: occupancy query or one trace+shade iteration. */
template <bool COUNT, bool DIAG, int GEO, int LDSN>
static hipError_t wf_variant(bool query, int& bpc, const LaunchArgs& a, const WfBuffers& b, uint32_t trace_grid,
                             uint32_t shade_grid, hipStream_t stream)
{
    if (query) return trace_blocks_per_cu<COUNT, DIAG, GEO, LDSN>(bpc);
    wf_iteration<COUNT, DIAG, GEO, LDSN>(a, b, trace_grid, shade_grid, stream);
    return hipGetLastError();
}

/* The path-persistent trace (PERSIST): one launch for every segment of the pipeline's paths; GEO 2 or 3. */
template <int GEO>
static hipError_t wf_persist_variant(bool query, int& bpc, const LaunchArgs& a, const WfBuffers& b, uint32_t grid,
                                     hipStream_t stream)
{
    if (query)
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, dev::wf_trace<false, false, GEO, 10, true>, 64, 0);
    hipLaunchKernelGGL((dev::wf_trace<false, false, GEO, 10, true>), dim3(grid), dim3(64), 0, stream, a.sd, a.draws,
                       a.tri_records, b, a.status, a.counters, a.wf_refill_persist, a.materials, a.spheres, a.image, a.W,
                       a.H);
    return hipGetLastError();
}
static hipError_t wf_persist_dispatch(int geo, bool query, int& bpc, const LaunchArgs& a, const WfBuffers& b,
                                      uint32_t grid, hipStream_t stream)
{
    return geo == 3 ? wf_persist_variant<3>(query, bpc, a, b, grid, stream)
                    : wf_persist_variant<2>(query, bpc, a, b, grid, stream);
}

static hipError_t wf_dispatch(int mode, int geo, int ldsn, bool query, int& bpc, const LaunchArgs& a,
                              const WfBuffers& b, uint32_t tg, uint32_t sg, hipStream_t st)
{
    const bool single = geo >= 1;
    if (mode == kModeCount) return single ? wf_variant<true, false, 1, 10>(query, bpc, a, b, tg, sg, st)
                                          : wf_variant<true, false, 0, 10>(query, bpc, a, b, tg, sg, st);
    if (mode == kModeDiag) return single ? wf_variant<true, true, 1, 10>(query, bpc, a, b, tg, sg, st)
                                         : wf_variant<true, true, 0, 10>(query, bpc, a, b, tg, sg, st);
    if (!single) return wf_variant<false, false, 0, 10>(query, bpc, a, b, tg, sg, st);
    if (geo == 2) return wf_variant<false, false, 2, 10>(query, bpc, a, b, tg, sg, st);
    if (geo == 3) return wf_variant<false, false, 3, 10>(query, bpc, a, b, tg, sg, st);
    if (ldsn == 16) return wf_variant<false, false, 1, 16>(query, bpc, a, b, tg, sg, st);
    if (ldsn == 24) return wf_variant<false, false, 1, 24>(query, bpc, a, b, tg, sg, st);
    return wf_variant<false, false, 1, 10>(query, bpc, a, b, tg, sg, st);
}

/* The trace instantiation for this launch: 0 any draws, 1 one draw, 2 one draw on the fast layout (render build, the
 * default LDS stack; LaunchArgs::wf_fast). */
static int wf_geo(const LaunchArgs& a, int mode, int ldsn)
{
    if (a.sd.drawCommandCount != 1) return 0;
    return (WCPT_WF_GEO_FAST && a.wf_fast && mode == kModeRender && ldsn == 10) ? 2 : 1;
}

/* One fetch round per trace iteration (GEO 3) or two (GEO 2: a lane that descends into a leaf tests its first
 * triangle in the same iteration, after the interior lanes' fetch). One round overlaps the interior and leaf lanes'
 * fetches, which pays where fetch latency is exposed -- few queued rays per resident lane, so much of the launch is
 * its tail -- and costs an iteration per leaf descent, which loses where the chip is issue-bound on a long queue.
 * Measured (profiles/r05_fetch_once_ab.log): c3 (4.0 rays per lane per pipeline) 4.52 against 4.66 ms; c4 (15.8)
 * 203.6 against 199.6 ms. WCPT_OPTION_WF_FETCH: -1 (default) by that ratio, 0 two rounds, 1 one round. */
#ifndef WCPT_WF_FETCH_ONCE_RATIO
#define WCPT_WF_FETCH_ONCE_RATIO 8
#endif
static int wf_trace_geo(const LaunchArgs& a, int mode, int ldsn, uint32_t P, uint32_t trace_grid)
{
    const int geo = wf_geo(a, mode, ldsn);
    if (geo != 2 || a.wf_fetch == 0) return geo;
    if (a.wf_fetch > 0) return 3;
    return (uint64_t)P <= (uint64_t)WCPT_WF_FETCH_ONCE_RATIO * 64ull * trace_grid ? 3 : 2;
}

static hipError_t sort_queue(const LaunchArgs& a, WfState& s, const WfBuffers& b, uint32_t P, int cus,
                             hipStream_t stream)
{
    hipError_t r = wf_reserve_sort(s, P);
    if (r != hipSuccess) return r;
    const uint32_t grid = min((P + 255u) / 256u, (uint32_t)cus * 8u);
    hipLaunchKernelGGL(wf_sort_keys, dim3(grid), dim3(256), 0, stream, b, P, a.draws, s.sort_keys, s.sort_iota);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t temp = s.sort_temp_bytes;
    /* values: slot ids 0..P-1 -> the trace order of the input slots (b.order) */
    return hipcub::DeviceRadixSort::SortPairs(s.sort_temp, temp, s.sort_keys, s.sort_keys_alt, s.sort_iota,
                                              s.sort_order, (int)P, 0, 32, stream);
}

/* One pipeline: init (pipe_begin) + samples*(maxBounce+1) trace/shade iterations (pipe_iterate) over the tiles t with
 * t % npipes == pipe. */
static hipError_t pipe_begin(const LaunchArgs& a, int mode, WfState& s, const WfState& s0, float4* result, float4* prim_hit,
                             uint32_t pipe, uint32_t npipes, int cus, hipStream_t stream, WfBuffers& b)
{
    const uint32_t tilesX = (a.W + 7u) / 8u;
    const uint32_t tiles = tilesX * ((a.rows + 7u) / 8u);
    if (pipe >= tiles) return hipSuccess;
    const uint32_t total = ((tiles - pipe + npipes - 1u) / npipes) * 64u;
    /* live paths of this pipeline <= its pixels: the slot arrays are sized by its share of the tiles, not the frame */
    const uint32_t P = min(total, a.W * a.rows);
    hipError_t e = wf_reserve(s, P);
    if (e != hipSuccess) return e;
    const bool count = mode != kModeRender;
    /* The queue counters must start at zero. WCPT_WF_CTR_PARITY: the pipeline alternates between two counter sets,
     * and each frame's wf_init zeroes the set the next frame uses -- the frames of one pipeline run in order on its
     * stream (and a render's pipelines join before the next render forks), so the previous frame, the only other user
     * of that set, has finished; only a fresh allocation is zeroed with a memset. Otherwise one memset per pipeline
     * and frame (a fill kernel launch in the pipeline's chain). */
    uint32_t* ctr = s.ctr;
    uint32_t* zero_next = nullptr;
#if WCPT_WF_CTR_PARITY
    if (s.ctr_fresh) {
        e = hipMemsetAsync(s.ctr, 0, 8 * sizeof(uint32_t), stream);
        if (e != hipSuccess) return e;
        s.ctr_fresh = false;
        s.parity = 0;
    }
    ctr = s.ctr + 4u * s.parity;
    zero_next = s.ctr + 4u * (s.parity ^ 1u);
    s.parity ^= 1u;
#else
    e = hipMemsetAsync(s.ctr, 0, 4 * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
#endif
    b.in = s.soa[0];
    b.out = s.soa[1];
    b.result = result;
    b.prim_hit = prim_hit;
    b.hit = s.hit;
    b.order = nullptr;
    b.head = ctr + 2;
    b.diag = s0.diag;
    if (mode == kModeDiag) {
        e = hipMemsetAsync(s0.diag, 0, dev::kDiagTimers * sizeof(unsigned long long), stream);
        if (e != hipSuccess) return e;
    }
    b.wire = a.wire;
    b.wire_ch = a.wire_ch;
    b.wire_rows = a.wire_rows;
    b.count_in = ctr + 0;
    b.count_out = ctr + 1;
    const uint32_t init_grid = min((total + dev::kShadeBlock - 1) / dev::kShadeBlock, (uint32_t)cus * 16u);
    if (count)
        hipLaunchKernelGGL(dev::wf_init<true>, dim3(init_grid), dim3(dev::kShadeBlock), 0, stream, a.sd, a.spheres, b, a.image,
                           a.W, a.H, RowMap{a.y0, a.row_shift, a.row_gap}, a.rows, tilesX, total, pipe, npipes, a.counters,
                           zero_next);
    else
        hipLaunchKernelGGL(dev::wf_init<false>, dim3(init_grid), dim3(dev::kShadeBlock), 0, stream, a.sd, a.spheres, b, a.image,
                           a.W, a.H, RowMap{a.y0, a.row_shift, a.row_gap}, a.rows, tilesX, total, pipe, npipes, a.counters,
                           zero_next);
    return hipGetLastError();
}

static hipError_t pipe_iterate(const LaunchArgs& a, int mode, WfState& s, uint32_t pipe, uint32_t npipes,
                               bool sort_rays, int ldsn, int cus, uint32_t trace_grid, uint32_t shade_grid,
                               uint32_t persist_grid, hipStream_t stream, WfBuffers b)
{
    const uint32_t tilesX = (a.W + 7u) / 8u;
    const uint32_t tiles = tilesX * ((a.rows + 7u) / 8u);
    if (pipe >= tiles) return hipSuccess;
    const uint32_t P = min(((tiles - pipe + npipes - 1u) / npipes) * 64u, a.W * a.rows); /* as pipe_begin */
    /* one draw: the reference's case (PathTracingRenderer.jai:251) */
    const int geo = wf_trace_geo(a, mode, ldsn, P, trace_grid);
    hipError_t e = hipSuccess;
    if (persist_grid) { /* every segment in one launch (launch_wavefront) */
        int unused = 0;
        return wf_persist_dispatch(WCPT_WF_PERSIST_GEO, false, unused, a, b, persist_grid, stream);
    }
    /* each iteration advances every live path by one traced segment; a path needs <= samples*(maxBounce+1), or
     * with the primary records reused (wf_shade) maxBounce+1 for sample 0 and maxBounce for each later sample */
    uint64_t iters = (uint64_t)a.sd.samples * ((uint64_t)a.sd.maxBounceCount + 1ull);
    if (WCPT_WF_PRIMARY_REUSE && mode == kModeRender && a.sd.samples > 1u)
        iters = (uint64_t)a.sd.maxBounceCount + 1ull + (uint64_t)(a.sd.samples - 1u) * a.sd.maxBounceCount;
    if (iters > (1ull << 20)) iters = 1ull << 20; /* bounded; WCPT documents the cap */
    for (uint64_t it = 0; it < iters; it++) {
        b.order = nullptr;
        if (sort_rays && it > 0) { /* bounce rays; the primary queue is already in 8x8-tile order */
            e = sort_queue(a, s, b, P, cus, stream);
            if (e != hipSuccess) return e;
            b.order = s.sort_order;
        }
        int unused = 0;
        e = wf_dispatch(mode, geo, ldsn, false, unused, a, b, trace_grid, shade_grid, stream);
        if (e != hipSuccess) return e;
        std::swap(b.in, b.out);
        std::swap(b.count_in, b.count_out);
    }
    return hipSuccess;
}

#ifndef WCPT_WF_START_TOGETHER
#define WCPT_WF_START_TOGETHER 0
#endif

hipError_t wf_join(WfPipes& w, hipStream_t stream)
{
    if (!w.pending) return hipSuccess;
    w.pending = false;
    hipError_t first = hipSuccess;
    for (uint32_t j = 1; j < w.pending_pipes; j++) {
        hipError_t e = hipEventRecord(w.join[j], w.aux[j]);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, w.join[j], 0);
        if (e != hipSuccess && first == hipSuccess) first = e;
    }
    return first;
}

hipError_t launch_wavefront(const LaunchArgs& a, int mode, WfPipes& w, int pipes, bool sort_rays, int lds_stack,
                            hipStream_t stream, int overlap)
{
    const uint32_t tilesX = (a.W + 7u) / 8u;
    const uint32_t tilesY = (a.rows + 7u) / 8u;
    const uint64_t total64 = (uint64_t)tilesX * tilesY * 64ull;
    if (total64 == 0) return hipSuccess;
    if (total64 > 0xFFFFFFC0ull || (uint64_t)a.W * a.rows > 0xFFFFFFFFull) return hipErrorInvalidValue;
    WfState& s0 = w.pipe[0];
    int cus = 0;
    hipError_t e = cu_count(s0, cus);
    if (e != hipSuccess) return e;
    const int ldsn = (lds_stack == 16 || lds_stack == 24) ? lds_stack : 10;
    const int geo = wf_geo(a, mode, ldsn); /* GEO 3 (wf_trace_geo) runs at GEO 2's occupancy: both 8 waves/SIMD */
    int& bpc = s0.trace_bpc[mode][geo][ldsn == 10 ? 0 : (ldsn == 16 ? 1 : 2)];
    if (bpc == 0) {
        e = wf_dispatch(mode, geo, ldsn, true, bpc, a, WfBuffers{}, 0, 0, stream);
        if (e != hipSuccess) return e;
        if (bpc < 1) bpc = 1;
    }
    uint32_t trace_grid = (uint32_t)(bpc * cus);
/* Shade blocks per CU (grid-stride over the queue). The continuing paths are appended in roughly the order
 * the blocks walk their chunks, so a small grid keeps the next queue close to the input order (coherent rays
 * for the next trace). Measured on c3: 4 -> 7.98 ms, 8 -> 8.13, 16 -> 8.56, 32 -> 8.98, one thread per slot ->
 * 8.97. */
#ifndef WCPT_SHADE_BLOCKS_PER_CU
#define WCPT_SHADE_BLOCKS_PER_CU 4
#endif
    /* 0: one thread per path slot (no grid-stride loop) */
    const uint32_t P = a.W * a.rows;
    const uint32_t shade_grid = WCPT_SHADE_BLOCKS_PER_CU > 0 ? (uint32_t)(cus * WCPT_SHADE_BLOCKS_PER_CU)
                                                             : (P + dev::kShadeBlock - 1) / dev::kShadeBlock;
    sort_rays = sort_rays && a.sd.drawCommandCount > 0;
    /* the path-persistent trace (WCPT_OPTION_WF_PERSIST): one sample per pixel on the fast layout, and by default only
     * where the frame's paths about fit its resident lanes (row blocks): there the per-bounce
     * launches each last as long as their slowest ray, and one launch that lets each path run on lasts as long as its
     * slowest path (c3 135-row blocks 1.30 against 1.85 ms; the full c3 frame 6.64 against 4.55 ms,
     * profiles/r05_persist_ab.log) */
    const bool persist_ok = mode == kModeRender && geo == 2 && a.sd.samples == 1u && !sort_rays && a.wf_persist != 0;
    if (persist_ok && s0.persist_bpc == 0) {
        e = wf_persist_dispatch(WCPT_WF_PERSIST_GEO, true, s0.persist_bpc, a, WfBuffers{}, 0, stream);
        if (e != hipSuccess) return e;
        if (s0.persist_bpc < 1) s0.persist_bpc = 1;
    }
    const uint32_t persist_full = persist_ok ? (uint32_t)(s0.persist_bpc * cus) : 0u;
    /* at most 1.4 paths per resident lane: the lanes freed by the first paths take the rest (7- / 6-way c3 splits at
     * 1.13 / 1.32 paths per lane gain 7 % / 3 %, 5-way at 1.58 is flat, 4-way at 2.0 loses) */
    const bool persist = persist_ok && (a.wf_persist > 0 || (uint64_t)a.W * a.rows * 5ull <= 64ull * 7ull * persist_full);
    /* pipelines: the option's count, or (0, the default) for the path-persistent trace one when each frame joins its
     * pipelines (its blocks measured 1.30 / 1.40 / 1.40 ms with 1 / 2 / 3) and two under the frame overlap, where a
     * pipeline's persistent launch runs on into its next frame (c3 8-way shares, slowest of 8, region-timed: 8-row
     * stripes 1.254 / 1.246 ms with one, 1.219 / 1.218 with two, 1.218 / 1.214 with three -- a third stream would sit
     * past the four hardware queues beside a group's communication stream; profiles/r06_c3_persist_pipes.log); else 3
     * when the frame holds at most 8 paths per resident trace lane -- the launches are short and their tails weigh, so
     * a third chain overlaps them (c3 4.41-4.46 against 4.50-4.55 ms with two) -- and 2 on longer queues (c4 199.5
     * against 197.9 ms with two; profiles/r05_pipes_ab.log) */
    uint32_t K = (uint32_t)(pipes > kWfMaxPipes ? kWfMaxPipes : pipes);
    if (pipes < 1) {
        K = persist ? (overlap != 0 && mode == kModeRender ? 2u : 1u)
                    : ((uint64_t)a.W * a.rows <= (uint64_t)WCPT_WF_FETCH_ONCE_RATIO * 64ull * trace_grid ? 3u : 2u);
    }
    if (sort_rays || mode == kModeDiag) K = 1; /* one sort scratch and one diagnostics block */
    const uint32_t tiles = tilesX * tilesY;
    if (K > tiles) K = tiles;
#if WCPT_WF_TRACE_SHARE
    /* each pipeline's persistent trace grid holds 1/K of the resident-wave slots, so the K traces run side by side
     * instead of the first one taking every slot and the others only filling its tail (c3 6.58 -> 6.16 ms with two
     * pipelines; 5/8 or 3/4 of the slots per pipeline measured equal, 7/16 slower) */
    if (K > 1) trace_grid = trace_grid / K > 0 ? trace_grid / K : 1u;
#endif
    const uint32_t persist_grid = persist ? max(1u, persist_full / K) : 0u;
    /* Frame overlap (WCPT_OPTION_FRAME_OVERLAP; the megakernel's in pt_kernels.hip launch_megakernel): pipeline j
     * owns the tiles t % K == j, so while K and the frame's tiles stay, this render's pipelines need not wait for the
     * previous render's other pipelines -- each continues on its own stream, and the context's stream is joined to
     * them only when another entry point needs it (wf_join). On the per-bounce launches that recovers the frame's
     * ragged end (c3: its three pipelines end 0.3-0.5 ms apart, profiles/r06_c3_frame_timeline.log). */
    const bool cont = overlap != 0 && K > 1 && !WCPT_WF_START_TOGETHER && mode == kModeRender && w.pending &&
                      w.pending_pipes == K && w.pending_W == a.W && w.pending_rows == a.rows &&
                      w.pending_persist == (persist_grid != 0);
    if (w.pending && !cont) {
        e = wf_join(w, stream);
        if (e != hipSuccess) return e;
    }
    e = wf_reserve_result(w, (uint64_t)a.W * a.rows);
    if (e != hipSuccess) return e;
    WfBuffers bs[kWfMaxPipes];
    if (K == 1) {
        e = pipe_begin(a, mode, s0, s0, w.result, w.result + w.result_capacity, 0, 1, cus, stream, bs[0]);
        if (e != hipSuccess) return e;
        return pipe_iterate(a, mode, s0, 0, 1, sort_rays, ldsn, cus, trace_grid, shade_grid, persist_grid, stream, bs[0]);
    }

    /* fork: pipelines 1..K-1 run on their own streams after everything already queued on the context's stream */
    if (!w.fork) {
        e = hipEventCreateWithFlags(&w.fork, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    for (uint32_t j = 1; j < K; j++) {
        if (!w.aux[j]) {
            e = hipStreamCreateWithFlags(&w.aux[j], hipStreamNonBlocking);
            if (e != hipSuccess) return e;
        }
        if (!w.join[j]) {
            e = hipEventCreateWithFlags(&w.join[j], hipEventDisableTiming);
            if (e != hipSuccess) return e;
        }
    }
    if (!cont) {
        e = hipEventRecord(w.fork, stream);
        if (e != hipSuccess) return e;
        for (uint32_t j = 1; j < K; j++) {
            e = hipStreamWaitEvent(w.aux[j], w.fork, 0);
            if (e != hipSuccess) return e;
        }
    }
    hipError_t first = hipSuccess;
    for (uint32_t j = 0; j < K && first == hipSuccess; j++)
        first = pipe_begin(a, mode, w.pipe[j], s0, w.result, w.result + w.result_capacity, j, K, cus, j == 0 ? stream : w.aux[j], bs[j]);
    if (WCPT_WF_START_TOGETHER && first == hipSuccess) {
        /* every pipeline's first trace waits for all the inits: the persistent trace grids then start on an idle
         * chip together instead of the first one being placed around the other pipelines' init blocks */
        for (uint32_t j = 0; j < K && first == hipSuccess; j++) {
            if (!w.ready[j]) first = hipEventCreateWithFlags(&w.ready[j], hipEventDisableTiming);
            if (first == hipSuccess) first = hipEventRecord(w.ready[j], j == 0 ? stream : w.aux[j]);
        }
        for (uint32_t j = 0; j < K && first == hipSuccess; j++)
            for (uint32_t i = 0; i < K && first == hipSuccess; i++)
                if (i != j) first = hipStreamWaitEvent(j == 0 ? stream : w.aux[j], w.ready[i], 0);
    }
    for (uint32_t j = 0; j < K && first == hipSuccess; j++)
        first = pipe_iterate(a, mode, w.pipe[j], j, K, false, ldsn, cus, trace_grid, shade_grid, persist_grid,
                             j == 0 ? stream : w.aux[j], bs[j]);
    /* join: the context's stream continues after every pipeline (also after a failed enqueue) -- now, or with the
     * frame overlap when another entry point needs the stream (wf_join) */
    w.pending = true;
    w.pending_pipes = K;
    w.pending_W = a.W;
    w.pending_rows = a.rows;
    w.pending_persist = persist_grid != 0;
    if (!overlap || mode != kModeRender || first != hipSuccess) {
        e = wf_join(w, stream);
        if (e != hipSuccess && first == hipSuccess) first = e;
    }
    return first;
}

} // namespace wcpt
