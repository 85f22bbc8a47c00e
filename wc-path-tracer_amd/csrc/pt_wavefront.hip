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
 * changes. Path state lives in HBM as structure-of-arrays float4s (80 B/path + 24 B hit record).
 */
#include <hip/hip_runtime.h>

#include "pt_device.h"
#include "pt_kernels.h"

namespace wcpt {
namespace dev {

constexpr uint32_t kTraceChunk = 64;   /* queue entries a wave claims per atomicAdd */
constexpr int kShadeBlock = 256;

/* Hit record flags */
constexpr uint32_t kHitFlag = 1u, kFrontFlag = 2u;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ unsigned long long lanemask_lt() { return (1ull << lane_id()) - 1ull; }

__device__ __forceinline__ void store_ray(const WfBuffers& b, uint32_t p, const Ray& r, uint32_t bounce, uint32_t sample)
{
    b.ray0[p] = make_float4(r.origin.x, r.origin.y, r.origin.z, r.direction.x);
    b.ray1[p] = make_float4(r.direction.y, r.direction.z, __uint_as_float(bounce), __uint_as_float(sample));
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

/* ---- ray generation ------------------------------------------------------------------------------- */
template <bool COUNT>
__global__ __launch_bounds__(kShadeBlock) void wf_init(const wcpt_scene_data sd, WfBuffers b, float4* __restrict__ image,
                                                       uint32_t W, uint32_t H, uint32_t y0, uint32_t rows,
                                                       uint32_t tilesX, uint32_t total,
                                                       unsigned long long* __restrict__ counters)
{
    __shared__ uint32_t s_wave[kShadeBlock / 64], s_base;
    Counters cnt = {};
    for (uint32_t base = blockIdx.x * blockDim.x; base < total; base += gridDim.x * blockDim.x) {
        const uint32_t w = base + threadIdx.x;
        bool live = false;
        uint32_t p = 0;
        if (w < total) {
            const uint32_t t = w >> 6, q = w & 63u;           /* 8x8 tiles: coherent initial queue */
            const uint32_t lx = (t % tilesX) * 8u + (q & 7u);
            const uint32_t ly = (t / tilesX) * 8u + (q >> 3);
            if (lx < W && ly < rows) {
                p = ly * W + lx;
                const uint32_t y = y0 + ly;
                const uint32_t seed = pcg_hash(lx + y * W + sd.renderedFramesCount * 719393u); /* :304-305 */
                b.result[p] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (sd.samples > 0) {
                    PathState ps;
                    path_begin(ps, mk3(sd.position[0], sd.position[1], sd.position[2]),
                               primary_direction(sd, lx, y, W, H));
                    store_ray(b, p, ps.ray, 0u, 0u);
                    b.light[p] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(seed));
                    b.trans[p] = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
                    live = true;
                } else { /* samples == 0: result / 0 = NaN (:312), stored as the reference would */
                    const f3 r = mk3(0.0f, 0.0f, 0.0f) / (float)sd.samples;
                    if (!COUNT) image[(size_t)ly * W + lx] = make_float4(r.x, r.y, r.z, 1.0f);
                    if (COUNT) cnt.pixels++;
                }
            }
        }
        const uint32_t slot = block_append(b.count_in, live, s_wave, &s_base);
        if (live) b.queue_in[slot] = p;
    }
    if (COUNT) wave_add_u64(&counters[0], cnt.pixels);
}

/* ---- trace ------------------------------------------------------------------------------------------ */
enum : uint32_t { kModeInterior = 0, kModeLeaf = 1, kModePop = 2, kModeDone = 3 };

struct Trav {
    const wcpt_node* bvh;
    const uint32_t* indices;
    const float* vertices;
    uint32_t d, curLeft, curCount, k, mode;
};

/* Start draw command t.d (or the next one whose root survives the cull, :152-162); kModeDone past the last. */
template <bool COUNT, class Stack>
__device__ __forceinline__ void start_draw(Trav& t, const Ray& ray, float recT, const wcpt_scene_data& sd,
                                           const wcpt_draw_command* __restrict__ draws, Stack& stk, Counters& cnt)
{
    for (; t.d < sd.drawCommandCount; t.d++) {
        t.bvh = reinterpret_cast<const wcpt_node*>(draws[t.d].bvhBuffer);
        t.indices = reinterpret_cast<const uint32_t*>(draws[t.d].indexBuffer);
        t.vertices = reinterpret_cast<const float*>(draws[t.d].vertexBuffer);
        if (COUNT) { cnt.draw_fetches++; cnt.node_pops++; }
        const NodeV root = load_node(t.bvh, 0);
        float c0, c1;
        node_box(ray, root, c0, c1);
        if (c0 > c1 || c1 < 0.0f || c0 > recT) continue;
        t.curLeft = root.b.z;
        t.curCount = root.b.w;
        t.k = 0;
        t.mode = t.curCount > 0 ? kModeLeaf : kModeInterior;
        stk.reset();
        return;
    }
    t.mode = kModeDone;
}

template <bool COUNT, bool DIAG>
__global__ __launch_bounds__(64) void wf_trace(const wcpt_scene_data sd, const wcpt_sphere* __restrict__ spheres,
                                               const wcpt_draw_command* __restrict__ draws, WfBuffers b,
                                               uint32_t* __restrict__ status, unsigned long long* __restrict__ counters)
{
    __shared__ uint2 s_stack[kLdsStack * 64];
    if (blockIdx.x == 0 && threadIdx.x == 0) *b.count_out = 0; /* shade appends to it after this kernel */
    const uint32_t n = *b.count_in;
    const uint32_t lane = lane_id();
    LdsStack<kLdsStack, kSpillStack> stk;
    stk.base = s_stack + lane;
    Counters cnt = {};
    bool overflow = false;

    bool has = false, drained = false;
    uint32_t lo = 0, hi = 0; /* this wave's claimed queue range [lo, hi) (wave-uniform) */
    uint32_t p = 0;
    Ray ray;
    Hit rec;
    Trav t;
    t.mode = kModeDone;
    for (;;) {
        /* dynamic fetch: idle lanes take the next queued rays */
        if (!drained) {
            unsigned long long need = __ballot(!has);
            while (need) {
                if (lo == hi) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(b.head, kTraceChunk);
                    base = __shfl(base, 0, 64);
                    if (base >= n) {
                        drained = true;
                        break;
                    }
                    lo = base;
                    hi = min(base + kTraceChunk, n);
                }
                const uint32_t avail = hi - lo;
                const uint32_t rank = (uint32_t)__popcll(need & lanemask_lt());
                const bool take = ((need >> lane) & 1ull) && rank < avail;
                if (take) {
                    p = b.queue_in[lo + rank];
                    const float4 r0 = b.ray0[p], r1 = b.ray1[p];
                    ray.origin = mk3(r0.x, r0.y, r0.z);
                    ray.direction = mk3(r0.w, r1.x, r1.y);
                    ray.invDirection = rcp3(ray.direction);
                    /* Intersect prologue (:136-149): the sphere loop */
                    rec.t = kInfinity;
                    rec.hit = false;
                    rec.front = false;
                    rec.material = 0;
                    rec.normal = mk3(0.0f, 0.0f, 0.0f);
                    if (COUNT) {
                        cnt.segments++;
                        simd_step<DIAG>(cnt.wave_seg, cnt.lane_seg);
                    }
                    for (uint32_t i = 0; i < sd.sphereCount; i++) {
                        const wcpt_sphere& s = spheres[i];
                        const f3 spc = mk3(s.position[0], s.position[1], s.position[2]);
                        const float tempRec = raySphereNear(ray, spc, s.radius);
                        if (COUNT) cnt.sphere_tests++;
                        if (tempRec > 0.0f && tempRec < rec.t) {
                            rec.t = tempRec;
                            rec.p = ray.origin + rec.t * ray.direction;
                            rec.normal = (rec.p - spc) / s.radius;
                            rec.hit = true;
                            rec.material = s.material;
                        }
                    }
                    t.d = 0;
                    start_draw<COUNT>(t, ray, rec.t, sd, draws, stk, cnt);
                    has = true;
                }
                const uint32_t took = min(avail, (uint32_t)__popcll(need));
                lo += took;
                need &= ~__ballot(take);
            }
        }
        if (!__ballot(has)) break;
        if (has) {
            /* one traversal step (:157-200) */
            if (t.mode == kModeLeaf) {
                const uint32_t first = t.k + t.curLeft;
                const uint32_t ia = t.indices[first + 0];
                const uint32_t ib = t.indices[first + 1];
                const uint32_t ic = t.indices[first + 2];
                const f3 a = ld3(t.vertices + 3ull * ia);
                const f3 bb = ld3(t.vertices + 3ull * ib);
                const f3 c = ld3(t.vertices + 3ull * ic);
                const float tt = rayTriangle(ray, a, bb, c);
                if (COUNT) {
                    cnt.triangle_tests++;
                    simd_step<DIAG>(cnt.wave_tri, cnt.lane_tri);
                }
                if (tt != -1.0f && tt < rec.t) {
                    rec.t = tt;
                    rec.normal = normalize(cross(bb - a, c - a));
                    rec.hit = true;
                    rec.material = 0; /* :175 */
                }
                t.k += 3;
                if (t.k >= t.curCount) t.mode = kModePop;
            } else if (t.mode == kModeInterior) {
                const NodeV L = load_node(t.bvh, t.curLeft);
                const NodeV R = load_node(t.bvh, t.curLeft + 1);
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
                const uint32_t farIdx = leftFirst ? t.curLeft + 1 : t.curLeft;
                const bool passNear = leftFirst ? passL : passR;
                const bool passFar = leftFirst ? passR : passL;
                const float nearT0 = leftFirst ? l0 : r0;
                const float farT0 = leftFirst ? r0 : l0;
                if (passFar && !stk.push(farIdx, farT0)) overflow = true;
                if (passNear && !(nearT0 > rec.t)) {
                    const NodeV& N = leftFirst ? L : R;
                    t.curLeft = N.b.z;
                    t.curCount = N.b.w;
                    t.k = 0;
                    t.mode = t.curCount > 0 ? kModeLeaf : kModeInterior;
                } else {
                    t.mode = kModePop;
                }
            }
            if (t.mode == kModePop) {
                bool found = false;
                while (!stk.empty()) {
                    uint32_t ni;
                    float t0;
                    stk.pop(ni, t0);
                    if (t0 > rec.t) continue;
                    const uint2 lc = reinterpret_cast<const uint2*>(t.bvh + ni)[3];
                    t.curLeft = lc.x;
                    t.curCount = lc.y;
                    t.k = 0;
                    t.mode = t.curCount > 0 ? kModeLeaf : kModeInterior;
                    found = true;
                    break;
                }
                if (!found) {
                    t.d++;
                    start_draw<COUNT>(t, ray, rec.t, sd, draws, stk, cnt);
                }
            }
            if (t.mode == kModeDone) {
                /* Intersect epilogue (:204-208) */
                uint32_t flags = 0;
                if (rec.hit) {
                    rec.front = dot(ray.direction, rec.normal) < 0.0f;
                    if (!rec.front) rec.normal = rec.normal * -1.0f;
                    flags = kHitFlag | (rec.front ? kFrontFlag : 0u);
                    if (COUNT) cnt.hits++;
                }
                b.hit[p] = make_float4(rec.t, rec.normal.x, rec.normal.y, rec.normal.z);
                b.hitinfo[p] = make_uint2(rec.material, flags);
                has = false;
            }
        }
    }
    if (overflow) atomicOr(status, 1u);
    flush_counters<COUNT>(cnt, counters);
}

/* ---- shade ------------------------------------------------------------------------------------------ */
template <bool COUNT>
__global__ __launch_bounds__(kShadeBlock) void wf_shade(const wcpt_scene_data sd, const wcpt_material* __restrict__ mats,
                                                        WfBuffers b, float4* __restrict__ image, uint32_t W,
                                                        uint32_t H, uint32_t y0, unsigned long long* __restrict__ counters)
{
    __shared__ uint32_t s_wave[kShadeBlock / 64], s_base;
    if (blockIdx.x == 0 && threadIdx.x == 0) *b.head = 0; /* the trace of this iteration has finished */
    const uint32_t n = *b.count_in;
    Counters cnt = {};
    for (uint32_t base = blockIdx.x * blockDim.x; base < n; base += gridDim.x * blockDim.x) {
        const uint32_t w = base + threadIdx.x;
        bool cont = false;
        uint32_t p = 0;
        if (w < n) {
            p = b.queue_in[w];
            const float4 r0 = b.ray0[p], r1 = b.ray1[p], li = b.light[p], tr = b.trans[p], hi = b.hit[p];
            const uint2 hf = b.hitinfo[p];
            PathState ps;
            ps.ray.origin = mk3(r0.x, r0.y, r0.z);
            ps.ray.direction = mk3(r0.w, r1.x, r1.y);
            ps.ray.invDirection = rcp3(ps.ray.direction);
            ps.totalLight = mk3(li.x, li.y, li.z);
            ps.transmittance = mk3(tr.x, tr.y, tr.z);
            ps.bounce = __float_as_uint(r1.z);
            uint32_t sample = __float_as_uint(r1.w);
            uint32_t seed = __float_as_uint(li.w);
            Hit h;
            h.hit = (hf.y & kHitFlag) != 0u;
            h.front = (hf.y & kFrontFlag) != 0u;
            h.material = hf.x;
            h.t = hi.x;
            h.normal = mk3(hi.y, hi.z, hi.w);
            h.p = ps.ray.origin + h.t * ps.ray.direction; /* :205 */
            f3 L;
            if (!path_shade(ps, h, seed, sd, mats, L)) {
                cont = true;
            } else {
                const float4 rs = b.result[p];
                f3 result = mk3(rs.x, rs.y, rs.z) + L;                    /* :310 */
                sample++;
                const uint32_t lx = p % W, ly = p / W;
                if (sample < sd.samples) {                                  /* next sample, same primary ray */
                    path_begin(ps, mk3(sd.position[0], sd.position[1], sd.position[2]),
                               primary_direction(sd, lx, y0 + ly, W, H));
                    b.result[p] = make_float4(result.x, result.y, result.z, 0.0f);
                    cont = true;
                } else {
                    result = result / (float)sd.samples;                   /* :312 */
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
                        *px = make_float4(acc.x, acc.y, acc.z, 1.0f);
                    }
                    if (COUNT) cnt.pixels++;
                }
            }
            if (cont) {
                store_ray(b, p, ps.ray, ps.bounce, sample);
                b.light[p] = make_float4(ps.totalLight.x, ps.totalLight.y, ps.totalLight.z, __uint_as_float(seed));
                b.trans[p] = make_float4(ps.transmittance.x, ps.transmittance.y, ps.transmittance.z, 0.0f);
            }
        }
        const uint32_t slot = block_append(b.count_out, cont, s_wave, &s_base);
        if (cont) b.queue_out[slot] = p;
    }
    if (COUNT) wave_add_u64(&counters[0], cnt.pixels);
}

} // namespace dev

/* ---------------------------------------------------------------------------------------------------- */
static int g_cus = 0;

static hipError_t cu_count(int& cus)
{
    if (g_cus == 0) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
    }
    cus = g_cus;
    return hipSuccess;
}

hipError_t wf_reserve(WfState& s, uint32_t paths)
{
    if (paths <= s.capacity) return hipSuccess;
    wf_release(s);
    const size_t P = paths;
    const size_t bytes = P * (6 * sizeof(float4) + sizeof(uint2) + 2 * sizeof(uint32_t)) + 64;
    char* m = nullptr;
    hipError_t e = hipMalloc(&m, bytes);
    if (e != hipSuccess) return e;
    s.mem = m;
    float4* f = reinterpret_cast<float4*>(m);
    s.ray0 = f;
    s.ray1 = f + P;
    s.light = f + 2 * P;
    s.trans = f + 3 * P;
    s.result = f + 4 * P;
    s.hit = f + 5 * P;
    s.hitinfo = reinterpret_cast<uint2*>(f + 6 * P);
    s.queue[0] = reinterpret_cast<uint32_t*>(s.hitinfo + P);
    s.queue[1] = s.queue[0] + P;
    s.ctr = s.queue[1] + P; /* [0] count q0, [1] count q1, [2] trace head */
    s.capacity = paths;
    return hipSuccess;
}

void wf_release(WfState& s)
{
    if (s.mem) (void)hipFree(s.mem);
    s = WfState{};
}

template <bool COUNT, bool DIAG>
static void wf_iteration(const LaunchArgs& a, const WfBuffers& b, uint32_t trace_grid, uint32_t shade_grid,
                         hipStream_t stream)
{
    hipLaunchKernelGGL((dev::wf_trace<COUNT, DIAG>), dim3(trace_grid), dim3(64), 0, stream, a.sd, a.spheres, a.draws, b,
                       a.status, a.counters);
    hipLaunchKernelGGL(dev::wf_shade<COUNT>, dim3(shade_grid), dim3(dev::kShadeBlock), 0, stream, a.sd, a.materials, b,
                       a.image, a.W, a.H, a.y0, a.counters);
}

hipError_t launch_wavefront(const LaunchArgs& a, int mode, WfState& s, hipStream_t stream)
{
    const uint32_t tilesX = (a.W + 7u) / 8u;
    const uint32_t tilesY = (a.rows + 7u) / 8u;
    const uint64_t total64 = (uint64_t)tilesX * tilesY * 64ull;
    if (total64 == 0) return hipSuccess;
    if (total64 > 0xFFFFFFC0ull || (uint64_t)a.W * a.rows > 0xFFFFFFFFull) return hipErrorInvalidValue;
    const uint32_t total = (uint32_t)total64;
    const uint32_t P = a.W * a.rows;
    hipError_t e = wf_reserve(s, P);
    if (e != hipSuccess) return e;
    int cus = 0;
    e = cu_count(cus);
    if (e != hipSuccess) return e;
    const bool count = mode != kModeRender;
    static int trace_bpc[3] = {0, 0, 0};
    int& bpc = trace_bpc[mode];
    if (bpc == 0) {
        if (mode == kModeRender) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, dev::wf_trace<false, false>, 64, 0);
        else if (mode == kModeCount) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, dev::wf_trace<true, false>, 64, 0);
        else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, dev::wf_trace<true, true>, 64, 0);
        if (e != hipSuccess) return e;
        if (bpc < 1) bpc = 1;
    }
    const uint32_t trace_grid = (uint32_t)(bpc * cus);
    const uint32_t shade_grid = (uint32_t)(cus * 8);

    e = hipMemsetAsync(s.ctr, 0, 4 * sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    WfBuffers b;
    b.ray0 = s.ray0; b.ray1 = s.ray1; b.light = s.light; b.trans = s.trans; b.result = s.result;
    b.hit = s.hit; b.hitinfo = s.hitinfo; b.head = s.ctr + 2;
    b.queue_in = s.queue[0]; b.count_in = s.ctr + 0;
    b.queue_out = s.queue[1]; b.count_out = s.ctr + 1;
    const uint32_t init_grid = min((total + dev::kShadeBlock - 1) / dev::kShadeBlock, (uint32_t)cus * 16u);
    if (count)
        hipLaunchKernelGGL(dev::wf_init<true>, dim3(init_grid), dim3(dev::kShadeBlock), 0, stream, a.sd, b, a.image,
                           a.W, a.H, a.y0, a.rows, tilesX, total, a.counters);
    else
        hipLaunchKernelGGL(dev::wf_init<false>, dim3(init_grid), dim3(dev::kShadeBlock), 0, stream, a.sd, b, a.image,
                           a.W, a.H, a.y0, a.rows, tilesX, total, a.counters);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    /* each iteration advances every live path by one segment; a path needs <= samples*(maxBounce+1) */
    uint64_t iters = (uint64_t)a.sd.samples * ((uint64_t)a.sd.maxBounceCount + 1ull);
    if (iters > (1ull << 20)) iters = 1ull << 20; /* bounded; WCPT documents the cap */
    for (uint64_t it = 0; it < iters; it++) {
        if (mode == kModeRender) wf_iteration<false, false>(a, b, trace_grid, shade_grid, stream);
        else if (mode == kModeCount) wf_iteration<true, false>(a, b, trace_grid, shade_grid, stream);
        else wf_iteration<true, true>(a, b, trace_grid, shade_grid, stream);
        e = hipGetLastError();
        if (e != hipSuccess) return e;
        std::swap(b.queue_in, b.queue_out);
        std::swap(b.count_in, b.count_out);
    }
    return hipSuccess;
}

} // namespace wcpt
