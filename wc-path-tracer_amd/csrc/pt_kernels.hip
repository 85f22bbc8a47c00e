/*
 * pt_kernels.hip — the path-tracing megakernel for gfx950 (reference: src/shaders/pathTracer.comp:286-324).
 *
 * Launch shape: one 64-lane wave per 8x8 pixel tile (the reference's 4x4 = 16-invocation workgroups would
 * leave 48 of 64 lanes idle on wave64 CDNA). A bounds guard makes any width/height legal (the reference
 * has none, :289). SceneData arrives by value in the kernarg segment.
 *
 * Instantiations: COUNT=false renders; COUNT=true runs the same frame without writing the image and counts the
 * reference algorithm's work; DIAG=true additionally counts SIMD lane/wave steps with a
 * __ballot inside the traversal loop (tools/diag.py only — kept out of the COUNT build the parity tests use).
 */
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "pt_device.h"
#include "pt_kernels.h"

namespace wcpt {
namespace dev {

/* Pixel tile of one wave64: kTileW x kTileH. Measured on c2: 8x8 and 4x16 equal, 16x4 +3%, 32x2 +4%. */
#ifndef WCPT_TILE_W
#define WCPT_TILE_W 8
#endif
constexpr uint32_t kTileW = WCPT_TILE_W, kTileH = 64u / WCPT_TILE_W;

/* Pixel tile -> block mapping. Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
 * "Workgroup dispatch"); remapping the linear block id so that each XCD walks a contiguous band of tiles
 * keeps neighbouring (coherent) tiles on one XCD's L2. Speed only; any placement is correct. */
__device__ __forceinline__ void tile_of_block(uint32_t tilesX, uint32_t tilesTotal, uint32_t scatter,
                                              const uint32_t* __restrict__ order, uint32_t& tx, uint32_t& ty)
{
    const uint32_t b = blockIdx.x;
    uint32_t t = b;
    if (order != nullptr) {
        t = order[b]; /* cost-ordered: a permutation of [0, tilesTotal), longest tile first */
    } else if (scatter & 1u) {
        t = (uint32_t)(((uint64_t)b * scatter) % tilesTotal);   /* odd: scattered, multiplier `scatter` */
    } else if ((tilesTotal & 7u) == 0u) {
        /* blocks go to the XCDs round-robin (block b -> XCD b mod 8): XCD x walks the x-th eighth of a tile list */
        t = (b & 7u) * (tilesTotal >> 3) + (b >> 3);
        if (scatter != 0u) {
            /* even scatter = 2h: striped list. Stripes of h tile rows, listed by (stripe mod 8, stripe / 8), each in
             * raster order, so XCD x walks (about) the stripes s = x mod 8: neighbouring tiles stay together on an
             * XCD, and every XCD sees every part of the frame (one contiguous band per XCD can leave a few XCDs with
             * the heavy regions of the image) */
            const uint32_t h = scatter >> 1;
            const uint32_t tilesY = tilesTotal / tilesX;
            const uint32_t full = tilesY / (8u * h), rem = tilesY % (8u * h);
            for (uint32_t j = 0; j < 8u; j++) {
                const uint32_t part = rem > j * h ? min(rem - j * h, h) : 0u;
                const uint32_t seg = (full * h + part) * tilesX;   /* tiles of the rows in stripes s = j mod 8 */
                if (t < seg) {
                    const uint32_t lr = t / tilesX;
                    t = (((lr / h) * 8u + j) * h + lr % h) * tilesX + t % tilesX;
                    break;
                }
                t -= seg;
            }
        }
    }
    tx = t % tilesX;
    ty = t / tilesX;
}

/* Shade one pixel (pathTracer.comp:290-323) with the given traversal stack. */
template <bool COUNT, bool DIAG, bool PAIRS, bool SINGLE, bool REUSE, class Stack>
__device__ __forceinline__ void shade_pixel(const wcpt_scene_data& sd, const wcpt_material* __restrict__ mats,
                                            const wcpt_sphere* __restrict__ spheres,
                                            const wcpt_draw_command* __restrict__ draws,
                                            const uint64_t* __restrict__ tri_records, float4* __restrict__ image,
                                            float* __restrict__ wire, uint32_t wire_ch,
                                            uint32_t W, uint32_t H, const RowMap& rm, const RowMap& wm, uint32_t lx,
                                            uint32_t ly, Stack& stk, Counters& cnt, bool& overflow)
{
    const uint32_t x = lx, y = frame_row(rm, ly); /* the frame row: a row block or interleaved stripes (row_map.h) */
    const f3 dir = primary_direction(sd, x, y, W, H);
    const uint32_t pixel_index = x + y * W + sd.renderedFramesCount * 719393u; /* :304 */
    uint32_t seed = pcg_hash(pixel_index);
    /* The accumulation read (:314) is issued before the trace, so its HBM latency hides behind the segments
     * instead of stalling the wave at its end (the image is the one buffer that does not live in L2). */
    float4* px = image + (size_t)ly * W + lx;
    float4 old = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (!COUNT && sd.renderedFramesCount != 0) old = *px;
    phase_mark(cnt, 0);
    f3 result = mk3(0.0f, 0.0f, 0.0f);
    const f3 origin = mk3(sd.position[0], sd.position[1], sd.position[2]);
    float4 prim_rec = make_float4(0.0f, 0.0f, 0.0f, 0.0f); /* sample 0's primary Intersect record */
    for (uint32_t s = 0; s < sd.samples; s++) { /* :309-310, all samples share the primary ray */
        Ray r;
        r.origin = origin;
        r.direction = dir;
        r.invDirection = rcp3(dir);
        result = result + TraceRay<COUNT, DIAG, PAIRS, SINGLE, Stack, REUSE>(r, seed, sd, mats, spheres, draws, tri_records, stk, cnt, overflow,
                                                       s + 1u == sd.samples, prim_rec, s > 0u);
    }
    result = result / (float)sd.samples; /* :312 */
    if (!COUNT) {
        f3 acc;
        if (sd.renderedFramesCount == 0) { /* :318 — the loaded value would be discarded */
            acc = result;
        } else {
            const float4 o = old;                                             /* :314 */
            const float weight = 1.0f / (float)(sd.renderedFramesCount + 1u); /* :316 */
            const float iw = 1.0f - weight;
            acc = mk3(o.x * iw + result.x * weight, o.y * iw + result.y * weight, o.z * iw + result.z * weight);
        }
        store_pixel(image, wire, wire_ch, wm, W, lx, ly, acc); /* :323 */
    }
    if (COUNT) cnt.pixels++;
    phase_mark(cnt, 6);
}

/* Stack kinds: 0 = private (scratch) stack of kPrivateStack entries; 1 = LDS stack of kLdsStack entries per
 * lane with a kSpillStack-entry private spill. */
/* Occupancy floor for experiments (tools/ab_build.sh): __launch_bounds__'s minimum waves per SIMD. */
#ifndef WCPT_MK_WAVES
#define WCPT_MK_WAVES 1
#endif
template <bool COUNT, bool DIAG, int SK, bool PAIRS, bool SINGLE, bool REUSE>
__global__ __launch_bounds__(64, WCPT_MK_WAVES) void pt_megakernel(const wcpt_scene_data sd, const wcpt_material* __restrict__ mats,
                                                    const wcpt_sphere* __restrict__ spheres,
                                                    const wcpt_draw_command* __restrict__ draws,
                                                    const uint64_t* __restrict__ tri_records,
                                                    float4* __restrict__ image, float* __restrict__ wire,
                                                    uint32_t wire_ch, uint32_t W, uint32_t H, const RowMap rm,
                                                    const RowMap wm, uint32_t rows, uint32_t tilesX, uint32_t tilesTotal,
                                                    uint32_t scatter, const uint32_t* __restrict__ tile_order,
                                                    uint32_t* __restrict__ tile_cost, uint32_t* __restrict__ status,
                                                    unsigned long long* __restrict__ counters)
{
    const uint64_t c0 = (!COUNT && tile_cost) ? __builtin_amdgcn_s_memtime() : 0ull;
    uint32_t tx, ty;
    tile_of_block(tilesX, tilesTotal, scatter, tile_order, tx, ty);
    const uint32_t lx = tx * kTileW + (threadIdx.x % kTileW);
    const uint32_t ly = ty * kTileH + (threadIdx.x / kTileW);
    Counters cnt = {};
    phase_start(cnt);
    bool overflow = false;
    if (lx < W && ly < rows) {
        if constexpr (SK == 0) {
            uint64_t mem[kPrivateStack];
            PrivateStack<kPrivateStack> stk;
            stk.mem = (priv_u64_ptr)mem;
            shade_pixel<COUNT, DIAG, PAIRS, SINGLE, REUSE>(sd, mats, spheres, draws, tri_records, image, wire, wire_ch, W, H, rm, wm, lx, ly, stk,
                                            cnt, overflow);
        } else {
            __shared__ uint64_t s_stack[kLdsStack * 64];
            uint64_t spill[kSpillStack];
            LdsStack<kLdsStack, kSpillStack> stk;
            stk.base = (lds_u64_ptr)(s_stack + (threadIdx.x & 63u));
            stk.spill = (priv_u64_ptr)spill;
            shade_pixel<COUNT, DIAG, PAIRS, SINGLE, REUSE>(sd, mats, spheres, draws, tri_records, image, wire, wire_ch, W, H, rm, wm, lx, ly, stk,
                                            cnt, overflow);
        }
    }
    if (overflow) atomicOr(status, 1u);
    flush_counters<COUNT>(cnt, counters);
    if (!COUNT && tile_cost && (threadIdx.x & 63u) == 0u) {
        /* this tile's time, for the next renders' order: a running average (each frame draws new bounce directions,
         * the primary rays repeat), halved into the previous value */
        uint32_t* const tc = tile_cost + ty * tilesX + tx;
        const uint64_t c = (__builtin_amdgcn_s_memtime() - c0) >> 1;
        *tc = (*tc >> 1) + (c > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)c);
    }
#if WCPT_MK_TIMERS
    if (!COUNT && (threadIdx.x & 63u) == 0u)
        for (int k = 0; k < kPhaseTimers; k++) atomicAdd(&counters[k], (unsigned long long)cnt.tim[k]);
#endif
}

/* Derived triangle records (pt_device.h), single and pair formats: one thread per pair. Same subtractions as
 * rayTriangle (:122-123). The second slot of the last pair of an odd count is NaN (never inside a leaf's range:
 * leaf_record bounds leaves by the triangle count). A vertex index past the vertex buffer gives NaN vertices. */
__device__ __forceinline__ void tri_fields(const uint32_t* __restrict__ idx, const float* __restrict__ vtx, uint32_t nvert,
                                           uint64_t k, float f[9])
{
    const uint32_t ia = idx[3ull * k + 0], ib = idx[3ull * k + 1], ic = idx[3ull * k + 2];
    const float qnan = __uint_as_float(0x7fc00000u);
    const f3 nan3 = mk3(qnan, qnan, qnan);
    const f3 a = ia < nvert ? ld3(vtx + 3ull * ia) : nan3;
    const f3 b = ib < nvert ? ld3(vtx + 3ull * ib) : nan3;
    const f3 c = ic < nvert ? ld3(vtx + 3ull * ic) : nan3;
    const f3 e1 = b - a, e2 = c - a;
    f[0] = a.x; f[1] = a.y; f[2] = a.z;
    f[3] = e1.x; f[4] = e1.y; f[5] = e1.z;
    f[6] = e2.x; f[7] = e2.y; f[8] = e2.z;
}

/* The BVH's leaves against the fast layout's assumptions: *flags |= 1 when some leaf has triangleCount >= kRefFetch (a
 * stack entry of it would not carry its count), |= 2 when some leaf does not start at a triangle boundary or reaches
 * past the draw's derived records (first % 3 != 0 or first + count > lim3 = 3 * triangles: its triangles would need
 * the index path). */
__global__ __launch_bounds__(256) void scan_leaf_counts(const wcpt_node* __restrict__ bvh, uint32_t nodes, uint32_t lim3,
                                                        uint32_t* __restrict__ flags)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= nodes) return;
    const uint32_t first = bvh[i].leftNodeOrTriangleIndex, count = bvh[i].triangleCount;
    if (count == 0u) return;
    uint32_t f = count >= kRefFetch ? 1u : 0u;
    if (first % 3u != 0u || first > lim3 || count > lim3 - first) f |= 2u;
    if (f) atomicOr(flags, f);
}

__global__ __launch_bounds__(256) void build_tri_records(const uint32_t* __restrict__ idx, const float* __restrict__ vtx,
                                                         uint32_t ntri, uint32_t nvert, float4* __restrict__ singles,
                                                         float4* __restrict__ out)
{
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (2ull * j >= ntri) return;
    float v[2][9];
    for (uint32_t h = 0; h < 2; h++) {
        const uint64_t k = 2ull * j + h;
        if (k >= ntri) {
            for (int c = 0; c < 9; c++) v[h][c] = __uint_as_float(0x7fc00000u);
            continue;
        }
        tri_fields(idx, vtx, nvert, k, v[h]);
        const f3 e1 = mk3(v[h][3], v[h][4], v[h][5]), e2 = mk3(v[h][6], v[h][7], v[h][8]);
        const f3 n = normalize(cross(e1, e2)); /* :173 */
        singles[3ull * k + 0] = make_float4(v[h][0], v[h][1], v[h][2], v[h][3]);
        singles[3ull * k + 1] = make_float4(v[h][4], v[h][5], v[h][6], v[h][7]);
        singles[3ull * k + 2] = make_float4(v[h][8], n.x, n.y, n.z);
    }
    float4* o = out + (uint64_t)kPairRecordFloat4s * j;
    o[0] = make_float4(v[0][0], v[1][0], v[0][1], v[1][1]);
    o[1] = make_float4(v[0][2], v[1][2], v[0][3], v[1][3]);
    o[2] = make_float4(v[0][4], v[1][4], v[0][5], v[1][5]);
    o[3] = make_float4(v[0][6], v[1][6], v[0][7], v[1][7]);
    o[4] = make_float4(v[0][8], v[1][8], 0.0f, 0.0f);
}

/* Primary-ray pair records from pair records (one thread per pair): the origin terms of both triangles with
 * primary_terms, the same operations as rayTrianglePair's for that origin. */
__global__ __launch_bounds__(256) void build_primary_pairs(const float4* __restrict__ pairs, uint32_t npairs, float ox,
                                                           float oy, float oz, float4* __restrict__ out)
{
    const uint32_t j = blockIdx.x * 256u + threadIdx.x;
    if (j >= npairs) return;
    const float4* q = pairs + (uint64_t)kPairRecordFloat4s * j;
    const float4 r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
    /* pair record: (ax, ay) (az, e1x) (e1y, e1z) (e2x, e2y) (e2z, pad) as {tri 2j, tri 2j+1} float2 */
    const float ax[2] = {r0.x, r0.y}, ay[2] = {r0.z, r0.w}, az[2] = {r1.x, r1.y}, e1x[2] = {r1.z, r1.w};
    const float e1y[2] = {r2.x, r2.y}, e1z[2] = {r2.z, r2.w}, e2x[2] = {r3.x, r3.y}, e2y[2] = {r3.z, r3.w};
    const float e2z[2] = {r4.x, r4.y};
    float t[2][7];
    for (int h = 0; h < 2; h++)
        primary_terms(ox, oy, oz, ax[h], ay[h], az[h], e1x[h], e1y[h], e1z[h], e2x[h], e2y[h], e2z[h], t[h]);
    float4* o = out + (uint64_t)kPrimPairFloat4s * j;
    o[0] = make_float4(e1x[0], e1x[1], e1y[0], e1y[1]);
    o[1] = make_float4(e1z[0], e1z[1], e2x[0], e2x[1]);
    o[2] = make_float4(e2y[0], e2y[1], e2z[0], e2z[1]);
    o[3] = make_float4(t[0][0], t[1][0], t[0][1], t[1][1]); /* oax, oay */
    o[4] = make_float4(t[0][2], t[1][2], t[0][3], t[1][3]); /* oaz, qx */
    o[5] = make_float4(t[0][4], t[1][4], t[0][5], t[1][5]); /* qy, qz */
    o[6] = make_float4(t[0][6], t[1][6], 0.0f, 0.0f);       /* tq */
}

/* Device self-tests: evaluate the device definitions of the RNG and the deterministic libm on host inputs. */
__global__ __launch_bounds__(256) void pt_selftest(int fn, const uint32_t* __restrict__ in, const uint32_t* __restrict__ in2,
                                                   uint32_t* __restrict__ out, uint32_t n)
{
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint32_t a = in[i];
    switch (fn) {
    case 0: out[i] = pcg_hash(a); break;
    case 1: {
        uint32_t s = a;
        for (int k = 0; k < 4; k++) out[4u * i + (uint32_t)k] = __float_as_uint(rand_f(s));
        break;
    }
    case 2: out[i] = __float_as_uint(wcpt_logf(__uint_as_float(a))); break;
    case 3: out[i] = __float_as_uint(wcpt_cosf(__uint_as_float(a))); break;
    case 4: out[i] = __float_as_uint(wcpt_expf(__uint_as_float(a))); break;
    case 5: out[i] = __float_as_uint(sqrt_exact(__uint_as_float(a))); break;
    case 6: out[i] = __float_as_uint(__uint_as_float(a) / __uint_as_float(in2[i])); break;
    case 8: { /* exhaustive fast-reciprocal check: mismatches of rcp_exact's fast path vs IEEE 1/x over the 2^16
                 inputs (a << 16) | k inside the fast path's range */
        uint32_t bad = 0;
        for (uint32_t k = 0; k < 65536u; k++) {
            const float x = __uint_as_float((a << 16) | k);
            const float ax = fabsf(x);
            if (!(ax >= 0x1p-126f && ax < 0x1p126f)) continue;
            const float y = __builtin_amdgcn_rcpf(x);
            const float e = __builtin_fmaf(-x, y, 1.0f);
            const float r = __builtin_fmaf(e, y, y);
            bad += (__float_as_uint(r) != __float_as_uint(1.0f / x)) ? 1u : 0u;
        }
        out[i] = bad;
        break;
    }
    case 9: out[i] = __float_as_uint(rcp_exact(__uint_as_float(a))); break;
    case 10:   /* as 8, over every normal binary32 input (v_cmp_class range test) */
    case 11: { /* as 8, over every input (no range test) */
        uint32_t bad = 0;
        for (uint32_t k = 0; k < 65536u; k++) {
            const float x = __uint_as_float((a << 16) | k);
            if (fn == 10 && !__builtin_isnormal(x)) continue;
            const float y = __builtin_amdgcn_rcpf(x);
            const float e = __builtin_fmaf(-x, y, 1.0f);
            const float r = __builtin_fmaf(e, y, y);
            const float q = 1.0f / x;
            bad += (__float_as_uint(r) != __float_as_uint(q) && !(r != r && q != q)) ? 1u : 0u;
        }
        out[i] = bad;
        break;
    }
    case 12: { /* the kernels' reciprocals vs the IEEE quotient over the 2^16 inputs x = (a << 16) | k: rcp_exact(x), and
                  rcp2_exact on the pair (x, ~x) (every bit pattern in both halves); mismatches, NaN == NaN */
        uint32_t bad = 0;
        for (uint32_t k = 0; k < 65536u; k++) {
            const uint32_t bits = (a << 16) | k;
            const float x = __uint_as_float(bits), x2 = __uint_as_float(~bits);
            const float r = rcp_exact(x);
            v2f xx;
            xx.x = x;
            xx.y = x2;
            const v2f rr = rcp2_exact(xx);
            const float q = 1.0f / x, q2 = 1.0f / x2;
            bad += (__float_as_uint(r) != __float_as_uint(q) && !(r != r && q != q)) ? 1u : 0u;
            bad += (__float_as_uint(rr.x) != __float_as_uint(q) && !(rr.x != rr.x && q != q)) ? 1u : 0u;
            bad += (__float_as_uint(rr.y) != __float_as_uint(q2) && !(rr.y != rr.y && q2 != q2)) ? 1u : 0u;
        }
        out[i] = bad;
        break;
    }
    case 13: { /* how many of the 2^16 inputs (a << 16) | k fail the fast result's class check (general division) */
        uint32_t slow = 0;
        for (uint32_t k = 0; k < 65536u; k++)
            slow += rcp_fast_ok(rcp_fast_raw(__uint_as_float((a << 16) | k))) ? 0u : 1u;
        out[i] = slow;
        break;
    }
    case 14: { /* acceptance tests on (u, v) = (in, in2) with t = 1: bit 0 = accept_tri, bit 1 = accept_tri_w */
        const float u = __uint_as_float(a), v = __uint_as_float(in2[i]);
        const float uv = u + v;
        out[i] = (accept_tri(1.0f, u, v, uv) ? 1u : 0u) | (accept_tri_w(1.0f, u, v, 1.0f - uv) ? 2u : 0u);
        break;
    }
    case 15: { /* the kernels' sqrt (sqrt_exact) vs hipcc's correctly rounded sqrtf over the 2^16 inputs (a << 16) | k:
                  mismatches, NaN == NaN */
        uint32_t bad = 0;
        for (uint32_t k = 0; k < 65536u; k++) {
            const float x = __uint_as_float((a << 16) | k);
            const float r = sqrt_exact(x), q = sqrtf(x);
            bad += (__float_as_uint(r) != __float_as_uint(q) && !(r != r && q != q)) ? 1u : 0u;
        }
        out[i] = bad;
        break;
    }
    case 17: { /* the take's two forms (pt_device.h take_bits) over t = (a << 16) | k, k < 2^16, for rec.t = in2: mismatches
                  between (t > 0 && t < rec.t) and bits(t) - 1 < bits(rec.t) - 1 */
        const float rt = __uint_as_float(in2[i]);
        const uint32_t rb = take_bits(rt);
        uint32_t bad = 0;
        for (uint32_t k = 0; k < 65536u; k++) {
            const float t = __uint_as_float((a << 16) | k);
            bad += ((t > 0.0f && t < rt) != (take_bits(t) < rb)) ? 1u : 0u;
        }
        out[i] = bad;
        break;
    }
    case 16: { /* GLSL vector / scalar as the kernels evaluate it (pt_device.h operator/): in * RN(1 / in2) */
        const f3 q = mk3(__uint_as_float(a), 0.0f, 0.0f) / __uint_as_float(in2[i]);
        out[i] = __float_as_uint(q.x);
        break;
    }
    case 7: { /* RandomDirection: 3 words per input */
        uint32_t s = a;
        const f3 d = RandomDirection(s);
        out[3u * i + 0u] = __float_as_uint(d.x);
        out[3u * i + 1u] = __float_as_uint(d.y);
        out[3u * i + 2u] = __float_as_uint(d.z);
        break;
    }
    default: break;
    }
}

} // namespace dev

/* ------------------------------------------------------------------------------------------------ */
hipError_t launch_build_tri_records(const uint32_t* indices, const float* vertices, uint32_t triangles,
                                    uint32_t vertex_count, void* singles, void* pairs, hipStream_t stream)
{
    if (triangles == 0) return hipSuccess;
    const uint32_t npairs = (uint32_t)((triangles + 1ull) / 2ull);
    hipLaunchKernelGGL(dev::build_tri_records, dim3((npairs + 255u) / 256u), dim3(256), 0, stream, indices, vertices,
                       triangles, vertex_count, static_cast<float4*>(singles), static_cast<float4*>(pairs));
    return hipGetLastError();
}

hipError_t launch_scan_leaf_counts(const void* bvh, uint32_t nodes, uint32_t triangles, uint32_t* flags,
                                   hipStream_t stream)
{
    hipError_t e = hipMemsetAsync(flags, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess || nodes == 0) return e;
    hipLaunchKernelGGL(dev::scan_leaf_counts, dim3((nodes + 255u) / 256u), dim3(256), 0, stream,
                       static_cast<const wcpt_node*>(bvh), nodes, 3u * triangles, flags);
    return hipGetLastError();
}

static_assert(dev::kPrimPairRecordBytes == kPrimPairRecordBytes, "primary-ray pair record size");
static_assert(dev::kPairRecordBytes == kPairRecordBytes, "pair record size");
hipError_t launch_build_primary_pairs(const void* pairs, uint32_t npairs, float ox, float oy, float oz, void* out,
                                      hipStream_t stream)
{
    if (npairs == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::build_primary_pairs, dim3((npairs + 255u) / 256u), dim3(256), 0, stream,
                       static_cast<const float4*>(pairs), npairs, ox, oy, oz, static_cast<float4*>(out));
    return hipGetLastError();
}

/* list / grid: a frame-overlap pipe's share of the cost-ordered tiles (MkState::split); null: every tile, in the order
 * below */
template <bool COUNT, bool DIAG, int SK, bool PAIRS, bool SINGLE, bool REUSE = false>
static hipError_t launch_mega(const LaunchArgs& a, MkState& mk, hipStream_t stream, uint32_t tilesX, uint32_t tiles,
                              const uint32_t* list, uint32_t grid)
{
    /* scattered tile order: block b renders tile (b * m) mod tiles for an m coprime with tiles near 0.618 * tiles,
     * so the tiles resident on one CU at once come from all over the frame */
    /* 3, 4, 5, 6: striped XCD bands of 1, 2, 4, 8 tile rows (tile_of_block: even scatter = 2 x stripe height);
     * 2 (auto, default): scattered for a launch of about one round of resident waves (below), else stripes of one tile
     * row. Measured (round 3, 10 frames x 4 interleaved rounds): the reference's Init scene 1.91 ms (bands) -> 1.48 ms
     * (stripes of 1; 2 / 4 / 8 rows: 1.50 / 1.69 / 1.98 ms; scattered 1.52), the atrium on the megakernel 12.15 ->
     * 11.24 ms; the Cornell box 0.379 -> 0.382 ms (its tiles cost alike, so bands only keep neighbours together) */
    uint32_t scatter = a.mk_tile_order >= 3 ? (2u << (a.mk_tile_order - 3)) : (a.mk_tile_order == 2 ? 2u : 0u);
    const bool one_round = (uint64_t)tiles <= 16ull * (uint64_t)mk.cus; /* <= ~4 resident waves per SIMD */
    if ((a.mk_tile_order == 1 || (a.mk_tile_order == 2 && one_round)) && tiles > 2) {
        uint32_t m = (uint32_t)((uint64_t)tiles * 618034u / 1000000u) | 1u;
        auto gcd = [](uint32_t x, uint32_t y) { while (y) { const uint32_t r = x % y; x = y; y = r; } return x; };
        while (gcd(m, tiles) != 1u) m += 2u;
        scatter = m;
    }
    /* cost-ordered tiles (auto order, render launches): this render records every tile's time, and the renders after
     * a sort (launch_megakernel) take the tiles longest first */
    const bool cost_order = !COUNT && a.mk_tile_order == 2 && mk.cost != nullptr;
    const uint32_t* order = list ? list : (cost_order && mk.order_valid ? mk.order : nullptr);
    hipLaunchKernelGGL((dev::pt_megakernel<COUNT, DIAG, SK, PAIRS, SINGLE, REUSE>), dim3(list ? grid : tiles), dim3(64), 0,
                       stream, a.sd, a.materials, a.spheres, a.draws, a.tri_records, a.image, a.wire, a.wire_ch, a.W, a.H,
                       RowMap{a.y0, a.row_shift, a.row_gap}, a.wire_rows, a.rows, tilesX, tiles, scatter, order,
                       cost_order ? mk.cost : nullptr, a.status, a.counters);
    return hipGetLastError();
}

__global__ void fill_iota(uint32_t* __restrict__ v, uint32_t n)
{
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) v[i] = i;
}

__global__ void split_tiles(const uint32_t* __restrict__ order, uint32_t n, uint32_t* __restrict__ out)
{
    const uint32_t half = (n + 1u) / 2u;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        out[(i & 1u) ? half + (i >> 1) : (i >> 1)] = order[i];
}

/* the caller has synchronised the context's stream after mk_join */
void mk_release(MkState& mk)
{
    for (uint32_t p = 0; p < kMkPipes; p++) {
        if (mk.pipe[p]) (void)hipStreamDestroy(mk.pipe[p]);
        if (mk.join[p]) (void)hipEventDestroy(mk.join[p]);
    }
    if (mk.fork) (void)hipEventDestroy(mk.fork);
    if (mk.mem) (void)hipFree(mk.mem);
    const int cus = mk.cus;
    mk = MkState{};
    mk.cus = cus;
}

/* Longest-first tile order from the costs the renders record (tile time in shader cycles). Measured (round 3,
 * tools/tile_trace.py, 20 frames x 4 interleaved rounds): tile times vary with a coefficient of variation of 0.5-0.66
 * across a frame and repeat from frame to frame for a still camera (the same primary rays); starting the longest
 * tiles first leaves the short ones to fill the launch's last round: the Cornell box 0.3863 -> 0.3761 ms, its
 * 270-row block 0.1251 -> 0.1209 ms, the reference's scene 1.486 -> 1.284 ms. Sorted after the first render of a
 * geometry, after its 4th and 16th and then every kResortEvery renders (a radix sort of one key per tile, ~tens of
 * microseconds). */
constexpr uint32_t kResortEvery = 64;
static hipError_t cost_order_prepare(const LaunchArgs& a, MkState& mk, uint32_t tiles, hipStream_t stream)
{
    if (tiles > mk.cap) {
        if (mk.mem) {
            hipError_t e = hipStreamSynchronize(stream);
            if (e != hipSuccess) return e;
            (void)hipFree(mk.mem);
            mk.mem = nullptr;
            mk.cap = 0;
        }
        size_t temp = 0;
        hipError_t e = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, temp, (const uint32_t*)nullptr,
                                                                    (uint32_t*)nullptr, (const uint32_t*)nullptr,
                                                                    (uint32_t*)nullptr, (int)tiles, 0, 32, stream);
        if (e != hipSuccess) return e;
        const size_t words = 5ull * tiles;
        const size_t bytes = ((words * 4ull + 255ull) & ~255ull) + temp;
        void* m = nullptr;
        e = hipMalloc(&m, bytes);
        if (e != hipSuccess) return e;
        mk.mem = m;
        uint32_t* u = static_cast<uint32_t*>(m);
        mk.cost = u;
        mk.keys = u + tiles;
        mk.iota = u + 2ull * tiles;
        mk.order = u + 3ull * tiles;
        mk.split = u + 4ull * tiles;
        mk.temp = static_cast<char*>(m) + ((words * 4ull + 255ull) & ~255ull);
        mk.temp_bytes = temp;
        mk.cap = tiles;
        mk.geom_tiles = 0; /* forces the reset below */
    }
    if (mk.geom_tiles != tiles || mk.geom_w != a.W || mk.geom_rows != a.rows || mk.geom_y0 != a.y0 ||
        mk.geom_shift != a.row_shift || mk.geom_gap != a.row_gap) {
        mk.geom_tiles = tiles;
        mk.geom_w = a.W;
        mk.geom_rows = a.rows;
        mk.geom_y0 = a.y0;
        mk.geom_shift = a.row_shift;
        mk.geom_gap = a.row_gap;
        mk.renders = 0;
        mk.order_valid = false;
        mk.split_valid = false;
        return hipMemsetAsync(mk.cost, 0, (size_t)tiles * 4u, stream); /* the running averages start at 0 */
    }
    return hipSuccess;
}

static hipError_t cost_order_sort(MkState& mk, uint32_t tiles, hipStream_t stream)
{
    hipLaunchKernelGGL(fill_iota, dim3(std::min<uint32_t>((tiles + 255u) / 256u, 1024u)), dim3(256), 0, stream,
                       mk.iota, tiles);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    size_t temp = mk.temp_bytes;
    e = hipcub::DeviceRadixSort::SortPairsDescending(mk.temp, temp, mk.cost, mk.keys, mk.iota, mk.order, (int)tiles, 0,
                                                     32, stream);
    if (e != hipSuccess) return e;
    mk.order_valid = true;
    /* the frame-overlap pipes' tile lists: the order's even positions, then its odd ones (each list longest first) */
    hipLaunchKernelGGL(split_tiles, dim3(std::min<uint32_t>((tiles + 255u) / 256u, 1024u)), dim3(256), 0, stream,
                       mk.order, tiles, mk.split);
    e = hipGetLastError();
    mk.split_valid = e == hipSuccess;
    return e;
}

template <bool PAIRS, bool SINGLE>
static hipError_t launch_mega_sk(const LaunchArgs& a, int mode, int stack_kind, MkState& mk, hipStream_t stream,
                                 uint32_t tilesX, uint32_t tiles, const uint32_t* list = nullptr, uint32_t grid = 0)
{
    if (stack_kind == 0) {
        if (mode == kModeRender)
            return a.sd.samples > 1u && WCPT_MK_PRIMARY_REUSE
                       ? launch_mega<false, false, 0, PAIRS, SINGLE, true>(a, mk, stream, tilesX, tiles, list, grid)
                       : launch_mega<false, false, 0, PAIRS, SINGLE>(a, mk, stream, tilesX, tiles, list, grid);
        if (mode == kModeCount) return launch_mega<true, false, 0, PAIRS, SINGLE>(a, mk, stream, tilesX, tiles, list, grid);
        return launch_mega<true, true, 0, PAIRS, SINGLE>(a, mk, stream, tilesX, tiles, list, grid);
    }
    if (mode == kModeRender)
        return a.sd.samples > 1u && WCPT_MK_PRIMARY_REUSE
                   ? launch_mega<false, false, 1, PAIRS, SINGLE, true>(a, mk, stream, tilesX, tiles, list, grid)
                   : launch_mega<false, false, 1, PAIRS, SINGLE>(a, mk, stream, tilesX, tiles, list, grid);
    if (mode == kModeCount) return launch_mega<true, false, 1, PAIRS, SINGLE>(a, mk, stream, tilesX, tiles, list, grid);
    return launch_mega<true, true, 1, PAIRS, SINGLE>(a, mk, stream, tilesX, tiles, list, grid);
}

hipError_t mk_join(MkState& mk, hipStream_t stream)
{
    if (!mk.pending) return hipSuccess;
    mk.pending = false;
    hipError_t first = hipSuccess;
    for (uint32_t p = 1; p < kMkPipes; p++) { /* pipe 0 is the context's stream itself */
        hipError_t e = hipEventRecord(mk.join[p], mk.pipe[p]);
        if (e == hipSuccess) e = hipStreamWaitEvent(stream, mk.join[p], 0);
        if (e != hipSuccess && first == hipSuccess) first = e;
    }
    return first;
}

/* Frame overlap: a launch leaves its last round of waves with fewer and fewer tiles (the cost order puts the shortest
 * last) and the next frame's launch on the same stream cannot start before the last one ends -- the in-order queue
 * sets each dispatch's barrier bit, and gfx9 has no any-order launch (hip_ext.h). Two contexts rendering the Cornell
 * box round-robin finish 5.0 % more frames than one (0.3441 against 0.3614 ms, tools/stream_overlap.py,
 * profiles/r06_stream_overlap.log): that tail, overlapped by the other stream's work. Here one context does it with
 * two pipes: each takes half the cost-ordered tiles (every other position of the order, so both halves cost alike),
 * pipe 0 on the context's stream and pipe 1 on a stream of its own (one stream more per context: a one-rank group's
 * communication stream still fits the device's four hardware queues), and a pipe's next frame queues behind its own
 * previous frame only. A pixel belongs to the
 * same pipe in every frame while the order stands, so its frames accumulate in order; a re-sort, a new geometry,
 * another kernel or any other entry point first joins both pipes into the context's stream (mk_join). Auto: from 1.5
 * rounds of resident waves up (c2 4-way blocks, 2 rounds: 0.1168 -> 0.0916 ms, 2-way 0.1976 -> 0.1759 ms; an 8-way block
 * is one round, and there the overlap measured +0.9 %; profiles/r06_block_overlap.log). */
constexpr uint32_t kMkOverlapMinTilesPerCu = 24;

hipError_t launch_megakernel(const LaunchArgs& a, int mode, int stack_kind, MkState& mk, hipStream_t stream, int overlap)
{
    const uint32_t tilesX = (a.W + dev::kTileW - 1u) / dev::kTileW;
    const uint32_t tilesY = (a.rows + dev::kTileH - 1u) / dev::kTileH;
    const uint32_t tiles = tilesX * tilesY;
    if (mk.cus == 0) { /* CU count of the context's device, cached per context */
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e == hipSuccess) e = hipDeviceGetAttribute(&mk.cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (e != hipSuccess) return e;
    }
    const bool cost_order = mode == kModeRender && a.mk_tile_order == 2;
    const bool same_geometry = mk.geom_tiles == tiles && mk.geom_w == a.W && mk.geom_rows == a.rows &&
                               mk.geom_y0 == a.y0 && mk.geom_shift == a.row_shift && mk.geom_gap == a.row_gap;
    const bool pipes = overlap != 0 && cost_order && same_geometry && mk.order_valid && mk.split_valid && tiles >= 2u &&
                       (overlap == 2 || (uint64_t)tiles >= (uint64_t)kMkOverlapMinTilesPerCu * (uint64_t)mk.cus);
    hipError_t e = hipSuccess;
    if (mk.pending && !(pipes && mk.pending_tiles == tiles)) {
        e = mk_join(mk, stream);
        if (e != hipSuccess) return e;
    }
    if (tiles == 0) return hipSuccess;
    if (cost_order) {
        e = cost_order_prepare(a, mk, tiles, stream);
        if (e != hipSuccess) return e;
    }
    /* one draw command (the reference's case): the single-draw instantiation, without the draw loop */
    const bool single = a.sd.drawCommandCount == 1u;
    auto launch = [&](const LaunchArgs& la, hipStream_t s, const uint32_t* list, uint32_t grid) {
        if (la.pair_records)
            return single ? launch_mega_sk<true, true>(la, mode, stack_kind, mk, s, tilesX, tiles, list, grid)
                          : launch_mega_sk<true, false>(la, mode, stack_kind, mk, s, tilesX, tiles, list, grid);
        return single ? launch_mega_sk<false, true>(la, mode, stack_kind, mk, s, tilesX, tiles, list, grid)
                      : launch_mega_sk<false, false>(la, mode, stack_kind, mk, s, tilesX, tiles, list, grid);
    };
    if (pipes) {
        if (!mk.pending) { /* fork: pipe 1 after everything queued on the context's stream */
            for (uint32_t p = 1; p < kMkPipes && e == hipSuccess; p++) {
                if (!mk.pipe[p]) e = hipStreamCreateWithFlags(&mk.pipe[p], hipStreamNonBlocking);
                if (e == hipSuccess && !mk.join[p]) e = hipEventCreateWithFlags(&mk.join[p], hipEventDisableTiming);
            }
            if (e == hipSuccess && !mk.fork) e = hipEventCreateWithFlags(&mk.fork, hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventRecord(mk.fork, stream);
            for (uint32_t p = 1; p < kMkPipes && e == hipSuccess; p++) e = hipStreamWaitEvent(mk.pipe[p], mk.fork, 0);
            if (e != hipSuccess) return e;
        }
        const uint32_t half = (tiles + 1u) / 2u;
        e = launch(a, stream, mk.split, half);
        /* pending from the first enqueue on: a failed second launch still leaves the first to join */
        mk.pending = true;
        mk.pending_tiles = tiles;
        if (e == hipSuccess && a.pipe1_prepare) e = a.pipe1_prepare(a.pipe1_user, mk.pipe[1]);
        if (e == hipSuccess) {
            LaunchArgs a1 = a;
            if (a.tri_records_pipe1) a1.tri_records = a.tri_records_pipe1;
            e = launch(a1, mk.pipe[1], mk.split + half, tiles - half);
        }
    } else {
        e = launch(a, stream, nullptr, 0);
    }
    if (e != hipSuccess || !cost_order) return e;
    /* sorted after renders 1, 4 and 16 of a geometry (the running averages settle), then every kResortEvery; the sort
     * rewrites the order the pipes read, so they are joined first and the next render forks after it */
    const uint32_t r = ++mk.renders;
    if (r == 1u || r == 4u || r == 16u || r % kResortEvery == 0u) {
        e = mk_join(mk, stream);
        if (e != hipSuccess) return e;
        return cost_order_sort(mk, tiles, stream);
    }
    return hipSuccess;
}

hipError_t launch_selftest(int fn, const uint32_t* in, const uint32_t* in2, uint32_t* out, uint32_t n, hipStream_t stream)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(dev::pt_selftest, dim3((n + 255u) / 256u), dim3(256), 0, stream, fn, in, in2, out, n);
    return hipGetLastError();
}

} // namespace wcpt
