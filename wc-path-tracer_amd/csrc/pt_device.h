/*
 * pt_device.h — device-side building blocks of the path tracer (gfx950).
 *
 * Semantics follow src/shaders/pathTracer.comp and src/shaders/include/Random.glsl of the reference
 * exactly (cited per function). Every expression keeps the reference's operand order and is compiled
 * with -ffp-contract=off, so that the image is bit-identical to oracle/pt_oracle.c on the same inputs.
 *
 * Layout-level differences from the reference (results unchanged):
 *   - SceneData is a kernel argument (scalar loads from the kernarg segment) instead of a BDA buffer.
 *   - BVH traversal keeps the nearer child in registers and pushes only the farther one, with the box
 *     entry distance t0 on the stack. A child whose box test fails statically (t0 > t1 || t1 < 0) is never
 *     pushed; the dynamic cull (t0 > rt) is applied when the child would have been popped. This is
 *     exactly the reference's pop order and cull set (pathTracer.comp:157-200) with one 64-byte sibling
 *     fetch per interior node instead of 32 (pop) + 64 (children) bytes.
 */
#ifndef WCPT_PT_DEVICE_H
#define WCPT_PT_DEVICE_H

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/wcpt.h"
#include "row_map.h"
#include "wcpt_composite.h"
#include "wcpt_libm.h"

namespace wcpt {
namespace dev {

/* Scene buffers are reached through device addresses stored in DrawCommands (buffer device addresses in the
 * reference, pathTracer.comp:82-88). Casting them to address-space-1 (global) pointers makes hipcc emit
 * global_load_* instead of flat_load_*: flat loads count against lgkmcnt as well as vmcnt, so every LDS
 * stack access would otherwise also wait for outstanding node fetches. */
#define WCPT_GLOBAL __attribute__((address_space(1)))
typedef const WCPT_GLOBAL wcpt_node* gnode_ptr;
typedef const WCPT_GLOBAL uint32_t* gu32_ptr;
typedef const WCPT_GLOBAL float* gf32_ptr;
__device__ __forceinline__ gnode_ptr as_nodes(uint64_t a) { return (gnode_ptr)(uintptr_t)a; }
__device__ __forceinline__ gu32_ptr as_u32(uint64_t a) { return (gu32_ptr)(uintptr_t)a; }
__device__ __forceinline__ gf32_ptr as_f32(uint64_t a) { return (gf32_ptr)(uintptr_t)a; }

/* constants.glsl:4-9 */
constexpr float kBias = 1e-5f;
constexpr float kInfinity = 3.402823466e+38f;
constexpr float kPI = 3.14159265358979323846264338327950288f;

struct f3 { float x, y, z; };

__device__ __forceinline__ f3 mk3(float x, float y, float z) { f3 r; r.x = x; r.y = y; r.z = z; return r; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, f3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
/* Correctly rounded reciprocal 1/x: v_rcp_f32 followed by one FMA Newton step, with the general division for the
 * inputs where that fast sequence is not the IEEE quotient. 3 VALU + 1 check instead of the 11 of hipcc's
 * division sequence.
 *
 * The fast sequence equals 1.0f / x for every |x| in [2^-126, 2^126) (all 2^32 bit patterns checked on gfx950:
 * tools/rcp_exhaustive.hip and selftest fn 8/10). Outside that range it returns zero (|x| >= 2^126: the denormal
 * quotient is flushed) or NaN (x zero, denormal, infinite or NaN), never a normal number. So the fast result is
 * validated on its own class (one v_cmp_class): a normal result is the IEEE quotient, anything else takes the
 * general division. Checked over all 2^32 inputs: selftest fn 12 (0 mismatches), which also runs the packed pair
 * form rcp2_exact. WCPT_RCP_RANGE=1 selects the older input-range test (two compares). */
#ifndef WCPT_RCP_RANGE
#define WCPT_RCP_RANGE 0
#endif
__device__ __forceinline__ float rcp_fast_raw(float x)
{
    const float y = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, y, 1.0f);
    return __builtin_fmaf(e, y, y);
}
__device__ __forceinline__ bool rcp_fast_ok(float r) { return __builtin_isnormal(r); }
__device__ __forceinline__ float rcp_exact(float x)
{
#if WCPT_RCP_RANGE
    const float a = fabsf(x);
    if (__builtin_expect(a >= 0x1p-126f && a < 0x1p126f, 1)) return rcp_fast_raw(x);
    return 1.0f / x;
#else
    const float r = rcp_fast_raw(x);
    if (__builtin_expect(rcp_fast_ok(r), 1)) return r;
    return 1.0f / x;
#endif
}
typedef float v2f __attribute__((ext_vector_type(2)));
/* rcp_exact of both halves: two v_rcp_f32, the Newton step as two packed FMAs (v_pk_fma_f32: two independent
 * binary32 fused multiply-adds, the same operations as the scalar step) and one branch for both fallbacks. */
__device__ __forceinline__ v2f rcp2_exact(v2f x)
{
#if WCPT_RCP_RANGE
    v2f r;
    r.x = rcp_exact(x.x);
    r.y = rcp_exact(x.y);
    return r;
#else
    v2f y;
    y.x = __builtin_amdgcn_rcpf(x.x);
    y.y = __builtin_amdgcn_rcpf(x.y);
    const v2f one = {1.0f, 1.0f};
    const v2f e = __builtin_elementwise_fma(-x, y, one);
    v2f r = __builtin_elementwise_fma(e, y, y);
    const bool okx = rcp_fast_ok(r.x), oky = rcp_fast_ok(r.y);
    if (__builtin_expect(!(okx && oky), 0)) {
        if (!okx) r.x = 1.0f / x.x;
        if (!oky) r.y = 1.0f / x.y;
    }
    return r;
#endif
}
__device__ __forceinline__ f3 rcp3(f3 a) { return mk3(rcp_exact(a.x), rcp_exact(a.y), rcp_exact(a.z)); }
/* GLSL vector / scalar (normalize, the sphere normal :145, target.xyz / target.w :301, result / samples :312):
 * v * RN(1/s) with the correctly rounded reciprocal, one reciprocal and three multiplies instead of three
 * correctly rounded divisions. Vulkan allows 2.5 ULP for GLSL division; this is <= 1.5 ULP, and the oracle
 * defines vector / scalar the same way (oracle/pt_oracle.c div3s), so the two stay bit-identical. */
__device__ __forceinline__ f3 operator/(f3 a, float s)
{
    const float r = rcp_exact(s);
    return mk3(a.x * r, a.y * r, a.z * r);
}
/* GLSL dot: (x*x' + y*y') + z*z' */
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* GLSL cross (4.50 spec §8.5) */
__device__ __forceinline__ f3 cross(f3 a, f3 b)
{
    return mk3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
/* Correctly rounded sqrt. hipcc's sqrtf is v_sqrt_f32 (not correctly rounded alone) + a one-ulp correction from two
 * FMA residuals, wrapped in a 2^32 scaling for inputs below 2^-96 and a zero/infinity class fixup: 17 VALU. For
 * x >= 2^-96 (including +inf) the correction alone is the IEEE square root -- checked against sqrtf over every such
 * input on the device (selftest fn 15) -- so that range takes the 9-VALU core and everything else (tiny, zero,
 * negative, NaN) the full sequence. WCPT_SQRT_CORE=0 uses sqrtf everywhere. */
#ifndef WCPT_SQRT_CORE
#define WCPT_SQRT_CORE 1
#endif
__device__ __forceinline__ float sqrt_core(float x)
{
    const float s = __builtin_amdgcn_sqrtf(x);
    const float s_dn = __uint_as_float(__float_as_uint(s) - 1u);
    const float s_up = __uint_as_float(__float_as_uint(s) + 1u);
    const float r_dn = __builtin_fmaf(-s_dn, s, x);
    const float r_up = __builtin_fmaf(-s_up, s, x);
    float r = (r_dn <= 0.0f) ? s_dn : s;
    r = (r_up > 0.0f) ? s_up : r;
    return r;
}
__device__ __forceinline__ float sqrt_exact(float x)
{
#if WCPT_SQRT_CORE
    if (__builtin_expect(x >= 0x1p-96f, 1)) return sqrt_core(x);
#endif
    return sqrtf(x);
}
__device__ __forceinline__ f3 normalize(f3 v) { return v / sqrt_exact(dot(v, v)); }
__device__ __forceinline__ f3 reflect(f3 I, f3 N) { return I - N * (2.0f * dot(N, I)); }
__device__ __forceinline__ f3 refract(f3 I, f3 N, float eta)
{
    const float d = dot(N, I);
    const float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return mk3(0.0f, 0.0f, 0.0f);
    return eta * I - N * (eta * d + sqrt_exact(k));
}
__device__ __forceinline__ float sign1(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
__device__ __forceinline__ f3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }
__device__ __forceinline__ f3 ld3(gf32_ptr p) { return mk3(p[0], p[1], p[2]); } /* global_load_dwordx3 */
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

/* ---- Random.glsl:10-56 ------------------------------------------------------------------------- */
__device__ __forceinline__ uint32_t pcg_hash(uint32_t seed)
{
    const uint32_t state = seed * 747796405u + 2891336453u;
    const uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
/* rand_pcg's output word is the PCG permutation of the *current* state (Random.glsl:18-24); rand() then
 * overwrites the state with that output (Random.glsl:29-30), discarding the LCG step of :21. */
__device__ __forceinline__ uint32_t pcg_permute(uint32_t state)
{
    const uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}
__device__ __forceinline__ float rand_f(uint32_t& state)
{
    const uint32_t x = pcg_permute(state);
    state = x;
    return (float)x * 2.3283064365386963e-10f; /* uintBitsToFloat(0x2f800000u) = 2^-32 */
}

__device__ __forceinline__ float RandomValueNormalDistribution(uint32_t& seed)
{
    const float theta = 2.0f * kPI * rand_f(seed);
    const float rho = sqrt_exact(-2.0f * wcpt_logf_rand(rand_f(seed))); /* == wcpt_logf on rand()'s values */
    return rho * wcpt_cosf_2pi(theta);                              /* == wcpt_cosf on [0, 2*pi] */
}
/* wcpt_libm.h's wcpt_logf_rand and wcpt_cosf_2pi on two arguments at once: the same binary32 operations in the same
 * order per half, with the float arithmetic on packed FP32 instructions (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32
 * for the reciprocal's Newton step) and the integer and rounding steps per half. Bit-identical to the scalar
 * functions (and so to the oracle) by construction; selftest fn 7 checks RandomDirection against the oracle. */
#ifndef WCPT_RANDDIR_PAIRS
#define WCPT_RANDDIR_PAIRS 1
#endif
__device__ __forceinline__ v2f bcast2(float s) { v2f r = {s, s}; return r; }
__device__ __forceinline__ v2f logf_rand2(v2f x)
{
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f;
    const float Lg1 = 0.66666662693f, Lg2 = 0.40000972152f, Lg3 = 0.28498786688f, Lg4 = 0.24279078841f;
    uint32_t ix0 = __float_as_uint(x.x) + (0x3f800000u - 0x3f3504f3u);
    uint32_t ix1 = __float_as_uint(x.y) + (0x3f800000u - 0x3f3504f3u);
    const int k0 = (int)(ix0 >> 23) - 127, k1 = (int)(ix1 >> 23) - 127;
    ix0 = (ix0 & 0x007fffffu) + 0x3f3504f3u;
    ix1 = (ix1 & 0x007fffffu) + 0x3f3504f3u;
    const v2f m = {__uint_as_float(ix0), __uint_as_float(ix1)};
    const v2f f = m - bcast2(1.0f);
    const v2f den = bcast2(2.0f) + f;
    v2f y;
    y.x = __builtin_amdgcn_rcpf(den.x);
    y.y = __builtin_amdgcn_rcpf(den.y);
    const v2f e = __builtin_elementwise_fma(-den, y, bcast2(1.0f));
    const v2f rc = __builtin_elementwise_fma(e, y, y); /* wcpt_rcp1_2 per half */
    const v2f sv = f * rc;
    const v2f z = sv * sv;
    const v2f w = z * z;
    const v2f t1 = w * (bcast2(Lg2) + w * bcast2(Lg4));
    const v2f t2 = z * (bcast2(Lg1) + w * bcast2(Lg3));
    const v2f R = t2 + t1;
    const v2f hfsq = bcast2(0.5f) * f * f;
    const v2f dk = {(float)k0, (float)k1};
    v2f out = sv * (hfsq + R) + dk * bcast2(ln2_lo) - hfsq + f + dk * bcast2(ln2_hi);
    if (x.x == 0.0f) out.x = __uint_as_float(0xff800000u);
    if (x.y == 0.0f) out.y = __uint_as_float(0xff800000u);
    return out;
}
__device__ __forceinline__ float cos_quadrant(int j, float c, float s)
{
    switch (j & 3) {
    case 0: return c;
    case 1: return -s;
    case 2: return -c;
    default: return s;
    }
}
__device__ __forceinline__ v2f cosf_2pi2(v2f ax)
{
    const float two_over_pi = 0.63661977236758134f;
    const float pio2_1 = 1.5703125f, pio2_2 = 4.837512969970703125e-4f, pio2_3 = 7.5497899548e-8f;
    const float S1 = -1.6666654611e-1f, S2 = 8.3321608736e-3f, S3 = -1.9515295891e-4f;
    const float C1 = 4.166664568298827e-2f, C2 = -1.388731625493765e-3f, C3 = 2.443315711809948e-5f;
    const v2f q = ax * bcast2(two_over_pi) + bcast2(0.5f);
    const v2f jf = {floorf(q.x), floorf(q.y)};
    const int j0 = (int)jf.x, j1 = (int)jf.y;
    const v2f r = ((ax - jf * bcast2(pio2_1)) - jf * bcast2(pio2_2)) - jf * bcast2(pio2_3);
    const v2f z = r * r;
    v2f c = ((bcast2(C3) * z + bcast2(C2)) * z + bcast2(C1)) * z * z;
    c = c - bcast2(0.5f) * z;
    c = c + bcast2(1.0f);
    v2f sn = ((bcast2(S3) * z + bcast2(S2)) * z + bcast2(S1)) * z * r;
    sn = sn + r;
    v2f out;
    out.x = cos_quadrant(j0, c.x, sn.x);
    out.y = cos_quadrant(j1, c.y, sn.y);
    return out;
}
__device__ __forceinline__ f3 RandomDirection(uint32_t& seed)
{
#if WCPT_RANDDIR_PAIRS
    /* Random.glsl:43-56 with the draws in the reference order: theta_x, rho_x, theta_y, rho_y, theta_z, rho_z */
    const float ux0 = rand_f(seed), ux1 = rand_f(seed);
    const float uy0 = rand_f(seed), uy1 = rand_f(seed);
    const v2f theta = bcast2(2.0f * kPI) * (v2f){ux0, uy0};
    const v2f lg = logf_rand2((v2f){ux1, uy1});
    const v2f m2 = bcast2(-2.0f) * lg;
    const v2f rho = {sqrt_exact(m2.x), sqrt_exact(m2.y)};
    const v2f xy = rho * cosf_2pi2(theta);
    const float z = RandomValueNormalDistribution(seed);
    return normalize(mk3(xy.x, xy.y, z));
#else
    const float x = RandomValueNormalDistribution(seed);
    const float y = RandomValueNormalDistribution(seed);
    const float z = RandomValueNormalDistribution(seed);
    return normalize(mk3(x, y, z));
#endif
}

/* ---- pathTracer.comp:24-28, 50-58 ------------------------------------------------------------- */
struct Ray { f3 origin, direction, invDirection; };
struct Hit { f3 p, normal; float t; uint32_t material; bool hit, front; };

/* pathTracer.comp:97-108 — slab test; min/max are IEEE minNum/maxNum (v_min_f32 / v_max_f32). */
__device__ __forceinline__ void rayBox(const Ray& r, float mnx_, float mny_, float mnz_, float mxx_, float mxy_,
                                       float mxz_, float& t0, float& t1)
{
    const float bx = (mnx_ - r.origin.x) * r.invDirection.x;
    const float by = (mny_ - r.origin.y) * r.invDirection.y;
    const float bz = (mnz_ - r.origin.z) * r.invDirection.z;
    const float tx = (mxx_ - r.origin.x) * r.invDirection.x;
    const float ty = (mxy_ - r.origin.y) * r.invDirection.y;
    const float tz = (mxz_ - r.origin.z) * r.invDirection.z;
    const float mnx = fminf(tx, bx), mny = fminf(ty, by), mnz = fminf(tz, bz);
    const float mxx = fmaxf(tx, bx), mxy = fmaxf(ty, by), mxz = fmaxf(tz, bz);
    t0 = fmaxf(fmaxf(mnx, mny), fmaxf(mnx, mnz));
    t1 = fminf(fminf(mxx, mxy), fminf(mxx, mxz));
}

/* A BVH node (32 B) as two 16-byte loads: {min.xyz, max.x}, {max.yz, left, count}. */
struct NodeV { v4f a; v4u b; };
__device__ __forceinline__ NodeV load_node(gnode_ptr bvh, uint32_t i)
{
    const WCPT_GLOBAL v4f* p = reinterpret_cast<const WCPT_GLOBAL v4f*>(bvh + i);
    NodeV n;
    n.a = p[0];
    n.b = reinterpret_cast<const WCPT_GLOBAL v4u*>(p)[1];
    return n;
}
/* The child pair (left, left + 1) of an interior node through a buffer resource over the BVH (draws whose BVH is a
 * known context buffer of < 2^24 nodes: table word 2's high half holds the node count): the four loads take one VGPR
 * byte offset (buffer_load_dwordx4 v_off, s[rsrc] offen offset:0/16/32/48) instead of two 64-bit lane addresses
 * (v_lshlrev_b64 + v_lshl_add_u64 each), and an index past the buffer reads a zero node instead of other memory.
 * Same bytes for every node in the buffer. */
constexpr int kBufferDword3 = 0x00020000; /* gfx9 raw buffer resource word 3 (composable_kernel's value for gfx9) */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t node_rsrc(gnode_ptr bvh, uint32_t nodes)
{
    return __builtin_amdgcn_make_buffer_rsrc((void*)bvh, (short)0, (int)(nodes * 32u), kBufferDword3);
}
__device__ __forceinline__ void load_pair_rsrc(__amdgpu_buffer_rsrc_t r, uint32_t left, NodeV& L, NodeV& R)
{
    const int off = (int)(left << 5);
    L.a = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    L.b = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0));
    R.a = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(r, off + 32, 0, 0));
    R.b = __builtin_bit_cast(v4u, __builtin_amdgcn_raw_buffer_load_b128(r, off + 48, 0, 0));
}
/* (leftNodeOrTriangleIndex, triangleCount) of node i: bytes 24..31 */
__device__ __forceinline__ uint2 load_node_lc(gnode_ptr bvh, uint32_t i)
{
    const v2u v = reinterpret_cast<const WCPT_GLOBAL v2u*>(bvh + i)[3];
    return make_uint2(v.x, v.y);
}
/* Stack entry node references. Packed form (draws whose BVH has < 2^24 nodes and whose index count is < 2^24,
 * table flag kTriFlagPackedRefs): the deferred child's own (left, count) as (left << 8) | count when count < 255,
 * so that popping it needs no node fetch -- the pop path then has no dependent memory round trip; otherwise
 * (node index << 8) | 255 and the node's (left, count) is fetched at pop. Unpacked form: the node index. */
constexpr uint32_t kRefFetch = 255u;
__device__ __forceinline__ uint32_t node_ref(bool packed, uint32_t node_index, uint32_t left, uint32_t count)
{
    if (!packed) return node_index;
    return (count < kRefFetch && left < (1u << 24)) ? (left << 8) | count : (node_index << 8) | kRefFetch;
}
__device__ __forceinline__ uint2 node_ref_lc(bool packed, gnode_ptr bvh, uint32_t ref)
{
    if (!packed) return load_node_lc(bvh, ref);
    if ((ref & 255u) != kRefFetch) return make_uint2(ref >> 8, ref & 255u);
    return load_node_lc(bvh, ref >> 8);
}
/* The packed forms when every index and count fits (the wavefront fast layout: < 2^24 nodes and index positions,
 * every triangleCount < kRefFetch, kTriFlagSmallLeaves): no fetch case */
__device__ __forceinline__ uint32_t node_ref_small(uint32_t left, uint32_t count) { return (left << 8) | count; }
__device__ __forceinline__ uint2 node_ref_lc_small(uint32_t ref) { return make_uint2(ref >> 8, ref & 255u); }
__device__ __forceinline__ void node_box(const Ray& r, const NodeV& n, float& t0, float& t1)
{
    /* node = {min.xyz, max.x | max.yz, left, count} */
    rayBox(r, n.a.x, n.a.y, n.a.z, n.a.w, __uint_as_float(n.b.x), __uint_as_float(n.b.y), t0, t1);
}

/* pathTracer.comp:110-119, near root only (:141) */
__device__ __forceinline__ float raySphereNear(const Ray& r, f3 position, float radius)
{
    const f3 oc = r.origin - position;
    const float b = dot(oc, r.direction);
    const float c = dot(oc, oc) - radius * radius;
    const float t = b * b - c;
    if (t < 0.0f) return -1.0f;
    return -b - sqrt_exact(t);
}

/* The sphere loop of Intersect (pathTracer.comp:140-149) over spheres [0, count): the near root of each, accepted
 * iff 0 < t < rec.t, in sphere order. WCPT_SPHERE_PAIRS=1 (default) evaluates two spheres per step with packed
 * FP32 (v_pk_mul_f32 / v_pk_add_f32: per half exactly raySphereNear's binary32 operations), the square roots and
 * the ordered takes per sphere. */
constexpr uint32_t kNoPrim = 0xFFFFFFFFu, kSpherePrim = 0x80000000u;
#ifndef WCPT_SPHERE_PAIRS
#define WCPT_SPHERE_PAIRS 1
#endif
#ifndef WCPT_SPHERE_BSKIP
#define WCPT_SPHERE_BSKIP 1
#endif
__device__ __forceinline__ void sphere_loop(const Ray& r, uint32_t count, const wcpt_sphere* __restrict__ spheres,
                                            float& rt, uint32_t& prim)
{
    uint32_t i = 0;
#if WCPT_SPHERE_PAIRS
    const v2f ox = {r.origin.x, r.origin.x}, oy = {r.origin.y, r.origin.y}, oz = {r.origin.z, r.origin.z};
    const v2f dx = {r.direction.x, r.direction.x}, dy = {r.direction.y, r.direction.y},
                dz = {r.direction.z, r.direction.z};
    for (; i + 1u < count; i += 2u) {
        const wcpt_sphere& s0 = spheres[i];
        const wcpt_sphere& s1 = spheres[i + 1u];
        const v2f cx = {s0.position[0], s1.position[0]}, cy = {s0.position[1], s1.position[1]},
                    cz = {s0.position[2], s1.position[2]}, rad = {s0.radius, s1.radius};
        const v2f ocx = ox - cx, ocy = oy - cy, ocz = oz - cz;     /* oc = origin - position */
        const v2f b = (ocx * dx + ocy * dy) + ocz * dz;           /* dot(oc, d) */
        const v2f c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - rad * rad;
        const v2f t = b * b - c;
#if WCPT_SPHERE_BSKIP
        /* b >= 0 (the centre is not ahead of the origin) gives -b - sqrt(t) <= 0 exactly, so RN of it is <= 0 and the
         * `t0 > 0` test below fails either way: the square root is skipped (NaN b still takes the full path) */
        const float t0 = (t.x < 0.0f || b.x >= 0.0f) ? -1.0f : -b.x - sqrt_exact(t.x);
        const float t1 = (t.y < 0.0f || b.y >= 0.0f) ? -1.0f : -b.y - sqrt_exact(t.y);
#else
        const float t0 = t.x < 0.0f ? -1.0f : -b.x - sqrt_exact(t.x);
        const float t1 = t.y < 0.0f ? -1.0f : -b.y - sqrt_exact(t.y);
#endif
        if (t0 > 0.0f && t0 < rt) { rt = t0; prim = kSpherePrim | i; }
        if (t1 > 0.0f && t1 < rt) { rt = t1; prim = kSpherePrim | (i + 1u); }
    }
#endif
    for (; i < count; i++) {
        const wcpt_sphere& s = spheres[i];
        const float tempRec = raySphereNear(r, mk3(s.position[0], s.position[1], s.position[2]), s.radius);
        if (tempRec > 0.0f && tempRec < rt) {
            rt = tempRec;
            prim = kSpherePrim | i;
        }
    }
}

/* The acceptance test of :132 without its `u <= 1` term, which the other terms imply: with v >= 0, u + v >= u
 * exactly, so the rounded sum RN(u + v) >= RN(u) = u (rounding is monotonic), and u + v <= 1 then gives u <= 1.
 * A NaN u or v fails `u >= 0` / `v >= 0` either way, and u = +inf fails `u + v <= 1`. Same decision, one
 * compare less per triangle. */
__device__ __forceinline__ bool accept_tri(float t, float u, float v, float uv)
{
    return t > 0.0f && u >= 0.0f && v >= 0.0f && uv <= 1.0f;
}

/* The same decision with one compare for u, v and u + v: t > 0 && minimum3(u, v, 1 - (u + v)) >= 0, where minimum3
 * is v_minimum3_f32 (IEEE 754-2019 minimum: NaN-propagating, -0 < +0). Equivalence: a NaN u or v makes u + v and
 * 1 - (u + v) NaN, so the minimum is NaN and the test fails, as `u >= 0` / `v >= 0` does; u = +inf with v = -inf
 * fails both ways (v < 0, and the NaN sum). For non-NaN values minimum3 >= 0 is u >= 0 && v >= 0 && w >= 0 (-0 counts
 * as >= 0 in both), and w = RN(1 - uv) >= 0 exactly when uv <= 1: uv <= 1 makes 1 - uv >= 0, whose rounding stays
 * >= 0; uv > 1 means uv >= 1 + 2^-23, so 1 - uv <= -2^-23 rounds to a negative number; uv = -inf gives +inf and
 * passes as `uv <= 1` does. The device self-test fn 14 compares both forms on special and random operands. The
 * pair test forms w for both triangles with one packed subtraction: 4.5 VALU per triangle instead of 5. */
#ifndef WCPT_ACCEPT_MIN3
#define WCPT_ACCEPT_MIN3 1
#endif
__device__ __forceinline__ float minimum3(float a, float b, float c)
{
    return __builtin_elementwise_minimum(__builtin_elementwise_minimum(a, b), c);
}
__device__ __forceinline__ bool accept_tri_w(float t, float u, float v, float w)
{
    return t > 0.0f && minimum3(u, v, w) >= 0.0f;
}

/* Integer form of the take (WCPT_PAIR_ITAKE). The reference takes an accepted triangle iff t > 0 (:132) and t < rec.t
 * (:171). For rec.t a positive float (kInfinity at most, or an earlier accepted t > 0; never NaN), the two compares
 * are one unsigned compare of bit patterns minus one: bits(t) - 1 < bits(rec.t) - 1. Positive floats (denormals
 * included: IEEE compares them as nonzero) order like their bit patterns; t = +0 gives 0 - 1 = 0xFFFFFFFF, which is
 * never below; a negative t or -0 has the sign bit, so bits - 1 >= 0x7FFFFFFF > bits(rec.t) - 1 <= 0x7F7FFFFF;
 * a NaN t (positive 0x7F800001.. or negative) lies above every finite or infinite rec.t the same way. So the pair loop
 * carries rec.t as rb = bits(rec.t) - 1, takes with one v_add_u32 and one v_cmp_u32 per triangle instead of two float
 * compares and their mask AND, and converts back at the end of the leaf. The acceptance keeps its minimum3 >= 0 test
 * (which must pass -0 and reject NaN). Device check: selftest fn 17 compares both forms on all 2^32 t against a set of
 * rec.t values (tests/test_gpu_parity.py). Measured (round 5, 6 interleaved rounds on two boxes,
 * profiles/r05_itake_ab.log): c2 kernel 0.3635 against 0.3651 ms (-0.4 %), the reference's scene +0.3 %; the same
 * form confined to the uniform loop gained less on c2 (-0.15 %). */
#ifndef WCPT_PAIR_ITAKE
#define WCPT_PAIR_ITAKE 1
#endif
__device__ __forceinline__ uint32_t take_bits(float t) { return __float_as_uint(t) - 1u; }
__device__ __forceinline__ bool accept_uvw(float u, float v, float w) { return minimum3(u, v, w) >= 0.0f; }

/* pathTracer.comp:121-133 with the two edges given: e1 = b - a, e2 = c - a (:122-123); returns t or -1 */
__device__ __forceinline__ float rayTriangleE(const Ray& r, f3 a, f3 edgeAB, f3 edgeAC)
{
    const f3 oa = r.origin - a;
    const f3 crossRDE2 = cross(r.direction, edgeAC);
    const float inv = rcp_exact(dot(edgeAB, crossRDE2));
    const f3 crossROAE1 = cross(oa, edgeAB);
    const float u = dot(oa, crossRDE2) * inv;
    const float v = dot(r.direction, crossROAE1 * inv);
    const float t = dot(edgeAC, crossROAE1) * inv;
    return accept_tri(t, u, v, u + v) ? t : -1.0f;
}
__device__ __forceinline__ float rayTriangle(const Ray& r, f3 a, f3 b, f3 c) { return rayTriangleE(r, a, b - a, c - a); }

/* Derived triangle records. For each draw command the runtime derives from the draw's index and vertex buffers,
 * triangle k = index positions 3k..3k+2, with e1 = b - a and e2 = c - a computed by the same binary32
 * subtractions as :122-123, two record arrays:
 *   single records, 48 B per triangle: (a.xyz, e1.x) (e1.yz, e2.xy) (e2.z, n.xyz), where n = normalize(cross(e1,
 *     e2)) is the geometric normal of :173 evaluated once per triangle with the same operations (it depends on
 *     the triangle only), so the hit epilogue reads it instead of re-gathering three indices and vertices;
 *   pair records, 80 B per triangle pair (2j, 2j+1): the nine components of both triangles as float2
 *     {tri 2j, tri 2j+1} + 8 B pad. One lane then tests two triangles at once with packed-FP32 instructions
 *     (v_pk_mul_f32 / v_pk_add_f32 perform two independent binary32 ops each -- exactly the reference's ops),
 *     halving the VALU issue slots of the Möller-Trumbore arithmetic; the two results are applied in
 *     reference order (2j first, then 2j+1, strict <).
 * A leaf test reads aligned 16-byte loads instead of an index fetch plus three dependent vertex gathers, and
 * the edge subtractions leave the inner loop. Pairs pay off for fat leaves (the Cornell box: ~17 triangles per
 * leaf, VALU-bound); single records for thin leaves (the atrium: ~2 triangles per leaf, fetch-latency-bound).
 * The reference's BVH keeps each leaf's index triples contiguous (PathTracingRenderer.jai:233), so a leaf's
 * records are contiguous. A leaf whose first index position is not a multiple of 3 (never produced by the
 * reference's builder) or that reaches past the draw's indexCount uses the index path.
 * Per-draw table entry: {single record address, pair record address, triangle count, flags | vertex count << 32,
 * primary-ray pair record address or 0} (5 x u64). */
constexpr uint32_t kTriTableWords = 5;
constexpr uint64_t kTriFlagPackedRefs = 1u; /* table word 3: stack entries may carry (left, count) */
constexpr uint64_t kTriFlagIndex24 = 2u;    /* table word 3: the draw's indexCount is < 2^24 */
constexpr uint64_t kTriFlagSmallLeaves = 4u; /* table word 3: every node's triangleCount is < kRefFetch, so every packed
                                                stack entry carries its node's (left, count) */
constexpr uint64_t kTriFlagLeafRecords = 8u; /* table word 3: every leaf starts at a triangle boundary and ends within the
                                                draw's derived records, so each leaf triangle at index position p is
                                                single record p / 3 (byte offset 16 p) */
/* table word 3, bits 32..63: vertices in the draw's vertex buffer (0xFFFFFFFF: unknown, not a context buffer) */
__device__ __forceinline__ uint32_t draw_vertex_count(const uint64_t* __restrict__ tri_records, uint32_t draw)
{
    return (uint32_t)(tri_records[kTriTableWords * draw + 3u] >> 32);
}
typedef const WCPT_GLOBAL v4f* gtri_ptr;
struct TriE { f3 a, e1, e2; };
__device__ __forceinline__ TriE load_tri(gtri_ptr t, uint32_t k)
{
    const gtri_ptr q = t + 3ull * k;
    const v4f r0 = q[0], r1 = q[1], r2 = q[2];
    TriE e;
    e.a = mk3(r0.x, r0.y, r0.z);
    e.e1 = mk3(r0.w, r1.x, r1.y);
    e.e2 = mk3(r1.z, r1.w, r2.x);
    return e;
}
constexpr uint32_t kPairRecordFloat4s = 5;
struct TriPair { v2f ax, ay, az, e1x, e1y, e1z, e2x, e2y, e2z; };
__device__ __forceinline__ TriPair load_pair(gtri_ptr t, uint32_t j)
{
    const gtri_ptr q = t + (uint64_t)kPairRecordFloat4s * j;
    const v4f r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
    TriPair p;
    p.ax = r0.xy;  p.ay = r0.zw;
    p.az = r1.xy;  p.e1x = r1.zw;
    p.e1y = r2.xy; p.e1z = r2.zw;
    p.e2x = r3.xy; p.e2y = r3.zw;
    p.e2z = r4.xy;
    return p;
}
/* The pair record at byte offset `off` from the record base (pair j at off = 80 j). */
constexpr uint32_t kPairRecordBytes = 16u * kPairRecordFloat4s;
constexpr uint32_t kNoTag = 0xFFFFFFFFu;
#ifndef WCPT_PAIR_UNIFORM
#define WCPT_PAIR_UNIFORM 1
#endif
#ifndef WCPT_PAIR_SLOOP
#define WCPT_PAIR_SLOOP 1
#endif

__device__ __forceinline__ TriPair load_pair_at(const WCPT_GLOBAL char* base, uint32_t off)
{
    const gtri_ptr q = reinterpret_cast<gtri_ptr>(base + off);
    const v4f r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
    TriPair p;
    p.ax = r0.xy;  p.ay = r0.zw;
    p.az = r1.xy;  p.e1x = r1.zw;
    p.e1y = r2.xy; p.e1z = r2.zw;
    p.e2x = r3.xy; p.e2y = r3.zw;
    p.e2z = r4.xy;
    return p;
}
/* The same record through the constant address space (4): the records are read-only for the whole launch, and a
 * wave-uniform offset then lowers to scalar loads (s_load_dwordx16 / s_load_dwordx4 through the scalar cache) whose
 * values the packed-FP32 instructions read straight from SGPRs. */
typedef const __attribute__((address_space(4))) v4f* ctri_ptr;
__device__ __forceinline__ TriPair load_pair_const(const WCPT_GLOBAL char* base, uint32_t off)
{
    const ctri_ptr q = (ctri_ptr)(uintptr_t)(base + off);
    const v4f r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4];
    TriPair p;
    p.ax = r0.xy;  p.ay = r0.zw;
    p.az = r1.xy;  p.e1x = r1.zw;
    p.e1y = r2.xy; p.e1z = r2.zw;
    p.e2x = r3.xy; p.e2y = r3.zw;
    p.e2z = r4.xy;
    return p;
}
__device__ __forceinline__ v2f bc2(float s) { v2f r = {s, s}; return r; }
/* rayTriangleE for the two triangles of a pair: t for triangle 2j (.x) and 2j+1 (.y), and whether each passed
 * the reference's acceptance test (t > 0, u, v, u + v in range). A triangle is taken iff it passed and t < rec.t;
 * that equals the reference's `t != -1 && t < rec.t` on its -1-for-miss result (a pass implies t > 0). */
struct PairHit { v2f t; bool hit0, hit1; };
#ifndef WCPT_PAIR_PIN
#define WCPT_PAIR_PIN 1
#endif
__device__ __forceinline__ PairHit rayTrianglePair(const Ray& r, const TriPair& p)
{
    const v2f dx = bc2(r.direction.x), dy = bc2(r.direction.y), dz = bc2(r.direction.z);
    const v2f oax = bc2(r.origin.x) - p.ax, oay = bc2(r.origin.y) - p.ay, oaz = bc2(r.origin.z) - p.az;
    /* crossRDE2 = cross(d, e2) */
    const v2f px = dy * p.e2z - p.e2y * dz;
    const v2f py = dz * p.e2x - p.e2z * dx;
    const v2f pz = dx * p.e2y - p.e2x * dy;
    const v2f det = (p.e1x * px + p.e1y * py) + p.e1z * pz;
    /* crossROAE1 = cross(oa, e1) */
    const v2f qx = oay * p.e1z - p.e1y * oaz;
    const v2f qy = oaz * p.e1x - p.e1z * oax;
    const v2f qz = oax * p.e1y - p.e1x * oay;
    const v2f un = (oax * px + oay * py) + oaz * pz; /* dot(oa, crossRDE2) */
    const v2f tn = (p.e2x * qx + p.e2y * qy) + p.e2z * qz; /* dot(edgeAC, crossROAE1) */
#if WCPT_PAIR_PIN
    /* computed before the reciprocal: its fallback branch would otherwise split the block, and these independent
     * products would be sunk past it instead of filling the det -> rcp -> Newton chain's dependency stalls */
    asm volatile("" ::"v"(qx), "v"(qy), "v"(qz), "v"(un), "v"(tn));
#endif
    const v2f inv = rcp2_exact(det);
    const v2f u = un * inv;
    const v2f v = (dx * (qx * inv) + dy * (qy * inv)) + dz * (qz * inv);
    const v2f t = tn * inv;
    const v2f uv = u + v;
    PairHit h;
    h.t = t;
#if WCPT_PAIR_ITAKE
    /* t > 0 is part of the take's integer compare (take_bits) */
    const v2f w = bc2(1.0f) - uv;
    h.hit0 = accept_uvw(u.x, v.x, w.x);
    h.hit1 = accept_uvw(u.y, v.y, w.y);
#elif WCPT_ACCEPT_MIN3
    const v2f w = bc2(1.0f) - uv;
    h.hit0 = accept_tri_w(t.x, u.x, v.x, w.x);
    h.hit1 = accept_tri_w(t.y, u.y, v.y, w.y);
#else
    h.hit0 = accept_tri(t.x, u.x, v.x, uv.x);
    h.hit1 = accept_tri(t.y, u.y, v.y, uv.y);
#endif
    return h;
}
/* Primary-ray pair records. Every primary ray of a frame starts at the camera (pathTracer.comp:299-302, SceneData
 * position), so the terms of rayTrianglePair that depend only on the origin and the triangle -- oa = o - a, q =
 * cross(oa, e1) and the t numerator dot(e2, q) (:124-125, :127, :130) -- are the same for every primary ray. The
 * runtime derives them once per camera position (build_primary_pairs, the same binary32 operations in the same
 * order, so the values are bit-identical) and the first segment of each sample tests its leaves from these records:
 * 51 instead of 68 VALU per pair. 112 B per pair: (e1x, e1y) (e1z, e2x) (e2y, e2z) (oax, oay) (oaz, qx) (qy, qz)
 * (tq, pad), each a float2 {triangle 2j, 2j+1}. */
#ifndef WCPT_PRIMARY_PAIRS
#define WCPT_PRIMARY_PAIRS 1
#endif
constexpr uint32_t kPrimPairFloat4s = 7;
constexpr uint32_t kPrimPairRecordBytes = 16u * kPrimPairFloat4s;
struct TriPairP { v2f e1x, e1y, e1z, e2x, e2y, e2z, oax, oay, oaz, qx, qy, qz, tq; };
template <class P>
__device__ __forceinline__ TriPairP unpack_pairP(P q)
{
    const v4f r0 = q[0], r1 = q[1], r2 = q[2], r3 = q[3], r4 = q[4], r5 = q[5], r6 = q[6];
    TriPairP p;
    p.e1x = r0.xy; p.e1y = r0.zw;
    p.e1z = r1.xy; p.e2x = r1.zw;
    p.e2y = r2.xy; p.e2z = r2.zw;
    p.oax = r3.xy; p.oay = r3.zw;
    p.oaz = r4.xy; p.qx = r4.zw;
    p.qy = r5.xy;  p.qz = r5.zw;
    p.tq = r6.xy;
    return p;
}
__device__ __forceinline__ TriPairP load_pairP_at(const WCPT_GLOBAL char* base, uint32_t off)
{
    return unpack_pairP(reinterpret_cast<gtri_ptr>(base + off));
}
__device__ __forceinline__ TriPairP load_pairP_const(const WCPT_GLOBAL char* base, uint32_t off)
{
    return unpack_pairP((ctri_ptr)(uintptr_t)(base + off));
}
/* rayTrianglePair with the origin terms taken from the record: the remaining operations are rayTrianglePair's */
__device__ __forceinline__ PairHit rayTrianglePairP(const Ray& r, const TriPairP& p)
{
    const v2f dx = bc2(r.direction.x), dy = bc2(r.direction.y), dz = bc2(r.direction.z);
    const v2f px = dy * p.e2z - p.e2y * dz;
    const v2f py = dz * p.e2x - p.e2z * dx;
    const v2f pz = dx * p.e2y - p.e2x * dy;
    const v2f det = (p.e1x * px + p.e1y * py) + p.e1z * pz;
    const v2f inv = rcp2_exact(det);
    const v2f u = ((p.oax * px + p.oay * py) + p.oaz * pz) * inv;
    const v2f v = (dx * (p.qx * inv) + dy * (p.qy * inv)) + dz * (p.qz * inv);
    const v2f t = p.tq * inv;
    const v2f uv = u + v;
    PairHit h;
    h.t = t;
#if WCPT_PAIR_ITAKE
    /* t > 0 is part of the take's integer compare (take_bits) */
    const v2f w = bc2(1.0f) - uv;
    h.hit0 = accept_uvw(u.x, v.x, w.x);
    h.hit1 = accept_uvw(u.y, v.y, w.y);
#elif WCPT_ACCEPT_MIN3
    const v2f w = bc2(1.0f) - uv;
    h.hit0 = accept_tri_w(t.x, u.x, v.x, w.x);
    h.hit1 = accept_tri_w(t.y, u.y, v.y, w.y);
#else
    h.hit0 = accept_tri(t.x, u.x, v.x, uv.x);
    h.hit1 = accept_tri(t.y, u.y, v.y, uv.y);
#endif
    return h;
}
/* Exact sign pre-reject of a primary pair (WCPT_PRIM_SIGN_SKIP, VERDICT r05 item 3: execute fewer triangle tests).
 * The reference's t is RN(tn * RN(1 / det)) (:126, :130), and a take needs t > 0 (:132). The primary records hold tn
 * itself (tq, bit-identical to the test's), and det is the test's first result, so before the rest of the test: when
 * the sign bits of tq and det differ, t is negative, -0 (an underflow) or NaN (a NaN operand) -- never > 0 -- and when
 * det is +-0 or tq is +-0 with different signs the same holds (t = -inf, -0 or NaN). Such a triangle cannot be taken,
 * whatever rec.t is. A wave whose every lane has both triangles of a pair in that case skips the pair's remaining
 * operations (reciprocal, u, v, t, acceptance: 39 of its 53 VALU); a lane that may take either runs the whole test,
 * so every result is the reference's. On primary rays (all from the camera, directions within one 8x8 tile) the sign
 * of det -- which side of the triangle's plane the ray heads to -- is nearly uniform across a wave: on Cornell ~21 %
 * of the primary pair steps are skippable by the whole wave (tools/prereject_sim.py; under 3 % on bounce rays, whose
 * directions are random per lane, where the test therefore is not made). */
#ifndef WCPT_PRIM_SIGN_SKIP
#define WCPT_PRIM_SIGN_SKIP 1
#endif
#ifndef WCPT_PAIR_PREFETCH
#define WCPT_PAIR_PREFETCH 0
#endif
__device__ __forceinline__ v2f pairP_det(const Ray& r, const TriPairP& p, v2f& px, v2f& py, v2f& pz)
{
    const v2f dx = bc2(r.direction.x), dy = bc2(r.direction.y), dz = bc2(r.direction.z);
    px = dy * p.e2z - p.e2y * dz;
    py = dz * p.e2x - p.e2z * dx;
    pz = dx * p.e2y - p.e2x * dy;
    return (p.e1x * px + p.e1y * py) + p.e1z * pz;
}
/* the rest of rayTrianglePairP after det (the same operations in the same order) */
__device__ __forceinline__ PairHit pairP_finish(const Ray& r, const TriPairP& p, v2f px, v2f py, v2f pz, v2f det)
{
    const v2f dx = bc2(r.direction.x), dy = bc2(r.direction.y), dz = bc2(r.direction.z);
    const v2f inv = rcp2_exact(det);
    const v2f u = ((p.oax * px + p.oay * py) + p.oaz * pz) * inv;
    const v2f v = (dx * (p.qx * inv) + dy * (p.qy * inv)) + dz * (p.qz * inv);
    const v2f t = p.tq * inv;
    const v2f uv = u + v;
    PairHit h;
    h.t = t;
#if WCPT_PAIR_ITAKE
    const v2f w = bc2(1.0f) - uv;
    h.hit0 = accept_uvw(u.x, v.x, w.x);
    h.hit1 = accept_uvw(u.y, v.y, w.y);
#elif WCPT_ACCEPT_MIN3
    const v2f w = bc2(1.0f) - uv;
    h.hit0 = accept_tri_w(t.x, u.x, v.x, w.x);
    h.hit1 = accept_tri_w(t.y, u.y, v.y, w.y);
#else
    h.hit0 = accept_tri(t.x, u.x, v.x, uv.x);
    h.hit1 = accept_tri(t.y, u.y, v.y, uv.y);
#endif
    return h;
}
/* whether a lane may take either triangle of the pair: the sign bits of tq and det agree for at least one of them */
__device__ __forceinline__ bool pairP_may_take(const TriPairP& p, v2f det)
{
    return (int32_t)(__float_as_uint(det.x) ^ __float_as_uint(p.tq.x)) >= 0 ||
           (int32_t)(__float_as_uint(det.y) ^ __float_as_uint(p.tq.y)) >= 0;
}

/* The origin terms of one triangle (half h of pair record q) for origin o: build_primary_pairs */
__device__ __forceinline__ void primary_terms(float ox, float oy, float oz, float ax, float ay, float az, float e1x,
                                              float e1y, float e1z, float e2x, float e2y, float e2z, float out[7])
{
    const float oax = ox - ax, oay = oy - ay, oaz = oz - az;
    const float qx = oay * e1z - e1y * oaz;
    const float qy = oaz * e1x - e1z * oax;
    const float qz = oax * e1y - e1x * oay;
    out[0] = oax; out[1] = oay; out[2] = oaz;
    out[3] = qx;  out[4] = qy;  out[5] = qz;
    out[6] = (e2x * qx + e2y * qy) + e2z * qz;
}

/* Vertex i of a draw whose vertex buffer holds nvert vertices (table word 3, high half; 0xFFFFFFFF when the buffer
 * is not a context buffer): a vertex index past the buffer reads NaN instead of memory past it, so that triangle is
 * never accepted (every comparison with NaN fails) -- the same rule the derived records follow (tri_fields). */
__device__ __forceinline__ f3 ld_vertex(gf32_ptr vtx, uint32_t i, uint32_t nvert)
{
    if (__builtin_expect(i < nvert, 1)) return ld3(vtx + 3ull * i);
    const float qnan = __uint_as_float(0x7fc00000u);
    return mk3(qnan, qnan, qnan);
}
__device__ __forceinline__ TriE tri_from_indices(gu32_ptr idx, gf32_ptr vtx, uint32_t first, uint32_t nvert)
{
    const f3 a = ld_vertex(vtx, idx[first + 0], nvert);
    const f3 b = ld_vertex(vtx, idx[first + 1], nvert);
    const f3 c = ld_vertex(vtx, idx[first + 2], nvert);
    TriE e;
    e.a = a;
    e.e1 = b - a;
    e.e2 = c - a;
    return e;
}
/* Leaf cursor into the records: triangle index of the leaf's first triangle, or kNoRecord for a leaf that does not
 * start on a triangle boundary or is not fully covered by the draw's `ntri` records. The per-draw table entry
 * is {record address, ntri} (2 x u64). */
constexpr uint32_t kNoRecord = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t leaf_record(uint32_t first, uint32_t count, uint32_t ntri)
{
    const uint32_t k = first / 3u;
    return (k * 3u == first && (uint64_t)k + (count + 2u) / 3u <= ntri) ? k : kNoRecord;
}
/* The same validity as a byte offset into the single records (48 B per triangle = 16 B per index position, so the
 * leaf's first record is at 16 * first), without a division: for first < 2^24 (draws with kTriFlagIndex24),
 * first % 3 == 0 exactly when (first * 0xAAAAAB) mod 2^24 <= 0x555555 (0xAAAAAB is the inverse of 3 mod 2^24; checked
 * for every first < 2^24), one full-rate v_mul_u32_u24 instead of leaf_record's quarter-rate v_mul_hi_u32 pair.
 * The end test is leaf_record's k + ceil(count / 3) <= ntri for every count: with first = 3k and lim3 = 3 * ntri,
 * lim3 - first is a multiple of 3, and count <= M holds for a multiple M of 3 exactly when 3 * ceil(count / 3) <= M.
 * It is written as first <= lim3 && count <= lim3 - first, which cannot wrap; lim3 < 2^24 for these draws, so an
 * accepted first is < 2^24 and the 24-bit alignment test above is exact for it. */
/* v_mul_u32_u24 (full rate). __umul24 is not enough here: only the low 24 bits of its product are used, so the
 * optimizer drops its 24-bit operand masks and the backend then emits the quarter-rate v_mul_lo_u32 (seen in the ISA
 * of both kernels). */
#ifndef WCPT_MUL24_ASM
#define WCPT_MUL24_ASM 1
#endif
__device__ __forceinline__ uint32_t mul_u32_u24(uint32_t a, uint32_t b_uniform)
{
#if WCPT_MUL24_ASM
    uint32_t r;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(r) : "s"(b_uniform), "v"(a));
    return r;
#else
    return __umul24(a, b_uniform);
#endif
}
__device__ __forceinline__ uint32_t leaf_record_off24(uint32_t first, uint32_t count, uint32_t lim3)
{
    const bool aligned = (mul_u32_u24(first, 0xAAAAABu) & 0xFFFFFFu) <= 0x555555u;
    return (aligned && first <= lim3 && count <= lim3 - first) ? first * 16u : kNoRecord;
}
/* The single record of the triangle at index position `pos` (the reference reads indices pos..pos+2, :174-176) as a
 * byte offset, for kTriFlagIndex24 draws: record k = pos / 3 was derived from exactly those indices when pos is a
 * multiple of 3 and k < ntri (pos < lim3 = 3 * ntri); else kNoRecord (the index path). Per triangle, so a leaf's
 * cursor needs no record offset of its own. */
__device__ __forceinline__ uint32_t tri_record_off24(uint32_t pos, uint32_t lim3)
{
    const bool aligned = (mul_u32_u24(pos, 0xAAAAABu) & 0xFFFFFFu) <= 0x555555u;
    return (aligned && pos < lim3) ? pos * 16u : kNoRecord;
}
/* leaf_record as a byte offset for any draw (records beyond 4 GiB take the index path) */
__device__ __forceinline__ uint32_t leaf_record_off(uint32_t first, uint32_t count, uint32_t ntri)
{
    const uint32_t k = leaf_record(first, count, ntri);
    return (k != kNoRecord && k < (1u << 26)) ? k * 48u : kNoRecord;
}
/* Single records through a buffer resource of ntri records (48 B each; ntri < 2^24 / 3 for the draws that use it):
 * an offset past the records reads zeros (hardware range check), i.e. a = e1 = e2 = 0, whose det is 0 and whose test
 * never accepts (0 * inf = NaN fails every comparison) */
__device__ __forceinline__ __amdgpu_buffer_rsrc_t tri_rsrc(gtri_ptr t, uint32_t ntri)
{
    return __builtin_amdgcn_make_buffer_rsrc((void*)t, (short)0, (int)(ntri * 48u), kBufferDword3);
}
__device__ __forceinline__ TriE load_tri_rsrc(__amdgpu_buffer_rsrc_t r, uint32_t off)
{
    const v4f r0 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
    const v4f r1 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(r, off + 16, 0, 0));
    const v4f r2 = __builtin_bit_cast(v4f, __builtin_amdgcn_raw_buffer_load_b128(r, off + 32, 0, 0));
    TriE e;
    e.a = mk3(r0.x, r0.y, r0.z);
    e.e1 = mk3(r0.w, r1.x, r1.y);
    e.e2 = mk3(r1.z, r1.w, r2.x);
    return e;
}
__device__ __forceinline__ TriE load_tri_at(gtri_ptr t, uint32_t off)
{
    const gtri_ptr q = reinterpret_cast<gtri_ptr>(reinterpret_cast<const WCPT_GLOBAL char*>(t) + off);
    const v4f r0 = q[0], r1 = q[1], r2 = q[2];
    TriE e;
    e.a = mk3(r0.x, r0.y, r0.z);
    e.e1 = mk3(r0.w, r1.x, r1.y);
    e.e2 = mk3(r1.z, r1.w, r2.x);
    return e;
}

/* Megakernel phase timers (tools only: a library built with -DWCPT_MK_TIMERS=1, tools/mk_phases.py). Each wave
 * attributes the s_memtime ticks since its previous mark to the phase that just ended: 0 primary ray, 1 sphere
 * loop, 2 BVH interior steps + pops, 3 leaf triangle tests, 4 hit resolution, 5 shading, 6 accumulation/store.
 * Ticks include the time other waves of the SIMD issue in between: read the shares, not absolute costs. */
#ifndef WCPT_MK_TIMERS
#define WCPT_MK_TIMERS 0
#endif
constexpr int kPhaseTimers = 8;

/* Cost attribution (tools only, tools/ab_build.sh): WCPT_DUP_<part>=1 evaluates that part a second time on
 * laundered inputs and discards the result, so the A/B time difference is the part's cost. Never on by default. */
#ifndef WCPT_DUP_SPHERES
#define WCPT_DUP_SPHERES 0
#endif
#ifndef WCPT_DUP_RANDDIR
#define WCPT_DUP_RANDDIR 0
#endif
#ifndef WCPT_DUP_PAIR
#define WCPT_DUP_PAIR 0
#endif
#ifndef WCPT_DUP_BOX
#define WCPT_DUP_BOX 0
#endif
__device__ __forceinline__ float launder(float x) { asm volatile("" : "+v"(x)); return x; }
__device__ __forceinline__ uint32_t launder_u(uint32_t x) { asm volatile("" : "+v"(x)); return x; }
__device__ __forceinline__ void sink(float x) { asm volatile("" ::"v"(x)); }
__device__ __forceinline__ void sink_u(uint32_t x) { asm volatile("" ::"v"(x)); }

/* Per-lane work counters; reduced per wave and added to global u64 counters. */
struct Counters {
    uint32_t pixels, segments, sphere_tests, node_pops, interior_visits, triangle_tests, hits, draw_fetches;
    uint32_t wave_int, lane_int, wave_tri, lane_tri, wave_seg, lane_seg; /* SIMD-efficiency diagnostics */
    uint32_t ref_over;  /* segments whose reference stack (uint nodeStack[32], :151) is written past index 31 */
    uint32_t ref_max;   /* deepest reference stack (entries after a push), 0xFFFFFFFF when it could not be tracked */
    bool ref_seg;       /* the current segment overflowed the reference stack */
#if WCPT_MK_TIMERS
    uint64_t tim[kPhaseTimers], tprev;
#endif
};

/* The reference's traversal stack, tracked exactly in the counting builds.
 * pathTracer.comp pushes the root (:155) and, at every interior node that survives its box test, BOTH children
 * (:192-198), culling a child only when it is popped (:162). So while a node is visited, its stack index (the entries
 * below it) is the number of its ancestors whose second-popped child is still pending -- the ancestors where the walk
 * went into the first-popped ("near") child. The kernels push only far children that pass their box test, so this
 * index is kept as two path masks instead of a second stack: bit k of `near` = the ancestor at depth k was left
 * through its near child (its far child is still pending in the reference), bit k of `pushed` = that far child is on
 * this kernel's stack. An interior visit pushes at indices rs and rs + 1 with rs = popcount(near); rs >= 31 writes
 * nodeStack[32], out of bounds (undefined behaviour in the reference). A pop of this kernel's stack takes the far
 * child of the deepest `pushed` ancestor k; the reference pops (and culls) every pending entry above it first. */
struct RefStack {
    uint64_t nearm, pushed;
    uint32_t depth;
};
constexpr uint32_t kRefStackSize = 32u;  /* uint nodeStack[32] (pathTracer.comp:151) */
constexpr uint32_t kRefUnknown = 0xFFFFFFFFu;
template <bool COUNT>
__device__ __forceinline__ void ref_root(RefStack& r, Counters& cnt)
{
    if (!COUNT) return;
    r.nearm = 0;
    r.pushed = 0;
    r.depth = 0;
    if (cnt.ref_max < 1u) cnt.ref_max = 1u; /* the root push (:155) */
}
template <bool COUNT>
__device__ __forceinline__ void ref_interior(RefStack& r, bool pushed_far, Counters& cnt)
{
    if (!COUNT) return;
    const uint32_t rs = (uint32_t)__popcll(r.nearm);
    if (rs + 2u > kRefStackSize) cnt.ref_seg = true;
    if (r.depth < 64u) {
        if (cnt.ref_max != kRefUnknown && cnt.ref_max < rs + 2u) cnt.ref_max = rs + 2u;
        const uint64_t b = 1ull << r.depth;
        r.nearm |= b;
        if (pushed_far) r.pushed |= b;
    } else {
        cnt.ref_max = kRefUnknown; /* deeper than the masks: not tracked */
    }
    r.depth++;
}
template <bool COUNT>
__device__ __forceinline__ void ref_pop(RefStack& r)
{
    if (!COUNT || r.pushed == 0) return;
    const uint32_t k = 63u - (uint32_t)__clzll((long long)r.pushed);
    const uint64_t below = (1ull << k) - 1ull;
    r.nearm &= below;
    r.pushed &= below;
    r.depth = k + 1u;
}
template <bool COUNT>
__device__ __forceinline__ void ref_segment_end(Counters& cnt)
{
    if (!COUNT) return;
    if (cnt.ref_seg) cnt.ref_over++;
    cnt.ref_seg = false;
}

__device__ __forceinline__ void phase_start(Counters& c)
{
#if WCPT_MK_TIMERS
    for (int k = 0; k < kPhaseTimers; k++) c.tim[k] = 0;
    c.tprev = __builtin_amdgcn_s_memtime();
#else
    (void)c;
#endif
}
__device__ __forceinline__ void phase_mark(Counters& c, int k)
{
#if WCPT_MK_TIMERS
    const uint64_t t = __builtin_amdgcn_s_memtime();
    c.tim[k] += t - c.tprev;
    c.tprev = t;
#else
    (void)c;
    (void)k;
#endif
}

/* Diagnostic step counting (COUNT kernels only): every executing lane adds a lane-step, the lowest active
 * lane adds the wave-step. */
template <bool DIAG>
__device__ __forceinline__ void simd_step(uint32_t& wave, uint32_t& lane_steps)
{
    if (!DIAG) return;
    const unsigned long long m = __ballot(1);
    lane_steps++;
    if ((threadIdx.x & 63u) == (uint32_t)(__ffsll((long long)m) - 1)) wave++;
}

template <bool COUNT, bool DIAG>
__device__ __forceinline__ void count_tri(Counters& cnt)
{
    if (COUNT) {
        cnt.triangle_tests++;
        simd_step<DIAG>(cnt.wave_tri, cnt.lane_tri);
    }
}

/* Traversal stacks; entries = (node index, box entry distance t0) of deferred far children.
 *
 * PrivateStack keeps the entries in private (scratch) memory: simple, but every push/pop is a VMEM store/load
 * that the per-XCD L2 cannot hold at full occupancy (measured: ~6 GB of writes per 1080p atrium frame).
 * LdsStack keeps the first N entries in LDS, lane-interleaved ([entry][64 lanes] of 8-byte words: one
 * conflict-free ds_write_b64 / ds_read_b64 per wave), and only entries N..N+SPILL-1 in scratch. */
/* The entry storage is a separate private array owned by the caller (`mem` / `spill` point at it) so that the
 * stack pointer itself stays in a register: with the arrays inside the struct, the dynamic array indexing kept
 * the whole struct -- sp included -- in scratch, and every push/pop paid a scratch round trip for sp. */
typedef __attribute__((address_space(5))) uint64_t* priv_u64_ptr;
typedef __attribute__((address_space(3))) uint64_t* lds_u64_ptr;

template <int N>
struct PrivateStack {
    priv_u64_ptr mem; /* caller's private uint64_t[N], entries (node index | t0 bits << 32) */
    int sp;
    __device__ __forceinline__ void reset() { sp = 0; }
    __device__ __forceinline__ bool empty() const { return sp == 0; }
    __device__ __forceinline__ bool push(uint32_t i, float t)
    {
        if (sp >= N) return false;
        mem[sp] = (uint64_t)i | ((uint64_t)__float_as_uint(t) << 32);
        sp++;
        return true;
    }
    __device__ __forceinline__ void pop(uint32_t& i, float& t)
    {
        sp--;
        const uint64_t e = mem[sp];
        i = (uint32_t)e;
        t = __uint_as_float((uint32_t)(e >> 32));
    }
};

#ifndef WCPT_STACK_UNIFORM_FAST
#define WCPT_STACK_UNIFORM_FAST 0
#endif
/* Spill wait in the pop's spill branch (LdsStack::pop): measured c4 -1.2 % alone, c3 -1.4 % alone, and with the
 * deferred hit stores (pt_wavefront.hip WCPT_WF_DEFER_HIT) c3 -2.9 % / c4 -2.8 % (profiles/r05_store_wait_ab.log). */
#ifndef WCPT_STACK_SPILL_WAIT
#define WCPT_STACK_SPILL_WAIT 1
#endif
/* Entries are packed (node index | t0 bits << 32). The two storage classes are typed by address space so that
 * the compiler emits ds_read/ds_write for the LDS part and scratch_* for the spill instead of merging the two
 * into one flat access. */
template <int N, int SPILL>
struct LdsStack {
    lds_u64_ptr base;   /* &lds[0][lane] */
    priv_u64_ptr spill; /* caller's private uint64_t[SPILL] */
    int sp;
    __device__ __forceinline__ void reset() { sp = 0; }
    __device__ __forceinline__ bool empty() const { return sp == 0; }
    __device__ __forceinline__ bool push(uint32_t i, float t)
    {
        const uint64_t e = (uint64_t)i | ((uint64_t)__float_as_uint(t) << 32);
#if WCPT_STACK_UNIFORM_FAST
        /* wave-uniform fast path: no pushing lane has reached the spill region (one compare and a scalar branch
         * instead of the exec-mask bookkeeping of a divergent if/else) */
        if (!__ballot(sp >= N)) {
            base[sp * 64] = e;
            sp++;
            return true;
        }
#endif
        if (sp < N) {
            base[sp * 64] = e;
        } else if (sp < N + SPILL) {
            spill[sp - N] = e;
        } else {
            return false;
        }
        sp++;
        return true;
    }
    __device__ __forceinline__ void pop(uint32_t& i, float& t)
    {
        sp--;
        uint64_t e;
#if WCPT_STACK_UNIFORM_FAST
        if (!__ballot(sp >= N)) {
            e = base[sp * 64];
        } else
#endif
        if (sp < N) {
            e = base[sp * 64];
        } else {
            e = spill[sp - N];
#if WCPT_STACK_SPILL_WAIT && defined(__gfx9__)
            /* wait for the spill load inside its (rare) branch: otherwise the LDS read of the other lanes, which
             * writes the same registers, waits for vmcnt(0) on every pop -- and so for every store still in flight.
             * The immediate is the gfx9 s_waitcnt encoding (gfx950 is gfx9); other generations lay the counters out
             * differently and get no explicit wait. */
            __builtin_amdgcn_s_waitcnt(0x0F70); /* vmcnt(0), expcnt/lgkmcnt untouched (gfx9 encoding) */
#endif
        }
        i = (uint32_t)e;
        t = __uint_as_float((uint32_t)(e >> 32));
    }
};

/* Closest-hit record during traversal: (t, primitive) only; the winner's normal and material are rebuilt
 * once afterwards (resolve_hit) with the reference's expressions, which gives the values the reference
 * computes at each update (:145, :173) without paying a normalize per closer hit. */

/* Geometric normal of the triangle at index positions prim..prim+2 of draw `draw` (:173): from its single record
 * when the triangle starts on a triangle boundary inside the records (the record was derived from exactly these
 * three indices), else recomputed from the index and vertex buffers with the same expression. */
__device__ __forceinline__ f3 triangle_normal(uint32_t prim, uint32_t draw, const wcpt_draw_command* __restrict__ draws,
                                              const uint64_t* __restrict__ tri_records)
{
    const uint32_t k = prim / 3u;
    if (tri_records && k * 3u == prim && k < (uint32_t)tri_records[kTriTableWords * draw + 2u]) {
        const gtri_ptr t = (gtri_ptr)(uintptr_t)tri_records[kTriTableWords * draw];
        const v4f r2 = t[3ull * k + 2u];
        return mk3(r2.y, r2.z, r2.w);
    }
    const TriE e = tri_from_indices(as_u32(draws[draw].indexBuffer), as_f32(draws[draw].vertexBuffer), prim,
                                    tri_records ? draw_vertex_count(tri_records, draw) : 0xFFFFFFFFu);
    return normalize(cross(e.e1, e.e2));
}

/* Intersect epilogue (:204-208) for winner `prim` (kNoPrim, kSpherePrim | sphere, or the index position of
 * a triangle of draw `draw`) at distance t. */
__device__ __forceinline__ Hit resolve_hit(const Ray& ray, float t, uint32_t prim, uint32_t draw,
                                           const wcpt_sphere* __restrict__ spheres,
                                           const wcpt_draw_command* __restrict__ draws,
                                           const uint64_t* __restrict__ tri_records)
{
    Hit h;
    h.t = t;
    h.hit = prim != kNoPrim;
    h.front = false;
    h.material = 0;
    h.normal = mk3(0.0f, 0.0f, 0.0f);
    if (h.hit) {
        if (prim & kSpherePrim) {
            const wcpt_sphere& s = spheres[prim & ~kSpherePrim];
            const f3 c = mk3(s.position[0], s.position[1], s.position[2]);
            const f3 ph = ray.origin + t * ray.direction;
            h.normal = (ph - c) / s.radius;                        /* :145 */
            h.material = s.material;
        } else {
            h.normal = triangle_normal(prim, draw, draws, tri_records); /* :173, material 0 (:175) */
        }
        h.front = dot(ray.direction, h.normal) < 0.0f;
        if (!h.front) h.normal = h.normal * -1.0f;
    }
    h.p = ray.origin + t * ray.direction;                             /* :205 */
    return h;
}

/* One draw command's geometry (pathTracer.comp:152-156 and the derived records of its table entry). */
struct DrawGeom {
    gnode_ptr bvh;
    gu32_ptr indices;
    gf32_ptr vertices;
    gtri_ptr tris;  /* pair records (PAIRS) or single records */
    gtri_ptr ptris; /* primary-ray pair records (PAIRS, when the runtime built them; table word 4) or null */
    uint32_t ntri;
    uint32_t nvert; /* vertex count bound of the index path (draw_vertex_count) */
    bool packed; /* stack entries carry (left, count): kTriFlagPackedRefs */
};
template <bool PAIRS>
__device__ __forceinline__ DrawGeom draw_geom(const wcpt_draw_command* __restrict__ draws,
                                              const uint64_t* __restrict__ tri_records, uint32_t i)
{
    DrawGeom g;
    g.bvh = as_nodes(draws[i].bvhBuffer);
    g.indices = as_u32(draws[i].indexBuffer);
    g.vertices = as_f32(draws[i].vertexBuffer);
    g.tris = (gtri_ptr)(uintptr_t)tri_records[kTriTableWords * i + (PAIRS ? 1u : 0u)];
    g.ptris = PAIRS ? (gtri_ptr)(uintptr_t)tri_records[kTriTableWords * i + 4u] : nullptr;
    g.ntri = (uint32_t)tri_records[kTriTableWords * i + 2u];
    g.nvert = draw_vertex_count(tri_records, i);
    g.packed = (tri_records[kTriTableWords * i + 3u] & kTriFlagPackedRefs) != 0u;
    return g;
}

/* The pair-record part of a leaf (:164-178): triangles [k0, kend) in pair records (2j, 2j+1), from `recs` (pair
 * records, or primary-ray pair records when PRIM). A leaf that starts in the second slot of a pair tests that pair
 * for its first triangle, then whole pairs, then possibly the first slot of a last pair -- no per-iteration slot
 * checks; applied in index order, strict <. UNIFORM: lanes of a coherent wave walk the whole pairs with scalar loads
 * (the record base must be wave-uniform). */
/* The pair record last tested for a peeled (odd-boundary) triangle in this segment: a leaf that ends in slot 0 of a pair
 * and the leaf that starts in its slot 1 (two 17-triangle midpoint leaves share the pair (16, 17)) both need that
 * record's test. Its byte offset with the two acceptance bits in bits 0-1, and both t: the second leaf reuses the
 * values the first computed -- the same test of the same ray on the same record -- and still applies them against
 * its own rec.t in its own order. Reset per segment and per draw (the offsets are relative to a draw's records). */
#ifndef WCPT_PEEL_CACHE
#define WCPT_PEEL_CACHE 1
#endif
struct PeelCache { uint32_t tag; v2f t; };
constexpr uint32_t kNoPeel = 0xFFFFFFFFu;
/* Take the pair's triangles in reference order (2j, then 2j+1; each iff accepted with t < rec.t, strict):
 * the winner is tagged with the record offset (+1 for the second). WCPT_PAIR_MERGE=1 picks the pair's own winner first
 * (the second only when strictly nearer, as the reference's second `<` against the updated rec.t would) and compares
 * that one with rec.t: the same winner, with one compare-select on rec.t's dependency chain per pair instead of two. */
#ifndef WCPT_PAIR_MERGE
#define WCPT_PAIR_MERGE 0
#endif
#if WCPT_PAIR_ITAKE
/* rb = bits(rec.t) - 1 (take_bits); hit0/hit1 are the acceptance without t > 0 */
__device__ __forceinline__ void pair_take_bits(const PairHit& ph, uint32_t off, uint32_t& rb, uint32_t& tag)
{
    const uint32_t b0 = take_bits(ph.t.x), b1 = take_bits(ph.t.y);
    if (ph.hit0 && b0 < rb) { rb = b0; tag = off; }
    if (ph.hit1 && b1 < rb) { rb = b1; tag = off + 1u; }
}
#endif
__device__ __forceinline__ void pair_take(const PairHit& ph, uint32_t off, float& rt, uint32_t& tag)
{
#if WCPT_PAIR_MERGE
    const float c0 = ph.hit0 ? ph.t.x : __builtin_inff();
    const float c1 = ph.hit1 ? ph.t.y : __builtin_inff();
    const bool second = c1 < c0;
    const float cb = second ? c1 : c0;
    if (cb < rt) {
        rt = cb;
        tag = off + (second ? 1u : 0u);
    }
#else
    if (ph.hit0 && ph.t.x < rt) { rt = ph.t.x; tag = off; }
    if (ph.hit1 && ph.t.y < rt) { rt = ph.t.y; tag = off + 1u; }
#endif
}
template <bool COUNT, bool DIAG, bool UNIFORM, bool PRIM>
__device__ __forceinline__ void pair_leaf(const Ray& ray, gtri_ptr recs, uint32_t k0, uint32_t kend, float& rt,
                                          uint32_t& prim, Counters& cnt, PeelCache& pc)
{
    constexpr uint32_t kBytes = PRIM ? kPrimPairRecordBytes : kPairRecordBytes;
    const WCPT_GLOBAL char* pbase = reinterpret_cast<const WCPT_GLOBAL char*>(recs);
    auto test_at = [&](uint32_t off) {
        if constexpr (PRIM) return rayTrianglePairP(ray, load_pairP_at(pbase, off));
        else return rayTrianglePair(ray, load_pair_at(pbase, off));
    };
    /* the peeled pair at `off`, through the per-segment cache */
    auto peeled_at = [&](uint32_t off) {
#if WCPT_PEEL_CACHE
        PairHit ph;
        if ((pc.tag & ~3u) == off) {
            ph.t = pc.t;
            ph.hit0 = (pc.tag & 1u) != 0u;
            ph.hit1 = (pc.tag & 2u) != 0u;
        } else {
            ph = test_at(off);
            pc.tag = off | (ph.hit0 ? 1u : 0u) | (ph.hit1 ? 2u : 0u);
            pc.t = ph.t;
        }
        return ph;
#else
        (void)pc;
        return test_at(off);
#endif
    };
#if WCPT_PAIR_ITAKE
    uint32_t rb = take_bits(rt); /* rec.t as bits - 1 through the leaf (take_bits) */
#define WCPT_TAKES(T, I) (take_bits(T) < rb)
#define WCPT_SET_RT(T) (rb = take_bits(T))
#else
#define WCPT_TAKES(T, I) ((T) < rt)
#define WCPT_SET_RT(T) (rt = (T))
#endif
    uint32_t k = k0;
    if (k & 1u) {
        const PairHit ph = peeled_at((k >> 1) * kBytes);
        count_tri<COUNT, DIAG>(cnt);
        if (ph.hit1 && WCPT_TAKES(ph.t.y, 1)) { WCPT_SET_RT(ph.t.y); prim = 3u * k; }
        k++;
    }
    /* whole pairs: one 32-bit byte-offset induction variable from the draw's record base, and the winner recorded
     * as a tag -- the pair's offset for its first triangle, offset + 1 for its second -- decoded into the index
     * position once per leaf */
    const uint32_t kfull = kend & ~1u;
    const uint32_t offEnd = (kfull >> 1) * kBytes;
    uint32_t off = (k >> 1) * kBytes, tag = kNoTag;
#if WCPT_PAIR_UNIFORM
    if (UNIFORM) {
        /* Lanes whose whole-pair range equals the first active lane's (in a coherent wave: all of them) read the
         * records at wave-uniform offsets with scalar loads: they go through the scalar cache (no per-lane
         * addresses, no vector-memory return of 64 copies of the record) and the packed-FP32 instructions take the
         * record straight from SGPRs (c2 -6 %). The other lanes take the per-lane loop below. */
        const uint32_t offU = __builtin_amdgcn_readfirstlane(off);
        const uint32_t endU = __builtin_amdgcn_readfirstlane(offEnd);
        /* tested through an opaque value: a plain `off == offU` lets the compiler substitute the equal per-lane
         * value back into the loads */
        uint32_t diff = (off ^ offU) | (offEnd ^ endU);
        asm volatile("" : "+v"(diff));
        if (diff == 0u) {
            /* the loop counter itself in an SGPR (offU..endU): no per-lane offset arithmetic (70 -> 68 VALU per
             * pair, c2 -1.7 %). A wave-uniform loop like this one was mis-compiled inside the old nested draw loop;
             * in the flat traversal loop it is correct (tools/stack_probe.py) */
#if WCPT_PAIR_PREFETCH
            if constexpr (!PRIM) {
                /* software-pipelined scalar records: the next pair's record is requested before this pair is tested,
                 * so its scalar-cache latency hides behind the test. The record one past the leaf's whole pairs is
                 * inside the draw's allocation (runtime: ntri / 2 + 1 pair records) and is never used. */
                TriPair cur = load_pair_const(pbase, offU);
                for (uint32_t o = offU; o < endU; o += kBytes) {
                    const TriPair nxt = load_pair_const(pbase, o + kBytes);
                    const PairHit ph = rayTrianglePair(ray, cur);
                    count_tri<COUNT, DIAG>(cnt);
                    count_tri<COUNT, DIAG>(cnt);
#if WCPT_PAIR_ITAKE
                    pair_take_bits(ph, o, rb, tag);
#else
                    pair_take(ph, o, rt, tag);
#endif
                    cur = nxt;
                }
                off = offEnd;
            } else
#endif
            for (uint32_t o = offU; o < endU; o += kBytes) {
                PairHit ph;
#if WCPT_PRIM_SIGN_SKIP
                if constexpr (PRIM) {
                    const TriPairP p = load_pairP_const(pbase, o);
                    v2f px, py, pz;
                    const v2f det = pairP_det(ray, p, px, py, pz);
                    if (__builtin_amdgcn_ballot_w64(pairP_may_take(p, det)) == 0ull) {
                        /* no lane can take either triangle (t <= 0 or NaN for all): the reference's tests still
                         * ran (and are counted), and none would change rec.t */
                        count_tri<COUNT, DIAG>(cnt);
                        count_tri<COUNT, DIAG>(cnt);
                        continue;
                    }
                    ph = pairP_finish(ray, p, px, py, pz, det);
                } else {
                    ph = rayTrianglePair(ray, load_pair_const(pbase, o));
                }
#else
                if constexpr (PRIM) ph = rayTrianglePairP(ray, load_pairP_const(pbase, o));
                else ph = rayTrianglePair(ray, load_pair_const(pbase, o));
#endif
#if WCPT_DUP_PAIR
                {
                    Ray r2 = ray;
                    r2.direction.x = launder(r2.direction.x);
                    PairHit p2;
                    if constexpr (PRIM) p2 = rayTrianglePairP(r2, load_pairP_const(pbase, o));
                    else p2 = rayTrianglePair(r2, load_pair_const(pbase, o));
                    sink(p2.t.x + p2.t.y);
                    sink_u((p2.hit0 ? 1u : 0u) | (p2.hit1 ? 2u : 0u));
                }
#endif
                count_tri<COUNT, DIAG>(cnt);
                count_tri<COUNT, DIAG>(cnt);
#if WCPT_PAIR_ITAKE
                pair_take_bits(ph, o, rb, tag);
#else
                pair_take(ph, o, rt, tag);
#endif
            }
            off = offEnd;
        }
    }
#endif
    for (; off < offEnd; off += kBytes) {
        const PairHit ph = test_at(off);
#if WCPT_DUP_PAIR
        if constexpr (!PRIM) {
            Ray r2 = ray;
            r2.origin.x = launder(r2.origin.x);
            const PairHit p2 = rayTrianglePair(r2, load_pair_at(pbase, off));
            sink(p2.t.x + p2.t.y);
            sink_u((p2.hit0 ? 1u : 0u) | (p2.hit1 ? 2u : 0u));
        }
#endif
        count_tri<COUNT, DIAG>(cnt);
        count_tri<COUNT, DIAG>(cnt);
#if WCPT_PAIR_ITAKE
        pair_take_bits(ph, off, rb, tag);
#else
        pair_take(ph, off, rt, tag);
#endif
    }
    if (tag != kNoTag) prim = 3u * (2u * (tag / kBytes) + (tag & 1u));
    if (k < kfull) k = kfull;
    if (k < kend) {
        const PairHit ph = peeled_at((k >> 1) * kBytes);
        count_tri<COUNT, DIAG>(cnt);
        if (ph.hit0 && WCPT_TAKES(ph.t.x, 0)) { WCPT_SET_RT(ph.t.x); prim = 3u * k; }
    }
#if WCPT_PAIR_ITAKE
    rt = __uint_as_float(rb + 1u);
#endif
#undef WCPT_TAKES
#undef WCPT_SET_RT
}

/* Leaf (:164-178): every triangle of the leaf at index positions [curLeft, curLeft + curCount), in index order,
 * taken iff accepted with t < rec.t (strict). UNIFORM: the leaf's whole pairs may be read with scalar loads (the
 * draw's record base must then be wave-uniform). primary: the segment is a sample's first (origin = the camera,
 * wave-uniform), whose leaves are tested from the primary-ray pair records when the draw has them. */
template <bool COUNT, bool DIAG, bool PAIRS, bool UNIFORM>
__device__ __forceinline__ void leaf_step(const Ray& ray, const DrawGeom& g, uint32_t curLeft, uint32_t curCount,
                                          float& rt, uint32_t& prim, Counters& cnt, bool primary, PeelCache& pc)
{
    const uint32_t k0 = leaf_record(curLeft, curCount, g.ntri);
    if (PAIRS && k0 != kNoRecord) {
        const uint32_t kend = k0 + (curCount + 2u) / 3u;
#if WCPT_PRIMARY_PAIRS
        if (primary && g.ptris != nullptr)
            pair_leaf<COUNT, DIAG, UNIFORM, true>(ray, g.ptris, k0, kend, rt, prim, cnt, pc);
        else
#endif
            pair_leaf<COUNT, DIAG, UNIFORM, false>(ray, g.tris, k0, kend, rt, prim, cnt, pc);
    } else {
        for (uint32_t k = 0, j = 0; k < curCount; k += 3, j++) {
            const uint32_t first = k + curLeft;
            const TriE tr = (!PAIRS && k0 != kNoRecord) ? load_tri(g.tris, k0 + j)
                                                        : tri_from_indices(g.indices, g.vertices, first, g.nvert);
            const float t = rayTriangleE(ray, tr.a, tr.e1, tr.e2);
            count_tri<COUNT, DIAG>(cnt);
            if (t != -1.0f && t < rt) {
                rt = t;
                prim = first;
            }
        }
    }
    phase_mark(cnt, 3);
}

/* Interior (:179-199): fetch both children (64 contiguous bytes), test both boxes, push the farther child if it
 * passes, and return true with the cursor on the nearer child if that one passes and is not culled by rec.t. */
template <bool COUNT, bool DIAG, class Stack>
__device__ __forceinline__ bool interior_step(const Ray& ray, const DrawGeom& g, Stack& stk, uint32_t& curLeft,
                                              uint32_t& curCount, float rt, Counters& cnt, bool& overflow,
                                              RefStack& rf)
{
    const NodeV L = load_node(g.bvh, curLeft);
    const NodeV R = load_node(g.bvh, curLeft + 1);
    float l0, l1, r0, r1;
    node_box(ray, L, l0, l1);
    node_box(ray, R, r0, r1);
#if WCPT_DUP_BOX
    {
        Ray r2 = ray;
        r2.origin.x = launder(r2.origin.x);
        r2.origin.y = launder(r2.origin.y);
        r2.origin.z = launder(r2.origin.z);
        float a0, a1, b0, b1;
        node_box(r2, L, a0, a1);
        node_box(r2, R, b0, b1);
        sink(a0 + a1 + b0 + b1);
    }
#endif
    if (COUNT) {
        cnt.interior_visits++;
        cnt.node_pops += 2;
        simd_step<DIAG>(cnt.wave_int, cnt.lane_int);
    }
    const float leftDist = (l0 > 0.0f) ? l0 : l1;
    const float rightDist = (r0 > 0.0f) ? r0 : r1;
    const bool passL = !(l0 > l1 || l1 < 0.0f);
    const bool passR = !(r0 > r1 || r1 < 0.0f);
    /* reference order: left popped first iff leftDist < rightDist */
    const bool leftFirst = leftDist < rightDist;
    const uint32_t farIdx = leftFirst ? curLeft + 1 : curLeft;
    const bool passNear = leftFirst ? passL : passR;
    const bool passFar = leftFirst ? passR : passL;
    const float nearT0 = leftFirst ? l0 : r0;
    const float farT0 = leftFirst ? r0 : l0;
    const NodeV& F = leftFirst ? R : L;
    if (passFar && !stk.push(node_ref(g.packed, farIdx, F.b.z, F.b.w), farT0)) overflow = true;
    ref_interior<COUNT>(rf, passFar, cnt);
    phase_mark(cnt, 2);
    if (passNear && !(nearT0 > rt)) {
        const NodeV& N = leftFirst ? L : R;
        curLeft = N.b.z;
        curCount = N.b.w;
        return true;
    }
    return false;
}

#ifndef WCPT_MK_POP_ONCE
#define WCPT_MK_POP_ONCE 1
#endif
/* Pop (:157-162): the next deferred node whose box entry distance is not beyond rec.t; false when none is left. */
template <bool COUNT, class Stack>
__device__ __forceinline__ bool pop_step(const DrawGeom& g, Stack& stk, uint32_t& curLeft, uint32_t& curCount, float rt,
                                         Counters& cnt, RefStack& rf)
{
    bool found = false;
    while (!stk.empty()) {
        uint32_t ni;
        float t0;
        stk.pop(ni, t0);
        ref_pop<COUNT>(rf);
        if (t0 > rt) continue;
        const uint2 lc = node_ref_lc(g.packed, g.bvh, ni);
        curLeft = lc.x;
        curCount = lc.y;
        found = true;
        break;
    }
    phase_mark(cnt, 2);
    return found;
}

/* The root of draw d (:152-162): pushed untested, popped and tested. Returns true with the cursor on the root when it
 * survives the cull. */
template <bool COUNT>
__device__ __forceinline__ bool root_step(const Ray& ray, const DrawGeom& g, float rt, uint32_t& curLeft,
                                          uint32_t& curCount, Counters& cnt, RefStack& rf)
{
    if (COUNT) { cnt.draw_fetches++; cnt.node_pops++; }
    ref_root<COUNT>(rf, cnt);
    const NodeV cur = load_node(g.bvh, 0);
    float c0, c1;
    node_box(ray, cur, c0, c1);
    if (c0 > c1 || c1 < 0.0f || c0 > rt) return false;
    curLeft = cur.b.z;
    curCount = cur.b.w;
    return true;
}

/* pathTracer.comp:135-211. PAIRS: leaf tests on pair records (else single records).
 *
 * SINGLE (drawCommandCount == 1, the reference's own case, PathTracingRenderer.jai:251): the draw's geometry is
 * kernel-uniform and its traversal runs once, without the draw loop. Otherwise the draws are walked inside the one
 * traversal loop (the next draw starts when the stack of the current one is exhausted), like wf_trace: the nested
 * form -- a loop over draws containing the divergent traversal loops, inside the divergent bounce loop -- is
 * mis-compiled by this toolchain whenever the traversal grows (a DIAG build or the scalar-load leaf loop on the
 * atrium overflowed the stack, tools/stack_probe.py), while this flat form is not. */
/* Every sample of a pixel starts with the same primary ray (pathTracer.comp:302, :309-310), so its Intersect record is
 * the same too: the megakernel keeps sample 0's and later samples resolve their primary segment from it (render
 * builds for samples > 1 only, a separate instantiation -- keeping the record costs the one-sample kernel 20 VGPRs --
 * and never the COUNT build, which traces every segment as the reference does for the exact counters). */
#ifndef WCPT_MK_PRIMARY_REUSE
#define WCPT_MK_PRIMARY_REUSE 1
#endif
template <bool COUNT, bool DIAG, bool PAIRS, bool SINGLE, class Stack>
__device__ __forceinline__ Hit intersect(const Ray& ray, const wcpt_scene_data& sd, const wcpt_sphere* __restrict__ spheres,
                                         const wcpt_draw_command* __restrict__ draws,
                                         const uint64_t* __restrict__ tri_records, Stack& stk,
                                         Counters& cnt, bool& overflow, bool primary, float4& prim_rec,
                                         bool reuse_primary)
{
    float rt = kInfinity;
    uint32_t prim = kNoPrim, primDraw = 0;
    if (!COUNT && WCPT_MK_PRIMARY_REUSE && reuse_primary) { /* a later sample's primary segment (TraceRay) */
        rt = prim_rec.x;
        prim = __float_as_uint(prim_rec.y);
        primDraw = __float_as_uint(prim_rec.z);
    } else {
        if (COUNT) {
            cnt.segments++;
            simd_step<DIAG>(cnt.wave_seg, cnt.lane_seg);
        }

        sphere_loop(ray, sd.sphereCount, spheres, rt, prim);
        if (COUNT) cnt.sphere_tests += sd.sphereCount;
#if WCPT_DUP_SPHERES
        {
            Ray r2 = ray;
            r2.origin.x = launder(r2.origin.x);
            r2.direction.x = launder(r2.direction.x);
            float rt2 = kInfinity;
            uint32_t p2 = 0;
            for (uint32_t i = 0; i < sd.sphereCount; i++) {
                const wcpt_sphere& s = spheres[i];
                const float tr = raySphereNear(r2, mk3(s.position[0], s.position[1], s.position[2]), s.radius);
                if (tr > 0.0f && tr < rt2) { rt2 = tr; p2 = i; }
            }
            sink(rt2);
            sink_u(p2);
        }
#endif
        phase_mark(cnt, 1);

        uint32_t curLeft = 0, curCount = 0;
        PeelCache pc;
        pc.tag = kNoPeel;
        pc.t = bc2(0.0f);
        RefStack rf;
        if constexpr (SINGLE) {
            const DrawGeom g = draw_geom<PAIRS>(draws, tri_records, 0);
            /* one traversal step per iteration as sequential ifs on the lane's mode (pop -> interior -> leaf), like
             * wf_trace: a lane that pops an interior node visits it in the same iteration, one that descends into a
             * leaf tests it in the same iteration */
            enum : uint32_t { kInterior = 0, kLeaf = 1, kPop = 2, kDone = 3 };
            uint32_t mode = kDone;
            if (sd.drawCommandCount != 0u && root_step<COUNT>(ray, g, rt, curLeft, curCount, cnt, rf)) {
                stk.reset();
                mode = curCount > 0 ? kLeaf : kInterior;
            }
            while (mode != kDone) {
#if WCPT_MK_POP_ONCE
                if (mode == kPop) {
                    /* one stack entry per iteration (no inner pop loop): a culled entry (:162) keeps the lane popping */
                    if (stk.empty()) {
                        mode = kDone;
                    } else {
                        uint32_t ni;
                        float t0;
                        stk.pop(ni, t0);
                        ref_pop<COUNT>(rf);
                        if (!(t0 > rt)) {
                            const uint2 lc = node_ref_lc(g.packed, g.bvh, ni);
                            curLeft = lc.x;
                            curCount = lc.y;
                            mode = curCount > 0 ? kLeaf : kInterior;
                        }
                    }
                    phase_mark(cnt, 2);
                }
#else
                if (mode == kPop)
                    mode = pop_step<COUNT>(g, stk, curLeft, curCount, rt, cnt, rf) ? (curCount > 0 ? kLeaf : kInterior)
                                                                                    : kDone;
#endif
                if (mode == kInterior)
                    mode = interior_step<COUNT, DIAG>(ray, g, stk, curLeft, curCount, rt, cnt, overflow, rf)
                               ? (curCount > 0 ? kLeaf : kInterior) : kPop;
                if (mode == kLeaf) {
                    leaf_step<COUNT, DIAG, PAIRS, true>(ray, g, curLeft, curCount, rt, prim, cnt, primary, pc);
                    mode = kPop;
                }
            }
        } else {
            uint32_t d = 0;
            DrawGeom g;
            float rt_before = rt;
            /* first draw (from d on) whose root survives the cull */
            auto start_draw = [&]() {
                for (; d < sd.drawCommandCount; d++) {
                    g = draw_geom<PAIRS>(draws, tri_records, d);
                    rt_before = rt;
                    if (root_step<COUNT>(ray, g, rt, curLeft, curCount, cnt, rf)) {
                        stk.reset();
                        pc.tag = kNoPeel; /* offsets of another draw's records */
                        return true;
                    }
                }
                return false;
            };
            bool active = start_draw();
            while (active) {
                if (curCount > 0) {
                    leaf_step<COUNT, DIAG, PAIRS, false>(ray, g, curLeft, curCount, rt, prim, cnt, primary, pc);
                } else if (interior_step<COUNT, DIAG>(ray, g, stk, curLeft, curCount, rt, cnt, overflow, rf)) {
                    continue;
                }
                if (pop_step<COUNT>(g, stk, curLeft, curCount, rt, cnt, rf)) continue;
                if (rt != rt_before) primDraw = d; /* this draw lowered rt: it owns prim */
                d++;
                active = start_draw();
            }
        }
    }
    if (!COUNT && WCPT_MK_PRIMARY_REUSE && primary && sd.samples > 1u) prim_rec = make_float4(rt, __uint_as_float(prim), __uint_as_float(primDraw), 0.0f);
    if (COUNT && prim != kNoPrim) cnt.hits++;
    ref_segment_end<COUNT>(cnt);
    const Hit hit = resolve_hit(ray, rt, prim, primDraw, spheres, draws, tri_records);
    phase_mark(cnt, 4);
    return hit;
}

/* pathTracer.comp:213-234 */
__device__ __forceinline__ float CalculateReflectance(f3 inDir, f3 normal, float iorA, float iorB)
{
    const float refractRatio = iorA / iorB;
    const float cosAngleIn = -dot(inDir, normal);
    const float sinSqr = refractRatio * refractRatio * (1.0f - cosAngleIn * cosAngleIn);
    if (sinSqr >= 1.0f) return 1.0f;
    const float cosRefr = sqrt_exact(1.0f - sinSqr);
    const float dPerp = iorA * cosAngleIn + iorB * cosRefr;
    const float dPar = iorB * cosAngleIn + iorA * cosRefr;
    if (fminf(dPerp, dPar) < 1e-8f) return 1.0f;
    float rPerp = (iorA * cosAngleIn - iorB * cosRefr) / dPerp;
    rPerp *= rPerp;
    float rPar = (iorB * cosAngleIn - iorA * cosRefr) / dPar;
    rPar *= rPar;
    return (rPerp + rPar) / 2.0f;
}

/* pathTracer.comp:236-239 */
__device__ __forceinline__ f3 ray_color(const Ray& r)
{
    const float a = 0.5f * (r.direction.y + 1.0f);
    const float ia = 1.0f - a;
    return mk3(0.5f * ia + 1.0f * a, 0.7f * ia + 1.0f * a, 1.0f * ia + 1.0f * a);
}

/* State of one path between segments: the loop-carried variables of TraceRay (pathTracer.comp:241-245). */
struct PathState {
    Ray ray;
    f3 totalLight;
    f3 transmittance;
    uint32_t bounce; /* loop index i of :245 */
};

__device__ __forceinline__ void path_begin(PathState& ps, f3 origin, f3 dir)
{
    ps.ray.origin = origin;
    ps.ray.direction = dir;
    ps.ray.invDirection = rcp3(dir);
    ps.totalLight = mk3(0.0f, 0.0f, 0.0f);
    ps.transmittance = mk3(1.0f, 1.0f, 1.0f);
    ps.bounce = 0;
}

#ifndef WCPT_SHADE_SHARED
#define WCPT_SHADE_SHARED 1
#endif
/* The last segment of a pixel's last sample ends the path whatever it samples next: after its emission term
 * (:253) the reference still draws the BSDF sample of :256-280 -- the next direction, transmittance and RNG state --
 * but the loop then exits (:245, :283) and nothing reads them again (the RNG state carries over only into a next
 * sample, :309-310). WCPT_LAST_SEGMENT_SHORTCUT=1 returns right after the emission term there: the same radiance
 * bits, without the dead RandomDirection, reflection, normalize and 1/direction. The condition is wave-uniform in
 * the megakernel (the lanes of a wave start every sample together). */
#ifndef WCPT_LAST_SEGMENT_SHORTCUT
#define WCPT_LAST_SEGMENT_SHORTCUT 1
#endif
/* Shading after an Intersect (pathTracer.comp:248-280). Returns true when the path is finished, with its
 * radiance in L: on a miss (:248-249) or when the bounce loop is exhausted (:245, :283). lastSample: this is the
 * pixel's last sample (its RNG state is not read after the path). */
__device__ __forceinline__ bool path_shade(PathState& ps, const Hit& h, uint32_t& rng, const wcpt_scene_data& sd,
                                           const wcpt_material* __restrict__ mats, f3& L, bool lastSample)
{
    Ray& ray = ps.ray;
    if (!h.hit) {
        L = ps.totalLight + ray_color(ray) * ps.transmittance;
        return true;
    }
    const wcpt_material& m = mats[h.material];
    const uint32_t mtype = m.type;
    const f3 emission = ld3(m.emission);
    const float emissionStrength = m.emissionStrength;
    const float roughness = m.roughness;
    ps.totalLight = ps.totalLight + (emission * emissionStrength) * ps.transmittance;
#if WCPT_LAST_SEGMENT_SHORTCUT
    if (lastSample && ps.bounce + 1u > sd.maxBounceCount) { /* the loop's last iteration (:245): nothing below is read */
        L = ps.totalLight;
        return true;
    }
#else
    (void)lastSample;
#endif

#if WCPT_SHADE_SHARED
    /* Both branches of :256-280 end in normalize(base + roughness * RandomDirection(rng)) and a new 1/direction.
     * That tail is shared here, after the dielectric-only part (Fresnel, refract and the :273 rand, which must
     * precede RandomDirection in the lane's RNG sequence), so a wave whose lanes hit both kinds of material runs
     * RandomDirection (6 rand, 3 log, 3 cos, 4 sqrt) once instead of once per branch. Every lane performs the
     * reference's operations in the reference's order. */
    const bool metal = mtype == WCPT_MATERIAL_METAL;
    const f3 R = reflect(ray.direction, h.normal);
    f3 base = R;
    bool followReflection = true;
    if (!metal) {
        const float ior = m.ior;
        const float etaI = h.front ? 1.0f : ior;
        const float etaT = h.front ? ior : 1.0f;
        const float reflectProb = CalculateReflectance(ray.direction, h.normal, etaI, etaT);
        const f3 T = refract(ray.direction, h.normal, etaI / etaT);
        followReflection = (T.x == 0.0f && T.y == 0.0f && T.z == 0.0f);
        if (!followReflection) followReflection = (rand_f(rng) <= reflectProb); /* :273 short-circuit */
        if (!followReflection) base = T;
    }
    const f3 rd = RandomDirection(rng);
#if WCPT_DUP_RANDDIR
    {
        uint32_t r2 = launder_u(rng);
        const f3 d2 = RandomDirection(r2);
        sink(d2.x + d2.y + d2.z);
    }
#endif
    const f3 dir = normalize(base + roughness * rd);
    if (metal) {
        ray.origin = h.p + h.normal * kBias;                                  /* :257 */
        ps.transmittance = ps.transmittance * ld3(m.albedo);                  /* :261 */
    } else {
        if (!followReflection && !h.front) {                                  /* :276-278 */
            const f3 e = ((ld3(m.absorption) * -1.0f) * m.absorptionStrength) * h.t;
            ps.transmittance = ps.transmittance * mk3(wcpt_expf(e.x), wcpt_expf(e.y), wcpt_expf(e.z));
        }
        ray.origin = h.p + (kBias * h.normal) * sign1(dot(dir, h.normal));   /* :279 */
    }
    ray.direction = dir;
    ray.invDirection = rcp3(dir);
#else
    if (mtype == WCPT_MATERIAL_METAL) {
        ray.origin = h.p + h.normal * kBias;
        const f3 R = reflect(ray.direction, h.normal);
        const f3 rd = RandomDirection(rng);
        ray.direction = normalize(R + roughness * rd);
        ray.invDirection = rcp3(ray.direction);
        ps.transmittance = ps.transmittance * ld3(m.albedo);
    } else {
        const float ior = m.ior;
        const float etaI = h.front ? 1.0f : ior;
        const float etaT = h.front ? ior : 1.0f;
        const float reflectProb = CalculateReflectance(ray.direction, h.normal, etaI, etaT);
        const f3 R = reflect(ray.direction, h.normal);
        const f3 T = refract(ray.direction, h.normal, etaI / etaT);
        bool followReflection = (T.x == 0.0f && T.y == 0.0f && T.z == 0.0f);
        if (!followReflection) followReflection = (rand_f(rng) <= reflectProb); /* :273 short-circuit */
        const f3 rd = RandomDirection(rng);
        ray.direction = normalize((followReflection ? R : T) + roughness * rd);
        ray.invDirection = rcp3(ray.direction);
        if (!followReflection && !h.front) {
            const f3 e = ((ld3(m.absorption) * -1.0f) * m.absorptionStrength) * h.t;
            ps.transmittance = ps.transmittance * mk3(wcpt_expf(e.x), wcpt_expf(e.y), wcpt_expf(e.z));
        }
        ray.origin = h.p + (kBias * h.normal) * sign1(dot(ray.direction, h.normal));
    }
#endif
    ps.bounce++;
    if (ps.bounce > sd.maxBounceCount) { /* loop exhausted: no sky term (:283) */
        L = ps.totalLight;
        return true;
    }
    return false;
}

/* pathTracer.comp:241-284. prim_rec: the primary segment's Intersect record (t, primitive, draw), written by the
 * first sample; reuse_primary: a later sample, whose primary segment reads it instead of tracing the same ray again
 * (intersect). */
template <bool COUNT, bool DIAG, bool PAIRS, bool SINGLE, class Stack, bool REUSE = false>
__device__ __forceinline__ f3 TraceRay(Ray ray, uint32_t& rng, const wcpt_scene_data& sd,
                                       const wcpt_material* __restrict__ mats, const wcpt_sphere* __restrict__ spheres,
                                       const wcpt_draw_command* __restrict__ draws,
                                       const uint64_t* __restrict__ tri_records, Stack& stk,
                                       Counters& cnt, bool& overflow, bool lastSample, float4& prim_rec,
                                       bool reuse_primary)
{
    PathState ps;
    path_begin(ps, ray.origin, ray.direction);
    f3 L;
    /* segment counter of this sample: uniform across the wave's lanes (all start a sample together), so `primary`
     * (segment 0: origin = the camera) is a wave-uniform branch condition */
    for (uint32_t seg = 0;; seg++) {
        const Hit h = intersect<COUNT, DIAG, PAIRS, SINGLE>(ps.ray, sd, spheres, draws, tri_records, stk, cnt, overflow,
                                                           seg == 0u, prim_rec, REUSE && seg == 0u && reuse_primary);
        const bool done = path_shade(ps, h, rng, sd, mats, L, lastSample);
        phase_mark(cnt, 5);
        if (done) return L;
    }
}

/* pathTracer.comp:290-302 — primary ray direction for pixel (x, y) of a W x H frame. */
__device__ __forceinline__ f3 primary_direction(const wcpt_scene_data& sd, uint32_t x, uint32_t y, uint32_t W, uint32_t H)
{
    const float imgW = (float)W, imgH = (float)H;
    float cx = (float)x / imgW, cy = (float)y / imgH;
    cx = cx + (1.0f / imgW) * 0.5f;
    cy = cy + (1.0f / imgH) * 0.5f;
    cy = 1.0f - cy;
    cx = cx * 2.0f - 1.0f;
    cy = cy * 2.0f - 1.0f;
    const float* P = sd.inverseProjection;
    float tg[4];
#pragma unroll
    for (int r = 0; r < 4; r++) tg[r] = P[0 * 4 + r] * cx + P[1 * 4 + r] * cy + P[2 * 4 + r] * 1.0f + P[3 * 4 + r] * 1.0f;
    const f3 d = normalize(mk3(tg[0], tg[1], tg[2]) / tg[3]);
    const float* V = sd.inverseView;
    float wd[3];
#pragma unroll
    for (int r = 0; r < 3; r++) wd[r] = V[0 * 4 + r] * d.x + V[1 * 4 + r] * d.y + V[2 * 4 + r] * d.z + V[3 * 4 + r] * 0.0f;
    return normalize(mk3(wd[0], wd[1], wd[2]));
}

/* Final store of a pixel (pathTracer.comp:323, `vec4(acc, 1)`): the accumulation image, plus the gather payload
 * (wcpt_set_gather_output) when the host asked for one, same row-major pixel index: RGB (3 floats), RGBA (4 floats),
 * or WCPT_PAYLOAD_DISPLAY_RGBA8 -- the display step of composite.comp:36-53 (gamma 1/2.2 + PBR Neutral, then UNORM8)
 * applied to the accumulated value as it is stored, so a multi-device frame travels at 4 B/px
 * with no composite pass over the image. */
__device__ __noinline__ uint32_t display_rgba8(f3 acc)
{
    const float in[4] = {acc.x, acc.y, acc.z, 1.0f};
    float o[4];
    wcpt_composite_texel(in, o);
    return (uint32_t)wcpt_unorm8(o[0]) | ((uint32_t)wcpt_unorm8(o[1]) << 8) | ((uint32_t)wcpt_unorm8(o[2]) << 16) |
           (255u << 24);
}
/* Gather-output rows (row_map.h): the map {0, 31, 0} (row = ly) addresses a payload that holds the context's rows back
 * to back; the context's own row map addresses a whole frame (WCPT_OPTION_GATHER_FRAME_ROWS). */

/* :323 imageStore of pixel (lx, ly) of the context's rows into the accumulation image (index i = ly * W + lx), and
 * into the gather output (wcpt_set_gather_output) at row frame_row(wm, ly) of that output */
__device__ __forceinline__ void store_pixel(float4* __restrict__ image, float* __restrict__ wire, uint32_t wire_ch,
                                            const RowMap& wm, uint32_t W, uint32_t lx, uint32_t ly, f3 acc)
{
    const size_t i = (size_t)ly * W + lx;
    image[i] = make_float4(acc.x, acc.y, acc.z, 1.0f);
    if (wire) {
        const size_t j = (size_t)frame_row(wm, ly) * W + lx;
        if (wire_ch == 3u) {
            float* w = wire + 3u * j;
            w[0] = acc.x;
            w[1] = acc.y;
            w[2] = acc.z;
        } else if (wire_ch == 4u) {
            reinterpret_cast<float4*>(wire)[j] = make_float4(acc.x, acc.y, acc.z, 1.0f);
        } else {
            reinterpret_cast<uint32_t*>(wire)[j] = display_rgba8(acc);
        }
    }
}

/* Wave-level sum of a per-lane u32 counter, one u64 atomic per wave. */
__device__ __forceinline__ void wave_add_u64(unsigned long long* dst, uint32_t v)
{
    unsigned long long s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(dst, s);
}

/* Wave-reduce the per-lane counters into the 16 global u64 counters (wcpt_counters order; the last is a maximum).
 * All 64 lanes of the wave must call it. */
template <bool COUNT>
__device__ __forceinline__ void flush_counters(const Counters& cnt, unsigned long long* __restrict__ counters)
{
    if (COUNT) {
        wave_add_u64(&counters[0], cnt.pixels);
        wave_add_u64(&counters[1], cnt.segments);
        wave_add_u64(&counters[2], cnt.sphere_tests);
        wave_add_u64(&counters[3], cnt.node_pops);
        wave_add_u64(&counters[4], cnt.interior_visits);
        wave_add_u64(&counters[5], cnt.triangle_tests);
        wave_add_u64(&counters[6], cnt.hits);
        wave_add_u64(&counters[7], cnt.draw_fetches);
        wave_add_u64(&counters[8], cnt.wave_int);
        wave_add_u64(&counters[9], cnt.lane_int);
        wave_add_u64(&counters[10], cnt.wave_tri);
        wave_add_u64(&counters[11], cnt.lane_tri);
        wave_add_u64(&counters[12], cnt.wave_seg);
        wave_add_u64(&counters[13], cnt.lane_seg);
        wave_add_u64(&counters[14], cnt.ref_over);
        uint32_t m = cnt.ref_max;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, off, 64));
        if ((threadIdx.x & 63) == 0 && m) atomicMax(&counters[15], (unsigned long long)m);
    }
}

} // namespace dev
} // namespace wcpt

#endif /* WCPT_PT_DEVICE_H */
