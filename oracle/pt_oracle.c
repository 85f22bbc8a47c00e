/*
 * pt_oracle.c — CPU ORACLE for the WC-Path-tracer compute path.  TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and only as
 * the checker / the reported CPU baseline. The product (wc-path-tracer_amd/) never links or calls it.
 *
 * What it is: a scalar C restatement of the reference algorithm, IEEE binary32 with no contraction
 * (built with -ffp-contract=off), following
 *   - src/shaders/pathTracer.comp:97-324      (intersection, traversal, BSDF, TraceRay, main)
 *   - src/shaders/include/Random.glsl:10-56    (PCG hash / stepping, rand, Box-Muller, RandomDirection)
 *   - src/shaders/include/constants.glsl:4-9   (bias, kInfinity, PI)
 *   - src/PathTracingRenderer.jai:147-217      (UpdateNodeBounds / Subdivide midpoint BVH)
 * with GLSL 4.50 built-ins written out: dot = (x*x' + y*y') + z*z'; cross per the GLSL spec;
 * normalize(v) = v / sqrt(dot(v,v)) where vector / scalar = v * (1/s) (see div3s); reflect(I,N) =
 * I - (2*dot(N,I))*N; refract per the GLSL spec;
 * mix(x,y,a) = x*(1-a) + y*a; sign(0) = 0; min/max = IEEE minNum/maxNum (a NaN operand yields the other).
 * log/cos/exp are the deterministic definitions of wc-path-tracer_amd/csrc/wcpt_libm.h (GLSL leaves their
 * precision to the driver; see DESIGN.md "Parity").
 *
 * Parity pinning: the reference cannot be built or run here (Jai host, GLSL needing glslc + a Vulkan ICD;
 * SURVEY.md §8(c)). The RNG is pinned by the known-answer values of SURVEY.md §4 (tests/test_oracle.py);
 * the intersection primitives by hand-derived known answers; full images are "parity unpinned" against
 * reference execution and are pinned as committed golden fixtures of this oracle (tests/golden/).
 *
 * Instrumented with the per-frame counters of SURVEY.md §8(d) (wcpt_counters).
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/wcpt.h"
#include "../wc-path-tracer_amd/csrc/wcpt_libm.h"

/* ------------------------------------------------------------------------------------------------ */
/* constants.glsl:4-9                                                                               */
static const float kBias = 1e-5f;
static const float kInfinity = 3.402823466e+38f;
static const float kPI = 3.14159265358979323846264338327950288f;

typedef struct { float x, y, z; } v3;
typedef struct { float x, y; } v2;

static inline v3 mk3(float x, float y, float z) { v3 r; r.x = x; r.y = y; r.z = z; return r; }
static inline v3 add3(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub3(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul3(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 mul3s(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
static inline v3 smul3(float s, v3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
/* GLSL vector / scalar, implemented as v * RN(1/s) (Vulkan allows 2.5 ULP for division; this is <= 1.5 ULP). The
 * kernel evaluates the same expression with its correctly rounded reciprocal (pt_device.h operator/). */
static inline v3 div3s(v3 a, float s) { const float r = 1.0f / s; return mk3(a.x * r, a.y * r, a.z * r); }
static inline v3 sdiv3(float s, v3 a) { return mk3(s / a.x, s / a.y, s / a.z); }
static inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross3(v3 a, v3 b)
{
    return mk3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
static inline v3 normalize3(v3 v) { return div3s(v, sqrtf(dot3(v, v))); }
static inline v3 reflect3(v3 I, v3 N) { return sub3(I, mul3s(N, 2.0f * dot3(N, I))); }
static inline v3 refract3(v3 I, v3 N, float eta)
{
    const float d = dot3(N, I);
    const float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return mk3(0.0f, 0.0f, 0.0f);
    return sub3(smul3(eta, I), mul3s(N, eta * d + sqrtf(k)));
}
static inline float fmin_nn(float a, float b) { if (a != a) return b; if (b != b) return a; return b < a ? b : a; }
static inline float fmax_nn(float a, float b) { if (a != a) return b; if (b != b) return a; return b > a ? b : a; }
static inline float sign1(float x) { return x > 0.0f ? 1.0f : (x < 0.0f ? -1.0f : 0.0f); }
static inline v3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }

/* ------------------------------------------------------------------------------------------------ */
/* Random.glsl:10-56                                                                                */
uint32_t oracle_pcg_hash(uint32_t seed)
{
    uint32_t state = seed * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}

static inline uint32_t rand_pcg(uint32_t* rngState)
{
    uint32_t state = *rngState;
    *rngState = *rngState * 747796405u + 2891336453u;
    uint32_t word = ((state >> ((state >> 28u) + 4u)) ^ state) * 277803737u;
    return (word >> 22u) ^ word;
}

/* rand(): the output overwrites the state (Random.glsl:29-30), discarding the LCG step of :21. */
float oracle_rand(uint32_t* state)
{
    uint32_t x = rand_pcg(state);
    *state = x;
    return (float)x * 2.3283064365386963e-10f; /* uintBitsToFloat(0x2f800000) = 2^-32 */
}

static inline float RandomValueNormalDistribution(uint32_t* seed)
{
    const float theta = 2.0f * kPI * oracle_rand(seed);
    const float rho = sqrtf(-2.0f * wcpt_logf(oracle_rand(seed)));
    return rho * wcpt_cosf(theta);
}

static inline v3 RandomDirection(uint32_t* seed)
{
    const float x = RandomValueNormalDistribution(seed);
    const float y = RandomValueNormalDistribution(seed);
    const float z = RandomValueNormalDistribution(seed);
    return normalize3(mk3(x, y, z));
}

/* Exported for the libm / RNG known-answer tests. */
float oracle_logf(float x) { return wcpt_logf(x); }
float oracle_cosf(float x) { return wcpt_cosf(x); }
/* the kernel's domain-specialised variants (equal to the general ones on rand()'s values / [0, 2*pi]) */
float oracle_logf_rand(float x) { return wcpt_logf_rand(x); }
float oracle_cosf_2pi(float x) { return wcpt_cosf_2pi(x); }
/* Mismatches between the specialised and the general functions over the rand() outputs n * 2^-32 for
 * n = first, first + stride, ... < 2^32 (log of the value, cos of 2*PI times it, Random.glsl:45-46). */
uint64_t oracle_libm_domain_mismatches(uint32_t first, uint32_t stride)
{
    uint64_t bad = 0;
    for (uint64_t n = first; n < (1ull << 32); n += stride) {
        const float x = (float)(uint32_t)n * 2.3283064365386963e-10f;
        const float th = 2.0f * 3.14159265358979323846264338327950288f * x;
        const float l0 = wcpt_logf(x), l1 = wcpt_logf_rand(x);
        const float c0 = wcpt_cosf(th), c1 = wcpt_cosf_2pi(th);
        bad += (wcpt_f2u(l0) != wcpt_f2u(l1)) + (wcpt_f2u(c0) != wcpt_f2u(c1));
    }
    return bad;
}
float oracle_expf(float x) { return wcpt_expf(x); }
void oracle_random_direction(uint32_t* seed, float* out3)
{
    v3 d = RandomDirection(seed);
    out3[0] = d.x; out3[1] = d.y; out3[2] = d.z;
}

/* ------------------------------------------------------------------------------------------------ */
/* pathTracer.comp:24-28, 50-58                                                                     */
typedef struct { v3 origin, direction, invDirection; } Ray;
typedef struct { v3 p, normal; float t; int hit, front; uint32_t material; } HitInfo;

/* Host-side view of one DrawCommand (pathTracer.comp:82-87) with host pointers. */
typedef struct oracle_draw {
    const float* vertices;      /* vec3 stride 12 */
    const uint32_t* indices;
    const wcpt_node* bvh;
} oracle_draw;

typedef struct {
    const wcpt_scene_data* sd;
    const wcpt_material* materials;
    const wcpt_sphere* spheres;
    const oracle_draw* draws;
    wcpt_counters* cnt;
    int overflow;
} Scene;

/* pathTracer.comp:97-108 */
static inline v2 rayBoxIntersect(const Ray* ray, v3 bmin, v3 bmax)
{
    const v3 tbot = mul3(sub3(bmin, ray->origin), ray->invDirection);
    const v3 ttop = mul3(sub3(bmax, ray->origin), ray->invDirection);
    const v3 tmin = mk3(fmin_nn(ttop.x, tbot.x), fmin_nn(ttop.y, tbot.y), fmin_nn(ttop.z, tbot.z));
    const v3 tmax = mk3(fmax_nn(ttop.x, tbot.x), fmax_nn(ttop.y, tbot.y), fmax_nn(ttop.z, tbot.z));
    v2 t, r;
    t.x = fmax_nn(tmin.x, tmin.y); t.y = fmax_nn(tmin.x, tmin.z);
    r.x = fmax_nn(t.x, t.y);
    t.x = fmin_nn(tmax.x, tmax.y); t.y = fmin_nn(tmax.x, tmax.z);
    r.y = fmin_nn(t.x, t.y);
    return r;
}

/* pathTracer.comp:110-119 (only .x is used by the caller, :141) */
static inline float raySphereIntersectNear(const Ray* ray, v3 position, float radius)
{
    const v3 oc = sub3(ray->origin, position);
    const float b = dot3(oc, ray->direction);
    const float c = dot3(oc, oc) - radius * radius;
    const float t = b * b - c;
    if (t < 0.0f) return -1.0f;
    return -b - sqrtf(t);
}

/* pathTracer.comp:121-133; returns t or -1 */
static inline float rayTriangleIntersect(const Ray* ray, v3 a, v3 b, v3 c)
{
    const v3 edgeAB = sub3(b, a);
    const v3 edgeAC = sub3(c, a);
    const v3 oa = sub3(ray->origin, a);
    const v3 crossRDE2 = cross3(ray->direction, edgeAC);
    const float inv = 1.0f / dot3(edgeAB, crossRDE2);
    const v3 crossROAE1 = cross3(oa, edgeAB);
    const float u = dot3(oa, crossRDE2) * inv;
    const float v = dot3(ray->direction, mul3s(crossROAE1, inv));
    const float t = dot3(edgeAC, crossROAE1) * inv;
    return (t > 0.0f && u >= 0.0f && u <= 1.0f && v >= 0.0f && u + v <= 1.0f) ? t : -1.0f;
}

#define ORACLE_STACK 256

/* pathTracer.comp:135-211 */
static HitInfo Intersect(Scene* S, const Ray* ray)
{
    HitInfo rec;
    uint32_t nodeStack[ORACLE_STACK];
    const wcpt_scene_data* sd = S->sd;
    memset(&rec, 0, sizeof(rec));
    rec.t = kInfinity;
    rec.hit = 0;
    S->cnt->segments++;

    for (uint32_t i = 0; i < sd->sphereCount; i++) {
        const wcpt_sphere* sp = &S->spheres[i];
        const float tempRec = raySphereIntersectNear(ray, ld3(sp->position), sp->radius);
        S->cnt->sphere_tests++;
        if (tempRec > 0.0f && tempRec < rec.t) {
            rec.t = tempRec;
            rec.p = add3(ray->origin, smul3(rec.t, ray->direction));
            rec.normal = div3s(sub3(rec.p, ld3(sp->position)), sp->radius);
            rec.hit = 1;
            rec.material = sp->material;
        }
    }

    /* The reference's stack is uint nodeStack[32] (:151). This one is deeper, so the reference's out-of-bounds writes
     * are counted instead of performed: a segment that pushes at index >= 32 (ref_stack_overflow_segments), and the
     * deepest stack reached (ref_stack_max). */
    int ref_overflow = 0;
    for (uint32_t i = 0; i < sd->drawCommandCount; i++) {
        const oracle_draw* dc = &S->draws[i];
        int stackIndex = 0;
        S->cnt->draw_fetches++;
        nodeStack[stackIndex++] = 0;
        if (S->cnt->ref_stack_max < 1) S->cnt->ref_stack_max = 1;
        while (stackIndex > 0) {
            const uint32_t nodeIdx = nodeStack[--stackIndex];
            const wcpt_node* node = &dc->bvh[nodeIdx];
            const v2 bvhT = rayBoxIntersect(ray, ld3(node->min), ld3(node->max));
            S->cnt->node_pops++;
            if (bvhT.x > bvhT.y || bvhT.y < 0.0f || bvhT.x > rec.t) continue;
            if (node->triangleCount > 0) {
                for (uint32_t k = 0; k < node->triangleCount; k += 3) {
                    const uint32_t first = k + node->leftNodeOrTriangleIndex;
                    const v3 a = ld3(dc->vertices + 3u * (uint64_t)dc->indices[first + 0]);
                    const v3 b = ld3(dc->vertices + 3u * (uint64_t)dc->indices[first + 1]);
                    const v3 c = ld3(dc->vertices + 3u * (uint64_t)dc->indices[first + 2]);
                    const float t = rayTriangleIntersect(ray, a, b, c);
                    S->cnt->triangle_tests++;
                    if (t != -1.0f && t < rec.t) {
                        rec.t = t;
                        rec.normal = normalize3(cross3(sub3(b, a), sub3(c, a)));
                        rec.hit = 1;
                        rec.material = 0; /* :175 triangles always use material 0 */
                    }
                }
            } else {
                const uint32_t leftChild = node->leftNodeOrTriangleIndex;
                const uint32_t rightChild = leftChild + 1;
                const wcpt_node* leftNode = &dc->bvh[leftChild];
                const wcpt_node* rightNode = &dc->bvh[rightChild];
                const v2 leftT = rayBoxIntersect(ray, ld3(leftNode->min), ld3(leftNode->max));
                const v2 rightT = rayBoxIntersect(ray, ld3(rightNode->min), ld3(rightNode->max));
                const float leftDist = (leftT.x > 0.0f) ? leftT.x : leftT.y;
                const float rightDist = (rightT.x > 0.0f) ? rightT.x : rightT.y;
                S->cnt->interior_visits++;
                if (stackIndex + 2 > 32) ref_overflow = 1;
                if ((uint64_t)(stackIndex + 2) > S->cnt->ref_stack_max) S->cnt->ref_stack_max = (uint64_t)(stackIndex + 2);
                if (stackIndex + 2 > ORACLE_STACK) { S->overflow = 1; continue; }
                if (leftDist < rightDist) {
                    nodeStack[stackIndex++] = rightChild;
                    nodeStack[stackIndex++] = leftChild;
                } else {
                    nodeStack[stackIndex++] = leftChild;
                    nodeStack[stackIndex++] = rightChild;
                }
            }
        }
    }

    S->cnt->ref_stack_overflow_segments += (uint64_t)ref_overflow;
    if (rec.hit) {
        rec.p = add3(ray->origin, smul3(rec.t, ray->direction));
        rec.front = dot3(ray->direction, rec.normal) < 0.0f;
        if (!rec.front) rec.normal = mul3s(rec.normal, -1.0f);
        S->cnt->hits++;
    }
    return rec;
}

/* pathTracer.comp:213-234 */
static float CalculateReflectance(v3 inDir, v3 normal, float iorA, float iorB)
{
    const float refractRatio = iorA / iorB;
    const float cosAngleIn = -dot3(inDir, normal);
    const float sinSqrAngleOfRefraction = refractRatio * refractRatio * (1.0f - cosAngleIn * cosAngleIn);
    if (sinSqrAngleOfRefraction >= 1.0f) return 1.0f;
    const float cosAngleOfRefraction = sqrtf(1.0f - sinSqrAngleOfRefraction);
    const float denominatorPerpendicular = iorA * cosAngleIn + iorB * cosAngleOfRefraction;
    const float denominatorParallel = iorB * cosAngleIn + iorA * cosAngleOfRefraction;
    if (fmin_nn(denominatorPerpendicular, denominatorParallel) < 1e-8f) return 1.0f;
    float rPerpendicular = (iorA * cosAngleIn - iorB * cosAngleOfRefraction) / denominatorPerpendicular;
    rPerpendicular *= rPerpendicular;
    float rParallel = (iorB * cosAngleIn - iorA * cosAngleOfRefraction) / denominatorParallel;
    rParallel *= rParallel;
    return (rPerpendicular + rParallel) / 2.0f;
}

/* pathTracer.comp:236-239 */
static inline v3 ray_color(const Ray* ray)
{
    const float a = 0.5f * (ray->direction.y + 1.0f);
    const float ia = 1.0f - a;
    return mk3(0.5f * ia + 1.0f * a, 0.7f * ia + 1.0f * a, 1.0f * ia + 1.0f * a);
}

/* pathTracer.comp:241-284 */
static v3 TraceRay(Scene* S, Ray ray, uint32_t* rngState)
{
    v3 totalLight = mk3(0.0f, 0.0f, 0.0f);
    v3 transmittance = mk3(1.0f, 1.0f, 1.0f);
    for (uint32_t i = 0; i <= S->sd->maxBounceCount; i++) {
        const HitInfo hitInfo = Intersect(S, &ray);
        if (!hitInfo.hit) return add3(totalLight, mul3(ray_color(&ray), transmittance));

        const wcpt_material* material = &S->materials[hitInfo.material];
        totalLight = add3(totalLight, mul3(mul3s(ld3(material->emission), material->emissionStrength), transmittance));

        if (material->type == WCPT_MATERIAL_METAL) {
            ray.origin = add3(hitInfo.p, mul3s(hitInfo.normal, kBias));
            {
                const v3 R = reflect3(ray.direction, hitInfo.normal);
                const v3 rd = RandomDirection(rngState);
                ray.direction = normalize3(add3(R, smul3(material->roughness, rd)));
            }
            ray.invDirection = sdiv3(1.0f, ray.direction);
            transmittance = mul3(transmittance, ld3(material->albedo));
        } else {
            const float etaI = hitInfo.front ? 1.0f : material->ior;
            const float etaT = hitInfo.front ? material->ior : 1.0f;
            const float reflectProb = CalculateReflectance(ray.direction, hitInfo.normal, etaI, etaT);
            const v3 R = reflect3(ray.direction, hitInfo.normal);
            const v3 T = refract3(ray.direction, hitInfo.normal, etaI / etaT);
            /* :273 — `||` short-circuits: rand() is consumed only when T != 0 */
            const int followReflection = (T.x == 0.0f && T.y == 0.0f && T.z == 0.0f) ||
                                         (oracle_rand(rngState) <= reflectProb);
            {
                const v3 rd = RandomDirection(rngState);
                ray.direction = normalize3(add3(followReflection ? R : T, smul3(material->roughness, rd)));
            }
            ray.invDirection = sdiv3(1.0f, ray.direction);
            if (!followReflection && !hitInfo.front) {
                const v3 ab = mul3s(mul3s(ld3(material->absorption), -1.0f), material->absorptionStrength);
                const v3 e = mul3s(ab, hitInfo.t);
                transmittance = mul3(transmittance, mk3(wcpt_expf(e.x), wcpt_expf(e.y), wcpt_expf(e.z)));
            }
            ray.origin = add3(hitInfo.p, mul3s(smul3(kBias, hitInfo.normal), sign1(dot3(ray.direction, hitInfo.normal))));
        }
    }
    return totalLight;
}

/* pathTracer.comp:289-324 for one pixel. `px` points at the pixel's float4 in the caller's image. */
static void shade_pixel(Scene* S, uint32_t x, uint32_t y, uint32_t W, uint32_t H, float* px)
{
    const wcpt_scene_data* sd = S->sd;
    const float imgW = (float)W, imgH = (float)H;
    float cx = (float)x / imgW, cy = (float)y / imgH;
    cx = cx + (1.0f / imgW) * 0.5f;
    cy = cy + (1.0f / imgH) * 0.5f;
    cy = 1.0f - cy;
    cx = cx * 2.0f - 1.0f;
    cy = cy * 2.0f - 1.0f;

    /* target = inverseProjection * vec4(cx, cy, 1, 1); column-major m[c*4 + r] */
    const float* P = sd->inverseProjection;
    float tg[4];
    for (int r = 0; r < 4; r++) tg[r] = P[0 * 4 + r] * cx + P[1 * 4 + r] * cy + P[2 * 4 + r] * 1.0f + P[3 * 4 + r] * 1.0f;
    v3 d = normalize3(div3s(mk3(tg[0], tg[1], tg[2]), tg[3]));
    const float* V = sd->inverseView;
    float wd[3];
    for (int r = 0; r < 3; r++) wd[r] = V[0 * 4 + r] * d.x + V[1 * 4 + r] * d.y + V[2 * 4 + r] * d.z + V[3 * 4 + r] * 0.0f;
    const v3 rayDirection = normalize3(mk3(wd[0], wd[1], wd[2]));

    const uint32_t pixel_index = x + y * W + sd->renderedFramesCount * 719393u;
    uint32_t seed = oracle_pcg_hash(pixel_index);

    v3 result = mk3(0.0f, 0.0f, 0.0f);
    for (uint32_t i = 0; i < sd->samples; i++) {
        Ray ray;
        ray.origin = ld3(sd->position);
        ray.direction = rayDirection;
        ray.invDirection = sdiv3(1.0f, rayDirection);
        result = add3(result, TraceRay(S, ray, &seed));
    }
    result = div3s(result, (float)sd->samples);

    const v3 oldRender = mk3(px[0], px[1], px[2]);
    const float weight = 1.0f / (float)(sd->renderedFramesCount + 1u);
    v3 acc = add3(mul3s(oldRender, 1.0f - weight), mul3s(result, weight));
    if (sd->renderedFramesCount == 0) acc = result;
    px[0] = acc.x; px[1] = acc.y; px[2] = acc.z; px[3] = 1.0f;
    S->cnt->pixels++;
}

typedef struct {
    const wcpt_scene_data* sd;
    const wcpt_material* materials;
    const wcpt_sphere* spheres;
    const oracle_draw* draws;
    float* image;
    uint32_t W, H, y0, rows;
    uint32_t* next_row;          /* shared: the next local row to claim */
    wcpt_counters cnt;
    int overflow;
} Job;

static void* run_job(void* arg)
{
    Job* j = (Job*)arg;
    Scene S;
    S.sd = j->sd; S.materials = j->materials; S.spheres = j->spheres; S.draws = j->draws;
    S.cnt = &j->cnt; S.overflow = 0;
    for (;;) {
        const uint32_t ly = __atomic_fetch_add(j->next_row, 1u, __ATOMIC_RELAXED);
        if (ly >= j->rows) break;
        for (uint32_t x = 0; x < j->W; x++)
            shade_pixel(&S, x, j->y0 + ly, j->W, j->H, j->image + ((uint64_t)ly * j->W + x) * 4u);
    }
    j->overflow = S.overflow;
    return NULL;
}

/*
 * Render rows [y0, y0+rows) of a W x H frame into `image` (float4[rows][W], read-modify-write like the
 * reference's imageLoad/imageStore). `threads` host threads (at most 1024) claim rows one at a time, so rows of
 * unequal cost balance across them (every pixel is independent, pathTracer.comp:289-323, and the counters are sums).
 * Returns 0, or WCPT_ERROR_STACK_OVERFLOW if a BVH needed more than ORACLE_STACK entries.
 */
int oracle_render(const wcpt_scene_data* sd, const wcpt_material* materials, const wcpt_sphere* spheres,
                  const oracle_draw* draws, float* image, uint32_t W, uint32_t H, uint32_t y0, uint32_t rows,
                  int threads, wcpt_counters* out)
{
    if (threads < 1) threads = 1;
    if (threads > 1024) threads = 1024;
    if ((uint32_t)threads > rows && rows > 0) threads = (int)rows;
    Job* jobs = (Job*)calloc((size_t)threads, sizeof(Job));
    pthread_t* tids = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !tids) { free(jobs); free(tids); return WCPT_ERROR_OUT_OF_HOST_MEMORY; }
    uint32_t next_row = 0;
    for (int t = 0; t < threads; t++) {
        Job* j = &jobs[t];
        j->sd = sd; j->materials = materials; j->spheres = spheres; j->draws = draws; j->image = image;
        j->W = W; j->H = H; j->y0 = y0; j->rows = rows;
        j->next_row = &next_row;
    }
    if (threads == 1) {
        run_job(&jobs[0]);
    } else {
        for (int t = 0; t < threads; t++) pthread_create(&tids[t], NULL, run_job, &jobs[t]);
        for (int t = 0; t < threads; t++) pthread_join(tids[t], NULL);
    }
    int rc = 0;
    wcpt_counters sum;
    memset(&sum, 0, sizeof(sum));
    for (int t = 0; t < threads; t++) {
        sum.pixels += jobs[t].cnt.pixels;
        sum.segments += jobs[t].cnt.segments;
        sum.sphere_tests += jobs[t].cnt.sphere_tests;
        sum.node_pops += jobs[t].cnt.node_pops;
        sum.interior_visits += jobs[t].cnt.interior_visits;
        sum.triangle_tests += jobs[t].cnt.triangle_tests;
        sum.hits += jobs[t].cnt.hits;
        sum.draw_fetches += jobs[t].cnt.draw_fetches;
        sum.ref_stack_overflow_segments += jobs[t].cnt.ref_stack_overflow_segments;
        if (jobs[t].cnt.ref_stack_max > sum.ref_stack_max) sum.ref_stack_max = jobs[t].cnt.ref_stack_max;
        if (jobs[t].overflow) rc = WCPT_ERROR_STACK_OVERFLOW;
    }
    if (out) *out = sum;
    free(jobs);
    free(tids);
    return rc;
}

/* Known-answer helpers for the intersection primitives (tests/test_oracle.py). */
void oracle_ray_box(const float* o, const float* d, const float* bmin, const float* bmax, float* out2)
{
    Ray r;
    r.origin = ld3(o); r.direction = ld3(d); r.invDirection = sdiv3(1.0f, r.direction);
    v2 t = rayBoxIntersect(&r, ld3(bmin), ld3(bmax));
    out2[0] = t.x; out2[1] = t.y;
}
float oracle_ray_sphere(const float* o, const float* d, const float* c, float radius)
{
    Ray r;
    r.origin = ld3(o); r.direction = ld3(d); r.invDirection = sdiv3(1.0f, r.direction);
    return raySphereIntersectNear(&r, ld3(c), radius);
}
float oracle_ray_triangle(const float* o, const float* d, const float* a, const float* b, const float* c)
{
    Ray r;
    r.origin = ld3(o); r.direction = ld3(d); r.invDirection = sdiv3(1.0f, r.direction);
    return rayTriangleIntersect(&r, ld3(a), ld3(b), ld3(c));
}

/* ------------------------------------------------------------------------------------------------ */
/* PathTracingRenderer.jai:147-217 — midpoint BVH, restated with index-based node access (the reference
 * holds `node` across append(*bvh), :168 vs :196-210) and a signed `j` (the reference's u32 `j -= 3`
 * wraps when first == 0, :178,190). Jai's min/max on Vector3 are per component `a < b ? a : b`.      */
typedef struct {
    const float* pos;
    uint32_t* idx;
    wcpt_node* bvh;
    uint32_t nodesUsed, maxNodes;
    int overflow;
} BvhB;

static inline float jmin(float a, float b) { return a < b ? a : b; }
static inline float jmax(float a, float b) { return a > b ? a : b; }

static void UpdateNodeBounds(BvhB* B, uint32_t nodeIndex)
{
    wcpt_node* node = &B->bvh[nodeIndex];
    for (uint32_t i = 0; i < node->triangleCount; i += 3) {
        const uint32_t index = node->leftNodeOrTriangleIndex + i;
        for (int v = 0; v < 3; v++) {
            const float* p = B->pos + 3u * (uint64_t)B->idx[index + (uint32_t)v];
            for (int c = 0; c < 3; c++) {
                node->min[c] = jmin(node->min[c], p[c]);
                node->max[c] = jmax(node->max[c], p[c]);
            }
        }
    }
}

static void init_node(wcpt_node* n)
{
    for (int c = 0; c < 3; c++) { n->min[c] = 3.40282346638528859812e+38f; n->max[c] = -3.40282346638528859812e+38f; }
    n->leftNodeOrTriangleIndex = 0;
    n->triangleCount = 0;
}

static void Subdivide(BvhB* B, uint32_t nodeIndex, uint32_t depth)
{
    wcpt_node* node = &B->bvh[nodeIndex];
    if (node->triangleCount <= 6 || depth == 0) return;
    float extent[3];
    for (int c = 0; c < 3; c++) extent[c] = node->max[c] - node->min[c];
    int axis = 0;
    if (extent[1] > extent[0]) axis = 1;
    if (extent[2] > extent[axis]) axis = 2;
    const float splitPos = node->min[axis] + extent[axis] * 0.5f;

    int64_t i = node->leftNodeOrTriangleIndex;
    int64_t j = i + (int64_t)node->triangleCount - 3;
    while (i <= j) {
        const float a = B->pos[3u * (uint64_t)B->idx[i + 0] + (uint32_t)axis];
        const float b = B->pos[3u * (uint64_t)B->idx[i + 1] + (uint32_t)axis];
        const float c = B->pos[3u * (uint64_t)B->idx[i + 2] + (uint32_t)axis];
        if ((a + b + c) / 3.0f < splitPos) {
            i += 3;
        } else {
            for (int k = 0; k < 3; k++) { uint32_t t = B->idx[i + k]; B->idx[i + k] = B->idx[j + k]; B->idx[j + k] = t; }
            j -= 3;
        }
    }
    const uint32_t leftCount = (uint32_t)(i - (int64_t)node->leftNodeOrTriangleIndex);
    if (leftCount == 0 || leftCount == node->triangleCount) return;
    if (B->nodesUsed + 2 > B->maxNodes) { B->overflow = 1; return; }

    const uint32_t leftChildIdx = B->nodesUsed++;
    const uint32_t rightChildIdx = B->nodesUsed++;
    init_node(&B->bvh[leftChildIdx]);
    init_node(&B->bvh[rightChildIdx]);
    node = &B->bvh[nodeIndex];
    B->bvh[leftChildIdx].leftNodeOrTriangleIndex = node->leftNodeOrTriangleIndex;
    B->bvh[leftChildIdx].triangleCount = leftCount;
    B->bvh[rightChildIdx].leftNodeOrTriangleIndex = (uint32_t)i;
    B->bvh[rightChildIdx].triangleCount = node->triangleCount - leftCount;
    node->leftNodeOrTriangleIndex = leftChildIdx;
    node->triangleCount = 0;

    UpdateNodeBounds(B, leftChildIdx);
    UpdateNodeBounds(B, rightChildIdx);
    Subdivide(B, leftChildIdx, depth - 1);
    Subdivide(B, rightChildIdx, depth - 1);
}

/* LoadModel's BVH part (PathTracingRenderer.jai:228-232). Returns nodes used, or 0 on overflow. */
uint32_t oracle_bvh_build(const float* positions, uint32_t* indices, uint32_t index_count, wcpt_node* nodes,
                          uint32_t max_nodes)
{
    BvhB B;
    if (max_nodes < 1) return 0;
    B.pos = positions; B.idx = indices; B.bvh = nodes; B.nodesUsed = 0; B.maxNodes = max_nodes; B.overflow = 0;
    init_node(&nodes[0]);
    nodes[0].triangleCount = index_count;
    B.nodesUsed = 1;
    UpdateNodeBounds(&B, 0);
    Subdivide(&B, 0, 32);
    return B.overflow ? 0 : B.nodesUsed;
}

/* ---- composite.comp:3-54 (display step) ------------------------------------------
 * Restated here independently of the product's wcpt_composite.h; only log/exp are the shared deterministic
 * definitions (pow(x, y) = exp(y * log(x)); GLSL leaves pow's precision to the driver). */
static v3 oracle_pbr_neutral(v3 color)                       /* composite.comp:3-23 */
{
    const float startCompression = 0.8f - 0.04f;
    const float desaturation = 0.15f;
    float x = fminf(color.x, fminf(color.y, color.z));
    float offset = x < 0.08f ? x - 6.25f * x * x : 0.04f;
    color.x -= offset;
    color.y -= offset;
    color.z -= offset;
    float peak = fmaxf(color.x, fmaxf(color.y, color.z));
    if (peak < startCompression) return color;
    const float d = 1.0f - startCompression;
    float newPeak = 1.0f - d * d / (peak + d - startCompression);
    float s = newPeak / peak;
    color.x *= s;
    color.y *= s;
    color.z *= s;
    float g = 1.0f - 1.0f / (desaturation * (peak - newPeak) + 1.0f);
    /* GLSL mix(x, y, a) = x * (1 - a) + y * a, y = newPeak * vec3(1) */
    v3 r;
    r.x = color.x * (1.0f - g) + newPeak * g;
    r.y = color.y * (1.0f - g) + newPeak * g;
    r.z = color.z * (1.0f - g) + newPeak * g;
    return r;
}

static float oracle_pow(float x, float y) { return wcpt_expf(y * wcpt_logf(x)); }

/* img: n float4 texels; out32 (n float4) and/or out8 (n RGBA8), either may be NULL */
void oracle_composite(const float* img, uint64_t n, float* out32, uint8_t* out8)
{
    const float gamma = 1.0f / 2.2f;
    for (uint64_t i = 0; i < n; i++) {
        v3 c;
        c.x = oracle_pow(img[4 * i + 0], gamma);               /* composite.comp:47-48 */
        c.y = oracle_pow(img[4 * i + 1], gamma);
        c.z = oracle_pow(img[4 * i + 2], gamma);
        c = oracle_pbr_neutral(c);                             /* :50-51 */
        if (out32) {
            out32[4 * i + 0] = c.x;
            out32[4 * i + 1] = c.y;
            out32[4 * i + 2] = c.z;
            out32[4 * i + 3] = 1.0f;                           /* :53 */
        }
        if (out8) {
            const float v[3] = {c.x, c.y, c.z};
            for (int k = 0; k < 3; k++) {
                float f = v[k];
                uint8_t u;
                if (!(f > 0.0f)) u = 0;
                else if (f >= 1.0f) u = 255;
                else u = (uint8_t)(int)(f * 255.0f + 0.5f);
                out8[4 * i + k] = u;
            }
            out8[4 * i + 3] = 255;
        }
    }
}
