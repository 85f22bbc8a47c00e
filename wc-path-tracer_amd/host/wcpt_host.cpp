/*
 * wcpt_host.cpp — host-side inputs of the hot path: OBJ loader, midpoint BVH builder, camera, scenes.
 *
 *   wcpt_obj_parse      <- src/ModelLoader.jai:60-141   (parse_obj_file; (v,vt,vn) de-dup, fan triangulation)
 *   wcpt_bvh_build      <- src/PathTracingRenderer.jai:147-217 (UpdateNodeBounds / Subdivide), :228-232
 *   wcpt_camera_update  <- src/PathTracingRenderer.jai:22-36   (Camera Update)
 *   wcpt_scene_generate "default" <- src/PathTracingRenderer.jai:322-339 (Init's materials and spheres)
 *
 * No GPU is needed for anything in this file.
 */
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <algorithm>
#include <vector>

#include "../../include/wcpt.h"

namespace {

/* ------------------------------------------------------------------------------------------------ */
/* OBJ loader                                                                                       */

struct VertexKey {
    int64_t v = -1, vt = -1, vn = -1; /* ModelLoader.jai:12-16 */
    bool operator==(const VertexKey& o) const { return v == o.v && vt == o.vt && vn == o.vn; }
};

/* FNV-1a over the low 4 bytes of each index (ModelLoader.jai:20-56); only affects table speed. */
struct VertexKeyHash {
    size_t operator()(const VertexKey& k) const
    {
        uint32_t h = 2166136261u;
        const int64_t parts[3] = {k.v, k.vt, k.vn};
        for (int p = 0; p < 3; p++)
            for (int s = 0; s < 32; s += 8) {
                h ^= (uint32_t)((parts[p] >> s) & 0xFF);
                h *= 16777619u;
            }
        return h;
    }
};

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\v' || c == '\f'; }

struct Span {
    const char* p;
    size_t n;
};

inline Span trim(Span s)
{
    while (s.n && is_ws(s.p[0])) { s.p++; s.n--; }
    while (s.n && is_ws(s.p[s.n - 1])) s.n--;
    return s;
}

/* Jai split(s, sep): every separator splits, empty pieces are kept. */
inline void split(Span s, char sep, std::vector<Span>& out)
{
    out.clear();
    size_t start = 0;
    for (size_t i = 0; i <= s.n; i++) {
        if (i == s.n || s.p[i] == sep) {
            out.push_back(Span{s.p + start, i - start});
            start = i + 1;
        }
    }
}

inline bool eq(Span s, const char* lit)
{
    const size_t n = strlen(lit);
    return s.n == n && memcmp(s.p, lit, n) == 0;
}

/* string_to_float: leading float of the token, 0 when none parses. */
inline float to_float(Span s)
{
    char buf[128];
    const size_t n = s.n < sizeof(buf) - 1 ? s.n : sizeof(buf) - 1;
    memcpy(buf, s.p, n);
    buf[n] = 0;
    char* end = nullptr;
    const float v = strtof(buf, &end);
    return end == buf ? 0.0f : v;
}

/* string_to_int: optional sign then decimal digits; 0 when there are no digits. */
inline int64_t to_int(Span s)
{
    size_t i = 0;
    bool neg = false;
    if (i < s.n && (s.p[i] == '-' || s.p[i] == '+')) { neg = s.p[i] == '-'; i++; }
    int64_t v = 0;
    bool any = false;
    for (; i < s.n && s.p[i] >= '0' && s.p[i] <= '9'; i++) {
        v = v * 10 + (s.p[i] - '0');
        any = true;
    }
    if (!any) return 0;
    return neg ? -v : v;
}

int obj_parse(const char* text, uint64_t length, wcpt_mesh* out)
{
    std::vector<float> positions;  /* xyz */
    size_t texcoordCount = 0, normalCount = 0;
    std::vector<float> outPos;
    std::vector<uint32_t> outIdx;
    std::unordered_map<VertexKey, uint32_t, VertexKeyHash> vertexMap;
    std::vector<Span> lines, tokens, parts;
    std::vector<uint32_t> face;

    split(Span{text, (size_t)length}, '\n', lines);
    for (const Span& line : lines) {
        const Span t = trim(line);
        if (t.n == 0 || t.p[0] == '#') continue;
        split(t, ' ', tokens);
        if (tokens.empty()) continue;
        const Span cmd = tokens[0];
        if (eq(cmd, "v") && tokens.size() >= 4) {
            positions.push_back(to_float(tokens[1]));
            positions.push_back(to_float(tokens[2]));
            positions.push_back(to_float(tokens[3]));
        } else if (eq(cmd, "vt") && tokens.size() >= 3) {
            texcoordCount++;
        } else if (eq(cmd, "vn") && tokens.size() >= 4) {
            normalCount++;
        } else if (eq(cmd, "f") && tokens.size() >= 4) {
            face.clear();
            for (size_t i = 1; i < tokens.size(); i++) {
                split(tokens[i], '/', parts);
                VertexKey key;
                if (parts.size() >= 1 && parts[0].n > 0) key.v = to_int(parts[0]) - 1;
                if (parts.size() >= 2 && parts[1].n > 0) key.vt = to_int(parts[1]) - 1;
                if (parts.size() >= 3 && parts[2].n > 0) key.vn = to_int(parts[2]) - 1;
                auto it = vertexMap.find(key);
                uint32_t vi;
                if (it != vertexMap.end()) {
                    vi = it->second;
                } else {
                    float p[3] = {0.0f, 0.0f, 0.0f};
                    const int64_t np = (int64_t)(positions.size() / 3);
                    if (key.v >= 0 && key.v < np) {
                        p[0] = positions[3 * key.v + 0];
                        p[1] = positions[3 * key.v + 1];
                        p[2] = positions[3 * key.v + 2];
                    }
                    vi = (uint32_t)(outPos.size() / 3);
                    outPos.push_back(p[0]);
                    outPos.push_back(p[1]);
                    outPos.push_back(p[2]);
                    vertexMap.emplace(key, vi);
                }
                face.push_back(vi);
            }
            for (size_t i = 1; i + 1 < face.size(); i++) { /* fan (:132-136) */
                outIdx.push_back(face[0]);
                outIdx.push_back(face[i]);
                outIdx.push_back(face[i + 1]);
            }
        }
    }
    (void)texcoordCount;
    (void)normalCount;
    out->vertex_count = (uint32_t)(outPos.size() / 3);
    out->index_count = (uint32_t)outIdx.size();
    out->positions = (float*)malloc(outPos.size() * sizeof(float) + 4);
    out->indices = (uint32_t*)malloc(outIdx.size() * sizeof(uint32_t) + 4);
    if (!out->positions || !out->indices) {
        free(out->positions);
        free(out->indices);
        out->positions = nullptr;
        out->indices = nullptr;
        return WCPT_ERROR_OUT_OF_HOST_MEMORY;
    }
    if (!outPos.empty()) memcpy(out->positions, outPos.data(), outPos.size() * sizeof(float));
    if (!outIdx.empty()) memcpy(out->indices, outIdx.data(), outIdx.size() * sizeof(uint32_t));
    return WCPT_SUCCESS;
}

/* ------------------------------------------------------------------------------------------------ */
/* Binned SAH BVH (optional builder behind a flag). Same node format and numbering
 * convention as the midpoint builder: root 0, children allocated as a consecutive pair when their parent splits,
 * leaves = contiguous index-triple ranges, bounds = min/max over the leaf's vertices. The traversal kernels and the
 * oracle consume it unchanged; only the tree differs (and with it the work), so images differ from the midpoint
 * tree's only where two triangles hit at exactly the same t (the reference keeps the first one it tests).
 * Split search: 16 centroid bins per axis, cost = 1 + (A_L N_L + A_R N_R) / A (traversal 1, triangle 1);
 * a node becomes a leaf when no split beats its triangle count (up to kSahMaxLeaf triangles), at 1 triangle, or at
 * kSahMaxDepth (the traversal stack holds 48 entries). Degenerate centroid extents fall back to an object median. */
constexpr int kSahBins = 16;
constexpr uint32_t kSahMaxLeaf = 8;   /* triangles */
constexpr uint32_t kSahMaxDepth = 40;

struct Aabb {
    float lo[3], hi[3];
    void reset() { for (int c = 0; c < 3; c++) { lo[c] = 3.40282347e38f; hi[c] = -3.40282347e38f; } }
    void grow(const float* p) { for (int c = 0; c < 3; c++) { lo[c] = p[c] < lo[c] ? p[c] : lo[c]; hi[c] = p[c] > hi[c] ? p[c] : hi[c]; } }
    void grow(const Aabb& b) { for (int c = 0; c < 3; c++) { lo[c] = b.lo[c] < lo[c] ? b.lo[c] : lo[c]; hi[c] = b.hi[c] > hi[c] ? b.hi[c] : hi[c]; } }
    double area() const
    {
        if (hi[0] < lo[0]) return 0.0;
        const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
        return 2.0 * (x * y + y * z + z * x);
    }
};

int bvh_build_sah(const float* pos, uint32_t* idx, uint32_t index_count, wcpt_node* nodes, uint32_t max_nodes,
                  uint32_t* nodes_used)
{
    const uint32_t ntri = index_count / 3;
    std::vector<Aabb> tb(ntri);
    std::vector<float> cen(3ull * ntri);
    for (uint32_t t = 0; t < ntri; t++) {
        tb[t].reset();
        for (int v = 0; v < 3; v++) tb[t].grow(pos + 3ull * idx[3ull * t + v]);
        for (int c = 0; c < 3; c++) cen[3ull * t + c] = 0.5f * (tb[t].lo[c] + tb[t].hi[c]);
    }
    /* work on a triangle permutation, then rewrite the index buffer in leaf order at the end */
    std::vector<uint32_t> perm(ntri);
    for (uint32_t t = 0; t < ntri; t++) perm[t] = t;
    struct Work { uint32_t node, first, count, depth; };
    std::vector<Work> stack;
    uint32_t used = 1;
    stack.push_back({0, 0, ntri, 0});
    std::vector<uint32_t> tmp;
    while (!stack.empty()) {
        const Work w = stack.back();
        stack.pop_back();
        wcpt_node& node = nodes[w.node];
        Aabb box, cbox;
        box.reset();
        cbox.reset();
        for (uint32_t k = w.first; k < w.first + w.count; k++) {
            box.grow(tb[perm[k]]);
            cbox.grow(&cen[3ull * perm[k]]);
        }
        for (int c = 0; c < 3; c++) {
            node.min[c] = box.lo[c];
            node.max[c] = box.hi[c];
        }
        node.leftNodeOrTriangleIndex = 3u * w.first;
        node.triangleCount = 3u * w.count;
        if (w.count <= 1 || w.depth >= kSahMaxDepth) continue;
        /* best binned split over the three axes */
        double best = 1e300;
        int best_axis = -1, best_bin = -1;
        const double parent_area = box.area();
        for (int a = 0; a < 3; a++) {
            const float ext = cbox.hi[a] - cbox.lo[a];
            if (!(ext > 0.0f)) continue;
            Aabb bb[kSahBins];
            uint32_t bn[kSahBins] = {};
            for (int b = 0; b < kSahBins; b++) bb[b].reset();
            const float scale = (float)kSahBins / ext;
            for (uint32_t k = w.first; k < w.first + w.count; k++) {
                int b = (int)((cen[3ull * perm[k] + a] - cbox.lo[a]) * scale);
                b = b < 0 ? 0 : (b >= kSahBins ? kSahBins - 1 : b);
                bb[b].grow(tb[perm[k]]);
                bn[b]++;
            }
            double right_area[kSahBins];
            uint32_t right_n[kSahBins];
            Aabb acc;
            acc.reset();
            uint32_t n = 0;
            for (int b = kSahBins - 1; b > 0; b--) {
                acc.grow(bb[b]);
                n += bn[b];
                right_area[b] = acc.area();
                right_n[b] = n;
            }
            acc.reset();
            n = 0;
            for (int b = 0; b < kSahBins - 1; b++) {
                acc.grow(bb[b]);
                n += bn[b];
                if (n == 0 || right_n[b + 1] == 0) continue;
                const double cost = acc.area() * n + right_area[b + 1] * right_n[b + 1];
                if (cost < best) {
                    best = cost;
                    best_axis = a;
                    best_bin = b;
                }
            }
        }
        uint32_t left_n = 0;
        if (best_axis >= 0) {
            const double split_cost = 1.0 + best / (parent_area > 0.0 ? parent_area : 1.0);
            if (split_cost >= (double)w.count && w.count <= kSahMaxLeaf) continue; /* leaf is cheaper */
            const float ext = cbox.hi[best_axis] - cbox.lo[best_axis];
            const float scale = (float)kSahBins / ext;
            auto in_left = [&](uint32_t t) {
                int b = (int)((cen[3ull * t + best_axis] - cbox.lo[best_axis]) * scale);
                b = b < 0 ? 0 : (b >= kSahBins ? kSahBins - 1 : b);
                return b <= best_bin;
            };
            uint32_t* beg = perm.data() + w.first;
            left_n = (uint32_t)(std::stable_partition(beg, beg + w.count, in_left) - beg);
        }
        if (left_n == 0 || left_n == w.count) {
            if (w.count <= kSahMaxLeaf) continue;
            /* all centroids in one bin: object median along the longest centroid axis */
            int a = 0;
            for (int c = 1; c < 3; c++)
                if (cbox.hi[c] - cbox.lo[c] > cbox.hi[a] - cbox.lo[a]) a = c;
            uint32_t* beg = perm.data() + w.first;
            std::stable_sort(beg, beg + w.count, [&](uint32_t x, uint32_t y) { return cen[3ull * x + a] < cen[3ull * y + a]; });
            left_n = w.count / 2;
        }
        if (used + 2 > max_nodes) return WCPT_ERROR_OUT_OF_HOST_MEMORY;
        const uint32_t L = used++, R = used++;
        node.leftNodeOrTriangleIndex = L;
        node.triangleCount = 0;
        stack.push_back({R, w.first + left_n, w.count - left_n, w.depth + 1});
        stack.push_back({L, w.first, left_n, w.depth + 1});
    }
    /* index buffer in leaf order */
    tmp.assign(idx, idx + index_count);
    for (uint32_t k = 0; k < ntri; k++)
        for (int v = 0; v < 3; v++) idx[3ull * k + v] = tmp[3ull * perm[k] + v];
    *nodes_used = used;
    return WCPT_SUCCESS;
}

/* ------------------------------------------------------------------------------------------------ */
/* Midpoint BVH. Same node numbering as the reference's recursion (preorder, left subtree first,
 * children allocated as a consecutive pair when their parent splits), written iteratively. */

inline float jmin(float a, float b) { return a < b ? a : b; } /* Jai min: a < b ? a : b */
inline float jmax(float a, float b) { return a > b ? a : b; }

void node_reset(wcpt_node& n)
{
    for (int c = 0; c < 3; c++) {
        n.min[c] = 3.40282346638528859812e+38f;  /* FLOAT32_MAX, PathTracingRenderer.jai:126 */
        n.max[c] = -3.40282346638528859812e+38f;
    }
    n.leftNodeOrTriangleIndex = 0;
    n.triangleCount = 0;
}

void update_bounds(wcpt_node& n, const float* pos, const uint32_t* idx)
{
    for (uint32_t i = 0; i < n.triangleCount; i += 3) {
        for (uint32_t v = 0; v < 3; v++) {
            const float* p = pos + 3ull * idx[n.leftNodeOrTriangleIndex + i + v];
            for (int c = 0; c < 3; c++) {
                n.min[c] = jmin(n.min[c], p[c]);
                n.max[c] = jmax(n.max[c], p[c]);
            }
        }
    }
}

int bvh_build(const float* pos, uint32_t* idx, uint32_t index_count, wcpt_node* nodes, uint32_t max_nodes,
              uint32_t* nodes_used)
{
    struct Work { uint32_t node, depth; };
    std::vector<Work> stack;
    uint32_t used = 1;
    node_reset(nodes[0]);
    nodes[0].triangleCount = index_count;
    update_bounds(nodes[0], pos, idx);
    stack.push_back({0, 32});
    while (!stack.empty()) {
        const Work w = stack.back();
        stack.pop_back();
        wcpt_node& node = nodes[w.node];
        if (node.triangleCount <= 6 || w.depth == 0) continue;
        float extent[3];
        for (int c = 0; c < 3; c++) extent[c] = node.max[c] - node.min[c];
        int axis = 0;
        if (extent[1] > extent[0]) axis = 1;
        if (extent[2] > extent[axis]) axis = 2;
        const float splitPos = node.min[axis] + extent[axis] * 0.5f;
        /* in-place partition of index triples by centroid (:177-192); j is signed */
        int64_t i = node.leftNodeOrTriangleIndex;
        int64_t j = i + (int64_t)node.triangleCount - 3;
        while (i <= j) {
            const float a = pos[3ull * idx[i + 0] + axis];
            const float b = pos[3ull * idx[i + 1] + axis];
            const float c = pos[3ull * idx[i + 2] + axis];
            if ((a + b + c) / 3.0f < splitPos) {
                i += 3;
            } else {
                for (int k = 0; k < 3; k++) std::swap(idx[i + k], idx[j + k]);
                j -= 3;
            }
        }
        const uint32_t leftCount = (uint32_t)(i - (int64_t)node.leftNodeOrTriangleIndex);
        if (leftCount == 0 || leftCount == node.triangleCount) continue;
        if (used + 2 > max_nodes) return WCPT_ERROR_OUT_OF_HOST_MEMORY;
        const uint32_t L = used++, R = used++;
        node_reset(nodes[L]);
        node_reset(nodes[R]);
        nodes[L].leftNodeOrTriangleIndex = node.leftNodeOrTriangleIndex;
        nodes[L].triangleCount = leftCount;
        nodes[R].leftNodeOrTriangleIndex = (uint32_t)i;
        nodes[R].triangleCount = node.triangleCount - leftCount;
        node.leftNodeOrTriangleIndex = L;
        node.triangleCount = 0;
        update_bounds(nodes[L], pos, idx);
        update_bounds(nodes[R], pos, idx);
        stack.push_back({R, w.depth - 1}); /* right subtree after the whole left subtree */
        stack.push_back({L, w.depth - 1});
    }
    *nodes_used = used;
    return WCPT_SUCCESS;
}

/* ------------------------------------------------------------------------------------------------ */
/* Camera (PathTracingRenderer.jai:22-36). The reference uses Jai's Math module (make_look_at_matrix,
 * make_projection_matrix, inverse), which is not available here: this is a GL-convention look-at and
 * perspective (fov vertical, near 0.1, far 100 as at :32). Matrices are boundary data (SceneData), so the
 * parity surface starts after this function. */

struct M4 { double m[4][4]; }; /* row-major */

M4 identity()
{
    M4 r{};
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0;
    return r;
}

bool invert(const M4& a, M4& out)
{
    double t[4][8];
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 8; c++) t[r][c] = c < 4 ? a.m[r][c] : (c - 4 == r ? 1.0 : 0.0);
    for (int col = 0; col < 4; col++) {
        int piv = col;
        for (int r = col + 1; r < 4; r++)
            if (std::fabs(t[r][col]) > std::fabs(t[piv][col])) piv = r;
        if (std::fabs(t[piv][col]) < 1e-300) return false;
        if (piv != col)
            for (int c = 0; c < 8; c++) std::swap(t[piv][c], t[col][c]);
        const double d = t[col][col];
        for (int c = 0; c < 8; c++) t[col][c] /= d;
        for (int r = 0; r < 4; r++) {
            if (r == col) continue;
            const double f = t[r][col];
            if (f == 0.0) continue;
            for (int c = 0; c < 8; c++) t[r][c] -= f * t[col][c];
        }
    }
    for (int r = 0; r < 4; r++)
        for (int c = 0; c < 4; c++) out.m[r][c] = t[r][c + 4];
    return true;
}

void store_colmajor(const M4& a, float* dst)
{
    for (int c = 0; c < 4; c++)
        for (int r = 0; r < 4; r++) dst[c * 4 + r] = (float)a.m[r][c];
}

int camera_update(wcpt_camera* cam, float aspect)
{
    const double kPi = 3.14159265358979323846;
    const double yaw = cam->yaw * kPi / 180.0, pitch = cam->pitch * kPi / 180.0;
    double dir[3] = {std::cos(yaw) * std::cos(pitch), std::sin(pitch), std::sin(yaw) * std::cos(pitch)};
    double dl = std::sqrt(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    for (double& d : dir) d /= dl;
    for (int i = 0; i < 3; i++) cam->direction[i] = (float)dir[i];
    const double eye[3] = {cam->position[0], cam->position[1], cam->position[2]};
    const double up[3] = {0.0, 1.0, 0.0};
    /* s = normalize(cross(f, up)); u = cross(s, f) */
    double s[3] = {dir[1] * up[2] - dir[2] * up[1], dir[2] * up[0] - dir[0] * up[2], dir[0] * up[1] - dir[1] * up[0]};
    double sl = std::sqrt(s[0] * s[0] + s[1] * s[1] + s[2] * s[2]);
    if (sl < 1e-12) { s[0] = 1.0; s[1] = 0.0; s[2] = 0.0; sl = 1.0; } /* looking straight up/down */
    for (double& v : s) v /= sl;
    const double u[3] = {s[1] * dir[2] - s[2] * dir[1], s[2] * dir[0] - s[0] * dir[2], s[0] * dir[1] - s[1] * dir[0]};
    M4 view = identity();
    for (int c = 0; c < 3; c++) {
        view.m[0][c] = s[c];
        view.m[1][c] = u[c];
        view.m[2][c] = -dir[c];
    }
    view.m[0][3] = -(s[0] * eye[0] + s[1] * eye[1] + s[2] * eye[2]);
    view.m[1][3] = -(u[0] * eye[0] + u[1] * eye[1] + u[2] * eye[2]);
    view.m[2][3] = (dir[0] * eye[0] + dir[1] * eye[1] + dir[2] * eye[2]);
    const double fov = (cam->fov > 0.0f ? cam->fov : 90.0f) * kPi / 180.0;
    const double f = 1.0 / std::tan(fov * 0.5);
    const double zn = 0.1, zf = 100.0;
    M4 proj{};
    proj.m[0][0] = f / (double)aspect;
    proj.m[1][1] = f;
    proj.m[2][2] = (zf + zn) / (zn - zf);
    proj.m[2][3] = 2.0 * zf * zn / (zn - zf);
    proj.m[3][2] = -1.0;
    M4 iv, ip;
    if (!invert(view, iv) || !invert(proj, ip)) return WCPT_ERROR_INVALID_ARGUMENT;
    store_colmajor(view, cam->view);
    store_colmajor(proj, cam->projection);
    store_colmajor(iv, cam->inverseView);
    store_colmajor(ip, cam->inverseProjection);
    return WCPT_SUCCESS;
}

/* ------------------------------------------------------------------------------------------------ */
/* Scenes                                                                                           */

wcpt_material default_material() /* PathTracingRenderer.jai:58-70 field defaults */
{
    wcpt_material m;
    memset(&m, 0, sizeof(m));
    m.type = WCPT_MATERIAL_METAL;
    m.absorptionStrength = 1.0f;
    m.ior = 1.0f;
    return m;
}

wcpt_material metal(float r, float g, float b, float rough)
{
    wcpt_material m = default_material();
    m.albedo[0] = r; m.albedo[1] = g; m.albedo[2] = b;
    m.roughness = rough;
    return m;
}

wcpt_sphere sphere(float x, float y, float z, float radius, uint32_t mat)
{
    wcpt_sphere s;
    s.position[0] = x; s.position[1] = y; s.position[2] = z;
    s.radius = radius;
    s.material = mat;
    return s;
}

struct MeshBuilder {
    std::vector<float> pos;
    std::vector<uint32_t> idx;
    uint32_t vert(double x, double y, double z)
    {
        pos.push_back((float)x); pos.push_back((float)y); pos.push_back((float)z);
        return (uint32_t)(pos.size() / 3 - 1);
    }
    void tri(uint32_t a, uint32_t b, uint32_t c) { idx.push_back(a); idx.push_back(b); idx.push_back(c); }
    void quad(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { tri(a, b, c); tri(a, c, d); }
    /* oriented box (rotation about y by `ang` radians) */
    void box(double cx, double cy, double cz, double hx, double hy, double hz, double ang)
    {
        const double ca = std::cos(ang), sa = std::sin(ang);
        uint32_t v[8];
        for (int i = 0; i < 8; i++) {
            const double lx = (i & 1) ? hx : -hx, ly = (i & 2) ? hy : -hy, lz = (i & 4) ? hz : -hz;
            v[i] = vert(cx + ca * lx + sa * lz, cy + ly, cz - sa * lx + ca * lz);
        }
        quad(v[0], v[1], v[3], v[2]); /* -z */
        quad(v[4], v[6], v[7], v[5]); /* +z */
        quad(v[0], v[2], v[6], v[4]); /* -x */
        quad(v[1], v[5], v[7], v[3]); /* +x */
        quad(v[0], v[4], v[5], v[1]); /* -y */
        quad(v[2], v[3], v[7], v[6]); /* +y */
    }
    /* tessellated planar grid: origin + u*i/nu + v*j/nv; cells where skip(i,j) are left open */
    template <class Skip>
    void grid(const double o[3], const double u[3], const double v[3], int nu, int nv, Skip skip)
    {
        std::vector<uint32_t> ids((size_t)(nu + 1) * (nv + 1));
        for (int j = 0; j <= nv; j++)
            for (int i = 0; i <= nu; i++) {
                const double a = (double)i / nu, b = (double)j / nv;
                ids[(size_t)j * (nu + 1) + i] =
                    vert(o[0] + u[0] * a + v[0] * b, o[1] + u[1] * a + v[1] * b, o[2] + u[2] * a + v[2] * b);
            }
        for (int j = 0; j < nv; j++)
            for (int i = 0; i < nu; i++) {
                if (skip(i, j)) continue;
                const uint32_t p00 = ids[(size_t)j * (nu + 1) + i], p10 = ids[(size_t)j * (nu + 1) + i + 1];
                const uint32_t p01 = ids[(size_t)(j + 1) * (nu + 1) + i], p11 = ids[(size_t)(j + 1) * (nu + 1) + i + 1];
                quad(p00, p10, p11, p01);
            }
    }
    /* capped cylinder along +y */
    void cylinder(double cx, double cy, double cz, double r, double h, int seg, int rings)
    {
        const double kPi = 3.14159265358979323846;
        const uint32_t base = (uint32_t)(pos.size() / 3);
        for (int j = 0; j <= rings; j++)
            for (int i = 0; i < seg; i++) {
                const double a = 2.0 * kPi * i / seg;
                /* slight entasis so that the rings are not all coplanar-identical */
                const double rr = r * (1.0 - 0.08 * std::sin(kPi * j / rings));
                vert(cx + rr * std::cos(a), cy + h * j / rings, cz + rr * std::sin(a));
            }
        for (int j = 0; j < rings; j++)
            for (int i = 0; i < seg; i++) {
                const uint32_t a = base + (uint32_t)(j * seg + i), b = base + (uint32_t)(j * seg + (i + 1) % seg);
                const uint32_t c = a + (uint32_t)seg, d = b + (uint32_t)seg;
                quad(a, c, d, b);
            }
        const uint32_t top = vert(cx, cy + h, cz), bot = vert(cx, cy, cz);
        for (int i = 0; i < seg; i++) {
            tri(top, base + (uint32_t)(rings * seg + (i + 1) % seg), base + (uint32_t)(rings * seg + i));
            tri(bot, base + (uint32_t)i, base + (uint32_t)((i + 1) % seg));
        }
    }
    /* half-torus arch in the x-y plane spanning [x0, x1] at height y, depth z, tube radius tr */
    void arch(double x0, double x1, double y, double z, double tr, int seg, int tube)
    {
        const double kPi = 3.14159265358979323846;
        const double R = 0.5 * (x1 - x0), cx = 0.5 * (x0 + x1);
        const uint32_t base = (uint32_t)(pos.size() / 3);
        for (int i = 0; i <= seg; i++) {
            const double a = kPi * i / seg;
            const double px = cx - R * std::cos(a), py = y + R * std::sin(a);
            const double nx = -std::cos(a), ny = std::sin(a);
            for (int k = 0; k < tube; k++) {
                const double b = 2.0 * kPi * k / tube;
                vert(px + tr * std::cos(b) * nx, py + tr * std::cos(b) * ny, z + tr * std::sin(b));
            }
        }
        for (int i = 0; i < seg; i++)
            for (int k = 0; k < tube; k++) {
                const uint32_t a = base + (uint32_t)(i * tube + k), b = base + (uint32_t)(i * tube + (k + 1) % tube);
                quad(a, b, b + (uint32_t)tube, a + (uint32_t)tube);
            }
    }
};

struct Rng { /* xorshift32, deterministic */
    uint32_t s;
    explicit Rng(uint32_t seed) : s(seed ? seed : 0x5EEDu) {}
    uint32_t next() { s ^= s << 13; s ^= s >> 17; s ^= s << 5; return s; }
    double uni() { return (next() >> 8) * (1.0 / 16777216.0); }
};

int fill_scene(wcpt_scene* out, MeshBuilder& mb, const std::vector<wcpt_material>& mats,
               const std::vector<wcpt_sphere>& sph, const wcpt_camera& cam)
{
    memset(out, 0, sizeof(*out));
    out->mesh.vertex_count = (uint32_t)(mb.pos.size() / 3);
    out->mesh.index_count = (uint32_t)mb.idx.size();
    out->mesh.positions = (float*)malloc(mb.pos.size() * sizeof(float) + 4);
    out->mesh.indices = (uint32_t*)malloc(mb.idx.size() * sizeof(uint32_t) + 4);
    out->material_count = (uint32_t)mats.size();
    out->materials = (wcpt_material*)malloc(mats.size() * sizeof(wcpt_material) + 4);
    out->sphere_count = (uint32_t)sph.size();
    out->spheres = (wcpt_sphere*)malloc(sph.size() * sizeof(wcpt_sphere) + 4);
    if (!out->mesh.positions || !out->mesh.indices || !out->materials || !out->spheres) {
        wcpt_scene_free(out);
        return WCPT_ERROR_OUT_OF_HOST_MEMORY;
    }
    if (!mb.pos.empty()) memcpy(out->mesh.positions, mb.pos.data(), mb.pos.size() * sizeof(float));
    if (!mb.idx.empty()) memcpy(out->mesh.indices, mb.idx.data(), mb.idx.size() * sizeof(uint32_t));
    if (!mats.empty()) memcpy(out->materials, mats.data(), mats.size() * sizeof(wcpt_material));
    if (!sph.empty()) memcpy(out->spheres, sph.data(), sph.size() * sizeof(wcpt_sphere));
    out->camera = cam;
    return WCPT_SUCCESS;
}

wcpt_camera make_camera(float x, float y, float z, float yaw, float pitch, float fov)
{
    wcpt_camera c;
    memset(&c, 0, sizeof(c));
    c.position[0] = x; c.position[1] = y; c.position[2] = z;
    c.yaw = yaw;
    c.pitch = pitch;
    c.fov = fov;
    camera_update(&c, 16.0f / 9.0f);
    return c;
}

/* The reference's Init scene (PathTracingRenderer.jai:322-339). variant 1: the "glass" material really is
 * DIELECTRIC (the reference's SetDielectric never sets `type`, :78-82); variant 2: the "Left" sphere's
 * emission is switched on (emissionStrength defaults to 0, :62). */
int scene_default(int variant, wcpt_scene* out)
{
    std::vector<wcpt_material> mats(4, default_material());
    const uint32_t glass = 0, ground = 1, left = 2, right = 3;
    mats[ground].albedo[0] = 0.8f; mats[ground].albedo[1] = 0.8f; mats[ground].albedo[2] = 0.0f;
    mats[ground].roughness = 1.0f;
    for (int c = 0; c < 3; c++) mats[left].emission[c] = 0.8f * 2.0f;
    mats[right].albedo[0] = 0.8f; mats[right].albedo[1] = 0.6f; mats[right].albedo[2] = 0.2f; /* SetMetal */
    mats[right].roughness = 0.75f;
    mats[right].metallic = 0.02f;
    mats[glass].albedo[0] = 0.0f; mats[glass].albedo[1] = 0.5f; mats[glass].albedo[2] = 1.0f; /* SetDielectric */
    mats[glass].roughness = 0.07f;
    mats[glass].ior = 1.5f;
    if (variant == 1) {
        mats[glass].type = WCPT_MATERIAL_DIELECTRIC;
        mats[glass].absorption[0] = 0.8f; mats[glass].absorption[1] = 0.3f; mats[glass].absorption[2] = 0.1f;
    }
    if (variant == 2) mats[left].emissionStrength = 1.0f;
    std::vector<wcpt_sphere> sph = {sphere(0.0f, 0.0f, -1.0f, 0.5f, glass), sphere(-1.0f, 0.0f, -1.0f, 0.5f, left),
                                    sphere(1.0f, 0.0f, -1.0f, 0.5f, right), sphere(0.0f, -100.5f, -1.0f, 100.0f, ground)};
    MeshBuilder mb;
    return fill_scene(out, mb, mats, sph, make_camera(0.0f, 0.0f, 0.0f, -90.0f, 0.0f, 90.0f));
}

/* Cornell-class box: 5 walls + 2 rotated blocks = 34 triangles, open at +z. All triangles use material 0
 * (pathTracer.comp:175), so colour and light come from spheres: an emissive cap in the ceiling, a mirror,
 * a glass (dielectric) and a rough red sphere. Sky light enters through the open front. */
int scene_cornell(wcpt_scene* out)
{
    MeshBuilder mb;
    const double kPi = 3.14159265358979323846;
    auto wall = [&](double ax, double ay, double az, double bx, double by, double bz, double cx, double cy, double cz,
                    double dx, double dy, double dz) {
        mb.quad(mb.vert(ax, ay, az), mb.vert(bx, by, bz), mb.vert(cx, cy, cz), mb.vert(dx, dy, dz));
    };
    wall(-1, -1, 1, 1, -1, 1, 1, -1, -1, -1, -1, -1); /* floor   */
    wall(-1, 1, -1, 1, 1, -1, 1, 1, 1, -1, 1, 1);     /* ceiling */
    wall(-1, -1, -1, 1, -1, -1, 1, 1, -1, -1, 1, -1); /* back    */
    wall(-1, -1, 1, -1, -1, -1, -1, 1, -1, -1, 1, 1); /* left    */
    wall(1, -1, -1, 1, -1, 1, 1, 1, 1, 1, 1, -1);     /* right   */
    mb.box(-0.35, -0.4, -0.3, 0.3, 0.6, 0.3, 17.0 * kPi / 180.0);  /* tall block  */
    mb.box(0.35, -0.7, 0.3, 0.3, 0.3, 0.3, -17.0 * kPi / 180.0);   /* short block */

    std::vector<wcpt_material> mats;
    mats.push_back(metal(0.73f, 0.73f, 0.73f, 1.0f));       /* 0: every triangle */
    wcpt_material light = metal(0.0f, 0.0f, 0.0f, 1.0f);     /* 1: light */
    light.emission[0] = 1.0f; light.emission[1] = 0.85f; light.emission[2] = 0.6f;
    light.emissionStrength = 6.0f;
    mats.push_back(light);
    mats.push_back(metal(0.9f, 0.9f, 0.9f, 0.02f));          /* 2: mirror */
    wcpt_material glass = metal(1.0f, 1.0f, 1.0f, 0.0f);     /* 3: glass */
    glass.type = WCPT_MATERIAL_DIELECTRIC;
    glass.ior = 1.5f;
    glass.absorption[0] = 0.2f; glass.absorption[1] = 0.05f; glass.absorption[2] = 0.01f;
    mats.push_back(glass);
    mats.push_back(metal(0.65f, 0.05f, 0.05f, 0.9f));        /* 4: red */
    std::vector<wcpt_sphere> sph = {sphere(0.0f, 1.35f, 0.0f, 0.5f, 1), sphere(0.35f, -0.15f, 0.3f, 0.25f, 2),
                                    sphere(-0.5f, -0.75f, 0.55f, 0.25f, 3), sphere(0.6f, -0.8f, -0.6f, 0.2f, 4)};
    return fill_scene(out, mb, mats, sph, make_camera(0.0f, 0.0f, 3.4f, -90.0f, 0.0f, 40.0f));
}

/* Deterministic "Sponza-scale" atrium (~262k triangles): a two-storey colonnaded hall with an open roof,
 * tessellated floor and walls with window openings, 40 columns, 36 arches, galleries, draperies and
 * foliage clusters. Sponza itself is not in the container and there is no network. */
int scene_atrium(uint32_t seed, wcpt_scene* out)
{
    MeshBuilder mb;
    Rng rng(seed);
    const double kPi = 3.14159265358979323846;
    const double X = 12.0, Z = 5.0, H = 10.0;
    auto none = [](int, int) { return false; };
    {   /* floor */
        const double o[3] = {-X, 0.0, -Z}, u[3] = {2 * X, 0, 0}, v[3] = {0, 0, 2 * Z};
        mb.grid(o, u, v, 96, 48, none);
    }
    for (int side = 0; side < 2; side++) { /* long walls with two rows of windows */
        const double z = side ? Z : -Z;
        const double o[3] = {-X, 0.0, z}, u[3] = {2 * X, 0, 0}, v[3] = {0, H, 0};
        mb.grid(o, u, v, 96, 40, [](int i, int j) { return (i % 8 >= 3 && i % 8 <= 5) && ((j >= 8 && j < 14) || (j >= 26 && j < 32)); });
    }
    for (int side = 0; side < 2; side++) { /* end walls */
        const double x = side ? X : -X;
        const double o[3] = {x, 0.0, -Z}, u[3] = {0, 0, 2 * Z}, v[3] = {0, H, 0};
        mb.grid(o, u, v, 48, 40, [](int i, int j) { return i >= 20 && i < 28 && j >= 4 && j < 20; });
    }
    for (int level = 0; level < 2; level++) { /* colonnades + arches */
        const double y0 = level ? 5.0 : 0.0, ch = level ? 3.2 : 3.8;
        for (int row = 0; row < 2; row++) {
            const double z = row ? 2.6 : -2.6;
            for (int k = 0; k < 10; k++) {
                const double x = -9.9 + 2.2 * k;
                mb.cylinder(x, y0, z, 0.32, ch, 48, 39);
                if (k < 9) mb.arch(x, x + 2.2, y0 + ch, z, 0.22, 32, 12);
            }
        }
    }
    for (int row = 0; row < 2; row++) { /* gallery slabs */
        const double z = row ? 3.8 : -3.8;
        /* every face tessellated: a single slab-long triangle would give every BVH child the parent's
         * bounds and stall the midpoint split (PathTracingRenderer.jai:175-194) */
        const double top[3] = {-X, 5.0, z - 1.2}, bot[3] = {-X, 4.8, z - 1.2}, u[3] = {2 * X, 0, 0},
                     v[3] = {0, 0, 2.4}, e[3] = {0, 0.2, 0};
        mb.grid(top, u, v, 64, 8, none);
        mb.grid(bot, u, v, 64, 8, none);
        const double f0[3] = {-X, 4.8, z - 1.2}, f1[3] = {-X, 4.8, z + 1.2};
        mb.grid(f0, u, e, 64, 1, none);
        mb.grid(f1, u, e, 64, 1, none);
    }
    for (int d = 0; d < 6; d++) { /* draperies: wavy hanging cloth */
        const double x0 = -9.0 + 3.4 * d, z = (d & 1) ? 3.4 : -3.4;
        const uint32_t base = (uint32_t)(mb.pos.size() / 3);
        const int nu = 32, nv = 48;
        for (int j = 0; j <= nv; j++)
            for (int i = 0; i <= nu; i++) {
                const double a = (double)i / nu, b = (double)j / nv;
                mb.vert(x0 + 1.8 * a, 8.8 - 4.0 * b, z + 0.15 * std::sin(6.0 * kPi * a + 2.0 * b) * (0.3 + b));
            }
        for (int j = 0; j < nv; j++)
            for (int i = 0; i < nu; i++) {
                const uint32_t p00 = base + (uint32_t)(j * (nu + 1) + i);
                mb.quad(p00, p00 + 1, p00 + 1 + (uint32_t)(nu + 1), p00 + (uint32_t)(nu + 1));
            }
    }
    for (int c = 0; c < 24; c++) { /* foliage clusters in pots */
        const double cx = -10.5 + 21.0 * rng.uni(), cz = (c & 1) ? (1.0 + 1.0 * rng.uni()) : -(1.0 + 1.0 * rng.uni());
        mb.cylinder(cx, 0.0, cz, 0.35, 0.6, 16, 2);
        for (int l = 0; l < 1070; l++) {
            const double th = 2.0 * kPi * rng.uni(), ph = 0.5 * kPi * rng.uni(), rr = 0.2 + 0.7 * rng.uni();
            const double px = cx + rr * std::cos(th) * std::cos(ph), py = 0.6 + 0.1 + rr * std::sin(ph) * 1.4,
                         pz = cz + rr * std::sin(th) * std::cos(ph);
            const double s = 0.06 + 0.05 * rng.uni();
            const uint32_t a = mb.vert(px, py, pz);
            const uint32_t b = mb.vert(px + s * (rng.uni() - 0.5) * 2, py + s * rng.uni(), pz + s * (rng.uni() - 0.5) * 2);
            const uint32_t cc = mb.vert(px + s * (rng.uni() - 0.5) * 2, py - s * rng.uni(), pz + s * (rng.uni() - 0.5) * 2);
            mb.tri(a, b, cc);
        }
    }
    std::vector<wcpt_material> mats;
    mats.push_back(metal(0.78f, 0.74f, 0.66f, 0.95f)); /* 0: sandstone, every triangle */
    wcpt_material sun = metal(0.0f, 0.0f, 0.0f, 1.0f);
    sun.emission[0] = 1.0f; sun.emission[1] = 0.9f; sun.emission[2] = 0.7f;
    sun.emissionStrength = 4.0f;
    mats.push_back(sun);                                   /* 1: lantern */
    mats.push_back(metal(0.95f, 0.8f, 0.5f, 0.05f));       /* 2: brass */
    wcpt_material glass = metal(1.0f, 1.0f, 1.0f, 0.0f);
    glass.type = WCPT_MATERIAL_DIELECTRIC;
    glass.ior = 1.45f;
    mats.push_back(glass);                                 /* 3: glass */
    std::vector<wcpt_sphere> sph = {sphere(0.0f, 3.0f, 0.0f, 0.6f, 1), sphere(-4.0f, 0.8f, 0.0f, 0.8f, 2),
                                    sphere(4.0f, 0.8f, 0.0f, 0.8f, 3), sphere(7.5f, 7.5f, 0.0f, 0.5f, 1)};
    return fill_scene(out, mb, mats, sph, make_camera(-11.0f, 2.2f, 0.0f, 0.0f, 6.0f, 70.0f));
}

} // namespace

extern "C" {

int wcpt_obj_parse(const char* text, uint64_t length, wcpt_mesh* out)
{
    if (!out || (!text && length)) return WCPT_ERROR_INVALID_ARGUMENT;
    memset(out, 0, sizeof(*out));
    try {
        return obj_parse(text ? text : "", length, out);
    } catch (...) {
        return WCPT_ERROR_OUT_OF_HOST_MEMORY;
    }
}

int wcpt_obj_load(const char* path, wcpt_mesh* out)
{
    if (!path || !out) return WCPT_ERROR_INVALID_ARGUMENT;
    memset(out, 0, sizeof(*out));
    FILE* f = fopen(path, "rb");
    if (!f) return WCPT_ERROR_PARSE; /* ModelLoader.jai:74-77: "Could not read file" */
    std::string s;
    char buf[1 << 16];
    size_t n;
    while ((n = fread(buf, 1, sizeof(buf), f)) > 0) s.append(buf, n);
    fclose(f);
    return wcpt_obj_parse(s.data(), s.size(), out);
}

void wcpt_mesh_free(wcpt_mesh* mesh)
{
    if (!mesh) return;
    free(mesh->positions);
    free(mesh->indices);
    memset(mesh, 0, sizeof(*mesh));
}

int wcpt_bvh_build(const float* positions, uint32_t vertex_count, uint32_t* indices, uint32_t index_count,
                   wcpt_node* nodes, uint32_t max_nodes, uint32_t* nodes_used)
{
    if (!positions || !indices || !nodes || !nodes_used || max_nodes < 1) return WCPT_ERROR_INVALID_ARGUMENT;
    if (index_count == 0 || index_count % 3 != 0) return WCPT_ERROR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < index_count; i++)
        if (indices[i] >= vertex_count) return WCPT_ERROR_INVALID_ARGUMENT;
    try {
        return bvh_build(positions, indices, index_count, nodes, max_nodes, nodes_used);
    } catch (...) {
        return WCPT_ERROR_OUT_OF_HOST_MEMORY;
    }
}

int wcpt_bvh_build_sah(const float* positions, uint32_t vertex_count, uint32_t* indices, uint32_t index_count,
                       wcpt_node* nodes, uint32_t max_nodes, uint32_t* nodes_used)
{
    if (!positions || !indices || !nodes || !nodes_used || max_nodes < 1) return WCPT_ERROR_INVALID_ARGUMENT;
    if (index_count == 0 || index_count % 3 != 0) return WCPT_ERROR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < index_count; i++)
        if (indices[i] >= vertex_count) return WCPT_ERROR_INVALID_ARGUMENT;
    try {
        return bvh_build_sah(positions, indices, index_count, nodes, max_nodes, nodes_used);
    } catch (...) {
        return WCPT_ERROR_OUT_OF_HOST_MEMORY;
    }
}

int wcpt_camera_update(wcpt_camera* cam, float aspect_ratio)
{
    if (!cam || !(aspect_ratio > 0.0f)) return WCPT_ERROR_INVALID_ARGUMENT;
    return camera_update(cam, aspect_ratio);
}

int wcpt_scene_generate(const char* name, uint32_t seed, wcpt_scene* out)
{
    if (!name || !out) return WCPT_ERROR_INVALID_ARGUMENT;
    try {
        if (!strcmp(name, "default")) return scene_default(0, out);
        if (!strcmp(name, "default_dielectric")) return scene_default(1, out);
        if (!strcmp(name, "default_emissive")) return scene_default(2, out);
        if (!strcmp(name, "cornell")) return scene_cornell(out);
        if (!strcmp(name, "atrium")) return scene_atrium(seed ? seed : 0x5EEDu, out);
    } catch (...) {
        return WCPT_ERROR_OUT_OF_HOST_MEMORY;
    }
    return WCPT_ERROR_INVALID_ARGUMENT;
}

void wcpt_scene_free(wcpt_scene* scene)
{
    if (!scene) return;
    wcpt_mesh_free(&scene->mesh);
    free(scene->materials);
    free(scene->spheres);
    scene->materials = nullptr;
    scene->spheres = nullptr;
    scene->material_count = scene->sphere_count = 0;
}

int wcpt_mesh_to_obj(const wcpt_mesh* mesh, char** out_text, uint64_t* out_length)
{
    if (!mesh || !out_text || !out_length) return WCPT_ERROR_INVALID_ARGUMENT;
    try {
        std::string s;
        s.reserve((size_t)mesh->vertex_count * 40 + (size_t)mesh->index_count * 10 + 64);
        s += "# wcpt generated mesh\n";
        char line[160];
        for (uint32_t v = 0; v < mesh->vertex_count; v++) {
            const float* p = mesh->positions + 3ull * v;
            int n = snprintf(line, sizeof(line), "v %.9g %.9g %.9g\n", p[0], p[1], p[2]);
            s.append(line, (size_t)n);
        }
        for (uint32_t i = 0; i + 2 < mesh->index_count; i += 3) {
            int n = snprintf(line, sizeof(line), "f %u %u %u\n", mesh->indices[i] + 1, mesh->indices[i + 1] + 1,
                             mesh->indices[i + 2] + 1);
            s.append(line, (size_t)n);
        }
        char* t = (char*)malloc(s.size() + 1);
        if (!t) return WCPT_ERROR_OUT_OF_HOST_MEMORY;
        memcpy(t, s.data(), s.size());
        t[s.size()] = 0;
        *out_text = t;
        *out_length = s.size();
        return WCPT_SUCCESS;
    } catch (...) {
        return WCPT_ERROR_OUT_OF_HOST_MEMORY;
    }
}

void wcpt_string_free(char* text) { free(text); }

} /* extern "C" */
