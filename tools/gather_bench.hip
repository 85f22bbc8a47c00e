// gather_bench.hip — ceiling of scattered 16-byte-per-lane gathers on gfx950 (the BVH node access pattern).
//
// Each lane follows `steps` pseudo-random 64-byte-aligned records in a table of `table_bytes` and loads
// `loads` x 16 B from each record (global_load_dwordx4). With chain=1 the next record index depends on the
// loaded data (a dependent chain, like BVH traversal); with chain=0 the indices come from a PCG stream.
// coherent=1 makes all 64 lanes of a wave read the same record. Reports lane-loads/s and record-visits/s.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/gather_bench tools/gather_bench.hip && tools/gather_bench [KiB ...]
//
// The last line is a JSON summary: the L2-resident dependent-chain rate (4 MiB table, 4 x 16 B = one 64-B line per
// visit) is the `peak` of bench.py's memory_latency roofline (profiles/gather_ceiling.json).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__device__ __forceinline__ uint32_t pcg(uint32_t s)
{
    uint32_t st = s * 747796405u + 2891336453u;
    uint32_t w = ((st >> ((st >> 28u) + 4u)) ^ st) * 277803737u;
    return (w >> 22u) ^ w;
}

template <int LOADS, bool CHAIN, bool COHERENT>
__global__ __launch_bounds__(64) void gather(const uint4* __restrict__ table, uint32_t records, uint32_t steps,
                                             uint32_t* __restrict__ out)
{
    const uint32_t gid = blockIdx.x * 64u + threadIdx.x;
    uint32_t idx = pcg(COHERENT ? blockIdx.x : gid) % records;
    uint32_t acc = 0, s = gid;
    for (uint32_t k = 0; k < steps; k++) {
        const uint4* r = table + (size_t)idx * 4u;
        uint32_t x = 0;
#pragma unroll
        for (int l = 0; l < LOADS; l++) {
            const uint4 v = r[l];
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
        acc += x;
        if (CHAIN) {
            idx = pcg(x ^ (k * 977u) ^ (COHERENT ? blockIdx.x : gid)) % records;
            if (COHERENT) idx = __shfl(idx, 0, 64);
        } else {
            s = pcg(s);
            idx = (COHERENT ? pcg(blockIdx.x * 131u + k) : s) % records;
        }
    }
    out[gid] = acc;
}

template <int LOADS, bool CHAIN, bool COHERENT>
static double run(const uint4* table, uint32_t records, uint32_t steps, uint32_t waves, uint32_t* out)
{
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    hipLaunchKernelGGL((gather<LOADS, CHAIN, COHERENT>), dim3(waves), dim3(64), 0, 0, table, records, steps, out);
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL((gather<LOADS, CHAIN, COHERENT>), dim3(waves), dim3(64), 0, 0, table, records, steps, out);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return ms * 1e-3;
}

int main(int argc, char** argv)
{
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t waves = (uint32_t)cus * 32u;   // 8 waves/SIMD worth of 64-thread blocks
    const uint32_t steps = 256;
    uint32_t* out;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * waves * 64u));
    std::vector<size_t> sizes = {size_t(64) << 10, size_t(4) << 20, size_t(16) << 20, size_t(512) << 20};
    if (argc > 1) {
        sizes.clear();
        for (int i = 1; i < argc; i++) sizes.push_back((size_t)strtoull(argv[i], nullptr, 10) << 10);
    }
    std::vector<std::pair<size_t, double>> chain4;
    for (size_t table_bytes : sizes) {
        const uint32_t records = (uint32_t)(table_bytes / 64);
        uint4* table;
        CHECK(hipMalloc(&table, table_bytes));
        std::vector<uint32_t> h(table_bytes / 4);
        for (size_t i = 0; i < h.size(); i++) h[i] = (uint32_t)(i * 2654435761u);
        CHECK(hipMemcpy(table, h.data(), table_bytes, hipMemcpyHostToDevice));
        struct R { const char* name; double s; int loads; };
        std::vector<R> rs;
        rs.push_back({"indep  1x16B", run<1, false, false>(table, records, steps, waves, out), 1});
        rs.push_back({"indep  4x16B", run<4, false, false>(table, records, steps, waves, out), 4});
        rs.push_back({"chain  1x16B", run<1, true, false>(table, records, steps, waves, out), 1});
        rs.push_back({"chain  4x16B", run<4, true, false>(table, records, steps, waves, out), 4});
        rs.push_back({"cohrnt 4x16B", run<4, true, true>(table, records, steps, waves, out), 4});
        chain4.push_back({table_bytes, (double)waves * 64.0 * steps / rs[3].s * 1e-9});
        for (auto& r : rs) {
            const double visits = (double)waves * 64.0 * steps;
            const double lane_loads = visits * r.loads;
            printf("table %7zu KiB  %-13s %8.3f ms  %8.2f G record-visits/s  %8.2f G lane-loads/s  %6.3f lane-loads/clk/CU @2.4GHz  %7.1f GB/s\n",
                   table_bytes >> 10, r.name, r.s * 1e3, visits / r.s * 1e-9, lane_loads / r.s * 1e-9,
                   lane_loads / r.s / cus / 2.4e9, lane_loads * 16.0 / r.s * 1e-9);
        }
        CHECK(hipFree(table));
    }
    CHECK(hipFree(out));
    printf("{\"chain_64B_glines_per_s\": {");
    double l2 = 0.0;
    for (size_t i = 0; i < chain4.size(); i++) {
        printf("%s\"%zu KiB\": %.2f", i ? ", " : "", chain4[i].first >> 10, chain4[i].second);
        if (chain4[i].first == (size_t(4) << 20)) l2 = chain4[i].second;
    }
    printf("}, \"l2_resident_chain_glines_per_s\": %.2f, \"waves_per_simd\": 8}\n", l2);
    return 0;
}
