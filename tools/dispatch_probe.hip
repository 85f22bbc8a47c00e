// dispatch_probe.hip — where does block b of a one-round launch run? (XCD, SE, CU, SIMD of each wave via
// s_getreg HW_ID / XCC_ID), for a launch shaped like the megakernel's 135-row block (4080 blocks of 64 threads at
// 4 waves/SIMD). Prints, per SIMD, the blocks it ran, so a tile order can put a heavy and a light tile on each SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o tools/dispatch_probe tools/dispatch_probe.hip && tools/dispatch_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <map>
#include <vector>

__global__ __launch_bounds__(64, 4) void probe(uint32_t* out, uint32_t spin)
{
    __shared__ float pad[2048];                         /* 8 KiB of LDS per wave, like the megakernel */
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   /* HW_REG_HW_ID, 32 bits */
    const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | (0 << 6) | 20); /* HW_REG_XCC_ID */
    float acc = threadIdx.x;
    for (uint32_t i = 0; i < spin; i++) acc = acc * 1.0001f + pad[(threadIdx.x + i) & 2047];
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
    if (acc == 12345.0f) pad[threadIdx.x] = acc;
}

int main(int argc, char** argv)
{
    const uint32_t blocks = argc > 1 ? (uint32_t)atoi(argv[1]) : 4080u;
    uint32_t* d = nullptr;
    (void)hipMalloc(&d, blocks * 8u);
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, 0, d, 20000u);
    (void)hipDeviceSynchronize();
    std::vector<uint32_t> h(blocks * 2u);
    (void)hipMemcpy(h.data(), d, blocks * 8u, hipMemcpyDeviceToHost);
    std::map<uint64_t, std::vector<uint32_t>> simd;
    for (uint32_t b = 0; b < blocks; b++) {
        const uint32_t hw = h[2 * b], xcc = h[2 * b + 1] & 0xF;
        const uint32_t simd_id = (hw >> 4) & 3u, cu = (hw >> 8) & 15u, sh = (hw >> 12) & 1u, se = (hw >> 13) & 7u;
        const uint64_t key = ((uint64_t)xcc << 24) | (se << 16) | (sh << 12) | (cu << 4) | simd_id;
        simd[key].push_back(b);
    }
    printf("{\"blocks\": %u, \"simds_used\": %zu, \"first_blocks_of_simds\": [", blocks, simd.size());
    int k = 0;
    for (auto& kv : simd) {
        if (k++ >= 48) break;
        printf("%s[", k > 1 ? ", " : "");
        for (size_t i = 0; i < kv.second.size(); i++) printf("%s%u", i ? "," : "", kv.second[i]);
        printf("]");
    }
    std::map<size_t, int> hist;
    for (auto& kv : simd) hist[kv.second.size()]++;
    printf("], \"blocks_per_simd_hist\": {");
    k = 0;
    for (auto& kv : hist) printf("%s\"%zu\": %d", k++ ? ", " : "", kv.first, kv.second);
    printf("}}\n");
    (void)hipFree(d);
    return 0;
}
