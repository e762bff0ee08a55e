// Occupancy probe (diagnostics, gfx950): how many 256-thread workgroups of a kernel that
// holds V architectural VGPRs and A accumulator registers share a CU at once.  Each
// workgroup spins ~20 us, stamping s_memtime at its start and end with the CU it ran on
// (HW_ID / XCC_ID); the host counts, per CU, the largest number of overlapping intervals.
// Question it answers: does the accumulator file count against the same per-SIMD budget
// as the architectural VGPRs (occupancy = 512 / (V + A)) or not (the LightGlue attention
// tile, 192 + 96 registers, lost 34 % when a dynamic-LDS pad forced one workgroup per CU:
// profiles/r05q_ab_attention_vgpr_scores.txt).
//   hipcc -O3 --offload-arch=gfx950 -o tools/bin/occupancy_probe tools/occupancy_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <vector>

#define CHECK(x)                                                              \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

// V arch VGPRs and A AGPRs reserved through clobbers of the top register of each file
// (the register-usage analysis counts clobbers, not asm text)
#define SPIN(NAME, ...)                                                                   \
    __global__ __launch_bounds__(256) void NAME(unsigned long long* out, int iters) {      \
        const unsigned long long t0 = __builtin_amdgcn_s_memtime();                        \
        float x = threadIdx.x;                                                             \
        for (int i = 0; i < iters; ++i) x = x * 1.0000001f + 0.5f;                         \
        asm volatile("" ::: __VA_ARGS__);                                                      \
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();                        \
        if (threadIdx.x == 0) {                                                            \
            unsigned long long* o = out + (size_t)blockIdx.x * 4;                          \
            o[0] = t0;                                                                     \
            o[1] = t1;                                                                     \
            o[2] = (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11));          \
            o[3] = (unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11));         \
        }                                                                                  \
        if (x == 12345.f) out[0] = 0;                                                      \
    }
SPIN(k_v128, "v127")
SPIN(k_v192, "v191")
SPIN(k_v256, "v255")
SPIN(k_v192a64, "v191", "a63")
SPIN(k_v192a96, "v191", "a95")
SPIN(k_v128a128, "v127", "a127")
SPIN(k_v256a128, "v255", "a127")

typedef void (*KFN)(unsigned long long*, int);
void run(KFN k, const char* name, unsigned long long* d, int nwg) {
    std::vector<unsigned long long> h((size_t)nwg * 4);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k, dim3(nwg), dim3(256), 0, 0, d, 20000);
        CHECK(hipDeviceSynchronize());
    }
    CHECK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
    std::map<long, std::vector<std::pair<unsigned long long, int>>> ev;  // cu -> (time, +1/-1)
    for (int b = 0; b < nwg; ++b) {
        const unsigned long long hw = h[b * 4 + 2], xcc = h[b * 4 + 3];
        const long cu = (long)(xcc & 15) * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15);
        ev[cu].push_back({h[b * 4], +1});
        ev[cu].push_back({h[b * 4 + 1], -1});
    }
    int best = 0;
    for (auto& kv : ev) {
        std::sort(kv.second.begin(), kv.second.end(),
                  [](auto& a, auto& b) { return a.first < b.first || (a.first == b.first && a.second < b.second); });
        int c = 0;
        for (auto& e : kv.second) best = std::max(best, c += e.second);
    }
    printf("{\"kernel\": \"%s\", \"cus\": %zu, \"max_workgroups_per_cu\": %d}\n", name, ev.size(), best);
}

int main() {
    const int nwg = 256 * 8;
    unsigned long long* d;
    CHECK(hipMalloc(&d, (size_t)nwg * 4 * 8));
    run(k_v128, "v128", d, nwg);
    run(k_v192, "v192", d, nwg);
    run(k_v256, "v256", d, nwg);
    run(k_v192a64, "v192+a64", d, nwg);
    run(k_v192a96, "v192+a96", d, nwg);
    run(k_v128a128, "v128+a128", d, nwg);
    run(k_v256a128, "v256+a128", d, nwg);
    CHECK(hipFree(d));
    return 0;
}
