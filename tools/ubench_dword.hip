// ubench_dword.hip -- the SoA gate's stream on its own: 150,000,128 contiguous
// 4-B words (600 MB, the config-3 src array), each wave a contiguous range,
// K dwords per lane in flight, nt loads.  Prints ms and GB/s per shape; under
// `rocprofv3 --pmc FETCH_SIZE` it calibrates FETCH_SIZE for this access width
// (a known 600,000,512 B per launch, MI355X_MICROARCH.md §HBM).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)

template <int BLOCK, int K>
__global__ __launch_bounds__(BLOCK) void k_dword(const uint32_t* src, uint64_t iters, uint32_t* out)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    const uint32_t lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t NWT = (uint64_t)gridDim.x * NW, gw = (uint64_t)blockIdx.x * NW + wid;
    const uint64_t b0 = gw * iters / NWT, b1 = (gw + 1) * iters / NWT;
    uint32_t nxt[K], acc = 0;
    auto issue = [&](uint64_t b) {
        const uint32_t* p = src + b * IE;
#pragma unroll
        for (int k = 0; k < K; ++k) nxt[k] = __builtin_nontemporal_load(p + k * 64 + lane);
    };
    if (b0 < b1) issue(b0);
    for (uint64_t b = b0; b < b1; ++b) {
        uint32_t r[K];
#pragma unroll
        for (int k = 0; k < K; ++k) r[k] = nxt[k];
        if (b + 1 < b1) issue(b + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < K; ++k) acc ^= r[k] * (2u * k + 1u);
    }
    if (acc == 0x12345678u) out[gw] = acc;
}

typedef void (*L)(const uint32_t*, uint64_t, uint32_t*, int);
template <int B, int K>
void launch(const uint32_t* s, uint64_t n, uint32_t* o, int grid)
{
    hipLaunchKernelGGL((k_dword<B, K>), dim3(grid), dim3(B), 0, 0, s, n / (64 * K), o);
}

int main(int argc, char** argv)
{
    const uint64_t n = 150000128ull;
    uint32_t *src, *out;
    CK(hipMalloc(&src, (n + 65536) * 4));
    CK(hipMemset(src, 1, (n + 65536) * 4));
    CK(hipMalloc(&out, 1 << 22));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct V { const char* name; L f; int per_cu; };
    std::vector<V> vs = {
        {"512x8 x2/CU", launch<512, 8>, 2},   {"512x16 x2/CU", launch<512, 16>, 2},
        {"512x32 x2/CU", launch<512, 32>, 2}, {"256x16 x4/CU", launch<256, 16>, 4},
        {"256x32 x4/CU", launch<256, 32>, 4}, {"1024x16 x1/CU", launch<1024, 16>, 1},
        {"512x16 x3/CU", launch<512, 16>, 3}, {"512x16 x4/CU", launch<512, 16>, 4},
    };
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto& v : vs) {
        std::vector<float> t;
        for (int r = 0; r < rounds; ++r) {
            v.f(src, n, out, cus * v.per_cu);  // warm
            CK(hipEventRecord(a));
            v.f(src, n, out, cus * v.per_cu);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const float med = t[t.size() / 2];
        printf("%-16s median %.4f ms  min %.4f ms  %.0f GB/s\n", v.name, med, t[0], n * 4.0 / (med * 1e-3) / 1e9);
    }
    return 0;
}
