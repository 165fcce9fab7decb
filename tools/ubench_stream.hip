// ubench_stream.hip -- how the assignment of records to persistent waves
// affects the HBM stream rate (config-3 shape: 150M x 16-B records).
//   wave-range : each wave sweeps its own contiguous range (4096 streams)
//   wg-range   : each workgroup sweeps a contiguous range, its waves take
//                consecutive blocks in turn (512 streams, 8-block window)
//   front      : all waves sweep one front (block = round * waves + wave)
//   one-shot   : non-persistent, one block of records per wave
// dwordx4 (whole record) and dword (src word only) loads, nt.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <cstring>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); exit(1); } } while (0)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

enum { WAVE_RANGE = 0, WG_RANGE = 1, FRONT = 2, ONE_SHOT = 3 };

template <int BLOCK, int K, int MODE, bool X4>
__global__ __launch_bounds__(BLOCK) void k(const u32x4_t* syn, uint64_t nblk, uint32_t* out)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    const uint32_t lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint64_t NWT = (uint64_t)gridDim.x * NW, gw = (uint64_t)blockIdx.x * NW + wid;
    uint64_t b0, bend, step;
    if (MODE == WAVE_RANGE) { b0 = gw * nblk / NWT; bend = (gw + 1) * nblk / NWT; step = 1; }
    else if (MODE == WG_RANGE) {
        const uint64_t g0 = (uint64_t)blockIdx.x * nblk / gridDim.x, g1 = (uint64_t)(blockIdx.x + 1) * nblk / gridDim.x;
        b0 = g0 + wid; bend = g1; step = NW;
    } else if (MODE == FRONT) { b0 = gw; bend = nblk; step = NWT; }
    else { b0 = gw; bend = gw + 1 <= nblk ? gw + 1 : nblk; step = 1; }
    uint32_t acc = 0;
    if (X4) {
        u32x4_t nxt[K];
        auto issue = [&](uint64_t b) {
            const u32x4_t* p = syn + b * IE;
#pragma unroll
            for (int kk = 0; kk < K; ++kk) nxt[kk] = __builtin_nontemporal_load(p + kk * 64 + lane);
        };
        if (b0 < bend) issue(b0);
        for (uint64_t b = b0; b < bend; b += step) {
            u32x4_t r[K];
#pragma unroll
            for (int kk = 0; kk < K; ++kk) r[kk] = nxt[kk];
            if (b + step < bend) issue(b + step);
#pragma unroll
            for (int kk = 0; kk < K; ++kk) acc ^= r[kk].x + r[kk].y * 3u + r[kk].z;
        }
    } else {
        const uint32_t* sx = reinterpret_cast<const uint32_t*>(syn);
        uint32_t nxt[K];
        auto issue = [&](uint64_t b) {
            const uint32_t* p = sx + 4 * (b * IE);
#pragma unroll
            for (int kk = 0; kk < K; ++kk) nxt[kk] = __builtin_nontemporal_load(p + 4 * (kk * 64 + lane));
        };
        if (b0 < bend) issue(b0);
        for (uint64_t b = b0; b < bend; b += step) {
            uint32_t r[K];
#pragma unroll
            for (int kk = 0; kk < K; ++kk) r[kk] = nxt[kk];
            if (b + step < bend) issue(b + step);
#pragma unroll
            for (int kk = 0; kk < K; ++kk) acc ^= r[kk] * (kk + 1);
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

struct V { const char* name; void (*launch)(const u32x4_t*, uint64_t, uint32_t*, int); };
template <int BLOCK, int K, int MODE, bool X4>
void L(const u32x4_t* s, uint64_t nblk, uint32_t* o, int grid)
{
    if (MODE == ONE_SHOT) grid = (int)((nblk + BLOCK / 64 - 1) / (BLOCK / 64));
    hipLaunchKernelGGL((k<BLOCK, K, MODE, X4>), dim3(grid), dim3(BLOCK), 0, 0, s, nblk, o);
}

int main()
{
    const uint64_t n = 150000128ull;  // records; multiple of 512
    u32x4_t* syn;
    uint32_t* out;
    CK(hipMalloc(&syn, (n + 4096) * 16));
    CK(hipMemset(syn, 1, (n + 4096) * 16));
    CK(hipMalloc(&out, 1 << 20));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<V> vs = {
        {"x4 512x8 wave-range", L<512, 8, WAVE_RANGE, true>},
        {"x4 512x8 wg-range", L<512, 8, WG_RANGE, true>},
        {"x4 512x8 front", L<512, 8, FRONT, true>},
        {"x4 512x8 one-shot", L<512, 8, ONE_SHOT, true>},
        {"x1 512x8 wave-range", L<512, 8, WAVE_RANGE, false>},
        {"x1 512x8 wg-range", L<512, 8, WG_RANGE, false>},
        {"x1 512x8 front", L<512, 8, FRONT, false>},
        {"x1 512x16 wg-range", L<512, 16, WG_RANGE, false>},
        {"x1 1024x8 wg-range", L<1024, 8, WG_RANGE, false>},
        {"x1 512x8 one-shot", L<512, 8, ONE_SHOT, false>},
        {"x4 512x8 wave-range again", L<512, 8, WAVE_RANGE, true>},
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> t(vs.size());
    for (int round = 0; round < 5; ++round)
        for (size_t v = 0; v < vs.size(); ++v) {
            const int K = strstr(vs[v].name, "x16") ? 16 : 8;
            const uint64_t nblk = n / (64 * K);
            const int grid = cus * 2;
            vs[v].launch(syn, nblk, out, grid);
            CK(hipEventRecord(a));
            for (int r = 0; r < 5; ++r) vs[v].launch(syn, nblk, out, grid);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t[v].push_back(ms / 5);
        }
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-28s median %.4f ms  (%6.1f GB/s)\n", vs[v].name, t[v][2], n * 16 / (t[v][2] * 1e6));
    }
    return 0;
}
