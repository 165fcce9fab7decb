// ubench_random.hip -- the ceiling of random-edge mode's gather: independent
// uniformly random 4-B reads from a table of T bytes (the 4-GB src32 mirror
// at config 3 and smaller tables), 150M reads per launch, every lane keeping
// K reads in flight; indices from a cheap hash (memory only) or from the
// engine's Philox4x32-10 pick (memory + pick arithmetic).  Prints G reads/s.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_random tools/ubench_random.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#define CK(x)                                                    \
    do {                                                         \
        hipError_t e = (x);                                      \
        if (e != hipSuccess) {                                   \
            printf("%s (line %d)\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                             \
        }                                                        \
    } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint64_t philox_pick(uint64_t t, uint64_t pass, uint64_t key, uint64_t n)
{
    uint32_t x0 = (uint32_t)t, x1 = (uint32_t)(t >> 32), x2 = (uint32_t)pass, x3 = (uint32_t)(pass >> 32);
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, x0), lo0 = 0xD2511F53u * x0;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, x2), lo1 = 0xCD9E8D57u * x2;
        x0 = hi1 ^ x1 ^ k0;
        x1 = lo1;
        x2 = hi0 ^ x3 ^ k1;
        x3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return __umul64hi(((uint64_t)x1 << 32) | x0, n);
}

template <int K, bool kPhilox>
__global__ __launch_bounds__(1024) void k_gather(const uint32_t* tab, uint64_t n, uint64_t reads, uint64_t pass,
                                                 uint32_t* out)
{
    const uint64_t nthr = (uint64_t)gridDim.x * 1024, tid = (uint64_t)blockIdx.x * 1024 + threadIdx.x;
    uint32_t acc = 0;
    for (uint64_t base = tid; base < reads; base += nthr * K) {
        uint32_t v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t t = base + (uint64_t)k * nthr;
            const uint64_t i = kPhilox ? philox_pick(t, pass, 0x1234567ull, n) : __umul64hi(mix64(t + pass * reads), n);
            v[k] = t < reads ? __builtin_nontemporal_load(tab + i) : 0u;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc ^= v[k];
    }
    if (acc == 0x12345678u) out[0] = acc;  // keep the loads
}

template <int K, bool kP>
float run(const uint32_t* tab, uint64_t n, uint64_t reads, uint32_t* out, int grid)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_gather<K, kP>), dim3(grid), dim3(1024), 0, 0, tab, n, reads, w, out);
    CK(hipEventRecord(a));
    const int it = 10;
    for (int w = 0; w < it; ++w) hipLaunchKernelGGL((k_gather<K, kP>), dim3(grid), dim3(1024), 0, 0, tab, n, reads, 100 + w, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / it;
}

int main()
{
    const uint64_t reads = 150000000ull;
    const uint64_t maxn = 1000000000ull;  // 4 GB of u32 (the config-3 src32 mirror)
    uint32_t* tab;
    uint32_t* out;
    CK(hipMalloc(&tab, maxn * 4));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(tab, 1, maxn * 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("random 4-B reads, %llu per launch, mean of 10 launches\n", (unsigned long long)reads);
    for (uint64_t n : {maxn, maxn / 4, maxn / 16, (uint64_t)64 << 20}) {
        for (int g : {cus, 2 * cus}) {
            const float a = run<8, false>(tab, n, reads, out, g), b = run<16, false>(tab, n, reads, out, g);
            const float c = run<8, true>(tab, n, reads, out, g);
            printf("table %7.3f GB grid %3d: hash K8 %6.3f ms %5.1f G/s | hash K16 %6.3f ms %5.1f G/s | philox K8 %6.3f ms %5.1f G/s\n",
                   n * 4e-9, g, a, reads / a * 1e-6, b, reads / b * 1e-6, c, reads / c * 1e-6);
        }
    }
    CK(hipFree(tab));
    return 0;
}
