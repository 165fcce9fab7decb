// ubench_fetch_cal.hip -- calibration of rocprofv3's FETCH_SIZE on gfx950 for
// the access shapes of the pass kernel (MI355X_MICROARCH.md §HBM: the x2 rule is
// calibrated for wide coalesced streams only; "other access widths are
// uncalibrated").  Each kernel moves a KNOWN number of bytes / lines:
//   stream16 : coalesced 16-B-per-lane non-temporal loads over B bytes (the gate's lo stream)
//   stream8  : coalesced  8-B-per-lane non-temporal loads over B bytes (the gate's hi stream)
//   rand8_T  : R random 8-B loads, one per 128-B line at most (distinct lines
//              w.h.p.), from a table of T bytes (T = 8 GB: the {dst, w} gathers;
//              40 MB: the lastFired gathers; 640 KB: the bitmap words)
// Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace`; tools/fetch_cal.py
// divides each dispatch's FETCH_SIZE by the known bytes / reads.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_fetch_cal tools/ubench_fetch_cal.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#define CK(x)                                                         \
    do {                                                              \
        hipError_t e = (x);                                           \
        if (e != hipSuccess) {                                        \
            printf("%s (line %d)\n", hipGetErrorString(e), __LINE__); \
            exit(1);                                                  \
        }                                                             \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ __launch_bounds__(1024) void stream16(const u32x4* p, uint64_t n, uint32_t* out)
{
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 1024) {
        const u32x4 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(1024) void stream8(const u32x2* p, uint64_t n, uint32_t* out)
{
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 1024) {
        const u32x2 v = __builtin_nontemporal_load(p + i);
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// reads random 8-B words, each at the start of a random 128-B line of the table
__global__ __launch_bounds__(1024) void rand8(const uint64_t* tab, uint64_t lines, uint64_t reads, uint64_t salt,
                                              uint32_t* out)
{
    uint64_t acc = 0;
    const uint64_t nthr = (uint64_t)gridDim.x * 1024;
    for (uint64_t t = (uint64_t)blockIdx.x * 1024 + threadIdx.x; t < reads; t += nthr * 4) {
        uint64_t v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint64_t u = t + k * nthr;
            v[k] = u < reads ? tab[__umul64hi(mix64(u ^ salt), lines) * 16] : 0ull;
        }
        acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
    }
    if (acc == 0x12345678ull) out[0] = (uint32_t)acc;
}

int main()
{
    const uint64_t big = 8ull << 30;  // 8 GiB table
    char* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, big));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 1, big));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint64_t sb = 1ull << 30;  // 1 GiB streams
    for (int r = 0; r < 3; ++r) {
        hipLaunchKernelGGL(stream16, dim3(cus * 2), dim3(1024), 0, 0, (const u32x4*)buf, sb / 16, out);
        hipLaunchKernelGGL(stream8, dim3(cus * 2), dim3(1024), 0, 0, (const u32x2*)buf, sb / 8, out);
    }
    const uint64_t reads = 4000000;
    const uint64_t tabs[3] = {big, 40000000ull, 640000ull};
    for (int r = 0; r < 3; ++r)
        for (uint64_t T : tabs)
            hipLaunchKernelGGL(rand8, dim3(cus * 2), dim3(1024), 0, 0, (const uint64_t*)buf, T / 128, reads,
                               (uint64_t)r * 7919 + T, out);
    CK(hipDeviceSynchronize());
    printf("stream16 bytes %llu | stream8 bytes %llu | rand8 reads %llu from tables 8 GiB, 40 MB, 640 KB (dispatch order)\n",
           (unsigned long long)sb, (unsigned long long)sb, (unsigned long long)reads);
    CK(hipFree(buf));
    return 0;
}
