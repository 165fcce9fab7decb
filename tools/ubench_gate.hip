// ubench_gate.hip -- design-space micro-benchmark for the streaming gate kernel
// (not part of the product).  Synthetic data with the shape of config 3:
// 150M 16-B records streamed once per launch, 5,000,512 neurons, ~15k "recent"
// source neurons (the steady-state pre-gate density, ~0.2-0.3 % of events).
//
//   A  stream only                     : the HBM floor for 16 B/event
//   B  stream + global bitmap gather   : the r01 product design
//   C  stream + LDS filter (persistent): hashed 1-bit filter in LDS, exact
//                                        global-bitmap check only on a hit
// Each variant xor-folds what it read into one word per block (no DCE).
// build: hipcc --offload-arch=gfx950 -O3 -o /tmp/ubench tools/ubench_gate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e = (x);                                                          \
        if (e != hipSuccess) {                                                       \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4_t ld_nt(const u32x4_t* p) { return __builtin_nontemporal_load(p); }

constexpr int B = 256;

template <int K, bool NT>
__global__ __launch_bounds__(B) void k_stream(const u32x4_t* syn, uint64_t n, uint32_t* out)
{
    const uint64_t base = (uint64_t)blockIdx.x * B * K;
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint64_t t = base + k * B + threadIdx.x;
        if (t < n) {
            u32x4_t r = NT ? ld_nt(syn + t) : syn[t];
            acc ^= r.x + r.y * 3 + r.z;
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int K, bool NT>
__global__ __launch_bounds__(B) void k_stream_bitmap(const u32x4_t* syn, uint64_t n,
                                                     const uint32_t* bm, uint32_t* out)
{
    const uint64_t base = (uint64_t)blockIdx.x * B * K;
    u32x4_t r[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint64_t t = base + k * B + threadIdx.x;
        r[k] = t < n ? (NT ? ld_nt(syn + t) : syn[t]) : u32x4_t{0, 0, 0, 0};
    }
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uint32_t s = r[k].x;
        acc += (bm[s >> 5] >> (s & 31)) & 1u;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// Persistent: each block keeps a FILTER_BITS-bit hashed filter in LDS; a hit is
// confirmed against the exact global bitmap.  Grid-stride over chunks with the
// next chunk's loads issued before the current chunk's lookups.
template <int K, int FILTER_WORDS>
__global__ __launch_bounds__(B) void k_stream_lds(const u32x4_t* syn, uint64_t n, const uint32_t* bm,
                                                  const uint32_t* filt, uint32_t* out)
{
    __shared__ uint32_t f[FILTER_WORDS];
    for (int i = threadIdx.x; i < FILTER_WORDS; i += B) f[i] = filt[i];
    __syncthreads();
    const uint64_t chunk = (uint64_t)B * K;
    const uint64_t nch = (n + chunk - 1) / chunk;
    uint32_t acc = 0;
    u32x4_t r[K];
    uint64_t c = blockIdx.x;
    if (c < nch) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint64_t t = c * chunk + k * B + threadIdx.x;
            r[k] = t < n ? ld_nt(syn + t) : u32x4_t{0, 0, 0, 0};
        }
    }
    for (; c < nch; c += gridDim.x) {
        uint32_t src[K];
#pragma unroll
        for (int k = 0; k < K; ++k) src[k] = r[k].x;
        const uint64_t cn = c + gridDim.x;
        if (cn < nch) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                uint64_t t = cn * chunk + k * B + threadIdx.x;
                r[k] = t < n ? ld_nt(syn + t) : u32x4_t{0, 0, 0, 0};
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uint32_t h = (src[k] * 0x9E3779B1u) >> (32 - __builtin_ctz(FILTER_WORDS * 32));
            if ((f[h >> 5] >> (h & 31)) & 1u) acc += (bm[src[k] >> 5] >> (src[k] & 31)) & 1u;
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

__global__ void k_fill(u32x4_t* syn, uint64_t n, uint32_t n_nrn)
{
    for (uint64_t i = (uint64_t)blockIdx.x * B + threadIdx.x; i < n; i += (uint64_t)gridDim.x * B) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        syn[i] = u32x4_t{(uint32_t)((z >> 32) * n_nrn >> 32), (uint32_t)((z & 0xffffffffu) * n_nrn >> 32),
                         0x3e000000u, 0u};
    }
}

template <typename F>
float time_it(F f, int reps)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int main()
{
    const uint64_t n = 150000128ull;
    const uint32_t n_nrn = 5000512u;
    const int nwords = (n_nrn + 31) / 32;
    u32x4_t* syn;
    uint32_t *bm, *out, *filt64k, *filt128k;
    CK(hipMalloc(&syn, n * 16));
    CK(hipMalloc(&bm, nwords * 4));
    CK(hipMalloc(&out, 1 << 22));
    CK(hipMalloc(&filt64k, 65536));
    CK(hipMalloc(&filt128k, 131072));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(B), 0, 0, syn, n, n_nrn);
    std::vector<uint32_t> h(nwords, 0), f64(16384, 0), f128(32768, 0);
    srand(1);
    int set = 0;
    for (int i = 0; i < 15000; ++i) {
        uint32_t s = ((uint64_t)rand() * 2654435761u) % n_nrn;
        h[s >> 5] |= 1u << (s & 31);
        uint32_t h1 = (s * 0x9E3779B1u) >> (32 - 19);  // 512k bits
        uint32_t h2 = (s * 0x9E3779B1u) >> (32 - 20);  // 1M bits
        f64[h1 >> 5] |= 1u << (h1 & 31);
        f128[h2 >> 5] |= 1u << (h2 & 31);
        ++set;
    }
    CK(hipMemcpy(bm, h.data(), nwords * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(filt64k, f64.data(), 65536, hipMemcpyHostToDevice));
    CK(hipMemcpy(filt128k, f128.data(), 131072, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    const double gb = n * 16.0 / 1e9;
    auto rep = [&](const char* name, float ms) {
        printf("%-44s %8.4f ms  %7.1f GB/s stream  %6.1f Gev/s\n", name, ms, gb / ms * 1e3, n / ms / 1e6);
    };
#define RUN_STREAM(K, NT)                                                                          \
    rep("A stream K=" #K " nt=" #NT, time_it([&] {                                                 \
            hipLaunchKernelGGL((k_stream<K, NT>), dim3((n + B * K - 1) / (B * K)), dim3(B), 0, 0, syn, n, out); \
        }, 10));
    RUN_STREAM(4, true) RUN_STREAM(8, true) RUN_STREAM(16, true) RUN_STREAM(8, false) RUN_STREAM(16, false)
#define RUN_BM(K, NT)                                                                              \
    rep("B stream+global bitmap K=" #K " nt=" #NT, time_it([&] {                                   \
            hipLaunchKernelGGL((k_stream_bitmap<K, NT>), dim3((n + B * K - 1) / (B * K)), dim3(B), 0, 0, syn, n, bm, out); \
        }, 10));
    RUN_BM(4, true) RUN_BM(8, true) RUN_BM(16, true) RUN_BM(8, false)
#define RUN_LDS(K, W, FP, G)                                                                       \
    rep("C lds filter K=" #K " words=" #W " grid=" #G, time_it([&] {                               \
            hipLaunchKernelGGL((k_stream_lds<K, W>), dim3(G), dim3(B), 0, 0, syn, n, bm, FP, out); \
        }, 10));
    RUN_LDS(8, 16384, filt64k, 512) RUN_LDS(8, 16384, filt64k, 1024) RUN_LDS(16, 16384, filt64k, 512)
    RUN_LDS(8, 32768, filt128k, 256) RUN_LDS(16, 32768, filt128k, 256) RUN_LDS(4, 16384, filt64k, 512)
    printf("recent neurons: %d\n", set);
    return 0;
}
