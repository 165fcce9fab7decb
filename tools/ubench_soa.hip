// ubench_soa.hip -- ablation of the SoA gate loop (not product code).
// Config-3-shaped data: 150,000,128 src words (600 MB), the first 65,536 in
// the dense input block (src < 256, all recent), the rest uniform over
// [512, 5,000,512); ~15.6k recent neurons (the 256 inputs + random ones) as
// an exact 625-KB bitmap and a folded LDS filter.  Each variant times the
// same sweep and records per-wave end times (s_memrealtime, 100 MHz).
//
//   S  : stream only (K nt dwords per lane, one iteration prefetched)
//   F  : + LDS filter lookup per event
//   C  : + confirm of filter hits on the exact bitmap (branchy per-k loads)
//   L  : + confirm with a loop over the hit bits (one load per hit)
//   B  : two LDS filters (second hash), confirm only what passes both
//   G  : + stage survivors in LDS (ballot/mbcnt per k), counted
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_soa tools/ubench_soa.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e = (x);                                                              \
        if (e != hipSuccess) {                                                           \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

enum { F_FILTER = 1, F_CONFIRM = 2, F_LOOP = 4, F_BLOOM = 8, F_STAGE = 16, F_EARLY = 32, F_OPT = 64,
       F_SEQ = 128 /* conflict-free LDS addresses */, F_BCAST = 256 /* one LDS address */,
       F_NOCOPY = 512 /* filter not loaded into LDS */, F_NOLOOK = 1024 /* copy only, no lookups */,
       F_GUARD = 2048 /* no prefetch past the range */, F_NOSYNC = 4096, F_NOATOM = 8192,
       F_PRIO = 16384 /* s_setprio: younger waves of a SIMD get higher issue priority */,
       F_ROT = 32768 /* priority rotates with the iteration count: every wave spends equal time at every rank */ };
__device__ __forceinline__ void setprio_rt(uint32_t p)
{
    switch (p & 3) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}
constexpr uint32_t N_NRN = 5000512;

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__host__ __device__ __forceinline__ uint32_t hash2(uint32_t x) { return (x * 0x9E3779B1u) >> 17; }  // 15 high bits

template <int BLOCK, int K, int FW, int FLAGS, int PM = 0xE4 /* prio per age group, 2 bits each */, int ROTM = 7>
__global__ __launch_bounds__(BLOCK) void k_var(const uint32_t* src, uint64_t events, uint32_t iters,
                                               const uint32_t* bitmap, const uint32_t* filt, const uint32_t* filt2,
                                               uint32_t* tot, uint64_t* clk)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    constexpr int F2 = (FLAGS & F_BLOOM) ? FW : 1;
    __shared__ uint32_t s_f[(FLAGS & (F_FILTER | F_BLOOM)) ? FW : 1];
    __shared__ uint32_t s_f2[F2];
    __shared__ uint32_t s_stage[NW][(FLAGS & F_STAGE) ? 512 : 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t NR = gridDim.x * NW, r = blockIdx.x * NW + wid;
    const uint64_t itb = (uint64_t)r * iters / NR, ite = (uint64_t)(r + 1) * iters / NR;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if (FLAGS == 0) {  // exactly ubench_dword's loop
        uint32_t nxt[K], ac = 0;
        auto iss = [&](uint64_t b) {
            const uint32_t* p = src + b * IE;
#pragma unroll
            for (int k = 0; k < K; ++k) nxt[k] = __builtin_nontemporal_load(p + k * 64 + lane);
        };
        if (itb < ite) iss(itb);
        for (uint64_t b = itb; b < ite; ++b) {
            uint32_t rr[K];
#pragma unroll
            for (int k = 0; k < K; ++k) rr[k] = nxt[k];
            if (b + 1 < ite) iss(b + 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int k = 0; k < K; ++k) ac ^= rr[k] * (2u * k + 1u);
        }
        if (lane == 0) clk[r] = __builtin_amdgcn_s_memrealtime() - t0;
        if (ac == 0x12345678u) tot[2 + r] = ac;
        return;
    }
    if ((FLAGS & (F_FILTER | F_BLOOM)) && !(FLAGS & F_NOCOPY))
        for (int i = tid; i < FW; i += BLOCK) s_f[i] = filt[i];
    if (FLAGS & F_BLOOM)
        for (int i = tid; i < FW; i += BLOCK) s_f2[i] = filt2[i];
    uint32_t nx[K];
    auto issue = [&](uint64_t it) {
        if ((FLAGS & F_GUARD) && it >= ite) return;
        const uint32_t* b = src + it * IE;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            nx[k] = __builtin_nontemporal_load(b + k * 64 + lane);
            __builtin_amdgcn_sched_barrier(0);  // keep ascending address order
        }
    };
    if (FLAGS & F_PRIO) {
        const uint32_t age = wid / 4 > 3 ? 3 : wid / 4;  // waves of a workgroup go round-robin over the 4 SIMDs
        const uint32_t pr = (PM >> (2 * age)) & 3;
        if (pr == 1) __builtin_amdgcn_s_setprio(1);
        if (pr == 2) __builtin_amdgcn_s_setprio(2);
        if (pr == 3) __builtin_amdgcn_s_setprio(3);
    }
    issue(itb);
    if (!(FLAGS & F_NOSYNC)) __syncthreads();
    uint32_t acc = 0, pend = 0;
    for (uint64_t it = itb; it < ite; ++it) {
        uint32_t s[K];
#pragma unroll
        for (int k = 0; k < K; ++k) s[k] = nx[k];
        if ((FLAGS & F_ROT) && ((it - itb) & ROTM) == 0) setprio_rt((uint32_t)((it - itb) / (ROTM + 1)) + wid / 4);
        if (FLAGS & F_EARLY) issue(it + 1);
        if (!(FLAGS & (F_FILTER | F_BLOOM)) || (FLAGS & F_NOLOOK)) {
            if (!(FLAGS & F_EARLY)) issue(it + 1);
#pragma unroll
            for (int k = 0; k < K; ++k) acc ^= s[k];
            continue;
        }
        uint32_t fw[K];
        uint32_t fm = 0;
        if (FLAGS & F_OPT) {
            uint32_t f2[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                if (FLAGS & F_SEQ) fw[k] = s_f[((s[k] >> 31) + lane + k * 64) & (FW - 1)];
                else if (FLAGS & F_BCAST) fw[k] = s_f[(s[k] >> 31) + k];
                else fw[k] = s_f[(s[k] >> 5) & (FW - 1)];
                if (FLAGS & F_BLOOM) f2[k] = s_f2[((s[k] >> 5) ^ __umul24(s[k] >> 18, 0x9E5u)) & (FW - 1)];
            }
#pragma unroll
            for (int k = 0; k < K; ++k) {
                uint32_t b = __builtin_amdgcn_ubfe(fw[k], s[k], 1);
                if (FLAGS & F_BLOOM) b &= __builtin_amdgcn_ubfe(f2[k], s[k], 1);
                fm |= b << k;
            }
        } else {
#pragma unroll
        for (int k = 0; k < K; ++k) fw[k] = s_f[(s[k] >> 5) & (FW - 1)];
#pragma unroll
        for (int k = 0; k < K; ++k) fm |= ((fw[k] >> (s[k] & 31u)) & 1u) << k;
        }
        if ((FLAGS & F_BLOOM) && !(FLAGS & F_OPT)) {
            uint32_t f2[K];
#pragma unroll
            for (int k = 0; k < K; ++k) f2[k] = s_f2[hash2(s[k]) & (FW - 1)];
            uint32_t m2 = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) m2 |= ((f2[k] >> (s[k] & 31u)) & 1u) << k;
            fm &= m2;
        }
        uint32_t cw[K];
        if (FLAGS & F_CONFIRM) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                cw[k] = 0xFFFFFFFFu;
                if ((fm >> k) & 1u) cw[k] = bitmap[s[k] >> 5];
            }
        }
        uint32_t lw = 0;  // F_LOOP: confirmed bits
        uint32_t lm = fm, lcw[4], lk[4];
        int nl = 0;
        if (FLAGS & F_LOOP) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                lk[j] = lm ? __builtin_ctz(lm) : 0u;
                uint32_t sv = 0;
#pragma unroll
                for (int k = 0; k < K; ++k) sv = (lk[j] == (uint32_t)k) ? s[k] : sv;
                lcw[j] = lm ? bitmap[sv >> 5] : 0u;
                lm &= lm - 1;
            }
            nl = 4;
        }
        if (!(FLAGS & F_EARLY)) issue(it + 1);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t g = fm;
        if (FLAGS & F_CONFIRM) {
            g = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) g |= ((((fm >> k) & 1u) && ((cw[k] >> (s[k] & 31u)) & 1u)) ? 1u : 0u) << k;
        }
        if (FLAGS & F_LOOP) {
            g = 0;
            uint32_t m = fm;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (m) {
                    uint32_t sv = 0;
#pragma unroll
                    for (int k = 0; k < K; ++k) sv = (lk[j] == (uint32_t)k) ? s[k] : sv;
                    g |= ((lcw[j] >> (sv & 31u)) & 1u) << lk[j];
                }
                m &= m - 1;
            }
            g |= m;  // > 4 hits in one lane: treat the rest as passing (rare)
            (void)nl;
            (void)lw;
        }
        if (FLAGS & F_STAGE) {
            if (__ballot(g != 0) == 0) continue;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool b = (g >> k) & 1u;
                const uint64_t bl = __ballot(b);
                if (b) s_stage[wid][(pend + mbcnt64(bl)) & 511] = (uint32_t)(it * IE + k * 64 + lane);
                pend += (uint32_t)__popcll(bl);
            }
        } else {
            acc += __popc(g);
        }
    }
    if (FLAGS & F_STAGE) acc += pend + s_stage[wid][lane];
    if (lane == 0) clk[r] = __builtin_amdgcn_s_memrealtime() - t0;
    if (acc == 0x7fffffffu) tot[0] = acc;
    if (true) {  // a same-address atomic per wave stalls every concurrent stream (measured): plain store
        if (acc == 0x7ffffffeu) tot[3] = pend;
    } else if (FLAGS & F_STAGE) {
        if (lane == 0) atomicAdd(tot + 1, pend);
    } else {
        acc = acc;
        uint32_t a = acc;
        for (int o = 32; o; o >>= 1) a += __shfl_xor(a, o, 64);
        if (lane == 0) atomicAdd(tot + 1, a);
    }
}

__global__ void k_fill(uint32_t* src, uint64_t n, uint64_t seed)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n + 4096; i += (uint64_t)gridDim.x * 256) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        src[i] = i < 65536 ? (uint32_t)(i >> 8) : 512u + (uint32_t)(((z >> 32) * (N_NRN - 512)) >> 32);
    }
}

typedef void (*Fn)(const uint32_t*, uint64_t, uint32_t, const uint32_t*, const uint32_t*, const uint32_t*, uint32_t*,
                   uint64_t*, int);
template <int B, int K, int FW, int FL, int PM = 0xE4, int ROTM = 7>
void run(const uint32_t* s, uint64_t e, uint32_t it, const uint32_t* bm, const uint32_t* f, const uint32_t* f2,
         uint32_t* t, uint64_t* c, int grid)
{
    hipLaunchKernelGGL((k_var<B, K, FW, FL, PM, ROTM>), dim3(grid), dim3(B), 0, 0, s, e, it, bm, f, f2, t, c);
}

int main(int argc, char** argv)
{
    const uint64_t E = 150000128ull;
    uint32_t *src, *bm, *f, *f2, *tot;
    uint64_t* clk;
    CK(hipMalloc(&src, (E + 4096) * 4));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, src, E, 7ull);
    if (argc > 2 && argv[2][0] == 'm') CK(hipMemset(src, 1, (E + 4096) * 4));  // constant data (ubench_dword)
    const uint32_t words = (N_NRN + 31) / 32;
    std::vector<uint32_t> hb(words, 0);
    uint64_t z = 12345;
    for (int i = 0; i < 256; ++i) hb[i >> 5] |= 1u << (i & 31);
    for (int i = 0; i < 15360; ++i) {
        z = z * 6364136223846793005ull + 1442695040888963407ull;
        const uint32_t n = 512 + (uint32_t)((z >> 33) % (N_NRN - 512));
        hb[n >> 5] |= 1u << (n & 31);
    }
    CK(hipMalloc(&bm, words * 4));
    CK(hipMemcpy(bm, hb.data(), words * 4, hipMemcpyHostToDevice));
    auto fold = [&](int FW, bool second) {
        std::vector<uint32_t> hf(FW, 0);
        for (uint32_t n = 0; n < N_NRN; ++n)
            if ((hb[n >> 5] >> (n & 31)) & 1u) {
                const uint32_t wi = second ? (((n >> 5) ^ ((n >> 18) * 0x9E5u)) & (FW - 1)) : ((n >> 5) & (FW - 1));
                hf[wi] |= 1u << (n & 31);
            }
        return hf;
    };
    CK(hipMalloc(&f, 32768 * 4));
    CK(hipMalloc(&f2, 32768 * 4));
    CK(hipMalloc(&tot, 64));
    CK(hipMalloc(&clk, 65536 * 8));
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    struct V { const char* name; Fn fn; int block, k, fw, per_cu; };
    constexpr int BOGF = F_BLOOM | F_EARLY | F_OPT | F_STAGE | F_GUARD;
    std::vector<V> vs = {
        {"S  1024x8", run<1024, 8, 8192, 0>, 1024, 8, 8192, 1},
        {"BOG 1024x8", run<1024, 8, 8192, BOGF>, 1024, 8, 8192, 1},
        {"BOG prio 0123", run<1024, 8, 8192, BOGF | F_PRIO, 0xE4>, 1024, 8, 8192, 1},
        {"BOG rot 1", run<1024, 8, 8192, BOGF | F_ROT, 0, 0>, 1024, 8, 8192, 1},
        {"BOG rot 4", run<1024, 8, 8192, BOGF | F_ROT, 0, 3>, 1024, 8, 8192, 1},
        {"BOG rot 8", run<1024, 8, 8192, BOGF | F_ROT, 0, 7>, 1024, 8, 8192, 1},
        {"BOG rot 16", run<1024, 8, 8192, BOGF | F_ROT, 0, 15>, 1024, 8, 8192, 1},
    };
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    std::vector<uint64_t> hc(65536);
    for (auto& v : vs) {
        std::vector<uint32_t> hf = fold(v.fw, false), hf2 = fold(v.fw, true);
        CK(hipMemcpy(f, hf.data(), v.fw * 4, hipMemcpyHostToDevice));
        CK(hipMemcpy(f2, hf2.data(), v.fw * 4, hipMemcpyHostToDevice));
        const int grid = cus * v.per_cu;
        const uint32_t iters = (uint32_t)(E / (64ull * v.k));
        std::vector<float> t;
        uint32_t ht[2] = {0, 0};
        for (int r = 0; r < rounds; ++r) {
            CK(hipMemset(tot, 0, 64));
            v.fn(src, E, iters, bm, f, f2, tot, clk, grid);
            CK(hipEventRecord(a));
            v.fn(src, E, iters, bm, f, f2, tot, clk, grid);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms);
            CK(hipMemcpy(ht, tot, 8, hipMemcpyDeviceToHost));
        }
        const int nw = grid * v.block / 64;
        CK(hipMemcpy(hc.data(), clk, nw * 8, hipMemcpyDeviceToHost));
        std::vector<double> d(nw), gm(4, 0.0);
        std::vector<int> gn(4, 0);
        const int NWb = v.block / 64;
        for (int i = 0; i < nw; ++i) {
            d[i] = hc[i] * 0.01;
            const int g = std::min(3, (i % NWb) / 4);
            gm[g] += d[i];
            gn[g]++;
        }
        std::sort(d.begin(), d.end());
        std::sort(t.begin(), t.end());
        printf("%-16s median %.4f ms  (%.0f GB/s)  wave us p10 %.1f p50 %.1f p90 %.1f max %.1f  count %u\n", v.name,
               t[t.size() / 2], E * 4.0 / (t[t.size() / 2] * 1e-3) / 1e9, d[nw / 10], d[nw / 2], d[nw * 9 / 10],
               d[nw - 1], ht[1] / 2);
        printf("    age-group mean us: %.1f %.1f %.1f %.1f\n", gn[0] ? gm[0] / gn[0] : 0, gn[1] ? gm[1] / gn[1] : 0,
               gn[2] ? gm[2] / gn[2] : 0, gn[3] ? gm[3] / gn[3] : 0);
    }
    return 0;
}
