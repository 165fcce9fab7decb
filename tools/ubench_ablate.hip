#include <type_traits>
// ubench_ablate.hip -- ablation study of the gate kernel structure (not product
// code).  Data shaped like config 3 in steady state: 150M 16-B records over
// 5,000,512 neurons, ~15.6k recent source neurons (exact bitmap + 64 KiB
// folded filter), lastFired such that ~0.2 % of events pass the pre-gate.
//
// Variants (template flags) -- each times the same sweep:
//   STREAM   : loads only (floor)
//   FILTER   : + LDS filter lookups
//   CONFIRM  : + L2 bitmap confirm on filter hits
//   GATHER   : + lastFired[dst] gather on hits
//   STORE    : + compacted entry stores
// Prefetch depth PF (1 or 2 iterations ahead), K events per lane.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_ablate tools/ubench_ablate.hip
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

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
constexpr int FW = 16384;

__device__ __forceinline__ uint4 ldnt(const uint4* p)
{
    const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

enum { F_FILTER = 1, F_CONFIRM = 2, F_GATHER = 4, F_STORE = 8, F_STAGE = 16, F_PLAIN = 32, F_SKIP = 64,
       F_NOWRITE = 128 /* stage: no LDS write */, F_NOSTORE = 256 /* flush: LDS read, no global store */,
       F_T4 = 512 /* stage 4-B event offsets, 448 per wave: flush ~once per range */ };

template <int BLOCK, int K, int FLAGS, int PF>
__global__ __launch_bounds__(BLOCK) void k_var(const uint4* syn, uint64_t events, uint32_t iters,
                                               const uint32_t* bitmap, const uint32_t* filt,
                                               const uint64_t* lastF, uint4* out, uint32_t* tot,
                                               uint64_t now)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    __shared__ uint32_t s_filter[(FLAGS & F_FILTER) ? FW : 1];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t NR = gridDim.x * NW, r = blockIdx.x * NW + wid;
    const uint64_t itb = (uint64_t)r * iters / NR, ite = (uint64_t)(r + 1) * iters / NR;
    const uint64_t region = itb * IE;
    if (FLAGS & F_FILTER)
        for (int i = tid; i < FW / 4; i += BLOCK)
            reinterpret_cast<uint4*>(s_filter)[i] = reinterpret_cast<const uint4*>(filt)[i];
    uint4 b0[K], b1[K];
    auto issue = [&](uint4* dst, uint64_t it) {
#pragma unroll
        for (int k = 0; k < K; ++k) dst[k] = ldnt(syn + it * IE + k * 64 + lane);
    };
    if (itb < ite) issue(b0, itb);
    if (PF == 2 && itb + 1 < ite) issue(b1, itb + 1);
    __syncthreads();
    uint32_t acc = 0, g2_run = 0;
    for (uint64_t it = itb; it < ite; ++it) {
        uint4 rec[K];
#pragma unroll
        for (int k = 0; k < K; ++k) rec[k] = b0[k];
        if (PF == 2) {
#pragma unroll
            for (int k = 0; k < K; ++k) b0[k] = b1[k];
        }
        uint32_t fm = 0;
        if (FLAGS & F_FILTER) {
            uint32_t fw[K];
#pragma unroll
            for (int k = 0; k < K; ++k) fw[k] = s_filter[(rec[k].x >> 5) & (FW - 1)];
#pragma unroll
            for (int k = 0; k < K; ++k) fm |= ((fw[k] >> (rec[k].x & 31u)) & 1u) << k;
        } else {
#pragma unroll
            for (int k = 0; k < K; ++k) acc ^= rec[k].x + rec[k].y + rec[k].z;
        }
        uint32_t cw[K];
        uint64_t ld[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            cw[k] = 0xFFFFFFFFu;
            ld[k] = 0;
            if ((fm >> k) & 1u) {
                if (FLAGS & F_CONFIRM) cw[k] = bitmap[rec[k].x >> 5];
                if (FLAGS & F_GATHER) ld[k] = lastF[rec[k].y];
            }
        }
        if (PF == 1) {
            if (it + 1 < ite) issue(b0, it + 1);
        } else {
            if (it + 2 < ite) issue(b1, it + 2);
        }
        uint32_t g2m = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (((fm >> k) & 1u) && ((cw[k] >> (rec[k].x & 31u)) & 1u) && now - ld[k] > 2) g2m |= 1u << k;
        if (FLAGS & F_STORE) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint64_t bg = __ballot((g2m >> k) & 1u);
                if ((g2m >> k) & 1u)
                    out[region + g2_run + mbcnt64(bg)] =
                        make_uint4((uint32_t)(it * IE - region) + k * 64 + lane, 0u, rec[k].z, 0u);
                g2_run += (uint32_t)__popcll(bg);
            }
        } else {
            acc += __popc(g2m);
        }
    }
    if (lane == 0) tot[r] = g2_run;
    if (acc == 0x9876543u) tot[r] = acc;
}

// Production-structure loop: straight-line K-load prefetch (dummy block for
// masked lanes), LDS filter, L2 confirm before the prefetch, sched barrier,
// pre-gated events staged in LDS and flushed with nt (or plain) stores.
template <int BLOCK, int K, int FLAGS>
__global__ __launch_bounds__(BLOCK) void k_prod(const uint4* syn, uint64_t events, uint32_t iters,
                                                const uint32_t* bitmap, const uint32_t* filt,
                                                const uint4* dummy, uint4* out, uint32_t* tot)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    constexpr uint32_t kFlushAt = (FLAGS & F_T4) ? 384 : 32, kStage = kFlushAt + 64;
    using Entry = typename std::conditional<(FLAGS & F_T4) != 0, uint32_t, uint4>::type;
    __shared__ uint32_t s_filter[FW];
    __shared__ Entry s_stage[NW][kStage];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t NR = gridDim.x * NW, r = blockIdx.x * NW + wid;
    const uint64_t itb = (uint64_t)r * iters / NR, ite = (uint64_t)(r + 1) * iters / NR;
    const uint64_t region = itb * IE;
    Entry* stage = s_stage[wid];
    for (int i = tid; i < FW / 4; i += BLOCK)
        reinterpret_cast<uint4*>(s_filter)[i] = reinterpret_cast<const uint4*>(filt)[i];
    uint4 nxt[K];
    auto issue = [&](uint64_t it, bool live) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t t = it * IE + k * 64 + lane;
            nxt[k] = ldnt((live && t < events) ? syn + t : dummy + (k * 64 + lane));
        }
    };
    issue(itb, itb < ite);
    __syncthreads();
    uint32_t pend = 0, flushed = 0, sink = 0;
    auto flush = [&]() {
        if constexpr ((FLAGS & F_T4) != 0) {
            uint32_t* o = reinterpret_cast<uint32_t*>(out);
            for (uint32_t q = lane; q < pend; q += 64)
                __builtin_nontemporal_store(stage[q], o + region + flushed + q);
            flushed += pend;
            pend = 0;
            return;
        }
        for (uint32_t q = lane; q < pend; q += 64) {
            const uint4 v = reinterpret_cast<const uint4*>(stage)[q];
            if (FLAGS & F_NOSTORE) sink ^= v.x ^ v.y;
            else if (FLAGS & F_PLAIN) out[region + flushed + q] = v;
            else __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(out + region + flushed + q));
        }
        flushed += pend;
        pend = 0;
    };
    for (uint64_t it = itb; it < ite; ++it) {
        uint4 rec[K];
#pragma unroll
        for (int k = 0; k < K; ++k) rec[k] = nxt[k];
        const uint64_t base = it * IE;
        uint32_t fw[K];
#pragma unroll
        for (int k = 0; k < K; ++k) fw[k] = s_filter[(rec[k].x >> 5) & (FW - 1)];
        uint32_t fm = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) fm |= ((fw[k] >> (rec[k].x & 31u)) & 1u) << k;
        uint32_t cw[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            cw[k] = 0xFFFFFFFFu;
            if ((fm >> k) & 1u) cw[k] = bitmap[rec[k].x >> 5];
        }
        issue(it + 1, it + 1 < ite);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t g1m = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) g1m |= ((((fm >> k) & 1u) && ((cw[k] >> (rec[k].x & 31u)) & 1u)) ? 1u : 0u) << k;
        if (FLAGS & F_SKIP) {
            if (__ballot(g1m != 0) == 0) continue;
        }
        if (FLAGS & F_STAGE) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool g1 = (g1m >> k) & 1u;
                const uint64_t b1 = __ballot(g1);
                if constexpr ((FLAGS & F_T4) != 0) {
                    if (g1) stage[pend + mbcnt64(b1)] = (uint32_t)(base - region) + k * 64 + lane;
                } else {
                    if (!(FLAGS & F_NOWRITE) && g1)
                        reinterpret_cast<uint4*>(stage)[pend + mbcnt64(b1)] =
                            make_uint4((uint32_t)(base - region) + k * 64 + lane, rec[k].y, rec[k].z, 0u);
                }
                pend += (uint32_t)__popcll(b1);
                if (pend >= kFlushAt) flush();
            }
        } else {
            pend += __popc(g1m);
        }
    }
    if (FLAGS & F_STAGE) flush();
    if (lane == 0) tot[r] = flushed + pend;
    if (sink == 0x9876543u) tot[r] = sink;
}

// Software-pipelined production loop: iteration i waits once (record block i
// and the confirmations of i-1 both landed), issues the prefetch of i+1
// immediately, stages iteration i-1's pre-gated events, then runs the filter
// of i and issues its confirmations.
template <int BLOCK, int K, int FLAGS>
__global__ __launch_bounds__(BLOCK) void k_pipe(const uint4* syn, uint64_t events, uint32_t iters,
                                                const uint32_t* bitmap, const uint32_t* filt,
                                                const uint4* dummy, uint4* out, uint32_t* tot)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    constexpr uint32_t kFlushAt = (FLAGS & F_T4) ? 384 : 32, kStage = kFlushAt + 64;
    using Entry = typename std::conditional<(FLAGS & F_T4) != 0, uint32_t, uint4>::type;
    __shared__ uint32_t s_filter[FW];
    __shared__ Entry s_stage[NW][kStage];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t NR = gridDim.x * NW, r = blockIdx.x * NW + wid;
    const uint64_t itb = (uint64_t)r * iters / NR, ite = (uint64_t)(r + 1) * iters / NR;
    const uint64_t region = itb * IE;
    uint4* stage = s_stage[wid];
    for (int i = tid; i < FW / 4; i += BLOCK)
        reinterpret_cast<uint4*>(s_filter)[i] = reinterpret_cast<const uint4*>(filt)[i];
    uint4 nxt[K];
    auto issue = [&](uint64_t it, bool live) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t t = it * IE + k * 64 + lane;
            nxt[k] = ldnt((live && t < events) ? syn + t : dummy + (k * 64 + lane));
        }
    };
    issue(itb, itb < ite);
    __syncthreads();
    uint32_t pend = 0, flushed = 0;
    auto flush = [&]() {
        for (uint32_t q = lane; q < pend; q += 64) {
            const uint4 v = stage[q];
            __builtin_nontemporal_store(u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_t*>(out + region + flushed + q));
        }
        flushed += pend;
        pend = 0;
    };
    // carried from the previous iteration: filter hits, confirmation words, record fields
    uint32_t pfm = 0, pcw[K], px[K], py[K], pz[K];
    uint64_t pbase = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) pcw[k] = px[k] = py[k] = pz[k] = 0;
    for (uint64_t it = itb; it <= ite; ++it) {
        uint4 rec[K];
#pragma unroll
        for (int k = 0; k < K; ++k) rec[k] = nxt[k];   // waits: records of it + confirmations of it-1
        const bool live = it < ite;
        issue(it + 1, it + 1 < ite);                    // prefetch right away
        __builtin_amdgcn_sched_barrier(0);
        // stage iteration it-1
        uint32_t g1m = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) g1m |= ((((pfm >> k) & 1u) && ((pcw[k] >> (px[k] & 31u)) & 1u)) ? 1u : 0u) << k;
        if (__ballot(g1m != 0) != 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool g1 = (g1m >> k) & 1u;
                const uint64_t b1 = __ballot(g1);
                if (g1) stage[pend + mbcnt64(b1)] = make_uint4((uint32_t)(pbase - region) + k * 64 + lane, py[k], pz[k], 0u);
                pend += (uint32_t)__popcll(b1);
                if (pend >= kFlushAt) flush();
            }
        }
        if (!live) break;
        // filter of it, confirmations issued (consumed next iteration)
        uint32_t fm = 0;
        uint32_t fw[K];
#pragma unroll
        for (int k = 0; k < K; ++k) fw[k] = s_filter[(rec[k].x >> 5) & (FW - 1)];
#pragma unroll
        for (int k = 0; k < K; ++k) fm |= ((fw[k] >> (rec[k].x & 31u)) & 1u) << k;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pcw[k] = 0xFFFFFFFFu;
            if ((fm >> k) & 1u) pcw[k] = bitmap[rec[k].x >> 5];
            px[k] = rec[k].x;
            py[k] = rec[k].y;
            pz[k] = rec[k].z;
        }
        pfm = fm;
        pbase = it * IE;
    }
    flush();
    if (lane == 0) tot[r] = flushed;
}

// Pipelined loop with 4-B staged entries (event offset only; dst and w are
// re-read downstream): iteration i waits once, issues the prefetch of i+1
// at once, stages i-1 (its confirmations have landed), then filters i and
// issues its confirmations.  Carried state: confirmation words + bit indices.
template <int BLOCK, int K, int FLAGS>
__global__ __launch_bounds__(BLOCK) void k_pipe4(const uint4* syn, uint64_t events, uint32_t iters,
                                                 const uint32_t* bitmap, const uint32_t* filt,
                                                 const uint4* dummy, uint4* out, uint32_t* tot)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    constexpr uint32_t kFlushAt = 384, kStage = kFlushAt + 64;
    __shared__ uint32_t s_filter[FW];
    __shared__ uint32_t s_stage[NW][kStage];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t NR = gridDim.x * NW, r = blockIdx.x * NW + wid;
    const uint64_t itb = (uint64_t)r * iters / NR, ite = (uint64_t)(r + 1) * iters / NR;
    const uint64_t region = itb * IE;
    uint32_t* stage = s_stage[wid];
    for (int i = tid; i < FW / 4; i += BLOCK)
        reinterpret_cast<uint4*>(s_filter)[i] = reinterpret_cast<const uint4*>(filt)[i];
    uint4 nxt[K];
    auto issue = [&](uint64_t it, bool live) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t t = it * IE + k * 64 + lane;
            nxt[k] = ldnt((live && t < events) ? syn + t : dummy + (k * 64 + lane));
        }
    };
    issue(itb, itb < ite);
    __syncthreads();
    uint32_t pend = 0, flushed = 0;
    uint32_t* o = reinterpret_cast<uint32_t*>(out);
    auto flush = [&]() {
        for (uint32_t q = lane; q < pend; q += 64)
            __builtin_nontemporal_store(stage[q], o + region + flushed + q);
        flushed += pend;
        pend = 0;
    };
    uint32_t pfm = 0, pcw[K], pbit[K];
    uint32_t prel = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) pcw[k] = pbit[k] = 0;
    for (uint64_t it = itb; it <= ite; ++it) {
        uint4 rec[K];
#pragma unroll
        for (int k = 0; k < K; ++k) rec[k] = nxt[k];
        const bool live = it < ite;
        issue(it + 1, it + 1 < ite);
        __builtin_amdgcn_sched_barrier(0);
        uint32_t g1m = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) g1m |= ((((pfm >> k) & 1u) && ((pcw[k] >> pbit[k]) & 1u)) ? 1u : 0u) << k;
        if (__ballot(g1m != 0) != 0) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool g1 = (g1m >> k) & 1u;
                const uint64_t b1 = __ballot(g1);
                if (g1) stage[pend + mbcnt64(b1)] = prel + k * 64 + lane;
                pend += (uint32_t)__popcll(b1);
                if (pend >= kFlushAt) flush();
            }
        }
        if (!live) break;
        uint32_t fw[K];
#pragma unroll
        for (int k = 0; k < K; ++k) fw[k] = s_filter[(rec[k].x >> 5) & (FW - 1)];
        uint32_t fm = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) fm |= ((fw[k] >> (rec[k].x & 31u)) & 1u) << k;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            pcw[k] = 0u;
            if ((fm >> k) & 1u) pcw[k] = bitmap[rec[k].x >> 5];
            pbit[k] = rec[k].x & 31u;
        }
        pfm = fm;
        prel = (uint32_t)(it * IE - region);
    }
    flush();
    if (lane == 0) tot[r] = flushed;
}

__device__ __forceinline__ uint32_t ldnt32(const uint32_t* p) { return __builtin_nontemporal_load(p); }

// x-only gate loop: each lane loads just the src dword of its records (same
// lines from HBM, a quarter of the registers), stages 4-B event offsets.
// Loads use a wave-uniform base (the record buffer is padded, so the last
// iteration reads past the end instead of masking lanes).
// PIPE: stage iteration i-1 after issuing the prefetch of i+1.
template <int BLOCK, int K, int PIPE>
__global__ __launch_bounds__(BLOCK) void k_x(const uint4* syn, uint64_t events, uint32_t iters,
                                             const uint32_t* bitmap, const uint32_t* filt,
                                             const uint4* dummy, uint4* out, uint32_t* tot)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    constexpr uint32_t kStage = 448, kFlushAt = kStage - 64;
    __shared__ uint32_t s_filter[FW];
    __shared__ uint32_t s_stage[NW][kStage];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t NR = gridDim.x * NW, r = blockIdx.x * NW + wid;
    const uint64_t itb = (uint64_t)r * iters / NR, ite = (uint64_t)(r + 1) * iters / NR;
    const uint64_t region = itb * IE;
    uint32_t* stage = s_stage[wid];
    const uint32_t* sx = reinterpret_cast<const uint32_t*>(syn);
    const uint32_t* dx = reinterpret_cast<const uint32_t*>(dummy);
    for (int i = tid; i < FW / 4; i += BLOCK)
        reinterpret_cast<uint4*>(s_filter)[i] = reinterpret_cast<const uint4*>(filt)[i];
    uint32_t nxt[K];
    auto issue = [&](uint64_t it, bool live) {
        const uint32_t* base = live ? sx + 4 * (it * IE) : dx;  // wave-uniform
#pragma unroll
        for (int k = 0; k < K; ++k) nxt[k] = ldnt32(base + 4 * (k * 64 + lane));
    };
    issue(itb, itb < ite);
    __syncthreads();
    uint32_t pend = 0, flushed = 0;
    uint32_t* o = reinterpret_cast<uint32_t*>(out);
    auto flush = [&]() {
        for (uint32_t q = lane; q < pend; q += 64)
            __builtin_nontemporal_store(stage[q], o + region + flushed + q);
        flushed += pend;
        pend = 0;
    };
    auto stage_it = [&](uint32_t g1m, uint32_t rel) {
        if (__ballot(g1m != 0) == 0) return;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const bool g1 = (g1m >> k) & 1u;
            const uint64_t b1 = __ballot(g1);
            if (g1) stage[pend + mbcnt64(b1)] = rel + k * 64 + lane;
            pend += (uint32_t)__popcll(b1);
            if (pend >= kFlushAt) flush();
        }
    };
    if constexpr (PIPE == 0) {
        for (uint64_t it = itb; it < ite; ++it) {
            uint32_t x[K];
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = nxt[k];
            uint32_t vmask = 0xFFFFFFFFu;
            if (it * IE + IE > events) {
                vmask = 0;
#pragma unroll
                for (int k = 0; k < K; ++k) vmask |= (it * IE + k * 64 + lane < events ? 1u : 0u) << k;
            }
            uint32_t fw[K];
#pragma unroll
            for (int k = 0; k < K; ++k) fw[k] = s_filter[(x[k] >> 5) & (FW - 1)];
            uint32_t fm = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) fm |= ((fw[k] >> (x[k] & 31u)) & 1u) << k;
            fm &= vmask;
            uint32_t cw[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                cw[k] = 0u;
                if ((fm >> k) & 1u) cw[k] = bitmap[x[k] >> 5];
            }
            issue(it + 1, it + 1 < ite);
            __builtin_amdgcn_sched_barrier(0);
            uint32_t g1m = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) g1m |= ((cw[k] >> (x[k] & 31u)) & 1u) << k;
            stage_it(g1m, (uint32_t)(it * IE - region));
        }
    } else {
        uint32_t pcw[K], prel = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) pcw[k] = 0;
        for (uint64_t it = itb; it <= ite; ++it) {
            uint32_t x[K];
#pragma unroll
            for (int k = 0; k < K; ++k) x[k] = nxt[k];
            const bool live = it < ite;
            issue(it + 1, it + 1 < ite);
            __builtin_amdgcn_sched_barrier(0);
            // pcw[k] already holds the confirmed bit (shifted down) of iteration it-1
            uint32_t g1m = 0;
#pragma unroll
            for (int k = 0; k < K; ++k) g1m |= (pcw[k] & 1u) << k;
            stage_it(g1m, prel);
            if (!live) break;
            uint32_t vmask = 0xFFFFFFFFu;
            if (it * IE + IE > events) {
                vmask = 0;
#pragma unroll
                for (int k = 0; k < K; ++k) vmask |= (it * IE + k * 64 + lane < events ? 1u : 0u) << k;
            }
            uint32_t fw[K];
#pragma unroll
            for (int k = 0; k < K; ++k) fw[k] = s_filter[(x[k] >> 5) & (FW - 1)];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                // the bit position rides in the low 5 bits of x: keep it beside the word
                const bool hit = ((fw[k] >> (x[k] & 31u)) & 1u) && ((vmask >> k) & 1u);
                pcw[k] = 0u;
                if (hit) pcw[k] = bitmap[x[k] >> 5] >> (x[k] & 31u);
            }
            prel = (uint32_t)(it * IE - region);
        }
    }
    flush();
    if (lane == 0) tot[r] = flushed;
}

__global__ void k_fill(uint4* syn, uint64_t n, uint32_t n_nrn)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        uint64_t z = (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        syn[i] = make_uint4(512 + (uint32_t)(((z >> 32) * (n_nrn - 512)) >> 32),
                            512 + (uint32_t)(((z & 0xffffffffu) * (n_nrn - 512)) >> 32), 0x3e000000u, 0u);
    }
}

template <int BLOCK, int K, int FLAGS>
void launch_prod(int grid, const uint4* syn, uint64_t ev, uint32_t iters, const uint32_t* bm,
                 const uint32_t* f, const uint64_t* lf, uint4* out, uint32_t* tot, uint64_t now)
{
    (void)lf; (void)now;
    hipLaunchKernelGGL((k_prod<BLOCK, K, FLAGS>), dim3(grid), dim3(BLOCK), 0, 0, syn, ev, iters, bm, f,
                       out + ev, out, tot);
}

template <int BLOCK, int K, int FLAGS>
void launch_pipe(int grid, const uint4* syn, uint64_t ev, uint32_t iters, const uint32_t* bm,
                 const uint32_t* f, const uint64_t* lf, uint4* out, uint32_t* tot, uint64_t now)
{
    (void)lf; (void)now;
    hipLaunchKernelGGL((k_pipe<BLOCK, K, FLAGS>), dim3(grid), dim3(BLOCK), 0, 0, syn, ev, iters, bm, f,
                       out + ev, out, tot);
}

template <int BLOCK, int K, int FLAGS>
void launch_pipe4(int grid, const uint4* syn, uint64_t ev, uint32_t iters, const uint32_t* bm,
                  const uint32_t* f, const uint64_t* lf, uint4* out, uint32_t* tot, uint64_t now)
{
    (void)lf; (void)now;
    hipLaunchKernelGGL((k_pipe4<BLOCK, K, FLAGS>), dim3(grid), dim3(BLOCK), 0, 0, syn, ev, iters, bm, f,
                       out + ev, out, tot);
}

template <int BLOCK, int K, int PIPE>
void launch_x(int grid, const uint4* syn, uint64_t ev, uint32_t iters, const uint32_t* bm,
              const uint32_t* f, const uint64_t* lf, uint4* out, uint32_t* tot, uint64_t now)
{
    (void)lf; (void)now;
    hipLaunchKernelGGL((k_x<BLOCK, K, PIPE>), dim3(grid), dim3(BLOCK), 0, 0, syn, ev, iters, bm, f,
                       out + ev, out, tot);
}

struct Var {
    const char* name;
    void (*launch)(int, const uint4*, uint64_t, uint32_t, const uint32_t*, const uint32_t*,
                   const uint64_t*, uint4*, uint32_t*, uint64_t);
    int block, k;
};

template <int BLOCK, int K, int FLAGS, int PF>
void launch_var(int grid, const uint4* syn, uint64_t ev, uint32_t iters, const uint32_t* bm,
                const uint32_t* f, const uint64_t* lf, uint4* out, uint32_t* tot, uint64_t now)
{
    hipLaunchKernelGGL((k_var<BLOCK, K, FLAGS, PF>), dim3(grid), dim3(BLOCK), 0, 0, syn, ev, iters, bm, f, lf,
                       out, tot, now);
}

#define V(B, K, FL, PF, NAME) Var{NAME, launch_var<B, K, FL, PF>, B, K}
#define P(B, K, FL, NAME) Var{NAME, launch_prod<B, K, FL>, B, K}
#define Q(B, K, FL, NAME) Var{NAME, launch_pipe<B, K, FL>, B, K}
#define Q4(B, K, FL, NAME) Var{NAME, launch_pipe4<B, K, FL>, B, K}
#define X(B, K, PIPE, NAME) Var{NAME, launch_x<B, K, PIPE>, B, K}

int main()
{
    const uint64_t n = 150000128ull;
    const uint32_t n_nrn = 5000512u;
    const uint32_t nwords = (n_nrn + 31) / 32;
    uint4 *syn, *out;
    uint32_t *bm, *filt, *tot;
    uint64_t* lastF;
    CK(hipMalloc(&syn, (n + 4096) * 16));  // padded: the x-only loop reads past the end
    CK(hipMalloc(&out, n * 16 + 65536));
    CK(hipMemset(out, 0, n * 16 + 65536));
    CK(hipMalloc(&bm, nwords * 4 + 64));
    CK(hipMalloc(&filt, FW * 4));
    CK(hipMalloc(&tot, 1 << 20));
    CK(hipMalloc(&lastF, (uint64_t)n_nrn * 8));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, syn, n, n_nrn);
    std::vector<uint32_t> h(nwords, 0), f(FW, 0);
    std::vector<uint64_t> lf(n_nrn, 0);
    const uint64_t now = 1000;
    srand(7);
    for (int i = 0; i < 15600; ++i) {
        uint32_t s = 512 + (uint32_t)(((uint64_t)rand() * 2654435761ull) % (n_nrn - 512));
        h[s >> 5] |= 1u << (s & 31);
        lf[s] = now - 1 - (i % 5);
    }
    for (uint32_t w = 0; w < nwords; ++w) f[w & (FW - 1)] |= h[w];
    int fpop = 0;
    for (uint32_t w : f) fpop += __builtin_popcount(w);
    CK(hipMemcpy(bm, h.data(), nwords * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(filt, f.data(), FW * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(lastF, lf.data(), (uint64_t)n_nrn * 8, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    printf("filter density %.4f\n", fpop / (double)(FW * 32));

    std::vector<Var> vars = {
        V(512, 8, 0, 1, "512x8 stream pf1"),
        P(512, 8, F_STAGE | F_SKIP, "prod"),
        X(512, 8, 0, "x 512x8"),
        X(512, 16, 0, "x 512x16"),
        X(512, 8, 1, "x pipe 512x8"),
        X(512, 16, 1, "x pipe 512x16"),
        X(1024, 8, 1, "x pipe 1024x8"),
        X(512, 32, 1, "x pipe 512x32"),
        V(512, 8, 0, 1, "512x8 stream pf1 again"),
        P(512, 8, F_STAGE | F_SKIP, "prod again"),
    };
    int cus = 256;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<std::vector<float>> t(vars.size());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int round = 0; round < 5; ++round) {
        for (size_t v = 0; v < vars.size(); ++v) {
            const uint32_t iters = (uint32_t)((n + 64 * vars[v].k - 1) / (64 * vars[v].k));
            const int grid = cus * 2;
            vars[v].launch(grid, syn, n, iters, bm, filt, lastF, out, tot, now);
            CK(hipEventRecord(a));
            for (int rep = 0; rep < 5; ++rep)
                vars[v].launch(grid, syn, n, iters, bm, filt, lastF, out, tot, now);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipGetLastError());
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t[v].push_back(ms / 5);
        }
    }
    for (size_t v = 0; v < vars.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-26s median %.4f ms  min %.4f ms  (%6.1f GB/s stream)\n", vars[v].name, t[v][2], t[v][0],
               n * 16.0 / (t[v][2] * 1e6));
    }
    return 0;
}
