// raw.hip -- the reference kernel's buffer-index ABI (abnn.h,
// abnn_launch_traversal): one C1 pass over CALLER-OWNED buffers in the
// reference's own layouts -- 16-B SynapsePacked records and u32 lastF / clock /
// budget (brain.metal:42-58, bound by Brain::encode_traversal at
// brain.cpp:93-118; allocated by Brain::build_buffers at brain.cpp:54-60).
//
// The handle API (capi.hip, kernels.hip) re-lays the records out for the gate
// (3 B per event).  Here the caller owns the memory, so every visited event
// streams its whole 16-B record and gathers lastF[src] as the reference does.
// Three launches per pass, all on the caller's stream:
//
//   k_raw_gate  : tiles of 2048 events (8 per thread, record loads coalesced):
//                 pre-spike gate (brain.metal:73-77), refractory gate
//                 (brain.metal:79-83), spike-candidate test (brain.metal:91-92)
//                 and the u32 age (brain.metal:116); survivors compacted in
//                 event order into the tile's workspace region.
//   k_raw_scan  : one workgroup: the tiles' capped candidate prefix (the
//                 ordered budget of C1, brain.metal:85-98 without its races),
//                 then the pass end on the scalars, which nothing later in the
//                 pass reads: *budget left, rBar (brain.metal:110-113), one
//                 clock tick (brain.metal:129).  The pass-start values go to the
//                 workspace header for k_raw_apply.
//   k_raw_apply : one wave per tile with budget left: the weight update of its
//                 survivors below the budget (brain.metal:101-122) and the
//                 spikes' stamps (brain.metal:125-126) -- every lastF read of
//                 the pass was in k_raw_gate, so the stamps land after them (C1).
//
// renormalise_clock_and_times (brain.metal:135-145): k_raw_renorm subtracts
// the clock read by every thread, k_raw_zero_clock zeroes it afterwards (the
// reference zeroes it inside the same kernel, racing with the readers).
#include <algorithm>
#include <cstring>

#include "engine.h"
#include "device.h"

#pragma clang fp contract(off)

namespace abnn {
namespace {

constexpr uint32_t kRawThreads = 256, kRawK = 8, kRawTile = kRawThreads * kRawK;  // events per tile
constexpr uint32_t kRawWaves = kRawThreads / 64;
constexpr uint32_t kRawScanThreads = 1024;
constexpr uint32_t kRawApplyBlocks = 4096;  // x 4 waves, each walks tiles w, w + 16384, ...

// Workspace: header | tile counts {survivors, candidates} | capped candidate
// prefix per tile | survivors {event, age bits | candidate << 31, w, dst}.
struct RawHdr {
    uint32_t now, budget0, t0, ncand;  // pass-start clock and budget; event 0 survived; candidates below the budget
    float R, rb;                       // pass-start reward and rBar (brain.metal:105-106)
    uint32_t pad[10];
};
static_assert(sizeof(RawHdr) == 64, "workspace header");

struct RawWs {
    RawHdr* hdr;
    uint2* cnt;
    uint32_t* pre;
    uint4* surv;
};

__host__ __device__ inline uint64_t raw_tiles(uint64_t E) { return (E + kRawTile - 1) / kRawTile; }

__host__ __device__ inline RawWs raw_ws(void* base, uint64_t tiles)
{
    char* p = static_cast<char*>(base);
    RawWs w;
    w.hdr = reinterpret_cast<RawHdr*>(p);
    w.cnt = reinterpret_cast<uint2*>(p + 64);
    w.pre = reinterpret_cast<uint32_t*>(p + 64 + 8 * tiles);
    w.surv = reinterpret_cast<uint4*>(p + 64 + ((12 * tiles + 15) & ~15ull));
    return w;
}

inline uint64_t raw_ws_bytes(uint64_t E)
{
    const uint64_t tiles = raw_tiles(E);
    return 64 + ((12 * tiles + 15) & ~15ull) + 16 * tiles * kRawTile;
}

// visited events: min(roundup(events, 256), n_syn) (brain.cpp:116-118, brain.metal:60-61)
inline uint64_t raw_events(uint32_t n_syn, uint32_t events)
{
    const uint64_t grid = ((uint64_t)events + 255u) / 256u * 256u;
    return grid < n_syn ? grid : n_syn;
}

__global__ __launch_bounds__(kRawThreads) void k_raw_gate(const uint4* __restrict__ syn, const uint32_t* lastF,
                                                           const uint32_t* clock, uint32_t n_nrn, uint32_t E,
                                                           KernelParams kp, RawWs ws)
{
    __shared__ uint32_t s_cnt[kRawK * kRawWaves], s_cand[kRawK * kRawWaves];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t now = *clock;  // per-TG clock cache (brain.metal:63-68); C1: the pass-start value
    const uint64_t base = (uint64_t)blockIdx.x * kRawTile;
    uint4 rec[kRawK];
#pragma unroll
    for (uint32_t k = 0; k < kRawK; ++k) {  // brain.metal:70, all loads in flight at once
        const uint64_t t = base + k * kRawThreads + threadIdx.x;
        rec[k] = t < E ? syn[t] : make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
    }
    uint32_t lp[kRawK];
#pragma unroll
    for (uint32_t k = 0; k < kRawK; ++k) lp[k] = rec[k].x < n_nrn ? lastF[rec[k].x] : 0u;
    uint32_t ld[kRawK];
    bool g1[kRawK];
#pragma unroll
    for (uint32_t k = 0; k < kRawK; ++k) {
        // a record naming a neuron >= n_nrn (the {0xFFFFFFFF, 0xFFFFFFFF} tombstone of a
        // pruned synapse) never passes
        g1[k] = rec[k].x < n_nrn && rec[k].y < n_nrn && now - lp[k] <= kp.window_pre;  // brain.metal:73-77
        ld[k] = g1[k] ? lastF[rec[k].y] : now;
    }
    uint64_t m2[kRawK];  // wave-uniform: survivors of step k
#pragma unroll
    for (uint32_t k = 0; k < kRawK; ++k) {
        const bool g2 = g1[k] && now - ld[k] > kp.refractory;  // brain.metal:79-83
        const uint64_t t = base + k * kRawThreads + threadIdx.x;
        const float w = __uint_as_float(rec[k].z);
        const bool cand = g2 && spike_candidate(kp, w, t, now);  // brain.metal:91-92
        m2[k] = __ballot(g2);
        const uint64_t mc = __ballot(cand);
        rec[k] = make_uint4((uint32_t)t, __float_as_uint((float)(now - ld[k])) | (cand ? 0x80000000u : 0u),
                            rec[k].z, rec[k].y);
        if (lane == 0) {
            s_cnt[k * kRawWaves + wv] = (uint32_t)__popcll(m2[k]);
            s_cand[k * kRawWaves + wv] = (uint32_t)__popcll(mc);
        }
        if (t == 0) ws.hdr->t0 = g2 ? 1u : 0u;  // event 0 reached the budget test (brain.metal:110)
    }
    __syncthreads();
    // exclusive offsets in event order: (k, wave, lane)
    uint32_t off = 0;
    if (wv == 0) {
        const uint32_t c = lane < kRawK * kRawWaves ? s_cnt[lane] : 0u;
        const uint32_t inc = wave_incl_scan(c);
        const uint32_t cc = wave_incl_scan(lane < kRawK * kRawWaves ? s_cand[lane] : 0u);
        if (lane < kRawK * kRawWaves) s_cnt[lane] = inc - c;
        if (lane == 63)
            ws.cnt[blockIdx.x] = make_uint2(inc, cc);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kRawK; ++k) {
        off = s_cnt[k * kRawWaves + wv];
        if ((m2[k] >> lane) & 1u) ws.surv[base + off + mbcnt64(m2[k])] = rec[k];
    }
}

__global__ __launch_bounds__(kRawScanThreads) void k_raw_scan(RawWs ws, uint32_t tiles, uint32_t E, uint32_t* clock,
                                                              uint32_t* budget, const float* reward, float* rbar,
                                                              KernelParams kp)
{
    __shared__ uint32_t s_wave[kRawScanThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t b0 = *budget;
    const uint32_t per = (tiles + kRawScanThreads - 1) / kRawScanThreads, q0 = threadIdx.x * per;
    uint64_t sum = 0;
    for (uint32_t q = q0; q < q0 + per && q < tiles; ++q) sum += ws.cnt[q].y;
    // block exclusive scan of the per-thread sums (capped: budgets are u32)
    const uint32_t v = (uint32_t)(sum < 0xFFFFFFFFull ? sum : 0xFFFFFFFFull);
    uint32_t inc = wave_incl_scan(v);  // tiles x 2048 < 2^32 events: no overflow
    if (lane == 63) s_wave[wv] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < kRawScanThreads / 64; ++w) {
        before += w < wv ? s_wave[w] : 0u;
        total += s_wave[w];
    }
    uint32_t run = before + inc - v;
    for (uint32_t q = q0; q < q0 + per && q < tiles; ++q) {
        ws.pre[q] = run < b0 ? run : b0;
        run += ws.cnt[q].y;
    }
    if (threadIdx.x == 0) {
        const uint32_t now = *clock;
        const float R = *reward, rb = *rbar;
        const uint32_t t0 = E > 0 ? ws.hdr->t0 : 0u;
        const uint32_t nc = total < b0 ? total : b0;
        ws.hdr->now = now;
        ws.hdr->budget0 = b0;
        ws.hdr->ncand = nc;
        ws.hdr->R = R;
        ws.hdr->rb = rb;
        *budget = b0 - nc;                                               // brain.metal:95-98 (C1: no wrap)
        if (t0 && b0 > 0) *rbar = rb + kp.alpha_rbar * (R - rb);         // brain.metal:110-113
        if (E > 0) *clock = now + kp.clock_inc;                          // brain.metal:129
    }
}

__global__ __launch_bounds__(kRawThreads) void k_raw_apply(uint4* syn, uint32_t* lastF, uint32_t tiles, KernelParams kp,
                                                            RawWs ws)
{
    const uint32_t lane = threadIdx.x & 63;
    const RawHdr h = *ws.hdr;  // pass-start scalars (k_raw_scan)
    const uint32_t nw = gridDim.x * kRawWaves;
    for (uint32_t tile = blockIdx.x * kRawWaves + (threadIdx.x >> 6); tile < tiles; tile += nw) {  // wave-uniform
        uint32_t P = ws.pre[tile];
        if (P >= h.budget0) continue;
        const uint32_t n = ws.cnt[tile].x;
        const uint4* sv = ws.surv + (uint64_t)tile * kRawTile;
        for (uint32_t b0 = 0; b0 < n && P < h.budget0; b0 += 64) {
            const bool v = b0 + lane < n;
            const uint4 e = v ? sv[b0 + lane] : make_uint4(0u, 0u, 0u, 0u);
            const bool cand = v && (e.y >> 31);
            const uint64_t bc = __ballot(cand);
            const uint32_t pre = P + mbcnt64(bc);  // spike candidates before this event
            if (v && pre < h.budget0) {
                const float w = updated_weight(kp, __uint_as_float(e.z), cand, h.R, h.rb,
                                               __uint_as_float(e.y & 0x7FFFFFFFu));  // brain.metal:101-121
                reinterpret_cast<float*>(syn + e.x)[2] = w;  // brain.metal:122 (src, dst, pad unchanged)
                if (cand) lastF[e.w] = h.now;                // brain.metal:125-126
            }
            P += (uint32_t)__popcll(bc);
        }
    }
}

__global__ __launch_bounds__(256) void k_raw_renorm(uint32_t* lastF, const uint32_t* clock, uint32_t n)
{
    const uint32_t base = *clock;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) lastF[i] -= base;  // brain.metal:142-143 (u32 wrap for never-fired neurons)
}

__global__ void k_raw_zero_clock(uint32_t* clock) { *clock = 0u; }  // brain.metal:144

KernelParams raw_params(const abnn_traversal_args& a)
{
    abnn_params p;
    if (a.knobs) p = *a.knobs;
    else abnn_default_params(&p);
    p.a_ltp = a.a_ltp;
    p.a_ltd = a.a_ltd;
    p.w_min = a.w_min;
    p.w_max = a.w_max;
    return to_kernel_params(p);
}

}  // namespace
}  // namespace abnn

using namespace abnn;

extern "C" {

uint64_t abnn_traversal_workspace_bytes(uint32_t n_syn, uint32_t events)
{
    return raw_ws_bytes(raw_events(n_syn, events));
}

abnn_status abnn_launch_traversal(const abnn_traversal_args* a, void* stream)
{
    if (!a || !a->clock || !a->budget || !a->reward || !a->rbar || !a->workspace ||
        (a->n_syn && (!a->syn || !a->last_fired)))
        return ABNN_ERR_INVALID;
    const uint64_t E = raw_events(a->n_syn, a->events);
    if (a->workspace_bytes < raw_ws_bytes(E) || ((uintptr_t)a->workspace & 15u)) return ABNN_ERR_INVALID;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const uint64_t tiles = raw_tiles(E);
    const RawWs ws = raw_ws(a->workspace, tiles);
    const KernelParams kp = raw_params(*a);
    uint4* syn = reinterpret_cast<uint4*>(a->syn);
    if (tiles)
        hipLaunchKernelGGL(k_raw_gate, dim3((uint32_t)tiles), dim3(kRawThreads), 0, s, syn, a->last_fired, a->clock,
                           a->n_nrn, (uint32_t)E, kp, ws);
    hipLaunchKernelGGL(k_raw_scan, dim3(1), dim3(kRawScanThreads), 0, s, ws, (uint32_t)tiles, (uint32_t)E, a->clock,
                       a->budget, a->reward, a->rbar, kp);
    if (tiles) {
        const uint32_t g = (uint32_t)std::min<uint64_t>((tiles + kRawWaves - 1) / kRawWaves, kRawApplyBlocks);
        hipLaunchKernelGGL(k_raw_apply, dim3(g), dim3(kRawThreads), 0, s, syn, a->last_fired, (uint32_t)tiles, kp, ws);
    }
    return hipGetLastError() == hipSuccess ? ABNN_OK : ABNN_ERR_HIP;
}

abnn_status abnn_launch_renormalise(uint32_t* last_fired, uint32_t* last_visited, uint32_t* clock, uint32_t n_nrn,
                                    void* stream)
{
    (void)last_visited;  // bound but untouched by the reference (brain.metal:137,142-144)
    if (!clock || (n_nrn && !last_fired)) return ABNN_ERR_INVALID;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    if (n_nrn) hipLaunchKernelGGL(k_raw_renorm, dim3((n_nrn + 255) / 256), dim3(256), 0, s, last_fired, clock, n_nrn);
    hipLaunchKernelGGL(k_raw_zero_clock, dim3(1), dim3(1), 0, s, clock);
    return hipGetLastError() == hipSuccess ? ABNN_OK : ABNN_ERR_HIP;
}

}  // extern "C"
