// kernels.hip -- CDNA4 (gfx950) kernels of one C1 traversal pass.
//
// Reference hot path: monte_carlo_traversal (abnn/src/core/kernels/brain.metal:41-130)
// and renormalise_clock_and_times (brain.metal:135-145).  One pass = seven
// launches, each doing one HBM-friendly thing:
//
//   k_bitmap   : lastFired (u64, 8 B/neuron, read once) -> exact recent-spike
//                bitmap, bit i = (now - lastFired[i]) <= WINDOW_PRE, OR-folded
//                into the LDS filter image; the per-pass stimulus stamp is
//                fused here.
//   k_gate     : THE streaming kernel.  Persistent workgroups whose waves each
//                sweep one contiguous range of events, loading only the src
//                word of every 16-B SynapsePacked record (the same HBM lines,
//                one VGPR per event in flight).  Pre-spike gate
//                (brain.metal:73-77) = one LDS filter bit + an L2 bitmap word
//                on a filter hit; passing events are staged in event order as
//                4-B offsets and flushed once per range.  Random-edge mode:
//                the same loop on Philox-picked records.
//   k_tiles    : one workgroup: 64-entry tiles over the ranges (descriptors).
//   k_refrac   : per tile: the record re-read, the refractory gate
//                (brain.metal:79-83) with a real lastFired[dst] gather, the
//                spike-candidate test (brain.metal:91-92), isi.
//   k_scan     : one workgroup: exclusive candidate prefix over the tiles =
//                the ordered global spike budget of schedule C1
//                (brain.metal:85-98 without its races) + the shard summary.
//   k_apply    : weight update (brain.metal:101-122) of every gated event that
//                still had budget (non-temporal stores; pruning, synaptogenesis);
//                spikes land at their budget position.  k_claim precedes it in
//                random mode (highest event wins a record).
//   k_finalize : deferred lastFired stamps (brain.metal:125-126), rBar EWMA
//                (brain.metal:110-113), one clock tick (brain.metal:129).
//   k_renorm   : brain.metal:135-145 with the base read once (no race).
//
// All fp32 arithmetic is compiled with -ffp-contract=off and written operation
// for operation like the oracle, so weights are bit-identical to the CPU.
#include <type_traits>

#include "engine.h"

#pragma clang fp contract(off)

namespace abnn {

KernelParams to_kernel_params(const abnn_params& p)
{
    KernelParams k;
    k.base_scale = p.base_scale;
    k.target_rate_hz = p.target_rate_hz;
    k.eta_home = p.eta_home;
    k.eta_reward = p.eta_reward;
    k.alpha_rbar = p.alpha_rbar;
    k.a_ltp = p.a_ltp;
    k.a_ltd = p.a_ltd;
    k.w_min = p.w_min;
    k.w_max = p.w_max;
    k.refractory = p.refractory;
    k.window_pre = p.window_pre;
    k.clock_inc = p.clock_inc;
    k.max_spikes = p.max_spikes;
    k.track_visits = p.track_visits;
    k.w_prune = p.w_prune;
    k.p_new = p.p_new;
    k.w_init = p.w_init;
    k.compact_every = p.compact_every;
    return k;
}

namespace {

// rand01, brain.metal:15-19.
__device__ __forceinline__ float rand01(uint32_t s)
{
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return (float)(s & 0xFFFFFFu) * (1.0f / 16777216.0f);
}

// Metal clamp(x, lo, hi) = min(max(x, lo), hi), written as selects so the
// result is bit-identical to the C oracle (no NaN canonicalisation).
__device__ __forceinline__ float clampf(float x, float lo, float hi)
{
    float m = x > lo ? x : lo;
    return m < hi ? m : hi;
}

__device__ __forceinline__ bool spike_candidate(const KernelParams& kp, float w, uint64_t tg,
                                                uint64_t now)
{
    float prob = clampf((w * w) * kp.base_scale, 0.0f, 1.0f);      // brain.metal:91
    return prob > rand01((uint32_t)tg ^ (uint32_t)now);             // brain.metal:92
}

__device__ __forceinline__ float updated_weight(const KernelParams& kp, float w, bool fired,
                                                float R, float rb, float isi)
{
    float dW = fired ? kp.a_ltp * (1.0f - w) : (-kp.a_ltd) * w;     // brain.metal:101-102
    dW = dW + (kp.eta_reward * (R - rb)) * (fired ? 1.0f : 0.0f);   // brain.metal:105-107
    float est_hz = isi > 0.0f ? 1e6f / isi : 0.0f;                  // brain.metal:116-117
    dW = dW + (kp.eta_home * (kp.target_rate_hz - est_hz)) * w;     // brain.metal:118
    return clampf(w + dW, kp.w_min, kp.w_max);                      // brain.metal:121
}

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

__device__ __forceinline__ uint64_t splitmix64_at(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1u) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Random-edge mode pick (include/abnn/abnn.h): Philox4x32-10 of
// {t, pass} under key seed ^ shard offset, then Lemire multiply-shift onto
// [0, n_syn).  Only the first two output words are used.
__device__ __forceinline__ uint64_t pick_record(uint64_t seed, uint64_t stream, uint64_t pass,
                                                uint64_t t, uint64_t n_syn)
{
    uint32_t x0 = (uint32_t)t, x1 = (uint32_t)(t >> 32), x2 = (uint32_t)pass, x3 = (uint32_t)(pass >> 32);
    const uint64_t k = seed ^ stream;
    uint32_t k0 = (uint32_t)k, k1 = (uint32_t)(k >> 32);
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
    return __umul64hi(((uint64_t)x1 << 32) | x0, n_syn);
}

// Record visited by local event t: itself (sweep, brain.metal:70) or its pick.
__device__ __forceinline__ uint64_t rec_index(const DeviceState& d, uint64_t t, uint64_t pass)
{
    return d.mode == ABNN_MODE_RANDOM ? pick_record(d.seed, d.syn_offset, pass, t, d.n_syn) : t;
}

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ float unit24(uint64_t x)
{
    return (float)(x >> 40) * (1.0f / 16777216.0f);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Exclusive scan of one u64 per thread over a kScanThreads workgroup.
__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* total, uint64_t* s_wave)
{
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr uint32_t nw = kScanThreads / 64;
    uint64_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) s_wave[wid] = inc;
    __syncthreads();
    uint64_t before = 0, tot = 0;
    for (uint32_t w = 0; w < nw; ++w) {
        uint64_t x = s_wave[w];
        if (w < wid) before += x;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return before + inc - v;
}

__device__ __forceinline__ uint64_t range_begin(uint32_t b, uint32_t iters, uint32_t G)
{
    return (uint64_t)b * iters / G;
}

// ---------------------------------------------------------------------------
// k_bitmap: bit i = (now - lastFired[i]) <= window_pre; stimulus stamp fused.
// A wave covers 256 neurons = four bitmap words; lane l owns neurons
// base + 64q + l, so ballot q is word q (four coalesced 512-B loads per wave).
__global__ __launch_bounds__(256) void k_bitmap(DeviceState d, KernelParams kp,
                                                uint64_t stim_first, uint64_t stim_count)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = ((uint64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const uint64_t base = wave * 256 + lane;
    const uint64_t now = *d.clock;
    uint64_t L[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = base + 64 * q;
        L[q] = i < d.n_nrn ? __builtin_nontemporal_load(d.last_fired + i) : ~0ull;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint64_t i = base + 64 * q;
        bool bit = false;
        if (i < d.n_nrn) {
            if (i - stim_first < stim_count) {  // unsigned range test
                L[q] = now;
                d.last_fired[i] = now;          // Brain::inject_inputs, brain.cpp:82
            }
            bit = (now - L[q]) <= (uint64_t)kp.window_pre;
        }
        const uint64_t m = __ballot(bit);
        if (lane == 0 && (wave * 4 + q) * 64 < d.n_nrn) {
            reinterpret_cast<uint64_t*>(d.bitmap)[wave * 4 + q] = m;
            // fold into the LDS filter image: filter[j] |= bitmap[j + m * filter_words]
            // (zeroed by k_refrac of the previous pass; few words are non-zero)
            const uint32_t w0 = (uint32_t)(wave * 4 + q) * 2u, fm = d.filter_words - 1u;
            if ((uint32_t)m) atomicOr(d.filter + (w0 & fm), (uint32_t)m);
            if ((uint32_t)(m >> 32)) atomicOr(d.filter + ((w0 + 1u) & fm), (uint32_t)(m >> 32));
        }
    }
}

// ---------------------------------------------------------------------------
// Pre-gated entries are processed as tiles of kTile (= 64 = one wave)
// consecutive entries of one range; tile order = event order;
// tile_desc[t] = {range, first entry of the tile in its range, entries, 0}.
// These steps move a few MB per pass: they are bound by dependent-load
// latency, so every loop below keeps all of a thread's loads in flight at
// once, scans run on DPP over coalesced chunks, and no tile waits on another.

// Inclusive wave scan on DPP (row_shr within 16-lane rows, then the gfx9
// row broadcasts): six VALU ops, no LDS crossbar round trips.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
    int v = (int)x;
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xC, 0xF, false);  // row_bcast:31 -> rows 2, 3
    return (uint32_t)v;
}

__device__ __forceinline__ uint32_t lane63(uint32_t x)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

__device__ __forceinline__ uint32_t tiles_of(uint32_t n) { return (n + kTile - 1) / kTile; }

// Tile descriptors and the pre-gated total, by one workgroup of NT threads.
// Wave w owns a contiguous block of ranges read as
// coalesced 64-range chunks (at most 16 with NT = kScanThreads); the chunk scans are recomputed in the second sweep
// rather than kept.  `lds` is scratch of >= 64 + 3 * kBig words.
template <int NT>
__device__ void build_tiles(const DeviceState& d, uint32_t* lds)
{
    constexpr uint32_t NWv = NT / 64, kCh = kMaxRanges / NT, kBig = 256;
    uint32_t* s_wt = lds;                                       // [NWv] tiles per wave
    uint64_t* s_wg1 = reinterpret_cast<uint64_t*>(lds + 16);    // [NWv] entries per wave
    uint32_t* s_nbig = lds + 48;
    uint32_t* s_big = lds + 64;                                 // {range, first tile, entries} x kBig
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = wave_uniform(tid >> 6), NR = d.n_ranges;
    const uint32_t per = ((NR + NWv - 1) / NWv + 63) & ~63u, nch = per / 64;
    if (tid == 0) *s_nbig = 0;
    uint32_t cnt[kCh];
#pragma unroll
    for (uint32_t c = 0; c < kCh; ++c) {
        const uint32_t r = w * per + c * 64 + lane;
        cnt[c] = (c < nch && r < NR) ? d.range_cnt[r] : 0u;
    }
    uint32_t run = 0;
    uint64_t g1 = 0;
#pragma unroll
    for (uint32_t c = 0; c < kCh; ++c) {
        run += lane63(wave_incl_scan(tiles_of(cnt[c])));
        g1 += cnt[c];
    }
    g1 = wave_sum(g1);
    if (lane == 0) {
        s_wt[w] = run;
        s_wg1[w] = g1;
    }
    __syncthreads();
    uint32_t off = 0, total = 0;
#pragma unroll
    for (uint32_t v = 0; v < NWv; ++v) {
        off += v < w ? s_wt[v] : 0u;
        total += s_wt[v];
    }
    run = 0;
#pragma unroll
    for (uint32_t c = 0; c < kCh; ++c) {
        const uint32_t r = w * per + c * 64 + lane;
        const uint32_t n = cnt[c], nt = tiles_of(n), x = wave_incl_scan(nt);
        const uint32_t t0 = off + run + x - nt;
        run += lane63(x);
        uint32_t q = 0;
        if (nt > 4) {  // long ranges (the dense input block) are filled cooperatively
            const uint32_t slot = atomicAdd(s_nbig, 1u);
            if (slot < kBig) {
                s_big[3 * slot] = r;
                s_big[3 * slot + 1] = t0;
                s_big[3 * slot + 2] = n;
                q = nt;
            }
        }
        for (; q < nt; ++q) d.tile_desc[t0 + q] = make_uint4(r, q * kTile, min(n - q * kTile, (uint32_t)kTile), 0u);
    }
    __syncthreads();
    const uint32_t nbig = min(*s_nbig, kBig);
    for (uint32_t b = 0; b < nbig; ++b) {
        const uint32_t r = s_big[3 * b], t0 = s_big[3 * b + 1], n = s_big[3 * b + 2], nt = tiles_of(n);
        for (uint32_t q = tid; q < nt; q += NT)
            d.tile_desc[t0 + q] = make_uint4(r, q * kTile, min(n - q * kTile, (uint32_t)kTile), 0u);
    }
    if (tid == 0) {
        uint64_t tg1 = 0;
        for (uint32_t v = 0; v < NWv; ++v) tg1 += s_wg1[v];
        d.work->total_tiles = total;
        d.work->g1 = tg1;
    }
}

// ---------------------------------------------------------------------------
// k_gate: the streaming kernel (see file header).  Every wave owns one
// contiguous range of events.  The pre-spike gate needs only the src of each
// record, and the records are held as arrays (SynArrays), so the sweep
// streams 4 B per event: a wave keeps K events per lane in flight in K VGPRs,
// each load one coalesced 256-B line segment.  Loads use a wave-uniform base:
// the arrays are padded by kDummyRecords, so the sweep's last iteration reads
// past its end instead of masking lanes, and the prefetch after a range's
// last iteration reads the zero dummy block.  Pre-gated events (~0.2 % in
// steady state) are staged as 4-B event offsets, kStageEntries per wave, so a
// wave usually flushes once, at the end of its range (vmcnt retires in issue
// order, stores included: a store between the prefetch and its wait delays
// the whole stream).
template <int BLOCK, int K, int FW, bool kTrack, bool kRandom>
__global__ __launch_bounds__(BLOCK) void k_gate(DeviceState d, KernelParams kp)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    constexpr uint32_t kFlushAt = kStageEntries - 64;  // one k-step adds at most 64
    constexpr int KD = kTrack ? K : 1;                 // dst words in flight (track_visits)
    static_assert(IE <= (uint32_t)kDummyRecords, "dummy block / padding must cover one iteration");
    __shared__ uint32_t s_filter[FW];
    __shared__ uint32_t s_stage[NW][kStageEntries];

    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = wave_uniform(tid >> 6);
    const uint32_t NR = gridDim.x * NW, r = blockIdx.x * NW + wid;
    const uint64_t it_begin = range_begin(r, d.iters, NR), it_end = range_begin(r + 1, d.iters, NR);
    const uint64_t region = it_begin * IE;
    const uint64_t now = *d.clock;  // per-TG clock cache, brain.metal:63-68 (C1: pass start)
    const bool exact = d.filter_exact != 0;
    uint32_t* stage = s_stage[wid];

    {
        const uint4* src = reinterpret_cast<const uint4*>(d.filter);
        uint4* dst = reinterpret_cast<uint4*>(s_filter);
        for (int i = tid; i < FW / 4; i += BLOCK) dst[i] = src[i];
    }

    uint32_t nxs[K], nxd[KD];
    const uint64_t pass = kRandom ? *d.pass_index : 0;
    auto issue = [&](uint64_t it, bool live) {
        if constexpr (kRandom) {  // random-edge mode: a per-lane random record per event
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint64_t t = it * IE + k * 64 + lane;
                const bool real = live && t < d.events;
                const uint64_t e = real ? pick_record(d.seed, d.syn_offset, pass, t, d.n_syn) : 0;
                nxs[k] = __builtin_nontemporal_load(real ? d.syn.src + e : d.dummy + (k * 64 + lane));
                if constexpr (kTrack)
                    nxd[k] = __builtin_nontemporal_load(real ? d.syn.dst + e : d.dummy + (k * 64 + lane));
            }
        } else {
            const uint32_t* bs = live ? d.syn.src + it * IE : d.dummy;  // wave-uniform
#pragma unroll
            for (int k = 0; k < K; ++k) nxs[k] = __builtin_nontemporal_load(bs + k * 64 + lane);
            if constexpr (kTrack) {
                const uint32_t* bd = live ? d.syn.dst + it * IE : d.dummy;
#pragma unroll
                for (int k = 0; k < K; ++k) nxd[k] = __builtin_nontemporal_load(bd + k * 64 + lane);
            }
        }
    };
    issue(it_begin, it_begin < it_end);
    __syncthreads();

    const uint32_t nn = (uint32_t)d.n_nrn;  // N_NRN < 2^32 (checked at create)
    uint32_t pend = 0, flushed = 0;
    auto flush = [&]() {  // wave-uniform: write the staged offsets, in order
        for (uint32_t q = lane; q < pend; q += 64)
            __builtin_nontemporal_store(stage[q], d.g1idx + region + flushed + q);
        flushed += pend;
        pend = 0;
    };
    for (uint64_t it = it_begin; it < it_end; ++it) {
        uint32_t src[K];
        uint32_t dst[KD];
#pragma unroll
        for (int k = 0; k < K; ++k) src[k] = nxs[k];
#pragma unroll
        for (int k = 0; k < KD; ++k) dst[k] = kTrack ? nxd[k] : 0u;
        const uint64_t base = it * IE;
        uint32_t vmask = (K == 32) ? 0xFFFFFFFFu : ((1u << K) - 1u);  // events of this lane that exist
        if (base + IE > d.events) {  // only the sweep's last iteration
            vmask = 0;
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (base + k * 64 + lane < d.events) vmask |= 1u << k;
        }

        // Pre-spike gate, brain.metal:73-77, first on the LDS filter: all K
        // reads issued back to back (the word index is masked, so always in
        // bounds), no branches.
        uint32_t fw[K];
#pragma unroll
        for (int k = 0; k < K; ++k) fw[k] = s_filter[(src[k] >> 5) & (FW - 1)];
        uint32_t fm = 0;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const bool hit = ((fw[k] >> (src[k] & 31u)) & 1u) && src[k] < nn;
            fm |= (hit ? 1u : 0u) << k;
        }
        fm &= vmask;
        // Filter hits are confirmed on the exact bitmap word (L2-resident);
        // issued before the next iteration's stream loads.
        uint32_t cw[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            cw[k] = 0xFFFFFFFFu;
            if (!exact && ((fm >> k) & 1u)) cw[k] = d.bitmap[src[k] >> 5];
        }
        issue(it + 1, it + 1 < it_end);  // next iteration's records in flight
        // keep every prefetch load ahead of the first use of a confirmation
        // (otherwise the scheduler interleaves them and waits mid-prefetch)
        __builtin_amdgcn_sched_barrier(0);

        if constexpr (kTrack) {  // README §4: lastVisited[dst] = now (never read by a decision)
#pragma unroll
            for (int k = 0; k < K; ++k)
                if (((vmask >> k) & 1u) && dst[k] < nn) d.last_visited[dst[k]] = now;
        }
        uint32_t g1m = 0;
#pragma unroll
        for (int k = 0; k < K; ++k)
            g1m |= ((((fm >> k) & 1u) && ((cw[k] >> (src[k] & 31u)) & 1u)) ? 1u : 0u) << k;
        if (__ballot(g1m != 0) == 0) continue;  // ~a third of the wave-iterations: nothing to stage
        const uint32_t rel = (uint32_t)(base - region);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const bool g1 = (g1m >> k) & 1u;
            const uint64_t b1 = __ballot(g1);
            if (g1) stage[pend + mbcnt64(b1)] = rel + k * 64 + lane;
            pend += (uint32_t)__popcll(b1);
            if (pend >= kFlushAt) flush();
        }
    }
    flush();
    if (lane == 0) d.range_cnt[r] = flushed;
}

// k_tiles: one workgroup builds the tile descriptors (build_tiles).
__global__ __launch_bounds__(kScanThreads) void k_tiles(DeviceState d)
{
    __shared__ uint32_t s_scratch[64 + 3 * 256];
    build_tiles<kScanThreads>(d, s_scratch);
}

// k_refrac: one wave per tile.  Per pre-gated entry the refractory gate with a
// real 8-B gather of lastFired[dst] (brain.metal:79-83), the spike-candidate
// test (brain.metal:91-92) and the homeostasis input isi (brain.metal:116);
// per tile the two lane masks and, for the events that passed, the entry
// {offset, dst, w, isi} at the tile's slot.  The gate is done with the filter
// image, so it is zeroed here for the next k_bitmap.
__global__ __launch_bounds__(256) void k_refrac(DeviceState d, KernelParams kp)
{
    const uint32_t lane = threadIdx.x & 63, gtid = blockIdx.x * 256 + threadIdx.x;
    for (uint32_t i = gtid; i < d.filter_words; i += gridDim.x * 256) d.filter[i] = 0u;
    const uint32_t wave = wave_uniform(gtid >> 6), nwaves = gridDim.x * 4;
    const uint64_t now = *d.clock;
    const uint32_t T = d.work->total_tiles;
    const uint32_t nn = (uint32_t)d.n_nrn;
    const uint64_t pass = *d.pass_index;
    for (uint32_t tile = wave; tile < T; tile += nwaves) {
        const uint4 td = d.tile_desc[tile];
        const uint64_t region = range_begin(td.x, d.iters, d.n_ranges) * d.iter_events;
        bool valid = lane < td.z;
        const uint32_t rel = valid ? d.g1idx[region + td.y + lane] : 0u;
        // the gate kept only the event offset: dst and w come from the record
        const uint64_t ri = valid ? rec_index(d, region + rel, pass) : 0;
        const uint32_t dst = valid ? d.syn.dst[ri] : 0u;
        const float w = valid ? d.syn.w[ri] : 0.0f;
        valid = valid && dst < nn;  // tombstones (dst = 0xFFFFFFFF) never pass
        const uint64_t ld = valid ? d.last_fired[dst] : 0ull;
        const bool g2 = valid && (now - ld) > (uint64_t)kp.refractory;
        const uint64_t tg = d.syn_offset + region + rel;
        const bool cand = g2 && spike_candidate(kp, w, tg, now);
        const uint64_t bg = __ballot(g2), bc = __ballot(cand);
        if (g2 && tg == 0) d.work->t0_g2 = 1;
        if (g2) d.g2e[(uint64_t)tile * kTile + lane] = make_uint4(rel, dst, __float_as_uint(w), __float_as_uint((float)(now - ld)));
        if (g2 && d.g2src) d.g2src[(uint64_t)tile * kTile + lane] = d.syn.src[ri];  // synaptogenesis keeps src
        if (lane == 0)
            d.tile_mask[tile] = make_uint4((uint32_t)bg, (uint32_t)(bg >> 32), (uint32_t)bc, (uint32_t)(bc >> 32));
    }
}

// ---------------------------------------------------------------------------
// k_scan: ordered spike budget over the tiles (one workgroup, in event order).
// Up to kSuper tiles per round: wave w scans a contiguous block of 64-tile
// chunks held in registers; rounds carry the prefix (warm-up passes only).
__global__ __launch_bounds__(kScanThreads) void k_scan(DeviceState d, KernelParams kp,
                                                       int32_t* xchg_out)
{
    int64_t* summary_out = reinterpret_cast<int64_t*>(xchg_out);
    constexpr uint32_t NWv = kScanThreads / 64, kCh = 16, kSuper = NWv * kCh * 64;
    __shared__ uint32_t s_wt[NWv];
    __shared__ uint64_t s_red[NWv];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = wave_uniform(tid >> 6);
    const uint32_t T = d.work->total_tiles;
    const uint64_t budget = kp.max_spikes;
    uint64_t carry = 0, g2 = 0;
    for (uint32_t base = 0; base < T; base += kSuper) {
        const uint32_t n = min(T - base, kSuper);
        const uint32_t per = ((n + NWv - 1) / NWv + 63) & ~63u, nch = per / 64;
        uint32_t cg[kCh];  // candidates | passed-refractory << 16, per tile
#pragma unroll
        for (uint32_t c = 0; c < kCh; ++c) {
            const uint32_t i = w * per + c * 64 + lane;
            const uint4 m = (c < nch && i < n) ? d.tile_mask[base + i] : make_uint4(0u, 0u, 0u, 0u);
            cg[c] = (uint32_t)(__popc(m.z) + __popc(m.w)) | ((uint32_t)(__popc(m.x) + __popc(m.y)) << 16);
        }
        uint32_t excl[kCh], run = 0;
#pragma unroll
        for (uint32_t c = 0; c < kCh; ++c) {
            const uint32_t x = cg[c] & 0xFFFFu, inc = wave_incl_scan(x);
            excl[c] = run + inc - x;
            run += lane63(inc);
            g2 += cg[c] >> 16;
        }
        if (lane == 0) s_wt[w] = run;
        __syncthreads();
        uint64_t off = carry, tot = 0;
#pragma unroll
        for (uint32_t v = 0; v < NWv; ++v) {
            off += v < w ? s_wt[v] : 0u;
            tot += s_wt[v];
        }
#pragma unroll
        for (uint32_t c = 0; c < kCh; ++c) {
            const uint32_t i = w * per + c * 64 + lane;
            if (c < nch && i < n) {
                const uint64_t pre = off + excl[c];
                // a tile is applied iff some event in it passed the refractory
                // gate while the budget lasted; inactive tiles carry the budget
                d.tile_pre[base + i] = (uint32_t)((cg[c] >> 16) > 0 && pre < budget ? pre : budget);
            }
        }
        carry += tot;
        __syncthreads();  // s_wt is rewritten by the next round
    }
    const uint64_t wg2 = wave_sum(g2);
    if (lane == 0) s_red[w] = wg2;
    __syncthreads();
    if (tid == 0) {
        uint64_t tg2 = 0;
        for (uint32_t v = 0; v < NWv; ++v) tg2 += s_red[v];
        const uint64_t capped = carry < budget ? carry : budget;
        const uint32_t t0 = d.work->t0_g2;
        summary_out[0] = (int64_t)capped;
        summary_out[1] = (int64_t)t0;
        summary_out[2] = (int64_t)d.events;
        summary_out[3] = (int64_t)tg2;
        d.work->t0_g2 = 0;  // re-armed for the next pass
        d.work->events = d.events;
        d.work->g2 = tg2;
    }
}

// ---------------------------------------------------------------------------
// k_spikes (sharded passes only): this shard's spike list in local budget
// order, written into its exchange record before the all-gather, so that every
// rank can stamp every rank's spikes in k_finalize.  Same tile walk as k_apply.
// The single-GPU pass skips it: k_apply writes the list there, in the same
// order, at no extra launch.
__global__ __launch_bounds__(256) void k_spikes(DeviceState d, KernelParams kp, int32_t* spikes)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = wave_uniform((blockIdx.x * 256 + threadIdx.x) >> 6), nwaves = gridDim.x * 4;
    const uint64_t budget = kp.max_spikes;
    const uint32_t T = d.work->total_tiles;
    for (uint32_t tile = wave; tile < T; tile += nwaves) {
        const uint64_t P = d.tile_pre[tile];
        if (P >= budget) continue;
        const uint4 m = d.tile_mask[tile];
        const uint64_t bc = m.z | ((uint64_t)m.w << 32);
        if (!((bc >> lane) & 1u)) continue;
        const uint64_t pre = P + mbcnt64(bc);
        if (pre < budget) spikes[pre] = (int32_t)d.g2e[(uint64_t)tile * kTile + lane].y;
    }
}

// ---------------------------------------------------------------------------
// k_claim (random mode): every event that will reach the update raises its
// record's claim to its event index + 1, so k_apply lets only the highest
// store (the last writer in event order).  Same tile walk as k_apply.
__global__ __launch_bounds__(256) void k_claim(DeviceState d, KernelParams kp, const int32_t* gathered,
                                               uint32_t rank)
{
    const uint32_t words = xchg_words(kp.max_spikes);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = wave_uniform((blockIdx.x * 256 + threadIdx.x) >> 6), nwaves = gridDim.x * 4;
    const uint64_t budget = kp.max_spikes, pass = *d.pass_index;
    uint64_t off = 0;
    for (uint32_t q = 0; q < rank; ++q) off += (uint64_t)*reinterpret_cast<const int64_t*>(gathered + q * words);
    off = off < budget ? off : budget;
    const uint32_t T = d.work->total_tiles;
    for (uint32_t tile = wave; tile < T; tile += nwaves) {
        const uint64_t P = off + d.tile_pre[tile];
        if (P >= budget) continue;
        const uint4 m = d.tile_mask[tile];
        const uint64_t bg = m.x | ((uint64_t)m.y << 32), bc = m.z | ((uint64_t)m.w << 32);
        if (!((bg >> lane) & 1u) || P + mbcnt64(bc) >= budget) continue;
        const uint64_t region = range_begin(d.tile_desc[tile].x, d.iters, d.n_ranges) * d.iter_events;
        const uint64_t t = region + d.g2e[(uint64_t)tile * kTile + lane].x;
        atomicMax(d.claim + rec_index(d, t, pass), (uint32_t)(t + 1));
    }
}

// ---------------------------------------------------------------------------
// k_apply: weight update of the gated events that still had budget; one wave
// per tile, tiles past the budget skipped on one load.
__global__ __launch_bounds__(256) void k_apply(DeviceState d, KernelParams kp,
                                               const int32_t* gathered, uint32_t rank,
                                               int32_t* spikes)
{
    const uint32_t words = xchg_words(kp.max_spikes);
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = wave_uniform((blockIdx.x * 256 + threadIdx.x) >> 6), nwaves = gridDim.x * 4;
    const uint64_t budget = kp.max_spikes;
    const float R = *d.reward, rb = *d.rbar;  // pass-start values (C1), brain.metal:105-106
    uint64_t off = 0;
    for (uint32_t q = 0; q < rank; ++q) off += (uint64_t)*reinterpret_cast<const int64_t*>(gathered + q * words);
    off = off < budget ? off : budget;

    const uint32_t T = d.work->total_tiles;
    const uint64_t pass = *d.pass_index;
    const bool random = d.mode == ABNN_MODE_RANDOM;
    const bool prune = kp.w_prune > 0.0f, genesis = d.grown != nullptr && kp.p_new > 0.0f;
    uint32_t upd = 0, nf = 0, npr = 0;
    for (uint32_t tile = wave; tile < T; tile += nwaves) {
        const uint64_t P = off + d.tile_pre[tile];
        if (P >= budget) continue;
        const uint4 m = d.tile_mask[tile];
        const uint64_t bg = m.x | ((uint64_t)m.y << 32), bc = m.z | ((uint64_t)m.w << 32);
        if (!((bg >> lane) & 1u)) continue;   // no entry, or stopped by the refractory gate
        const uint64_t pre = P + mbcnt64(bc);  // spike candidates before this event
        if (pre >= budget) continue;           // budget == 0 at this event: brain.metal:85-88
        const uint64_t region = range_begin(d.tile_desc[tile].x, d.iters, d.n_ranges) * d.iter_events;
        const uint4 e = d.g2e[(uint64_t)tile * kTile + lane];
        const bool f = (bc >> lane) & 1u;
        const float w = updated_weight(kp, __uint_as_float(e.z), f, R, rb, __uint_as_float(e.w));
        const uint64_t t = region + e.x, ri = rec_index(d, t, pass);
        // random mode: of the events that updated one synapse this pass, the
        // highest (k_claim) stores its weight; every one of them still counts
        const bool store = !random || d.claim[ri] == (uint32_t)(t + 1);
        if (random && store) d.claim[ri] = 0u;  // re-armed for the next pass
        // brain.metal:122.  Non-temporal: a plain 4-B store leaves ~160k
        // scattered dirty partial lines per pass whose write-back lands in the
        // middle of the next pass's record stream (+30 us of gate time,
        // tools/exp_variants.py).
        if (store && prune && w < kp.w_prune) {  // README §5: the synapse is removed
            __builtin_nontemporal_store(0xFFFFFFFFu, d.syn.src + ri);
            __builtin_nontemporal_store(0xFFFFFFFFu, d.syn.dst + ri);
            __builtin_nontemporal_store(w, d.syn.w + ri);
            if (d.dead) atomicAdd(d.dead + ri / kCompactChunk, 1u);  // tally for the structural update
            ++npr;
        } else if (store) {
            __builtin_nontemporal_store(w, d.syn.w + ri);
        }
        ++upd;
        if (f) {  // its stamp comes from the exchange record (k_finalize)
            if (spikes) spikes[pre] = (int32_t)e.y;  // single GPU: off == 0, local order
            ++nf;
            if (genesis) {  // README §5 synaptogenesis: slot `pre` of this pass
                const uint64_t x = splitmix64_at(d.seed ^ ABNN_GENESIS_KEY, (pass << 32) | pre);
                if (unit24(x) < kp.p_new) {
                    const uint64_t span = d.n_nrn - d.n_input;
                    d.grown[(pass % kp.compact_every) * kp.max_spikes + pre] =
                        make_uint4(d.g2src[(uint64_t)tile * kTile + lane],
                                   d.n_input + (uint32_t)(((x & 0xFFFFFFFFull) * span) >> 32),
                                   __float_as_uint(kp.w_init), 1u);
                }
            }
        }
    }
    // per-workgroup partials (atomics from every wave on one address serialise)
    __shared__ uint32_t s_u[4], s_f[4], s_p[4];
    const uint32_t wu = wave_sum(upd), wf = wave_sum(nf), wp = wave_sum(npr);
    if (lane == 0) {
        s_u[threadIdx.x >> 6] = wu;
        s_f[threadIdx.x >> 6] = wf;
        s_p[threadIdx.x >> 6] = wp;
    }
    __syncthreads();
    if (threadIdx.x == 0)
        d.apply_partial[blockIdx.x] = make_uint4(s_u[0] + s_u[1] + s_u[2] + s_u[3], s_f[0] + s_f[1] + s_f[2] + s_f[3],
                                                 s_p[0] + s_p[1] + s_p[2] + s_p[3], 0u);
}

// ---------------------------------------------------------------------------
// k_finalize: stamps, rBar, clock tick, statistics (one workgroup).
__global__ __launch_bounds__(kScanThreads) void k_finalize(DeviceState d, KernelParams kp,
                                                           const int32_t* gathered, uint32_t world)
{
    constexpr uint32_t kU = 4;
    const uint32_t tid = threadIdx.x, words = xchg_words(kp.max_spikes);
    const uint64_t now = *d.clock;
    const uint64_t budget = kp.max_spikes;
    uint64_t events = 0, off = 0;
    int64_t t0 = 0;
    for (uint32_t r = 0; r < world; ++r) {
        const int64_t* sm = reinterpret_cast<const int64_t*>(gathered + r * words);
        const int32_t* sp = gathered + r * words + 2 * ABNN_SUMMARY_WORDS;
        events += (uint64_t)sm[2];
        t0 |= sm[1];
        // rank r's spikes fill budget slots [off, off + n): brain.metal:125-126, deferred
        const uint64_t room = budget - off, n = (uint64_t)sm[0] < room ? (uint64_t)sm[0] : room;
        for (uint64_t i0 = 0; i0 < n; i0 += kU * kScanThreads) {
            uint32_t nrn[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u) {
                const uint64_t i = i0 + u * kScanThreads + tid;
                nrn[u] = i < n ? (uint32_t)sp[i] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u)
                if (nrn[u] < d.n_nrn) d.last_fired[nrn[u]] = now;
        }
        off += n;
    }
    uint32_t upd = 0, nf = 0, npr = 0;
#pragma unroll
    for (uint32_t u = 0; u < kTileBlocks / kScanThreads; ++u) {
        const uint4 v = d.apply_partial[u * kScanThreads + tid];
        upd += v.x;
        nf += v.y;
        npr += v.z;
    }
    __shared__ uint32_t s_u[kScanThreads / 64], s_f[kScanThreads / 64], s_p[kScanThreads / 64];
    upd = wave_sum(upd);
    nf = wave_sum(nf);
    npr = wave_sum(npr);
    if ((tid & 63) == 0) {
        s_u[tid >> 6] = upd;
        s_f[tid >> 6] = nf;
        s_p[tid >> 6] = npr;
    }
    __syncthreads();
    if (tid == 0) {
        uint64_t tu = 0, tf = 0, tp = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) {
            tu += s_u[w];
            tf += s_f[w];
            tp += s_p[w];
        }
        const float R = *d.reward, rb = *d.rbar;
        if (t0 != 0 && budget > 0)
            *d.rbar = rb + kp.alpha_rbar * (R - rb);  // brain.metal:110-113
        if (events > 0) *d.clock = now + kp.clock_inc; // brain.metal:129
        *d.pass_index += 1;
        PassWork* w = d.work;
        w->stats.passes += 1;
        w->stats.events += w->events;
        w->stats.pre_gated += w->g1;
        w->stats.post_gated += w->g2;
        w->stats.updated += tu;
        w->stats.fired += tf;
        w->stats.pruned += tp;
    }
}

// ---------------------------------------------------------------------------
// k_renorm: brain.metal:135-145; base (= the ticked clock) passed by the host.
__global__ __launch_bounds__(256) void k_renorm(DeviceState d, uint64_t base)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < d.n_nrn) d.last_fired[i] -= base;
    if (i == 0) *d.clock = 0;
}

// ---------------------------------------------------------------------------
// Structural update (README §5): stable removal of the tombstones.  Block b
// moves records [b * kCompactChunk, (b + 1) * kCompactChunk) to dst from
// offsets[b] on, in four coalesced rounds of kCompactThreads consecutive
// records (one block scan of the live flags per round), streaming both ways.
__global__ __launch_bounds__(kCompactThreads) void k_compact(SynArrays syn, uint64_t n, const uint64_t* offsets,
                                                             SynArrays dst)
{
    static_assert(kCompactThreads == kScanThreads, "block_exclusive_scan is sized for kScanThreads");
    __shared__ uint64_t s_wave[kCompactThreads / 64];
    const uint64_t base = (uint64_t)blockIdx.x * kCompactChunk;
    uint32_t rs[4], rd[4];
    float rw[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // all loads in flight first
        const uint64_t i = base + (uint64_t)j * kCompactThreads + threadIdx.x;
        const bool in = i < n;
        rs[j] = in ? __builtin_nontemporal_load(syn.src + i) : 0xFFFFFFFFu;
        rd[j] = in ? __builtin_nontemporal_load(syn.dst + i) : 0u;
        rw[j] = in ? __builtin_nontemporal_load(syn.w + i) : 0.0f;
    }
    uint64_t o = offsets[blockIdx.x];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const bool live = rs[j] != 0xFFFFFFFFu;
        uint64_t tot;
        const uint64_t pre = block_exclusive_scan(live ? 1u : 0u, &tot, s_wave);
        if (live) {
            __builtin_nontemporal_store(rs[j], dst.src + o + pre);
            __builtin_nontemporal_store(rd[j], dst.dst + o + pre);
            __builtin_nontemporal_store(rw[j], dst.w + o + pre);
        }
        o += tot;
    }
}

// ---------------------------------------------------------------------------
// k_generate: synthetic graph (recipe of brain-engine.cpp:31-53, portable RNG).
__global__ __launch_bounds__(256) void k_generate(DeviceState d, uint32_t n_in, uint32_t n_out,
                                                  uint64_t seed)
{
    const uint64_t n_io = (uint64_t)n_in * n_out;
    const uint64_t lo = (uint64_t)n_in + n_out;
    const uint64_t range = d.n_nrn - lo;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < d.n_syn; k += stride) {
        const uint64_t i = d.syn_offset + k;
        const uint64_t x2 = splitmix64_at(seed, 3u * i + 2u);
        uint32_t src, dst;
        float w;
        if (i < n_io) {
            src = (uint32_t)(i / n_out);
            dst = n_in + (uint32_t)(i % n_out);
            w = 0.4f + unit24(x2) * (0.8f - 0.4f);
        } else {
            const uint64_t x0 = splitmix64_at(seed, 3u * i + 0u);
            const uint64_t x1 = splitmix64_at(seed, 3u * i + 1u);
            src = (uint32_t)(lo + (((x0 >> 32) * range) >> 32));
            dst = (uint32_t)(lo + (((x1 >> 32) * range) >> 32));
            w = 0.1f + unit24(x2) * (0.2f - 0.1f);
        }
        d.syn.src[k] = src;
        d.syn.dst[k] = dst;
        d.syn.w[k] = w;
    }
}

__global__ __launch_bounds__(256) void k_checksum(DeviceState d, uint64_t* out)
{
    __shared__ uint64_t s[4];
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t acc = 0;
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < d.n_syn; k += stride) {
        const uint64_t i = d.syn_offset + k;
        const uint64_t a = ((uint64_t)d.syn.src[k] << 32) | d.syn.dst[k];
        const uint64_t b = (uint64_t)__float_as_uint(d.syn.w[k]) << 32;  // pad = 0
        acc += mix64(a ^ mix64(b + i * 0x9E3779B97F4A7C15ull));
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0)
        atomicAdd((unsigned long long*)out, (unsigned long long)(s[0] + s[1] + s[2] + s[3]));
}

__global__ __launch_bounds__(256) void k_stamp_list(DeviceState d, const uint32_t* idx,
                                                    uint64_t n, const uint64_t* value_dev,
                                                    uint64_t value)
{
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t v = value_dev ? *value_dev : value;
    if (i < n && idx[i] < d.n_nrn) d.last_fired[idx[i]] = v;
}

inline uint32_t blocks_for(uint64_t n) { return (uint32_t)((n + 255) / 256); }

template <int BLOCK, int K, int FW>
hipError_t launch_gate_shape(const DeviceState& d, const KernelParams& kp, hipStream_t s)
{
    const dim3 g(d.gate_blocks), b(BLOCK);
    const bool random = d.mode == ABNN_MODE_RANDOM;
    if (kp.track_visits) {
        if (random) hipLaunchKernelGGL((k_gate<BLOCK, K, FW, true, true>), g, b, 0, s, d, kp);
        else hipLaunchKernelGGL((k_gate<BLOCK, K, FW, true, false>), g, b, 0, s, d, kp);
    } else {
        if (random) hipLaunchKernelGGL((k_gate<BLOCK, K, FW, false, true>), g, b, 0, s, d, kp);
        else hipLaunchKernelGGL((k_gate<BLOCK, K, FW, false, false>), g, b, 0, s, d, kp);
    }
    return hipGetLastError();
}

template <int BLOCK, int K, int FW>
int occupancy_shape(bool track, bool random)
{
    int n = 0;
    hipError_t e;
    if (track)
        e = random ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, true, true>, BLOCK, 0)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, true, false>, BLOCK, 0);
    else
        e = random ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, false, true>, BLOCK, 0)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, false, false>, BLOCK, 0);
    return e == hipSuccess ? n : 0;
}

// Compiled gate shapes: threads per workgroup x events per lane x filter words.
#define ABNN_GATE_SHAPES(X) \
    X(512, 8, 16384)        \
    X(512, 16, 16384)       \
    X(512, 4, 16384)        \
    X(512, 8, 8192)         \
    X(512, 16, 8192)        \
    X(1024, 8, 8192)        \
    X(1024, 4, 8192)        \
    X(256, 16, 8192)        \
    X(256, 8, 8192)         \
    X(512, 32, 8192)        \
    X(256, 32, 8192)        \
    X(1024, 16, 8192)

constexpr uint64_t shape_key(uint32_t b, uint32_t k, uint32_t fw) { return ((uint64_t)b << 40) | ((uint64_t)k << 32) | fw; }

}  // namespace

int gate_blocks_per_cu(uint32_t block, uint32_t k, uint32_t fw, bool track, bool random)
{
    switch (shape_key(block, k, fw)) {
#define X(B, K, F) case shape_key(B, K, F): return occupancy_shape<B, K, F>(track, random);
        ABNN_GATE_SHAPES(X)
#undef X
    }
    return 0;
}

bool gate_shape_supported(uint32_t block, uint32_t k, uint32_t fw)
{
    switch (shape_key(block, k, fw)) {
#define X(B, K, F) case shape_key(B, K, F): return true;
        ABNN_GATE_SHAPES(X)
#undef X
    }
    return false;
}

hipError_t launch_bitmap(const DeviceState& d, const KernelParams& kp, uint64_t stim_first,
                         uint64_t stim_count, hipStream_t s)
{
    if (d.n_nrn == 0) return hipSuccess;
    hipLaunchKernelGGL(k_bitmap, dim3((uint32_t)((d.n_nrn + 1023) / 1024)), dim3(256), 0, s, d, kp,
                       stim_first, stim_count);
    return hipGetLastError();
}

hipError_t launch_refrac(const DeviceState& d, const KernelParams& kp, hipStream_t s)
{
    hipLaunchKernelGGL(k_tiles, dim3(1), dim3(kScanThreads), 0, s, d);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_refrac, dim3(kTileBlocks), dim3(256), 0, s, d, kp);
    return hipGetLastError();
}

hipError_t launch_gate(const DeviceState& d, const KernelParams& kp, hipStream_t s)
{
    if (d.gate_blocks == 0) return hipSuccess;  // no events: n_ranges = 0, k_tiles writes no tiles
    switch (shape_key(d.gate_block, d.gate_k, d.filter_words)) {
#define X(B, K, F) case shape_key(B, K, F): return launch_gate_shape<B, K, F>(d, kp, s);
        ABNN_GATE_SHAPES(X)
#undef X
    }
    return hipErrorInvalidValue;
}

hipError_t launch_scan(const DeviceState& d, const KernelParams& kp, int32_t* xchg_out,
                       bool spike_list, hipStream_t s)
{
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(kScanThreads), 0, s, d, kp, xchg_out);
    if (!spike_list) return hipGetLastError();
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_spikes, dim3(kTileBlocks), dim3(256), 0, s, d, kp,
                       xchg_out + 2 * ABNN_SUMMARY_WORDS);
    return hipGetLastError();
}

hipError_t launch_apply(const DeviceState& d, const KernelParams& kp, const int32_t* gathered,
                        uint32_t world, uint32_t rank, int32_t* spikes, hipStream_t s)
{
    if (spikes && (world != 1 || rank != 0)) return hipErrorInvalidValue;
    if (d.mode == ABNN_MODE_RANDOM) {
        hipLaunchKernelGGL(k_claim, dim3(kTileBlocks), dim3(256), 0, s, d, kp, gathered, rank);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_apply, dim3(kTileBlocks), dim3(256), 0, s, d, kp, gathered, rank, spikes);
    return hipGetLastError();
}

hipError_t launch_finalize(const DeviceState& d, const KernelParams& kp, const int32_t* gathered,
                           uint32_t world, hipStream_t s)
{
    hipLaunchKernelGGL(k_finalize, dim3(1), dim3(kScanThreads), 0, s, d, kp, gathered, world);
    return hipGetLastError();
}

hipError_t launch_renorm(const DeviceState& d, uint64_t base, hipStream_t s)
{
    hipLaunchKernelGGL(k_renorm, dim3(blocks_for(d.n_nrn > 0 ? d.n_nrn : 1)), dim3(256), 0, s, d,
                       base);
    return hipGetLastError();
}

hipError_t launch_compact(const SynArrays& syn, uint64_t n, const uint64_t* offsets, const SynArrays& dst,
                          hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_compact, dim3((uint32_t)((n + kCompactChunk - 1) / kCompactChunk)),
                       dim3(kCompactThreads), 0, s, syn, n, offsets, dst);
    return hipGetLastError();
}

hipError_t launch_generate(const DeviceState& d, uint32_t n_in, uint32_t n_out, uint64_t seed,
                           hipStream_t s)
{
    if (d.n_syn == 0) return hipSuccess;
    uint32_t grid = blocks_for(d.n_syn);
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(k_generate, dim3(grid), dim3(256), 0, s, d, n_in, n_out, seed);
    return hipGetLastError();
}

hipError_t launch_checksum(const DeviceState& d, uint64_t* out_dev, hipStream_t s)
{
    hipError_t e = hipMemsetAsync(out_dev, 0, sizeof(uint64_t), s);
    if (e != hipSuccess || d.n_syn == 0) return e;
    uint32_t grid = blocks_for(d.n_syn);
    if (grid > 4096) grid = 4096;
    hipLaunchKernelGGL(k_checksum, dim3(grid), dim3(256), 0, s, d, out_dev);
    return hipGetLastError();
}

hipError_t launch_stamp_list(const DeviceState& d, const uint32_t* idx_dev, uint64_t n,
                             const uint64_t* value_dev, uint64_t value, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_stamp_list, dim3(blocks_for(n)), dim3(256), 0, s, d, idx_dev, n, value_dev,
                       value);
    return hipGetLastError();
}

}  // namespace abnn
