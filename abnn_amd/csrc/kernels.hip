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
#include <algorithm>
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
// Per-range results of the gate.  A range is the contiguous block of events
// one gate wave sweeps; range order = event order.  The pre-gated events of a
// range are cut, in event order, into chunks of kChunk: chunk c occupies
// [region + c kChunk, region + (c + 1) kChunk) of the range's region in g1idx
// (offsets, full chunks only) and g2x (refractory survivors, compacted to the
// chunk's start).  g2x entry = {event - region, isi bits | candidate << 31,
// w bits, dst}, with isi = (float)(now - lastFired[dst]) >= 0 (its sign bit is
// free) and w, dst as read at pass start (C1).  chunk_cnt[chunk_slot] =
// {survivors, candidates} of a full chunk (slots of full chunks never
// collide; the last chunk's survivors are the range's total minus theirs);
// range_info[r] = {pre-gated, survivors, candidates, full chunks}.  The last (partial) chunk of a range is processed by its gate wave
// at the end of its range; full chunks (dense parts of the graph, warm-up
// passes) are queued for k_refrac so that no wave's stream waits on them.

__device__ __forceinline__ uint64_t region_of(const DeviceState& d, uint32_t r)
{
    return range_begin(r, d.iters, d.n_ranges) * d.iter_events;
}

__device__ __forceinline__ uint64_t chunk_slot(uint64_t region, uint32_t c)
{
    return (region + (uint64_t)c * kChunk) / kChunkSlotDiv;
}

// Refractory stage (brain.metal:79-83, 91-92, 116) of n <= kChunk pre-gated
// offsets of one chunk, by one wave, in event order: dst and w gathered from
// the record arrays, the 8-B lastFired[dst] gather, the candidate test; the
// survivors are written compacted from g2x[base] on.  `rel_at(q)` yields the
// q-th offset.  Batches of R rounds of 64 keep every load of a lane in flight
// at once.  Returns {survivors, candidates}.
template <int R, bool kRandom, class RelAt>
__device__ __forceinline__ uint2 refrac_chunk(const DeviceState& d, const KernelParams& kp, uint64_t region,
                                              uint64_t base, uint32_t n, uint64_t now, uint64_t pass,
                                              RelAt&& rel_at)
{
    const uint32_t lane = threadIdx.x & 63, nn = (uint32_t)d.n_nrn;
    uint32_t n_g2 = 0, n_cand = 0;
    auto record_of = [&](uint32_t rel) -> uint64_t {
        const uint64_t t = region + rel;
        return kRandom ? pick_record(d.seed, d.syn_offset, pass, t, d.n_syn) : t;
    };
    for (uint32_t b0 = 0; b0 < n; b0 += R * 64) {
        uint32_t rel[R], dst[R];
        float w[R];
        uint64_t ld[R];
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const uint32_t q = b0 + j * 64 + lane;
            const bool v = q < n;
            rel[j] = v ? rel_at(q) : 0u;
            const uint64_t ri = v ? record_of(rel[j]) : 0;
            dst[j] = v ? d.syn.dst[ri] : 0xFFFFFFFFu;  // tombstones (dst = 0xFFFFFFFF) never pass
            w[j] = v ? d.syn.w[ri] : 0.0f;
        }
#pragma unroll
        for (int j = 0; j < R; ++j) ld[j] = dst[j] < nn ? d.last_fired[dst[j]] : 0ull;
#pragma unroll
        for (int j = 0; j < R; ++j) {
            if (b0 + (uint32_t)j * 64 >= n) break;  // wave-uniform
            const bool g2 = dst[j] < nn && (now - ld[j]) > (uint64_t)kp.refractory;  // brain.metal:79-83
            const uint64_t tg = d.syn_offset + region + rel[j];
            const bool cand = g2 && spike_candidate(kp, w[j], tg, now);
            const uint64_t bg = __ballot(g2);
            if (g2) {
                const uint64_t o = base + n_g2 + mbcnt64(bg);
                const uint32_t isi = __float_as_uint((float)(now - ld[j])) | (cand ? 0x80000000u : 0u);
                d.g2x[o] = make_uint4(rel[j], isi, __float_as_uint(w[j]), dst[j]);
                if (d.g2src) d.g2src[o] = d.syn.src[record_of(rel[j])];  // synaptogenesis keeps src
                if (tg == 0) d.work->t0_g2 = 1u;
            }
            n_g2 += (uint32_t)__popcll(bg);
            n_cand += (uint32_t)__popcll(__ballot(cand));
        }
    }
    return make_uint2(n_g2, n_cand);
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
// steady state) are staged in LDS as 4-B event offsets; a full chunk goes to
// g1idx and onto the k_refrac queue, and the range's last chunk is run
// through the refractory stage by the wave itself once its stream is done.
// (vmcnt retires in issue order, stores included: a store between the
// prefetch and its wait delays the whole stream, so chunks are rare.)
template <int BLOCK, int K, int FW, bool kTrack, bool kRandom>
__global__ __launch_bounds__(BLOCK, 4) void k_gate(DeviceState d, KernelParams kp)  // >= 4 waves per SIMD: <= 128 VGPRs
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    constexpr int KD = kTrack ? K : 1;                 // dst words in flight (track_visits)
    static_assert(IE <= (uint32_t)kDummyRecords, "dummy block / padding must cover one iteration");
    __shared__ uint32_t s_filter[FW];
    __shared__ uint32_t s_stage[NW][kChunk + 64];      // a chunk + one k-step

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
    const uint64_t t_start = d.wave_clock ? __builtin_amdgcn_s_memrealtime() : 0;
    issue(it_begin, it_begin < it_end);
    __syncthreads();

    const uint32_t nn = (uint32_t)d.n_nrn;  // N_NRN < 2^32 (checked at create)
    uint32_t pend = 0, nch = 0, oslot = 0;
    // wave-uniform: a full chunk of staged offsets to g1idx and the k_refrac
    // queue; the (< 64) entries past it move to the front of the stage
    auto chunk_out = [&]() {
        const uint64_t base = region + (uint64_t)nch * kChunk;
#pragma unroll
        for (uint32_t q = 0; q < kChunk; q += 64) __builtin_nontemporal_store(stage[q + lane], d.g1idx + base + q + lane);
        const uint32_t rest = pend - kChunk;
        const uint32_t x = lane < rest ? stage[kChunk + lane] : 0u;
        if (lane < rest) stage[lane] = x;
        // queue slot: claimed now, written at the next chunk or the range's
        // end, so the stream never waits on the atomic's return
        if (lane == 0) {
            if (nch > 0) d.ovf[oslot] = make_uint2(r, nch - 1);
            oslot = atomicAdd(&d.work->n_ovf, 1u);
        }
        ++nch;
        pend = rest;
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
            if (pend >= kChunk) chunk_out();  // a k-step stages at most 64
        }
    }
    const uint64_t t_stream = d.wave_clock ? __builtin_amdgcn_s_memrealtime() : 0;
    // the range's last chunk: refractory stage by this wave
    const uint64_t tb = region + (uint64_t)nch * kChunk;
    const uint2 c = refrac_chunk<4, kRandom>(d, kp, region, tb, pend, now, pass,
                                             [&](uint32_t q) { return stage[q]; });
    if (lane == 0) {
        if (nch > 0) d.ovf[oslot] = make_uint2(r, nch - 1);
        d.range_info[r] = make_uint4(nch * kChunk + pend, c.x, c.y, nch);
        if (d.wave_clock) {  // diagnostics (ABNN_WAVE_CLOCK): 100 MHz wall clock per wave
            d.wave_clock[4 * r] = t_start;
            d.wave_clock[4 * r + 1] = t_stream;
            d.wave_clock[4 * r + 2] = __builtin_amdgcn_s_memrealtime();
            d.wave_clock[4 * r + 3] = __smid();
        }
    }
}

// k_refrac: the queued full chunks (k_gate), one wave per chunk; adds each
// chunk's counts to its range.
__global__ __launch_bounds__(256) void k_refrac(DeviceState d, KernelParams kp)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = wave_uniform((blockIdx.x * 256 + threadIdx.x) >> 6), nwaves = gridDim.x * 4;
    const uint64_t now = *d.clock, pass = *d.pass_index;
    const uint32_t n = d.work->n_ovf;
    for (uint32_t i = wave; i < n; i += nwaves) {
        const uint2 q = d.ovf[i];
        const uint64_t region = region_of(d, q.x), base = region + (uint64_t)q.y * kChunk;
        const uint32_t* rel = d.g1idx + base;
        const uint2 c = d.mode == ABNN_MODE_RANDOM
            ? refrac_chunk<kChunk / 64, true>(d, kp, region, base, kChunk, now, pass, [&](uint32_t j) { return rel[j]; })
            : refrac_chunk<kChunk / 64, false>(d, kp, region, base, kChunk, now, pass, [&](uint32_t j) { return rel[j]; });
        if (lane == 0) {
            d.chunk_cnt[chunk_slot(region, q.y)] = c;
            atomicAdd(&d.range_info[q.x].y, c.x);
            atomicAdd(&d.range_info[q.x].z, c.y);
        }
    }
}

// ---------------------------------------------------------------------------
// The ordered spike budget of schedule C1 (brain.metal:85-98 without its
// races): an event that passed both gates is updated iff fewer than
// max_spikes spike candidates precede it in global event order.  Walked by
// k_spikes, k_claim and k_apply alike.  Every workgroup first builds the
// capped exclusive candidate prefix of all ranges in LDS (a few KB read from
// L2; cheaper than a separate single-workgroup scan launch).  The work items
// are the last chunk of every range and every queued full chunk, one per wave
// at a time: an item adds the candidates of its range's lower full chunks,
// leaves at once if the budget is spent, and otherwise visits its (<= kChunk)
// survivors in event order, calling f(region, entry, candidate, budget
// position, g2x index) for each one whose position is below the budget.
constexpr uint32_t kWalkWaves = kApplyThreads / 64;
constexpr uint32_t kPrePerThread = kMaxRanges / kApplyThreads;

// s_pre[r] = min(off + candidates of ranges < r, budget), r < n_ranges.
__device__ void range_prefix(const DeviceState& d, uint64_t off, uint64_t budget, uint32_t* s_pre, uint64_t* s_red)
{
    const uint32_t NR = d.n_ranges, per = (NR + kApplyThreads - 1) / kApplyThreads, q0 = threadIdx.x * per;
    uint32_t c[kPrePerThread];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < kPrePerThread; ++j) {
        c[j] = (j < per && q0 + j < NR) ? d.range_info[q0 + j].z : 0u;
        sum += c[j];
    }
    uint64_t tot;
    uint64_t run = off + block_exclusive_scan(sum, &tot, s_red);
#pragma unroll
    for (uint32_t j = 0; j < kPrePerThread; ++j) {
        if (j < per && q0 + j < NR) s_pre[q0 + j] = (uint32_t)(run < budget ? run : budget);
        run += c[j];
    }
    __syncthreads();
}

template <class F>
__device__ void budget_walk(const DeviceState& d, uint64_t off, uint64_t budget, uint32_t* s_pre, uint64_t* s_red,
                            F&& f)
{
    range_prefix(d, off, budget, s_pre, s_red);
    const uint32_t lane = threadIdx.x & 63, w = wave_uniform(threadIdx.x >> 6);
    const uint32_t NR = d.n_ranges, items = NR + d.work->n_ovf;
    for (uint32_t i = blockIdx.x * kWalkWaves + w; i < items; i += gridDim.x * kWalkWaves) {
        uint32_t r, c;
        if (i < NR) {
            r = i;
            c = d.range_info[r].w;  // the last chunk follows the full ones
        } else {
            const uint2 q = d.ovf[i - NR];
            r = q.x;
            c = q.y;
        }
        uint64_t P = s_pre[r];
        if (P >= budget) continue;
        const uint4 ri = d.range_info[r];
        const uint64_t region = region_of(d, r);
        const bool last = c == ri.w;
        uint32_t cl = 0, gl = 0;  // candidates / survivors of the lower full chunks
        for (uint32_t c0 = 0; c0 < c; c0 += 64)
            if (c0 + lane < c) {
                const uint2 cc = d.chunk_cnt[chunk_slot(region, c0 + lane)];
                cl += cc.y;
                gl += cc.x;
            }
        P += wave_sum(cl);
        if (P >= budget) continue;
        // survivors of this chunk: the last one holds what the full ones do not
        const uint32_t n = last ? ri.y - wave_sum(gl) : d.chunk_cnt[chunk_slot(region, c)].x;
        const uint64_t base = region + (uint64_t)c * kChunk;
        constexpr uint32_t RW = kChunk / 64;
        uint4 e[RW];
#pragma unroll
        for (uint32_t j = 0; j < RW; ++j)
            e[j] = j * 64 + lane < n ? d.g2x[base + j * 64 + lane] : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
        for (uint32_t j = 0; j < RW; ++j) {
            if (j * 64 >= n || P >= budget) break;  // wave-uniform
            const bool v = j * 64 + lane < n, cand = v && (e[j].y >> 31);
            const uint64_t bc = __ballot(cand);
            const uint64_t pre = P + mbcnt64(bc);  // spike candidates before this event
            if (v && pre < budget) f(region, e[j], cand, pre, base + j * 64 + lane);
            P += (uint64_t)__popcll(bc);
        }
    }
}

// Budget slots taken by the lower ranks of a sharded pass (their gathered
// exchange summaries), capped at the budget; 0 without an exchange.
__device__ uint64_t rank_offset(const KernelParams& kp, const int32_t* gathered, uint32_t rank)
{
    const uint32_t words = xchg_words(kp.max_spikes);
    uint64_t off = 0;
    if (gathered)
        for (uint32_t q = 0; q < rank; ++q) off += (uint64_t)*reinterpret_cast<const int64_t*>(gathered + q * words);
    return off < kp.max_spikes ? off : kp.max_spikes;
}

// ---------------------------------------------------------------------------
// k_scan (sharded passes): this shard's exchange summary -- candidates capped
// at the budget, the event-0-updated flag, events visited, refractory passes.
__global__ __launch_bounds__(kScanThreads) void k_scan(DeviceState d, KernelParams kp, int32_t* xchg_out)
{
    __shared__ uint64_t s_c[kScanThreads / 64], s_g[kScanThreads / 64];
    int64_t* summary_out = reinterpret_cast<int64_t*>(xchg_out);
    uint64_t c = 0, g = 0;
    for (uint32_t q = threadIdx.x; q < d.n_ranges; q += kScanThreads) {
        const uint4 ri = d.range_info[q];
        c += ri.z;
        g += ri.y;
    }
    c = wave_sum(c);
    g = wave_sum(g);
    if ((threadIdx.x & 63) == 0) {
        s_c[threadIdx.x >> 6] = c;
        s_g[threadIdx.x >> 6] = g;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t tc = 0, tg = 0;
        for (uint32_t v = 0; v < kScanThreads / 64; ++v) {
            tc += s_c[v];
            tg += s_g[v];
        }
        const uint64_t budget = kp.max_spikes;
        summary_out[0] = (int64_t)(tc < budget ? tc : budget);
        summary_out[1] = (int64_t)d.work->t0_g2;
        summary_out[2] = (int64_t)d.events;
        summary_out[3] = (int64_t)tg;
    }
}

// ---------------------------------------------------------------------------
// k_spikes (sharded passes only): this shard's spike list in local budget
// order, written into its exchange record before the all-gather, so that every
// rank can stamp every rank's spikes in k_finalize.
__global__ __launch_bounds__(kApplyThreads) void k_spikes(DeviceState d, KernelParams kp, int32_t* spikes)
{
    extern __shared__ uint32_t s_pre[];
    __shared__ uint64_t s_red[kWalkWaves];
    budget_walk(d, 0, kp.max_spikes, s_pre, s_red, [&](uint64_t, const uint4& e, bool cand, uint64_t pre, uint64_t) {
        if (cand) spikes[pre] = (int32_t)e.w;
    });
}

// ---------------------------------------------------------------------------
// k_claim (random mode): every event that will reach the update raises its
// record's claim to its event index + 1, so k_apply lets only the highest
// store (the last writer in event order).
__global__ __launch_bounds__(kApplyThreads) void k_claim(DeviceState d, KernelParams kp, const int32_t* gathered,
                                                         uint32_t rank)
{
    extern __shared__ uint32_t s_pre[];
    __shared__ uint64_t s_red[kWalkWaves];
    const uint64_t pass = *d.pass_index;
    budget_walk(d, rank_offset(kp, gathered, rank), kp.max_spikes, s_pre, s_red,
                [&](uint64_t region, const uint4& e, bool, uint64_t, uint64_t) {
                    const uint64_t t = region + e.x;
                    atomicMax(d.claim + rec_index(d, t, pass), (uint32_t)(t + 1));
                });
}

// ---------------------------------------------------------------------------
// k_apply: weight update (brain.metal:101-122) of the gated events that still
// had budget.  Single GPU (no exchange): the spikes are stamped here
// (brain.metal:125-126, deferred to after every lastFired read of the pass);
// sharded passes stamp from the gathered spike lists in k_finalize.
__global__ __launch_bounds__(kApplyThreads) void k_apply(DeviceState d, KernelParams kp,
                                                         const int32_t* gathered, uint32_t rank)
{
    extern __shared__ uint32_t s_pre[];
    __shared__ uint64_t s_red[kWalkWaves];
    __shared__ uint32_t s_u[kWalkWaves], s_f[kWalkWaves], s_p[kWalkWaves];
    // every gate workgroup has its copy of the filter image: zero it for the next k_bitmap
    for (uint32_t i = blockIdx.x * kApplyThreads + threadIdx.x; i < d.filter_words; i += gridDim.x * kApplyThreads)
        d.filter[i] = 0u;
    const float R = *d.reward, rb = *d.rbar;  // pass-start values (C1), brain.metal:105-106
    const uint64_t now = *d.clock, pass = *d.pass_index;
    const bool random = d.mode == ABNN_MODE_RANDOM, stamp = gathered == nullptr;
    const bool prune = kp.w_prune > 0.0f, genesis = d.grown != nullptr && kp.p_new > 0.0f;
    uint32_t upd = 0, nf = 0, npr = 0;
    budget_walk(d, rank_offset(kp, gathered, rank), kp.max_spikes, s_pre, s_red,
                [&](uint64_t region, const uint4& e, bool f, uint64_t pre, uint64_t slot) {
        const float w = updated_weight(kp, __uint_as_float(e.z), f, R, rb, __uint_as_float(e.y & 0x7FFFFFFFu));
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
        if (f) {
            if (stamp) d.last_fired[e.w] = now;  // brain.metal:125-126
            ++nf;
            if (genesis) {  // README §5 synaptogenesis: slot `pre` of this pass
                const uint64_t x = splitmix64_at(d.seed ^ ABNN_GENESIS_KEY, (pass << 32) | pre);
                if (unit24(x) < kp.p_new) {
                    const uint64_t span = d.n_nrn - d.n_input;
                    d.grown[(pass % kp.compact_every) * kp.max_spikes + pre] =
                        make_uint4(d.g2src[slot], d.n_input + (uint32_t)(((x & 0xFFFFFFFFull) * span) >> 32),
                                   __float_as_uint(kp.w_init), 1u);
                }
            }
        }
    });
    // per-workgroup partials (atomics from every wave on one address serialise)
    const uint32_t wu = wave_sum(upd), wf = wave_sum(nf), wp = wave_sum(npr);
    if ((threadIdx.x & 63) == 0) {
        s_u[threadIdx.x >> 6] = wu;
        s_f[threadIdx.x >> 6] = wf;
        s_p[threadIdx.x >> 6] = wp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        uint4 t = make_uint4(0u, 0u, 0u, 0u);
        for (uint32_t v = 0; v < kWalkWaves; ++v) {
            t.x += s_u[v];
            t.y += s_f[v];
            t.z += s_p[v];
        }
        d.apply_partial[blockIdx.x] = t;
    }
}

// ---------------------------------------------------------------------------
// k_finalize: rBar (brain.metal:110-113), clock tick (brain.metal:129),
// statistics; in sharded passes also the deferred stamps of every rank's
// spikes from the gathered exchange records (brain.metal:125-126).  One
// workgroup.
__global__ __launch_bounds__(kScanThreads) void k_finalize(DeviceState d, KernelParams kp,
                                                           const int32_t* gathered, uint32_t world)
{
    constexpr uint32_t kU = 4;
    const uint32_t tid = threadIdx.x, words = xchg_words(kp.max_spikes);
    const uint64_t now = *d.clock;
    const uint64_t budget = kp.max_spikes;
    uint64_t events = d.events, off = 0;
    int64_t t0 = d.work->t0_g2;
    if (gathered) {
        events = 0;
        t0 = 0;
        for (uint32_t r = 0; r < world; ++r) {
            const int64_t* sm = reinterpret_cast<const int64_t*>(gathered + r * words);
            const int32_t* sp = gathered + r * words + 2 * ABNN_SUMMARY_WORDS;
            events += (uint64_t)sm[2];
            t0 |= sm[1];
            // rank r's spikes fill budget slots [off, off + n)
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
    }
    uint64_t g1 = 0, g2 = 0;
    for (uint32_t q = tid; q < d.n_ranges; q += kScanThreads) {
        const uint4 ri = d.range_info[q];
        g1 += ri.x;
        g2 += ri.y;
    }
    uint32_t upd = 0, nf = 0, npr = 0;
    if (tid < kWalkBlocks) {
        const uint4 v = d.apply_partial[tid];
        upd = v.x;
        nf = v.y;
        npr = v.z;
    }
    __shared__ uint64_t s_a[kScanThreads / 64], s_b[kScanThreads / 64];
    __shared__ uint32_t s_u[kScanThreads / 64], s_f[kScanThreads / 64], s_p[kScanThreads / 64];
    g1 = wave_sum(g1);
    g2 = wave_sum(g2);
    upd = wave_sum(upd);
    nf = wave_sum(nf);
    npr = wave_sum(npr);
    if ((tid & 63) == 0) {
        s_a[tid >> 6] = g1;
        s_b[tid >> 6] = g2;
        s_u[tid >> 6] = upd;
        s_f[tid >> 6] = nf;
        s_p[tid >> 6] = npr;
    }
    __syncthreads();
    if (tid == 0) {
        uint64_t ta = 0, tb = 0, tu = 0, tf = 0, tp = 0;
        for (int w = 0; w < kScanThreads / 64; ++w) {
            ta += s_a[w];
            tb += s_b[w];
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
        w->t0_g2 = 0;  // re-armed for the next pass
        w->n_ovf = 0;
        w->stats.passes += 1;
        w->stats.events += d.events;
        w->stats.pre_gated += ta;
        w->stats.post_gated += tb;
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

// budget walks: s_pre holds one u32 per range
inline size_t walk_lds(const DeviceState& d) { return (size_t)std::max(1u, d.n_ranges) * 4; }

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
    hipLaunchKernelGGL(k_refrac, dim3(kRefracBlocks), dim3(256), 0, s, d, kp);
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

hipError_t launch_scan(const DeviceState& d, const KernelParams& kp, int32_t* xchg_out, hipStream_t s)
{
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(kScanThreads), 0, s, d, kp, xchg_out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // at least one workgroup: it also zeroes the filter image (no ranges: a no-op walk)
    hipLaunchKernelGGL(k_spikes, dim3(kWalkBlocks), dim3(kApplyThreads), walk_lds(d), s, d, kp,
                       xchg_out + 2 * ABNN_SUMMARY_WORDS);
    return hipGetLastError();
}

hipError_t launch_apply(const DeviceState& d, const KernelParams& kp, const int32_t* gathered,
                        uint32_t rank, hipStream_t s)
{
    const dim3 g(kWalkBlocks), b(kApplyThreads);
    if (d.mode == ABNN_MODE_RANDOM) {
        hipLaunchKernelGGL(k_claim, g, b, walk_lds(d), s, d, kp, gathered, rank);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_apply, g, b, walk_lds(d), s, d, kp, gathered, rank);
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
