// kernels.hip -- CDNA4 (gfx950) kernels of one C1 traversal pass (handle API).
//
// Reference hot path: monte_carlo_traversal (abnn/src/core/kernels/brain.metal:41-130)
// and renormalise_clock_and_times (brain.metal:135-145).  DESIGN.md §5 has the
// measured story; in short:
//
//   k_gate<..., kFused> : THE pass of a single-GPU sweep, one launch.
//                Persistent workgroups (one per CU) whose waves each sweep one
//                contiguous range of events (adaptive partition).  Per event
//                the 3-B packed src code (engine.h: a u16 lo and a u8 hi
//                stream) is tested against one 64-bit block of an LDS
//                blocked Bloom filter of the recent-spike bitmap (the
//                pre-spike gate, brain.metal:73-77, pre-selected); hits are
//                staged in LDS and run through the refractory stage by the
//                same wave (exact bitmap bit, {dst, w} gather, lastFired[dst],
//                brain.metal:79-83, candidate test brain.metal:91-92, the
//                updated weight brain.metal:101-121).  A workgroup-level
//                decoupled look-back resolves the ordered spike budget of
//                schedule C1 (brain.metal:85-98 without its races); every wave
//                walks its own survivors, the workgroups owning spikes stamp
//                them once every look-back word is published
//                (brain.metal:125-126), workgroup 0 ends the pass (rBar
//                brain.metal:110-113, clock brain.metal:129).  The next pass's
//                bitmap and filter are built on the way (set-only atomics).
//   k_gate<..., !kFused> + k_apply : the two-kernel pass (sharded passes,
//                random-edge mode, ABNN_FUSED=0): the gate writes per-chunk
//                survivor slots, k_apply walks the budget over them, updates
//                weights (non-temporal stores; pruning, synaptogenesis), stamps,
//                builds the next bitmap and partition, and its last workgroup
//                ends the pass.  Sharded passes add k_scan + k_spikes (the
//                exchange record) after the gate; k_apply then stamps every
//                rank's spikes from the gathered records.  k_claim precedes
//                k_apply in random mode (highest event wins).
//   k_bitmap   : lastFired (8 B/neuron, read once) -> the exact recent-spike
//                bitmap and the filter, with the stimulus stamp; only when the
//                bitmap cannot come from the last passes' spike lists (the
//                first passes, host writes).
//   k_renorm   : brain.metal:135-145 with the base passed by the host (no race).
//   k_compact_inplace / k_span_* / k_tally_dead : the structural update (README §5).
//   k_visits_delta / k_visits_merge : the sharded lastVisited merge.
//
// All fp32 arithmetic is compiled with -ffp-contract=off and written operation
// for operation like the oracle, so weights are bit-identical to the CPU.
// Timestamps are u64; every decision on them is u32 arithmetic (age32,
// device.h), as the reference's `uint` buffers.
#include <algorithm>
#include <type_traits>

#include "engine.h"
#include "device.h"

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

// Global-memory views for agent-scope atomics (sc1 loads and stores).
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;

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

// The packed src of record i (engine.h, SynArrays): 24 bits, kSrcNone for a
// tombstone; src32 widens it to the interchange value (0xFFFFFFFF).
__device__ __forceinline__ uint32_t src_of(const SynArrays& a, uint64_t i)
{
    return code_src(a.lo[i], a.hi[hi_pos(i)]);
}

__device__ __forceinline__ uint32_t src32(uint32_t v) { return v == kSrcNone ? 0xFFFFFFFFu : v; }

__device__ __forceinline__ void set_src(const SynArrays& a, uint64_t i, uint32_t v)
{
    const uint32_t c = src_code(v);
    a.lo[i] = (uint16_t)c;
    a.hi[hi_pos(i)] = (uint8_t)(c >> 16);
    if (a.src32) a.src32[i] = v;
}

// A weight store (brain.metal:122), non-temporal: a plain 4-B store leaves
// scattered dirty partial lines whose write-back lands in the middle of the
// next pass's record stream (write-through sc1 stores measured equal,
// profiles/r03c_ab_wt_sc1.txt).
__device__ __forceinline__ void store_w(const DeviceState& d, uint64_t i, float w)
{
    __builtin_nontemporal_store(w, w_ptr(d.syn, i));
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

// Workgroup barrier for LDS communication only: unlike __syncthreads() it does
// not wait for the wave's outstanding global stores and atomics (a
// workgroup-scope release fence on global memory waits for vmcnt(0)).
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Sum of one u64 per thread over an NT-thread workgroup (every thread gets it).
template <int NT>
__device__ uint64_t block_sum(uint64_t v, uint64_t* s_wave)
{
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = v;
    __syncthreads();
    uint64_t t = 0;
#pragma unroll
    for (uint32_t w = 0; w < NT / 64; ++w) t += s_wave[w];
    __syncthreads();
    return t;
}

// Exclusive scan of one u64 per thread over an NT-thread workgroup.  kLds:
// LDS-only barriers (the waves' outstanding global loads and stores stay in
// flight).
template <int NT = kScanThreads, bool kLds = false>
__device__ uint64_t block_exclusive_scan(uint64_t v, uint64_t* total, uint64_t* s_wave)
{
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    constexpr uint32_t nw = NT / 64;
    uint64_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint64_t y = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += y;
    }
    if (lane == 63) s_wave[wid] = inc;
    if (kLds) lds_barrier();
    else __syncthreads();
    uint64_t before = 0, tot = 0;
    for (uint32_t w = 0; w < nw; ++w) {
        uint64_t x = s_wave[w];
        if (w < wid) before += x;
        tot += x;
    }
    if (kLds) lds_barrier();
    else __syncthreads();
    *total = tot;
    return before + inc - v;
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));  // (the nontemporal builtins take vector types)
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// Pre-spike filter: a blocked Bloom filter of the exact
// recent-spike bitmap, FB 64-bit blocks {low, high} (2 FB u32 words, one LDS
// image).  Bitmap word j (neurons 32 j .. 32 j + 31) is folded into block
// g(j) = (j ^ t) mod FB, t = 0x9E5 (j >> log2 FB) (24-bit multiply): low |=
// the word, high |= the word rotated left by r(j) = t mod 32.  Neuron n (word
// j, bit b) passes iff low bit b and high bit (b + r) mod 32 are set -- one
// 8-B LDS read per event.  Words of one j >> log2 FB share t, so two of them
// never share a block and one other neuron never sets both bits: a false
// positive needs two set neurons in the block (~0.2 % at config 3, 64 KiB),
// no false negatives; the exact bitmap confirms the staged events in the
// refractory stage.
__device__ __forceinline__ uint32_t filter_t(uint32_t j, uint32_t lg) { return __umul24(j >> lg, 0x9E5u); }

// Lane-contiguous sweep (record layout 4, engine.h): a lane's 8 events of a
// 512-event block come as four lo dwords (event k's lo in half k & 1 of dword
// k >> 1) and two hi dwords (event k's hi in byte k & 3 of dword k >> 2).
// The filter block's LDS byte address of the event in half `half` of lo
// dword w: lo & 0xFFF8 (SDWA word select for the high half: one VALU).
__device__ __forceinline__ uint32_t code_addr(uint32_t w, int half)
{
    if (half == 0) return w & 0xFFF8u;
    uint32_t a;
    asm("v_and_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
        : "=v"(a) : "v"(w), "v"(0xFFF8u));
    return a;
}

__device__ __forceinline__ uint2 filter_block_at(const uint2* s_fb, uint32_t addr)
{
    return *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(s_fb) + addr);
}

// The filter test of four consecutive events of a lane (blocks f[0..3]; lo
// dwords w0 = events 0, 1 and w1 = events 2, 3; hi dword h): bit 0 of byte m
// of the result is set iff event m passes.  lb = hi[4:0] is the shift amount
// straight from hi's byte m (SDWA src0_sel); hb = lo[2:0] | hi[7:6] << 3 for
// all four at once: one v_perm gathers the lo bytes, one v_bfi inserts
// hi >> 3 (bits 5..7 of each byte are don't-cares: shifts use [4:0]).  4 VALU
// per event (the layout-3 gate took 6.25: a v_perm per event to assemble the
// code, a shift and a v_bfi for hb).
#define ABNN_SHR_SEL(acc, amt, val, BYTE, KEEP)                                                       \
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:" BYTE " dst_unused:" KEEP " src0_sel:" BYTE           \
        " src1_sel:DWORD"                                                                             \
        : "+v"(acc)                                                                                   \
        : "v"(amt), "v"(val))
__device__ __forceinline__ uint32_t quad_filter(const uint2* f, uint32_t w0, uint32_t w1, uint32_t h)
{
    const uint32_t A = __builtin_amdgcn_perm(w1, w0, 0x06040200u);  // lo[7:0] of events 0..3
    const uint32_t R = (A & 0x07070707u) | ((h >> 3) & ~0x07070707u);  // byte m: hb of event m
    uint32_t HA, HB;
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
        : "=v"(HA) : "v"(h), "v"(f[0].x));
    asm("v_lshrrev_b32_sdwa %0, %1, %2 dst_sel:BYTE_0 dst_unused:UNUSED_PAD src0_sel:BYTE_0 src1_sel:DWORD"
        : "=v"(HB) : "v"(R), "v"(f[0].y));
    ABNN_SHR_SEL(HA, h, f[1].x, "BYTE_1", "UNUSED_PRESERVE");
    ABNN_SHR_SEL(HB, R, f[1].y, "BYTE_1", "UNUSED_PRESERVE");
    ABNN_SHR_SEL(HA, h, f[2].x, "BYTE_2", "UNUSED_PRESERVE");
    ABNN_SHR_SEL(HB, R, f[2].y, "BYTE_2", "UNUSED_PRESERVE");
    ABNN_SHR_SEL(HA, h, f[3].x, "BYTE_3", "UNUSED_PRESERVE");
    ABNN_SHR_SEL(HB, R, f[3].y, "BYTE_3", "UNUSED_PRESERVE");
    return HA & HB & 0x01010101u;
}
#undef ABNN_SHR_SEL

__device__ __forceinline__ void filter_set(uint32_t* f, uint32_t j, uint32_t bits, uint32_t FB, uint32_t lg)
{
    const uint32_t t = filter_t(j, lg), g = (j ^ t) & (FB - 1), r = t & 31u;
    atomicOr(f + 2 * g, bits);
    atomicOr(f + 2 * g + 1, (bits << r) | (bits >> ((32u - r) & 31u)));
    // the second-level filter (engine.h kF2Words), after the blocks: per neuron
    uint32_t* f2 = f + 2 * FB;
    for (uint32_t m = bits; m; m &= m - 1u) {
        const uint32_t n = 32u * j + (uint32_t)__builtin_ctz(m), h1 = f2_hash1(n), h2 = f2_hash2(n);
        atomicOr(f2 + (h1 >> 5), 1u << (h1 & 31u));
        atomicOr(f2 + (h2 >> 5), 1u << (h2 & 31u));
    }
}

// The second-level filter test on an LDS copy: false for no recent neuron
// (no false negatives), true for ~a tenth of the others.
__device__ __forceinline__ bool f2_test(const uint32_t* s_f2, uint32_t n)
{
    const uint32_t h1 = f2_hash1(n), h2 = f2_hash2(n);
    return ((s_f2[h1 >> 5] >> (h1 & 31u)) & (s_f2[h2 >> 5] >> (h2 & 31u)) & 1u) != 0u;
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
            bit = age32(now, L[q]) <= kp.window_pre;
        }
        const uint64_t m = __ballot(bit);
        if (lane == 0 && (wave * 4 + q) * 64 < d.n_nrn) {
            reinterpret_cast<uint64_t*>(d.bitmap)[wave * 4 + q] = m;
            // fold into the filter (zeroed by the pass before; few words are
            // non-zero)
            const uint32_t w0 = (uint32_t)(wave * 4 + q) * 2u;
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t part = (uint32_t)(m >> (32 * h));
                if (part) filter_set(d.filter, w0 + h, part, d.filter_words, d.filter_log2);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Steady state: the next pass's bitmap and filter images are
// built by k_apply instead of k_bitmap.  With the clock advancing by one per
// pass and no host-written stamp recent (the host checks, capi.hip
// build_next_ok), neuron n is recent at pass p+1 iff it was stamped by a spike
// of passes p+1-W..p (the spike lists: fired_ring, and this pass's spikes as
// k_apply stamps them) or by the stimulus of passes p+1-W..p+1 (W =
// window_pre).  Both buffers of pass p+1 were zeroed by the gate of pass p,
// so the build only sets bits: the order of the word atomics does not matter.
__device__ __forceinline__ void recent_set_next_word(const DeviceState& d, uint32_t j, uint32_t bits)
{
    atomicOr(d.bitmap_next + j, bits);
    filter_set(d.filter_next, j, bits, d.filter_words, d.filter_log2);
}

// Wave-converged form: the lanes with act set neuron n.  The spike lists
// repeat neurons (a neuron fires from many synapses, and the dense
// input->output block makes the 256 outputs fire over and over in the first
// passes), and same-address atomics serialise (~12 ns each): the lanes that
// share the first active lane's bitmap word are merged into one set of three
// atomics, for up to kMerge rounds while merging pays (a group of one ends it).
__device__ __forceinline__ void wave_set_next(const DeviceState& d, bool act, uint32_t n)
{
    constexpr int kMerge = 8;
    const uint32_t lane = threadIdx.x & 63, j = n >> 5;
    for (int it = 0; it < kMerge; ++it) {
        const uint64_t m = __ballot(act);
        if (m == 0) return;
        const uint32_t lead = (uint32_t)__builtin_ctzll(m);
        const uint32_t jl = (uint32_t)__builtin_amdgcn_readlane((int)j, (int)lead);
        const bool same = act && j == jl;
        const uint64_t g = __ballot(same);
        if (__popcll(g) == 1) break;  // no repeats at the head: plain atomics
        uint32_t bits = same ? 1u << (n & 31u) : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) bits |= __shfl_xor(bits, o, 64);
        if (lane == lead) recent_set_next_word(d, jl, bits);
        act = act && !same;
    }
    if (act) recent_set_next_word(d, j, 1u << (n & 31u));
}

// Fused pass: wave_set_next behind a per-workgroup LDS cache of the bitmap
// words this workgroup has already set this pass (a direct-mapped {word, bits}
// per slot, written whole as one 8-B LDS word, so an entry never claims a bit
// it has not set; a lost update only costs a repeated atomic).  The dense
// input->output ranges fire the 256 outputs over and over: without it their
// same-word atomics serialise the walk.
constexpr uint32_t kSetCache = 256;

__device__ __forceinline__ void wave_set_next_dedup(const DeviceState& d, bool act, uint32_t n, uint64_t* cache)
{
    const uint32_t j = n >> 5, bit = 1u << (n & 31u);
    uint64_t* c = cache + (j & (kSetCache - 1));
    if (act) {
        const uint64_t e = *c;
        if ((uint32_t)(e >> 32) == j && ((uint32_t)e & bit)) act = false;
    }
    if (__ballot(act) == 0) return;
    wave_set_next(d, act, n);
    if (act) {
        const uint64_t e = *c;
        const uint32_t b = (uint32_t)(e >> 32) == j ? (uint32_t)e | bit : bit;
        *c = (uint64_t)j << 32 | b;
    }
}

// The items of the build that do not depend on this pass: the spike lists of
// passes p+1-W..p-1 and the stimulus ranges.  Item x of k_apply thread t of
// workgroup g is x = t * gridDim + g (every workgroup gets a few), its loads
// issued at kernel entry (next_item_load, both at once: the list entry is read
// whether or not it is below the list's length) so they land during the walk
// prefix; the atomics follow the walk (next_item_set).  Items beyond one per
// thread (more than 256 K) are walked after it.
struct NextItem {
    uint32_t n, lim, i;  // neuron; valid iff i < lim
};

__device__ __forceinline__ uint64_t next_items(const DeviceState& d, const KernelParams& kp)
{
    const uint32_t W = kp.window_pre, nl = W > 0 ? W - 1 : 0;
    uint64_t items = (uint64_t)nl * kp.max_spikes;
    for (uint32_t r = 0; r < d.n_next_stim; ++r) items += d.next_stim[r][1];
    return items;
}

__device__ __forceinline__ NextItem next_item_load(const DeviceState& d, const KernelParams& kp, uint64_t pass, uint64_t x)
{
    const uint32_t M = kp.max_spikes, W = kp.window_pre, nl = W > 0 ? W - 1 : 0;
    if (x < (uint64_t)nl * M) {
        const uint32_t k = (uint32_t)(x / M), i = (uint32_t)(x - (uint64_t)k * M);
        const uint64_t q = (pass - nl + k) & (kFiredRing - 1);  // passes p+1-W .. p-1
        return NextItem{d.fired_ring[q * M + i], d.n_fired_ring[q], i};
    }
    uint64_t y = x - (uint64_t)nl * M;
    uint32_t r = 0;
    while (y >= d.next_stim[r][1]) y -= d.next_stim[r++][1];
    return NextItem{(uint32_t)(d.next_stim[r][0] + y), 1u, 0u};
}

// ---------------------------------------------------------------------------
// Per-range results of the gate.  A range is the contiguous block of events
// one gate wave sweeps; range order = event order.  Events that pass the LDS
// filter are staged as {offset, src} and cut, in event order, into chunks of
// kChunk, each run through the refractory stage by the gate wave itself: a
// full chunk as soon as it fills (dense parts of the graph, warm-up passes;
// the adaptive partition gives such ranges fewer events), the range's last
// chunk once its stream is done.  Chunk c's survivors occupy [region + c
// kChunk, ...) of g2x.  No atomics anywhere near the stream: a same-address
// atomic per wave stalls every concurrent stream
// (profiles/r01n_ubench_soa_atomic.txt).
//   g2x entry       = {event - region, isi bits | candidate << 31, w bits, dst},
//                     isi = (float)(now - lastFired[dst]) >= 0 (sign bit free),
//                     w, dst as read at pass start (C1)
//   range_info[r]   = {gate time, survivors, candidates, full chunks}, whole range;
//   range_g1[r]     = its pre-gated events (statistics)
//   chunk_cnt[slot] = {pre-gated, survivors, candidates, 0} of a full chunk;
//                     slots of full chunks never collide; the last chunk holds
//                     the range's survivors minus the full chunks'.

__device__ __forceinline__ uint64_t region_of(const DeviceState& d, uint32_t r)
{
    return (uint64_t)d.range_bounds[r] * d.iter_events;
}

__device__ __forceinline__ uint64_t chunk_slot(uint64_t region, uint32_t c)
{
    return (region + (uint64_t)c * kChunk) / kChunkSlotDiv;
}

// Counts of a whole range (the gate wave sums its chunks).
__device__ __forceinline__ uint4 range_totals(const DeviceState& d, uint32_t r) { return d.range_info[r]; }

// Refractory stage of n <= kChunk staged events of one chunk, by one wave, in
// event order: the exact pre-spike gate on the bitmap word of src
// (brain.metal:73-77; the filter only pre-selected), then for the events that
// pass: dst and w gathered from the record arrays, the 8-B lastFired[dst]
// gather, the refractory gate (brain.metal:79-83), the candidate test
// (brain.metal:91-92) and isi (brain.metal:116); survivors are written
// compacted from g2x[base] on.  `at(q)` yields the q-th staged {offset, src}.
// Batches of R rounds of 64 keep every load of a lane in flight at once.
// Returns {pre-gated, survivors, candidates, 0}.
// kFused: the entry is {offset | candidate << 31, w, updated w, dst} -- every
// input of the update (brain.metal:101-121) is known here (w, the candidate
// bit, isi, the pass-start reward and rBar); the budget walk only decides
// whether the event is below the budget (then fired = candidate).  With spec
// (the workgroup is predicted to lie below the pass's budget cut) the updated
// weight is stored here already; the walk restores w where the prediction was
// wrong.
template <int R, bool kRandom, bool kFused, bool kTail, class At>
__device__ __forceinline__ uint4 refrac_chunk(const DeviceState& d, const KernelParams& kp, uint64_t region,
                                              uint64_t base, uint32_t n, uint64_t now, uint64_t pass, float Rw,
                                              float rbw, bool spec, uint32_t crange, uint32_t c0,
                                              const uint32_t* s_f2, At&& at, uint4* lds_out = nullptr)
{
    const uint32_t lane = threadIdx.x & 63, nn = (uint32_t)d.n_nrn;
    uint32_t n_g1 = 0, n_g2 = 0, n_cand = 0;
    auto record_of = [&](uint32_t rel) -> uint64_t {
        const uint64_t t = region + rel;
        return kRandom ? pick_record(d.seed, d.syn_offset, pass, t, d.n_syn) : t;
    };
    for (uint32_t b0 = 0; b0 < n; b0 += R * 64) {
        uint32_t rel[R], src[R], bw[R], dst[R];
        float w[R];
        uint64_t ld[R];
        uint2 dw[R];
        bool f2[R];
        // one dependent round trip for both, only for the events the
        // second-level filter passes (LDS: the recent ones and ~a tenth of the
        // blocked filter's false positives; it holds every recent neuron, so
        // it has no false negatives): the exact bitmap word of src and the
        // record's {dst, w}.  (Round 4 read the bitmap word for every staged
        // event: each random read costs the CU's vector-memory path)
        if constexpr (!kTail) {
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const uint32_t q = b0 + j * 64 + lane;
                const uint2 e = q < n ? at(q) : make_uint2(0u, 0xFFFFFFFFu);
                rel[j] = e.x;
                // the sweep stages the record's code (engine.h, src_code), random mode its src
                src[j] = kRandom || q >= n ? e.y : code_src(e.y & 0xFFFFu, e.y >> 16);
                f2[j] = src[j] < nn && f2_test(s_f2, src[j]);
                bw[j] = f2[j] ? d.bitmap[src[j] >> 5] : 0u;
                dw[j] = f2[j] ? d.syn.dw[record_of(rel[j])] : make_uint2(0xFFFFFFFFu, 0u);  // one access for both
            }
        } else {
            // the range's tail (after its stream: no stream registers live):
            // straight-line (no per-round branches, so every access of a phase is
            // in flight at once): lanes past n and rejected events read a safe
            // address (the stage's spare slots, word 0, record 0) and discard it.
            // (n <= kChunk <= R * 64 entries of a stage of kChunk + 128)
            uint2 e[R];
#pragma unroll
            for (int j = 0; j < R; ++j) e[j] = at(b0 + j * 64 + lane);
            uint32_t fa[R], fb[R];
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const bool v = b0 + j * 64 + lane < n;
                rel[j] = e[j].x;
                // the sweep stages the record's code (engine.h, src_code), random mode its src
                src[j] = !v ? 0xFFFFFFFFu : (kRandom ? e[j].y : code_src(e[j].y & 0xFFFFu, e[j].y >> 16));
                const uint32_t sn = src[j] < nn ? src[j] : 0u;
                fa[j] = s_f2[f2_hash1(sn) >> 5];
                fb[j] = s_f2[f2_hash2(sn) >> 5];
            }
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const uint32_t sn = src[j] < nn ? src[j] : 0u;
                f2[j] = src[j] < nn && ((fa[j] >> (f2_hash1(sn) & 31u)) & (fb[j] >> (f2_hash2(sn) & 31u)) & 1u);
                bw[j] = d.bitmap[f2[j] ? sn >> 5 : 0u];
                dw[j] = d.syn.dw[f2[j] ? record_of(rel[j]) : 0];
            }
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const bool g1 = f2[j] && src[j] < nn && ((bw[j] >> (src[j] & 31u)) & 1u);  // brain.metal:73-77, exact
            bw[j] = g1;
            if (!g1) dw[j] = make_uint2(0xFFFFFFFFu, 0u);
            dst[j] = dw[j].x;  // tombstones (dst = 0xFFFFFFFF) never pass
            w[j] = __uint_as_float(dw[j].y);
        }
        // the stimulus of this pass is stamped `now` (brain.cpp:82) by k_bitmap
        // or, in steady state, by the gate itself at some point of the pass
        if constexpr (!kTail) {
#pragma unroll
            for (int j = 0; j < R; ++j)
                ld[j] = dst[j] - d.stim_first < d.stim_count ? now : (dst[j] < nn ? d.last_fired[dst[j]] : 0ull);
        } else {
#pragma unroll
            for (int j = 0; j < R; ++j) {
                ld[j] = d.last_fired[dst[j] < nn ? dst[j] : 0u];
            }
#pragma unroll
            for (int j = 0; j < R; ++j)
                ld[j] = dst[j] - d.stim_first < d.stim_count ? now : (dst[j] < nn ? ld[j] : 0ull);
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {
            if (b0 + (uint32_t)j * 64 >= n) break;  // wave-uniform
            n_g1 += (uint32_t)__popcll(__ballot(bw[j] != 0u));
            const bool g2 = dst[j] < nn && age32(now, ld[j]) > kp.refractory;  // brain.metal:79-83
            const uint64_t tg = d.syn_offset + region + rel[j];
            const bool cand = g2 && spike_candidate(kp, w[j], tg, now);
            const uint64_t bg = __ballot(g2), bcd = __ballot(cand);
            if (g2) {
                const uint64_t o = base + n_g2 + mbcnt64(bg);
                if constexpr (kFused) {
                    const float wn = updated_weight(kp, w[j], cand, Rw, rbw, (float)age32(now, ld[j]));
                    const uint4 ent = make_uint4(rel[j] | (cand ? 0x80000000u : 0u), __float_as_uint(w[j]),
                                                 __float_as_uint(wn), dst[j]);
                    if (kTail && lds_out) {
                        // the fused tail keeps its survivors in LDS (fused_end's
                        // walk reads them there, and stores the weights)
                        lds_out[n_g2 + mbcnt64(bg)] = ent;
                    } else {
                        d.g2x[o] = ent;
                        if (spec) store_w(d, region + rel[j], wn);  // brain.metal:122
                        const uint32_t ci = c0 + n_cand + mbcnt64(bcd);  // the range's candidate index
                        if (cand && ci < kCandCap)
                            d.cand_list[crange * kCandCap + ci] =
                                make_uint2((uint32_t)(base - region) + n_g2 + mbcnt64(bg), dst[j]);
                    }
                } else {
                    const uint32_t isi = __float_as_uint((float)age32(now, ld[j])) | (cand ? 0x80000000u : 0u);
                    d.g2x[o] = make_uint4(rel[j], isi, __float_as_uint(w[j]), dst[j]);
                }
                if (d.g2src) d.g2src[o] = src[j];  // synaptogenesis keeps src
                if (tg == 0) {  // read by workgroup 0 at the pass's end (fused pass): write-through,
                                // drained before this wave reaches the barrier its workgroup's
                                // look-back word is published behind (the sc1 hand-off form,
                                // MI355X_MICROARCH.md §inter-workgroup visibility); once per pass
                    __hip_atomic_store((gu32*)&d.work->t0_g2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
            n_g2 += (uint32_t)__popcll(bg);
            n_cand += (uint32_t)__popcll(bcd);
        }
    }
    return make_uint4(n_g1, n_g2, n_cand, 0u);
}

// ---------------------------------------------------------------------------
// The weight update of one event that reached it (brain.metal:101-126), shared
// by k_apply and the fused pass.  Per-pass inputs are the pass-start scalars
// (C1); the counters are the caller's.
struct ApplyCtx {
    float R, rb;
    uint64_t now, pass;
    bool random;     // random-edge mode: only the claim's winner stores
    bool stamp;      // stamp lastFired[dst] = now here (k_apply, single GPU)
    bool ring;       // write the spike list (fired_ring, budget position)
    bool ring_sc1;   // ... write-through: the fused pass's last workgroup reads it in-launch
    bool prune, genesis;
    bool precomputed;  // the entry holds the updated weight (fused pass: refrac_chunk<..., kFused>)
    uint32_t upd, nf, npr;
    uint32_t* lds_spk = nullptr;  // fused pass: the workgroup's spikes also go to LDS (fused_end stamps
    uint32_t lds_s0 = 0;          // them from there), budget position pre at lds_spk[pre - lds_s0]
};

// A spike of the pass (brain.metal:125-126): stamp (k_apply), the spike list
// (budget position pre), synaptogenesis.
__device__ __forceinline__ void record_spike(const DeviceState& d, const KernelParams& kp, ApplyCtx& c,
                                             const uint4& e, uint64_t pre, uint64_t slot)
{
    if (c.stamp) d.last_fired[e.w] = c.now;  // brain.metal:125-126
    if (c.lds_spk) c.lds_spk[pre - c.lds_s0] = e.w;
    if (c.ring) {
        uint32_t* q = d.fired_ring + (c.pass & (kFiredRing - 1)) * kp.max_spikes + pre;
        if (c.ring_sc1) __hip_atomic_store((gu32*)q, e.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else *q = e.w;
    }
    ++c.nf;
    if (c.genesis) {  // README §5 synaptogenesis: slot `pre` of this pass
        const uint64_t x = splitmix64_at(d.seed ^ ABNN_GENESIS_KEY, (c.pass << 32) | pre);
        if (unit24(x) < kp.p_new) {
            const uint64_t span = d.n_nrn - d.n_input;
            d.grown[(c.pass % kp.compact_every) * kp.max_spikes + pre] =
                make_uint4(d.g2src[slot], d.n_input + (uint32_t)(((x & 0xFFFFFFFFull) * span) >> 32),
                           __float_as_uint(kp.w_init), 1u);
        }
    }
}

__device__ __forceinline__ void apply_event(const DeviceState& d, const KernelParams& kp, ApplyCtx& c,
                                            uint64_t region, const uint4& e, bool f, uint64_t pre, uint64_t slot)
{
    const float w = c.precomputed ? __uint_as_float(e.z)
                                  : updated_weight(kp, __uint_as_float(e.z), f, c.R, c.rb, __uint_as_float(e.y & 0x7FFFFFFFu));
    const uint64_t t = region + e.x, ri = c.random ? rec_index(d, t, c.pass) : t;
    // random mode: of the events that updated one synapse this pass, the
    // highest (k_claim) stores its weight; every one of them still counts
    const bool store = !c.random || d.claim[ri] == (uint32_t)(t + 1);
    if (c.random && store) d.claim[ri] = 0u;  // re-armed for the next pass
    // brain.metal:122.  Non-temporal: a plain 4-B store leaves ~160k
    // scattered dirty partial lines per pass whose write-back lands in the
    // middle of the next pass's record stream (+30 us of gate time,
    // tools/exp_variants.py).
    if (store && c.prune && w < kp.w_prune) {  // README §5: the synapse is removed
        set_src(d.syn, ri, kSrcNone);
        __builtin_nontemporal_store((uint64_t)__float_as_uint(w) << 32 | 0xFFFFFFFFull,
                                    reinterpret_cast<uint64_t*>(d.syn.dw + ri));  // {dst, w} as one 8-B store
        if (d.dead) atomicAdd(d.dead + ri / kCompactChunk, 1u);  // tally for the structural update
        ++c.npr;
    } else if (store) {
        store_w(d, ri, w);
    }
    ++c.upd;
    if (f) record_spike(d, kp, c, e, pre, slot);
}

// One boundary of the adaptive sweep partition (partition_bounds below, and
// the fused pass's prologue): boundary k moves adapt_gain / 4 of the way from
// `from` (its place this pass) towards the iteration where a measured
// cumulative gate cost cc (exclusive prefix over the ranges of bounds rb,
// cc[NR] = total) reaches k / NR of the total, rounded to the nearest
// iteration.
__device__ __forceinline__ uint32_t adapted_bound(const DeviceState& d, const uint32_t* cc, const uint32_t* rb,
                                                  uint32_t NR, uint32_t k, uint32_t total_cost, uint32_t from,
                                                  uint32_t gain = 0)
{
    uint32_t nb = from;
    if (d.adapt_ranges && k > 0 && k < NR && total_cost > 0) {
        const uint32_t T = (uint32_t)((uint64_t)k * total_cost / NR);
        uint32_t lo = 0, hi = NR;  // last range with cc <= T (its cost is > 0)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (cc[mid] <= T) lo = mid;
            else hi = mid;
        }
        // target in 1/256 iterations; both terms of the move are monotonic
        // in k, so ranges never overlap
        const uint32_t cr = cc[lo + 1] - cc[lo];
        const uint64_t tfp = (uint64_t)rb[lo] * 256u +
                             (cr ? (uint64_t)(T - cc[lo]) * (rb[lo + 1] - rb[lo]) * 256u / cr : 0u);
        const uint32_t g = gain ? gain : d.adapt_gain;
        nb = (uint32_t)(((uint64_t)from * 256u * (4u - g) + tfp * g + 512u) >> 10);
    }
    return nb;
}

// ---------------------------------------------------------------------------
// Fused single-GPU sweep pass (k_gate<..., kFused>): the budget
// walk of k_apply moves into the gate waves, with a decoupled look-back at
// workgroup level.  When every wave of workgroup b is through its refractory
// stage, b publishes the spike candidates of its ranges (capped at the
// budget) in its look-back word; wave 0 then sweeps the words of ALL lower
// workgroups in one poll (up to 8 per lane, write-through loads) until they are
// all published -- their sum (capped) is the candidates before b -- and every
// wave walks its own survivors from there.  The words are tagged with the
// pass's epoch, so none is reset between passes.  Every published value is a
// lower bound of the candidates before b, so a workgroup stops waiting as soon
// as the published ones reach the budget: workgroups past the budget's end
// never wait for stragglers.  Once EVERY word is published, every refractory
// stage of the pass (the lastFired reads) is done: the workgroups that own
// spikes stamp them (brain.metal:125-126) and workgroup 0 ends the pass --
// no ticket, no last workgroup.
constexpr uint32_t kLbMaxWords = 8;  // look-back words per lane: gate_blocks <= 512

// One wave sweeps the words of workgroups [0, n): their values (capped sum)
// once all carry `tag`, or as soon as the published ones reach the budget
// (stop_at_budget).  vals: this lane's words (q = 64 i + lane), for the caller.
// pub != 0: this workgroup's own word, published by lane 0 right after the
// first sweep's loads are issued (a load issued after a store waits for it:
// vmcnt counts both, in order).
__device__ uint32_t wg_poll(const DeviceState& d, uint32_t n, uint32_t tag, uint32_t budget, bool stop_at_budget,
                            uint32_t (&vals)[kLbMaxWords], uint64_t pub = 0)
{
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t spins = 0;; ++spins) {  // wave-uniform
        uint64_t sum = 0;
        bool ok = true;
        uint64_t raw[kLbMaxWords];
#pragma unroll
        for (uint32_t i = 0; i < kLbMaxWords; ++i) {
            const uint32_t q = i * 64 + lane;
            raw[i] = 0;
            if (i * 64 < n && q < n)
                raw[i] = __hip_atomic_load((gu64*)(d.lb_status + q), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (pub && spins == 0) {
            __builtin_amdgcn_sched_barrier(0);
            if (lane == 0)
                __hip_atomic_store((gu64*)(d.lb_status + blockIdx.x), pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (uint32_t i = 0; i < kLbMaxWords; ++i) {
            const uint32_t q = i * 64 + lane;
            vals[i] = 0u;
            if (i * 64 < n && q < n) {
                const bool mine = (uint32_t)(raw[i] >> 32) == tag;
                vals[i] = mine ? (uint32_t)raw[i] & 0x3FFFFFFFu : 0u;
                sum += vals[i];
                ok = ok && mine;
            }
        }
        const uint64_t tot = wave_sum<uint64_t>(sum);
        if (__ballot(!ok) == 0 || (stop_at_budget && tot >= budget)) return (uint32_t)(tot < budget ? tot : budget);
        if (spins >= kLbSpinLimit) {  // never hang the GPU: report and go on
            if (lane == 0) __hip_atomic_store(d.err_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return budget;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// The NEXT pass's boundaries of this workgroup's ranges, range_bounds_next[k]
// for k in [b NW, (b + 1) NW) (and NR by the last workgroup), by ONE wave --
// the first of the workgroup through its refractory stage, so off the
// critical path.  With prologue_adapt they move from this pass's bounds
// towards the cost curve the previous pass measured over its bounds (cost_in
// over range_bounds_prev: one pass more lag than k_apply's partition_bounds,
// which moves from the bounds its costs were measured over); cc: the LDS
// exclusive cost prefix (NR + 1 u32).  Otherwise they stay.
template <int NW>
__device__ void fused_next_bounds(const DeviceState& d, uint32_t* cc)
{
    const uint32_t lane = threadIdx.x & 63, NR = d.n_ranges, k = blockIdx.x * NW + lane;
    const bool mine = (lane < (uint32_t)NW || k == NR) && k <= NR;  // this workgroup's boundaries
    if (!d.prologue_adapt || !d.adapt_ranges || NR < 2) {  // wave-uniform
        if (mine) d.range_bounds_next[k] = d.range_bounds[k];
        return;
    }
    // the costs are in cc already (the prologue's LDS-DMA): rows of 64, 8
    // rows read at once, each row scanned across the wave (DPP) on top of the
    // rows before it, in place
    const uint32_t rows = (NR + 63) / 64;  // NR <= kFusedMaxRanges
    uint32_t run = 0, cmax = 0;
    for (uint32_t j0 = 0; j0 < rows; j0 += 8) {  // wave-uniform
        uint32_t v[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            const uint32_t q = (j0 + u) * 64 + lane;
            v[u] = q < NR ? cc[q] : 0u;
            cmax = v[u] > cmax ? v[u] : cmax;
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; ++u) {
            const uint32_t q = (j0 + u) * 64 + lane;
            const uint32_t inc = wave_incl_scan(v[u]);
            if (q < NR) cc[q] = run + inc - v[u];
            run += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        }
    }
    const uint32_t total = run;
    if (lane == 0) cc[NR] = total;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
    // a range above 4x the mean cost (a dense stretch the records just grew:
    // a structural update's hole takes the array's last records, the grown
    // ones of the update before, whose src fired -- all pre-gated, refractory
    // chunk after chunk) moves every boundary the whole way to the measured
    // target this pass, instead of a quarter of it for ~10 passes at twice
    // the pass time; one gain for every boundary keeps the ranges ordered.
    // Steady-state noise (the slowest range ~1.2x the mean) never reaches it.
    for (int o = 32; o > 0; o >>= 1) {
        const uint32_t x = (uint32_t)__shfl_xor((int)cmax, o, 64);
        cmax = x > cmax ? x : cmax;
    }
    const uint32_t gain = (uint64_t)cmax * NR > 4ull * total ? 4u : 0u;
    if (mine) d.range_bounds_next[k] = adapted_bound(d, cc, d.range_bounds_prev, NR, k, total, d.range_bounds[k], gain);
}

// The walk of one range's survivors (the fused pass's g2x entries, contiguous
// from g2x[region]; C of them spike candidates) in event order from budget
// position P: the ordered budget of C1 (brain.metal:85-98), the weight update
// (brain.metal:101-122; stored by refrac_chunk already when spec) and the
// spikes (brain.metal:125-126: spike list, synaptogenesis; set_next: into the
// next pass's bitmap).  Returns the survivors below the budget that were
// stored by refrac_chunk and not visited (wave-uniform); ac counts the rest.
__device__ __forceinline__ uint32_t range_walk(const DeviceState& d, const KernelParams& kp, ApplyCtx& ac, uint32_t r,
                                               uint64_t region, uint32_t S, uint32_t C, uint64_t P, bool spec,
                                               bool set_next, uint64_t* setc)
{
    constexpr uint32_t RW = 4;  // rounds of survivors per walk batch (two batches in flight)
    const uint32_t lane = threadIdx.x & 63, budget = kp.max_spikes;
    // batches of RW x 64 survivors; the next batch's loads are issued before
    // this one's stores (gfx9's vmcnt also counts stores: a load issued after
    // them would wait for them)
    uint4 e[RW];
    auto load_batch = [&](uint32_t b0, uint4 (&x)[RW]) {
#pragma unroll
        for (uint32_t j = 0; j < RW; ++j) {
            const uint32_t q = b0 + j * 64 + lane;
            x[j] = q < S ? d.g2x[region + q] : make_uint4(0u, 0u, 0u, 0u);
        }
    };
    // spec (refrac_chunk stored every updated weight already): only the
    // spikes, and a restore of w from the budget's end on; once every
    // candidate of the range is below the budget the rest needs nothing.
    // Otherwise the walk of k_apply, which ends at the budget.
    uint32_t upd_rest = 0;  // spec: survivors below the budget not visited (wave-uniform)
    uint32_t seen = 0;      // candidates visited
    // spec, below the budget, every candidate of the range listed (cand_list):
    // the spikes come from the list, not from a walk of every survivor (a
    // dense range holds thousands, a walk of them is a chain of dependent
    // batches).  Survivors up to the budget's last candidate were stored by
    // refrac_chunk; the ones after it are restored.
    const bool listed = spec && C <= kCandCap && P < budget;
    if (listed) {
        const uint32_t k = (uint32_t)(budget - P);  // budget left, >= 1
        const uint32_t nb = C < k ? C : k;          // candidates below the budget
        const uint2* cl = d.cand_list + (uint64_t)r * kCandCap;
        for (uint32_t i0 = 0; i0 < nb; i0 += 64) {  // wave-uniform
            const uint32_t i = i0 + lane;
            const uint2 c = i < nb ? cl[i] : make_uint2(0u, 0xFFFFFFFFu);
            if (i < nb) record_spike(d, kp, ac, make_uint4(0u, 0u, 0u, c.y), P + i, region + c.x);
            if (set_next) wave_set_next_dedup(d, i < nb, c.y, setc);  // this pass's spikes
        }
        // survivors below the budget: all, or through the k-th candidate
        upd_rest = C < k ? S : wave_uniform(cl[k - 1].x) + 1u;
        for (uint32_t q = upd_rest + lane; q < S; q += 64) {  // mispredicted tail: w stays (brain.metal:85-88)
            const uint2 x = *reinterpret_cast<const uint2*>(d.g2x + region + q);  // {offset | cand, w}
            store_w(d, region + (x.x & 0x7FFFFFFFu), __uint_as_float(x.y));
        }
    }
    const bool walk = !listed && (spec ? !(C == 0 && P < budget) : P < budget) && S > 0;
    if (!walk && spec && !listed) upd_rest = S;
    if (!walk) return upd_rest;
    // (every load issued here is consumed before the function returns: a
    // load left pending would make the compiler wait for it -- and, vmcnt
    // being in order, for every store before it -- where the walk paths
    // merge, on every path, the LDS-only ones included)
    load_batch(0, e);
    for (uint32_t b0 = 0; b0 < S; b0 += RW * 64) {  // wave-uniform
        if (!spec && P >= budget) break;
        if (spec && P < budget && seen == C) {
            upd_rest = S - b0;
            break;
        }
        uint4 en[RW];
        if (b0 + RW * 64 < S) load_batch(b0 + RW * 64, en);
#pragma unroll
        for (uint32_t j = 0; j < RW; ++j) {
            if (b0 + j * 64 >= S || (!spec && P >= budget)) break;  // wave-uniform
            const uint32_t q = b0 + j * 64 + lane;
            const bool v = q < S, cand = v && (e[j].x >> 31);
            const uint4 x = make_uint4(e[j].x & 0x7FFFFFFFu, e[j].y, e[j].z, e[j].w);
            const uint64_t bc = __ballot(cand);
            const uint64_t pre = P + mbcnt64(bc);  // spike candidates before this event
            const bool below = v && pre < budget;
            if (!spec) {
                if (below) apply_event(d, kp, ac, region, x, cand, pre, region + q);
            } else if (below) {
                ++ac.upd;
                if (cand) record_spike(d, kp, ac, x, pre, region + q);
            } else if (v) {  // mispredicted: past the budget, w stays (brain.metal:85-88)
                store_w(d, region + x.x, __uint_as_float(x.y));
            }
            if (set_next) wave_set_next_dedup(d, cand && pre < budget, x.w, setc);  // this pass's spikes
            P += (uint64_t)__popcll(bc);
            seen += (uint32_t)__popcll(bc);
        }
#pragma unroll
        for (uint32_t j = 0; j < RW; ++j) e[j] = en[j];
    }
#pragma unroll
    for (uint32_t j = 0; j < RW; ++j) asm volatile("" ::"v"(e[j].x), "v"(e[j].y), "v"(e[j].z), "v"(e[j].w));
    return upd_rest;
}

// The fused tail's survivors (refrac_chunk lds_out: S entries {offset |
// candidate << 31, w, updated w, dst} in LDS, event order) from budget
// position P: the ordered budget (brain.metal:85-98), the weight stores of the
// ones below it (brain.metal:122; nothing was stored speculatively for them)
// and their spikes.  LDS only: no load waits behind the wave's stores.
__device__ __forceinline__ void lds_walk(const DeviceState& d, const KernelParams& kp, ApplyCtx& ac, uint64_t region,
                                         const uint4* e, uint32_t S, uint64_t P, bool set_next, uint64_t* setc)
{
    const uint32_t lane = threadIdx.x & 63, budget = kp.max_spikes;
    for (uint32_t q0 = 0; q0 < S && P < budget; q0 += 64) {  // wave-uniform
        const uint32_t q = q0 + lane;
        const bool v = q < S;
        const uint4 x = v ? e[q] : make_uint4(0u, 0u, 0u, 0u);
        const bool cand = v && (x.x >> 31);
        const uint64_t bc = __ballot(cand);
        const uint64_t pre = P + mbcnt64(bc);
        if (v && pre < budget) apply_event(d, kp, ac, region, make_uint4(x.x & 0x7FFFFFFFu, x.y, x.z, x.w), cand, pre, 0);
        if (set_next) wave_set_next_dedup(d, cand && pre < budget, x.w, setc);  // this pass's spikes
        P += (uint64_t)__popcll(bc);
    }
}

// Sharded pass, first launch: the dst of this range's spike candidates whose
// LOCAL budget position P + i is below the budget, in that order, into the
// exchange record's spike list (the lower ranks' offset is added by every
// rank when it stamps: stamp_gathered).  From cand_list when the range listed
// all its candidates, else by a walk of its survivors.
__device__ __forceinline__ void range_spikes_local(const DeviceState& d, const KernelParams& kp, uint32_t r,
                                                   uint64_t region, uint32_t S, uint32_t C, uint64_t P, int32_t* spikes)
{
    constexpr uint32_t RW = 4;
    const uint32_t lane = threadIdx.x & 63, budget = kp.max_spikes;
    if (P >= budget || C == 0) return;
    if (C <= kCandCap) {
        const uint32_t k = (uint32_t)(budget - P), nb = C < k ? C : k;
        const uint2* cl = d.cand_list + (uint64_t)r * kCandCap;
        for (uint32_t i = lane; i < nb; i += 64) spikes[P + i] = (int32_t)cl[i].y;
        return;
    }
    for (uint32_t b0 = 0; b0 < S && P < budget; b0 += RW * 64) {  // wave-uniform
        uint4 e[RW];
#pragma unroll
        for (uint32_t j = 0; j < RW; ++j) {
            const uint32_t q = b0 + j * 64 + lane;
            e[j] = q < S ? d.g2x[region + q] : make_uint4(0u, 0u, 0u, 0u);
        }
#pragma unroll
        for (uint32_t j = 0; j < RW; ++j) {
            const bool cand = b0 + j * 64 + lane < S && (e[j].x >> 31);
            const uint64_t bc = __ballot(cand);
            const uint64_t pre = P + mbcnt64(bc);
            if (cand && pre < budget) spikes[pre] = (int32_t)e[j].w;
            P += (uint64_t)__popcll(bc);
        }
    }
}

// The next pass's speculative workgroups (refrac_chunk's spec) from the
// workgroup `cut` where this pass's budget ran out: the ones below it, moved
// by spec_margin (default -1: the cut's own workgroup and one below it walk).
__device__ __forceinline__ uint32_t spec_prediction(const DeviceState& d, uint32_t cut, uint32_t G)
{
    if (cut >= G) return G;
    const int64_t v = (int64_t)cut + d.spec_margin;
    return v < 0 ? 0u : (v > (int64_t)G ? G : (uint32_t)v);
}

// The bitmap and filter images of the pass after next (the next pass builds
// them: k_apply, the fused pass, or k_bitmap) zeroed, a slice per workgroup;
// this pass's stimulus stamped by workgroup 0 (every refractory stage of the
// pass reads a stimulus neuron's lastFired as now without loading it).
__device__ __forceinline__ void zero_next_images(const DeviceState& d, uint32_t FW, uint32_t BLOCK, uint64_t now)
{
    const uint32_t tid = threadIdx.x;
    const uint32_t nz = d.n_bitmap_words + 2 * FW + kF2Words, per = (nz + gridDim.x - 1) / gridDim.x;
    for (uint32_t i = blockIdx.x * per + tid; i < min(nz, (blockIdx.x + 1) * per); i += BLOCK) {
        if (i < d.n_bitmap_words) d.bitmap_clear[i] = 0u;
        else d.filter_clear[i - d.n_bitmap_words] = 0u;
    }
    if (blockIdx.x == 0)
        for (uint64_t i = tid; i < d.stim_count; i += BLOCK) d.last_fired[d.stim_first + i] = now;
}

// s_waitcnt vmcnt(N) lgkmcnt(0) for the counts of record loads the gate's
// prologue leaves in flight.  The builtin, not inline asm: the compiler's
// wait-count tracking then knows the older LDS-DMAs are done (after an asm
// wait it would still count them pending and drain vmcnt(0) before the
// stream loop's first LDS read, every iteration).  gfx9 encoding: vmcnt
// [3:0] and [15:14], expcnt [6:4] (7: no wait), lgkmcnt [11:8].
template <int N>
__device__ __forceinline__ void wait_vm_lgkm0()
{
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
    asm volatile("" ::: "memory");
}

// LDS of the fused pass's end (per workgroup).
template <int NW>
struct FusedLds {
    uint64_t setc[kSetCache];          // wave_set_next_dedup's cache
    alignas(16) uint32_t cc[kFusedMaxRanges + 4];  // fused_next_bounds: the previous pass's range costs
                                                   // (LDS-DMA in the prologue), scanned in place
    uint32_t cand[NW];                 // spike candidates of each wave's range (capped at the budget)
    uint32_t stat[5];                  // pre-gated, survivors, updated, fired, pruned
    uint32_t excl;                     // candidates of all lower workgroups (capped)
    uint32_t done;                     // waves through their refractory stage
    uint32_t total;                    // candidates of the pass (capped; workgroup 0)
    uint32_t sg2;                      // sharded pass: the workgroup's refractory survivors
};

// Fused pass: range r's wave after its refractory stage (g1 pre-gated; Sg
// survivors contiguous from g2x[region] with Cg spike candidates among them,
// then -- when the tail kept them in LDS, tl -- St more at tl with Ct
// candidates; its stream took `stream_cost` 40-ns units, the next pass's
// partition cost): the next partition (first wave of the workgroup), its share
// of the next bitmap build, the workgroup look-back, the walk of its own
// survivors, statistics, the stamps of the workgroup's spikes once every
// refractory stage of the pass is done, and (workgroup 0) the pass's end.
// Pass-start scalars (C1) as read at kernel entry.
//
// gfx9's vmcnt counts loads and stores in issue order, so a load waits for
// every store the wave issued before it.  The path from the last refractory
// stage to the pass's end therefore issues no load behind a store where it
// can: the look-back's first sweep is issued before the publishing store, the
// tail's survivors and the workgroup's spikes stay in LDS, LDS-only barriers,
// and wave 0 sees every word published before it walks (and stores).
template <int BLOCK, int NW, bool kLean, bool kShard>
__device__ __forceinline__ void fused_end(const DeviceState& d, const KernelParams& kp, uint32_t r, uint64_t region,
                                          uint32_t g1, uint32_t Sg, uint32_t Cg, uint32_t St, uint32_t Ct,
                                          const uint4* tl, uint32_t stream_cost, bool empty, bool spec, uint64_t now,
                                          float R, float rb, uint64_t pass, uint32_t epoch, FusedLds<NW>& L,
                                          uint64_t t_stream, uint32_t h0, uint32_t chunk_t, uint32_t nch,
                                          uint64_t* wcb)
{
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, budget = kp.max_spikes;
    const uint32_t tag = epoch + 1u;
    // kLean: the single-GPU pass without plasticity (less code: the end of
    // the pass runs from a cold instruction cache)
    // kShard (with kLean): the sharded pass's first launch without plasticity
    const bool shard = kShard || (!kLean && d.shard_mode);
    const uint64_t t_tail = __builtin_amdgcn_s_memrealtime();
    const uint32_t S = Sg + St, C = Cg + Ct;  // the range's survivors and spike candidates
    uint32_t order = 0;
    if (lane == 0) {
        L.cand[wid] = C < budget ? C : budget;
        if (shard) atomicAdd(&L.sg2, S);
        order = atomicAdd(&L.done, 1u);
    }
    if (wave_uniform(order) == 0) fused_next_bounds<NW>(d, L.cc);
    lds_barrier();  // every range of the workgroup through its refractory stage
    uint32_t vals[kLbMaxWords];
    // The next pass's bitmap build items that do not depend on this pass (the
    // spike lists of passes p+1-W..p-1, the stimulus): item x to workgroup
    // h0 + x % (G - h0), by waves [w0, NW) of it.  With h0 > 0 only the
    // workgroups past the predicted budget cut take them (they have no walk),
    // with h0 = 0 every workgroup.
    auto next_share = [&](uint32_t w0) {
        const uint64_t nitems = next_items(d, kp), HG = gridDim.x - h0, hb = blockIdx.x - h0;
        for (uint64_t s0 = (uint64_t)(wid - w0) * 64; s0 * HG + hb < nitems; s0 += (uint64_t)(NW - w0) * 64) {
            const uint64_t x = (s0 + lane) * HG + hb;  // wave-uniform trip count (lane 0's item)
            const NextItem it = x < nitems ? next_item_load(d, kp, pass, x) : NextItem{0u, 0u, 0u};
            wave_set_next_dedup(d, it.i < it.lim, it.n, L.setc);
        }
    };
    // (waves 1.. take them while wave 0 publishes and polls: the workgroups
    // past the predicted cut have no walk after it, so the items would
    // otherwise come after their look-back, on the pass's critical path)
    if (wid != 0 && d.build_next && (h0 == 0 || blockIdx.x >= h0)) next_share(1);
    if (wid == 0) {
        uint32_t c = lane < (uint32_t)NW ? L.cand[lane] : 0u;
        c = wave_sum(c);
        const uint64_t word = (uint64_t)tag << 32 | (uint64_t)kLbAggregate << 30 | (c < budget ? c : budget);
        uint32_t e;
        if (shard) {
            // the pass's refractory survivors for the exchange summary: added
            // before this workgroup's word is published (workgroup 0 sums
            // them once every word is)
            if (lane == 0) {
                __hip_atomic_fetch_add(&d.work->shard_g2, (unsigned long long)L.sg2, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store((gu64*)(d.lb_status + blockIdx.x), word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            e = wg_poll(d, blockIdx.x, tag, budget, true, vals);
        } else {
            e = wg_poll(d, blockIdx.x, tag, budget, true, vals, word);
        }
        if (lane == 0) L.excl = e;
    }
    lds_barrier();
    const uint32_t excl_wg = L.excl;
    uint64_t P = excl_wg;
    uint64_t c_wg = 0;  // the workgroup's candidates
    for (uint32_t w = 0; w < (uint32_t)NW; ++w) {
        if (w < wid) P += L.cand[w];
        c_wg += L.cand[w];
    }
    const uint64_t t_lb = __builtin_amdgcn_s_memrealtime();
    // the workgroup's spikes: budget positions [s0, s1) of the spike list
    const uint32_t s0 = excl_wg, s1 = (uint32_t)(excl_wg + c_wg < budget ? excl_wg + c_wg : budget);
    const bool first = blockIdx.x == 0;
    const bool stamping = !shard && (s1 > s0 || first);
    // the spikes go to LDS too (L.cc: the partition's cost prefix is done)
    // unless the budget is larger than it
    const bool spk_lds = !shard && budget <= kFusedMaxRanges;
    // every workgroup's word published = every refractory stage of the pass
    // done: no lastFired read is left, the stamps may land.  Wave 0 waits for
    // that before its walk (its loads then wait for no store of the walk).
    uint32_t tot = 0, t0 = 0;
    if (wid == 0 && stamping) {
        tot = wg_poll(d, gridDim.x, tag, budget, false, vals);
        if (first) {
            // the next pass's prediction (refrac_chunk's spec): the workgroups
            // below the one where the budget ran out, less one
            uint32_t run = 0, cut = gridDim.x;
#pragma unroll
            for (uint32_t i = 0; i < kLbMaxWords; ++i) {
                const uint32_t inc = wave_incl_scan(vals[i]) + run;  // prefix through word 64 i + lane
                const uint64_t hit = __ballot(inc >= budget && inc - vals[i] < budget);
                if (hit && cut == gridDim.x) cut = i * 64 + (uint32_t)__builtin_ctzll(hit);
                run = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            }
            // the event-0 flag (refrac_chunk): stored and drained before its
            // workgroup's word was published
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            t0 = __hip_atomic_load((gu32*)&d.work->t0_g2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("" ::"v"(t0));  // consumed here, before any store of the walk (see range_walk)
            if (lane == 0) d.work->spec_wgs = spec_prediction(d, cut, gridDim.x);
        }
    }
    const uint64_t t_seen = __builtin_amdgcn_s_memrealtime();
    // the budget walk of k_apply over this range alone, in event order
    ApplyCtx ac{R, rb, now, pass, false, false, true, false, !kLean && kp.w_prune > 0.0f,
                !kLean && d.grown != nullptr && kp.p_new > 0.0f, true, 0u, 0u, 0u};
    if (spk_lds) {
        ac.lds_spk = L.cc;
        ac.lds_s0 = s0;
    }
    uint32_t upd_rest = 0;
    uint64_t t_rw = 0;
    if (!shard) {
        upd_rest = range_walk(d, kp, ac, r, region, Sg, Cg, P, spec, d.build_next != 0, L.setc);
        t_rw = __builtin_amdgcn_s_memrealtime();
        if (tl) lds_walk(d, kp, ac, region, tl, St, P + Cg, d.build_next != 0, L.setc);
    } else {
        // sharded pass (the first of its two launches): the global budget
        // offset is unknown until the exchange, so this range's local budget
        // position, survivors and candidates go to range_info for
        // k_shard_walk, and its candidates below the budget (local order)
        // into the exchange record's spike list (abnn.h)
        if (lane == 0)
            d.range_info[r] = make_uint4((uint32_t)(P < budget ? P : budget), S, C, (spec ? 1u : 0u) | (empty ? 2u : 0u));
        range_spikes_local(d, kp, r, region, S, C, P, d.xchg + 2 * ABNN_SUMMARY_WORDS);
    }
    const uint64_t t_walk = __builtin_amdgcn_s_memrealtime();
    const uint32_t wu = wave_sum(ac.upd) + upd_rest, wf = wave_sum(ac.nf), wp = wave_sum(ac.npr);
    if (lane == 0) {
        atomicAdd(&L.stat[0], g1);
        atomicAdd(&L.stat[1], S);
        atomicAdd(&L.stat[2], wu);
        atomicAdd(&L.stat[3], wf);
        atomicAdd(&L.stat[4], wp);
        d.cost_out[r] = empty ? 0u : (stream_cost < 1 ? 1u : (stream_cost > 0xFFFFu ? 0xFFFFu : stream_cost));
    }
    if (lane == 0 && d.wave_clock_on) {
        uint64_t* wc = wcb + (uint64_t)kWaveClock * r;  // diagnostics (tools/wave_clock.py)
        wc[1] = t_stream;  // wc[0], wc[3]: stored by k_gate at the stream's start
        wc[2] = t_tail;
        wc[4] = t_lb;
        wc[5] = t_walk;
        wc[6] = chunk_t;
        wc[7] = nch;
        wc[8] = S;
        wc[9] = C;
        wc[10] = excl_wg;
        wc[11] = wu;
        if (wid == 0) wc[12] = stamping ? t_seen : 0;
        wc[14] = t_rw;  // range_walk done (then the LDS tail's walk, the helpers' items: t_walk)
    }
    // LDS only (the statistics, the LDS spike list): the walks' stores stay in flight
    if (shard || (stamping && !spk_lds)) __syncthreads();
    else lds_barrier();
    if (threadIdx.x == 0) {
        typedef unsigned long long ull;
        abnn_stats* st = d.wg_stats + blockIdx.x % kWalkBlocks;
        atomicAdd((ull*)&st->pre_gated, (ull)L.stat[0]);
        atomicAdd((ull*)&st->post_gated, (ull)L.stat[1]);
        if (L.stat[2]) atomicAdd((ull*)&st->updated, (ull)L.stat[2]);
        if (L.stat[3]) atomicAdd((ull*)&st->fired, (ull)L.stat[3]);
        if (L.stat[4]) atomicAdd((ull*)&st->pruned, (ull)L.stat[4]);
        if (first) {
            atomicAdd((ull*)&st->passes, 1ull);
            atomicAdd((ull*)&st->events, (ull)d.events);
        }
    }
    if (shard) {
        // sharded pass: no stamps, no pass end here (k_shard_walk, after the
        // exchange); workgroup 0 writes the exchange summary (abnn.h) once
        // every word is published
        zero_next_images(d, kCodeFilterWords, BLOCK, now);
        if (!first || wid != 0) return;
        const uint32_t tt = wg_poll(d, gridDim.x, tag, budget, false, vals);
        if (lane == 0) {
            int64_t* sm = reinterpret_cast<int64_t*>(d.xchg);
            sm[0] = (int64_t)tt;  // candidates, capped at the budget
            sm[1] = (int64_t)__hip_atomic_load((gu32*)&d.work->t0_g2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sm[2] = (int64_t)d.events;
            sm[3] = (int64_t)__hip_atomic_load(&d.work->shard_g2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            d.work->shard_g2 = 0;
            d.work->epoch = epoch + 1u;
            d.work->ps_now = now;  // the pass-start scalars for k_shard_walk (C1)
            d.work->ps_pass = pass;
            d.work->ps_R = R;
            d.work->ps_rb = rb;
        }
        return;
    }
    uint64_t* wc0 = wcb + (uint64_t)kWaveClock * r;  // diagnostics, wave 0: exit
    if (stamping) {
        if (spk_lds) {
            for (uint32_t i = s0 + threadIdx.x; i < s1; i += BLOCK) {
                const uint32_t nrn = L.cc[i - s0];
                if (nrn < d.n_nrn) d.last_fired[nrn] = now;  // brain.metal:125-126
            }
        } else {
            const uint32_t* ring = d.fired_ring + (pass & (kFiredRing - 1)) * (uint64_t)budget;
            for (uint32_t i = s0 + threadIdx.x; i < s1; i += BLOCK) {
                const uint32_t nrn = ring[i];
                if (nrn < d.n_nrn) d.last_fired[nrn] = now;  // brain.metal:125-126
            }
        }
    }
    if (first && threadIdx.x == 0) {  // the pass's end: every workgroup has read the pass-start scalars
        d.n_fired_ring[pass & (kFiredRing - 1)] = tot;
        if (t0 != 0u && budget > 0) *d.rbar = rb + kp.alpha_rbar * (R - rb);  // brain.metal:110-113
        *d.clock = now + kp.clock_inc;                                        // brain.metal:129
        *d.pass_index = pass + 1;
        __hip_atomic_store((gu32*)&d.work->t0_g2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        d.work->epoch = epoch + 1u;
    }
    // last: no load of this pass follows these stores
    zero_next_images(d, kCodeFilterWords, BLOCK, now);
    if (threadIdx.x == 0 && d.wave_clock_on) wc0[13] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------------------
// k_gate: the streaming kernel (see file header).  Every wave owns one
// contiguous range of events.  The pre-spike gate needs only the src of each
// record, held as a 3-B filter code in two streams (engine.h, SynArrays): per
// 512-event block a lane loads its 8 consecutive events' lo words (16 B) and
// hi bytes (8 B) from wave-uniform bases, non-temporal, kDepth iterations in
// flight, and tests each against ONE 8-B block of the LDS filter
// (quad_filter: 4 VALU per event, no global load).  The arrays are padded by
// kDummyRecords, so the sweep's last iteration reads past its end instead of
// masking lanes, and the prefetch after a range's last iteration reads the
// zero dummy block.  Events that pass the filter (under 1 % at config 3 in
// steady state; the exact bitmap decides) are staged in LDS as {offset,
// code} in event order (lane order is event order within a block); every
// chunk of them goes through the refractory stage in the wave itself (a full
// one at once, the last one -- the range's tail -- after the stream).
// Instruction-issue priority (s_setprio takes an immediate).
__device__ __forceinline__ void set_priority(uint32_t p)
{
    switch (p & 3u) {
        case 0: __builtin_amdgcn_s_setprio(0); break;
        case 1: __builtin_amdgcn_s_setprio(1); break;
        case 2: __builtin_amdgcn_s_setprio(2); break;
        default: __builtin_amdgcn_s_setprio(3); break;
    }
}

// kFused (sweep mode, blocked range map): the whole single-GPU pass in this
// launch -- after its refractory stage every wave joins its workgroup's
// look-back (wg_lookback above), walks its own survivors up to the budget (the
// weight update of k_apply: apply_event), and the last workgroup ends the pass
// (fused_finalize).  Its survivors are written contiguously from the range's
// region start (no per-chunk slots: the wave walks them itself).
template <int BLOCK, int K, int FW, bool kTrack, bool kRandom, bool kFused, bool kLean = false, bool kShard = false>
__global__ __launch_bounds__(BLOCK) void k_gate(DeviceState d, KernelParams kp)
{
    constexpr int NW = BLOCK / 64;
    constexpr uint32_t IE = 64 * K;
    constexpr int KD = kTrack ? K : 1;                 // dst words in flight (track_visits)
    constexpr int NB8 = K / 8;                         // sweep: 512-event blocks per iteration
    constexpr uint32_t LG = __builtin_ctz(FW);
    constexpr uint32_t SE = kChunk + 128;              // a chunk + one staging step (<= 128 events)
    static_assert(K % 8 == 0, "the packed src stream is read in 512-event blocks (8 events per lane)");
    static_assert(kRandom || FW == kCodeFilterWords, "the sweep tests the stored code (engine.h, src_code)");
    static_assert(IE <= (uint32_t)kDummyRecords, "dummy block / padding must cover one iteration");
    static_assert(!(kFused && kRandom), "the fused pass is sweep-mode only");
    __shared__ uint2 s_fb[FW];  // the filter's FW 64-bit blocks
    __shared__ uint32_t s_f2[kF2Words];  // the second-level filter (refrac_chunk)
    // a wave's stage: SE offsets, then SE codes (one 8-SE-byte block, so the
    // fused tail can reuse it for its survivors, refrac_chunk lds_out)
    __shared__ uint32_t s_stage[NW][2 * SE];
    __shared__ FusedLds<NW> s_fz;            // fused: the pass end's workgroup state

    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const uint32_t wid = wave_uniform(tid >> 6);
    const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();  // diagnostics: the prologue
    // The filter goes global -> LDS directly (LDS-DMA), first: loads return
    // in order, so behind the first records' HBM burst it would hold the
    // prologue.  One wave-instruction copies 1 KiB (LDS: wave-uniform base +
    // 16 B per lane); the first use of an ordinary load's result waits for it.
    static_assert((FW / 2) % BLOCK == 0, "the filter copy is FW / 2 / BLOCK uint4 per thread");
#pragma unroll
    for (int c = 0; c < FW / 2 / BLOCK; ++c)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(d.filter) + c * BLOCK + tid,
                                         reinterpret_cast<uint4*>(s_fb) + c * BLOCK + (tid & ~63u), 16, 0, 0);
    // the second-level filter, stored after the blocks (engine.h kF2Words)
    static_assert(kF2Words % 4 == 0 && kF2Words / 4 <= 2048, "second-level filter copy");
    for (uint32_t i0 = 0; i0 < kF2Words / 4; i0 += BLOCK)  // workgroup-uniform
        if (i0 + tid < kF2Words / 4)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(d.filter + 2 * FW) + i0 + tid,
                                             reinterpret_cast<uint4*>(s_f2) + i0 + (tid & ~63u), 16, 0, 0);
    // fused: the previous pass's range costs (the next partition's input,
    // fused_next_bounds) go to LDS the same way
    if constexpr (kFused) {
        if (d.prologue_adapt && d.adapt_ranges && d.n_ranges >= 2) {
            const uint32_t nq = (d.n_ranges + 3) / 4;  // cost_in holds a multiple of 16 ranges
            for (uint32_t i0 = 0; i0 < nq; i0 += BLOCK)  // workgroup-uniform
                if (i0 + tid < nq)
                    __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(d.cost_in) + i0 + tid,
                                                     reinterpret_cast<uint4*>(s_fz.cc) + i0 + (tid & ~63u), 16, 0, 0);
        }
    }
    // range of this wave: blocked (a workgroup's waves sweep neighbouring
    // ranges) or interleaved (neighbouring ranges on different CUs / XCDs, so
    // a dense stretch of the graph does not land on one CU)
    const uint32_t r = (!kFused && d.range_map) ? wid * gridDim.x + blockIdx.x : blockIdx.x * NW + wid;
    // (iteration counts < 2^31, checked at create; wave-uniform, held in SGPRs)
    const uint32_t it_begin = sload(d.range_bounds + r), it_end = sload(d.range_bounds + r + 1);
    const uint64_t region = (uint64_t)it_begin * IE;
    const uint64_t now = sload(d.clock);  // per-TG clock cache, brain.metal:63-68 (C1: pass start)
    // fused: the pass-start reward and rBar (brain.metal:105-106; C1) for the
    // updated weights of the refractory stage
    // (pass-start scalars are moved to SGPRs: held through the stream in
    // VGPRs they would spill)
    const float Rw = kFused ? sload(d.reward) : 0.0f;
    const float rbw = kFused ? sload(d.rbar) : 0.0f;
    // fused: the pass index and epoch (workgroup 0 advances both at the end,
    // once every workgroup has read them), and whether this workgroup is
    // predicted below the budget cut (the previous pass's cut, less one); never
    // with pruning (a pruned record's src and dst change, which a restore would
    // have to undo too)
    const uint64_t pass_f = kFused ? sload(d.pass_index) : 0;
    const uint32_t epoch = kFused ? sload(&d.work->epoch) : 0u;
    const uint32_t spec_wgs = kFused ? sload(&d.work->spec_wgs) : 0u;
    const bool spec = kFused && !(kp.w_prune > 0.0f) && (d.spec_mode == 2 || (d.spec_mode == 1 && blockIdx.x < spec_wgs));
    // fused: the first workgroup past the predicted cut (spec_wgs = cut - 1)
    // and a margin -- the ones from it on take the next bitmap's
    // pass-independent items (fused_end); 0: every workgroup does
    uint32_t hw0 = 0;
    if (kFused && !d.shard_mode && spec_wgs + 3u + gridDim.x / 4u <= gridDim.x) hw0 = spec_wgs + 3u;
    uint32_t* st_off = s_stage[wid];
    uint32_t* st_src = s_stage[wid] + SE;
    // Records in flight.  Sweep (layout 4, engine.h SynArrays): lane-
    // contiguous -- per 512-event block b of an iteration, lane L holds events
    // 512 b + 8 L .. 8 L + 7: their eight lo words in one 16-B load and their
    // eight hi bytes in one 8-B load, 3 B per event, both in natural record
    // order (a wave-instruction reads 1 KiB / 512 B contiguous).  Random mode:
    // per event k (t = 64 k + lane) the u32 src of its picked record (the
    // src32 mirror).
    // kDepth iterations of records in flight per wave (sweep: two, ping-pong
    // buffers A/B; a wave's memory-level parallelism bounds its stream rate)
#ifndef ABNN_DEPTH
#define ABNN_DEPTH 2
#endif
    constexpr int kDepth = (kRandom || kTrack) ? 1 : ABNN_DEPTH;
    struct RecsSweep {
        u32x4 lo[NB8];
        u32x2 hi[NB8];
        uint32_t dd[KD];
    };
    struct RecsRandom {
        uint32_t s[K];
        uint32_t dd[KD];
    };
    using Recs = std::conditional_t<kRandom, RecsRandom, RecsSweep>;
    Recs bufs[kDepth];
    const uint64_t pass = kRandom ? sload(d.pass_index) : 0;
    auto issue = [&](Recs& x, uint64_t it, bool live) __attribute__((always_inline)) {
        if constexpr (kRandom) {  // random-edge mode: a per-lane random record per event
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const uint64_t t = it * IE + k * 64 + lane;
                const bool real = live && t < d.events;
                const uint64_t e = real ? pick_record(d.seed, d.syn_offset, pass, t, d.n_syn) : 0;
                x.s[k] = __builtin_nontemporal_load(d.syn.src32 + e);  // one access per pick
                if constexpr (kTrack)
                    x.dd[k] = __builtin_nontemporal_load(real ? reinterpret_cast<const uint32_t*>(d.syn.dw + e)
                                                              : d.dummy + (k * 64 + lane));
            }
        } else {
            // wave-uniform bases; past the range the zero dummy block
            const u32x4* bl = live ? reinterpret_cast<const u32x4*>(d.syn.lo) + it * (IE / 8)
                                   : reinterpret_cast<const u32x4*>(d.dummy);
            const u32x2* bh = live ? reinterpret_cast<const u32x2*>(d.syn.hi) + it * (IE / 8)
                                   : reinterpret_cast<const u32x2*>(d.dummy);
#pragma unroll
            for (int b = 0; b < NB8; ++b) {
                x.lo[b] = __builtin_nontemporal_load(bl + b * 64 + lane);
                x.hi[b] = __builtin_nontemporal_load(bh + b * 64 + lane);
            }
            if constexpr (kTrack) {  // dst of the same events: 8 {dst, w} pairs per lane and block
                const u32x4* bd = reinterpret_cast<const u32x4*>(live ? reinterpret_cast<const uint32_t*>(d.syn.dw + (uint64_t)it * IE)
                                                                      : d.dummy);
#pragma unroll
                for (int b = 0; b < NB8; ++b)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const u32x4 v = __builtin_nontemporal_load(bd + b * 256 + lane * 4 + j);
                        x.dd[8 * b + 2 * j] = v.x;
                        x.dd[8 * b + 2 * j + 1] = v.z;
                    }
            }
        }
    };
    __builtin_amdgcn_sched_barrier(0);  // the LDS-DMAs above stay older than the records (see the wait below)
#pragma unroll
    for (int j = 0; j < kDepth; ++j) issue(bufs[j], it_begin + j, it_begin + j < it_end);
    if constexpr (!kFused) {
        // the bitmap and images of the pass after next are zeroed here (the
        // next pass builds them: k_apply or k_bitmap), a slice per workgroup;
        // this pass's stimulus is stamped by workgroup 0 (the refractory stage
        // reads it as now).  The fused pass does both at its end (fused_end).
        zero_next_images(d, FW, BLOCK, now);
        lds_barrier();
    } else {
        if (tid < 5) s_fz.stat[tid] = 0u;
        if (tid == 0) s_fz.done = 0u;
        if (tid == 0) s_fz.sg2 = 0u;
        if (tid < kSetCache) s_fz.setc[tid] = ~0ull;
        // the filter images in LDS for every wave, the first records still in
        // flight: this wave's LDS-DMAs are older than its kDepth iterations of
        // record loads, and vmcnt retires in order.  (A release fence here
        // would wait for vmcnt(0): the records' whole round trip, and until
        // round 4 the prologue's zeroing stores too, before the stream began.)
        // (kTrack: the {dst, w} pairs of the same events too, one iteration deep)
        constexpr int kRecLoads = kDepth * (kRandom ? K * (kTrack ? 2 : 1) : NB8 * (2 + (kTrack ? 4 : 0)));
        __builtin_amdgcn_sched_barrier(0);
        wait_vm_lgkm0<kRecLoads>();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    }
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    // diagnostics (tools/wave_clock.py): the fused pass keeps the last
    // kWaveClockPasses passes' clocks (slot pass % kWaveClockPasses)
    uint64_t* wcb = d.wave_clock + (kFused ? (pass_f % kWaveClockPasses) * (uint64_t)kWaveClock * kMaxRanges : 0);
    if (lane == 0 && d.wave_clock_on) {  // stored now, not held through the stream
        wcb[kWaveClock * r] = t_start;
        wcb[kWaveClock * r + 3] = t_entry;
    }
    const uint64_t len = it_end - it_begin;

    const uint32_t nn = (uint32_t)d.n_nrn;  // N_NRN < 2^32 (checked at create)
    uint32_t pend = 0, nch = 0;
    uint4 tot = make_uint4(0u, 0u, 0u, 0u);
    auto stage_at = [&](uint32_t q) { return make_uint2(st_off[q], st_src[q]); };
    // wave-uniform: a full chunk through the refractory stage now; the (< 128)
    // entries past it move to the front of the stage
    // survivors go to chunk c's slots (the walk of k_apply takes chunks as
    // work items), or, fused, right after the range's earlier survivors
    uint32_t chunk_t = 0;  // diagnostics: 10-ns units spent in mid-stream refractory chunks
    auto chunk_out = [&]() {
        const uint64_t tc = __builtin_amdgcn_s_memrealtime();
        const uint64_t at = kFused ? region + tot.y : region + (uint64_t)nch * kChunk;
        const uint4 c = refrac_chunk<kChunk / 64, kRandom, kFused, false>(d, kp, region, at, kChunk, now, pass, Rw, rbw,
                                                                   spec, r, tot.z, s_f2, stage_at);
        if (!kFused && lane == 0) d.chunk_cnt[chunk_slot(region, nch)] = c;
        tot.x += c.x;
        tot.y += c.y;
        tot.z += c.z;
        const uint32_t rest = pend - kChunk;
#pragma unroll
        for (uint32_t h = 0; h < 128; h += 64) {
            const uint32_t q = h + lane;
            const uint32_t xo = q < rest ? st_off[kChunk + q] : 0u, xs = q < rest ? st_src[kChunk + q] : 0u;
            if (q < rest) {
                st_off[q] = xo;
                st_src[q] = xs;
            }
        }
        ++nch;
        pend = rest;
        chunk_t += (uint32_t)(__builtin_amdgcn_s_memrealtime() - tc);
    };
    // fused: every staged event through the refractory stage once flush_at
    // are staged (survivors go right after the range's earlier ones)
    auto flush_all = [&]() {
        const uint64_t tc = __builtin_amdgcn_s_memrealtime();
        const uint4 c = refrac_chunk<kChunk / 64, kRandom, kFused, false>(d, kp, region, region + tot.y, pend, now, pass, Rw,
                                                                   rbw, spec, r, tot.z, s_f2, stage_at);
        tot.x += c.x;
        tot.y += c.y;
        tot.z += c.z;
        nch += pend >= kChunk;
        pend = 0;
        chunk_t += (uint32_t)(__builtin_amdgcn_s_memrealtime() - tc);
    };
    auto step = [&](Recs& x, uint32_t it) __attribute__((always_inline)) {
        // The SIMD arbiter issues strictly by priority, then age: with a fixed
        // order the last of a SIMD's four waves streams ~15 % slower than the
        // first.  Rotating every wave through the four ranks every four
        // iterations equalises them (tools/ubench_soa.hip, profiles/r01p_*).
        if (((it - it_begin) & 3u) == 0) set_priority((uint32_t)((it - it_begin) >> 2) + wid / 4u);
        uint32_t dst[KD];
#pragma unroll
        for (int k = 0; k < KD; ++k) dst[k] = kTrack ? x.dd[k] : 0u;
        const uint64_t base = (uint64_t)it * IE;
        const uint32_t rel = (uint32_t)(base - region);
        const bool last = base + IE > d.events;  // only the sweep's last iteration (wave-uniform)
        if constexpr (kRandom) {
            // event k of this lane: idx = 64 k + lane (event order = (k, lane))
            uint32_t src[K];
#pragma unroll
            for (int k = 0; k < K; ++k) src[k] = x.s[k];
            issue(x, it + kDepth, it + kDepth < it_end);  // the buffer's next iteration in flight first
            uint32_t vmask = (K == 32) ? 0xFFFFFFFFu : ((1u << K) - 1u);  // events of this lane that exist
            if (last) {
                vmask = 0;
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (base + (uint32_t)(k * 64) + lane < d.events) vmask |= 1u << k;
            }
            // Pre-spike filter (brain.metal:73-77 pre-selection): every
            // event's block read back to back; the block index is masked, so
            // any src (tombstones included) stays in bounds; ubfe takes the
            // bit offset mod 32: low bit src mod 32, high bit (src + t) mod 32
            uint2 fb[K];
            uint32_t ft[K];
#pragma unroll
            for (int k = 0; k < K; ++k) {
                ft[k] = filter_t(src[k] >> 5, LG);
                fb[k] = s_fb[((src[k] >> 5) ^ ft[k]) & (FW - 1)];
            }
            uint32_t fm = 0;
#pragma unroll
            for (int k = 0; k < K; ++k)
                fm |= (__builtin_amdgcn_ubfe(fb[k].x, src[k], 1) & __builtin_amdgcn_ubfe(fb[k].y, src[k] + ft[k], 1)) << k;
            fm &= vmask;
            if constexpr (kTrack) {  // README §4: lastVisited[dst] = now (never read by a decision)
#pragma unroll
                for (int k = 0; k < K; ++k)
                    if (((vmask >> k) & 1u) && dst[k] < nn) d.last_visited[dst[k]] = now;
                // a shard handle also marks the neuron visited since the last
                // lastVisited merge (k_visits_delta)
                if (d.visit_mark) {
#pragma unroll
                    for (int k = 0; k < K; ++k)
                        if (((vmask >> k) & 1u) && dst[k] < nn) d.visit_mark[dst[k]] = 1u;
                }
            }
            if (__ballot(fm != 0) == 0) return;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const bool h = (fm >> k) & 1u;
                const uint64_t b1 = __ballot(h);
                if (h) {
                    const uint32_t q = pend + mbcnt64(b1);
                    st_off[q] = rel + (uint32_t)(k * 64) + lane;
                    st_src[q] = src[k];
                }
                pend += (uint32_t)__popcll(b1);
                if (pend >= kChunk) chunk_out();  // a k-step stages at most 64
            }
        } else {
            // this iteration's words (the buffer is refilled right away)
            u32x4 lo[NB8];
            u32x2 hi[NB8];
#pragma unroll
            for (int b = 0; b < NB8; ++b) {
                lo[b] = x.lo[b];
                hi[b] = x.hi[b];
            }
            issue(x, it + kDepth, it + kDepth < it_end);  // the buffer's next iteration in flight first
            // Pre-spike filter (brain.metal:73-77 pre-selection) on the stored
            // codes (engine.h, src_code), every block read issued before the
            // first test (the reads are independent; SQ_LDS_BANK_CONFLICT is
            // half of SQ_LDS_IDX_ACTIVE, so they queue): 4 VALU per event
            // (quad_filter), no v_perm to assemble the codes
            uint2 fb[K];
#pragma unroll
            for (int b = 0; b < NB8; ++b) {
                const uint32_t w[4] = {lo[b].x, lo[b].y, lo[b].z, lo[b].w};
#pragma unroll
                for (int k = 0; k < 8; ++k) fb[8 * b + k] = filter_block_at(s_fb, code_addr(w[k >> 1], k & 1));
            }
            uint32_t H[2 * NB8];  // bit 0 of byte m of H[2 b + q]: event 8 L + 4 q + m of block b passed
#pragma unroll
            for (int b = 0; b < NB8; ++b) {
                H[2 * b] = quad_filter(fb + 8 * b, lo[b].x, lo[b].y, hi[b].x);
                H[2 * b + 1] = quad_filter(fb + 8 * b + 4, lo[b].z, lo[b].w, hi[b].y);
            }
            if (last) {  // events past the sweep pass nothing
#pragma unroll
                for (int b = 0; b < NB8; ++b) {
                    const uint64_t e0 = base + 512u * b + 8u * lane;
                    const uint32_t nv = e0 >= d.events ? 0u : (uint32_t)std::min<uint64_t>(8u, d.events - e0);
                    H[2 * b] &= nv >= 4 ? 0xFFFFFFFFu : (1u << (8 * nv)) - 1u;
                    H[2 * b + 1] &= nv >= 8 ? 0xFFFFFFFFu : nv <= 4 ? 0u : (1u << (8 * (nv - 4))) - 1u;
                }
            }
            if constexpr (kTrack) {  // README §4: lastVisited[dst] = now (never read by a decision)
#pragma unroll
                for (int b = 0; b < NB8; ++b) {
                    const uint64_t e0 = base + 512u * b + 8u * lane;
                    const uint32_t nv = !last ? 8u : e0 >= d.events ? 0u : (uint32_t)std::min<uint64_t>(8u, d.events - e0);
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        if ((uint32_t)k < nv && dst[8 * b + k] < nn) d.last_visited[dst[8 * b + k]] = now;
                    // a shard handle also marks the neuron visited since the
                    // last lastVisited merge (k_visits_delta)
                    if (d.visit_mark) {
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            if ((uint32_t)k < nv && dst[8 * b + k] < nn) d.visit_mark[dst[8 * b + k]] = 1u;
                    }
                }
            }
            // Staging in event order.  Event order within a block is (lane,
            // k), so a lane's hits go to consecutive slots from the exclusive
            // prefix of the per-lane hit counts, in k order: round j writes
            // every lane's j-th hit (ffbl of the first quad's hits, then the
            // second's, each cleared when taken).  In the steady state
            // (~0.7 % of events pass) no lane holds two hits: one mbcnt is the
            // prefix and one round places them all; else (a lane with 2+
            // hits: ~8 % of blocks, and the dense input->output stretch) four
            // bit-plane ballots give the prefix and the rounds repeat.  A
            // block that would overflow the stage (dense) goes in 128-event
            // quarters (16 lanes each), the stage flushed between them.
            // (Runtime loops, not unrolled: the compiler hoisted an unrolled
            // slow path's per-event work in front of the common case.)
#pragma unroll
            for (int b = 0; b < NB8; ++b) {
                // event 4 q + m: bit 8 m of H[2 b + q]
                const uint64_t bb = __ballot((H[2 * b] | H[2 * b + 1]) != 0);
                if (bb == 0) continue;  // wave-uniform
                const uint32_t relb = rel + 512u * b + 8u * lane;  // this lane's first event of the block
                const uint32_t cb = __builtin_popcount(H[2 * b]) + __builtin_popcount(H[2 * b + 1]);
                uint32_t P, tot;  // exclusive prefix of the counts, their total
                if (__ballot(cb > 1u) == 0) {
                    P = mbcnt64(bb);
                    tot = (uint32_t)__popcll(bb);
                } else {
                    P = 0;
                    tot = 0;
#pragma unroll
                    for (int i = 0; i < 4; ++i) {  // counts <= 8: four bit planes
                        const uint64_t bi = __ballot((cb >> i) & 1u);
                        P += mbcnt64(bi) << i;
                        tot += (uint32_t)__popcll(bi) << i;
                    }
                }
                const bool split = pend + tot > SE;  // wave-uniform (dense)
                const uint32_t w0 = lo[b].x, w1 = lo[b].y, w2 = lo[b].z, w3 = lo[b].w, v0 = hi[b].x, v1 = hi[b].y;
#pragma unroll 1
                for (uint32_t u = 0; u < (split ? 4u : 1u); ++u) {  // wave-uniform
                    const uint32_t p0 = split ? (uint32_t)__builtin_amdgcn_readlane((int)P, (int)(16u * u)) : 0u;
                    const uint32_t p1 = !split || u == 3 ? tot
                                                         : (uint32_t)__builtin_amdgcn_readlane((int)P, (int)(16u * u + 16u));
                    const bool mine = !split || (lane >> 4) == u;
                    uint32_t x0 = mine ? H[2 * b] : 0u, x1 = mine ? H[2 * b + 1] : 0u;
                    uint32_t q = pend + P - p0;
                    do {  // one round: every lane's next hit (wave-uniform trip count)
                        if ((x0 | x1) != 0u) {
                            const bool hs = x0 == 0u;  // the block's second quad (events 4..7)
                            const uint32_t xx = hs ? x1 : x0, m = (uint32_t)__builtin_ctz(xx) >> 3;
                            const uint32_t xn = xx & (xx - 1u);
                            x0 = hs ? x0 : xn;
                            x1 = hs ? xn : x1;
                            const uint32_t e0 = hs ? w2 : w0, e1 = hs ? w3 : w1;
                            const uint32_t lo16 = __builtin_amdgcn_perm(e1, e0, 0x0C0C0100u + m * 0x0202u);
                            st_off[q] = relb + (hs ? 4u : 0u) + m;
                            st_src[q] = __builtin_amdgcn_perm(hs ? v1 : v0, lo16, 0x0C040100u + (m << 16));
                            ++q;
                        }
                    } while (__ballot((x0 | x1) != 0u) != 0);
                    pend += p1 - p0;
                    if (kFused ? pend >= d.flush_at : pend >= kChunk) {  // at most 128 past the threshold
                        if constexpr (kFused) flush_all();
                        else chunk_out();
                    }
                }
            }
        }
    };
    for (uint32_t it = it_begin; it < it_end; it += kDepth) {  // wave-uniform
#pragma unroll
        for (int j = 0; j < kDepth; ++j)
            if (j == 0 || it + j < it_end) step(bufs[j], it + j);
    }
    const uint64_t t_stream = __builtin_amdgcn_s_memrealtime();
    if (!kFused && lane == 0 && d.wave_clock_on) {  // diagnostics (tools/wave_clock.py; the fused pass stores them in fused_end)
        d.wave_clock[kWaveClock * r + 6] = chunk_t;
        d.wave_clock[kWaveClock * r + 7] = nch;
    }
    // the tail (a latency-bound chain of two gathers, few instructions) and
    // the pass's end run at the highest issue priority.  At the lowest (round
    // 3) a SIMD's tails lost every tie to its streams and then went by wave
    // age: the youngest waves' tails took 10-13 us against 6-8 for the oldest
    // (tools/wc_multi.py), and the partition, which balances stream + tail,
    // could not correct a cost that follows the wave slot, not the range
    // (profiles/r04k_*: tails 6-7.5 us, -0.4 us per pass)
    __builtin_amdgcn_s_setprio(3);
    // the range's last chunk: refractory stage by this wave
    const uint64_t tb = kFused ? region + tot.y : region + (uint64_t)nch * kChunk;
    // fused, single GPU, no synaptogenesis (its src list is global): the
    // tail's survivors stay in the stage's LDS (its entries are all read
    // before the first survivor is written: pend <= 256 <= one batch)
    uint4* tail_lds = nullptr;
    if constexpr (kFused) {
        static_assert(2 * SE * 4 >= 256 * sizeof(uint4), "the stage holds 256 tail survivors");
        // (the lean instance runs neither: shard mode and synaptogenesis are off)
        // (the shard instance's walk is the next launch: its tail goes to g2x)
        const bool lds_ok = kShard ? false : (kLean || (!d.shard_mode && !d.g2src));
        if (lds_ok && pend <= 256u) tail_lds = reinterpret_cast<uint4*>(s_stage[wid]);
    }
    const uint4 c = refrac_chunk<kChunk / 64, kRandom, kFused, true>(d, kp, region, tb, pend, now, pass, Rw, rbw, spec,
                                                               r, tot.z, s_f2, stage_at, tail_lds);
    const uint64_t gt = ((t_stream - t_start) >> 2) + (uint64_t)nch * d.chunk_penalty;
    const uint32_t cost = len ? (uint32_t)(gt < 1 ? 1 : (gt > 0xFFFFu ? 0xFFFFu : gt)) : 0u;
    if constexpr (kFused) {
        // fused: the look-back waits for stream + tail, so the partition
        // balances that (the tail's length follows the range's staged events)
        const uint64_t gf = ((__builtin_amdgcn_s_memrealtime() - t_start) >> 2) + (uint64_t)nch * d.chunk_penalty;
        const bool tl = tail_lds != nullptr;
        fused_end<BLOCK, NW, kLean, kShard>(d, kp, r, region, tot.x + c.x, tl ? tot.y : tot.y + c.y, tl ? tot.z : tot.z + c.z,
                             tl ? c.y : 0u, tl ? c.z : 0u, tail_lds, (uint32_t)gf, len == 0, spec, now, Rw, rbw, pass_f,
                             epoch, s_fz, t_stream, hw0, chunk_t, nch, wcb);
        return;
    }
    if (lane == 0) {
        // this wave's gate time (start to stream done, full chunks included;
        // the last chunk's refractory stage after the stream costs every wave
        // about the same and would bias short ranges) drives the next pass's
        // partition (partition_bounds): 40-ns units, clamped to [1, 0xFFFF],
        // 0 for an empty range.  Every full chunk adds chunk_penalty: the
        // dense stretch's time varies from pass to pass by more than the
        // stream's (the partition follows one pass late), so its ranges are
        // made shorter than the average, leaving room for that variation.
        d.range_info[r] = make_uint4(cost, tot.y + c.y, tot.z + c.z, nch);
        d.range_g1[r] = tot.x + c.x;
        if (d.wave_clock_on) {  // diagnostics (tools/wave_clock.py): 100 MHz wall clock
            d.wave_clock[kWaveClock * r + 1] = t_stream;
            d.wave_clock[kWaveClock * r + 2] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// ---------------------------------------------------------------------------
// The ordered spike budget of schedule C1 (brain.metal:85-98 without its
// races): an event that passed both gates is updated iff fewer than
// max_spikes spike candidates precede it in global event order.  Walked by
// k_spikes, k_claim and k_apply alike.  Every workgroup first builds, in LDS,
// per range: the capped exclusive candidate prefix, the exclusive prefix of
// full chunks and the survivor count (one packed scan over range_info, 64 KB
// read from L2 per workgroup at 4096 ranges -- cheaper than a separate
// single-workgroup scan launch, but L2-bandwidth-bound: every byte added per
// range costs every workgroup).
// The work items are the last chunk of every range and every full chunk, one
// per wave at a time: an item adds the candidates of its range's lower full
// chunks, leaves at once if the budget is spent, and otherwise visits its
// (<= kChunk) survivors in event order, calling f(region, entry, candidate,
// budget position, g2x index) for each one whose position is below the budget.
// A range without full chunks costs its item one global round trip (g2x).
constexpr uint32_t kWalkWaves = kApplyThreads / 64;

struct WalkLds {
    uint32_t* pre;   // [NR]     min(off + candidates of ranges < r, budget)
    uint32_t* cpre;  // [NR + 1] full chunks of ranges < r
    uint32_t* surv;  // [NR]     refractory survivors of range r
};

__device__ __forceinline__ WalkLds walk_lds_view(uint32_t* s, uint32_t NR)
{
    return WalkLds{s, s + NR, s + 2 * NR + 1};
}

// The next pass's sweep partition (k_apply only; part = its LDS, else null),
// computed from the same per-thread slice of ranges as the walk prefix, so
// its loads share the prefix's round trip and its cost scan the prefix's
// barriers.  Every k_apply workgroup then computes its own slice of boundaries
// into the other bounds buffer (range_bounds_next; the host swaps the two
// after the launch), so no workgroup waits for another.
//
// Equal ranges do not finish together: a wave's stream rate depends on how
// the SIMD arbiter treats it (the gate rotates priorities) and dense parts of
// the graph (the input->output block: every event pre-gated) stage more
// events.  So range r's measured gate time (range_info[r].x, written by this
// pass's gate), spread evenly over its iterations, gives a cumulative
// cost curve, and boundary k moves adapt_gain / 4 of the way (default half)
// from its old place towards the iteration where the curve reaches k / NR of
// the total, rounded to the nearest iteration (a floor never moves a boundary
// right by one iteration, and in the dense stretch one iteration is ~9 % of a
// range).  Results do not depend on the partition (event order is global, C1).
struct PartLds {
    uint32_t* cc;  // [NR + 1] exclusive cumulative cost
    uint32_t* rb;  // [NR + 1] current bounds
};

__device__ void partition_bounds(const DeviceState& d, const PartLds& P, uint32_t total_cost)
{
    const uint32_t NR = d.n_ranges;
    // this workgroup's boundaries k in [k0, k1); bounds 0 and NR never move
    const uint32_t slice = (NR + 1 + gridDim.x - 1) / gridDim.x;
    const uint32_t k0 = min(blockIdx.x * slice, NR + 1), k1 = min(k0 + slice, NR + 1);
    for (uint32_t k = k0 + threadIdx.x; k < k1; k += kApplyThreads) {
        const uint32_t nb = adapted_bound(d, P.cc, P.rb, NR, k, total_cost, P.rb[k]);
        d.range_bounds_next[k] = nb;
    }
}

// Builds the WalkLds arrays (and, with part, the partition curve); returns the
// number of full chunks.  With totals, also the pass's pre-gated and survivor
// counts (every thread gets them).
__device__ uint32_t walk_prefix(const DeviceState& d, uint64_t off, uint64_t budget, const WalkLds& L, uint64_t* s_red,
                                uint64_t* tot_g1, uint64_t* tot_g2, const PartLds* part, uint64_t* tot_cand)
{
    constexpr uint32_t kRound = 4;
    __shared__ uint32_t s_cw[kApplyThreads / 64];
    const uint32_t NR = d.n_ranges, per = (NR + kApplyThreads - 1) / kApplyThreads, q0 = threadIdx.x * per;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const bool adapt = part && d.adapt_ranges && NR >= 2;  // workgroup-uniform
    // pass 1: this thread's ranges' raw counts into LDS (pre = candidates,
    // cpre = full chunks, cc = cost), their sums into registers; pass 2 turns
    // its own LDS entries into exclusive prefixes in place (no per-range
    // register arrays: k_apply runs at 128 VGPRs)
    const bool totals = tot_g1 != nullptr;  // workgroup-uniform
    uint64_t sum = 0, g1 = 0, g2 = 0;
    uint32_t csum = 0;
    for (uint32_t j0 = 0; j0 < per; j0 += kRound) {
        uint4 ri[kRound];
        uint32_t b0[kRound], x1[kRound];
#pragma unroll
        for (uint32_t u = 0; u < kRound; ++u) {
            const uint32_t q = min(q0 + j0 + u, NR - 1);  // clamped: loads never depend on a branch
            ri[u] = range_totals(d, q);
            if (part) b0[u] = d.range_bounds[q];
            if (totals) x1[u] = d.range_g1[q];
        }
#pragma unroll
        for (uint32_t u = 0; u < kRound; ++u) {
            const uint32_t j = j0 + u, q = q0 + j;
            const bool in = j < per && q < NR;
            const uint64_t x = in ? (uint64_t)ri[u].z | ((uint64_t)ri[u].w << 32) : 0u;
            const uint32_t c = in && adapt ? ri[u].x : 0u;
            if (in) {
                L.pre[q] = ri[u].z;
                L.cpre[q] = ri[u].w;
                L.surv[q] = ri[u].y;
                if (part) part->rb[q] = b0[u];
                if (adapt) part->cc[q] = c;
            }
            sum += x;
            csum += c;
            if (totals) {
                g1 += in ? x1[u] : 0u;
                g2 += in ? ri[u].y : 0u;
            }
        }
    }
    if (part && threadIdx.x == 0) d.apply_clock[8 * blockIdx.x + 4] = __builtin_amdgcn_s_memrealtime();
    // the cost scan (DPP, u32: costs below 2^30) shares the prefix's barriers
    const uint32_t cin = wave_incl_scan(csum);
    if (lane == 63) s_cw[wv] = cin;
    uint64_t tot;
    uint64_t run = block_exclusive_scan<kApplyThreads>(sum, &tot, s_red);
    uint64_t cand = off + (uint32_t)run;
    uint32_t chunks = (uint32_t)(run >> 32);
    uint32_t before = 0, total_cost = 0;
    if (adapt) {
#pragma unroll
        for (uint32_t w = 0; w < kApplyThreads / 64; ++w) {
            before += w < wv ? s_cw[w] : 0u;
            total_cost += s_cw[w];
        }
    }
    uint32_t crun = before + cin - csum;
    for (uint32_t q = q0; q < min(q0 + per, NR); ++q) {
        const uint32_t nc = L.pre[q], nk = L.cpre[q];
        L.pre[q] = (uint32_t)(cand < budget ? cand : budget);
        L.cpre[q] = chunks;
        cand += nc;
        chunks += nk;
        if (adapt) {
            const uint32_t c = part->cc[q];
            part->cc[q] = crun;
            crun += c;
        }
    }
    if (threadIdx.x == 0) {
        if (tot_cand) *tot_cand = off + (uint32_t)tot;  // candidates before and in this shard
        L.cpre[NR] = (uint32_t)(tot >> 32);
        if (part) {
            part->cc[NR] = total_cost;
            part->rb[NR] = d.iters;
        }
    }
    if (totals) {  // LDS targets (a local's address would live in scratch)
        const uint64_t a = block_sum<kApplyThreads>(g1, s_red), b = block_sum<kApplyThreads>(g2, s_red);
        if (threadIdx.x == 0) {
            *tot_g1 = a;
            *tot_g2 = b;
        }
    }
    __syncthreads();
    if (part && threadIdx.x == 0) d.apply_clock[8 * blockIdx.x + 7] = __builtin_amdgcn_s_memrealtime();
    if (part) partition_bounds(d, *part, adapt ? total_cost : 0u);
    return (uint32_t)(tot >> 32);
}

// item j of the full chunks belongs to the last range r with cpre[r] <= j
__device__ __forceinline__ uint32_t chunk_range(const uint32_t* cpre, uint32_t NR, uint32_t j)
{
    uint32_t lo = 0, hi = NR;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cpre[mid] <= j) lo = mid;
        else hi = mid;
    }
    return lo;
}

struct NoWaveHook {
    __device__ void operator()(bool, const uint4&) const {}
};

// f(region, entry, candidate, budget position, g2x index) per visited event;
// h(visited and a candidate, entry) by the whole wave after every round.
template <class F, class H = NoWaveHook>
__device__ void budget_walk(const DeviceState& d, uint64_t off, uint64_t budget, uint32_t* s_lds, uint64_t* s_red,
                            F&& f, H h = H{}, uint64_t* tot_g1 = nullptr, uint64_t* tot_g2 = nullptr, uint64_t* tclock = nullptr,
                            bool partition = false, uint64_t* tot_cand = nullptr)
{
    const uint32_t NR = d.n_ranges;
    const WalkLds L = walk_lds_view(s_lds, NR);
    const PartLds P{s_lds + 3 * NR + 1, s_lds + 4 * NR + 2};
    const uint32_t items =
        NR + walk_prefix(d, off, budget, L, s_red, tot_g1, tot_g2, partition ? &P : nullptr, tot_cand);
    if (tclock && threadIdx.x == 0) *tclock = __builtin_amdgcn_s_memrealtime();
    const uint32_t lane = threadIdx.x & 63, w = wave_uniform(threadIdx.x >> 6);
    // consecutive items on different workgroups: the ranges that hold the
    // budget (the first ones) and the first full chunks spread over the chip
    for (uint32_t i = w * gridDim.x + blockIdx.x; i < items; i += gridDim.x * kWalkWaves) {
        uint32_t r, c;
        if (i < NR) {
            r = i;
            c = L.cpre[r + 1] - L.cpre[r];  // the last chunk follows the full ones
        } else {
            r = chunk_range(L.cpre, NR, i - NR);
            c = i - NR - L.cpre[r];
        }
        uint64_t P = L.pre[r];
        if (P >= budget) continue;
        const uint64_t region = region_of(d, r);
        const uint32_t nfull = L.cpre[r + 1] - L.cpre[r];
        uint32_t n = 0;
        if (nfull) {  // candidates of the lower full chunks; survivors of this one
            uint32_t cl = 0, gl = 0, own = 0;
            for (uint32_t c0 = 0; c0 < nfull; c0 += 64)
                if (c0 + lane < nfull && c0 + lane <= c) {
                    const uint4 x = d.chunk_cnt[chunk_slot(region, c0 + lane)];
                    if (c0 + lane < c) cl += x.z;
                    else own = x.y;
                    gl += x.y;
                }
            P += wave_sum(cl);
            if (P >= budget) continue;
            // the last chunk holds what the full ones do not
            n = c == nfull ? L.surv[r] - wave_sum(gl) : wave_sum(own);
        } else {
            n = L.surv[r];
        }
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
            h(cand && pre < budget, e[j]);
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

// Sharded passes: stamp rank r's first min(count_r, budget - offset_r) spikes
// (the gathered exchange records, rank order); workgroups take slices.
// The merged list is also this pass's spike list (fired_ring, global budget
// order) and, in steady state, goes into the next pass's bitmap like a
// single-GPU pass's spikes.  Returns the list's length (every thread).
__device__ uint64_t stamp_gathered(const DeviceState& d, const KernelParams& kp, const int32_t* gathered,
                                   uint32_t world, uint64_t now, uint64_t pass)
{
    const uint32_t words = xchg_words(kp.max_spikes);
    const uint64_t budget = kp.max_spikes;
    uint32_t* ring = d.fired_ring + (pass & (kFiredRing - 1)) * (uint64_t)kp.max_spikes;
    const uint32_t lane = threadIdx.x & 63;
    uint64_t off = 0;
    for (uint32_t r = 0; r < world && off < budget; ++r) {
        const int64_t cnt = *reinterpret_cast<const int64_t*>(gathered + r * words);
        const int32_t* sp = gathered + r * words + 2 * ABNN_SUMMARY_WORDS;
        const uint64_t room = budget - off, n = (uint64_t)cnt < room ? (uint64_t)cnt : room;
        // wave-uniform trip count (wave_set_next is wave-converged); the
        // list's 64-entry slices go to the waves in workgroup-interleaved
        // order, so that the stamps and the bitmap atomics of a few thousand
        // spikes spread over as many CUs (in workgroup order three CUs took
        // them all: their stores drained 5 us after every other workgroup's)
        const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
        for (uint64_t i0 = ((uint64_t)(threadIdx.x >> 6) * gridDim.x + blockIdx.x) * 64; i0 < n; i0 += nw * 64) {
            const uint64_t i = i0 + lane;
            const uint32_t nrn = i < n ? (uint32_t)sp[i] : 0xFFFFFFFFu;
            if (nrn < d.n_nrn) {
                d.last_fired[nrn] = now;
                ring[off + i] = nrn;
            }
            if (d.build_next) wave_set_next(d, nrn < d.n_nrn, nrn);
        }
        off += n;
    }
    return off;
}

// The end of a pass, by one thread of the last k_apply workgroup (every other
// one has read the pass-start scalars): rBar (brain.metal:110-113), clock tick
// (brain.metal:129).
__device__ void finalize_pass(const DeviceState& d, const KernelParams& kp, const int32_t* gathered, uint32_t world,
                              uint64_t now, float R, float rbar, uint64_t pass)
{
    uint64_t events = d.events;
    int64_t t0 = d.work->t0_g2;
    if (gathered) {
        const uint32_t words = xchg_words(kp.max_spikes);
        events = 0;
        t0 = 0;
        for (uint32_t r = 0; r < world; ++r) {
            const int64_t* sm = reinterpret_cast<const int64_t*>(gathered + r * words);
            events += (uint64_t)sm[2];
            t0 |= sm[1];
        }
    }
    if (t0 != 0 && kp.max_spikes > 0)
        *d.rbar = rbar + kp.alpha_rbar * (R - rbar);  // brain.metal:110-113
    if (events > 0) *d.clock = now + kp.clock_inc;     // brain.metal:129
    *d.pass_index = pass + 1;
    d.work->t0_g2 = 0;  // re-armed for the next pass
    __hip_atomic_store((gu32*)(&d.work->ticket), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
        const uint4 ri = range_totals(d, q);
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
// rank can stamp every rank's spikes in k_apply.
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
// sharded passes stamp from the gathered spike lists (stamp_gathered).
__global__ __launch_bounds__(kApplyThreads) void k_apply(DeviceState d, KernelParams kp,
                                                         const int32_t* gathered, uint32_t world, uint32_t rank)
{
    extern __shared__ uint32_t s_lds[];
    __shared__ uint64_t s_red[kWalkWaves];
    __shared__ uint32_t s_u[kWalkWaves], s_f[kWalkWaves], s_p[kWalkWaves];
    __shared__ uint64_t s_now, s_pass;
    __shared__ float s_R, s_rb;
    // per-workgroup timeline (diagnostics, abnn_debug_apply_clock): entry,
    // scalars, walk prefix, walk done, partition, ticket, pass end
    uint64_t* tc = d.apply_clock + 8 * blockIdx.x;
    // pass-start scalars (C1, brain.metal:105-106), read by one lane and used
    // through LDS only: the last workgroup rewrites them
    if (threadIdx.x == 0) {
        tc[0] = __builtin_amdgcn_s_memrealtime();
        s_R = *d.reward;
        s_rb = *d.rbar;
        s_now = *d.clock;
        s_pass = *d.pass_index;
    }
    __syncthreads();
    if (threadIdx.x == 0) tc[1] = __builtin_amdgcn_s_memrealtime();
    const float R = s_R, rb = s_rb;
    const uint64_t now = s_now, pass = s_pass;
    const bool random = d.mode == ABNN_MODE_RANDOM, stamp = gathered == nullptr;
    const bool prune = kp.w_prune > 0.0f, genesis = d.grown != nullptr && kp.p_new > 0.0f;
    __shared__ uint64_t s_g1, s_g2;  // the pass's gate totals (workgroup 0)
    __shared__ uint64_t s_cand;      // spike candidates up to and including this shard
    const bool first = blockIdx.x == 0;  // workgroup 0 also counts the pass's gate totals
    // the next pass's bitmap build (steady state): this thread's first item, loads in flight
    const uint64_t nitems = d.build_next ? next_items(d, kp) : 0;
    // counted from the workgroup's last thread down: the items land in the last
    // wave, away from wave 0 (the walk's heavy items) and the ticket wave --
    // gfx9's vmcnt covers stores and atomics, so a later load in the same wave
    // would wait for these atomics
    const uint32_t tr = kApplyThreads - 1 - threadIdx.x;
    const uint64_t x0 = (uint64_t)tr * gridDim.x + blockIdx.x, xs = (uint64_t)gridDim.x * kApplyThreads;
    const NextItem it0 = x0 < nitems ? next_item_load(d, kp, pass, x0) : NextItem{0u, 0u, 0u};
    ApplyCtx ac{R, rb, now, pass, random, stamp, stamp, false, prune, genesis, false, 0u, 0u, 0u};
    budget_walk(d, rank_offset(kp, gathered, rank), kp.max_spikes, s_lds, s_red,
                [&](uint64_t region, const uint4& e, bool f, uint64_t pre, uint64_t slot) {
        apply_event(d, kp, ac, region, e, f, pre, slot);
    }, [&](bool fired, const uint4& e) {  // this pass's spikes into the next pass's bitmap
        if (d.build_next && stamp) wave_set_next(d, fired, e.w);
    }, first ? &s_g1 : nullptr, first ? &s_g2 : nullptr, tc + 2, true, &s_cand);
    wave_set_next(d, it0.i < it0.lim, it0.n);
    const uint64_t xw = x0 - (uint64_t)(63 - (threadIdx.x & 63)) * gridDim.x;  // the wave's lowest item (lane 63)
    for (uint64_t k = xs; xw + k < nitems; k += xs) {  // wave-uniform
        const NextItem it = x0 + k < nitems ? next_item_load(d, kp, pass, x0 + k) : NextItem{0u, 0u, 0u};
        wave_set_next(d, it.i < it.lim, it.n);
    }
    // the spike list's length (positions below the budget)
    if (stamp && first && threadIdx.x == 0)
        d.n_fired_ring[pass & (kFiredRing - 1)] = (uint32_t)(s_cand < kp.max_spikes ? s_cand : kp.max_spikes);
    // sharded passes: every rank's spikes from the gathered exchange records,
    // budget order across ranks = global event order (brain.metal:125-126);
    // nothing of this kernel reads lastFired
    if (gathered) {
        const uint64_t nsp = stamp_gathered(d, kp, gathered, world, now, pass);
        if (first && threadIdx.x == 0) d.n_fired_ring[pass & (kFiredRing - 1)] = (uint32_t)nsp;
    }
    if (threadIdx.x == 0) tc[3] = __builtin_amdgcn_s_memrealtime();
    // statistics: every workgroup adds into its own slot (no cross-workgroup
    // sum; abnn_get_stats adds the slots)
    const uint32_t wu = wave_sum(ac.upd), wf = wave_sum(ac.nf), wp = wave_sum(ac.npr);
    if ((threadIdx.x & 63) == 0) {
        s_u[threadIdx.x >> 6] = wu;
        s_f[threadIdx.x >> 6] = wf;
        s_p[threadIdx.x >> 6] = wp;
    }
    lds_barrier();  // the weight stores and bitmap atomics stay in flight
    // one lane of the second-to-last wave (no build items, rarely a walk
    // store) takes the ticket, adds the statistics (no-return atomics into this
    // workgroup's own slot: no load waits behind the pass's stores) and, in the
    // last workgroup to arrive, ends the pass
    constexpr uint32_t kLeader = kApplyThreads - 128;
    if (threadIdx.x == kLeader) {
        const uint32_t ticket = __hip_atomic_fetch_add((gu32*)(&d.work->ticket), 1u, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
        uint32_t tu = 0, tf = 0, tp = 0;
        for (uint32_t v = 0; v < kWalkWaves; ++v) {
            tu += s_u[v];
            tf += s_f[v];
            tp += s_p[v];
        }
        abnn_stats* st = d.wg_stats + blockIdx.x;
        typedef unsigned long long ull;
        if (tu) atomicAdd((ull*)&st->updated, (ull)tu);
        if (tf) atomicAdd((ull*)&st->fired, (ull)tf);
        if (tp) atomicAdd((ull*)&st->pruned, (ull)tp);
        if (first) {
            atomicAdd((ull*)&st->passes, 1ull);
            atomicAdd((ull*)&st->events, (ull)d.events);
            atomicAdd((ull*)&st->pre_gated, (ull)s_g1);
            atomicAdd((ull*)&st->post_gated, (ull)s_g2);
        }
        tc[5] = __builtin_amdgcn_s_memrealtime();
        if (ticket == gridDim.x - 1) {
            finalize_pass(d, kp, gathered, world, now, R, rb, pass);
            tc[6] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// ---------------------------------------------------------------------------
// k_shard_walk: the second launch of a sharded pass on the fused path (the
// first is k_gate<..., kFused> in shard mode, then the all-gather).  One wave
// per range, as in the gate: the range's global budget position = the lower
// ranks' capped candidates (rank_offset) + its local position (range_info,
// written by the first launch); the walk of its survivors (range_walk: weight
// updates below the budget or the restore of mispredicted speculative stores,
// synaptogenesis at the global slot); every rank's spikes stamped from the
// gathered records in global budget order (stamp_gathered: no lastFired read
// is left in the pass) and set into the next pass's bitmap; the last
// workgroup ends the pass (finalize_pass) and predicts the next pass's
// speculative workgroups from the global cut.
template <int NW>
__global__ __launch_bounds__(NW * 64) void k_shard_walk(DeviceState d, KernelParams kp, const int32_t* gathered,
                                                        uint32_t world, uint32_t rank)
{
    __shared__ uint64_t s_setc[1];
    __shared__ uint32_t s_stat[3];
    __shared__ uint64_t s_now, s_pass;
    __shared__ float s_R, s_rb;
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, budget = kp.max_spikes;
    // diagnostics (tools/shard_clock.py): per workgroup, 100-MHz ticks
    uint64_t* ck = d.apply_clock + 8ull * (blockIdx.x % kWalkBlocks);
    if (threadIdx.x == 0) ck[0] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {  // pass-start scalars (C1), as the gate launch read them: workgroup 0
        s_R = d.work->ps_R;   // rewrites the live ones (finalize_pass) while others still start
        s_rb = d.work->ps_rb;
        s_now = d.work->ps_now;
        s_pass = d.work->ps_pass;
    }
    if (threadIdx.x < 3) s_stat[threadIdx.x] = 0u;
    __syncthreads();
    const float R = s_R, rb = s_rb;
    const uint64_t now = s_now, pass = s_pass;
    const uint64_t off = rank_offset(kp, gathered, rank);
    const uint32_t r = blockIdx.x * NW + wid;
    const uint4 ri = d.range_info[r];  // {local budget position (capped), survivors, candidates, spec | empty << 1}
    const uint64_t P = off + ri.x, region = (uint64_t)d.range_bounds[r] * d.iter_events;
    const bool spec = ri.w & 1u;
    ApplyCtx ac{R, rb, now, pass, false, false, false, false, kp.w_prune > 0.0f, d.grown != nullptr && kp.p_new > 0.0f,
                true, 0u, 0u, 0u};
    if (threadIdx.x == 0) ck[1] = __builtin_amdgcn_s_memrealtime();
    const uint32_t upd_rest = range_walk(d, kp, ac, r, region, ri.y, ri.z, P, spec, false, s_setc);
    if (threadIdx.x == 0) ck[2] = __builtin_amdgcn_s_memrealtime();
    // the next pass's spec prediction: the workgroup holding the global cut
    // (its first range's position below the budget, its last range's end at
    // or past it) names the ones below it, less one, as the fused pass does
    if (wid == NW - 1 && lane == 0) {
        const uint4 r0 = d.range_info[blockIdx.x * NW];
        if (off + r0.x < budget && P + ri.z >= budget) d.work->spec_wgs = spec_prediction(d, blockIdx.x, gridDim.x);
    }
    const uint32_t wu = wave_sum(ac.upd) + upd_rest, wf = wave_sum(ac.nf), wp = wave_sum(ac.npr);
    if (lane == 0) {
        atomicAdd(&s_stat[0], wu);
        atomicAdd(&s_stat[1], wf);
        atomicAdd(&s_stat[2], wp);
    }
    // every rank's spikes (global budget order) and, in steady state, into
    // the next pass's bitmap
    const uint64_t nsp = stamp_gathered(d, kp, gathered, world, now, pass);
    if (threadIdx.x == 0) ck[3] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (threadIdx.x == 0) ck[4] = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        typedef unsigned long long ull;
        abnn_stats* st = d.wg_stats + blockIdx.x % kWalkBlocks;
        if (s_stat[0]) atomicAdd((ull*)&st->updated, (ull)s_stat[0]);
        if (s_stat[1]) atomicAdd((ull*)&st->fired, (ull)s_stat[1]);
        if (s_stat[2]) atomicAdd((ull*)&st->pruned, (ull)s_stat[2]);
        ck[5] = __builtin_amdgcn_s_memrealtime();
        ck[6] = blockIdx.x == 0;
        if (blockIdx.x == 0) {  // the pass's end: no workgroup reads the live scalars (ps_* above)
            d.n_fired_ring[pass & (kFiredRing - 1)] = (uint32_t)nsp;
            const int64_t mine = *reinterpret_cast<const int64_t*>(gathered + rank * xchg_words(kp.max_spikes));
            if (off >= budget) d.work->spec_wgs = 0u;                        // the whole shard past the cut
            else if (off + (uint64_t)mine < budget) d.work->spec_wgs = gridDim.x;  // ... below it
            finalize_pass(d, kp, gathered, world, now, R, rb, pass);
        }
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
// The sharded lastVisited merge.  Unsharded, lastVisited[n] is
// the value of the LAST write: the `now` of the last pass that visited n, or
// what the host wrote after it.  A shard knows which neurons it visited since
// the last merge (visit_mark, set beside the lastVisited store); the others
// hold the replicated value of the last merge or host write.  Between two
// merges the clock only moves forward (a renormalisation is always followed
// by a merge), so of the shards that visited n the latest pass wrote the
// largest value: delta = visited ? value + 1 : 0 (clock values never reach
// 2^64 - 1), all-reduce MAX over the shards, then a non-zero result replaces
// the value on every shard and the marks clear.
__global__ __launch_bounds__(256) void k_visits_delta(const uint64_t* lv, const uint8_t* mark, uint64_t* delta,
                                                      uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        delta[i] = mark[i] ? lv[i] + 1u : 0u;
}

__global__ __launch_bounds__(256) void k_visits_merge(uint64_t* lv, uint8_t* mark, const uint64_t* reduced, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint64_t r = reduced[i];
        if (r) lv[i] = r - 1u;
        mark[i] = 0u;
    }
}

// ---------------------------------------------------------------------------
// The structural update's removal (abnn.h, round 6): with D tombstones and
// m = n - D, the k-th tombstone below m (index order) takes the k-th live
// record of the tail [m, n) (index order) and the array ends at m.  Holes lie
// below m and their fill above it, so no record is both read and written:
// every hole block moves its records at once, no inter-workgroup waits.
// Only the filled holes' records move (O(D)); the update reads the codes of
// the blocks holding tombstones (in a sweep: the visited window) to find the
// holes.  Round 4-5 closed the tombstones' span up in order (O(span) moves,
// 1.65 GB at config 5, in rounds that waited on lower blocks: ~0.8 ms).
// The update's words sp: [0] first block with a tombstone bf, [1] last such
// block + 1 bl, [2] tombstones D, [3] tombstones of block m / C below m,
// [4] records appended, [5] tombstones in the tail [m, n).
constexpr uint32_t kSwapThreads = 256;
constexpr uint32_t kSwapPer = kCompactChunk / kSwapThreads;  // records per thread (contiguous)
static_assert(kSwapPer == 16, "a thread loads its codes as 2 x 16 B (lo) + 16 B (hi)");

// the 24-bit code of the tombstone src (engine.h src_code(kSrcNone)), split
__device__ __forceinline__ uint32_t tomb_code() { return src_code(kSrcNone); }

// Records [base + 16 t, +16) of thread t: bit k of the result = record
// base + 16 t + k is a tombstone (tomb) or live, within [lo, hi).
__device__ __forceinline__ uint32_t swap_mask(const SynArrays& a, uint64_t base, uint64_t lo, uint64_t hi, bool tomb)
{
    const uint64_t i0 = base + (uint64_t)kSwapPer * threadIdx.x;
    if (i0 >= hi || i0 + kSwapPer <= lo) return 0u;
    const u32x4* pl = reinterpret_cast<const u32x4*>(a.lo + i0);
    const u32x4 l0 = __builtin_nontemporal_load(pl), l1 = __builtin_nontemporal_load(pl + 1);
    const u32x4 h = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.hi + hi_pos(i0)));
    const uint32_t lw[8] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w}, hw[4] = {h.x, h.y, h.z, h.w};
    const uint32_t tc = tomb_code();
    uint32_t m = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSwapPer; ++k) {
        const uint32_t code = ((lw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu) | ((hw[k >> 2] >> (8 * (k & 3))) & 0xFFu) << 16;
        const uint64_t i = i0 + k;
        if (i >= lo && i < hi && (code == tc) == tomb) m |= 1u << k;
    }
    return m;
}

__device__ __forceinline__ void move_record(const SynArrays& a, uint64_t from, uint64_t to)
{
    set_src(a, to, src_of(a, from));
    __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(a.dw + from)),
                                reinterpret_cast<uint64_t*>(a.dw + to));
}

__global__ void k_span_init(unsigned long long* sp)
{
    if (threadIdx.x < 8) sp[threadIdx.x] = threadIdx.x == 0 ? ~0ull : 0ull;
}

// Block mb = m / C (the one m falls in): its tombstones below m (sp[3]), the
// tally checked against it, and the tail's tombstones (sp[5]) from the tally
// of the blocks above it.
__global__ __launch_bounds__(kSwapThreads) void k_swap_mb(SynArrays a, uint64_t n, const uint32_t* dead, uint64_t nb,
                                                          unsigned long long* sp, uint32_t* err)
{
    __shared__ uint64_t s_wave[kSwapThreads / 64];
    const uint64_t D = sp[2];
    if (D == 0) return;
    if (D > n) {  // the tally disagrees with the records
        if (threadIdx.x == 0) __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    const uint64_t m = n - D, mb = m / kCompactChunk, base = mb * kCompactChunk;
    const uint64_t end = n < base + kCompactChunk ? n : base + kCompactChunk;
    const uint64_t below = __popc(swap_mask(a, base, base, m, true));
    const uint64_t above = __popc(swap_mask(a, base, m, end, true));
    const uint64_t tm = block_sum<kSwapThreads>(below, s_wave), ta = block_sum<kSwapThreads>(above, s_wave);
    uint64_t up = 0;  // tallied tombstones of the blocks above mb
    for (uint64_t b = mb + 1 + threadIdx.x; b < nb; b += kSwapThreads) up += dead[b];
    up = block_sum<kSwapThreads>(up, s_wave);
    if (threadIdx.x == 0) {
        sp[3] = tm;
        sp[5] = ta + up;
        if (tm + ta != (mb < nb ? dead[mb] : 0u)) __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The holes' ranks: off[b] = tallied tombstones of blocks [bf, b), for the
// hole blocks [bf, min(bl, mb + 1)) -- a two-launch scan over slices of 1024
// blocks (part[] = each slice's sum; the second launch adds the lower slices').
__device__ __forceinline__ void swap_hole_range(const unsigned long long* sp, uint64_t n, uint64_t& b0, uint64_t& b1)
{
    const uint64_t D = sp[2];
    b0 = b1 = 0;
    if (D == 0 || D >= n) return;  // (D = n: no record stays, nothing to fill)
    const uint64_t mb = (n - D) / kCompactChunk;
    b0 = sp[0];
    b1 = sp[1] < mb + 1 ? sp[1] : mb + 1;
    if (b1 < b0) b1 = b0;
}

__global__ __launch_bounds__(kScanThreads) void k_swap_scan1(const uint32_t* dead, uint64_t n,
                                                             const unsigned long long* sp, uint64_t* part)
{
    __shared__ uint64_t s_wave[kScanThreads / 64];
    uint64_t b0, b1;
    swap_hole_range(sp, n, b0, b1);
    const uint64_t b = b0 + (uint64_t)blockIdx.x * kScanThreads + threadIdx.x;
    if (b0 + (uint64_t)blockIdx.x * kScanThreads >= b1) return;  // workgroup-uniform
    const uint64_t t = block_sum<kScanThreads>(b < b1 ? dead[b] : 0u, s_wave);
    if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ __launch_bounds__(kScanThreads) void k_swap_scan2(const uint32_t* dead, uint64_t n,
                                                             const unsigned long long* sp, const uint64_t* part,
                                                             uint64_t* off)
{
    __shared__ uint64_t s_wave[kScanThreads / 64];
    uint64_t b0, b1;
    swap_hole_range(sp, n, b0, b1);
    if (b0 + (uint64_t)blockIdx.x * kScanThreads >= b1) return;  // workgroup-uniform
    uint64_t lower = 0;
    for (uint32_t s = threadIdx.x; s < blockIdx.x; s += kScanThreads) lower += part[s];
    lower = block_sum<kScanThreads>(lower, s_wave);
    const uint64_t b = b0 + (uint64_t)blockIdx.x * kScanThreads + threadIdx.x;
    uint64_t tot;
    const uint64_t pre = block_exclusive_scan<kScanThreads>(b < b1 ? dead[b] : 0u, &tot, s_wave);
    if (b < b1) off[b] = lower + pre;
}

// Tail blocks' live prefix (only when the tail holds tombstones: else the k-th
// live tail record is m + k): toff[b - mb] = live records of [m, b C) for the
// tail blocks b of [mb, ceil(n / C)) and one past them.  One workgroup.
__global__ __launch_bounds__(kScanThreads) void k_swap_tail(const uint32_t* dead, uint64_t n,
                                                            const unsigned long long* sp, uint64_t* toff)
{
    __shared__ uint64_t s_wave[kScanThreads / 64];
    const uint64_t D = sp[2];
    if (D == 0 || D >= n || sp[5] == 0) return;
    const uint64_t m = n - D, mb = m / kCompactChunk, nbn = (n + kCompactChunk - 1) / kCompactChunk;
    uint64_t run = 0;
    for (uint64_t j0 = 0; j0 <= nbn - mb; j0 += kScanThreads) {  // workgroup-uniform
        const uint64_t j = j0 + threadIdx.x, b = mb + j;
        uint64_t live = 0;
        if (b < nbn) {
            const uint64_t lo = b == mb ? m : b * kCompactChunk;
            const uint64_t hi = n < (b + 1) * kCompactChunk ? n : (b + 1) * kCompactChunk;
            const uint64_t tombs = b == mb ? dead[b] - sp[3] : dead[b];
            live = (hi - lo) - tombs;
        }
        uint64_t tot;
        const uint64_t pre = block_exclusive_scan<kScanThreads>(live, &tot, s_wave);
        if (j <= nbn - mb) toff[j] = run + pre;
        run += tot;
    }
}

// The fill: hole blocks [bf, min(bl, mb + 1)) over a persistent grid, one
// workgroup per block at a time.  A block's holes get the consecutive ranks
// off[b] + (their order in the block); its tombstones must match the tally
// (err = 2: the tally and the records disagree).
__global__ __launch_bounds__(kSwapThreads) void k_swap_fill(SynArrays a, uint64_t n, const uint32_t* dead,
                                                            const unsigned long long* sp, const uint64_t* off,
                                                            const uint64_t* toff, uint32_t* err)
{
    __shared__ uint64_t s_wave[kSwapThreads / 64];
    __shared__ uint16_t s_hole[kCompactChunk];  // the block's holes by rank (slow path)
    uint64_t b0, b1;
    swap_hole_range(sp, n, b0, b1);
    const uint64_t D = sp[2], m = n - D, mb = m / kCompactChunk, tail_tombs = sp[5];
    for (uint64_t b = b0 + blockIdx.x; b < b1; b += gridDim.x) {  // workgroup-uniform
        const uint32_t tally = dead[b];
        if (tally == 0) continue;
        const uint64_t base = b * kCompactChunk, hi = m < base + kCompactChunk ? m : base + kCompactChunk;
        const uint32_t hm = swap_mask(a, base, base, hi, true);
        uint64_t h;
        const uint64_t pre = block_exclusive_scan<kSwapThreads, true>((uint64_t)__popc(hm), &h, s_wave);
        // block mb: its tombstones below m (checked against the tally by k_swap_mb)
        if (h != (b == mb ? sp[3] : tally)) {
            if (threadIdx.x == 0) __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            continue;
        }
        const uint64_t k0 = off[b];
        const uint64_t i0 = base + (uint64_t)kSwapPer * threadIdx.x;
        if (tail_tombs == 0) {  // the tail is all live: the k-th live tail record is m + k
            uint32_t x = hm;
            for (uint64_t r = k0 + pre; x; x &= x - 1u, ++r) move_record(a, m + r, i0 + (uint32_t)__builtin_ctz(x));
            continue;
        }
        // the tail holds tombstones: the holes' offsets in LDS by rank, then
        // the tail blocks covering ranks [k0, k0 + h), each scanned for its
        // live records' ranks
        {
            uint32_t x = hm;
            for (uint64_t q = pre; x; x &= x - 1u, ++q)
                s_hole[q] = (uint16_t)(kSwapPer * threadIdx.x + (uint32_t)__builtin_ctz(x));
        }
        __syncthreads();
        const uint64_t nt = (n + kCompactChunk - 1) / kCompactChunk - mb;  // tail blocks
        uint64_t lo_j = 0, hi_j = nt;  // the last j with toff[j] <= k0
        while (hi_j - lo_j > 1) {
            const uint64_t mid = (lo_j + hi_j) >> 1;
            if (toff[mid] <= k0) lo_j = mid;
            else hi_j = mid;
        }
        for (uint64_t j = lo_j; j < nt && toff[j] < k0 + h; ++j) {  // workgroup-uniform
            const uint64_t tb = (mb + j) * kCompactChunk;
            const uint64_t tlo = j == 0 ? m : tb, thi = n < tb + kCompactChunk ? n : tb + kCompactChunk;
            const uint32_t lm = swap_mask(a, tb, tlo, thi, false);
            uint64_t lt;
            const uint64_t lp = block_exclusive_scan<kSwapThreads, true>((uint64_t)__popc(lm), &lt, s_wave);
            if (lt != toff[j + 1] - toff[j]) {
                if (threadIdx.x == 0) __hip_atomic_store(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            const uint64_t t0 = tb + (uint64_t)kSwapPer * threadIdx.x;
            uint32_t x = lm;
            for (uint64_t r = toff[j] + lp; x; x &= x - 1u, ++r)
                if (r >= k0 && r < k0 + h) move_record(a, t0 + (uint32_t)__builtin_ctz(x), base + s_hole[r - k0]);
        }
        __syncthreads();  // s_hole is reused by the next block
    }
}

// After the fill: no tombstone is left below m, and the blocks from m on hold
// the appended (live) records next: their tally is cleared.
__global__ __launch_bounds__(256) void k_dead_clear(uint32_t* dead, uint64_t n, const unsigned long long* sp)
{
    const uint64_t D = sp[2];
    if (D == 0) return;
    const uint64_t mb = (D <= n ? n - D : 0) / kCompactChunk, bf = sp[0] < mb ? sp[0] : mb;
    const uint64_t nbn = (n + kCompactChunk - 1) / kCompactChunk;
    for (uint64_t b = bf + (uint64_t)blockIdx.x * 256 + threadIdx.x; b < nbn; b += (uint64_t)gridDim.x * 256) dead[b] = 0u;
}

// The grown records (slots in (pass, slot) order, w = 1: used) appended after
// the n - D live records while capacity lasts; sp[4] = how many; the slots
// cleared for the next period.  Two launches over 1024-slot blocks: the used
// count of each, then each block's records at the lower blocks' count.
__global__ __launch_bounds__(kScanThreads) void k_grown_counts(const uint4* grown, uint64_t slots, uint32_t* cnt)
{
    __shared__ uint64_t s_wave[kScanThreads / 64];
    const uint64_t j = (uint64_t)blockIdx.x * kScanThreads + threadIdx.x;
    const uint64_t c = block_sum<kScanThreads>(j < slots && grown[j].w == 1u ? 1u : 0u, s_wave);
    if (threadIdx.x == 0) cnt[blockIdx.x] = (uint32_t)c;
}

__global__ __launch_bounds__(kScanThreads) void k_append_grown(SynArrays a, uint64_t n, uint64_t cap, uint4* grown,
                                                               uint64_t slots, const uint32_t* cnt,
                                                               unsigned long long* sp, unsigned long long* stats_grown,
                                                               const uint32_t* err)
{
    __shared__ uint64_t s_wave[kScanThreads / 64];
    __shared__ uint32_t s_err;
    // a failed removal (err: a compaction wait gave up, or the tally and the
    // records disagree) leaves n - D meaningless: append nothing.  err is the
    // host-mapped error word: ONE read per workgroup (a read per thread
    // crossed PCIe 1024 times per workgroup, 360 us per update)
    if (threadIdx.x == 0) s_err = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (s_err != 0u) return;
    const uint64_t live = n - sp[2];
    uint64_t below = 0;  // used slots in the lower blocks
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += kScanThreads) below += cnt[b];
    below = block_sum<kScanThreads>(below, s_wave);
    const uint64_t j = (uint64_t)blockIdx.x * kScanThreads + threadIdx.x;
    const uint4 g = j < slots ? grown[j] : make_uint4(0u, 0u, 0u, 0u);
    const bool used = g.w == 1u;
    uint64_t tot;
    const uint64_t pre = block_exclusive_scan<kScanThreads>(used ? 1u : 0u, &tot, s_wave);
    const uint64_t pos = live + below + pre;
    if (used && pos < cap) {
        set_src(a, pos, g.x);
        a.dw[pos] = make_uint2(g.y, g.z);
    }
    if (j < slots) grown[j] = make_uint4(0u, 0u, 0u, 0u);
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {  // the last block knows the total
        const uint64_t run = below + tot, added = live + run <= cap ? run : cap - live;
        sp[4] = added;
        *stats_grown += added;  // abnn_stats.grown (host-kept counter block)
    }
}

// The structural update's span (abnn.h contract): out = {first block with a
// tombstone, last such block + 1, tombstones} from the per-block tally.
__global__ __launch_bounds__(256) void k_dead_bounds(const uint32_t* dead, uint64_t nb, unsigned long long* out)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    unsigned long long lo = ~0ull, hi = 0, sum = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x; b < nb; b += stride) {
        const uint32_t c = dead[b];
        if (c) {
            lo = lo < b ? lo : b;
            hi = b + 1;
            sum += c;
        }
    }
    if (sum) {
        atomicMin(out, lo);
        atomicMax(out + 1, hi);
        atomicAdd(out + 2, sum);
    }
}

// The structural update's tombstone tally recounted from the records (after a
// host upload, which may hold tombstones: a saved pruned brain): dead[b] =
// tombstones among records [b kCompactChunk, (b + 1) kCompactChunk) of the
// first n, for blocks b0 + blockIdx.x.
__global__ __launch_bounds__(256) void k_tally_dead(SynArrays a, uint64_t n, uint32_t* dead, uint64_t b0)
{
    __shared__ uint64_t s_wave[4];
    const uint64_t b = b0 + blockIdx.x, base = b * kCompactChunk;
    uint64_t c = 0;
    for (uint32_t k = threadIdx.x; k < (uint32_t)kCompactChunk; k += 256) {
        const uint64_t i = base + k;
        c += i < n && src_of(a, i) == kSrcNone;
    }
    c = block_sum<256>(c, s_wave);
    if (threadIdx.x == 0) dead[b] = (uint32_t)c;
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
        set_src(d.syn, k, src);
        d.syn.dw[k] = make_uint2(dst, __float_as_uint(w));
    }
}

__global__ __launch_bounds__(256) void k_checksum(DeviceState d, uint64_t* out)
{
    __shared__ uint64_t s[4];
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t acc = 0;
    for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < d.n_syn; k += stride) {
        const uint64_t i = d.syn_offset + k;
        const uint2 dw = d.syn.dw[k];
        const uint64_t a = ((uint64_t)src32(src_of(d.syn, k)) << 32) | dw.x;
        const uint64_t b = (uint64_t)dw.y << 32;  // pad = 0
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

// budget walks: WalkLds (three u32 per range; the finalizing workgroup reuses two)
// dynamic LDS of the budget walk (k_spikes, k_claim): its prefix arrays;
// k_apply adds the partition curve and bounds
inline size_t walk_lds(const DeviceState& d, bool partition = false)
{
    const size_t nr = std::max(1u, d.n_ranges);
    return (3 * nr + 1 + (partition ? 2 * (nr + 1) : 0)) * 4;
}

template <int BLOCK, int K, int FW>
hipError_t launch_gate_shape(const DeviceState& d, const KernelParams& kp, hipStream_t s)
{
    const dim3 g(d.gate_blocks), b(BLOCK);
    const bool random = d.mode == ABNN_MODE_RANDOM;
    if (kp.track_visits) {
        if (random) hipLaunchKernelGGL((k_gate<BLOCK, K, FW, true, true, false>), g, b, 0, s, d, kp);
        else hipLaunchKernelGGL((k_gate<BLOCK, K, FW, true, false, false>), g, b, 0, s, d, kp);
    } else {
        if (random) hipLaunchKernelGGL((k_gate<BLOCK, K, FW, false, true, false>), g, b, 0, s, d, kp);
        else hipLaunchKernelGGL((k_gate<BLOCK, K, FW, false, false, false>), g, b, 0, s, d, kp);
    }
    return hipGetLastError();
}

template <int BLOCK, int K, int FW>
hipError_t launch_fused_shape(const DeviceState& d, const KernelParams& kp, hipStream_t s)
{
    const dim3 g(d.gate_blocks), b(BLOCK);
    // lean: the pass without pruning or synaptogenesis -- single-GPU, or the
    // first launch of a sharded pass (less code in the pass end)
    const bool plastic = kp.w_prune > 0.0f || (d.grown != nullptr && kp.p_new > 0.0f);
    const bool lean = d.lean && !plastic;
    if (kp.track_visits) hipLaunchKernelGGL((k_gate<BLOCK, K, FW, true, false, true>), g, b, 0, s, d, kp);
    else if (lean && !d.shard_mode) hipLaunchKernelGGL((k_gate<BLOCK, K, FW, false, false, true, true>), g, b, 0, s, d, kp);
    else if (lean) hipLaunchKernelGGL((k_gate<BLOCK, K, FW, false, false, true, true, true>), g, b, 0, s, d, kp);
    else hipLaunchKernelGGL((k_gate<BLOCK, K, FW, false, false, true>), g, b, 0, s, d, kp);
    return hipGetLastError();
}

template <int BLOCK, int K, int FW>
int occupancy_shape(bool track, bool random)
{
    int n = 0;
    hipError_t e;
    if (track)
        e = random ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, true, true, false>, BLOCK, 0)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, true, false, false>, BLOCK, 0);
    else
        e = random ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, false, true, false>, BLOCK, 0)
                   : hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, false, false, false>, BLOCK, 0);
    return e == hipSuccess ? n : 0;
}

template <int BLOCK, int K, int FW>
int occupancy_fused_shape(bool track)
{
    // every instance launch_fused_shape may select for these knobs: the
    // look-back needs all gate workgroups resident, whichever one runs
    int n = 0, m = 0;
    if (track) {
        const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, true, false, true>, BLOCK, 0);
        return e == hipSuccess ? n : 0;
    }
    int q = 0;
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_gate<BLOCK, K, FW, false, false, true>, BLOCK, 0);
    const hipError_t f = hipOccupancyMaxActiveBlocksPerMultiprocessor(&m, k_gate<BLOCK, K, FW, false, false, true, true>, BLOCK, 0);
    const hipError_t h = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &q, k_gate<BLOCK, K, FW, false, false, true, true, true>, BLOCK, 0);
    return e == hipSuccess && f == hipSuccess && h == hipSuccess ? std::min(n, std::min(m, q)) : 0;
}

// Compiled gate shapes: threads per workgroup x events per lane x filter words.
#define ABNN_GATE_SHAPES(X) \
    X(1024, 8, 8192)        \
    X(1024, 16, 8192)       \
    X(512, 8, 8192)         \
    X(512, 16, 8192)        \
    X(256, 16, 8192)

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

// Fused pass shapes: 1024-thread workgroups, at most 512 of them (one
// look-back poll) and 4096 ranges (the partition's LDS prefix), all resident
// (one per CU: the look-back waits only on other workgroups of the launch,
// which are resident or done; the wait is bounded anyway).
#define ABNN_FUSED_SHAPES(X) \
    X(1024, 8, 8192)         \
    X(1024, 16, 8192)

int fused_blocks_per_cu(uint32_t block, uint32_t k, uint32_t fw, bool track)
{
    switch (shape_key(block, k, fw)) {
#define X(B, K, F) case shape_key(B, K, F): return occupancy_fused_shape<B, K, F>(track);
        ABNN_FUSED_SHAPES(X)
#undef X
    }
    return 0;
}

bool fused_pass_supported(const DeviceState& d)
{
    bool shape = false;
    switch (shape_key(d.gate_block, d.gate_k, d.filter_words)) {
#define X(B, K, F) case shape_key(B, K, F): shape = true; break;
        ABNN_FUSED_SHAPES(X)
#undef X
    }
    // the look-back waits on other workgroups of the launch: every one must be
    // resident at once (fused_max_blocks: the occupancy of the fused kernel)
    return shape && d.mode == ABNN_MODE_SWEEP && d.range_map == 0 && d.gate_blocks > 0 &&
           d.gate_blocks <= kLbMaxWords * 64 && d.n_ranges <= kFusedMaxRanges && d.gate_blocks <= d.fused_max_blocks;
}

hipError_t launch_fused_pass(const DeviceState& d, const KernelParams& kp, hipStream_t s)
{
    switch (shape_key(d.gate_block, d.gate_k, d.filter_words)) {
#define X(B, K, F) case shape_key(B, K, F): return launch_fused_shape<B, K, F>(d, kp, s);
        ABNN_FUSED_SHAPES(X)
#undef X
    }
    return hipErrorInvalidValue;
}

hipError_t launch_shard_walk(const DeviceState& d, const KernelParams& kp, const int32_t* gathered, uint32_t world,
                             uint32_t rank, hipStream_t s)
{
    if (d.gate_block != 1024) return hipErrorInvalidValue;  // one wave per range of the 1024-thread fused gate
    hipLaunchKernelGGL(k_shard_walk<16>, dim3(d.gate_blocks), dim3(1024), 0, s, d, kp, gathered, world, rank);
    return hipGetLastError();
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
                        uint32_t world, uint32_t rank, hipStream_t s)
{
    const dim3 g(d.apply_blocks ? d.apply_blocks : kWalkBlocks), b(kApplyThreads);
    if (d.mode == ABNN_MODE_RANDOM) {
        hipLaunchKernelGGL(k_claim, g, b, walk_lds(d), s, d, kp, gathered, rank);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_apply, g, b, walk_lds(d, true), s, d, kp, gathered, world, rank);
    return hipGetLastError();
}

hipError_t launch_renorm(const DeviceState& d, uint64_t base, hipStream_t s)
{
    hipLaunchKernelGGL(k_renorm, dim3(blocks_for(d.n_nrn > 0 ? d.n_nrn : 1)), dim3(256), 0, s, d,
                       base);
    return hipGetLastError();
}

// Interchange src values (u32, 0xFFFFFFFF = tombstone) <-> the packed
// streams, records [first, first + n).
__global__ __launch_bounds__(256) void k_pack_src(SynArrays a, const uint32_t* in, uint64_t first, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        const uint32_t v = in[i];
        set_src(a, first + i, v >= kSrcNone ? kSrcNone : v);
    }
}

__global__ __launch_bounds__(256) void k_unpack_src(SynArrays a, uint32_t* out, uint64_t first, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256)
        out[i] = src32(src_of(a, first + i));
}

hipError_t launch_pack_src(const SynArrays& a, const uint32_t* in_dev, uint64_t first, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_pack_src, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, s, a,
                       in_dev, first, n);
    return hipGetLastError();
}

hipError_t launch_unpack_src(const SynArrays& a, uint32_t* out_dev, uint64_t first, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_unpack_src, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, s, a,
                       out_dev, first, n);
    return hipGetLastError();
}

// The structural update's removal and append, all on `s` (sp: 5 device words,
// see k_span_init): span bounds, offsets, z, the in-place compaction (one
// workgroup per CU), the hole, the grown records.
hipError_t launch_structural_update(const SynArrays& syn, uint64_t n, uint64_t cap, uint32_t* dead, uint64_t nb,
                                    uint64_t* offsets, uint64_t* part, uint64_t* toff, unsigned long long* sp,
                                    uint32_t* err, uint32_t cus, uint4* grown, uint64_t slots, uint32_t* grown_cnt,
                                    unsigned long long* stats_grown, hipStream_t s)
{
    hipLaunchKernelGGL(k_span_init, dim3(1), dim3(64), 0, s, sp);
    if (dead && nb && n) {
        hipLaunchKernelGGL(k_dead_bounds, dim3((uint32_t)std::min<uint64_t>((nb + 255) / 256, 1024)), dim3(256), 0, s,
                           dead, nb, sp);
        hipLaunchKernelGGL(k_swap_mb, dim3(1), dim3(kSwapThreads), 0, s, syn, n, dead, nb, sp, err);
        const uint32_t slices = (uint32_t)((nb + kScanThreads - 1) / kScanThreads);  // covers any hole range
        hipLaunchKernelGGL(k_swap_scan1, dim3(slices), dim3(kScanThreads), 0, s, dead, n, sp, part);
        hipLaunchKernelGGL(k_swap_scan2, dim3(slices), dim3(kScanThreads), 0, s, dead, n, sp, part, offsets);
        hipLaunchKernelGGL(k_swap_tail, dim3(1), dim3(kScanThreads), 0, s, dead, n, sp, toff);
        hipLaunchKernelGGL(k_swap_fill, dim3(std::max(1u, cus) * 8u), dim3(kSwapThreads), 0, s, syn, n, dead, sp, offsets,
                           toff, err);
        hipLaunchKernelGGL(k_dead_clear, dim3((uint32_t)std::min<uint64_t>((nb + 255) / 256, 1024)), dim3(256), 0, s,
                           dead, n, sp);
    }
    if (grown && slots) {
        const uint32_t gb = (uint32_t)((slots + kScanThreads - 1) / kScanThreads);
        hipLaunchKernelGGL(k_grown_counts, dim3(gb), dim3(kScanThreads), 0, s, grown, slots, grown_cnt);
        hipLaunchKernelGGL(k_append_grown, dim3(gb), dim3(kScanThreads), 0, s, syn, n, cap, grown, slots, grown_cnt, sp,
                           stats_grown, err);
    }
    return hipGetLastError();
}

hipError_t launch_visits_delta(const uint64_t* lv, const uint8_t* mark, uint64_t* delta, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_visits_delta, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, s, lv,
                       mark, delta, n);
    return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_reduce_u64(uint64_t* acc, const uint64_t* x, uint64_t n, uint32_t max)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const uint64_t a = acc[i], b = x[i];
        acc[i] = max ? (a > b ? a : b) : a + b;
    }
}

hipError_t launch_reduce_u64(uint64_t* acc, const uint64_t* x, uint64_t n, bool max, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_reduce_u64, dim3(blocks), dim3(256), 0, s, acc, x, n, max ? 1u : 0u);
    return hipGetLastError();
}

hipError_t launch_visits_merge(uint64_t* lv, uint8_t* mark, const uint64_t* reduced, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_visits_merge, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 4096)), dim3(256), 0, s, lv,
                       mark, reduced, n);
    return hipGetLastError();
}

hipError_t launch_tally_dead(const SynArrays& a, uint64_t n, uint32_t* dead, uint64_t first, uint64_t count,
                             hipStream_t s)
{
    if (count == 0 || first >= n) return hipSuccess;
    const uint64_t b0 = first / kCompactChunk, b1 = (std::min(first + count, n) + kCompactChunk - 1) / kCompactChunk;
    hipLaunchKernelGGL(k_tally_dead, dim3((uint32_t)(b1 - b0)), dim3(256), 0, s, a, n, dead, b0);
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
