// raw.hip -- the reference kernel's buffer-index ABI (abnn.h,
// abnn_launch_traversal): one C1 pass over CALLER-OWNED buffers in the
// reference's own layouts -- 16-B SynapsePacked records and u32 lastF / clock /
// budget (brain.metal:42-58, bound by Brain::encode_traversal at
// brain.cpp:93-118; allocated by Brain::build_buffers at brain.cpp:54-60).
//
// The handle API (capi.hip, kernels.hip) re-lays the records out for the gate
// (3 B per event).  Here the caller owns the memory, so every visited event
// streams its whole 16-B record (brain.metal:70) -- the compulsory traffic.
// What is not compulsory is the reference's 4-B lastF[src] gather per event
// (brain.metal:73): the pass answers the pre-spike gate from an LDS filter of
// the recent neurons and gathers lastF only for the ~1 % of events the filter
// passes.  Launches per pass, all on the caller's stream:
//
//   k_raw_filter : lastF (read once, 4 B per neuron) -> the blocked Bloom
//                  filter of the neurons with age <= window_pre (the same
//                  filter as the handle API's; each filter block
//                  built by one workgroup from its ~20 bitmap words: no
//                  atomics, no zeroing); resets the pass's workspace counters.
//   k_raw_pass   : (round 5, the default) the rest of the pass in ONE
//                  persistent launch -- see its comment below: one
//                  adaptive contiguous range per workgroup, groups claimed by
//                  its waves, the gates in one round trip per ~192 staged
//                  hits, survivors in a bounded pool, a decoupled look-back
//                  for the ordered budget, the walks, the stamps, the pass end.
//
// The round-4 pass (ABNN_RAW_FUSED=0, or where 256 workgroups of ~158 KB LDS
// cannot be resident at once) keeps five launches after the filter:
//   k_raw_gate   : persistent, one 1024-thread workgroup per CU; every wave
//                  sweeps groups of 1024 events (interleaved over the CUs):
//                  16-B records four iterations ahead, the filter test per
//                  event (one 8-B LDS read), hits staged in LDS in event
//                  order; per group the staged hits' lastF[src] and lastF[dst]
//                  in ONE round trip -> exact pre-spike gate (brain.metal:
//                  73-77), refractory gate (brain.metal:79-83), spike
//                  candidate (brain.metal:91-92), u32 age (brain.metal:116);
//                  survivors appended to the wave's survivor sequence, held
//                  in 4-KiB chunks of a BOUNDED pool (one atomic per chunk).
//   k_raw_scan_local + k_raw_scan : the groups' capped candidate prefix
//                  (the ordered budget of C1, brain.metal:85-98 without its
//                  races) in 4096-group blocks, then one workgroup: the
//                  blocks' prefix, the budget cut, the pass end on the
//                  scalars: *budget left, rBar (brain.metal:110-113), one
//                  clock tick (brain.metal:129).
//   k_raw_apply  : the groups below the cut: the weight update of their
//                  survivors below the budget (brain.metal:101-122) and the
//                  spikes' stamps (brain.metal:125-126): it reads no lastF.
//                  A group whose survivors did not fit the pool is recomputed
//                  from its records with the pass-start lastF; in such a pass
//                  the spikes go to a list in budget order instead and
//   k_raw_stamp  : stamps them after every lastF read of the pass (C1).
//
// renormalise_clock_and_times (brain.metal:135-145): k_raw_renorm subtracts
// the clock read by every thread, k_raw_zero_clock zeroes it afterwards (the
// reference zeroes it inside the same kernel, racing with the readers).
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <atomic>
#include <vector>

#include "engine.h"
#include "device.h"

#pragma clang fp contract(off)

namespace abnn {
namespace {

constexpr uint32_t kRawBlock = 1024;                 // gate threads per workgroup (16 waves)
constexpr uint32_t kRawGateWGs = 256;                // gate workgroups (one per CU; no inter-WG dependency)
constexpr uint32_t kRawWaves = kRawGateWGs * (kRawBlock / 64);  // 4096 gate waves
constexpr uint32_t kRawK = 4;                        // records per lane per iteration (256 events)
constexpr uint32_t kRawIt = 64 * kRawK;              // events per iteration
constexpr uint32_t kRawD = 4;                        // iterations per group = buffers in flight
constexpr uint32_t kRawGroup = kRawIt * kRawD;       // 1024 events: the scan / apply unit
constexpr uint32_t kRawChunk = 256;                  // survivor entries (16 B) per pool chunk
constexpr uint32_t kRawStage = 256;                  // staged hits per wave (flush above 192)
constexpr uint32_t kRawOpen = 32;                    // groups whose hits may wait in the stage (gate)
constexpr uint32_t kRawFB = 8192;                    // filter blocks (64 KiB of LDS)
constexpr uint32_t kRawFLg = 13;
constexpr uint32_t kRawSpikeCap = 65536;             // spike list entries (deferred stamps)
constexpr uint32_t kRawScanThreads = 1024;
constexpr uint32_t kRawScanBlock = 4 * kRawScanThreads;  // groups per k_raw_scan_local workgroup
constexpr uint32_t kRfNR = kRawGateWGs;              // fused pass: one contiguous range per workgroup
constexpr uint32_t kRfMaxG = 2048;                   // fused pass: groups per workgroup range (LDS tallies)
#ifndef ABNN_RF_D
#define ABNN_RF_D 3
#endif
constexpr uint32_t kRfD = ABNN_RF_D;                 // fused pass: iterations in flight per wave
#ifndef ABNN_RF_G
#define ABNN_RF_G 2
#endif
constexpr uint32_t kRfG = ABNN_RF_G;                 // fused pass: the least group (iterations, a power of two)
constexpr uint32_t kRfCt = 16;                       // fused pass: chunk ids of a wave's sequence kept in LDS
constexpr uint32_t kRfWB = 4;                        // fused pass: chunks a walk loads at once
constexpr uint32_t kRfLink = kRawChunk - 1;          // fused pass: a pool chunk holds 255 survivors + the next chunk's id
constexpr uint32_t kRfClk = 8;  // fused pass, diagnostics words per gate wave: entry, stream start / end, look-back,
                                // walk, end (100 MHz), iterations, survivors
static_assert(kRawWaves % kRawScanThreads == 0, "k_raw_scan sums the gate waves' statistics in whole rounds");
constexpr uint32_t kRawApplyWGs = 1024;              // x 4 waves, grid-stride over the groups below the cut
constexpr uint32_t kRawNone = 0xFFFFFFFFu;
constexpr uint32_t kRawCtab = 0xFFFFFFFEu;  // ginfo: the group's survivors span > 2 chunks (ctab lookup)
constexpr uint32_t kRawRedo = 0xFFFFFFFDu;  // ginfo: not all stored (the pool ran out): recompute
constexpr uint32_t kRawInit = 0x52415731u;  // RawHdr::init of a workspace whose err word is live

// Workspace (16-B aligned pieces):
//   hdr | filter (FB uint2) | lb | bounds | cost | clk (E-independent: raw_state_bytes) | gcand[NG] | gpre[NG] | btot[NG / 4096] | ginfo[NG] {S, seq, chunks} |
//   wlim[W] | wstat[W] | ctab[W][maxc] | spikes[L] | pool[cap][kRawChunk] uint4
struct RawHdr {
    uint32_t now, budget0, t0, ncand;  // pass-start clock and budget; event 0 survived; spikes (capped)
    float R, rb;                       // pass-start reward and rBar (brain.metal:105-106)
    uint32_t chunks;                   // pool chunks handed out this pass
    uint32_t gcut;                     // groups below the budget's cut: [0, gcut)
    uint32_t direct;                   // the spikes exceed the spike list: apply stamps itself
    uint32_t err;                      // sticky: a recomputed group met direct stamps in some pass since the
                                       // last abnn_traversal_workspace_error (which clears it)
    uint32_t ovf;                      // some wave's survivors overflowed the pool this pass (groups recomputed)
    uint32_t init;                     // kRawInit once err has been initialised (the workspace starts as garbage)
    uint64_t g1, g2;                   // the pass's pre-gated and refractory-surviving events (diagnostics)
    // the fused pass (k_raw_pass): its state across passes, on the device
    uint32_t pass;                     // fused passes run on this workspace (rotates bounds / costs, tags the look-back)
    uint32_t pvalid;                   // kRawInit: bounds[pass % 3] hold a partition of pE events; costs of pass - 1 valid
    uint32_t pE;                       // events the partition was made for
    uint32_t wdone;                    // workgroups whose walk is done (this pass; pool-overflow passes wait for it)
    uint32_t pad2[12];
};
static_assert(sizeof(RawHdr) == 128, "workspace header");

struct RawWs {
    RawHdr* hdr;
    uint2* filter;
    uint32_t* gcand;   // spike candidates per group
    uint32_t* gpre;    // exclusive candidate prefix per group within its scan block of 4096 groups
    uint32_t* btot;    // per scan block: its candidates; then (k_raw_scan) the blocks before it, capped
    uint4* ginfo;      // {survivors, first index in the owning wave's survivor sequence, pool chunk of
                       //  that entry, the next chunk} (kRawCtab: > 2 chunks, kRawRedo: not all stored)
    uint32_t* wlim;    // per wave: survivor-sequence entries stored (the rest overflowed the pool)
    uint2* wstat;      // per wave: {pre-gated, survivors} of its groups (k_raw_scan sums them)
    uint32_t* ctab;    // per wave: pool chunk of every 256 entries of its sequence
    uint32_t* spikes;  // dst per budget position (deferred stamps)
    unsigned long long* lb;  // fused pass: per gate workgroup its look-back word (epoch-tagged, never reset)
    uint32_t* bounds;  // fused pass: 3 x (kRfNR + 1) range bounds (iterations), rotated by pass % 3
    uint32_t* cost;    // fused pass: 2 x kRfNR range costs (40-ns units), by pass % 2
    uint64_t* clk;     // fused pass, diagnostics: kRfClk words per gate wave (abnn_debug_raw_wave_clock)
    uint4* pool;       // survivors {event, age bits | candidate << 31, w bits, dst}
    uint32_t ng, maxc, spike_cap, pool_chunks;
};

__host__ __device__ inline uint64_t raw_groups(uint64_t E) { return (E + kRawGroup - 1) / kRawGroup; }
__host__ __device__ inline uint32_t raw_maxc(uint64_t ng)
{
    const uint64_t per_wave = (ng + kRawWaves - 1) / kRawWaves;  // groups of one wave
    return (uint32_t)(per_wave * (kRawGroup / kRawChunk) + 1);
}
inline constexpr uint64_t al16(uint64_t x) { return (x + 15) & ~15ull; }

// The part of the workspace whose offsets do not depend on E: the header, the
// filter and the fused pass's state kept across passes (look-back words,
// bounds, costs, wave clocks).  A workspace reused with another n_syn or
// events keeps its look-back words where they were, so an epoch tag is never
// compared against a spike list or a bound of a differently sized pass
// (ADVICE r5).
inline constexpr uint64_t raw_state_bytes()
{
    return 128 + kRawFB * 8 + 8ull * kRawGateWGs + al16(4ull * 3 * (kRfNR + 1)) + 4ull * 2 * kRfNR +
           8ull * kRfClk * kRawWaves;
}

inline uint64_t raw_fixed_bytes(uint64_t E)
{
    const uint64_t ng = raw_groups(E);
    const uint64_t L = std::min<uint64_t>(E, kRawSpikeCap);
    return raw_state_bytes() + al16(4 * ng) * 2 + al16(4 * ((ng + kRawScanBlock - 1) / kRawScanBlock)) +
           al16(16 * ng) + al16(4ull * kRawWaves) + al16(8ull * kRawWaves) + al16(4ull * kRawWaves * raw_maxc(ng)) +
           al16(4 * L);
}

// Recommended pool: a partial chunk per wave plus 1/64 of the events (config
// 3 keeps ~0.3 % of them); a larger workspace only makes overflow rarer.
inline uint64_t raw_pool_chunks_recommended(uint64_t E)
{
    return E ? kRawWaves + (E / 64 + kRawChunk - 1) / kRawChunk + 64 : 0;
}

inline uint64_t raw_ws_bytes(uint64_t E)
{
    return raw_fixed_bytes(E) + raw_pool_chunks_recommended(E) * kRawChunk * 16;
}

inline RawWs raw_ws(void* base, uint64_t E, uint64_t bytes)
{
    char* p = static_cast<char*>(base);
    const uint64_t ng = raw_groups(E);
    RawWs w;
    w.ng = (uint32_t)ng;
    w.maxc = raw_maxc(ng);
    w.spike_cap = (uint32_t)std::min<uint64_t>(E, kRawSpikeCap);
    w.hdr = reinterpret_cast<RawHdr*>(p);
    p += 128;
    w.filter = reinterpret_cast<uint2*>(p);
    p += kRawFB * 8;
    w.lb = reinterpret_cast<unsigned long long*>(p);
    p += 8ull * kRawGateWGs;
    w.bounds = reinterpret_cast<uint32_t*>(p);
    p += al16(4ull * 3 * (kRfNR + 1));
    w.cost = reinterpret_cast<uint32_t*>(p);
    p += 4ull * 2 * kRfNR;
    w.clk = reinterpret_cast<uint64_t*>(p);
    p += 8ull * kRfClk * kRawWaves;
    w.gcand = reinterpret_cast<uint32_t*>(p);
    p += al16(4 * ng);
    w.gpre = reinterpret_cast<uint32_t*>(p);
    p += al16(4 * ng);
    w.btot = reinterpret_cast<uint32_t*>(p);
    p += al16(4 * ((ng + kRawScanBlock - 1) / kRawScanBlock));
    w.ginfo = reinterpret_cast<uint4*>(p);
    p += al16(16 * ng);
    w.wlim = reinterpret_cast<uint32_t*>(p);
    p += al16(4ull * kRawWaves);
    w.wstat = reinterpret_cast<uint2*>(p);
    p += al16(8ull * kRawWaves);
    w.ctab = reinterpret_cast<uint32_t*>(p);
    p += al16(4ull * kRawWaves * w.maxc);
    w.spikes = reinterpret_cast<uint32_t*>(p);
    p += al16(4ull * w.spike_cap);
    w.pool = reinterpret_cast<uint4*>(p);
    const uint64_t fixed = (uint64_t)(p - static_cast<char*>(base));
    w.pool_chunks = (uint32_t)std::min<uint64_t>((bytes - fixed) / (kRawChunk * 16), 0xFFFFFFFEu);
    return w;
}

// visited events: min(roundup(events, 256), n_syn) (brain.cpp:116-118, brain.metal:60-61)
inline uint64_t raw_events(uint32_t n_syn, uint32_t events)
{
    const uint64_t grid = ((uint64_t)events + 255u) / 256u * 256u;
    return grid < n_syn ? grid : n_syn;
}

// The filter block of word j (neurons 32 j .. 32 j + 31): g(j) = (j ^ t) mod
// FB, t = 0x9E5 (j >> 13); its high half holds the word rotated left by t mod
// 32 (kernels.hip filter_set).
__device__ __forceinline__ uint32_t raw_t(uint32_t j) { return __umul24(j >> kRawFLg, 0x9E5u); }

// One 8-B LDS read per event; no false negatives.  Any src (tombstones
// included) reads inside the filter.
__device__ __forceinline__ bool raw_filter_pass(const uint2* s_fb, uint32_t src)
{
    const uint32_t j = src >> 5, t = raw_t(j);
    const uint2 f = s_fb[(j ^ t) & (kRawFB - 1)];
    return (__builtin_amdgcn_ubfe(f.x, src, 1) & __builtin_amdgcn_ubfe(f.y, src + t, 1)) != 0u;
}

// ---------------------------------------------------------------------------
// k_raw_filter: workgroup b builds filter blocks [4 b, 4 b + 4).  The words
// of block g are j = h << 13 | ((g ^ t(h)) & 8191), h = 0 .. H-1 (t depends on
// h only); half a wave reads one word's 32 lastF values (128 B), so a wave
// instruction covers two words and the ballot returns both; a wave issues
// all its reads at once (config 3: H = 20, 20 words per wave, one round
// trip).  Every lastF value is read once by the whole grid.
constexpr uint32_t kRawFilterBlocks = 4;  // filter blocks per workgroup
__global__ __launch_bounds__(256) void k_raw_filter(const uint32_t* lastF, const uint32_t* clock, uint32_t n_nrn,
                                                    KernelParams kp, RawWs ws)
{
    constexpr uint32_t NB = kRawFilterBlocks, kU = 12;  // word pairs in flight per wave
    __shared__ uint32_t s_lo[NB], s_hi[NB];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (threadIdx.x < NB) {
        s_lo[threadIdx.x] = 0u;
        s_hi[threadIdx.x] = 0u;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // this pass's counters (the gate and the scan set them)
        ws.hdr->chunks = 0u;
        ws.hdr->t0 = 0u;
        ws.hdr->ovf = 0u;
        ws.hdr->wdone = 0u;
        ws.hdr->g1 = 0ull;
        ws.hdr->g2 = 0ull;
        if (ws.hdr->init != kRawInit) {  // first use of this workspace: err is sticky from here on, and the
            ws.hdr->err = 0u;            // fused pass's state starts over
            ws.hdr->init = kRawInit;
            ws.hdr->pass = 0u;
            ws.hdr->pvalid = 0u;
            for (uint32_t i = 0; i < kRawGateWGs; ++i) ws.lb[i] = 0ull;
        }
    }
    __syncthreads();
    const uint32_t now = *clock;
    const uint32_t words = (n_nrn + 31u) / 32u, H = (words + kRawFB - 1) >> kRawFLg;
    const uint32_t tasks = NB * H;  // (block, h) pairs of this workgroup
    for (uint32_t x0 = wv * 2u * kU; x0 < tasks; x0 += 4u * 2u * kU) {  // wave-uniform
        uint32_t v[kU];
        uint32_t jw[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t x = x0 + 2u * u + (lane >> 5);  // this half-wave's task
            const uint32_t gl = x % NB, h = x / NB, g = blockIdx.x * NB + gl;
            const uint32_t t = __umul24(h, 0x9E5u);
            const uint32_t j = h << kRawFLg | ((g ^ t) & (kRawFB - 1));
            const uint64_t n = (uint64_t)j * 32u + (lane & 31u);
            const bool ok = x < tasks && n < n_nrn;
            jw[u] = x < tasks ? j : kRawNone;
            v[u] = ok ? lastF[n] : now;
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t x = x0 + 2u * u + (lane >> 5);
            const uint64_t n = (uint64_t)(jw[u] == kRawNone ? 0u : jw[u]) * 32u + (lane & 31u);
            const bool bit = jw[u] != kRawNone && n < n_nrn && (now - v[u]) <= kp.window_pre;  // brain.metal:73-77 (u32)
            const uint64_t m = __ballot(bit);
            if ((lane & 31u) == 0 && jw[u] != kRawNone) {
                const uint32_t bits = (uint32_t)(m >> (lane & 32u));
                if (bits) {
                    const uint32_t gl = x % NB, r = raw_t(jw[u]) & 31u;
                    atomicOr(&s_lo[gl], bits);
                    atomicOr(&s_hi[gl], (bits << r) | (bits >> ((32u - r) & 31u)));
                }
            }
        }
    }
    __syncthreads();
    if (threadIdx.x < NB) ws.filter[blockIdx.x * NB + threadIdx.x] = make_uint2(s_lo[threadIdx.x], s_hi[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// k_raw_gate (see the file header).  Wave v = wid * gridDim + blockIdx sweeps
// groups v, v + W, v + 2W, ... (W = all gate waves): the dense stretches of a
// graph spread over the CUs.  Its survivors form one sequence in group order,
// stored 256 entries per pool chunk (ctab: the chunk of every 256 entries);
// when the pool runs out the rest of the wave's sequence is not stored
// (wlim), and k_raw_apply recomputes those groups.
__global__ __launch_bounds__(kRawBlock) void k_raw_gate(const uint4* __restrict__ syn, const uint32_t* lastF,
                                                         const uint32_t* clock, uint32_t n_nrn, uint32_t E,
                                                         KernelParams kp, RawWs ws)
{
    constexpr uint32_t NW = kRawBlock / 64;
    __shared__ uint2 s_fb[kRawFB];
    __shared__ uint4 s_st[NW][kRawStage];  // staged hits {event, src, dst, w}
    __shared__ uint4 s_og[NW][kRawOpen];   // pending groups {group, first stage entry, survivors, candidates}
    __shared__ uint32_t s_oseq[NW][kRawOpen];  // ... their first survivor's place in the wave's sequence
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = wave_uniform(tid >> 6);
    // the filter global -> LDS (LDS-DMA) before the first records are requested
#pragma unroll
    for (uint32_t c = 0; c < kRawFB / 2 / kRawBlock; ++c)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(ws.filter) + c * kRawBlock + tid,
                                         reinterpret_cast<uint4*>(s_fb) + c * kRawBlock + (tid & ~63u), 16, 0, 0);
    const uint32_t now = sload(clock);  // per-TG clock cache (brain.metal:63-68); C1: the pass-start value
    const uint32_t v = wid * gridDim.x + blockIdx.x, W = gridDim.x * NW;
    const uint32_t NG = ws.ng;
    uint4* st = s_st[wid];
    uint4 R[kRawD][kRawK];
    // iteration d of group g: events g * 1024 + d * 256 + k * 64 + lane;
    // past E a tombstone-like record that never passes
    auto issue = [&](uint32_t d, uint32_t g) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t k = 0; k < kRawK; ++k) {
            const uint64_t t = (uint64_t)g * kRawGroup + d * kRawIt + k * 64 + lane;
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            u32x4 x = {kRawNone, kRawNone, 0u, 0u};
            if (t < E) x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(syn) + t);
            R[d][k] = make_uint4(x.x, x.y, x.z, x.w);
        }
    };
    if (v < NG) {
#pragma unroll
        for (uint32_t d = 0; d < kRawD; ++d) issue(d, v);
    }
    __syncthreads();  // the filter in LDS (every wave's LDS-DMA done: vmcnt is waited by the barrier's release)
    uint32_t seq = 0;           // survivors of this wave so far (its sequence)
    uint32_t have = 0;          // chunks held
    uint32_t cur = kRawNone, prev = kRawNone;  // the last two chunks' pool ids
    uint32_t lim = kRawNone;    // sequence entries stored (kRawNone: all so far)
    uint32_t n_g1 = 0;          // pre-gated events of this wave (diagnostics)
    const uint32_t window = kp.window_pre, refr = kp.refractory;
    // The staged hits go through the gates only when the stage fills or
    // kRawOpen groups with hits are pending (round 3 did it at the end of every
    // group: its lastF round trip was issued behind the next group's record
    // loads, and vmcnt retires in order, so each wave drained its whole
    // pipeline once per 1024 events -- 13 % of the gate's time).  Per pending
    // group (in this wave's LDS): {group, first stage entry, survivors so far,
    // candidates so far} and its first survivor's place in the sequence.
    uint4* og = s_og[wid];
    uint32_t* oseq = s_oseq[wid];
    uint32_t nopen = 0;   // pending groups (the last may be the current one)
    bool cur_open = false;  // the current group is the last pending one
    uint32_t pend = 0;
    // ginfo of a finished group: where its survivors are
    auto write_ginfo = [&](uint32_t g, uint32_t S, uint32_t C, uint32_t seq0) {
        if (lane == 0) {
            uint32_t ia = kRawNone, ib = kRawNone;
            if (S) {
                const uint32_t c0 = seq0 / kRawChunk;
                if (lim != kRawNone && seq0 + S > lim) ia = kRawRedo;
                else if (c0 + 1 == have) ia = cur;  // every survivor in the last chunk
                else if (c0 + 2 == have) { ia = prev; ib = cur; }
                else ia = kRawCtab;
            }
            ws.gcand[g] = C;
            ws.ginfo[g] = make_uint4(S, seq0, ia, ib);
        }
    };
    // every staged hit through the gates; survivors appended to the sequence
    // and counted to their groups; the finished groups' ginfo written (keep:
    // the current group stays pending, its next hits staged from entry 0)
    auto flush = [&](bool keep_current) {
        constexpr uint32_t RR = kRawStage / 64;
        uint4 e[RR];
        uint32_t a[RR], b[RR];
#pragma unroll
        for (uint32_t r = 0; r < RR; ++r) {
            const uint32_t q = r * 64 + lane;
            e[r] = q < pend ? st[q] : make_uint4(0u, kRawNone, kRawNone, 0u);
            const bool ok = e[r].y < n_nrn && e[r].z < n_nrn;
            a[r] = ok ? lastF[e[r].y] : now;  // brain.metal:73 (exact, for the filter's hits)
            b[r] = ok ? lastF[e[r].z] : now;  // brain.metal:79, in the same round trip
        }
        uint64_t m2[RR], mc[RR];
        uint32_t n = 0;
#pragma unroll
        for (uint32_t r = 0; r < RR; ++r) {
            const bool ok = e[r].y < n_nrn && e[r].z < n_nrn;
            const bool g1 = ok && now - a[r] <= window;          // brain.metal:73-77
            const bool g2 = g1 && now - b[r] > refr;             // brain.metal:79-83
            const bool cand = g2 && spike_candidate(kp, __uint_as_float(e[r].w), e[r].x, now);  // brain.metal:91-92
            m2[r] = __ballot(g2);
            mc[r] = __ballot(cand);
            n_g1 += (uint32_t)__popcll(__ballot(g1));
            if (g2 && e[r].x == 0u) ws.hdr->t0 = 1u;             // event 0 reached the budget test (brain.metal:110)
            e[r] = make_uint4(e[r].x, __float_as_uint((float)(now - b[r])) | (cand ? 0x80000000u : 0u), e[r].w,
                              e[r].z);
            n += (uint32_t)__popcll(m2[r]);
        }
        const uint32_t seq_before = seq;
        if (n) {
            // chunks for entries [seq, seq + n)
            if (lim == kRawNone) {
                while (have * kRawChunk < seq + n) {  // wave-uniform
                    uint32_t id = 0;
                    if (lane == 0) id = atomicAdd(&ws.hdr->chunks, 1u);
                    id = wave_uniform(id);
                    if (id >= ws.pool_chunks) {  // the pool is spent: the rest of the sequence is not stored
                        lim = have * kRawChunk;
                        if (lane == 0) __hip_atomic_store(&ws.hdr->ovf, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // k_raw_apply will recompute: stamps deferred
                        break;
                    }
                    if (lane == 0) ws.ctab[(uint64_t)v * ws.maxc + have] = id;
                    prev = cur;
                    cur = id;
                    ++have;
                }
            }
            uint32_t o = seq;
#pragma unroll
            for (uint32_t r = 0; r < RR; ++r) {
                const uint32_t x = o + mbcnt64(m2[r]);
                if (((m2[r] >> lane) & 1u) && (lim == kRawNone || x < lim)) {
                    const uint32_t c = x / kRawChunk;
                    const uint32_t id = c + 1 == have ? cur
                                      : c + 2 == have ? prev
                                                      : ws.ctab[(uint64_t)v * ws.maxc + c];
                    ws.pool[(uint64_t)id * kRawChunk + (x % kRawChunk)] = e[r];
                }
                o += (uint32_t)__popcll(m2[r]);
            }
            seq += n;
        }
        // the pending groups' shares (stage entries [st0_j, st0_j+1) are group j's)
        auto range_mask = [](uint32_t lo, uint32_t hi, uint32_t r) -> uint64_t {  // lanes q in [lo, hi) of round r
            const uint32_t b0 = r * 64;
            const uint32_t l = lo > b0 ? (lo - b0 < 64 ? lo - b0 : 64) : 0, h = hi > b0 ? (hi - b0 < 64 ? hi - b0 : 64) : 0;
            const uint64_t mh = h >= 64 ? ~0ull : ((1ull << h) - 1), ml = l >= 64 ? ~0ull : ((1ull << l) - 1);
            return mh & ~ml;
        };
        uint32_t kept = 0;
        for (uint32_t j = 0; j < nopen; ++j) {  // wave-uniform
            uint4 oj = og[j];  // {group, first entry, survivors, candidates}
            const uint32_t hi = j + 1 < nopen ? og[j + 1].y : pend;
            uint32_t sj = 0, cj = 0, before = 0;
#pragma unroll
            for (uint32_t r = 0; r < RR; ++r) {
                const uint64_t m = range_mask(oj.y, hi, r);
                sj += (uint32_t)__popcll(m2[r] & m);
                cj += (uint32_t)__popcll(mc[r] & m);
                before += (uint32_t)__popcll(m2[r] & range_mask(0, oj.y, r));
            }
            if (oj.z == 0 && sj) oseq[j] = seq_before + before;  // its first survivor's place
            oj.z += sj;
            oj.w += cj;
            if (keep_current && cur_open && j + 1 == nopen) {  // the current group stays pending
                og[0] = make_uint4(oj.x, 0u, oj.z, oj.w);
                oseq[0] = oseq[j];
                kept = 1;
            } else {
                write_ginfo(oj.x, oj.z, oj.w, oj.z ? oseq[j] : seq);
            }
        }
        nopen = kept;
        cur_open = kept != 0;
        pend = 0;
    };
    for (uint32_t g = v; g < NG; g += W) {  // wave-uniform
#pragma unroll
        for (uint32_t d = 0; d < kRawD; ++d) {
            uint32_t src[kRawK];
            uint4 rc[kRawK];
#pragma unroll
            for (uint32_t k = 0; k < kRawK; ++k) rc[k] = R[d][k];
            // this buffer's next group in flight first
            if (g + W < NG) issue(d, g + W);
            const uint32_t rel = g * kRawGroup + d * kRawIt;
#pragma unroll
            for (uint32_t k = 0; k < kRawK; ++k) src[k] = rc[k].x;
#pragma unroll
            for (uint32_t k = 0; k < kRawK; ++k) {
                const bool h = raw_filter_pass(s_fb, src[k]);
                const uint64_t bm = __ballot(h);
                if (bm == 0) continue;  // wave-uniform
                if (!cur_open) {  // the group's first staged hit: it becomes pending
                    if (lane == 0) {
                        og[nopen] = make_uint4(g, pend, 0u, 0u);
                        oseq[nopen] = 0u;
                    }
                    ++nopen;
                    cur_open = true;
                }
                if (h) st[pend + mbcnt64(bm)] = make_uint4(rel + k * 64 + lane, rc[k].x, rc[k].y, rc[k].z);
                pend += (uint32_t)__popcll(bm);
                if (pend > kRawStage - 64) flush(true);
            }
        }
        // the group is done: without a pending share, its ginfo now (its
        // survivors, if a flush inside it kept any, are all counted)
        if (cur_open && nopen == 1 && pend == 0) {  // (a flush inside it took every hit: og[0] is it)
            const uint4 oj = og[0];
            write_ginfo(oj.x, oj.z, oj.w, oj.z ? oseq[0] : seq);
            nopen = 0;
        } else if (!cur_open) {
            write_ginfo(g, 0u, 0u, seq);
        }
        cur_open = false;
        if (nopen >= kRawOpen) flush(false);
    }
    if (nopen) flush(false);
    if (lane == 0) {
        ws.wlim[v] = lim;
        ws.wstat[v] = make_uint2(n_g1, seq);
    }
}

// The ordered budget in two launches.  k_raw_scan_local: workgroup b scans
// groups [4096 b, 4096 b + 4096) -- one coalesced 16-B load per thread --
// into gpre (exclusive, within the block) and the block's total (btot[b]).
__global__ __launch_bounds__(kRawScanThreads) void k_raw_scan_local(RawWs ws)
{
    __shared__ uint32_t s_wave[kRawScanThreads / 64];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t g0 = blockIdx.x * kRawScanBlock + 4 * threadIdx.x, NG = ws.ng;
    uint4 c = make_uint4(0u, 0u, 0u, 0u);
    if (g0 + 3 < NG) {
        c = *reinterpret_cast<const uint4*>(ws.gcand + g0);  // 16-B aligned: g0 % 4 == 0, gcand 16-B aligned
    } else {
        if (g0 < NG) c.x = ws.gcand[g0];
        if (g0 + 1 < NG) c.y = ws.gcand[g0 + 1];
        if (g0 + 2 < NG) c.z = ws.gcand[g0 + 2];
    }
    const uint32_t v = c.x + c.y + c.z + c.w;  // a group holds <= 1024 candidates: no overflow in a block
    const uint32_t inc = wave_incl_scan(v);
    if (lane == 63) s_wave[wv] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < kRawScanThreads / 64; ++w) {
        before += w < wv ? s_wave[w] : 0u;
        total += s_wave[w];
    }
    const uint32_t e = before + inc - v;
    if (g0 + 3 < NG) {
        *reinterpret_cast<uint4*>(ws.gpre + g0) = make_uint4(e, e + c.x, e + c.x + c.y, e + c.x + c.y + c.z);
    } else {
        if (g0 < NG) ws.gpre[g0] = e;
        if (g0 + 1 < NG) ws.gpre[g0 + 1] = e + c.x;
        if (g0 + 2 < NG) ws.gpre[g0 + 2] = e + c.x + c.y;
    }
    if (threadIdx.x == 0) ws.btot[blockIdx.x] = total;
}

// k_raw_scan: one workgroup.  The blocks' totals become capped exclusive
// prefixes (btot), the cut (the groups below the budget, [0, gcut): the
// prefix is monotone) is found inside the block where the budget runs out,
// then the pass end on the scalars, which nothing later in the pass reads:
// *budget left, rBar (brain.metal:110-113), one clock tick (brain.metal:129).
// A group's capped budget position is min(btot[g / 4096] + gpre[g], budget).
__global__ __launch_bounds__(kRawScanThreads) void k_raw_scan(RawWs ws, uint32_t E, uint32_t* clock, uint32_t* budget,
                                                              const float* reward, float* rbar, KernelParams kp)
{
    __shared__ uint32_t s_wave[kRawScanThreads / 64], s_cut[kRawScanThreads / 64];
    __shared__ uint32_t s_blk[2];  // the block where the budget runs out, its offset
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t b0 = *budget, NG = ws.ng, NB = (NG + kRawScanBlock - 1) / kRawScanBlock;
    __shared__ unsigned long long s_g[2];
    if (threadIdx.x == 0) {
        s_blk[0] = NB;
        s_blk[1] = 0u;
        s_g[0] = s_g[1] = 0ull;
    }
    // the gate waves' statistics (a wave past the last group wrote zeros),
    // loaded beside the block totals (one round trip)
    uint2 wst[kRawWaves / kRawScanThreads];
#pragma unroll
    for (uint32_t i = 0; i < kRawWaves / kRawScanThreads; ++i) wst[i] = ws.wstat[i * kRawScanThreads + threadIdx.x];
    // blocks: NB <= 1024 at any u32 record count
    const uint32_t bt = threadIdx.x < NB ? ws.btot[threadIdx.x] : 0u;
    const uint64_t bt64 = bt;
    uint32_t inc = wave_incl_scan(bt);  // per-block totals <= 4096 x 1024: u32 prefix is exact below 2^32 events
    if (lane == 63) s_wave[wv] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (uint32_t w = 0; w < kRawScanThreads / 64; ++w) {
        before += w < wv ? s_wave[w] : 0u;
        total += s_wave[w];
    }
    const uint32_t ex = before + inc - (uint32_t)bt64;
    if (threadIdx.x < NB) {
        ws.btot[threadIdx.x] = ex < b0 ? ex : b0;
        if (ex < b0 && ex + bt >= b0) {  // the budget runs out inside this block
            s_blk[0] = threadIdx.x;
            s_blk[1] = ex;
        }
    }
    __syncthreads();
    // gcut: the groups with a budget position below b0
    uint32_t gcut;
    const uint32_t cb = s_blk[0];
    if (b0 == 0) {
        gcut = 0;   // no budget: no update (C1)
    } else if (cb >= NB) {
        gcut = NG;  // the budget never runs out
    } else {
        uint32_t below = 0;
        for (uint32_t q = threadIdx.x; q < kRawScanBlock; q += kRawScanThreads) {
            const uint32_t g = cb * kRawScanBlock + q;
            below += (g < NG && s_blk[1] + ws.gpre[g] < b0) ? 1u : 0u;
        }
        const uint32_t bw = wave_incl_scan(below);
        if (lane == 63) s_cut[wv] = bw;
        __syncthreads();
        uint32_t nb = 0;
        for (uint32_t w = 0; w < kRawScanThreads / 64; ++w) nb += s_cut[w];
        gcut = cb * kRawScanBlock + nb;
    }
    uint64_t a1 = 0, a2 = 0;
#pragma unroll
    for (uint32_t i = 0; i < kRawWaves / kRawScanThreads; ++i) {
        a1 += wst[i].x;
        a2 += wst[i].y;
    }
    if (a1) atomicAdd(&s_g[0], (unsigned long long)a1);
    if (a2) atomicAdd(&s_g[1], (unsigned long long)a2);
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t now = *clock;
        const float R = *reward, rb = *rbar;
        const uint32_t t0 = E > 0 ? ws.hdr->t0 : 0u;
        const uint32_t nc = total < b0 ? total : b0;
        RawHdr* h = ws.hdr;
        h->now = now;
        h->budget0 = b0;
        h->ncand = nc;
        h->R = R;
        h->rb = rb;
        h->gcut = gcut;
        // no group recomputed (nothing overflowed the pool): k_raw_apply reads
        // no lastF, so it stamps the spikes itself; else they wait for
        // k_raw_stamp, unless this pass's spikes (nc <= b0) exceed the list
        h->direct = (nc > ws.spike_cap || h->ovf == 0u) ? 1u : 0u;
        h->g1 = ws.ng ? s_g[0] : 0ull;
        h->g2 = ws.ng ? s_g[1] : 0ull;
        *budget = b0 - nc;                                               // brain.metal:95-98 (C1: no wrap)
        if (t0 && b0 > 0) *rbar = rb + kp.alpha_rbar * (R - rb);         // brain.metal:110-113
        if (E > 0) *clock = now + kp.clock_inc;                          // brain.metal:129
    }
}

// One survivor below the budget's cut at budget position pre (< budget0):
// the weight update (brain.metal:101-122, the record's w only) and, for a
// spike, its budget slot.
__device__ __forceinline__ void raw_apply_one(uint4* syn, uint32_t* lastF, const RawWs& ws, const RawHdr& h,
                                              const KernelParams& kp, const uint4& e, bool cand, uint32_t pre)
{
    const float w = updated_weight(kp, __uint_as_float(e.z), cand, h.R, h.rb, __uint_as_float(e.y & 0x7FFFFFFFu));
    reinterpret_cast<float*>(syn + e.x)[2] = w;  // brain.metal:122 (src, dst, pad unchanged)
    if (cand) {
        if (h.direct) lastF[e.w] = h.now;  // brain.metal:125-126 (k_raw_scan: no lastF read is left)
        else ws.spikes[pre] = e.w;
    }
}

// k_raw_apply: every wave takes kRawApplyGroups groups below the cut at a
// time (strided over the waves): their {survivors, place} and budget positions in one round
// trip (a lane per group), the survivors of all of them in a second (a group
// keeps ~3 at config 3, the dense input->output groups up to 1024), then the
// walk in event order.  The groups below the cut are ~25 % of all at config
// 3, so per-group round trips would be a chain of ~9 per wave.
constexpr uint32_t kRawApplyGroups = 16;

__device__ __forceinline__ uint4 raw_pool_entry(const RawWs& ws, const uint4& gi, uint32_t v, uint32_t q)
{
    const uint32_t x = gi.y + q, c = x / kRawChunk;
    const uint32_t id = gi.z == kRawCtab ? ws.ctab[(uint64_t)v * ws.maxc + c]
                                         : (c == gi.y / kRawChunk ? gi.z : gi.w);
    return ws.pool[(uint64_t)id * kRawChunk + x % kRawChunk];
}

// One group below the cut with more than 64 survivors (a dense stretch), or
// whose survivors did not fit the pool (recomputed from its records with the
// pass-start lastF: the stamps then wait for k_raw_stamp).
__device__ __forceinline__ void raw_apply_group(uint4* syn, uint32_t* lastF, uint32_t n_nrn, uint32_t E,
                                             const KernelParams& kp, const RawWs& ws, const RawHdr& h, uint32_t g,
                                             uint4 gi, uint32_t P)
{
    const uint32_t lane = threadIdx.x & 63, S = gi.x, v = g % kRawWaves;
    if (gi.z != kRawRedo) {  // stored: the wave's sequence [s0, s0 + S), 4 x 64 in flight
        constexpr uint32_t RW = 4;
        for (uint32_t b0 = 0; b0 < S && P < h.budget0; b0 += RW * 64) {  // wave-uniform
            uint4 x[RW];
#pragma unroll
            for (uint32_t j = 0; j < RW; ++j)
                x[j] = b0 + j * 64 + lane < S ? raw_pool_entry(ws, gi, v, b0 + j * 64 + lane) : make_uint4(0u, 0u, 0u, 0u);
#pragma unroll
            for (uint32_t j = 0; j < RW; ++j) {
                if (b0 + j * 64 >= S || P >= h.budget0) break;  // wave-uniform
                const bool ok = b0 + j * 64 + lane < S;
                const bool cand = ok && (x[j].y >> 31);
                const uint64_t bc = __ballot(cand);
                const uint32_t pre = P + mbcnt64(bc);
                if (ok && pre < h.budget0) raw_apply_one(syn, lastF, ws, h, kp, x[j], cand, pre);
                P += (uint32_t)__popcll(bc);
            }
        }
        return;
    }
    if (h.direct && lane == 0) ws.hdr->err = 1u;  // (direct here only with a budget beyond the list)
    constexpr uint32_t RH = kRawGroup / 64 / 2;  // two halves: records and their lastF in flight
    for (uint32_t h0 = 0; h0 < 2 * RH && P < h.budget0; h0 += RH) {  // wave-uniform
        uint4 rc[RH];
#pragma unroll
        for (uint32_t j = 0; j < RH; ++j) {
            const uint64_t t = (uint64_t)g * kRawGroup + (h0 + j) * 64 + lane;
            rc[j] = t < E ? syn[t] : make_uint4(kRawNone, kRawNone, 0u, 0u);
        }
        uint32_t la[RH], lb[RH];
#pragma unroll
        for (uint32_t j = 0; j < RH; ++j) {
            const bool ok = rc[j].x < n_nrn && rc[j].y < n_nrn;
            la[j] = ok ? lastF[rc[j].x] : h.now;
            lb[j] = ok ? lastF[rc[j].y] : h.now;
        }
#pragma unroll
        for (uint32_t j = 0; j < RH; ++j) {
            if (P >= h.budget0) break;  // wave-uniform
            const uint64_t t = (uint64_t)g * kRawGroup + (h0 + j) * 64 + lane;
            const bool ok = rc[j].x < n_nrn && rc[j].y < n_nrn;
            const bool g2 = ok && h.now - la[j] <= kp.window_pre && h.now - lb[j] > kp.refractory;  // brain.metal:73-83
            const bool cand = g2 && spike_candidate(kp, __uint_as_float(rc[j].z), t, h.now);        // brain.metal:91-92
            const uint64_t bc = __ballot(cand);
            const uint32_t pre = P + mbcnt64(bc);
            if (g2 && pre < h.budget0)
                raw_apply_one(syn, lastF, ws, h, kp,
                              make_uint4((uint32_t)t, __float_as_uint((float)(h.now - lb[j])), rc[j].z, rc[j].y), cand,
                              pre);
            P += (uint32_t)__popcll(bc);
        }
    }
}

__global__ __launch_bounds__(256) void k_raw_apply(uint4* syn, uint32_t* lastF, uint32_t n_nrn, uint32_t E,
                                                   KernelParams kp, RawWs ws)
{
    constexpr uint32_t GA = kRawApplyGroups;
    const uint32_t lane = threadIdx.x & 63;
    const RawHdr h = *ws.hdr;  // pass-start scalars (k_raw_scan)
    const uint32_t nw = gridDim.x * 4u;
    // slot i of round r of wave w: group (r GA + i) nw + w -- strided, so the
    // dense groups at the start of the sweep spread over many waves
    const uint32_t w = blockIdx.x * 4u + (threadIdx.x >> 6);
    for (uint32_t r0 = 0; r0 * nw < h.gcut; r0 += GA) {  // wave-uniform
        const uint32_t g0 = r0 * nw + w;  // the round's first group; slot i is g0 + i nw
        // lane i < GA: slot i
        const uint32_t gl = g0 + (lane < GA ? lane : 0u) * nw;
        const bool mine = lane < GA && gl < h.gcut;
        const uint4 gi_l = mine ? ws.ginfo[gl] : make_uint4(0u, 0u, 0u, 0u);
        const uint32_t pre_l = mine ? ws.btot[gl / kRawScanBlock] + ws.gpre[gl] : h.budget0;
        // survivors of every group with at most 64 (one per lane), all in flight
        uint4 e[GA];
#pragma unroll
        for (uint32_t i = 0; i < GA; ++i) {
            const uint32_t S = (uint32_t)__builtin_amdgcn_readlane((int)gi_l.x, (int)i);
            const uint4 gi = make_uint4(S, (uint32_t)__builtin_amdgcn_readlane((int)gi_l.y, (int)i),
                                        (uint32_t)__builtin_amdgcn_readlane((int)gi_l.z, (int)i),
                                        (uint32_t)__builtin_amdgcn_readlane((int)gi_l.w, (int)i));
            const bool direct_load = S <= 64 && gi.z != kRawRedo;
            e[i] = direct_load && lane < S ? raw_pool_entry(ws, gi, (g0 + i * nw) % kRawWaves, lane) : make_uint4(0u, 0u, 0u, 0u);
        }
        uint32_t slow = 0;  // groups for raw_apply_group (wave-uniform bit mask)
#pragma unroll
        for (uint32_t i = 0; i < GA; ++i) {
            const uint32_t g = g0 + i * nw;
            const uint32_t S = (uint32_t)__builtin_amdgcn_readlane((int)gi_l.x, (int)i);
            const uint32_t gz = (uint32_t)__builtin_amdgcn_readlane((int)gi_l.z, (int)i);
            if (g >= h.gcut || S == 0) continue;  // wave-uniform
            if (S > 64 || gz == kRawRedo) {
                slow |= 1u << i;
                continue;
            }
            // the common case: prefetched above
            const uint32_t P = (uint32_t)__builtin_amdgcn_readlane((int)pre_l, (int)i);  // < budget0: g < gcut
            const bool ok = lane < S;
            const bool cand = ok && (e[i].y >> 31);
            const uint64_t bc = __ballot(cand);
            const uint32_t pre = P + mbcnt64(bc);  // spike candidates before this event
            if (ok && pre < h.budget0) raw_apply_one(syn, lastF, ws, h, kp, e[i], cand, pre);
        }
        // groups are independent (each one's budget position is known), so
        // the rare big or recomputed ones may come last
        while (slow) {  // wave-uniform
            const uint32_t i = (uint32_t)__builtin_ctz(slow);
            slow &= slow - 1u;
            const uint4 gi = make_uint4((uint32_t)__builtin_amdgcn_readlane((int)gi_l.x, (int)i),
                                        (uint32_t)__builtin_amdgcn_readlane((int)gi_l.y, (int)i),
                                        (uint32_t)__builtin_amdgcn_readlane((int)gi_l.z, (int)i),
                                        (uint32_t)__builtin_amdgcn_readlane((int)gi_l.w, (int)i));
            raw_apply_group(syn, lastF, n_nrn, E, kp, ws, h, g0 + i * nw, gi,
                            (uint32_t)__builtin_amdgcn_readlane((int)pre_l, (int)i));
        }
    }
}

__global__ __launch_bounds__(1024) void k_raw_stamp(uint32_t* lastF, RawWs ws)
{
    const RawHdr* h = ws.hdr;
    if (h->direct) return;
    const uint32_t now = h->now, n = h->ncand;
    for (uint32_t i = threadIdx.x; i < n; i += 1024) lastF[ws.spikes[i]] = now;  // brain.metal:125-126
}

// ---------------------------------------------------------------------------
// k_raw_pass: the fused reference-layout pass (round 5).  After k_raw_filter,
// ONE launch does the rest of the pass with the handle path's design
// (kernels.hip k_gate<..., kFused>): persistent workgroups (one per CU), one
// contiguous range of 256-event iterations per WORKGROUP -- an adaptive
// partition kept in the workspace (each pass moves the next pass's bounds
// towards equal measured costs; the dense input->output stretch gets a short
// range) -- split into up to kRfMaxG groups that the workgroup's 16 waves
// claim in order from an LDS counter.  Per-wave ranges (the first version)
// left 80 us between a workgroup's first and last wave: the CU's oldest waves
// issue first, so the waves of one workgroup stream at rates 0.39-0.50
// iterations/us by age, which no cost-driven partition kept up with; claimed
// groups even that out.  Each wave streams its groups kRawD iterations ahead;
// the LDS filter test per event; hits staged in LDS in event order and,
// every ~192, through the gates in ONE round trip (lastF[src] and
// lastF[dst]: both come with the record); the survivors appended to the
// wave's sequence in the bounded pool (chunks of 255 entries + the next
// chunk's id), each group's candidates and {first place, wave candidates
// before it} tallied in LDS.  Then the workgroup's decoupled look-back
// (epoch-tagged words in the workspace, never reset) and an LDS scan over its
// groups give every survivor its budget position, every wave walks its own
// sequence (the weight update into the record's w, brain.metal:101-122;
// spikes into the workgroup's list), and once every look-back word is
// published -- every lastF read of the pass done -- the spikes are stamped
// (brain.metal:125-126) and workgroup 0 ends the pass (*budget, rBar, clock;
// brain.metal:95-98, 110-113, 129).  Round 4 ran five launches (gate, two
// scans, apply, stamp) with 71 us per pass outside the gate.
constexpr uint32_t kRfSpkLds = 2560;     // spikes of a workgroup kept in LDS (budgets up to kMaxSpikes, brain.h:18)
constexpr uint32_t kRfSpinLimit = 1u << 22;

struct RfLds {
    uint32_t next;   // the next group to claim
    uint32_t tmax;   // the workgroup's longest stream (40-ns units)
    uint32_t g1, g2; // the workgroup's pre-gated and surviving events
    uint32_t done;   // waves through their tail
    uint32_t excl;   // candidates of every lower workgroup (capped)
    uint32_t cwg;    // the workgroup's candidates
    uint32_t tot;    // the pass's candidates (capped; stamping workgroups)
};

// One wave polls the look-back words of workgroups [0, n) (64 per lane-round,
// up to 4 rounds: 256 workgroups) until all carry `tag` or, with
// stop_at_budget, the published ones reach the budget; their capped sum.
__device__ uint32_t rf_poll(const RawWs& ws, uint32_t n, uint32_t tag, uint32_t budget, bool stop_at_budget,
                            uint64_t pub)
{
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t spins = 0;; ++spins) {  // wave-uniform
        uint64_t raw[kRawGateWGs / 64];
#pragma unroll
        for (uint32_t i = 0; i < kRawGateWGs / 64; ++i) {
            const uint32_t q = i * 64 + lane;
            raw[i] = q < n ? __hip_atomic_load(ws.lb + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        }
        if (pub && spins == 0 && lane == 0)  // this workgroup's word, behind the first sweep's loads
            __hip_atomic_store(ws.lb + blockIdx.x, (unsigned long long)pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t sum = 0;
        bool ok = true;
#pragma unroll
        for (uint32_t i = 0; i < kRawGateWGs / 64; ++i) {
            const uint32_t q = i * 64 + lane;
            if (q < n) {
                const bool mine = (uint32_t)(raw[i] >> 32) == tag;
                sum += mine ? (raw[i] & 0x3FFFFFFFull) : 0ull;
                ok = ok && mine;
            }
        }
        uint64_t tot = sum;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o, 64);
        if (__ballot(!ok) == 0 || (stop_at_budget && tot >= budget)) return (uint32_t)(tot < budget ? tot : budget);
        if (spins >= kRfSpinLimit) {  // never hang the GPU: report (abnn_traversal_workspace_error) and go on
            if (lane == 0)  // (every workgroup is resident: never expected)
                __hip_atomic_store(&ws.hdr->err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return budget;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// The next pass's bound k from this pass's bound `from`, the previous pass's
// costs (exclusive prefix cc over its bounds rb, NR ranges, total T): a
// quarter of the way (or, gain 4, all of it) to where the cost curve reaches
// k / NR of the total (kernels.hip adapted_bound).
__device__ __forceinline__ uint32_t rf_bound(const uint32_t* cc, const uint32_t* rb, uint32_t NR, uint32_t k,
                                             uint32_t total, uint32_t from, uint32_t gain)
{
    if (k == 0 || k >= NR || total == 0) return from;
    const uint32_t T = (uint32_t)((uint64_t)k * total / NR);
    uint32_t lo = 0, hi = NR;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (cc[mid] <= T) lo = mid;
        else hi = mid;
    }
    const uint32_t cr = cc[lo + 1] - cc[lo];
    const uint64_t tfp = (uint64_t)rb[lo] * 256u + (cr ? (uint64_t)(T - cc[lo]) * (rb[lo + 1] - rb[lo]) * 256u / cr : 0u);
    return (uint32_t)(((uint64_t)from * 256u * (4u - gain) + tfp * gain + 512u) >> 10);
}

__global__ __launch_bounds__(kRawBlock) void k_raw_pass(uint4* __restrict__ syn, uint32_t* lastF, uint32_t* clock,
                                                        uint32_t* budget_p, const float* reward, float* rbar,
                                                        uint32_t n_nrn, uint32_t E, KernelParams kp, RawWs ws)
{
    constexpr uint32_t NW = kRawBlock / 64, NR = kRfNR, RR = kRawStage / 64, MG = kRfMaxG;
    __shared__ uint2 s_fb[kRawFB];
    __shared__ uint4 s_st[NW][kRawStage];          // staged hits {event, src, dst, w}
    __shared__ alignas(16) uint32_t s_cc[NR + 4];  // the previous pass's workgroup costs, scanned in place
    __shared__ uint32_t s_spk[kRfSpkLds];          // the workgroup's spikes, budget order
    __shared__ uint32_t s_gc[MG];                  // per group: its candidates, then their exclusive prefix
    __shared__ uint32_t s_gk[MG];                  // per group: the sweeping wave's candidates before its first
                                                   // survivor (the least over its survivors)
    __shared__ uint8_t s_gw[MG];                   // per group: the wave that swept it
    __shared__ uint32_t s_ct[NW][kRfCt];           // per wave: its sequence's first chunks' pool ids
    __shared__ RfLds L;
    const uint64_t t_entry = __builtin_amdgcn_s_memrealtime();
    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = wave_uniform(tid >> 6);
    // the filter global -> LDS (LDS-DMA) before the first records are requested
#pragma unroll
    for (uint32_t c = 0; c < kRawFB / 2 / kRawBlock; ++c)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(ws.filter) + c * kRawBlock + tid,
                                         reinterpret_cast<uint4*>(s_fb) + c * kRawBlock + (tid & ~63u), 16, 0, 0);
    // the pass's state and scalars (C1: pass-start values; nothing this launch
    // writes them before every workgroup has read them)
    const uint32_t pass = sload(&ws.hdr->pass), pvalid = sload(&ws.hdr->pvalid), pE = sload(&ws.hdr->pE);
    const uint32_t now = sload(clock), b0 = sload(budget_p);
    const float R = sload(reward), rb = sload(rbar);
    const uint32_t tag = pass + 1u;
    const uint32_t NI = (E + kRawIt - 1) / kRawIt;  // iterations of the sweep
    // bounds[pass % 3] partition these events; the previous pass wrote its
    // bounds into bounds[(pass + 2) % 3] and its costs over them
    const bool valid = pvalid == kRawInit && pE == E;
    uint32_t* bcur = ws.bounds + (pass % 3u) * (NR + 1);
    uint32_t* bnext = ws.bounds + ((pass + 1u) % 3u) * (NR + 1);
    const uint32_t* bprev = ws.bounds + ((pass + 2u) % 3u) * (NR + 1);
    const uint32_t* cost_in = ws.cost + ((pass + 1u) % 2u) * NR;
    uint32_t* cost_out = ws.cost + (pass % 2u) * NR;
    if (valid && tid < NR / 4)  // the previous pass's costs to LDS (the next partition's input)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(cost_in) + tid,
                                         reinterpret_cast<uint4*>(s_cc) + (tid & ~63u), 16, 0, 0);
    const uint32_t ib = valid ? sload(bcur + blockIdx.x) : (uint32_t)((uint64_t)blockIdx.x * NI / NR);
    const uint32_t ie = valid ? sload(bcur + blockIdx.x + 1) : (uint32_t)((uint64_t)(blockIdx.x + 1) * NI / NR);
    const uint32_t nit = ie - ib;  // the workgroup's iterations
    // groups of gsz = 2^gsh iterations (at least kRfG), at most MG of them
    uint32_t gsh = 31 - __builtin_clz(kRfG);
    while (((uint64_t)MG << gsh) < nit) ++gsh;
    const uint32_t gsz = 1u << gsh;
    const uint32_t ngrp = (nit + gsz - 1) / gsz;
    for (uint32_t i = tid; i < ngrp; i += kRawBlock) {
        s_gc[i] = 0u;
        s_gk[i] = ~0u;
    }
    uint4* st = s_st[wid];
    uint4 Rc[kRfD][kRawK];
    // iteration it (of the workgroup's range): events (ib + it) * 256 + k * 64
    // + lane.  Lanes past the range or E load record 0 (every call issues
    // exactly kRawK loads, which the prologue's wait counts; an iteration past
    // the range is never swept, and the sweep's lanes past E are masked where
    // the records are consumed, so no use of a load follows it here)
    auto issue = [&](uint32_t d, uint32_t it) __attribute__((always_inline)) {
#pragma unroll
        for (uint32_t k = 0; k < kRawK; ++k) {
            const uint64_t t = (uint64_t)(ib + it) * kRawIt + k * 64 + lane;
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            const bool live = it < nit && t < E;
            const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(syn) + (live ? t : 0ull));
            Rc[d][k] = make_uint4(x.x, x.y, x.z, x.w);
        }
    };
    // the wave's iterations: its groups' in order, kRfD in flight (buffer d
    // holds itb[d]).  Wave w starts with the m0 groups [w m0, w m0 + m0) --
    // enough for the kRfD iterations fetched before the barrier, so no claim
    // comes before the counter is set --, then the fetch cursor {fg, fi}
    // claims the next group from the workgroup's counter whenever it needs one
    const uint32_t m0 = (kRfD + gsz - 1) / gsz;
    uint32_t fg = wid * m0 < ngrp ? wid * m0 : kRawNone, fi = 0, fstat = m0 - 1;
    if (fg != kRawNone && lane == 0) s_gw[fg] = (uint8_t)wid;
    auto next_fetch = [&]() -> uint32_t {  // wave-uniform: the next iteration of the wave, kRawNone past its last
        if (fg == kRawNone) return kRawNone;
        if (fi == gsz || fg * gsz + fi >= nit) {  // past the group: the next one
            uint32_t g = fg + 1;
            if (fstat) --fstat;
            else {
                if (lane == 0) g = atomicAdd(&L.next, 1u);
                g = wave_uniform(g);
            }
            fg = g < ngrp ? g : kRawNone;
            fi = 0;
            if (fg == kRawNone) return kRawNone;
            if (lane == 0) s_gw[fg] = (uint8_t)wid;
        }
        return fg * gsz + fi++;
    };
    if (tid == 0) {
        L.next = NW * m0;
        L.tmax = 0u;
        L.g1 = 0u;
        L.g2 = 0u;
        L.done = 0u;
    }
    uint32_t itb[kRfD];
    __builtin_amdgcn_sched_barrier(0);  // the LDS-DMAs above stay older than the records
#pragma unroll
    for (uint32_t d = 0; d < kRfD; ++d) {
        itb[d] = next_fetch();
        issue(d, itb[d]);  // (kRawNone: past the range, loads counted all the same)
    }
    // the filter, the costs and the tallies' zeros in LDS for every wave, the
    // first records still in flight: this wave's LDS-DMAs are older than its
    // kRfD * kRawK record loads and vmcnt retires in order (a __syncthreads
    // would wait for the records' whole round trip, ~5 us at config 3).  The
    // builtin wait, not inline asm: the compiler's own count then knows the
    // DMAs are done (kernels.hip wait_vm_lgkm0)
    __builtin_amdgcn_sched_barrier(0);
    {
        constexpr int N = kRfD * kRawK;
        static_assert(N < 64, "vmcnt is 6 bits");
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4));
        asm volatile("" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    const uint32_t window = kp.window_pre, refr = kp.refractory;
    uint32_t pend = 0, n_g1 = 0, S = 0, Kw = 0, n_it = 0;
    // the survivor sequence: chunk ids of its first and current chunk, entries
    // stored (kRawNone: all so far), the first unstored survivor's event and
    // the wave's candidates before it
    uint32_t first_id = kRawNone, cur_id = kRawNone, lim = kRawNone, resume = kRawNone, kres = 0;
    auto new_chunk = [&]() -> uint32_t {  // wave-uniform; kRawNone when the pool is spent
        uint32_t id = 0;
        if (lane == 0) id = atomicAdd(&ws.hdr->chunks, 1u);
        id = wave_uniform(id);
        return id < ws.pool_chunks ? id : kRawNone;
    };
    // every staged hit through the gates (one round trip), the survivors
    // appended to the sequence in event order and tallied to their groups
    auto flush = [&]() {
        // the gathers first, from the stage's {src, dst} alone (the records in
        // flight keep most registers: the entries are re-read from LDS below)
        uint32_t a[RR], bl[RR];
#pragma unroll
        for (uint32_t j = 0; j < RR; ++j) {
            const uint32_t q = j * 64 + lane;
            const uint32_t src = q < pend ? st[q].y : kRawNone, dst = q < pend ? st[q].z : kRawNone;
            const bool ok = src < n_nrn && dst < n_nrn;
            a[j] = ok ? lastF[src] : now;   // brain.metal:73 (exact, for the filter's hits)
            bl[j] = ok ? lastF[dst] : now;  // brain.metal:79, in the same round trip
        }
        // the gates; each entry rewritten in place as its pool entry; places
        // and tallies: survivor x of the sequence, K(x) = the wave's
        // candidates before it
        uint64_t m2[RR], mc[RR];
        uint32_t n = 0, nc = 0;
#pragma unroll
        for (uint32_t j = 0; j < RR; ++j) {
            const uint32_t q = j * 64 + lane;
            uint4 e = q < pend ? st[q] : make_uint4(0u, kRawNone, kRawNone, 0u);
            const bool ok = e.y < n_nrn && e.z < n_nrn;
            const bool g1 = ok && now - a[j] <= window;    // brain.metal:73-77 (u32 ages)
            const bool g2 = g1 && now - bl[j] > refr;      // brain.metal:79-83
            const bool cand = g2 && spike_candidate(kp, __uint_as_float(e.w), e.x, now);  // brain.metal:91-92
            m2[j] = __ballot(g2);
            mc[j] = __ballot(cand);
            n_g1 += (uint32_t)__popcll(__ballot(g1));
            if (g2 && e.x == 0u) {  // event 0 reached the budget test (brain.metal:110): drained before
                                    // this workgroup's look-back word is published
                __hip_atomic_store(&ws.hdr->t0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            st[q] = make_uint4(e.x, __float_as_uint((float)(now - bl[j])) | (cand ? 0x80000000u : 0u), e.w, e.z);
            if (g2) {
                const uint32_t gl = ((e.x >> 8) - ib) >> gsh;
                atomicMin(&s_gk[gl], Kw + nc + mbcnt64(mc[j]));  // K never decreases along the sequence
                if (cand) atomicAdd(&s_gc[gl], 1u);
            }
            n += (uint32_t)__popcll(m2[j]);
            nc += (uint32_t)__popcll(mc[j]);
        }
        if (n && lim == kRawNone) {
            // chunks for entries [S, S + n): the current one and up to two more
            // (n <= 256, 255 per chunk); a new chunk's id goes into its
            // predecessor's link slot
            uint32_t ids[3] = {cur_id, kRawNone, kRawNone};
            const uint32_t c0 = S / kRfLink, c1 = (S + n - 1) / kRfLink;
            if (S % kRfLink == 0) {  // S starts a new chunk
                ids[0] = new_chunk();
                if (ids[0] != kRawNone) {
                    if (first_id == kRawNone) first_id = ids[0];
                    else if (lane == 0) ws.pool[(uint64_t)cur_id * kRawChunk + kRfLink].x = ids[0];
                    if (lane == 0 && c0 < kRfCt) s_ct[wid][c0] = ids[0];
                }
            }
            for (uint32_t c = 1; c <= c1 - c0 && ids[c - 1] != kRawNone; ++c) {  // wave-uniform
                ids[c] = new_chunk();
                if (ids[c] != kRawNone && lane == 0) {
                    ws.pool[(uint64_t)ids[c - 1] * kRawChunk + kRfLink].x = ids[c];
                    if (c0 + c < kRfCt) s_ct[wid][c0 + c] = ids[c];
                }
            }
            uint32_t stored = n;  // the first chunk that could not be had ends the stored entries
            for (uint32_t c = 0; c <= c1 - c0; ++c)
                if (ids[c] == kRawNone) {
                    stored = (c0 + c) * kRfLink > S ? (c0 + c) * kRfLink - S : 0u;
                    break;
                }
            uint32_t o = 0, oc = 0;
#pragma unroll
            for (uint32_t j = 0; j < RR; ++j) {
                const uint32_t x = o + mbcnt64(m2[j]);  // this survivor's place among the flush's
                typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
                const u32x4 e = reinterpret_cast<const u32x4*>(st)[j * 64 + lane];
                if (((m2[j] >> lane) & 1u) && x < stored) {
                    const uint32_t xs = S + x, c = xs / kRfLink - c0;
                    const uint32_t id = c == 0 ? ids[0] : (c == 1 ? ids[1] : ids[2]);
                    reinterpret_cast<u32x4*>(ws.pool)[(uint64_t)id * kRawChunk + xs % kRfLink] = e;
                }
                if (stored < n && o <= stored && stored < o + (uint32_t)__popcll(m2[j])) {  // wave-uniform
                    // the survivor at place `stored` is the first one not stored
                    const uint64_t mm = m2[j];
                    const uint32_t want = stored - o;  // its rank among this round's survivors
                    const bool me = ((mm >> lane) & 1u) && mbcnt64(mm) == want;
                    const int src_lane = (int)__builtin_ctzll(__ballot(me));
                    resume = (uint32_t)__builtin_amdgcn_readlane((int)e.x, src_lane);
                    kres = (uint32_t)__builtin_amdgcn_readlane((int)(Kw + oc + mbcnt64(mc[j])), src_lane);
                }
                o += (uint32_t)__popcll(m2[j]);
                oc += (uint32_t)__popcll(mc[j]);
            }
            cur_id = ids[c1 - c0] != kRawNone ? ids[c1 - c0] : cur_id;
            if (stored < n) {
                lim = S + stored;
                if (lane == 0) __hip_atomic_store(&ws.hdr->ovf, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the walk recomputes the rest: the stamps wait for every walk
            }
        }
        S += n;
        Kw += nc;
        pend = 0;
    };
    for (bool more = itb[0] != kRawNone; more;) {  // wave-uniform: kRfD iterations per step
#pragma unroll
        for (uint32_t d = 0; d < kRfD; ++d) {
            const uint32_t it = itb[d];
            if (it == kRawNone) {  // (fetch order: so is every later buffer)
                more = false;
                break;
            }
            uint4 rc[kRawK];
#pragma unroll
            for (uint32_t k = 0; k < kRawK; ++k) rc[k] = Rc[d][k];
            itb[d] = next_fetch();  // this buffer's next iteration in flight first
            if (itb[d] != kRawNone) issue(d, itb[d]);
            ++n_it;
            const uint32_t rel = (ib + it) * kRawIt;
            if (rel + kRawIt > E) {  // wave-uniform: the sweep's last iteration, lanes past E
#pragma unroll
                for (uint32_t k = 0; k < kRawK; ++k)
                    if (rel + k * 64 + lane >= E) rc[k] = make_uint4(kRawNone, kRawNone, 0u, 0u);
            }
#pragma unroll
            for (uint32_t k = 0; k < kRawK; ++k) {
                const bool h = raw_filter_pass(s_fb, rc[k].x);
                const uint64_t bm = __ballot(h);
                if (bm == 0) continue;  // wave-uniform
                if (h) st[pend + mbcnt64(bm)] = make_uint4(rel + k * 64 + lane, rc[k].x, rc[k].y, rc[k].z);
                pend += (uint32_t)__popcll(bm);
                if (pend > kRawStage - 64) flush();
            }
        }
    }
    if (pend) flush();  // the wave's tail
    // ---- the workgroup: next partition, look-back, walks, stamps, pass end ----
    const uint64_t t_tail = __builtin_amdgcn_s_memrealtime();
    uint32_t order = 0;
    if (lane == 0) {
        atomicAdd(&L.g1, n_g1);
        atomicAdd(&L.g2, S);
        const uint64_t gt = (t_tail - t_start) >> 2;  // 40-ns units
        atomicMax(&L.tmax, (uint32_t)(gt < 1 ? 1 : (gt > 0xFFFFu ? 0xFFFFu : gt)));  // (+ the walk, below)
        order = atomicAdd(&L.done, 1u);
    }
    if (wave_uniform(order) == 0) {
        // the first wave through its tail: the next pass's bound of this
        // workgroup's range (off the critical path)
        const uint32_t k = blockIdx.x + lane;
        const bool mine = lane == 0 || (lane == 1 && k == NR);
        if (valid) {
            // the previous pass's costs (LDS) scanned in place into an
            // exclusive prefix; a range above 4x the mean moves every bound the
            // whole way (kernels.hip fused_next_bounds)
            uint32_t run = 0, cmax = 0;
#pragma unroll
            for (uint32_t u = 0; u < NR / 64; ++u) {
                const uint32_t v = s_cc[u * 64 + lane];
                cmax = v > cmax ? v : cmax;
                const uint32_t inc = wave_incl_scan(v);
                s_cc[u * 64 + lane] = run + inc - v;
                run += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            }
            if (lane == 0) s_cc[NR] = run;
            for (int o = 32; o > 0; o >>= 1) {
                const uint32_t x = (uint32_t)__shfl_xor((int)cmax, o, 64);
                cmax = x > cmax ? x : cmax;
            }
            const uint32_t gain = (uint64_t)cmax * NR > 4ull * run ? 4u : 1u;  // (gain 2 / 4 measured equal)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
            if (mine) bnext[k] = k == NR ? NI : rf_bound(s_cc, bprev, NR, k, run, bcur[k], gain);
        } else if (mine) {
            // no costs to adapt from: the bounds stay (the first pass writes
            // its uniform ones as this pass's, so the next one has both)
            const uint32_t cur = k == NR ? NI : (uint32_t)((uint64_t)k * NI / NR);
            bnext[k] = cur;
            bcur[k] = cur;
        }
    }
    __syncthreads();  // every wave of the workgroup through its tail: the tallies complete
    if (wid == 0) {
        // the workgroup's flag stores (hdr->ovf, hdr->err) are agent-scope
        // atomics, performed at the coherence point, and the barrier above
        // drained them (s_waitcnt vmcnt(0)) before this wave publishes the
        // look-back word below: the stampers' acquire after their poll reads
        // them with agent-scope loads.  Not an agent-scope release
        // fence: on gfx950 that is an L2 write-back (buffer_wbl2) on every
        // workgroup's critical path, +7 us per pass measured
        // (profiles/r06g_raw_release_fence_ab.txt)
        // the groups' candidates -> their exclusive prefix in the workgroup
        // (each lane a run of consecutive groups)
        const uint32_t per = (ngrp + 63) / 64, g0 = lane * per;
        uint32_t sum = 0;
        for (uint32_t i = 0; i < per; ++i)
            if (g0 + i < ngrp) sum += s_gc[g0 + i];
        const uint32_t inc = wave_incl_scan(sum);
        uint32_t run = inc - sum;
        for (uint32_t i = 0; i < per; ++i)
            if (g0 + i < ngrp) {
                const uint32_t c = s_gc[g0 + i];
                s_gc[g0 + i] = run;
                run += c;
            }
        const uint32_t c_wg = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
        if (lane == 0) {
            atomicAdd(reinterpret_cast<unsigned long long*>(&ws.hdr->g1), (unsigned long long)L.g1);
            atomicAdd(reinterpret_cast<unsigned long long*>(&ws.hdr->g2), (unsigned long long)L.g2);
            L.cwg = c_wg;
        }
        const uint32_t cv = c_wg < b0 ? c_wg : b0;
        const uint64_t word = (uint64_t)tag << 32 | (cv < 0x3FFFFFFFu ? cv : 0x3FFFFFFFu);
        const uint32_t e = rf_poll(ws, blockIdx.x, tag, b0, true, word);
        if (lane == 0) L.excl = e;
    }
    __syncthreads();
    const uint64_t t_lb = __builtin_amdgcn_s_memrealtime();
    const uint32_t excl = L.excl, c_wg = L.cwg;
    // the workgroup's spikes: budget positions [s0, s1)
    const uint32_t s0 = excl, s1 = (uint32_t)(excl + (uint64_t)c_wg < b0 ? excl + c_wg : b0);
    const bool spk_lds = b0 <= kRfSpkLds;
    auto spike = [&](uint32_t pre, uint32_t dst) {  // the spike at budget position pre < b0
        if (spk_lds) s_spk[pre - s0] = dst;
        else if (pre < ws.spike_cap) ws.spikes[pre] = dst;
        else {  // beyond the list (a budget above 65536 and more spikes than that): stamped now,
                // which may race with another workgroup's refractory reads -- reported
            lastF[dst] = now;
            __hip_atomic_store(&ws.hdr->err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    // budget position of the survivor of group gl with K wave candidates
    // before it: every candidate of lower workgroups, of lower groups, and of
    // its group before it (its group's survivors are consecutive in the
    // wave's sequence, from the tallied first place on)
    auto base_of = [&](uint32_t gl) -> uint32_t { return excl + s_gc[gl] - s_gk[gl]; };
    // the walk of this wave's survivors in event order (brain.metal:85-122):
    // the weight update into the record's w, the spikes; budget positions
    // never decrease along the sequence
    if (excl < b0 && S > 0) {
        const uint32_t ns = lim == kRawNone ? S : lim;  // stored survivors
        uint32_t id = first_id, K = 0;  // (id: the next chunk past the LDS table)
        bool more = true;
        for (uint32_t x0 = 0; x0 < ns && more;) {  // wave-uniform: up to kRfWB chunks in flight
            const uint32_t c = x0 / kRfLink, left = (ns - x0 + kRfLink - 1) / kRfLink;
            uint32_t nb = 1;
            if (c + 1 < kRfCt) nb = left < kRfWB ? left : kRfWB;
            if (c < kRfCt && c + nb > kRfCt) nb = kRfCt - c;
            uint32_t cid[kRfWB];
#pragma unroll
            for (uint32_t b = 0; b < kRfWB; ++b) cid[b] = b < nb ? (c + b < kRfCt ? s_ct[wid][c + b] : id) : 0u;
            uint4 ex[kRfWB][4];
#pragma unroll
            for (uint32_t b = 0; b < kRfWB; ++b)
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    const uint32_t x = x0 + b * kRfLink + j * 64 + lane;
                    ex[b][j] = b < nb && j * 64 + lane < kRfLink && x < ns ? ws.pool[(uint64_t)cid[b] * kRawChunk + j * 64 + lane]
                                                                          : make_uint4(0u, 0u, 0u, 0u);
                }
            const uint32_t xl = x0 + nb * kRfLink;  // the sequence past this batch
            if (xl < ns && c + nb >= kRfCt) {      // past the table: the last chunk's link
                uint32_t last = cid[0];
#pragma unroll
                for (uint32_t b = 1; b < kRfWB; ++b) last = b + 1 == nb ? cid[b] : last;
                id = ws.pool[(uint64_t)last * kRawChunk + kRfLink].x;
            }
#pragma unroll
            for (uint32_t b = 0; b < kRfWB; ++b) {
                if (b >= nb || !more) break;  // wave-uniform
                const uint32_t xb = x0 + b * kRfLink, nc = ns - xb < kRfLink ? ns - xb : kRfLink;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if (j * 64 >= nc) break;  // wave-uniform
                    const bool v = j * 64 + lane < nc, cand = v && (ex[b][j].y >> 31);
                    const uint64_t bc = __ballot(cand);
                    const uint32_t pre = v ? base_of(((ex[b][j].x >> 8) - ib) >> gsh) + K + mbcnt64(bc) : kRawNone;
                    if ((uint32_t)__builtin_amdgcn_readfirstlane((int)pre) >= b0) {  // lane 0: the round's first
                        more = false;
                        break;
                    }
                    if (v && pre < b0) {
                        const float w = updated_weight(kp, __uint_as_float(ex[b][j].z), cand, R, rb,
                                                       __uint_as_float(ex[b][j].y & 0x7FFFFFFFu));
                        reinterpret_cast<float*>(syn + ex[b][j].x)[2] = w;  // brain.metal:122 (src, dst, pad unchanged)
                        if (cand) spike(pre, ex[b][j].w);
                    }
                    K += (uint32_t)__popcll(bc);
                }
            }
            x0 = xl;
        }
        if (lim != kRawNone && more) {
            // the pool ran out: the rest recomputed from the records of this
            // wave's groups from the first unstored survivor's event on, with
            // the pass-start lastF (every stamp of this pass waits for every
            // walk: hdr->ovf)
            K = kres;
            for (uint32_t gl = 0; gl < ngrp && more; ++gl) {  // wave-uniform
                if (s_gw[gl] != wid) continue;
                const uint32_t ge_it = gl * gsz + gsz < nit ? gl * gsz + gsz : nit;
                const uint32_t gs = (ib + gl * gsz) * kRawIt, ge = (ib + ge_it) * kRawIt < E ? (ib + ge_it) * kRawIt : E;
                if (ge <= resume) continue;
                const uint32_t base = base_of(gl);  // (a group with no survivor never gets here with one)
                for (uint32_t t0 = gs > resume ? gs : resume; t0 < ge; t0 += 64) {  // wave-uniform
                    const uint32_t t = t0 + lane;
                    const uint4 rc = t < ge ? syn[t] : make_uint4(kRawNone, kRawNone, 0u, 0u);
                    const bool ok = rc.x < n_nrn && rc.y < n_nrn;
                    const uint32_t la = ok ? lastF[rc.x] : now, lb2 = ok ? lastF[rc.y] : now;
                    const bool g2 = ok && now - la <= window && now - lb2 > refr;
                    const bool cand = g2 && spike_candidate(kp, __uint_as_float(rc.z), t, now);
                    const uint64_t bc = __ballot(cand);
                    const uint64_t b2 = __ballot(g2);
                    if (b2) {
                        // the round's first survivor already past the budget: so is the rest
                        const uint32_t pre0 = base + K + mbcnt64(bc & ((1ull << __builtin_ctzll(b2)) - 1ull));
                        if (base + K >= b0 || pre0 >= b0) {
                            more = false;
                            break;
                        }
                    }
                    const uint32_t pre = base + K + mbcnt64(bc);
                    if (g2 && pre < b0) {
                        const float w = updated_weight(kp, __uint_as_float(rc.z), cand, R, rb, (float)(now - lb2));
                        reinterpret_cast<float*>(syn + t)[2] = w;
                        if (cand) spike(pre, rc.y);
                    }
                    K += (uint32_t)__popcll(bc);
                }
            }
        }
    }
    __syncthreads();  // the workgroup's walks (and its LDS spike list) done
    const uint64_t t_walk = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        __hip_atomic_fetch_add(&ws.hdr->wdone, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        // the workgroup's cost: its longest stream and its walk (the dense
        // input stretch's walk is long: its range shrinks for it)
        const uint32_t c = L.tmax + (uint32_t)((t_walk - t_lb) >> 2);
        cost_out[blockIdx.x] = nit == 0 ? 0u : (c > 0xFFFFu ? 0xFFFFu : c);
    }
    uint64_t* clk = ws.clk + (uint64_t)kRfClk * (blockIdx.x * NW + wid);  // diagnostics (abnn_debug_raw_wave_clock)
    if (lane < kRfClk) {
        const uint64_t vals[kRfClk] = {t_entry, t_start, t_tail, t_lb, t_walk, t_walk, n_it, S};
        uint64_t x = vals[0];
#pragma unroll
        for (uint32_t j = 1; j < kRfClk; ++j) x = lane == j ? vals[j] : x;
        clk[lane] = x;
    }
    const bool first = blockIdx.x == 0;
    if (!(s1 > s0 || first)) return;
    // every look-back word published = every refractory stage (lastF read) of
    // the pass done; with a pool overflow, every walk too (recomputes read lastF)
    if (wid == 0) {
        const uint32_t tot = rf_poll(ws, gridDim.x, tag, b0, false, 0ull);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (__hip_atomic_load(&ws.hdr->ovf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            bool all_walked = false;
            for (uint32_t spins = 0; spins < kRfSpinLimit && !all_walked; ++spins) {
                all_walked = __hip_atomic_load(&ws.hdr->wdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= gridDim.x;
                if (!all_walked) __builtin_amdgcn_s_sleep(1);
            }
            // gave up (never expected: every workgroup is resident): the stamps
            // may race with a recompute's lastF reads -- reported, as a look-back
            // timeout is (abnn_traversal_workspace_error = 2)
            if (!all_walked && lane == 0)
                __hip_atomic_store(&ws.hdr->err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        if (lane == 0) L.tot = tot;
    }
    __syncthreads();
    const uint32_t lim_list = spk_lds ? s1 : (s1 < ws.spike_cap ? s1 : ws.spike_cap);
    for (uint32_t i = s0 + tid; i < lim_list; i += kRawBlock)
        lastF[spk_lds ? s_spk[i - s0] : ws.spikes[i]] = now;  // brain.metal:125-126
    if (first && tid == 0) {  // the pass's end: every workgroup has read the pass-start scalars
        const uint32_t tot = L.tot;
        RawHdr* h = ws.hdr;
        const uint32_t t0 = __hip_atomic_load(&h->t0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        h->now = now;
        h->budget0 = b0;
        h->ncand = tot;
        *budget_p = b0 - tot;                                   // brain.metal:95-98 (C1: no wrap)
        if (t0 && b0 > 0) *rbar = rb + kp.alpha_rbar * (R - rb);  // brain.metal:110-113
        *clock = now + kp.clock_inc;                             // brain.metal:129 (E > 0)
        h->pass = pass + 1u;
        h->pvalid = kRawInit;
        h->pE = E;
    }
    if (lane == 0) clk[5] = __builtin_amdgcn_s_memrealtime();
}

__global__ __launch_bounds__(256) void k_raw_renorm(uint32_t* lastF, const uint32_t* clock, uint32_t n)
{
    const uint32_t base = *clock;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) lastF[i] -= base;  // brain.metal:142-143 (u32 wrap for never-fired neurons)
}

__global__ void k_raw_zero_clock(uint32_t* clock) { *clock = 0u; }  // brain.metal:144

// abnn_debug_raw_gate_timing: an event pair around every gate launch (host
// state of the diagnostics only; the pass never reads it).
struct RawTiming {
    bool on = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev;
};
RawTiming& raw_timing()
{
    static RawTiming t;
    return t;
}

// The fused pass needs every one of its kRawGateWGs workgroups resident at
// once (the look-back): one per CU.  ABNN_RAW_FUSED=0 (or
// abnn_debug_raw_fused(0)) selects the five-launch pass of round 4 (A/B, and
// the fallback where 256 workgroups of 158 KB LDS do not fit at once).
int g_raw_fused = -1;  // abnn_debug_raw_fused: -1 the environment, 0 off, 1 on

bool raw_fused_ok()
{
    if (g_raw_fused == 0) return false;
    // per device (a process may drive several): 0 unknown, 1 fits, 2 does not
    constexpr int kMaxDev = 64;
    static std::atomic<int8_t> fits_by_dev[kMaxDev];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return false;
    int8_t f = dev < kMaxDev ? fits_by_dev[dev].load(std::memory_order_relaxed) : 0;
    if (f == 0) {
        int cus = 0, per = 0;
        const bool ok = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k_raw_pass, kRawBlock, 0) == hipSuccess &&
                        (uint64_t)cus * (uint64_t)per >= kRawGateWGs;
        f = ok ? 1 : 2;
        if (dev < kMaxDev) fits_by_dev[dev].store(f, std::memory_order_relaxed);
    }
    if (f != 1) return false;
    if (g_raw_fused == 1) return true;
    static const bool env_on = [] {
        const char* env = std::getenv("ABNN_RAW_FUSED");
        return !env || std::atoi(env) != 0;
    }();
    return env_on;
}

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

uint64_t abnn_traversal_workspace_min_bytes(uint32_t n_syn, uint32_t events)
{
    return raw_fixed_bytes(raw_events(n_syn, events));
}

abnn_status abnn_launch_traversal(const abnn_traversal_args* a, void* stream)
{
    if (!a || !a->clock || !a->budget || !a->reward || !a->rbar || !a->workspace ||
        (a->n_syn && (!a->syn || !a->last_fired)))
        return ABNN_ERR_INVALID;
    const uint64_t E = raw_events(a->n_syn, a->events);
    if (a->workspace_bytes < raw_fixed_bytes(E) || ((uintptr_t)a->workspace & 15u)) return ABNN_ERR_INVALID;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const RawWs ws = raw_ws(a->workspace, E, a->workspace_bytes);
    const KernelParams kp = raw_params(*a);
    uint4* syn = reinterpret_cast<uint4*>(a->syn);
    hipLaunchKernelGGL(k_raw_filter, dim3(kRawFB / kRawFilterBlocks), dim3(256), 0, s, a->last_fired, a->clock,
                       a->n_nrn, kp, ws);
    if (ws.ng && raw_fused_ok()) {  // the fused pass: the rest in one launch
        RawTiming& tm = raw_timing();
        std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
        if (tm.on && hipEventCreate(&ev.first) == hipSuccess && hipEventCreate(&ev.second) == hipSuccess)
            (void)hipEventRecord(ev.first, s);
        hipLaunchKernelGGL(k_raw_pass, dim3(kRawGateWGs), dim3(kRawBlock), 0, s, syn, a->last_fired, a->clock, a->budget,
                           a->reward, a->rbar, a->n_nrn, (uint32_t)E, kp, ws);
        if (ev.second) {
            (void)hipEventRecord(ev.second, s);
            tm.ev.push_back(ev);
        }
        return hipGetLastError() == hipSuccess ? ABNN_OK : ABNN_ERR_HIP;
    }
    if (ws.ng) {
        RawTiming& tm = raw_timing();
        std::pair<hipEvent_t, hipEvent_t> ev{nullptr, nullptr};
        if (tm.on && hipEventCreate(&ev.first) == hipSuccess && hipEventCreate(&ev.second) == hipSuccess)
            (void)hipEventRecord(ev.first, s);
        hipLaunchKernelGGL(k_raw_gate, dim3(kRawGateWGs), dim3(kRawBlock), 0, s, syn, a->last_fired, a->clock, a->n_nrn,
                           (uint32_t)E, kp, ws);
        if (ev.second) {
            (void)hipEventRecord(ev.second, s);
            tm.ev.push_back(ev);
        }
    }
    if (ws.ng)
        hipLaunchKernelGGL(k_raw_scan_local, dim3((ws.ng + kRawScanBlock - 1) / kRawScanBlock), dim3(kRawScanThreads), 0,
                           s, ws);
    hipLaunchKernelGGL(k_raw_scan, dim3(1), dim3(kRawScanThreads), 0, s, ws, (uint32_t)E, a->clock, a->budget, a->reward,
                       a->rbar, kp);
    if (ws.ng) {
        const uint32_t g = (uint32_t)std::min<uint64_t>((ws.ng + 4 * kRawApplyGroups - 1) / (4 * kRawApplyGroups), kRawApplyWGs);
        hipLaunchKernelGGL(k_raw_apply, dim3(g), dim3(256), 0, s, syn, a->last_fired, a->n_nrn, (uint32_t)E, kp, ws);
        hipLaunchKernelGGL(k_raw_stamp, dim3(1), dim3(1024), 0, s, a->last_fired, ws);
    }
    return hipGetLastError() == hipSuccess ? ABNN_OK : ABNN_ERR_HIP;
}

abnn_status abnn_traversal_workspace_error(const void* workspace, uint32_t* err, void* stream)
{
    if (!workspace || !err) return ABNN_ERR_INVALID;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    RawHdr* h = static_cast<RawHdr*>(const_cast<void*>(workspace));
    RawHdr hh;
    if (hipMemcpyAsync(&hh, h, sizeof(hh), hipMemcpyDeviceToHost, s) != hipSuccess) return ABNN_ERR_HIP;
    if (hipStreamSynchronize(s) != hipSuccess) return ABNN_ERR_HIP;
    *err = hh.init == kRawInit ? hh.err : 0u;  // (never launched on: nothing to report)
    // sticky until read: cleared here, not by the next launch
    if (hh.init == kRawInit && hh.err && hipMemsetAsync(&h->err, 0, 4, s) != hipSuccess) return ABNN_ERR_HIP;
    return hipStreamSynchronize(s) == hipSuccess ? ABNN_OK : ABNN_ERR_HIP;
}

// Diagnostics (abnn_debug.h): the last pass's pre-gated / surviving events
// from the workspace header, and HIP events around every k_raw_gate launch.
abnn_status abnn_debug_raw_stats(const void* workspace, uint64_t* out2, void* stream)
{
    if (!workspace || !out2) return ABNN_ERR_INVALID;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const RawHdr* h = static_cast<const RawHdr*>(workspace);
    if (hipMemcpyAsync(out2, &h->g1, 16, hipMemcpyDeviceToHost, s) != hipSuccess) return ABNN_ERR_HIP;
    return hipStreamSynchronize(s) == hipSuccess ? ABNN_OK : ABNN_ERR_HIP;
}

abnn_status abnn_debug_raw_gate_timing(int enable)
{
    RawTiming& t = raw_timing();
    for (auto& e : t.ev) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    t.ev.clear();
    t.on = enable != 0;
    return ABNN_OK;
}

abnn_status abnn_debug_raw_gate_time(double* total_ms, uint32_t* launches)
{
    if (!total_ms || !launches) return ABNN_ERR_INVALID;
    RawTiming& t = raw_timing();
    double ms = 0.0;
    for (auto& e : t.ev) {
        if (hipEventSynchronize(e.second) != hipSuccess) return ABNN_ERR_HIP;
        float x = 0.0f;
        if (hipEventElapsedTime(&x, e.first, e.second) != hipSuccess) return ABNN_ERR_HIP;
        ms += x;
    }
    *total_ms = ms;
    *launches = (uint32_t)t.ev.size();
    return ABNN_OK;
}

abnn_status abnn_debug_raw_fused(int mode)
{
    if (mode < -1 || mode > 1) return ABNN_ERR_INVALID;
    g_raw_fused = mode;
    return ABNN_OK;
}

int abnn_debug_raw_fused_active(void) { return raw_fused_ok() ? 1 : 0; }

abnn_status abnn_debug_raw_wave_clock(const void* workspace, uint64_t workspace_bytes, uint32_t n_syn, uint32_t events,
                                      uint64_t* out, uint64_t n, void* stream)
{
    const uint64_t E = raw_events(n_syn, events);
    if (!workspace || !out || workspace_bytes < raw_fixed_bytes(E)) return ABNN_ERR_INVALID;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const RawWs ws = raw_ws(const_cast<void*>(workspace), E, workspace_bytes);
    const uint64_t words = std::min<uint64_t>(n, (uint64_t)kRfClk * kRawWaves);
    if (hipMemcpyAsync(out, ws.clk, words * 8, hipMemcpyDeviceToHost, s) != hipSuccess) return ABNN_ERR_HIP;
    return hipStreamSynchronize(s) == hipSuccess ? ABNN_OK : ABNN_ERR_HIP;
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
