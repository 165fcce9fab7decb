// engine.h -- internal declarations shared by the kernels (kernels.hip) and the
// C-ABI implementation (capi.hip).  Not installed; the public surface is
// include/abnn/abnn.h.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/abnn/abnn.h"

namespace abnn {

// Pre-spike filter kept in LDS by every gate workgroup: two images of the exact
// recent-spike bitmap, each folded onto filter_words 32-bit words with its own
// word hash (kernels.hip; 8192 words = 32 KiB each by default).
constexpr int kMaxFilterWords = 16384;  // per image
// Second-level filter of the refractory stage (kernels.hip refrac_chunk): a
// 2-probe Bloom filter of the same recent set over kF2Words words (64 Ki bits),
// stored after the blocked filter in each filter buffer and copied to LDS by
// the gate's prologue.  Staged events it rejects gather nothing; the ones it
// passes gather {dst, w} beside the exact bitmap word (one dependent round
// trip less).  Its hashes are independent of the blocked filter's.
constexpr uint32_t kF2Words = 2048;
__host__ __device__ inline uint32_t f2_hash1(uint32_t n) { return (n * 0x9E3779B1u) >> 16; }
__host__ __device__ inline uint32_t f2_hash2(uint32_t n) { return (n * 0x85EBCA77u + 0x165667B1u) >> 16; }
constexpr int kScanThreads = 1024; // k_scan is one workgroup
constexpr int kMaxGateBlocks = 1024;
constexpr int kMaxRanges = 16384;  // kMaxGateBlocks x up to 16 waves (one range per gate wave)
constexpr int kApplyThreads = 1024;  // budget-walk workgroups (k_spikes, k_claim, k_apply)
constexpr uint32_t kCandCap = 256;      // fused pass: spike candidates listed per range (more: the full walk)
constexpr uint32_t kFusedMaxRanges = 4096;  // fused pass: ranges (the partition's LDS cost prefix)
constexpr uint32_t kWalkBlocks = 256; // their grid: 4096 waves, one work item (chunk) per wave at a time
constexpr int kMaxApplyBlocks = kWalkBlocks;
static_assert(kMaxApplyBlocks <= kApplyThreads, "the finalizing workgroup reads one apply partial per thread");
static_assert(kMaxRanges % kApplyThreads == 0, "range prefix: whole ranges per thread");
constexpr int kDummyRecords = 64 * 32;  // >= 64 lanes x max events per lane; also the record-buffer padding
                                         // (the dummy block itself holds 2x as many words: {dst, w} loads)
constexpr uint32_t kFiredRing = 8;     // spike lists kept (the bitmap build needs window_pre < kFiredRing)
constexpr uint32_t kChunk = 384;        // pre-gated events per chunk (staged in LDS by a gate wave)
constexpr uint32_t kWaveClock = 16;     // diagnostics: u64 words per gate wave (wave_clock)
constexpr uint32_t kWaveClockPasses = 8; // ... per pass slot; the fused pass keeps the last 8 passes' (pass % 8)
constexpr uint32_t kChunkSlotDiv = 128; // chunk_cnt index = (region + c * kChunk) / 128 (unique per chunk)

// Per-pass bookkeeping in device memory (one per handle).
struct alignas(16) PassWork {
    uint32_t t0_g2;        // global event 0 passed both gates this pass (re-armed by finalize_pass)
    uint32_t ticket;       // k_apply (fused pass: gate) workgroups done this pass (the last one finalizes, re-arms it)
    uint32_t epoch;        // fused passes run so far: tags this pass's look-back words (never set by the host)
    uint32_t error;        // unused (the error word is host-mapped: DeviceState::err_word)
    uint32_t spec_wgs;     // fused pass: gate workgroups predicted below the budget cut (the last pass's, less one)
    uint32_t pad;
    unsigned long long shard_g2;  // sharded fused pass: refractory survivors of the shard (the summary's word 3)
    // sharded fused pass: the pass-start scalars as the gate launch read them
    // (written by its workgroup 0), so every k_shard_walk workgroup reads
    // these and its workgroup 0 ends the pass at once, without a ticket
    unsigned long long ps_now, ps_pass;
    float ps_R, ps_rb;
    uint32_t pad2[2];
    abnn_stats stats;      // host-kept counters (grown); the device ones live in DeviceState::wg_stats
};

// Fused single-GPU sweep pass (k_gate<..., kFused>): per gate
// workgroup one look-back word {tag = epoch + 1 : 32 | kind : 2 | value : 30},
// kind 1 = the spike candidates of the workgroup's ranges (capped at the
// budget).  max_spikes < 2^30.
constexpr uint32_t kLbAggregate = 1u;
constexpr uint32_t kLbSpinLimit = 1u << 22;  // ~1 s of polls: then error, never a hang

// Synapse records on the device, structure of arrays: record
// i is {src[i], dst[i], w[i]} (SynapsePacked without its never-read pad).
// src is held in 24 bits (N_NRN < 2^24 - 1, checked at create; the tombstone
// src is kSrcNone) as two streams, so the sweep's gate reads 3 B per visited
// event: a u16 word lo[i] and a u8 byte hi[i], together the *filter code* of
// src -- a bijection of the 24 bits laid out so that the gate's pre-spike
// filter test (kernels.hip, quad_filter / filter_set) needs no hashing:
// neuron n = 32 j + b sits in filter block g = (j ^ t) mod 8192,
// t = 0x9E5 (j >> 13), at low bit lb = b and high bit hb = (b + t) mod 32;
//   lo = g << 3 | hb[2:0]                 (lo & 0xFFF8 = the block's LDS byte address)
//   hi = lb | x << 5 | hb[4:3] << 6       (x = bit 5 of j >> 13, i.e. n >= 2^23)
// Record layout 4: both streams in natural record order; a gate lane loads
// 8 consecutive records' lo words (16 B) and hi bytes (8 B) per 512-record
// block (lane-contiguous events: lane order is event order within a block,
// kernels.hip k_gate).  Layout 3 permuted hi within 256-record groups for a
// lane-interleaved gate.
// Each array holds capacity + kDummyRecords entries (zero padding: the gate's
// last iteration reads past the sweep; hi rounded up to whole 256-record groups).
constexpr uint32_t kSrcNone = 0xFFFFFFu;   // 24-bit tombstone src (downloads as 0xFFFFFFFF)
constexpr uint64_t kMaxNeurons = kSrcNone; // N_NRN < 2^24 - 1
constexpr uint32_t kCodeFilterWords = 8192; // the filter the code is laid out for (sweep gate shapes)

__host__ __device__ inline uint32_t src_code(uint32_t n)  // 24-bit src -> lo | hi << 16
{
    const uint32_t b = n & 31u, j = (n >> 5) & 0x7FFFFu, jh = j >> 13;
    const uint32_t t = jh * 0x9E5u, g = (j ^ t) & 8191u, hb = (b + t) & 31u;
    return (g << 3 | (hb & 7u)) | (b | (jh >> 5) << 5 | (hb >> 3) << 6) << 16;
}

__host__ __device__ inline uint32_t code_src(uint32_t lo, uint32_t hi)  // inverse of src_code
{
    const uint32_t g = (lo >> 3) & 8191u, lb = hi & 31u, hb = (lo & 7u) | ((hi >> 6) & 3u) << 3;
    const uint32_t jh = (((hb - lb) * 13u) & 31u) | ((hi >> 5) & 1u) << 5;  // 13 = 0x9E5^-1 mod 32
    const uint32_t j = ((g ^ jh * 0x9E5u) & 8191u) | jh << 13;
    return j << 5 | lb;
}

struct SynArrays {
    uint16_t* lo;
    uint8_t* hi;
    uint2* dw;        // {dst, w bits} of each record: the refractory stage gathers both
                      // with one access (one DRAM line per event, not two)
    uint32_t* src32;  // random mode only: the same src as one u32 per record, so a pick is
                      // one random DRAM access, not two (kept in step by set_src)
};

// w of record i inside its {dst, w} pair
__host__ __device__ inline float* w_ptr(const SynArrays& a, uint64_t i) { return reinterpret_cast<float*>(a.dw + i) + 1; }

__host__ __device__ inline uint64_t hi_pos(uint64_t i) { return i; }  // layout 4: natural order

__host__ __device__ inline uint64_t hi_bytes(uint64_t count) { return (count + 255) & ~255ull; }

// Kernel-facing view of a handle's device state.
struct DeviceState {
    SynArrays syn;            // [capacity + kDummyRecords] each
    uint64_t* last_fired;     // [n_nrn]
    uint64_t* last_visited;   // [n_nrn]
    uint8_t* visit_mark;      // shard handles with track_visits: [n_nrn] visited since the last merge (else null)
    uint64_t* clock;          // [1]
    uint64_t* pass_index;     // [1] passes run (keys the random-mode picks)
    float* reward;            // [1]
    float* rbar;              // [1]
    uint32_t* bitmap;         // [n_bitmap_words] exact recent-spike bitmap of this pass
    uint32_t* filter;         // [2 * filter_words] the two folded bitmap images of this pass
    uint32_t* bitmap_next;    // the next pass's (triple-buffered by pass % 3; zeroed by the pass before)
    uint32_t* filter_next;
    uint32_t* bitmap_clear;   // the one after it (pass + 2): zeroed by this pass's gate
    uint32_t* filter_clear;
    uint64_t stim_first, stim_count;  // this pass's stimulus range (stamped `now` at pass start)
    uint32_t build_next;      // k_apply builds bitmap_next / filter_next (steady state)
    uint32_t n_next_stim;     // stimulus ranges of passes p+1-W..p+1 (distinct), for the build
    uint64_t next_stim[kFiredRing][2];
    uint4* range_info;        // [n_ranges] {gate time (40 ns), passed refractory, candidates, chunks} per gate wave
    uint32_t* range_g1;       // [n_ranges] pre-gated events per gate wave (statistics)
    uint4* g2x;               // [iters * iter_events] per-range regions: {event - region, isi | cand << 31, w, dst}
    uint4* chunk_cnt;         // [iters * iter_events / kChunkSlotDiv + 8] {pre-gated, survivors, candidates, 0}
    const uint32_t* dummy;    // [kDummyRecords] zeros: target of the stream loads past a range
    abnn_stats* wg_stats;     // [kWalkBlocks] statistics, one slot per k_apply workgroup (summed by abnn_get_stats)
    uint32_t* g2src;          // genesis on: [iters * iter_events] src of the g2x entry's record
    uint4* grown;             // genesis on: [compact_every * max_spikes] grown records (w = 1: used)
    uint32_t* dead;           // pruning on: tombstones per kCompactChunk records (structural update)
    uint32_t* claim;          // random mode: [n_syn] highest updating event + 1 (0 = none)
    PassWork* work;
    uint32_t* err_word;       // host-mapped: a fused pass's look-back wait gave up (capi.hip pass_error)
    uint64_t* wave_clock;     // [kWaveClockPasses][kWaveClock * kMaxRanges] per-wave gate times {start, stream done, refractory
                              // tail done, entry, (fused) look-back done, walk done} (100 MHz, diagnostics)
    uint32_t wave_clock_on;   // record them (abnn_debug_set_wave_clock; off by default: their stores cost
                              // ~1.2 us per fused pass, profiles/r06l_ab_wave_clock_stores.txt)
    uint32_t* fired_ring;     // [kFiredRing * max_spikes] spike list of pass q at (q % kFiredRing), budget order
    uint32_t* n_fired_ring;   // [kFiredRing] their lengths (k_apply workgroup 0)
    uint64_t* apply_clock;    // [8 * kWalkBlocks] per-workgroup k_apply timeline (diagnostics, 100 MHz)
    uint32_t* range_bounds;   // [n_ranges + 1] first iteration of each range (this pass)
    uint32_t* range_bounds_next;  // [n_ranges + 1] the next pass's (k_apply's partition_bounds, or the fused
                                  // pass's prologue; the host rotates the three)
    uint32_t* range_bounds_prev;  // [n_ranges + 1] the previous pass's (the fused prologue's cost curve)
    uint32_t adapt_ranges;    // rebalance the partition after every pass (default on; ABNN_STATIC_RANGES=1: off)
    uint32_t adapt_gain;      // a boundary moves adapt_gain / 4 of the way to its target (1..4, ABNN_ADAPT_GAIN; default 1)
    uint32_t chunk_penalty;   // partition cost added per full chunk, 40-ns units (ABNN_CHUNK_PENALTY)
    uint32_t apply_blocks;    // k_claim / k_apply grid (<= kWalkBlocks; ABNN_APPLY_BLOCKS)
    uint32_t range_map;       // gate wave -> range: 0 blocked (workgroup b: ranges b*NW..), 1 interleaved (ABNN_RANGE_MAP=1)
    // fused pass: look-back words [gate_blocks]; gate costs of the previous
    // pass (read by the prologue when prologue_adapt) and of this one
    uint64_t* lb_status;
    const uint32_t* cost_in;
    uint32_t* cost_out;
    uint2* cand_list;         // fused: per range its first kCandCap spike candidates {survivor index, dst}
                              // ([kFusedMaxRanges * kCandCap]; the walk reads these, not every survivor)
    uint32_t flush_at;        // fused: staged events that send a wave's stage through the refractory stage
                              // (<= kChunk; ABNN_FLUSH_AT)
    int32_t spec_margin;      // fused: workgroups predicted below the cut = last cut + spec_margin (ABNN_SPEC_MARGIN, -1)
    uint32_t spec_mode;       // fused: speculative weight stores 0 off, 1 below the predicted cut (default),
                              // 2 everywhere (ABNN_SPEC; 2 exercises the restore path)
    uint32_t lean;            // fused single-GPU pass without plasticity: the lean kernel (ABNN_LEAN, default 1)
    uint32_t shard_mode;      // fused pass = the first launch of a sharded pass (k_gate: no stamps, exchange record)
    int32_t* xchg;            // ... its exchange record (abnn.h: summary + local spike list)
    uint32_t prologue_adapt;  // the previous pass was fused over the same ranges: its costs move the next
                              // pass's partition (computed in this one's prologue)
    uint64_t n_syn;           // local records
    uint64_t n_nrn;
    uint32_t n_input;
    uint64_t events;          // visited events per pass (local)
    uint64_t syn_offset;
    uint64_t seed;            // random-mode pick key (abnn_params.seed)
    uint32_t mode;            // ABNN_MODE_SWEEP / ABNN_MODE_RANDOM
    uint32_t n_bitmap_words;  // 2 * ceil(n_nrn / 64)
    uint32_t filter_words;    // words per LDS filter image (a power of two, compiled per gate shape)
    uint32_t filter_log2;     // log2(filter_words)
    uint32_t gate_blocks;     // persistent gate workgroups G
    uint32_t n_ranges;        // G * waves per workgroup: one contiguous range per wave
    uint32_t iters;           // ceil(events / iter_events)
    uint32_t iter_events;     // 64 * gate_k events per wave iteration
    uint32_t gate_block;      // threads per gate workgroup
    uint32_t gate_k;          // events per thread per iteration
    uint32_t fused_max_blocks;  // fused-pass workgroups resident at once (all must be: the look-back)
};

struct KernelParams {
    float base_scale, target_rate_hz, eta_home, eta_reward, alpha_rbar;
    float a_ltp, a_ltd, w_min, w_max;
    uint32_t refractory, window_pre, clock_inc, max_spikes;
    uint32_t track_visits;
    float w_prune, p_new, w_init;  // structural plasticity (README §5)
    uint32_t compact_every;
};

// Shard exchange record (abnn.h): ABNN_SUMMARY_WORDS int64, then max_spikes
// int32 spikes padded to 8 B -- in int32 words:
__host__ __device__ constexpr uint32_t xchg_words(uint32_t max_spikes)
{
    return 2 * ABNN_SUMMARY_WORDS + ((max_spikes + 1u) & ~1u);
}

constexpr int kCompactThreads = 1024;  // structural update: 4 consecutive records per thread
constexpr int kCompactChunk = 4 * kCompactThreads;

KernelParams to_kernel_params(const abnn_params& p);

// Gate kernel shapes compiled in (threads per workgroup x events per thread).
bool gate_shape_supported(uint32_t block, uint32_t k, uint32_t filter_words);
// Resident gate workgroups per CU for a shape (occupancy API; 0 on failure).
int gate_blocks_per_cu(uint32_t block, uint32_t k, uint32_t filter_words, bool track, bool random);

// Launchers (all asynchronous on `s`).
hipError_t launch_bitmap(const DeviceState& d, const KernelParams& kp, uint64_t stim_first,
                         uint64_t stim_count, hipStream_t s);
hipError_t launch_gate(const DeviceState& d, const KernelParams& kp, hipStream_t s);
// The whole single-GPU sweep pass in one launch (gate + look-back budget walk +
// weight update + stamps + pass end).  fused_pass_supported: the shape and
// range count it is compiled for.
bool fused_pass_supported(const DeviceState& d);
// Resident fused-pass workgroups per CU (occupancy API; 0 on failure or an uncompiled shape).
int fused_blocks_per_cu(uint32_t block, uint32_t k, uint32_t filter_words, bool track);
hipError_t launch_fused_pass(const DeviceState& d, const KernelParams& kp, hipStream_t s);
// Sharded passes on the fused path: the first launch is launch_fused_pass with
// d.shard_mode = 1 (writes d.xchg); after the all-gather, this one walks every
// range from its global budget position, stamps every rank's spikes and ends
// the pass.
hipError_t launch_shard_walk(const DeviceState& d, const KernelParams& kp, const int32_t* gathered, uint32_t world,
                             uint32_t rank, hipStream_t s);
// Sharded passes: this shard's exchange record (summary + local spike list).
hipError_t launch_scan(const DeviceState& d, const KernelParams& kp, int32_t* xchg_out, hipStream_t s);
// The rest of the pass: budget walk, weight update, stamps and, in its last
// workgroup, the pass's end (rBar, clock, statistics, next partition).
// gathered == nullptr: single-GPU pass (no exchange).
hipError_t launch_apply(const DeviceState& d, const KernelParams& kp, const int32_t* gathered,
                        uint32_t world, uint32_t rank, hipStream_t s);
hipError_t launch_renorm(const DeviceState& d, uint64_t base, hipStream_t s);
hipError_t launch_pack_src(const SynArrays& a, const uint32_t* in_dev, uint64_t first, uint64_t n, hipStream_t s);
hipError_t launch_unpack_src(const SynArrays& a, uint32_t* out_dev, uint64_t first, uint64_t n, hipStream_t s);
// Structural update (abnn.h contract, capi.hip structural_update), all on `s`:
// the tally's tombstones D and their blocks into sp, the holes' ranks (offsets,
// part: the scan's per-slice sums), the tail's live prefix when the tail holds
// tombstones (toff), the fill of every tombstone below m = n - D from the tail
// [m, n) (*err = 2: the tally and the records disagree), the tally cleared, then
// the grown records appended -- skipped when *err is set.
hipError_t launch_structural_update(const SynArrays& syn, uint64_t n, uint64_t cap, uint32_t* dead, uint64_t nb,
                                    uint64_t* offsets, uint64_t* part, uint64_t* toff, unsigned long long* sp,
                                    uint32_t* err, uint32_t cus, uint4* grown, uint64_t slots, uint32_t* grown_cnt,
                                    unsigned long long* stats_grown, hipStream_t s);
// The sharded lastVisited merge (kernels.hip k_visits_delta / k_visits_merge):
// delta[i] = mark[i] ? lv[i] + 1 : 0; after the all-reduce(MAX), lv[i] =
// reduced[i] - 1 where it is non-zero, and every mark clears.
hipError_t launch_visits_delta(const uint64_t* lv, const uint8_t* mark, uint64_t* delta, uint64_t n, hipStream_t s);
hipError_t launch_visits_merge(uint64_t* lv, uint8_t* mark, const uint64_t* reduced, uint64_t n, hipStream_t s);
// acc[i] = max(acc[i], x[i]) (max) or acc[i] + x[i]: the in-process
// communicator's all-reduce (capi.hip, abnn_comm_group), one peer at a time
hipError_t launch_reduce_u64(uint64_t* acc, const uint64_t* x, uint64_t n, bool max, hipStream_t s);
// dead[] (pruning tally) recounted for the blocks that hold records [first, first + count) of n
hipError_t launch_tally_dead(const SynArrays& a, uint64_t n, uint32_t* dead, uint64_t first, uint64_t count,
                             hipStream_t s);
hipError_t launch_generate(const DeviceState& d, uint32_t n_in, uint32_t n_out, uint64_t seed,
                           hipStream_t s);
hipError_t launch_checksum(const DeviceState& d, uint64_t* out_dev, hipStream_t s);
hipError_t launch_stamp_list(const DeviceState& d, const uint32_t* idx_dev, uint64_t n,
                             const uint64_t* value_dev, uint64_t value, hipStream_t s);

}  // namespace abnn
