// engine.h -- internal declarations shared by the kernels (kernels.hip) and the
// C-ABI implementation (capi.hip).  Not installed; the public surface is
// include/abnn/abnn.h.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/abnn/abnn.h"

namespace abnn {

// Pre-spike filter kept in LDS by every gate workgroup: the exact recent-spike
// bitmap folded modulo filter_words 32-bit words (16384 words = 512 Ki bits =
// 32 KiB by default).  When the bitmap itself fits, the filter IS the bitmap.
constexpr int kMaxFilterWords = 16384;
constexpr int kTile = 64;          // one tile = 64 consecutive pre-gated events of a range = one wave
constexpr int kTileBlocks = 2048;  // grid of the tile kernels (x 4 waves = 8192 waves, all resident)
constexpr int kScanThreads = 1024; // the range and tile scans are one workgroup each
constexpr int kMaxGateBlocks = 1024;
constexpr int kMaxRanges = 16384;  // kMaxGateBlocks x up to 16 waves; k_tiles holds them in registers
static_assert(kTileBlocks % kScanThreads == 0, "k_finalize sums the apply partials in whole rounds");
constexpr int kDummyRecords = 64 * 32;  // >= 64 lanes x max events per lane; also the record-buffer padding
constexpr int kStageEntries = 448;      // per gate wave: 4-B event offsets staged in LDS

// Per-pass bookkeeping in device memory (one per handle).
struct alignas(16) PassWork {
    uint32_t total_tiles;  // tiles of pre-gated entries this pass
    uint32_t t0_g2;        // global event 0 passed both gates this pass
    uint64_t events;       // visited events of this shard this pass
    uint64_t g1;           // passed the pre-gate
    uint64_t g2;           // passed the refractory gate
    abnn_stats stats;      // cumulative (finalize adds)
};

// Synapse records on the device, structure of arrays: record i is
// {src[i], dst[i], w[i]} (SynapsePacked without its never-read pad).  The
// sweep's gate streams only src: 4 B per visited event instead of 16.  Each
// array holds capacity + kDummyRecords entries (zero padding: the gate's last
// iteration reads past the sweep).
struct SynArrays {
    uint32_t* src;
    uint32_t* dst;
    float* w;
};

// Kernel-facing view of a handle's device state.
struct DeviceState {
    SynArrays syn;            // [capacity + kDummyRecords] each
    uint64_t* last_fired;     // [n_nrn]
    uint64_t* last_visited;   // [n_nrn]
    uint64_t* clock;          // [1]
    uint64_t* pass_index;     // [1] passes run (keys the random-mode picks)
    float* reward;            // [1]
    float* rbar;              // [1]
    uint32_t* bitmap;         // [n_bitmap_words] exact recent-spike bitmap
    uint32_t* filter;         // [filter_words] folded bitmap
    uint32_t* range_cnt;      // [n_ranges] pre-gated entries of each range
    uint4* tile_desc;         // [max_tiles] {range, first entry in the range, entries, 0}
    uint4* tile_mask;         // [max_tiles] {passed refractory, spike candidate} lane masks (2 x u64)
    uint32_t* tile_pre;       // [max_tiles] exclusive candidate prefix (capped; = budget: skip)
    uint32_t* g1idx;          // [iters * iter_events] pre-gated event offsets (event - region), per-range regions
    uint4* g2e;               // [max_tiles * kTile] {event - region, dst, w, isi} of the events that passed
    const uint32_t* dummy;    // [kDummyRecords] zeros: target of the stream loads past a range
    uint4* apply_partial;     // [kTileBlocks] {updated, fired, pruned, 0} per apply workgroup
    uint32_t* g2src;          // genesis on: [max tiles * kTile] src of the visited record
    uint4* grown;             // genesis on: [compact_every * max_spikes] grown records (w = 1: used)
    uint32_t* dead;           // pruning on: tombstones per kCompactChunk records (structural update)
    uint32_t* claim;          // random mode: [n_syn] highest updating event + 1 (0 = none)
    int32_t* xchg;            // internal exchange record (world = 1): summary + spike list
    PassWork* work;
    uint64_t n_syn;           // local records
    uint64_t n_nrn;
    uint32_t n_input;
    uint64_t events;          // visited events per pass (local)
    uint64_t syn_offset;
    uint64_t seed;            // random-mode pick key (abnn_params.seed)
    uint32_t mode;            // ABNN_MODE_SWEEP / ABNN_MODE_RANDOM
    uint32_t n_bitmap_words;  // 2 * ceil(n_nrn / 64)
    uint32_t filter_words;    // LDS filter size (a power of two, compiled per gate shape)
    uint32_t filter_exact;    // bitmap fits the filter: no global confirmation
    uint32_t gate_blocks;     // persistent gate workgroups G
    uint32_t n_ranges;        // G * waves per workgroup: one contiguous range per wave
    uint32_t iters;           // ceil(events / iter_events)
    uint32_t iter_events;     // 64 * gate_k events per wave iteration
    uint32_t gate_block;      // threads per gate workgroup
    uint32_t gate_k;          // events per thread per iteration
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
hipError_t launch_refrac(const DeviceState& d, const KernelParams& kp, hipStream_t s);
// launch_scan writes the exchange record's summary; with `spike_list` also its
// spike list (sharded passes).  launch_apply writes the list into `spikes`
// when non-null (the single-GPU pass, where it is the only rank).
hipError_t launch_scan(const DeviceState& d, const KernelParams& kp, int32_t* xchg_out,
                       bool spike_list, hipStream_t s);
hipError_t launch_apply(const DeviceState& d, const KernelParams& kp, const int32_t* gathered,
                        uint32_t world, uint32_t rank, int32_t* spikes, hipStream_t s);
hipError_t launch_finalize(const DeviceState& d, const KernelParams& kp, const int32_t* gathered,
                           uint32_t world, hipStream_t s);
hipError_t launch_renorm(const DeviceState& d, uint64_t base, hipStream_t s);
// Structural update: stable compaction into `dst`, block b of kCompactChunk
// records starting at offsets[b] (live counts from the k_apply tombstone tally).
hipError_t launch_compact(const SynArrays& syn, uint64_t n, const uint64_t* offsets, const SynArrays& dst,
                          hipStream_t s);
hipError_t launch_generate(const DeviceState& d, uint32_t n_in, uint32_t n_out, uint64_t seed,
                           hipStream_t s);
hipError_t launch_checksum(const DeviceState& d, uint64_t* out_dev, hipStream_t s);
hipError_t launch_stamp_list(const DeviceState& d, const uint32_t* idx_dev, uint64_t n,
                             const uint64_t* value_dev, uint64_t value, hipStream_t s);

}  // namespace abnn
