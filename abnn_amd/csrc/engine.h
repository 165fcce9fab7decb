// engine.h -- internal declarations shared by the kernels (kernels.hip) and the
// C-ABI implementation (capi.hip).  Not installed; the public surface is
// include/abnn/abnn.h.
#pragma once

#include <hip/hip_runtime.h>
#include <cstdint>

#include "../../include/abnn/abnn.h"

namespace abnn {

// One 256-thread workgroup streams one chunk of kChunk consecutive events,
// kEvPerThread per lane, lane-contiguous (event = chunk*kChunk + k*256 + tid)
// so every wave-instruction reads 1 KiB of consecutive 16-B records.
constexpr int kBlock = 256;
constexpr int kEvPerThread = 8;
constexpr int kChunk = kBlock * kEvPerThread;  // 2048 events
constexpr int kWaves = kBlock / 64;
constexpr int kApplyGrid = 1024;    // persistent grid of the apply kernel
constexpr int kScanThreads = 1024;  // single-workgroup chunk scan

// Per-pass bookkeeping in device memory (one per handle).
struct alignas(16) PassWork {
    uint32_t n_active;     // chunks queued for the apply kernel
    uint32_t t0_g2;        // global event 0 passed both gates this pass
    uint64_t events;       // visited events of this shard this pass
    uint64_t g1;           // passed the pre-gate
    uint64_t g2;           // passed the refractory gate
    abnn_stats stats;      // cumulative (finalize adds)
};

// Kernel-facing view of a handle's device state.
struct DeviceState {
    uint4* syn;               // abnn_synapse[n_syn] viewed as 16-B vectors
    uint64_t* last_fired;     // [n_nrn]
    uint64_t* last_visited;   // [n_nrn]
    uint64_t* clock;          // [1]
    float* reward;            // [1]
    float* rbar;              // [1]
    uint64_t* bitmap;         // [ceil(n_nrn/64)] recent-spike bit per neuron
    uint4* chunk_cnt;         // [n_chunks] {g2, candidates, g1, 0}
    uint32_t* chunk_pre;      // [n_chunks] exclusive candidate prefix (capped)
    uint32_t* active;         // [n_chunks] chunk ids for the apply kernel
    uint4* g2buf;             // [n_chunks*kChunk] gated entries, per-chunk regions
    uint2* apply_partial;     // [kApplyGrid] {updated, fired} per apply block
    int32_t* fired;           // [max_spikes] internal spike list (world = 1)
    int64_t* summary;         // [ABNN_SUMMARY_WORDS] internal (world = 1)
    PassWork* work;
    uint64_t n_syn;           // local records
    uint64_t n_nrn;
    uint64_t events;          // visited events per pass (local)
    uint64_t syn_offset;
    uint32_t n_chunks;
};

struct KernelParams {
    float base_scale, target_rate_hz, eta_home, eta_reward, alpha_rbar;
    float a_ltp, a_ltd, w_min, w_max;
    uint32_t refractory, window_pre, clock_inc, max_spikes;
    uint32_t track_visits;
};

KernelParams to_kernel_params(const abnn_params& p);

// Launchers (all asynchronous on `s`).
hipError_t launch_bitmap(const DeviceState& d, const KernelParams& kp, uint64_t stim_first,
                         uint64_t stim_count, hipStream_t s);
hipError_t launch_gate(const DeviceState& d, const KernelParams& kp, hipStream_t s);
hipError_t launch_scan(const DeviceState& d, const KernelParams& kp, int64_t* summary_out,
                       hipStream_t s);
hipError_t launch_apply(const DeviceState& d, const KernelParams& kp, const int64_t* summaries,
                        uint32_t world, uint32_t rank, int32_t* fired, hipStream_t s);
hipError_t launch_finalize(const DeviceState& d, const KernelParams& kp, const int64_t* summaries,
                           uint32_t world, const int32_t* fired, hipStream_t s);
hipError_t launch_renorm(const DeviceState& d, uint64_t base, hipStream_t s);
hipError_t launch_generate(const DeviceState& d, uint32_t n_in, uint32_t n_out, uint64_t seed,
                           hipStream_t s);
hipError_t launch_checksum(const DeviceState& d, uint64_t* out_dev, hipStream_t s);
hipError_t launch_stamp_list(const DeviceState& d, const uint32_t* idx_dev, uint64_t n,
                             const uint64_t* value_dev, uint64_t value, hipStream_t s);

}  // namespace abnn
