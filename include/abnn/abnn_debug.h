/*
 * abnn_debug.h -- diagnostics exported by libabnn_hip.so beside the C-ABI of
 * abnn.h.  NOT part of the stable boundary: their layouts follow the kernels
 * (abnn_amd/csrc/engine.h) and change without an ABI version bump.  Used by
 * tools/ (wave_clock.py, apply_clock.py, pass_stats.py) and the GPU tests.
 * Every call is synchronous (waits for the device) and copies at most n words.
 */
#ifndef ABNN_ABNN_DEBUG_H
#define ABNN_ABNN_DEBUG_H

#include "abnn.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Record the per-wave gate timeline of the following passes (on != 0) or not
 * (the default: the timeline's stores cost ~1.2 us per fused pass). */
abnn_status abnn_debug_set_wave_clock(abnn_brain* b, int on);
/* The last pass's per-wave gate timeline: 12 u64 per range (100-MHz ticks:
 * start, stream done, tail done, entry, look-back done, walk done, ...),
 * recorded while abnn_debug_set_wave_clock is on. */
abnn_status abnn_debug_wave_clock(abnn_brain* b, uint64_t* out, uint64_t n);
/* The same for pass p of the fused single-GPU pass, slot = p % 8 (the last
 * eight fused passes are kept). */
abnn_status abnn_debug_wave_clock_slot(abnn_brain* b, uint32_t slot, uint64_t* out, uint64_t n);
/* The last two-kernel pass's per-workgroup k_apply timeline, 8 u64 each. */
abnn_status abnn_debug_apply_clock(abnn_brain* b, uint64_t* out, uint64_t n);
/* The recent-spike bitmap the last pass read (bit i: neuron i recent at its
 * start), and whether the next pass's was built in-pass (1) or will be
 * rebuilt from lastFired (0). */
abnn_status abnn_debug_bitmap(abnn_brain* b, uint32_t* out, uint64_t n, int* incremental_next);
/* The current sweep partition: n_ranges + 1 iteration bounds. */
abnn_status abnn_debug_range_bounds(abnn_brain* b, uint32_t* out, uint64_t n);

/* Buffer-index launcher (abnn_launch_traversal): the last pass's pre-gated
 * and refractory-surviving events {g1, g2} from its workspace (synchronises
 * `stream`); HIP events around every k_raw_gate launch while enabled (enable
 * also clears them), their summed milliseconds and count. */
abnn_status abnn_debug_raw_stats(const void* workspace, uint64_t* out2, void* stream);
abnn_status abnn_debug_raw_gate_timing(int enable);
abnn_status abnn_debug_raw_gate_time(double* total_ms, uint32_t* launches);
/* The buffer-index pass in one launch after the filter (k_raw_pass) or the
 * five-launch pass of round 4: mode 1 / 0, or -1 = the ABNN_RAW_FUSED
 * environment variable (default: the fused pass when its 256 workgroups fit
 * the device at once). */
abnn_status abnn_debug_raw_fused(int mode);
/* 1 when the next abnn_launch_traversal runs the fused pass, else 0. */
int abnn_debug_raw_fused_active(void);
/* The last fused buffer-index pass's per-range timeline from its workspace:
 * 8 u64 per range (100-MHz ticks: entry, stream start, stream done, look-back
 * done, walk done, end; then iterations, survivors). */
abnn_status abnn_debug_raw_wave_clock(const void* workspace, uint64_t workspace_bytes, uint32_t n_syn,
                                      uint32_t events, uint64_t* out, uint64_t n, void* stream);

/* The sharded pass's exchange alone: `count` in-place all-gathers of
 * `bytes` per rank on the library's RCCL communicator (enqueued on `stream`;
 * buf holds world x bytes, this rank's record at rank x bytes). */
abnn_status abnn_debug_comm_allgather(abnn_comm* c, void* buf, uint64_t bytes, uint32_t count, void* stream);

#ifdef __cplusplus
} /* extern "C" */
#endif
#endif /* ABNN_ABNN_DEBUG_H */
