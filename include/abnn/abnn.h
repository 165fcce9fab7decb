/*
 * abnn.h -- C-ABI of the MI355X-native Monte-Carlo synapse traversal engine.
 *
 * This is the drop-in boundary for the reference's hot path:
 *   - the host class `Brain`            (abnn/src/core/brain/brain.h:24-83,
 *                                        abnn/src/core/brain/brain.cpp:21-178)
 *   - the kernel buffer-index ABI of    `monte_carlo_traversal`
 *                                       (abnn/src/core/kernels/brain.metal:41-58)
 *     and `renormalise_clock_and_times` (brain.metal:135-145)
 * Paths are relative to the reference root.  Every entry point below names the
 * reference interface it replaces.
 *
 * Rules of the boundary:
 *   - plain C types only (no torch, no HIP types: streams are `void*` that hold
 *     a hipStream_t, NULL = the default stream).  Pass functions
 *     (abnn_traverse, abnn_shard_*) only enqueue on that stream; every other
 *     function is synchronous and first waits for all work on the device;
 *   - every function returns an abnn_status; no exception crosses the ABI
 *     (the reference threw a *pointer* `new std::exception()` from Brain::load,
 *     brain.cpp:174 -- here that case is ABNN_ERR_SIZE_MISMATCH);
 *   - device pointers returned by abnn_state_ptrs are BORROWED (the handle
 *     owns them), exactly like the unretained MTL::Buffer getters of
 *     brain.h:54-58;
 *   - a handle is not thread-safe: the caller serialises (the reference drove
 *     one Brain from one worker thread, brain-engine.cpp:193-201).
 *
 * Semantics: every pass executes the deterministic legal schedule "C1" of the
 * reference kernel: events in increasing tid order, an
 * ordered global spike budget, all reads of lastFired/clock/rBar observe the
 * pass-start values, stores become visible at pass end.  Timestamps are
 * stored as u64 (README lastFiredNS) and every decision on them is the
 * reference's u32 arithmetic on their low 32 bits (brain.metal:43-45 declare
 * them `uint`): ages `now - ts` wrap at 2^32 (brain.metal:74,80,116),
 * read_outputs and the renormalisation test compare u32 values
 * (brain.cpp:127-128,149-154).
 */
#ifndef ABNN_ABNN_H
#define ABNN_ABNN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ABNN_ABI_VERSION 10

typedef enum abnn_status {
    ABNN_OK = 0,
    ABNN_ERR_INVALID = 1,        /* bad argument / shape                          */
    ABNN_ERR_HIP = 2,            /* a HIP runtime call failed (see abnn_last_error) */
    ABNN_ERR_OOM = 3,            /* device or host allocation failed              */
    ABNN_ERR_SIZE_MISMATCH = 4,  /* .bnn header does not match (brain.cpp:174)    */
    ABNN_ERR_IO = 5,             /* file open/read/write failed                   */
    ABNN_ERR_NO_DEVICE = 6       /* no HIP device / bad ordinal                   */
} abnn_status;

/* SynapsePacked -- brain.metal:11, brain.h:21, README §2.2.  16 bytes, AoS.
 * This is the INTERCHANGE format (upload/download, .bnn, the C++ wrapper).
 * On the device the records are held as arrays (abnn_state):
 * the sweep's gate needs only `src`, held in 24 bits, so it streams 3 B per
 * event instead of 16.  `pad` is not stored; downloads return 0 (the
 * reference never writes or reads it: brain.metal:11, brain-engine.cpp:31-53).
 * N_NRN = n_input + n_output + n_hidden must be below 2^24 - 1 (16,777,215;
 * the reference's configurations reach 5,000,512): abnn_brain_create returns
 * ABNN_ERR_INVALID above. */
typedef struct abnn_synapse {
    uint32_t src;
    uint32_t dst;
    float w;
    float pad; /* always 0, never read (brain.metal:11) */
} abnn_synapse;

/* Sizes fixed at construction: Brain(nInput, nOutput, nHidden, nSynapses,
 * eventsPerPass), brain.h:27-31.  N_NRN = n_input + n_output + n_hidden
 * (brain.cpp:24).  64-bit where the reference used uint32_t (4B synapses). */
typedef struct abnn_dims {
    uint32_t n_input;            /* 256 (constants.h:2)                         */
    uint32_t n_output;           /* 256 (constants.h:3)                         */
    uint64_t n_hidden;           /* 5'000'000 (constants.h:4)                   */
    uint64_t n_syn;              /* synapses held by THIS handle (its shard)    */
    uint64_t events_per_pass;    /* EVENTS_PER_PASS (constants.h:11); visited
                                    events per pass are
                                    min(roundup(events,256), n_syn) (brain.cpp:117,
                                    brain.metal:61) in sweep mode and exactly
                                    events_per_pass in random mode              */
    uint64_t syn_offset;         /* global id of local synapse 0 (sharding; 0)   */
    uint64_t global_events;      /* sum over shards of visited events per pass;
                                    0 = this handle alone (used for the clock
                                    tick rule, brain.metal:61,129)             */
    uint64_t syn_capacity;       /* records this handle may grow to by
                                    synaptogenesis; 0 = n_syn (no growth)     */
} abnn_dims;

/* Every knob of the path with the reference default (abnn_default_params). */
typedef struct abnn_params {
    float base_scale;        /* 0.8f    BASE_SCALE      brain.metal:22 */
    uint32_t refractory;     /* 2       REFRACTORY      brain.metal:23 */
    uint32_t window_pre;     /* 5       WINDOW_PRE      brain.metal:24 */
    uint32_t clock_inc;      /* 1       CLOCK_INC       brain.metal:26 */
    float target_rate_hz;    /* 1000    TARGET_RATE_HZ  brain.metal:28 */
    float eta_home;          /* 1e-6    ETA_HOME        brain.metal:29 */
    float eta_reward;        /* 1e-3    ETA_REWARD      brain.metal:30 */
    float alpha_rbar;        /* 1e-3    ALPHA_RBAR      brain.metal:31 */
    float a_ltp;             /* 0.04f   _aLTP           constants.h:16 */
    float a_ltd;             /* 0.02f   _aLTD           constants.h:17 */
    float w_min;             /* 0.001f  _wMin           constants.h:18 */
    float w_max;             /* 1.0f    _wMax           constants.h:19 */
    uint32_t max_spikes;     /* 2560    kMaxSpikes      brain.h:18     */
    uint32_t tick_ns;        /* 1000    kTickNS         brain.h:17     */
    uint32_t tau_vis;        /* 50000   brain.cpp:102 (bound, unused: brain.metal:47) */
    uint32_t tau_pre;        /* 50000   brain.cpp:102 (bound, unused: brain.metal:48) */
    uint64_t renorm_thresh;  /* 4000000 kRenormThresh   brain.h:19     */
    uint32_t track_visits;   /* 0: lastVisited untouched (reference code,
                                brain.metal:44); 1: lastVisited[dst] = now for
                                every visited event (README §4)        */
    uint32_t mode;           /* ABNN_MODE_SWEEP (the reference code: event t
                                visits synapse t) or ABNN_MODE_RANDOM (README
                                §4, SURVEY §8(a) A14: event t visits a uniform
                                random synapse, below)                 */
    uint64_t seed;           /* seed of the handle's host RNG (inject_inputs)
                                and of the random-mode picks           */
    /* structural plasticity (README §5; build-defined, below) */
    float w_prune;           /* 0: off; updated weight < w_prune removes the synapse */
    float p_new;             /* 0: off; probability that a spike grows a synapse     */
    float w_init;            /* weight of a grown synapse                            */
    uint32_t compact_every;  /* structural update after every N-th pass; 0 = never   */
} abnn_params;

/* Structural plasticity (README §5 "Plasticity & Rewiring"; no reference code,
 * so the build defines it; the CPU oracle restates it):
 *   pruning: an event that reached the weight update and whose stored weight
 *     (random mode: the winning store) is < w_prune removes its synapse: the
 *     record becomes the tombstone {src = dst = 0xFFFFFFFF, w, 0}, which never
 *     passes the pre-spike gate but still counts as a visited event;
 *   synaptogenesis: the spike in global budget slot k of pass p grows a
 *     synapse iff unit24(x) < p_new, x = splitmix64_at(seed ^ ABNN_GENESIS_KEY,
 *     (p << 32) | k) (the generator's SplitMix64, unit24 = top 24 bits / 2^24):
 *     record {src of the firing synapse, n_input + ((x & 0xFFFFFFFF) *
 *     (N_NRN - n_input) >> 32), w_init, 0};
 *   structural update, after every pass whose ticked pass_index is a multiple
 *     of compact_every: the D tombstones are removed -- the array ends at
 *     m = n_syn - D, and the tombstones below m, in index order, take the
 *     live records of the tail [m, n_syn), in index order (only the filled
 *     holes' records move: O(D); ABI 10 -- until ABI 9 the tombstones' span
 *     closed up in order, O(span)); then the synapses grown since the
 *     previous update are appended in (pass, slot) order while n_syn <
 *     syn_capacity.  n_syn and
 *     the visited events change here; the records are compacted in place (no
 *     second buffer), so the borrowed synapse pointer (abnn_state_ptrs) stays
 *     valid.  Sweep-mode event ids stay syn_offset + local index (syn_offset
 *     is fixed). */
#define ABNN_GENESIS_KEY 0xA24BAED4963EE407ull

/* Random-edge mode (README §4 "pick a random synapse"; no reference code, so
 * the build defines it):
 *   E = events_per_pass events per pass; event t (local index) visits record
 *   e(t) = mulhi64(x, n_syn), x = (out[1] << 32) | out[0] of
 *   Philox4x32-10(counter = {t_lo, t_hi, pass_lo, pass_hi},
 *                 key = {seed_lo ^ off_lo, seed_hi ^ off_hi}),
 *   pass = abnn_scalars.pass_index, off = abnn_dims.syn_offset (a shard picks
 *   within its own records, with its own stream).
 *   Gates, budget, candidate test (rand01((u32)(syn_offset + t) ^ now)) and
 *   stamps follow schedule C1 with t as the event id.  Every event reads the
 *   pass-start record; when several events that reached the update picked
 *   the same synapse, the weight stored is the one computed by the highest
 *   event index (a legal serialisation of the racy kernel: all reads before
 *   all writes, writes in event order).                                      */
#define ABNN_MODE_SWEEP 0u
#define ABNN_MODE_RANDOM 1u

/* Scalar state (brain.cpp:57-60): clock, reward, running-average reward,
 * plus the pass counter that keys the random-mode picks. */
typedef struct abnn_scalars {
    uint64_t clock;          /* u64 storage; decisions use its low 32 bits (the
                                reference's u32 clock, brain.cpp:57)          */
    float reward;
    float rbar;
    uint64_t pass_index;     /* passes run by this handle (+1 per pass; not
                                reset by renormalisation or reset_stats)    */
} abnn_scalars;

/* Cumulative per-handle pass statistics (for the roofline byte count). */
typedef struct abnn_stats {
    uint64_t passes;
    uint64_t events;         /* E: visited events                        */
    uint64_t pre_gated;      /* G1: passed the pre-spike gate (brain.metal:73-77) */
    uint64_t post_gated;     /* passed the refractory gate (brain.metal:79-83)   */
    uint64_t updated;        /* G2: reached the weight update (budget > 0)       */
    uint64_t fired;          /* F: spikes emitted (lastFired stamps)             */
    uint64_t pruned;         /* synapses removed (tombstoned)                    */
    uint64_t grown;          /* synapses appended by structural updates          */
} abnn_stats;

/* Borrowed device pointers (brain.h:54-58 buffer getters).  The neuron state
 * and the scalars are plain arrays (u64 timestamps, README lastFiredNS; every
 * decision takes their low 32 bits, as the reference's `uint` arithmetic,
 * brain.metal:43-45,74,80,116).  The synapse records (bufSyn_) are held in a
 * kernel-specific device layout: `synapses` is opaque.  Read and write
 * records through abnn_upload_synapses / abnn_download_synapses (the
 * SynapsePacked interchange format), or describe the layout with
 * abnn_synapse_layout (versioned separately from the ABI: a layout change
 * does not change this header).  Taking the pointers makes every later pass
 * rebuild the recent-spike bitmap from lastFired (the caller may write it
 * behind the handle's back). */
typedef struct abnn_state {
    void* synapses;          /* opaque: the device record arrays (abnn_synapse_layout) */
    uint64_t* last_fired;    /* N_NRN (bufLastFire_)                     */
    uint64_t* last_visited;  /* N_NRN (bufLastVisit_)                    */
    uint64_t* clock;         /* 1 (bufClock_)                            */
    float* reward;           /* 1 (bufReward_)                           */
    float* rbar;             /* 1 (bufRBar_)                             */
} abnn_state;

/* The device record layout behind abnn_state.synapses, for tools that must
 * address it directly (profilers, debuggers, custom kernels).  `version`
 * names the layout (DESIGN.md §4 documents each; ABNN_LAYOUT_VERSION is the
 * one this library writes); arrays[i] = {device pointer, bytes, element
 * bytes, name}.  A caller that does not know `version` must not touch them. */
#define ABNN_LAYOUT_VERSION 4
#define ABNN_LAYOUT_MAX_ARRAYS 4
typedef struct abnn_array_desc {
    void* ptr;
    uint64_t bytes;
    uint32_t elem_bytes;
    char name[20];
} abnn_array_desc;
typedef struct abnn_layout {
    uint32_t version;
    uint32_t n_arrays;
    abnn_array_desc arrays[ABNN_LAYOUT_MAX_ARRAYS];
} abnn_layout;

typedef struct abnn_brain abnn_brain;

/* ---- library ------------------------------------------------------------ */
int abnn_abi_version(void);
const char* abnn_status_string(abnn_status s);
/* Last error message of the calling thread (empty string if none). */
const char* abnn_last_error(void);
/* Reference defaults for every knob (brain.metal:22-31, constants.h:16-19,
 * brain.h:17-19, brain.cpp:102). */
void abnn_default_params(abnn_params* out);
/* Number of HIP devices visible (0 without a GPU; never fails). */
int abnn_device_count(void);

/* ---- lifetime: Brain::Brain + build_pipeline + build_buffers -------------
 * brain.cpp:21-26 (ctor), brain.cpp:38-48 (build_pipeline: kernels are
 * compiled in, nothing to build), brain.cpp:52-69 (build_buffers: allocate
 * and zero; budget = kMaxSpikes; reward = rBar = 0; clock = 0).            */
abnn_status abnn_brain_create(const abnn_dims* dims, const abnn_params* params,
                              int device, abnn_brain** out);
/* ~Brain / release_all, brain.cpp:27-34. */
abnn_status abnn_brain_destroy(abnn_brain* b);
abnn_status abnn_get_dims(const abnn_brain* b, abnn_dims* out);
abnn_status abnn_get_params(const abnn_brain* b, abnn_params* out);
abnn_status abnn_state_ptrs(abnn_brain* b, abnn_state* out);
abnn_status abnn_synapse_layout(abnn_brain* b, abnn_layout* out);
/* n_neuron() = n_input + n_output + n_hidden (brain.h:51). */
uint64_t abnn_n_neuron(const abnn_brain* b);

/* ---- synapses ------------------------------------------------------------ */
/* Host -> device copy of records [first, first+n) (the reference wrote the
 * Managed buffer directly, brain-engine.cpp:37-52). */
abnn_status abnn_upload_synapses(abnn_brain* b, uint64_t first,
                                 const abnn_synapse* src, uint64_t n);
abnn_status abnn_download_synapses(abnn_brain* b, uint64_t first,
                                   abnn_synapse* dst, uint64_t n);
/* Synthetic graph with the recipe of build_random_graph (brain-engine.cpp:31-53)
 * and this library's portable counter-based RNG: global record
 * i < n_input*n_output is the dense block {i/n_out, n_in + i%n_out,
 * w~U(0.4,0.8)}; the rest {src,dst ~ U[n_in+n_out, N_NRN-1], w~U(0.1,0.2)}.
 * Generated on the device, shard-aware (uses syn_offset).                   */
abnn_status abnn_generate_synapses(abnn_brain* b, uint64_t seed);
/* Order-sensitive 64-bit checksum of the local synapse array (device-side). */
abnn_status abnn_checksum_synapses(abnn_brain* b, uint64_t* out);

/* ---- neuron timestamps / scalars ----------------------------------------- */
abnn_status abnn_get_last_fired(abnn_brain* b, uint64_t first, uint64_t* out, uint64_t n);
abnn_status abnn_set_last_fired(abnn_brain* b, uint64_t first, const uint64_t* src, uint64_t n);
abnn_status abnn_get_last_visited(abnn_brain* b, uint64_t first, uint64_t* out, uint64_t n);
abnn_status abnn_set_last_visited(abnn_brain* b, uint64_t first, const uint64_t* src, uint64_t n);
/* (A shard's abnn_set_last_visited clears the visit marks of what it writes,
 * and a write of [0, N_NRN) leaves none unmerged.  Writes through the
 * abnn_state_ptrs pointers bypass the marks and the host's bookkeeping: use
 * the setters on sharded brains.) */
/* lastFired[idx[i]] = value for i < n (teacher / input spikes written by the
 * host, brain.cpp:82, brain-engine.cpp:131). */
abnn_status abnn_set_timestamps(abnn_brain* b, const uint32_t* idx, uint64_t n, uint64_t value);
abnn_status abnn_get_scalars(abnn_brain* b, abnn_scalars* out);
abnn_status abnn_set_scalars(abnn_brain* b, const abnn_scalars* in);
/* *reward = r (brain-engine.cpp:180-182). */
abnn_status abnn_set_reward(abnn_brain* b, float r);

/* ---- pass-boundary hooks --------------------------------------------------
 * Brain::inject_inputs(vals, hz), brain.cpp:73-83: for every input i,
 * lastFired[i] = clock when uni() < hz*kTickNS*NSEC_PER_SEC * v[i]; uni() is
 * the handle's seeded host RNG (params.seed) instead of a random_device mt19937.
 * n must equal n_input (the reference asserts it, brain.cpp:75).            */
abnn_status abnn_inject_inputs(abnn_brain* b, const float* v, uint32_t n, float hz);
/* Brain::read_outputs(), brain.cpp:145-157: out[o] = 1 iff
 * ts = lastFired[n_input+o] != 0 && start <= ts < now, start = now>1 ? now-1 : 0.
 * n must equal n_output.                                                     */
abnn_status abnn_read_outputs(abnn_brain* b, uint8_t* out, uint32_t n);
/* Stamp lastFired[first, first+count) = clock at the start of EVERY pass
 * (fused into the pass; the bench stimulus of SURVEY §8d).  count = 0 = off. */
abnn_status abnn_set_auto_stimulus(abnn_brain* b, uint64_t first, uint64_t count);

/* ---- passes: Brain::encode_traversal + commit/wait ------------------------
 * brain.cpp:87-141 + brain-engine.cpp:136-141.  Enqueues `passes` whole C1
 * passes (traversal + clock tick + renormalisation when the pass-start clock
 * exceeds renorm_thresh) on `stream` (NULL = the default stream).  Returns
 * without waiting; abnn_synchronize waits for `stream` and the device.       */
abnn_status abnn_traverse(abnn_brain* b, uint32_t passes, void* stream);
abnn_status abnn_synchronize(abnn_brain* b, void* stream);

/* ---- sharded passes (synapse-shard data parallelism) --------
 * One pass on rank r of W = three calls around ONE exchange:
 *   abnn_shard_gate   -> writes this shard's exchange record to `xchg_dev`
 *                        (abnn_exchange_bytes(b) bytes): ABNN_SUMMARY_WORDS
 *                        int64 {spike candidates capped at the budget, global
 *                        event 0 reached the update, visited events, passed the
 *                        refractory gate}, then the shard's spikes (dst, int32)
 *                        in local budget order, max_spikes slots (padded to 8 B);
 *   [all-gather the W records, rank order, into `gathered_dev`]
 *   abnn_shard_apply  -> weight updates of this shard's events that fall inside
 *                        the global budget (offset = capped sum of lower ranks);
 *   abnn_shard_commit -> stamps every shard's spikes in rank order (= global
 *                        budget order, the first max_spikes), updates rBar,
 *                        ticks the clock, renormalises if due.
 * All pointers are device pointers; the exchange is the caller's (RCCL via
 * torch.distributed in abnn_amd/shard.py).  W = 1 with the local record is
 * exactly abnn_traverse.                                                     */
#define ABNN_SUMMARY_WORDS 4
uint64_t abnn_exchange_bytes(const abnn_brain* b);
/* abnn_dims.global_events after the shards' record counts changed (structural
 * updates): the visited events of all shards per pass (the clock-tick rule,
 * brain.metal:61,129).  The caller sums the shards' visited events (an
 * all-reduce) and sets it on every rank.                                    */
abnn_status abnn_set_global_events(abnn_brain* b, uint64_t global_events);
abnn_status abnn_shard_gate(abnn_brain* b, void* xchg_dev, void* stream);
abnn_status abnn_shard_apply(abnn_brain* b, const void* gathered_dev, uint32_t world,
                             uint32_t rank, void* stream);
abnn_status abnn_shard_commit(abnn_brain* b, const void* gathered_dev, uint32_t world,
                              void* stream);

/* The lastVisited merge of a sharded brain with track_visits.
 * Unsharded, lastVisited[n] holds the last value written: the clock of the
 * last pass that visited n, or what the host wrote after it.  Each shard
 * marks the neurons its passes visit; between merges the clock only moves
 * forward (abnn_set_scalars refuses to move it back over unmerged visits, and
 * abnn_shard_traverse merges after every renormalisation), so the shard that
 * visited n last wrote the largest value:
 *   abnn_shard_visits_delta -> delta_dev[i] = visited since the last merge ?
 *                              lastVisited[i] + 1 : 0   (u64 x N_NRN, device)
 *   [all-reduce(MAX) of the deltas over the shards]
 *   abnn_shard_visits_merge -> lastVisited[i] = reduced[i] - 1 where reduced[i]
 *                              != 0; every mark clears.
 * A caller driving the shard phases itself merges whenever
 * abnn_renormalisations changed after a pass, and before reading lastVisited
 * (abnn_comm_sync_visits does all three steps over RCCL).  Host writes
 * (abnn_set_last_visited, abnn_load_flat) must be the same on every shard;
 * they clear the marks of what they write.  Without track_visits both calls
 * are no-ops (delta = 0).                                                    */
abnn_status abnn_shard_visits_delta(abnn_brain* b, void* delta_dev, void* stream);
abnn_status abnn_shard_visits_merge(abnn_brain* b, const void* reduced_dev, void* stream);
/* Renormalisations run by this handle (host-side count, no synchronisation). */
uint64_t abnn_renormalisations(const abnn_brain* b);

/* Spike budget left by the last pass: max_spikes minus the spikes it emitted
 * (the reference's bufBudget_ after a pass, brain.h:58; the host resets it to
 * kMaxSpikes before every pass, brain.cpp:90, here the max_spikes knob; C1 never
 * lets it wrap).  max_spikes before the first pass (brain.cpp:66). */
abnn_status abnn_get_budget(abnn_brain* b, uint32_t* remaining);
/* Structural updates run by this handle (host-side count, no synchronisation):
 * a sharded caller re-sums abnn_dims.global_events when it changes. */
uint64_t abnn_structural_updates(const abnn_brain* b);

/* ---- buffer-index launcher (the reference's kernel ABI) ---------------------
 * monte_carlo_traversal's 14 buffers (brain.metal:42-58, bound by
 * Brain::encode_traversal at brain.cpp:93-118) as CALLER-OWNED device memory
 * in the reference's own layouts: 16-B SynapsePacked records and u32
 * lastF / clock / budget (brain.cpp:54-60).  One call enqueues one pass of
 * schedule C1 over the first min(roundup(events,256), n_syn) records on
 * `stream`: gates, ordered budget (the first *budget spike candidates fire;
 * *budget is left at the remainder), STDP + reward + homeostasis, write-back
 * (the whole 16-B record, brain.metal:122), deferred stamps, rBar and one
 * clock tick.  The knobs the reference compiles in (#define BASE_SCALE ...,
 * brain.metal:22-31) come from `knobs` (NULL = the reference defaults; only
 * the #define fields are read -- aLTP..wMax are the buffer arguments).
 * Scratch: `workspace` of device memory (any contents on first use; reused
 * every pass: it carries the pass's adaptive partition and look-back epoch),
 * 16-B aligned: abnn_traversal_workspace_bytes(n_syn, events) is the
 * recommended size (~61 MB at config 3: a bounded pool of refractory
 * survivors, 1/64 of the visited events, plus per-1024-event counters),
 * abnn_traversal_workspace_min_bytes the least accepted (no pool).  Survivors
 * that do not fit the pool are recomputed from the records (slower, same
 * results).  The spikes are stamped after the pass's last lastF read from a
 * list of min(events, 65536) entries; a pass with more spikes than that
 * stamps the rest directly, which may land before another workgroup's lastF
 * reads (the fused pass), or (the five-launch pass) before a recomputed
 * group's when survivors also overflowed the pool -- such a pass is reported
 * by abnn_traversal_workspace_error (1); the host's kMaxSpikes = 2560,
 * brain.cpp:90, never comes near it.  This is the reference's memory
 * layout, so it streams 16 B per visited event; the pre-spike test is
 * answered from an LDS filter of lastF, which is gathered only for the ~1 %
 * of events the filter passes (the handle API's layout moves
 * 3 B per event).
 * The single-launch pass after the filter keeps one workgroup per CU resident
 * for the whole pass (its look-back waits on every other workgroup): run it
 * with the device to itself -- not beside another stream's persistent kernels
 * (a second handle's pass, RCCL) -- or select the five-launch pass
 * (ABNN_RAW_FUSED=0), and check abnn_traversal_workspace_error now and then:
 * a starved pass is not hung but reported there (2).
 * renormalise_clock_and_times (brain.metal:135-145) on the same buffers:
 * lastF[i] -= *clock for i < n_nrn, then *clock = 0 (the host decides when,
 * brain.cpp:127-128).                                                         */
typedef struct abnn_traversal_args {
    abnn_synapse* syn;          /* buffer(0)  SynapsePacked[n_syn]           rw */
    uint32_t* last_fired;       /* buffer(1)  atomic_uint lastF[n_nrn]       rw */
    uint32_t* last_visited;     /* buffer(2)  unused (brain.metal:44)           */
    uint32_t* clock;            /* buffer(3)  atomic_uint                    rw */
    uint32_t n_syn;             /* buffer(4)                                    */
    uint32_t tau_vis, tau_pre;  /* buffer(5,6) unused (brain.metal:47-48)       */
    float a_ltp, a_ltd;         /* buffer(7,8)                                  */
    float w_min, w_max;         /* buffer(9,10)                                 */
    uint32_t* budget;           /* buffer(11) atomic_uint                    rw */
    const float* reward;        /* buffer(12)                                   */
    float* rbar;                /* buffer(13) atomic_float                   rw */
    uint32_t n_nrn;             /* lastF length (src/dst >= n_nrn never pass)    */
    uint32_t events;            /* EVENTS_PER_PASS: grid roundup(events,256)    */
    const abnn_params* knobs;   /* #define knobs, NULL = reference defaults     */
    void* workspace;            /* device scratch                               */
    uint64_t workspace_bytes;
} abnn_traversal_args;
uint64_t abnn_traversal_workspace_bytes(uint32_t n_syn, uint32_t events);
uint64_t abnn_traversal_workspace_min_bytes(uint32_t n_syn, uint32_t events);
/* synchronises `stream`: 1 if any pass on this workspace since the last call
 * (or since its first launch) stamped directly where that may race (see
 * above), 2 if a pass's look-back wait gave up (never expected:
 * every workgroup of the pass is resident), else 0; the flag is sticky until
 * this call reads and clears it, so one check after many passes sees every
 * pass */
abnn_status abnn_traversal_workspace_error(const void* workspace, uint32_t* err, void* stream);
abnn_status abnn_launch_traversal(const abnn_traversal_args* a, void* stream);
abnn_status abnn_launch_renormalise(uint32_t* last_fired, uint32_t* last_visited, uint32_t* clock,
                                    uint32_t n_nrn, void* stream);

/* ---- sharded passes driven from C over RCCL ---------------------------------
 * One process per GPU (xGMI), one communicator per shard handle.  The
 * library's own RCCL communicator (RCCL = NCCL on ROCm; the one already
 * loaded in the process, e.g. by torch, else librccl.so.1): one rank calls
 * abnn_comm_unique_id, every rank gets those ABNN_COMM_ID_BYTES bytes (any
 * channel: torch.distributed broadcast, a file, MPI) and calls
 * abnn_comm_create.  abnn_shard_traverse then enqueues `passes` whole sharded
 * passes on `stream` -- per pass: abnn_shard_gate, ONE ncclAllGather of the
 * exchange records (in place, on the stream), abnn_shard_apply,
 * abnn_shard_commit -- with no host round trip except after a structural
 * update (an all-reduce of the shards' visited events for the clock-tick
 * rule, then abnn_set_global_events) and, with track_visits, the lastVisited
 * merge after every renormalisation (above).  abnn_comm_sync_visits is that
 * merge on demand (lastVisited is never read by a decision, brain.metal:44;
 * merge before reading or saving it).
 * An error on any rank (a failed launch or collective, a pass error flag)
 * leaves the other ranks inside the pass's collectives: the communicator is
 * then marked unusable (every later abnn_shard_traverse on it returns
 * ABNN_ERR_INVALID) and the caller must abort / destroy it on every rank, as
 * after any NCCL error. */
#define ABNN_COMM_ID_BYTES 128
typedef struct abnn_comm abnn_comm;
abnn_status abnn_comm_unique_id(void* id_out);
abnn_status abnn_comm_create(const void* id, uint32_t world, uint32_t rank, int device, abnn_comm** out);
abnn_status abnn_comm_destroy(abnn_comm* c);
abnn_status abnn_shard_traverse(abnn_brain* b, abnn_comm* c, uint32_t passes, void* stream);
abnn_status abnn_comm_sync_visits(abnn_brain* b, abnn_comm* c, void* stream);

/* In-process communicator group: `world` ranks in ONE process, one host
 * thread per rank, each calling abnn_shard_traverse / abnn_comm_sync_visits
 * on its own shard handle with the communicator of abnn_comm_create_local
 * (the same calls, in the same order, on every rank -- as with RCCL).  The
 * collectives are device copies and a reduction kernel on each rank's stream
 * between host barriers (no RCCL): the sharded pass at world > 1 on ONE GPU
 * (k handles share the device), or over several GPUs of one process.  Ranks
 * on one device must pass the same stream (a pass keeps one workgroup per CU
 * resident: two must not run at once); a rank that fails, or one that does
 * not reach a collective within 300 s, breaks the group and every rank's
 * next collective fails (ABNN_ERR_INVALID).  Destroy every rank's
 * communicator before the group.                                             */
typedef struct abnn_comm_group abnn_comm_group;
abnn_status abnn_comm_group_create(uint32_t world, abnn_comm_group** out);
abnn_status abnn_comm_group_destroy(abnn_comm_group* g);
abnn_status abnn_comm_create_local(abnn_comm_group* g, uint32_t rank, int device, abnn_comm** out);

/* ---- statistics / timing ---------------------------------------------------- */
abnn_status abnn_get_stats(abnn_brain* b, abnn_stats* out);   /* synchronises */
abnn_status abnn_reset_stats(abnn_brain* b);
/* every > 0: HIP events around the gate (streaming) kernel, on the stream it
 * is launched on, for every launch (every = 1) or every `every`-th launch
 * starting with the second after this call (an event pair costs stream time,
 * so sampling keeps it out of the rate; the first launch is skipped because
 * it is the one most likely to carry a transient); 0: off.
 * abnn_get_kernel_time returns the summed milliseconds and the count of timed
 * launches since the last call; abnn_get_kernel_times the same launches one by
 * one (up to `cap` of them into out_ms; *launches = how many were timed).
 * Either call resets the record.                                            */
abnn_status abnn_enable_timing(abnn_brain* b, int every);
abnn_status abnn_get_kernel_time(abnn_brain* b, double* ms_total, uint64_t* launches);
abnn_status abnn_get_kernel_times(abnn_brain* b, float* out_ms, uint64_t cap, uint64_t* launches);

/* ---- persistence ------------------------------------------------------------
 * .bnn = u32 N_SYN, u32 N_NRN, N_SYN x 16-B SynapsePacked (Brain::save/load,
 * brain.cpp:161-178).  Load of a mismatched header -> ABNN_ERR_SIZE_MISMATCH.  */
abnn_status abnn_save_bnn(abnn_brain* b, const char* path);
abnn_status abnn_load_bnn(abnn_brain* b, const char* path);
/* README §2 flat buffer: 16-B header {u32 N_SYN, u32 N_NRN, 8 B pad},
 * synapses (u32 src, u32 dst) x N_SYN, weights f32 x N_SYN,
 * lastFiredNS u64 x N_NRN, lastVisitedNS u64 x N_NRN.                         */
abnn_status abnn_save_flat(abnn_brain* b, const char* path);
abnn_status abnn_load_flat(abnn_brain* b, const char* path);

#ifdef __cplusplus
} /* extern "C" */
#endif
#endif /* ABNN_ABNN_H */
