// capi.hip -- implementation of the C-ABI (include/abnn/abnn.h) over the HIP
// kernels of kernels.hip.  Replaces the Metal host class Brain
// (abnn/src/core/brain/brain.{h,cpp}); each function cites what it replaces.
#include <dlfcn.h>
#include <link.h>
#include <rccl/rccl.h>  // types only: the entry points are resolved at run time (rccl_api)

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "engine.h"

using namespace abnn;

namespace {

thread_local std::string g_err;

void set_err(const std::string& m) { g_err = m; }

#define HIP_TRY(expr)                                                                  \
    do {                                                                               \
        hipError_t _e = (expr);                                                        \
        if (_e != hipSuccess) {                                                        \
            set_err(std::string(#expr) + ": " + hipGetErrorString(_e));                \
            return ABNN_ERR_HIP;                                                       \
        }                                                                              \
    } while (0)

#define REQUIRE(cond, msg)                                                             \
    do {                                                                               \
        if (!(cond)) {                                                                 \
            set_err(msg);                                                              \
            return ABNN_ERR_INVALID;                                                   \
        }                                                                              \
    } while (0)

uint64_t visited_events(const abnn_dims& d, uint32_t mode)
{
    if (mode == ABNN_MODE_RANDOM) return d.n_syn ? d.events_per_pass : 0;  // README §4: EVENTS picks
    uint64_t grid = (d.events_per_pass + 255u) / 256u * 256u;  // brain.cpp:116-118
    return grid < d.n_syn ? grid : d.n_syn;                     // brain.metal:61
}

struct EventPair {
    hipEvent_t a, b;
};

}  // namespace

struct abnn_brain {
    abnn_dims dims{};
    abnn_params params{};
    KernelParams kp{};
    int device = 0;
    hipStream_t stream = nullptr;  // default stream of state accessors (the null stream)
    uint64_t n_nrn = 0;
    DeviceState d{};
    void* scalar_block = nullptr;  // clock | reward | rbar
    uint64_t clock_host = 0;       // mirror, for the renormalisation decision (brain.cpp:127)
    uint64_t rng = 0;              // host RNG of inject_inputs
    uint64_t stim_first = 0, stim_count = 0;
    // steady-state bitmap build by k_apply (build_next_ok): consecutive
    // single-GPU passes whose spike lists are in fired_ring with no clock
    // discontinuity, the highest lastFired value the host wrote (creation's
    // zeros included), the stimulus of the last kFiredRing passes, whether
    // the next pass's bitmap was built (and for which stimulus), borrowed
    // state pointers handed out.  Bitmap and images are triple-buffered by
    // pass % 3: read by pass p, built by pass p - 1, zeroed by pass p - 2.
    uint64_t clean_passes = 0, max_host_stamp = 0;
    uint64_t stim_ring[kFiredRing][2] = {};
    bool next_built = false;
    uint64_t built_stim[2] = {};
    bool ext_ptrs = false, force_full_bitmap = false;
    uint32_t* bitmap_buf[3] = {};
    uint32_t* filter_buf[3] = {};
    // fused single-GPU sweep passes (ABNN_FUSED=0: gate + apply launches):
    // whether the previous pass was fused (its gate costs are in cost_buf[cost
    // parity ^ 1] and its prologue adapts the partition), the look-back words
    bool use_fused = true, last_pass_fused = false;
    uint32_t* cost_buf[2] = {};
    uint32_t cost_parity = 0;
    bool pending_renorm = false;   // shard protocol: decided at gate time
    int timing = 0;                // time every timing-th gate launch (0: off)
    uint64_t timing_count = 0;
    std::vector<EventPair> events;
    size_t events_used = 0;
    uint32_t* idx_scratch = nullptr;
    uint64_t idx_cap = 0;
    uint64_t* u64_scratch = nullptr;
    int cus = 256, per_cu = 1;     // gate partition inputs (configure)
    uint64_t pass_host = 0;        // mirror of pass_index (structural-update schedule)
    uint64_t rot = 0;              // passes run by this handle: the bitmap buffers' rotation (never reset)
    // structural updates (compact_every > 0, in place: kernels.hip
    // launch_structural_update): the hole blocks' ranks (k_swap_scan2), the
    // scan's per-slice sums, the tail blocks' live prefix (k_swap_tail)
    uint64_t* compact_offsets = nullptr;
    uint64_t* swap_part = nullptr;
    uint64_t* swap_toff = nullptr;
    unsigned long long* span_words = nullptr;  // the update's device words (kernels.hip k_span_init)
    uint32_t* grown_cnt = nullptr;             // used grown slots per 1024-slot block (k_grown_counts)
    uint64_t structural_updates = 0;  // run so far (abnn_structural_updates)
    uint64_t last_pass = ~0ull;       // pass_index of the last pass (its spike list: abnn_get_budget)
    // host-mapped error word: a fused pass whose look-back wait gave up sets it
    // (kernels.hip wg_poll); abnn_traverse sees it without synchronising
    uint32_t* err_host = nullptr;
    // a sharded pass on the fused path: its first launch (k_gate in shard
    // mode) ran, k_shard_walk follows the exchange (abnn_shard_apply)
    bool pending_walk = false;
    // the sharded lastVisited merge: a track_visits shard marks
    // the neurons it visits (d.visit_mark); marks_dirty = a pass ran since the
    // last merge or host write of lastVisited
    bool marks_dirty = false;
    uint64_t renorms = 0;  // renormalisations run (abnn_renormalisations)
    // a structural update that failed part-way left the records invalid (the
    // compaction works in place): every pass is refused until they are
    // reloaded (abnn_load_bnn / abnn_load_flat / abnn_generate_synapses / an
    // upload of every record)
    bool records_invalid = false;
};

namespace {

// Pass functions run on the caller's stream (NULL = the default stream).
hipStream_t pick(abnn_brain*, void* s) { return static_cast<hipStream_t>(s); }

// A fused pass whose look-back wait gave up (never expected: every gate
// workgroup is resident, checked at create) reports it once, here, instead of
// hanging the GPU; the word is re-armed, so only that failure is reported.
abnn_status pass_error(abnn_brain* b)
{
    if (!b->err_host || __atomic_load_n(b->err_host, __ATOMIC_ACQUIRE) == 0) return ABNN_OK;
    __atomic_store_n(b->err_host, 0u, __ATOMIC_RELEASE);
    set_err("fused pass: a look-back wait timed out; the state after that pass is invalid "
            "(reload it: abnn_load_bnn / abnn_load_flat)");
    return ABNN_ERR_HIP;
}

// State accessors are synchronous: they wait for all work on the handle's
// device (whatever stream it was enqueued on), then copy on the default stream.
abnn_status sync_all(abnn_brain* b)
{
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipDeviceSynchronize());
    return pass_error(b);
}

void free_all(abnn_brain* b)
{
    if (!b) return;
    (void)hipSetDevice(b->device);
    void* ptrs[] = {b->d.syn.lo,    b->d.syn.hi,     b->d.syn.dw,     b->d.syn.src32,
                    b->d.last_fired, b->d.last_visited, b->d.visit_mark, b->scalar_block,
                    b->bitmap_buf[0], b->bitmap_buf[1], b->bitmap_buf[2], b->filter_buf[0], b->filter_buf[1],
                    b->filter_buf[2], b->cost_buf[0], b->cost_buf[1], b->d.lb_status, b->d.cand_list,
                    b->d.range_info,    b->d.range_g1,  b->d.g2x,
                    b->d.chunk_cnt,
                    b->d.wg_stats, b->d.claim,  b->d.g2src,      b->d.grown,
                    b->d.dead,      b->compact_offsets, b->swap_part, b->swap_toff, b->span_words, b->grown_cnt,
                    b->d.work,      b->idx_scratch,
                    b->u64_scratch,  b->d.wave_clock,  b->d.apply_clock, b->d.fired_ring, b->d.n_fired_ring, b->d.range_bounds,  b->d.range_bounds_next, b->d.range_bounds_prev,
                    const_cast<uint32_t*>(b->d.dummy)};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (auto& e : b->events) {
        (void)hipEventDestroy(e.a);
        (void)hipEventDestroy(e.b);
    }
    if (b->err_host) (void)hipHostFree(b->err_host);
}

template <typename T>
abnn_status dalloc(T** p, uint64_t count)
{
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
    if (e != hipSuccess) {
        *p = nullptr;
        set_err(std::string("hipMalloc(") + std::to_string(count * sizeof(T)) + " B): " +
                hipGetErrorString(e));
        return ABNN_ERR_OOM;
    }
    e = hipMemset(*p, 0, count * sizeof(T));
    if (e != hipSuccess) {
        set_err(std::string("hipMemset: ") + hipGetErrorString(e));
        return ABNN_ERR_HIP;
    }
    return ABNN_OK;
}

#define ST_TRY(expr)                        \
    do {                                    \
        abnn_status _s = (expr);            \
        if (_s != ABNN_OK) return _s;       \
    } while (0)

abnn_status ensure_idx_scratch(abnn_brain* b, uint64_t n)
{
    if (n <= b->idx_cap) return ABNN_OK;
    if (b->idx_scratch) (void)hipFree(b->idx_scratch);
    b->idx_scratch = nullptr;
    b->idx_cap = 0;
    ST_TRY(dalloc(&b->idx_scratch, n));
    b->idx_cap = n;
    return ABNN_OK;
}

// Device records are the packed src streams, dst and w (SynArrays, engine.h);
// abnn_synapse is the host interchange format.  Capacity `count` records.
abnn_status alloc_syn(SynArrays* a, uint64_t count, bool random_mode)
{
    ST_TRY(dalloc(&a->lo, count));
    ST_TRY(dalloc(&a->hi, hi_bytes(count)));
    if (random_mode) ST_TRY(dalloc(&a->src32, count));
    return dalloc(&a->dw, count);
}

// src values of records [first, first + m) <-> host u32 (interchange form),
// through a device staging buffer and the pack / unpack kernels.
struct SrcStage {
    uint32_t* dev = nullptr;
    ~SrcStage() { if (dev) (void)hipFree(dev); }
};

// Chunked copies between device arrays [first, first + n) and host records.
constexpr uint64_t kXferRecs = 1u << 22;

abnn_status records_d2h(const SynArrays& a, uint64_t first, uint64_t n, abnn_synapse* out)
{
    std::vector<uint32_t> s;
    std::vector<uint2> dw;
    SrcStage st;
    if (n) ST_TRY(dalloc(&st.dev, std::min<uint64_t>(kXferRecs, n)));
    for (uint64_t i = 0; i < n; i += kXferRecs) {
        const uint64_t m = std::min<uint64_t>(kXferRecs, n - i);
        s.resize(m);
        dw.resize(m);
        HIP_TRY(launch_unpack_src(a, st.dev, first + i, m, nullptr));
        HIP_TRY(hipMemcpy(s.data(), st.dev, m * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(dw.data(), a.dw + first + i, m * 8, hipMemcpyDeviceToHost));
        for (uint64_t k = 0; k < m; ++k) {
            float w;
            std::memcpy(&w, &dw[k].y, 4);
            out[i + k] = {s[k], dw[k].x, w, 0.0f};
        }
    }
    return ABNN_OK;
}

abnn_status records_h2d(const SynArrays& a, uint64_t first, uint64_t n, const abnn_synapse* in)
{
    std::vector<uint32_t> s;
    std::vector<uint2> dw;
    SrcStage st;
    if (n) ST_TRY(dalloc(&st.dev, std::min<uint64_t>(kXferRecs, n)));
    for (uint64_t i = 0; i < n; i += kXferRecs) {
        const uint64_t m = std::min<uint64_t>(kXferRecs, n - i);
        s.resize(m);
        dw.resize(m);
        for (uint64_t k = 0; k < m; ++k) {
            s[k] = in[i + k].src;
            dw[k].x = in[i + k].dst;
            std::memcpy(&dw[k].y, &in[i + k].w, 4);
        }
        HIP_TRY(hipMemcpy(st.dev, s.data(), m * 4, hipMemcpyHostToDevice));
        HIP_TRY(launch_pack_src(a, st.dev, first + i, m, nullptr));
        HIP_TRY(hipDeviceSynchronize());  // the staging buffer is reused
        HIP_TRY(hipMemcpy(a.dw + first + i, dw.data(), m * 8, hipMemcpyHostToDevice));
    }
    return ABNN_OK;
}

// Every record names two neurons, or is the pruning tombstone {src = dst =
// 0xFFFFFFFF} that downloads, .bnn and flat saves of a pruned brain hold
// between structural updates (abnn.h; k_pack_src maps it to kSrcNone).
abnn_status validate_records(const abnn_brain* b, const abnn_synapse* s, uint64_t n)
{
    for (uint64_t i = 0; i < n; ++i)
        if ((s[i].src >= b->n_nrn || s[i].dst >= b->n_nrn) &&
            !(s[i].src == 0xFFFFFFFFu && s[i].dst == 0xFFFFFFFFu)) {
            set_err("synapse " + std::to_string(i) + " has src/dst >= N_NRN (" +
                    std::to_string(b->n_nrn) + ")");
            return ABNN_ERR_INVALID;
        }
    return ABNN_OK;
}

// Host-written records may hold tombstones (a saved pruned brain): recount the
// structural update's per-block tally over them (structural updates on only:
// d.dead exists when compact_every > 0).
abnn_status retally(abnn_brain* b, uint64_t first, uint64_t n)
{
    if (!b->d.dead || n == 0) return ABNN_OK;
    HIP_TRY(launch_tally_dead(b->d.syn, b->dims.n_syn, b->d.dead, first, n, nullptr));
    HIP_TRY(hipDeviceSynchronize());
    return ABNN_OK;
}

uint64_t tick_events(const abnn_brain* b)
{
    return b->dims.global_events ? b->dims.global_events : b->d.events;
}

// renormalise_if_needed (brain.cpp:127-128) on the pass-start clock: the
// reference's clock is a u32, so the test is on its low 32 bits
bool renorm_due(const abnn_brain* b) { return (uint64_t)(uint32_t)b->clock_host > b->params.renorm_thresh; }

constexpr const char* kRecordsInvalid =
    "a failed structural update left the records invalid: reload them (abnn_load_bnn / abnn_load_flat / "
    "abnn_generate_synapses / abnn_upload_synapses of every record) before the next pass";

// A shard that tracks visits keeps per-neuron visit marks for the lastVisited
// merge; allocated at creation when global_events is set, else
// by the first sharded pass (zeros: nothing visited yet).
abnn_status ensure_visit_marks(abnn_brain* b)
{
    if (!b->params.track_visits || b->d.visit_mark) return ABNN_OK;
    return dalloc(&b->d.visit_mark, b->n_nrn);
}

void host_tick(abnn_brain* b)
{
    if (tick_events(b) > 0) b->clock_host += b->params.clock_inc;  // brain.metal:129
}

abnn_status time_begin(abnn_brain* b, hipStream_t s, EventPair** out)
{
    *out = nullptr;
    if (b->timing <= 0) return ABNN_OK;
    // sampling every n-th launch starts at the second one: the first launch
    // after enable_timing is the one most likely to carry a transient
    const uint64_t n = (uint64_t)b->timing, c = b->timing_count++;
    if (c % n != (n > 1 ? 1u : 0u)) return ABNN_OK;
    if (b->events_used == b->events.size()) {
        EventPair p;
        HIP_TRY(hipEventCreate(&p.a));
        HIP_TRY(hipEventCreate(&p.b));
        b->events.push_back(p);
    }
    *out = &b->events[b->events_used++];
    HIP_TRY(hipEventRecord((*out)->a, s));
    return ABNN_OK;
}

// Sweep partition for the current record count: visited events, wave
// iterations and the persistent gate grid (one range per wave).  Run at
// creation and after every structural update.
void configure(abnn_brain* b)
{
    DeviceState& d = b->d;
    d.n_syn = b->dims.n_syn;
    d.events = visited_events(b->dims, b->params.mode);
    const uint64_t iters = (d.events + d.iter_events - 1) / d.iter_events;
    d.iters = (uint32_t)iters;
    uint64_t G = std::min<uint64_t>(iters, std::min<uint64_t>((uint64_t)b->cus * b->per_cu, kMaxGateBlocks));
    // ranges are per wave; the last workgroup may own fewer than one iteration each
    const uint64_t waves = d.gate_block / 64;
    G = std::min<uint64_t>(G, (iters + waves - 1) / waves);
    if (G == 0 && iters > 0) G = 1;
    d.gate_blocks = (uint32_t)G;
    d.n_ranges = (uint32_t)(G * waves);  // <= kMaxGateBlocks * 16 = kMaxRanges
}

// Uniform sweep partition: range r starts at iteration floor(r * iters / NR)
// (k_apply then adapts it pass by pass, partition_bounds).
abnn_status reset_ranges(abnn_brain* b)
{
    const DeviceState& d = b->d;
    std::vector<uint32_t> rb(d.n_ranges + 1);
    for (uint32_t r = 0; r <= d.n_ranges; ++r) rb[r] = (uint32_t)((uint64_t)r * d.iters / std::max(1u, d.n_ranges));
    HIP_TRY(hipMemcpy(d.range_bounds, rb.data(), rb.size() * 4, hipMemcpyHostToDevice));
    return ABNN_OK;
}

// README §5 structural update (contract in abnn.h): the tombstones' span
// [a, z) closes up in order and the hole at its end takes the array's last D
// records (or the tail shifts down), then the grown records are appended in
// (pass, slot) order while capacity lasts.  Synchronous; runs between passes.
// Only the span and D records move: the tally's bounds give the span's blocks,
// whose live records move down to their final places in place (one pass over
// the span, no spare buffer), so a sweep's update costs O(events), not
// O(n_syn), and the records take their own size in HBM, not twice it.
abnn_status structural_update(abnn_brain* b)
{
    DeviceState& d = b->d;
    const uint64_t n = b->dims.n_syn, cap = b->dims.syn_capacity;
    ST_TRY(sync_all(b));
    const uint64_t nb = (n + kCompactChunk - 1) / kCompactChunk;
    const uint64_t slots = d.grown ? (uint64_t)b->params.compact_every * b->params.max_spikes : 0;
    // the whole update on the device (kernels.hip launch_structural_update):
    // the tally's span, its offsets, the in-place compaction, the hole, the
    // grown records; one synchronisation reads D and the records appended
    *b->err_host = 0;
    unsigned long long* sp = b->span_words;
    hipError_t e = launch_structural_update(d.syn, n, cap, d.dead, nb, b->compact_offsets, b->swap_part, b->swap_toff,
                                            sp, d.err_word, (uint32_t)b->cus, d.grown, slots, b->grown_cnt,
                                            reinterpret_cast<unsigned long long*>(&d.work->stats.grown), nullptr);
    unsigned long long w[5] = {0, 0, 0, 0, 0};
    if (e == hipSuccess) e = hipMemcpy(w, sp, sizeof(w), hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e != hipSuccess) {
        b->records_invalid = true;  // the update may have stopped part-way through its in-place moves
        set_err(std::string("structural update: ") + hipGetErrorString(e) +
                "; the records are not valid, reload them (abnn_load_bnn / abnn_load_flat)");
        return ABNN_ERR_HIP;
    }
    if (const uint32_t err = *b->err_host) {
        // the compaction moves records in place, so a part-done update cannot
        // be rolled back: passes are refused until the records are reloaded
        *b->err_host = 0;
        b->records_invalid = true;
        set_err("structural update: the tombstone tally and the records disagree; "
                "the records are not valid, reload them (abnn_load_bnn / abnn_load_flat)");
        return ABNN_ERR_HIP;
    }
    b->dims.n_syn = n - w[2] + w[4];
    b->structural_updates += 1;
    const uint32_t old_iters = d.iters, old_ranges = d.n_ranges;
    configure(b);
    if (d.n_ranges == old_ranges && old_iters > 0) {
        // the same ranges over (nearly) the same records: keep the adapted
        // partition -- rescaled if the sweep's length changed -- and the
        // measured costs, instead of restarting from a uniform partition
        // (a uniform one costs ~3 passes at several times the pass time)
        if (d.iters != old_iters) {
            std::vector<uint32_t> rb(d.n_ranges + 1);
            for (uint32_t* buf : {d.range_bounds, d.range_bounds_prev}) {
                HIP_TRY(hipMemcpy(rb.data(), buf, rb.size() * 4, hipMemcpyDeviceToHost));
                for (auto& v : rb) v = (uint32_t)((uint64_t)v * d.iters / old_iters);
                rb[d.n_ranges] = d.iters;
                HIP_TRY(hipMemcpy(buf, rb.data(), rb.size() * 4, hipMemcpyHostToDevice));
            }
        }
        return ABNN_OK;
    }
    b->last_pass_fused = false;  // new ranges: the measured costs do not apply
    return reset_ranges(b);
}

// A host write to lastFired (or a clock change) up to `stamp`: the recent-spike
// bitmap is rebuilt from all of lastFired (k_bitmap) until k_apply's build is
// exact again.
void state_written(abnn_brain* b, uint64_t stamp)
{
    b->clean_passes = 0;
    b->max_host_stamp = std::max(b->max_host_stamp, stamp);
    b->next_built = false;
}

// k_apply of pass p may build pass p+1's bitmap from the spike lists
// (kernels.hip, build_next_lists) iff: the clock advances by one per pass; the
// last window_pre - 1 passes were single-GPU passes after the last
// discontinuity, so their spike lists are in fired_ring; and no value the
// host wrote is recent at pass p+1 (clock >= max_host_stamp + window_pre).
bool build_next_ok(const abnn_brain* b)
{
    const uint64_t W = b->params.window_pre;
    return !b->ext_ptrs && !b->force_full_bitmap && b->params.clock_inc == 1 && W >= 1 && W < kFiredRing &&
           b->clean_passes + 1 >= W && b->clock_host >= b->max_host_stamp + W &&
           b->clock_host + W < (1ull << 32);  // ages are u32 (age32): the stamp order above holds below 2^32
}

// This pass's recent-spike buffers (triple-buffered by pass % 3) and, unless
// the previous pass built them, the bitmap from lastFired (k_bitmap).
abnn_status pass_buffers(abnn_brain* b, hipStream_t s)
{
    DeviceState& d = b->d;
    const uint64_t p = b->rot;  // not pass_host: set_scalars may move that
    d.bitmap = b->bitmap_buf[p % 3];
    d.filter = b->filter_buf[p % 3];
    d.bitmap_next = b->bitmap_buf[(p + 1) % 3];
    d.filter_next = b->filter_buf[(p + 1) % 3];
    d.bitmap_clear = b->bitmap_buf[(p + 2) % 3];
    d.filter_clear = b->filter_buf[(p + 2) % 3];
    d.stim_first = b->stim_first;
    d.stim_count = b->stim_count;
    const bool prebuilt = b->next_built && b->built_stim[0] == b->stim_first &&
                          b->built_stim[1] == b->stim_count;
    b->next_built = false;
    if (!prebuilt) HIP_TRY(launch_bitmap(d, b->kp, b->stim_first, b->stim_count, s));
    b->stim_ring[b->pass_host % kFiredRing][0] = b->stim_first;
    b->stim_ring[b->pass_host % kFiredRing][1] = b->stim_count;
    return ABNN_OK;
}

// Whether this pass builds the next one's bitmap, and from which stimulus ranges.
void plan_build(abnn_brain* b)
{
    DeviceState& d = b->d;
    d.build_next = build_next_ok(b) ? 1u : 0u;
    d.n_next_stim = 0;
    if (d.build_next) {  // distinct stimulus ranges of passes p+1-W .. p+1 (p+1: the current one)
        const uint64_t W = b->params.window_pre, p = b->pass_host;
        auto add = [&](uint64_t f, uint64_t c) {
            if (c == 0) return;
            for (uint32_t r = 0; r < d.n_next_stim; ++r)
                if (d.next_stim[r][0] == f && d.next_stim[r][1] == c) return;
            d.next_stim[d.n_next_stim][0] = f;
            d.next_stim[d.n_next_stim++][1] = c;
        };
        for (uint64_t q = p + 1 - W; q <= p; ++q) add(b->stim_ring[q % kFiredRing][0], b->stim_ring[q % kFiredRing][1]);
        add(b->stim_first, b->stim_count);
    }
}

// A sharded pass takes the fused path (two launches around the exchange:
// k_gate in shard mode, k_shard_walk) where a single-GPU pass would.
bool shard_fused(const abnn_brain* b)
{
    return b->use_fused && fused_pass_supported(b->d) && b->d.gate_block == 1024;
}

abnn_status run_shard_fused_gate(abnn_brain* b, int32_t* xchg, hipStream_t s);

// bitmap + streaming gate (with the refractory stage) [+ the exchange record
// of a sharded pass]: the first half of every pass.
abnn_status run_gate(abnn_brain* b, int32_t* xchg_out, hipStream_t s)
{
    if (xchg_out && shard_fused(b)) return run_shard_fused_gate(b, xchg_out, s);
    ST_TRY(pass_buffers(b, s));
    b->last_pass_fused = false;
    EventPair* ev = nullptr;
    ST_TRY(time_begin(b, s, &ev));
    HIP_TRY(launch_gate(b->d, b->kp, s));
    if (ev) HIP_TRY(hipEventRecord(ev->b, s));
    if (xchg_out) HIP_TRY(launch_scan(b->d, b->kp, xchg_out, s));
    return ABNN_OK;
}

// After a pass: the partition it computed for the next one becomes current
// (kernel arguments are captured at launch), its own becomes the previous one.
void rotate_bounds(abnn_brain* b)
{
    DeviceState& d = b->d;
    uint32_t* prev = d.range_bounds_prev;
    d.range_bounds_prev = d.range_bounds;
    d.range_bounds = d.range_bounds_next;
    d.range_bounds_next = prev;
}

// budget walk, weight update, stamps, pass end; k_apply writes the next
// pass's partition into range_bounds_next (rotate_bounds)
abnn_status run_apply(abnn_brain* b, const int32_t* gathered, uint32_t world, uint32_t rank, hipStream_t s)
{
    DeviceState& d = b->d;
    if (b->pending_walk) {  // the sharded fused pass's second launch
        b->pending_walk = false;
        HIP_TRY(launch_shard_walk(d, b->kp, gathered, world, rank, s));
        b->next_built = d.build_next != 0;
        b->built_stim[0] = b->stim_first;
        b->built_stim[1] = b->stim_count;
        rotate_bounds(b);
        return ABNN_OK;
    }
    plan_build(b);
    HIP_TRY(launch_apply(d, b->kp, gathered, world, rank, s));
    b->next_built = d.build_next != 0;
    b->built_stim[0] = b->stim_first;
    b->built_stim[1] = b->stim_count;
    rotate_bounds(b);
    return ABNN_OK;
}

// The whole single-GPU sweep pass in one launch (kernels.hip, k_gate<...,
// kFused>): gate, look-back budget walk, weight update, stamps, pass end.  Its
// prologue computes the next pass's partition (range_bounds_next) from the
// previous fused pass's gate costs.
abnn_status run_fused(abnn_brain* b, hipStream_t s)
{
    DeviceState& d = b->d;
    ST_TRY(pass_buffers(b, s));
    plan_build(b);
    d.prologue_adapt = b->last_pass_fused && d.adapt_ranges ? 1u : 0u;
    d.cost_in = b->cost_buf[b->cost_parity ^ 1u];
    d.cost_out = b->cost_buf[b->cost_parity];
    EventPair* ev = nullptr;
    ST_TRY(time_begin(b, s, &ev));
    HIP_TRY(launch_fused_pass(d, b->kp, s));
    if (ev) HIP_TRY(hipEventRecord(ev->b, s));
    b->next_built = d.build_next != 0;
    b->built_stim[0] = b->stim_first;
    b->built_stim[1] = b->stim_count;
    rotate_bounds(b);
    b->cost_parity ^= 1u;
    b->last_pass_fused = true;
    return ABNN_OK;
}

// The first launch of a sharded pass on the fused path: gate, refractory
// stage, look-back over this shard's workgroups with local budget positions,
// this shard's exchange record (kernels.hip fused_end, shard mode).  Like
// run_fused, but the walk, the stamps and the pass end wait for the exchange.
abnn_status run_shard_fused_gate(abnn_brain* b, int32_t* xchg, hipStream_t s)
{
    DeviceState& d = b->d;
    ST_TRY(pass_buffers(b, s));
    plan_build(b);
    d.prologue_adapt = b->last_pass_fused && d.adapt_ranges ? 1u : 0u;
    d.cost_in = b->cost_buf[b->cost_parity ^ 1u];
    d.cost_out = b->cost_buf[b->cost_parity];
    d.shard_mode = 1;
    d.xchg = xchg;
    EventPair* ev = nullptr;
    ST_TRY(time_begin(b, s, &ev));
    const hipError_t e = launch_fused_pass(d, b->kp, s);
    d.shard_mode = 0;
    d.xchg = nullptr;
    HIP_TRY(e);
    if (ev) HIP_TRY(hipEventRecord(ev->b, s));
    b->cost_parity ^= 1u;
    b->last_pass_fused = true;
    b->pending_walk = true;
    return ABNN_OK;
}

abnn_status run_commit(abnn_brain* b, const int32_t* gathered, uint32_t world, bool renorm,
                       hipStream_t s)
{
    host_tick(b);
    // sharded passes write the merged spike list into fired_ring too
    b->clean_passes += 1;
    if (renorm) {  // renormalise_if_needed, brain.cpp:125-141; kernel brain.metal:135-145
        HIP_TRY(launch_renorm(b->d, b->clock_host, s));
        b->renorms += 1;
        const uint64_t base = b->clock_host;
        b->max_host_stamp = b->max_host_stamp > base ? b->max_host_stamp - base : 0;
        b->clean_passes = 0;  // the clock jumps back
        b->next_built = false;
        b->clock_host = 0;
    }
    b->last_pass = b->pass_host;
    b->pass_host += 1;
    b->rot += 1;
    const uint32_t ce = b->params.compact_every;
    if (ce != 0 && b->pass_host % ce == 0) ST_TRY(structural_update(b));  // README §5
    return ABNN_OK;
}

// RCCL entry points, resolved once: the librccl already loaded in the process
// (torch's, when the caller imported it: one RCCL per process), else the
// system's librccl.so.1.
struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId*);
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*comm_destroy)(ncclComm_t);
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t);
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    const char* (*error_string)(ncclResult_t);
    bool ok;
};

int find_loaded_rccl(struct dl_phdr_info* info, size_t, void* out)
{
    if (info->dlpi_name && std::strstr(info->dlpi_name, "librccl.so")) {
        *static_cast<std::string*>(out) = info->dlpi_name;
        return 1;
    }
    return 0;
}

const RcclApi& rccl_api()
{
    static RcclApi api = [] {
        RcclApi a{};
        std::string loaded;
        dl_iterate_phdr(find_loaded_rccl, &loaded);
        void* h = loaded.empty() ? nullptr : dlopen(loaded.c_str(), RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return a;
        a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        a.comm_init_rank = reinterpret_cast<decltype(a.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
        a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        a.all_gather = reinterpret_cast<decltype(a.all_gather)>(dlsym(h, "ncclAllGather"));
        a.all_reduce = reinterpret_cast<decltype(a.all_reduce)>(dlsym(h, "ncclAllReduce"));
        a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(h, "ncclGetErrorString"));
        a.ok = a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.all_gather && a.all_reduce && a.error_string;
        return a;
    }();
    return api;
}

#define RCCL_TRY(expr)                                                                 \
    do {                                                                               \
        ncclResult_t _r = (expr);                                                      \
        if (_r != ncclSuccess) {                                                       \
            set_err(std::string(#expr) + ": " + rccl_api().error_string(_r));          \
            return ABNN_ERR_HIP;                                                       \
        }                                                                              \
    } while (0)

// Chunked host<->device copies for the file formats.
constexpr uint64_t kIoRecs = 1u << 22;  // 4M records (64 MiB) per piece

}  // namespace

extern "C" {

int abnn_abi_version(void) { return ABNN_ABI_VERSION; }

const char* abnn_status_string(abnn_status s)
{
    switch (s) {
        case ABNN_OK: return "ok";
        case ABNN_ERR_INVALID: return "invalid argument";
        case ABNN_ERR_HIP: return "HIP runtime error";
        case ABNN_ERR_OOM: return "out of memory";
        case ABNN_ERR_SIZE_MISMATCH: return "size mismatch";
        case ABNN_ERR_IO: return "I/O error";
        case ABNN_ERR_NO_DEVICE: return "no HIP device";
    }
    return "unknown status";
}

const char* abnn_last_error(void) { return g_err.c_str(); }

void abnn_default_params(abnn_params* p)
{
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->base_scale = 0.8f;         // brain.metal:22
    p->refractory = 2u;           // brain.metal:23
    p->window_pre = 5u;           // brain.metal:24
    p->clock_inc = 1u;            // brain.metal:26
    p->target_rate_hz = 1000.0f;  // brain.metal:28
    p->eta_home = 1.0e-6f;        // brain.metal:29
    p->eta_reward = 1.0e-3f;      // brain.metal:30
    p->alpha_rbar = 0.001f;       // brain.metal:31
    p->a_ltp = 0.04f;             // constants.h:16
    p->a_ltd = 0.02f;             // constants.h:17
    p->w_min = 0.001f;            // constants.h:18
    p->w_max = 1.0f;              // constants.h:19
    p->max_spikes = 2560u;        // brain.h:18
    p->tick_ns = 1000u;           // brain.h:17
    p->tau_vis = 50000u;          // brain.cpp:102
    p->tau_pre = 50000u;          // brain.cpp:102
    p->renorm_thresh = 4000000u;  // brain.h:19
    p->track_visits = 0u;
    p->seed = 1u;
}

int abnn_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

abnn_status abnn_brain_create(const abnn_dims* dims, const abnn_params* params, int device,
                              abnn_brain** out)
{
    REQUIRE(dims && out, "null argument");
    *out = nullptr;
    REQUIRE(dims->n_input > 0 || dims->n_output > 0 || dims->n_hidden > 0, "no neurons");
    const uint64_t n_nrn = (uint64_t)dims->n_input + dims->n_output + dims->n_hidden;
    REQUIRE(n_nrn < kMaxNeurons, "N_NRN must be below 2^24 - 1 (src is held in 24 bits on the device, DESIGN.md 4)");
    abnn_params p;
    if (params) p = *params;
    else abnn_default_params(&p);
    REQUIRE(p.max_spikes < (1u << 30), "max_spikes too large");
    REQUIRE(p.mode == ABNN_MODE_SWEEP || p.mode == ABNN_MODE_RANDOM, "unknown mode");
    const uint64_t cap = std::max<uint64_t>(dims->syn_capacity, dims->n_syn);  // 0 = creation size
    abnn_dims dmax = *dims;
    dmax.n_syn = cap;
    const uint64_t E = visited_events(dmax, p.mode);  // the most events a pass can visit
    REQUIRE(p.mode != ABNN_MODE_RANDOM || E < 0xFFFFFFFFull, "random mode: events per pass must fit u32");
    const bool genesis = p.p_new > 0.0f && p.compact_every > 0;
    // Gate kernel shape: threads per workgroup x events per lane x KiB per LDS
    // filter image (ABNN_GATE="1024x16f32"; tuning knob, the default is the measured best:
    // profiles/r01s_shape_sweep.txt).
    uint32_t gate_block = 1024, gate_k = 8, filter_kib = 32;  // profiles/r03l_ab_k8.txt: 1024x8 -1.7 us against 1024x16
    if (const char* env = std::getenv("ABNN_GATE")) {
        unsigned gb = 0, gk = 0, fk = 0;
        const int got = std::sscanf(env, "%ux%uf%u", &gb, &gk, &fk);
        if (got >= 2) {
            gate_block = gb;
            gate_k = gk;
            if (got == 3) filter_kib = fk;
        }
    }
    const uint32_t filter_words = filter_kib * 256;
    REQUIRE(gate_shape_supported(gate_block, gate_k, filter_words), "unsupported ABNN_GATE shape");
    const uint64_t iter_events = 64ull * gate_k;  // one wave iteration
    const uint64_t iters = (E + iter_events - 1) / iter_events;
    REQUIRE(iters < 0x7FFFFFFFull, "too many events for one handle");

    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
        set_err("no HIP device visible");
        return ABNN_ERR_NO_DEVICE;
    }
    REQUIRE(device >= 0 && device < ndev, "device ordinal out of range");

    abnn_brain* b = new (std::nothrow) abnn_brain();
    if (!b) return ABNN_ERR_OOM;
    b->dims = *dims;
    b->dims.syn_capacity = cap;
    b->params = p;
    b->kp = to_kernel_params(p);
    b->device = device;
    b->n_nrn = n_nrn;
    b->rng = p.seed;
    auto fail = [&](abnn_status s) {
        free_all(b);
        delete b;
        return s;
    };
    if (hipSetDevice(device) != hipSuccess) {
        set_err("hipSetDevice failed");
        return fail(ABNN_ERR_HIP);
    }
    DeviceState& d = b->d;
    d.n_nrn = n_nrn;
    d.n_input = dims->n_input;
    d.syn_offset = dims->syn_offset;
    d.seed = p.seed;
    d.mode = p.mode;
    d.gate_block = gate_block;
    d.gate_k = gate_k;
    d.iter_events = (uint32_t)iter_events;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0)
        cus = 256;
    // one wave of persistent workgroups: as many as are resident (each keeps the
    // 64 KiB filter in LDS, so at most two per CU)
    int per_cu = gate_blocks_per_cu(gate_block, gate_k, filter_words, p.track_visits != 0,
                                    p.mode == ABNN_MODE_RANDOM);
    if (per_cu <= 0) per_cu = 1;
    if (per_cu > 4) per_cu = 4;
    // at most kFusedMaxRanges ranges (the fused pass's partition prefix in LDS)
    per_cu = std::min<int>(per_cu, std::max<int>(1, (int)(kFusedMaxRanges / ((uint32_t)cus * (gate_block / 64)))));
    b->cus = cus;
    b->per_cu = per_cu;
    // partition A-B knobs: wave -> range map, adaptation gain
    if (const char* env = std::getenv("ABNN_RANGE_MAP")) d.range_map = std::atoi(env) ? 1u : 0u;
    d.adapt_gain = 1;  // profiles/r03g_*: 1 with tail priority 0 is -1 us against 2 with the rank kept
    if (const char* env = std::getenv("ABNN_ADAPT_GAIN")) d.adapt_gain = (uint32_t)std::min(4, std::max(1, std::atoi(env)));
    d.chunk_penalty = 600;  // 24 us per full chunk: the dense input->output stretch spread over more
                            // ranges (ABNN_CHUNK_PENALTY: 25 -> 350 measured -6 us per pass in round 2;
                            // 600 with the 1024x8 gate, profiles/r03l_ab_k8.txt)
    d.apply_blocks = kWalkBlocks;
    if (const char* env = std::getenv("ABNN_APPLY_BLOCKS"))
        d.apply_blocks = (uint32_t)std::min<int>(kWalkBlocks, std::max(1, std::atoi(env)));
    if (const char* env = std::getenv("ABNN_CHUNK_PENALTY")) d.chunk_penalty = (uint32_t)std::max(0, std::atoi(env));
    d.fused_max_blocks = (uint32_t)std::max(0, fused_blocks_per_cu(gate_block, gate_k, filter_words, p.track_visits != 0)) *
                         (uint32_t)cus;
    configure(b);  // sweep partition for the creation size
    const uint64_t max_ranges = (uint64_t)std::min<int>(kMaxGateBlocks, cus * per_cu) * (gate_block / 64);
    d.n_bitmap_words = (uint32_t)(2 * ((n_nrn + 63) / 64));
    d.filter_words = filter_words;
    d.filter_log2 = (uint32_t)__builtin_ctz(filter_words);
    abnn_status s;
    // build_buffers, brain.cpp:52-69: allocate and zero every buffer.
    // padded: the gate's last iteration reads up to one iteration past the sweep
    if ((s = alloc_syn(&d.syn, cap + kDummyRecords, p.mode == ABNN_MODE_RANDOM)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.last_fired, n_nrn)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.last_visited, n_nrn)) != ABNN_OK) return fail(s);
    // a shard (global_events set) that tracks visits marks them for the merge
    if (p.track_visits && dims->global_events && (s = dalloc(&d.visit_mark, n_nrn)) != ABNN_OK) return fail(s);
    uint64_t* sb = nullptr;
    if ((s = dalloc(&sb, 3)) != ABNN_OK) return fail(s);  // {clock, reward|rbar, pass_index}
    b->scalar_block = sb;
    d.clock = sb;
    d.reward = reinterpret_cast<float*>(sb + 1);
    d.rbar = d.reward + 1;
    d.pass_index = sb + 2;
    for (int i = 0; i < 3; ++i) {
        if ((s = dalloc(&b->bitmap_buf[i], (uint64_t)d.n_bitmap_words + 2)) != ABNN_OK) return fail(s);
        if ((s = dalloc(&b->filter_buf[i], 2 * kMaxFilterWords)) != ABNN_OK) return fail(s);
    }
    for (int i = 0; i < 2; ++i)
        if ((s = dalloc(&b->cost_buf[i], max_ranges)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.lb_status, kMaxGateBlocks)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.cand_list, (uint64_t)kFusedMaxRanges * kCandCap)) != ABNN_OK) return fail(s);
    if (const char* env = std::getenv("ABNN_FUSED")) b->use_fused = std::atoi(env) != 0;
    d.spec_mode = 1;
    d.spec_margin = -1;
    if (const char* env = std::getenv("ABNN_SPEC_MARGIN")) d.spec_margin = std::atoi(env);
    d.flush_at = kChunk;
    if (const char* env = std::getenv("ABNN_FLUSH_AT"))
        d.flush_at = (uint32_t)std::min<int>((int)kChunk, std::max(64, std::atoi(env)));
    d.lean = 1;
    if (const char* env = std::getenv("ABNN_LEAN")) d.lean = std::atoi(env) != 0;
    if (const char* env = std::getenv("ABNN_SPEC")) d.spec_mode = (uint32_t)std::min(2, std::max(0, std::atoi(env)));
    d.bitmap = b->bitmap_buf[0];
    d.filter = b->filter_buf[0];
    if ((s = dalloc(&d.range_info, max_ranges)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.range_g1, max_ranges)) != ABNN_OK) return fail(s);
    // per-range regions of refractory survivors (16 B per event: every event of
    // a range may pass in the warm-up passes)
    if ((s = dalloc(&d.g2x, iters * iter_events)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.chunk_cnt, iters * iter_events / kChunkSlotDiv + 8)) != ABNN_OK) return fail(s);
    uint32_t* dummy = nullptr;
    if ((s = dalloc(&dummy, 2 * kDummyRecords)) != ABNN_OK) return fail(s);
    d.dummy = dummy;
    if ((s = dalloc(&d.wg_stats, kWalkBlocks)) != ABNN_OK) return fail(s);
    if (p.mode == ABNN_MODE_RANDOM && (s = dalloc(&d.claim, cap)) != ABNN_OK) return fail(s);
    if (p.compact_every > 0) {  // structural updates (in place): the span's offsets, read flags, words
        const uint64_t nb = (cap + kCompactChunk - 1) / kCompactChunk;
        if ((s = dalloc(&b->compact_offsets, nb + 4)) != ABNN_OK) return fail(s);  // <= nb used (+ slack)
        if ((s = dalloc(&b->swap_part, (nb + kScanThreads - 1) / kScanThreads + 1)) != ABNN_OK) return fail(s);
        if ((s = dalloc(&b->swap_toff, nb + 4)) != ABNN_OK) return fail(s);  // tail blocks + 1 <= nb + 2
        if ((s = dalloc(&b->span_words, 8)) != ABNN_OK) return fail(s);
        // the tombstone tally: pruning's, and an upload's (a saved pruned brain)
        if ((s = dalloc(&d.dead, nb)) != ABNN_OK) return fail(s);
    }
    if (genesis) {
        if ((s = dalloc(&d.g2src, iters * iter_events)) != ABNN_OK) return fail(s);
        if ((s = dalloc(&d.grown, (uint64_t)p.compact_every * p.max_spikes)) != ABNN_OK) return fail(s);
        if ((s = dalloc(&b->grown_cnt, ((uint64_t)p.compact_every * p.max_spikes + kScanThreads - 1) / kScanThreads + 1)) !=
            ABNN_OK)
            return fail(s);
    }
    if ((s = dalloc(&d.work, 1)) != ABNN_OK) return fail(s);
    if (hipHostMalloc(reinterpret_cast<void**>(&b->err_host), 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(reinterpret_cast<void**>(&d.err_word), b->err_host, 0) != hipSuccess) {
        set_err("hipHostMalloc (error word) failed");
        return fail(ABNN_ERR_OOM);
    }
    *b->err_host = 0;
    if ((s = dalloc(&b->u64_scratch, 4)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.wave_clock, (uint64_t)kWaveClockPasses * kWaveClock * kMaxRanges + 32)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.apply_clock, 8 * (uint64_t)kWalkBlocks)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.fired_ring, (uint64_t)kFiredRing * std::max(1u, p.max_spikes))) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.n_fired_ring, kFiredRing)) != ABNN_OK) return fail(s);
    b->force_full_bitmap = std::getenv("ABNN_FULL_BITMAP") != nullptr;
    if ((s = dalloc(&d.range_bounds, max_ranges + 1)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.range_bounds_next, max_ranges + 1)) != ABNN_OK) return fail(s);
    if ((s = dalloc(&d.range_bounds_prev, max_ranges + 1)) != ABNN_OK) return fail(s);
    d.adapt_ranges = std::getenv("ABNN_STATIC_RANGES") ? 0u : 1u;
    if ((s = reset_ranges(b)) != ABNN_OK) return fail(s);
    *out = b;
    return ABNN_OK;
}

abnn_status abnn_brain_destroy(abnn_brain* b)
{
    if (!b) return ABNN_OK;
    (void)hipSetDevice(b->device);
    (void)hipDeviceSynchronize();
    free_all(b);
    delete b;
    return ABNN_OK;
}

abnn_status abnn_get_dims(const abnn_brain* b, abnn_dims* out)
{
    REQUIRE(b && out, "null argument");
    *out = b->dims;
    return ABNN_OK;
}

abnn_status abnn_get_params(const abnn_brain* b, abnn_params* out)
{
    REQUIRE(b && out, "null argument");
    *out = b->params;
    return ABNN_OK;
}

abnn_status abnn_state_ptrs(abnn_brain* b, abnn_state* out)
{
    REQUIRE(b && out, "null argument");
    // the caller may write lastFired or the clock behind the handle's back:
    // rebuild the recent-spike bitmap from lastFired every pass from now on
    b->ext_ptrs = true;
    out->synapses = b->d.syn.lo;  // opaque (abnn_synapse_layout describes the arrays)
    out->last_fired = b->d.last_fired;
    out->last_visited = b->d.last_visited;
    out->clock = b->d.clock;
    out->reward = b->d.reward;
    out->rbar = b->d.rbar;
    return ABNN_OK;
}

// The device record layout (layout 3): the 24-bit src as its
// filter code in two streams (lo u16 in record order, hi u8 permuted within
// every 256-record group) and the {dst, w} pairs; random mode adds the u32 src
// mirror.  Each array holds capacity + padding entries.
abnn_status abnn_synapse_layout(abnn_brain* b, abnn_layout* out)
{
    REQUIRE(b && out, "null argument");
    std::memset(out, 0, sizeof(*out));
    b->ext_ptrs = true;  // as abnn_state_ptrs: the caller may write behind the handle's back
    const uint64_t n = b->dims.syn_capacity + kDummyRecords;
    auto put = [&](void* p, uint64_t bytes, uint32_t eb, const char* name) {
        abnn_array_desc& a = out->arrays[out->n_arrays++];
        a.ptr = p;
        a.bytes = bytes;
        a.elem_bytes = eb;
        std::strncpy(a.name, name, sizeof(a.name) - 1);
    };
    out->version = ABNN_LAYOUT_VERSION;
    put(b->d.syn.lo, n * 2, 2, "src_code_lo");
    put(b->d.syn.hi, hi_bytes(n), 1, "src_code_hi");
    put(b->d.syn.dw, n * 8, 8, "dst_w");
    if (b->d.syn.src32) put(b->d.syn.src32, n * 4, 4, "src32");
    return ABNN_OK;
}

uint64_t abnn_n_neuron(const abnn_brain* b) { return b ? b->n_nrn : 0; }

abnn_status abnn_get_budget(abnn_brain* b, uint32_t* remaining)
{
    REQUIRE(b && remaining, "null argument");
    ST_TRY(sync_all(b));
    uint32_t used = 0;
    if (b->last_pass != ~0ull)  // spikes of the last pass (its spike list's length, in fired_ring)
        HIP_TRY(hipMemcpy(&used, b->d.n_fired_ring + (b->last_pass & (kFiredRing - 1)), 4, hipMemcpyDeviceToHost));
    *remaining = b->params.max_spikes - std::min(used, b->params.max_spikes);
    return ABNN_OK;
}

uint64_t abnn_structural_updates(const abnn_brain* b) { return b ? b->structural_updates : 0; }

uint64_t abnn_renormalisations(const abnn_brain* b) { return b ? b->renorms : 0; }

abnn_status abnn_upload_synapses(abnn_brain* b, uint64_t first, const abnn_synapse* src, uint64_t n)
{
    REQUIRE(b && (src || n == 0), "null argument");
    REQUIRE(first <= b->dims.n_syn && n <= b->dims.n_syn - first, "range out of bounds");
    ST_TRY(validate_records(b, src, n));
    ST_TRY(sync_all(b));
    ST_TRY(records_h2d(b->d.syn, first, n, src));
    if (first == 0 && n == b->dims.n_syn) b->records_invalid = false;  // every record rewritten
    return retally(b, first, n);
}

abnn_status abnn_download_synapses(abnn_brain* b, uint64_t first, abnn_synapse* dst, uint64_t n)
{
    REQUIRE(b && (dst || n == 0), "null argument");
    REQUIRE(first <= b->dims.n_syn && n <= b->dims.n_syn - first, "range out of bounds");
    ST_TRY(sync_all(b));
    return records_d2h(b->d.syn, first, n, dst);
}

abnn_status abnn_generate_synapses(abnn_brain* b, uint64_t seed)
{
    REQUIRE(b, "null argument");
    const uint64_t n_io = (uint64_t)b->dims.n_input * b->dims.n_output;
    REQUIRE(b->dims.syn_offset + b->dims.n_syn <= n_io || b->dims.n_hidden > 0,
            "sparse hidden synapses need n_hidden > 0 (brain-engine.cpp:46-47)");
    REQUIRE(b->dims.n_output > 0 || b->dims.syn_offset + b->dims.n_syn <= n_io,
            "dense block needs n_output > 0");
    ST_TRY(sync_all(b));
    HIP_TRY(launch_generate(b->d, b->dims.n_input, b->dims.n_output, seed, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    b->records_invalid = false;
    return retally(b, 0, b->dims.n_syn);
}

abnn_status abnn_checksum_synapses(abnn_brain* b, uint64_t* out)
{
    REQUIRE(b && out, "null argument");
    ST_TRY(sync_all(b));
    HIP_TRY(launch_checksum(b->d, b->u64_scratch, b->stream));
    HIP_TRY(hipMemcpyAsync(out, b->u64_scratch, sizeof(uint64_t), hipMemcpyDeviceToHost, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    return ABNN_OK;
}

abnn_status abnn_get_last_fired(abnn_brain* b, uint64_t first, uint64_t* out, uint64_t n)
{
    REQUIRE(b && (out || n == 0), "null argument");
    REQUIRE(first <= b->n_nrn && n <= b->n_nrn - first, "range out of bounds");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(out, b->d.last_fired + first, n * 8, hipMemcpyDeviceToHost));
    return ABNN_OK;
}

abnn_status abnn_set_last_fired(abnn_brain* b, uint64_t first, const uint64_t* src, uint64_t n)
{
    REQUIRE(b && (src || n == 0), "null argument");
    REQUIRE(first <= b->n_nrn && n <= b->n_nrn - first, "range out of bounds");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(b->d.last_fired + first, src, n * 8, hipMemcpyHostToDevice));
    state_written(b, n ? *std::max_element(src, src + n) : 0);
    return ABNN_OK;
}

abnn_status abnn_get_last_visited(abnn_brain* b, uint64_t first, uint64_t* out, uint64_t n)
{
    REQUIRE(b && (out || n == 0), "null argument");
    REQUIRE(first <= b->n_nrn && n <= b->n_nrn - first, "range out of bounds");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(out, b->d.last_visited + first, n * 8, hipMemcpyDeviceToHost));
    return ABNN_OK;
}

abnn_status abnn_set_last_visited(abnn_brain* b, uint64_t first, const uint64_t* src, uint64_t n)
{
    REQUIRE(b && (src || n == 0), "null argument");
    REQUIRE(first <= b->n_nrn && n <= b->n_nrn - first, "range out of bounds");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(b->d.last_visited + first, src, n * 8, hipMemcpyHostToDevice));
    // a host write is replicated on every shard (the neuron state is): it
    // replaces whatever this shard visited before it
    if (b->d.visit_mark && n) HIP_TRY(hipMemset(b->d.visit_mark + first, 0, n));
    // a write of the whole array leaves no unmerged mark (as abnn_load_flat):
    // a single-rank restore may then move the clock back (abnn_set_scalars)
    if (first == 0 && n == b->n_nrn) b->marks_dirty = false;
    return ABNN_OK;
}

abnn_status abnn_set_timestamps(abnn_brain* b, const uint32_t* idx, uint64_t n, uint64_t value)
{
    REQUIRE(b && (idx || n == 0), "null argument");
    for (uint64_t i = 0; i < n; ++i) REQUIRE(idx[i] < b->n_nrn, "neuron index out of range");
    ST_TRY(sync_all(b));
    ST_TRY(ensure_idx_scratch(b, n));
    HIP_TRY(hipMemcpy(b->idx_scratch, idx, n * 4, hipMemcpyHostToDevice));
    HIP_TRY(launch_stamp_list(b->d, b->idx_scratch, n, nullptr, value, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    state_written(b, value);
    return ABNN_OK;
}

abnn_status abnn_get_scalars(abnn_brain* b, abnn_scalars* out)
{
    REQUIRE(b && out, "null argument");
    ST_TRY(sync_all(b));
    uint64_t blk[3];
    HIP_TRY(hipMemcpy(blk, b->scalar_block, sizeof(blk), hipMemcpyDeviceToHost));
    out->clock = blk[0];
    std::memcpy(&out->reward, reinterpret_cast<char*>(blk) + 8, 4);
    std::memcpy(&out->rbar, reinterpret_cast<char*>(blk) + 12, 4);
    out->pass_index = blk[2];
    return ABNN_OK;
}

abnn_status abnn_set_scalars(abnn_brain* b, const abnn_scalars* in)
{
    REQUIRE(b && in, "null argument");
    // the merge takes the largest value among the shards that visited a
    // neuron: the clock must not move back over unmerged visits
    REQUIRE(!(b->marks_dirty && in->clock < b->clock_host),
            "the clock moves back over unmerged lastVisited stamps: merge them first "
            "(abnn_comm_sync_visits, or abnn_shard_visits_delta / _merge) on every rank");
    ST_TRY(sync_all(b));
    uint64_t blk[3];
    blk[0] = in->clock;
    std::memcpy(reinterpret_cast<char*>(blk) + 8, &in->reward, 4);
    std::memcpy(reinterpret_cast<char*>(blk) + 12, &in->rbar, 4);
    blk[2] = in->pass_index;
    HIP_TRY(hipMemcpy(b->scalar_block, blk, sizeof(blk), hipMemcpyHostToDevice));
    state_written(b, b->clock_host);  // every stamp so far is <= the old clock
    b->clock_host = in->clock;
    b->pass_host = in->pass_index;
    return ABNN_OK;
}

abnn_status abnn_set_reward(abnn_brain* b, float r)
{
    REQUIRE(b, "null argument");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(b->d.reward, &r, 4, hipMemcpyHostToDevice));
    return ABNN_OK;
}

abnn_status abnn_inject_inputs(abnn_brain* b, const float* v, uint32_t n, float hz)
{
    REQUIRE(b && (v || n == 0), "null argument");
    REQUIRE(n == b->dims.n_input, "inject_inputs: size must equal n_input (brain.cpp:75)");
    // pTick = hz * kTickNS * NSEC_PER_SEC, all in float (brain.cpp:76)
    float p_tick = hz * (float)b->params.tick_ns;
    p_tick = p_tick * (float)1000000000ull;
    std::vector<uint32_t> idx;
    for (uint32_t i = 0; i < n; ++i) {
        b->rng += 0x9E3779B97F4A7C15ull;  // SplitMix64 step
        uint64_t z = b->rng;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z = z ^ (z >> 31);
        const float uni = (float)(z >> 40) * (1.0f / 16777216.0f);
        if (uni < p_tick * v[i]) idx.push_back(i);  // brain.cpp:82
    }
    ST_TRY(sync_all(b));
    if (idx.empty()) return ABNN_OK;
    ST_TRY(ensure_idx_scratch(b, idx.size()));
    HIP_TRY(hipMemcpy(b->idx_scratch, idx.data(), idx.size() * 4, hipMemcpyHostToDevice));
    // lastFired[i] = clock, read on the device
    HIP_TRY(launch_stamp_list(b->d, b->idx_scratch, idx.size(), b->d.clock, 0, b->stream));
    HIP_TRY(hipStreamSynchronize(b->stream));
    state_written(b, b->clock_host);
    return ABNN_OK;
}

abnn_status abnn_read_outputs(abnn_brain* b, uint8_t* out, uint32_t n)
{
    REQUIRE(b && (out || n == 0), "null argument");
    REQUIRE(n == b->dims.n_output, "read_outputs: size must equal n_output");
    ST_TRY(sync_all(b));
    std::vector<uint64_t> lf(n);
    uint64_t clk = 0;
    if (n) HIP_TRY(hipMemcpy(lf.data(), b->d.last_fired + b->dims.n_input, n * 8, hipMemcpyDeviceToHost));
    HIP_TRY(hipMemcpy(&clk, b->d.clock, 8, hipMemcpyDeviceToHost));
    // u32 timestamps, as the reference's (brain.cpp:149-153): the low 32 bits
    const uint32_t now = (uint32_t)clk, start = now > 1 ? now - 1 : 0;  // brain.cpp:151
    for (uint32_t o = 0; o < n; ++o) {
        const uint32_t ts = (uint32_t)lf[o];
        out[o] = (ts != 0 && ts >= start && ts < now) ? 1 : 0;  // brain.cpp:153-154
    }
    return ABNN_OK;
}

abnn_status abnn_set_auto_stimulus(abnn_brain* b, uint64_t first, uint64_t count)
{
    REQUIRE(b, "null argument");
    REQUIRE(count == 0 || (first < b->n_nrn && count <= b->n_nrn - first), "range out of bounds");
    b->stim_first = count ? first : 0;
    b->stim_count = count;
    return ABNN_OK;
}

abnn_status abnn_traverse(abnn_brain* b, uint32_t passes, void* stream)
{
    REQUIRE(b, "null argument");
    REQUIRE(!b->records_invalid, kRecordsInvalid);
    ST_TRY(pass_error(b));  // a pass already completed failed: enqueue nothing more
    if (b->d.visit_mark && passes) b->marks_dirty = true;
    HIP_TRY(hipSetDevice(b->device));
    hipStream_t s = pick(b, stream);
    for (uint32_t i = 0; i < passes; ++i) {
        // the host reads the clock at encode time, before the pass (brain.cpp:127-128)
        const bool renorm = renorm_due(b);
        if (b->use_fused && fused_pass_supported(b->d)) {
            ST_TRY(run_fused(b, s));
        } else {
            ST_TRY(run_gate(b, nullptr, s));
            ST_TRY(run_apply(b, nullptr, 1, 0, s));
        }
        ST_TRY(run_commit(b, nullptr, 1, renorm, s));
    }
    return ABNN_OK;
}

abnn_status abnn_synchronize(abnn_brain* b, void* stream)
{
    REQUIRE(b, "null argument");
    HIP_TRY(hipSetDevice(b->device));
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return sync_all(b);
}

uint64_t abnn_exchange_bytes(const abnn_brain* b)
{
    return b ? 4ull * xchg_words(b->params.max_spikes) : 0;
}

abnn_status abnn_set_global_events(abnn_brain* b, uint64_t global_events)
{
    REQUIRE(b, "null argument");
    b->dims.global_events = global_events;
    return ABNN_OK;
}

abnn_status abnn_shard_gate(abnn_brain* b, void* xchg_dev, void* stream)
{
    REQUIRE(b && xchg_dev, "null argument");
    REQUIRE(((uintptr_t)xchg_dev & 7u) == 0, "exchange record must be 8-B aligned");
    REQUIRE(!b->records_invalid, kRecordsInvalid);
    HIP_TRY(hipSetDevice(b->device));
    ST_TRY(ensure_visit_marks(b));
    if (b->d.visit_mark) b->marks_dirty = true;
    hipStream_t s = pick(b, stream);
    b->pending_renorm = renorm_due(b);
    return run_gate(b, static_cast<int32_t*>(xchg_dev), s);
}

abnn_status abnn_shard_apply(abnn_brain* b, const void* gathered_dev, uint32_t world, uint32_t rank,
                             void* stream)
{
    REQUIRE(b && gathered_dev, "null argument");
    REQUIRE(world >= 1 && rank < world, "bad world/rank");
    HIP_TRY(hipSetDevice(b->device));
    hipStream_t s = pick(b, stream);
    return run_apply(b, static_cast<const int32_t*>(gathered_dev), world, rank, s);
}

abnn_status abnn_shard_commit(abnn_brain* b, const void* gathered_dev, uint32_t world, void* stream)
{
    REQUIRE(b && gathered_dev, "null argument");
    REQUIRE(world >= 1, "bad world");
    HIP_TRY(hipSetDevice(b->device));
    hipStream_t s = pick(b, stream);
    const bool renorm = b->pending_renorm;
    b->pending_renorm = false;
    return run_commit(b, static_cast<const int32_t*>(gathered_dev), world, renorm, s);
}

// The lastVisited merge over a caller's exchange (abnn.h): this shard's deltas,
// then the all-reduced ones applied.
abnn_status abnn_shard_visits_delta(abnn_brain* b, void* delta_dev, void* stream)
{
    REQUIRE(b && delta_dev, "null argument");
    HIP_TRY(hipSetDevice(b->device));
    hipStream_t s = pick(b, stream);
    uint64_t* delta = static_cast<uint64_t*>(delta_dev);
    if (!b->params.track_visits) {  // lastVisited is never written: nothing to merge
        HIP_TRY(hipMemsetAsync(delta, 0, b->n_nrn * 8, s));
        return ABNN_OK;
    }
    ST_TRY(ensure_visit_marks(b));
    HIP_TRY(launch_visits_delta(b->d.last_visited, b->d.visit_mark, delta, b->n_nrn, s));
    return ABNN_OK;
}

abnn_status abnn_shard_visits_merge(abnn_brain* b, const void* reduced_dev, void* stream)
{
    REQUIRE(b && reduced_dev, "null argument");
    HIP_TRY(hipSetDevice(b->device));
    if (!b->params.track_visits) return ABNN_OK;
    ST_TRY(ensure_visit_marks(b));
    HIP_TRY(launch_visits_merge(b->d.last_visited, b->d.visit_mark, static_cast<const uint64_t*>(reduced_dev), b->n_nrn,
                                pick(b, stream)));
    b->marks_dirty = false;
    return ABNN_OK;
}

// ---- sharded passes over RCCL ------------------------------------------------

struct abnn_comm {
    ncclComm_t comm = nullptr;
    abnn_comm_group* local = nullptr;  // in-process group (abnn_comm_create_local): no RCCL
    uint32_t world = 1, rank = 0;
    int device = 0;
    char* gathered = nullptr;   // world exchange records, rank order
    uint64_t rec_bytes = 0;
    uint64_t* scratch = nullptr;  // visited-events all-reduce
    uint64_t* visits = nullptr;   // the lastVisited merge's deltas (n_nrn words, sized on first use)
    uint64_t visits_n = 0;
    bool broken = false;          // an earlier pass failed on this rank (abnn.h: abort on every rank)
    // in-process group: this rank's events (its stream reached the collective /
    // its reads of the peers' buffers are enqueued) and the all-reduce's
    // accumulator and peer staging buffer (sized on first use)
    hipEvent_t ev_ready = nullptr, ev_done = nullptr;
    uint64_t* red_acc = nullptr;
    uint64_t* red_in = nullptr;
    uint64_t red_n = 0;
};

// ---- in-process communicator group (abnn.h abnn_comm_group) -----------------
// `world` ranks in ONE process, one host thread per rank (SURVEY §4 item 4's
// fake communicator behind the same comm interface): the collectives
// abnn_shard_traverse / abnn_comm_sync_visits need -- the in-place all-gather
// of the exchange records and the all-reduce(MAX / SUM) of u64 words -- are
// device copies and a reduction kernel on each rank's own stream, between two
// host barriers:
//   1. every rank records ev_ready on its stream (its inputs are enqueued),
//      barrier;
//   2. every rank's stream waits for the peers' ev_ready, copies / reduces the
//      peers' buffers into its own (rank order), records ev_done, barrier;
//   3. every rank's stream waits for the peers' ev_done (no rank overwrites a
//      buffer a peer still reads).
// No GPU work ever waits for the host, so a rank blocked in a host
// synchronisation never holds up a peer.  Ranks on one device must pass one
// stream (a pass keeps one workgroup per CU resident for its look-back: two
// passes must not run at once); ranks on different devices copy over
// xGMI/PCIe (hipMemcpyDefault).  A barrier that waits longer than
// kGroupTimeout, or a rank that fails (abnn_shard_traverse error), breaks the
// group: every later collective on it fails at once.
struct abnn_comm_group {
    uint32_t world = 0;
    std::mutex m;
    std::condition_variable cv;
    uint64_t gen = 0;       // barrier generation
    uint32_t arrived = 0;
    bool broken = false;
    std::string why;
    std::vector<abnn_comm*> ranks;     // registered communicators (null: free slot)
    std::vector<const char*> buf;      // this collective's buffer of every rank
    std::vector<hipStream_t> streams;  // ... and its stream
};

namespace {

constexpr auto kGroupTimeout = std::chrono::seconds(300);

void group_break(abnn_comm_group* g, const std::string& why)
{
    std::lock_guard<std::mutex> lk(g->m);
    if (!g->broken) g->why = why;
    g->broken = true;
    g->cv.notify_all();
}

abnn_status group_barrier(abnn_comm_group* g)
{
    std::unique_lock<std::mutex> lk(g->m);
    if (g->broken) {
        set_err("local communicator group is broken: " + g->why);
        return ABNN_ERR_INVALID;
    }
    const uint64_t my = g->gen;
    if (++g->arrived == g->world) {
        g->arrived = 0;
        ++g->gen;
        g->cv.notify_all();
        return ABNN_OK;
    }
    if (!g->cv.wait_for(lk, kGroupTimeout, [&] { return g->gen != my || g->broken; })) {
        g->broken = true;
        g->why = "a rank did not reach a collective within 300 s";
        g->cv.notify_all();
    }
    if (g->broken) {
        set_err("local communicator group is broken: " + g->why);
        return ABNN_ERR_INVALID;
    }
    return ABNN_OK;
}

// Steps 1-2 of a collective: publish (buf, s), wait for every rank, check the
// stream rule, and make s wait for every peer's inputs.
abnn_status group_enter(abnn_comm* c, const void* buf, hipStream_t s)
{
    abnn_comm_group* g = c->local;
    g->buf[c->rank] = static_cast<const char*>(buf);
    g->streams[c->rank] = s;
    HIP_TRY(hipEventRecord(c->ev_ready, s));
    ST_TRY(group_barrier(g));
    for (uint32_t j = 0; j < g->world; ++j) {
        if (j == c->rank) continue;
        if (g->ranks[j]->device == c->device && g->streams[j] != s) {
            // every rank sees the same mismatch and fails the same way
            set_err("local communicator: ranks on one device must pass the same stream (their passes must not "
                    "run at once)");
            return ABNN_ERR_INVALID;
        }
        HIP_TRY(hipStreamWaitEvent(s, g->ranks[j]->ev_ready, 0));
    }
    return ABNN_OK;
}

// Step 3: the peers' reads of this rank's buffer are enqueued before s goes on.
abnn_status group_leave(abnn_comm* c, hipStream_t s)
{
    abnn_comm_group* g = c->local;
    HIP_TRY(hipEventRecord(c->ev_done, s));
    ST_TRY(group_barrier(g));
    for (uint32_t j = 0; j < g->world; ++j)
        if (j != c->rank) HIP_TRY(hipStreamWaitEvent(s, g->ranks[j]->ev_done, 0));
    return ABNN_OK;
}

abnn_status local_all_gather(abnn_comm* c, char* recv, uint64_t bytes, hipStream_t s)
{
    abnn_comm_group* g = c->local;
    ST_TRY(group_enter(c, recv, s));
    for (uint32_t j = 0; j < g->world; ++j)  // slot j of every rank's buffer = rank j's record
        if (j != c->rank)
            HIP_TRY(hipMemcpyAsync(recv + bytes * j, g->buf[j] + bytes * j, bytes, hipMemcpyDefault, s));
    return group_leave(c, s);
}

abnn_status local_all_reduce_u64(abnn_comm* c, uint64_t* buf, uint64_t n, bool max, hipStream_t s)
{
    abnn_comm_group* g = c->local;
    if (c->red_n < n) {  // before the barrier: a failed allocation must not leave peers waiting in step 2
        if (c->red_acc) (void)hipFree(c->red_acc);
        if (c->red_in) (void)hipFree(c->red_in);
        c->red_acc = c->red_in = nullptr;
        c->red_n = 0;
        if (dalloc(&c->red_acc, n) != ABNN_OK || dalloc(&c->red_in, n) != ABNN_OK) {
            group_break(g, "rank " + std::to_string(c->rank) + " could not allocate the all-reduce buffers");
            return ABNN_ERR_OOM;
        }
        c->red_n = n;
    }
    ST_TRY(group_enter(c, buf, s));
    HIP_TRY(hipMemcpyAsync(c->red_acc, buf, n * 8, hipMemcpyDefault, s));
    for (uint32_t j = 0; j < g->world; ++j) {
        if (j == c->rank) continue;
        HIP_TRY(hipMemcpyAsync(c->red_in, g->buf[j], n * 8, hipMemcpyDefault, s));
        HIP_TRY(launch_reduce_u64(c->red_acc, c->red_in, n, max, s));
    }
    ST_TRY(group_leave(c, s));
    HIP_TRY(hipMemcpyAsync(buf, c->red_acc, n * 8, hipMemcpyDefault, s));
    return ABNN_OK;
}

}  // namespace

// The collectives of the sharded pass, over RCCL or the in-process group.
static abnn_status comm_all_gather(abnn_comm* c, char* recv, uint64_t bytes, hipStream_t s)
{
    if (c->local) return local_all_gather(c, recv, bytes, s);
    RCCL_TRY(rccl_api().all_gather(recv + bytes * c->rank, recv, bytes, ncclInt8, c->comm, s));  // in place
    return ABNN_OK;
}

static abnn_status comm_all_reduce_u64(abnn_comm* c, uint64_t* buf, uint64_t n, bool max, hipStream_t s)
{
    if (c->local) return local_all_reduce_u64(c, buf, n, max, s);
    RCCL_TRY(rccl_api().all_reduce(buf, buf, n, ncclUint64, max ? ncclMax : ncclSum, c->comm, s));
    return ABNN_OK;
}

// The lastVisited merge on the stream: every rank's deltas
// (k_visits_delta), one all-reduce(MAX) of n_nrn words in place, the merge.
static abnn_status merge_visits(abnn_brain* b, abnn_comm* c, hipStream_t s)
{
    if (!b->params.track_visits) return ABNN_OK;  // lastVisited is never written
    ST_TRY(ensure_visit_marks(b));
    if (c->visits_n != b->n_nrn) {
        if (c->visits) HIP_TRY(hipFree(c->visits));
        c->visits = nullptr;
        c->visits_n = 0;
        ST_TRY(dalloc(&c->visits, b->n_nrn));
        c->visits_n = b->n_nrn;
    }
    HIP_TRY(launch_visits_delta(b->d.last_visited, b->d.visit_mark, c->visits, b->n_nrn, s));
    ST_TRY(comm_all_reduce_u64(c, c->visits, b->n_nrn, true, s));
    HIP_TRY(launch_visits_merge(b->d.last_visited, b->d.visit_mark, c->visits, b->n_nrn, s));
    b->marks_dirty = false;
    return ABNN_OK;
}

abnn_status abnn_comm_unique_id(void* id_out)
{
    REQUIRE(id_out, "null argument");
    const RcclApi& r = rccl_api();
    if (!r.ok) {
        set_err("RCCL (librccl) not found");
        return ABNN_ERR_NO_DEVICE;
    }
    ncclUniqueId id;
    RCCL_TRY(r.get_unique_id(&id));
    std::memcpy(id_out, &id, sizeof(id));
    return ABNN_OK;
}

abnn_status abnn_comm_create(const void* id, uint32_t world, uint32_t rank, int device, abnn_comm** out)
{
    REQUIRE(id && out && world >= 1 && rank < world, "bad argument");
    static_assert(sizeof(ncclUniqueId) == ABNN_COMM_ID_BYTES, "unique id size");
    *out = nullptr;
    const RcclApi& r = rccl_api();
    if (!r.ok) {
        set_err("RCCL (librccl) not found");
        return ABNN_ERR_NO_DEVICE;
    }
    HIP_TRY(hipSetDevice(device));
    abnn_comm* c = new (std::nothrow) abnn_comm();
    if (!c) return ABNN_ERR_OOM;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    const ncclResult_t e = r.comm_init_rank(&c->comm, (int)world, uid, (int)rank);
    if (e != ncclSuccess) {
        set_err(std::string("ncclCommInitRank: ") + r.error_string(e));
        delete c;
        return ABNN_ERR_HIP;
    }
    c->world = world;
    c->rank = rank;
    c->device = device;
    if (dalloc(&c->scratch, 1) != ABNN_OK) {
        abnn_comm_destroy(c);
        return ABNN_ERR_OOM;
    }
    *out = c;
    return ABNN_OK;
}

abnn_status abnn_comm_destroy(abnn_comm* c)
{
    if (!c) return ABNN_OK;
    (void)hipSetDevice(c->device);
    (void)hipDeviceSynchronize();
    if (c->comm) rccl_api().comm_destroy(c->comm);
    if (c->local) {
        std::lock_guard<std::mutex> lk(c->local->m);
        c->local->ranks[c->rank] = nullptr;
    }
    for (void* p : {(void*)c->gathered, (void*)c->scratch, (void*)c->visits, (void*)c->red_acc, (void*)c->red_in})
        if (p) (void)hipFree(p);
    if (c->ev_ready) (void)hipEventDestroy(c->ev_ready);
    if (c->ev_done) (void)hipEventDestroy(c->ev_done);
    delete c;
    return ABNN_OK;
}

abnn_status abnn_comm_group_create(uint32_t world, abnn_comm_group** out)
{
    REQUIRE(out && world >= 1 && world <= 4096, "bad argument");
    abnn_comm_group* g = new (std::nothrow) abnn_comm_group();
    if (!g) return ABNN_ERR_OOM;
    g->world = world;
    g->ranks.assign(world, nullptr);
    g->buf.assign(world, nullptr);
    g->streams.assign(world, nullptr);
    *out = g;
    return ABNN_OK;
}

abnn_status abnn_comm_group_destroy(abnn_comm_group* g)
{
    if (!g) return ABNN_OK;
    {
        std::lock_guard<std::mutex> lk(g->m);
        for (abnn_comm* c : g->ranks)
            REQUIRE(c == nullptr, "abnn_comm_group_destroy: destroy every rank's communicator first");
    }
    delete g;
    return ABNN_OK;
}

abnn_status abnn_comm_create_local(abnn_comm_group* g, uint32_t rank, int device, abnn_comm** out)
{
    REQUIRE(g && out, "null argument");
    REQUIRE(rank < g->world, "rank out of range");
    *out = nullptr;
    HIP_TRY(hipSetDevice(device));
    abnn_comm* c = new (std::nothrow) abnn_comm();
    if (!c) return ABNN_ERR_OOM;
    c->local = g;
    c->world = g->world;
    c->rank = rank;
    c->device = device;
    if (hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming) != hipSuccess ||
        dalloc(&c->scratch, 1) != ABNN_OK) {
        c->local = nullptr;
        abnn_comm_destroy(c);
        set_err("abnn_comm_create_local: event or buffer allocation failed");
        return ABNN_ERR_OOM;
    }
    {
        std::lock_guard<std::mutex> lk(g->m);
        if (g->ranks[rank] != nullptr) {
            c->local = nullptr;
            abnn_comm_destroy(c);
            set_err("abnn_comm_create_local: rank already has a communicator in this group");
            return ABNN_ERR_INVALID;
        }
        g->ranks[rank] = c;
    }
    *out = c;
    return ABNN_OK;
}

// One sharded pass per iteration.  An error part-way through a pass leaves
// the other ranks inside (or about to enter) the pass's collectives, so the
// communicator is marked broken: every later call on it fails at once, and
// the caller must abort / destroy it on every rank (abnn.h).  The handle's
// half-done pass is dropped (no walk of a gate whose exchange never came).
static abnn_status shard_traverse_passes(abnn_brain* b, abnn_comm* c, uint32_t passes, hipStream_t s)
{
    const uint64_t rec = abnn_exchange_bytes(b);
    if (rec != c->rec_bytes) {  // the records' size follows the budget: sized on first use
        if (c->gathered) HIP_TRY(hipFree(c->gathered));
        c->gathered = nullptr;
        ST_TRY(dalloc(&c->gathered, rec * c->world));
        c->rec_bytes = rec;
    }
    char* mine = c->gathered + rec * c->rank;
    for (uint32_t i = 0; i < passes; ++i) {
        ST_TRY(abnn_shard_gate(b, mine, s));
        ST_TRY(comm_all_gather(c, c->gathered, rec, s));  // in place, rank order
        ST_TRY(abnn_shard_apply(b, c->gathered, c->world, c->rank, s));
        const uint64_t updates = b->structural_updates, renorms = b->renorms;
        ST_TRY(abnn_shard_commit(b, c->gathered, c->world, s));
        // the clock went back: merge lastVisited before the next pass stamps
        // smaller values than this epoch's
        if (b->renorms != renorms && b->params.track_visits) ST_TRY(merge_visits(b, c, s));
        if (b->structural_updates != updates) {
            // every shard's record count changed (all ranks update after the
            // same pass): re-sum the visited events for the clock-tick rule
            uint64_t mine_ev = visited_events(b->dims, b->params.mode), tot = 0;
            HIP_TRY(hipMemcpyAsync(c->scratch, &mine_ev, 8, hipMemcpyHostToDevice, s));
            ST_TRY(comm_all_reduce_u64(c, c->scratch, 1, false, s));
            HIP_TRY(hipMemcpyAsync(&tot, c->scratch, 8, hipMemcpyDeviceToHost, s));
            HIP_TRY(hipStreamSynchronize(s));
            b->dims.global_events = tot;
        }
    }
    return ABNN_OK;
}

static abnn_status shard_traverse_checked(abnn_brain* b, abnn_comm* c, uint32_t passes, void* stream)
{
    REQUIRE(b, "null argument");
    REQUIRE(c->device == b->device, "communicator and handle are on different devices");
    REQUIRE(!c->broken, "communicator unusable after an earlier error on this rank: abort / destroy it on every rank");
    HIP_TRY(hipSetDevice(b->device));
    ST_TRY(pass_error(b));
    return shard_traverse_passes(b, c, passes, pick(b, stream));
}

abnn_status abnn_shard_traverse(abnn_brain* b, abnn_comm* c, uint32_t passes, void* stream)
{
    REQUIRE(c, "null argument");
    const abnn_status st = shard_traverse_checked(b, c, passes, stream);
    if (st != ABNN_OK) {
        c->broken = true;
        if (b) b->pending_walk = false;
        // the peers are in (or about to enter) this pass's collectives: an
        // in-process group lets them fail at once (RCCL ranks abort)
        if (c->local) group_break(c->local, "rank " + std::to_string(c->rank) + ": " + g_err);
    }
    return st;
}

// Diagnostics (abnn_debug.h): `count` in-place all-gathers of `bytes` per
// rank from `buf` (rank order, world x bytes), the sharded pass's exchange
// alone (tools/allgather_time.py).
abnn_status abnn_debug_comm_allgather(abnn_comm* c, void* buf, uint64_t bytes, uint32_t count, void* stream)
{
    REQUIRE(c && buf, "null argument");
    REQUIRE(!c->broken, "communicator unusable after an earlier error on this rank: abort / destroy it on every rank");
    HIP_TRY(hipSetDevice(c->device));
    const hipStream_t s = static_cast<hipStream_t>(stream);
    char* base = static_cast<char*>(buf);
    for (uint32_t i = 0; i < count; ++i) ST_TRY(comm_all_gather(c, base, bytes, s));
    return ABNN_OK;
}

abnn_status abnn_comm_sync_visits(abnn_brain* b, abnn_comm* c, void* stream)
{
    REQUIRE(b && c, "null argument");
    REQUIRE(c->device == b->device, "communicator and handle are on different devices");
    REQUIRE(!c->broken, "communicator unusable after an earlier error on this rank: abort / destroy it on every rank");
    ST_TRY(sync_all(b));
    hipStream_t s = pick(b, stream);
    abnn_status st = merge_visits(b, c, s);
    if (st == ABNN_OK && hipStreamSynchronize(s) != hipSuccess) {
        set_err("hipStreamSynchronize failed after the lastVisited merge");
        st = ABNN_ERR_HIP;
    }
    if (st != ABNN_OK) {
        c->broken = true;
        if (c->local) group_break(c->local, "rank " + std::to_string(c->rank) + ": " + g_err);
    }
    return st;
}

// Diagnostics (not part of abnn.h): record the per-wave gate times of the
// following passes (on) or not (off, the default).
abnn_status abnn_debug_set_wave_clock(abnn_brain* b, int on)
{
    REQUIRE(b, "null argument");
    b->d.wave_clock_on = on ? 1u : 0u;
    return ABNN_OK;
}

// Diagnostics (not part of abnn.h): the last pass's per-wave gate times,
// kWaveClock u64 per range (engine.h, DeviceState::wave_clock), 100 MHz ticks.
abnn_status abnn_debug_wave_clock_slot(abnn_brain* b, uint32_t slot, uint64_t* out, uint64_t n)
{
    REQUIRE(b && out, "null argument");
    REQUIRE(slot < kWaveClockPasses, "slot out of range");
    ST_TRY(sync_all(b));
    const uint64_t per = (uint64_t)kWaveClock * kMaxRanges;
    HIP_TRY(hipMemcpy(out, b->d.wave_clock + slot * per, std::min<uint64_t>(n, per) * 8, hipMemcpyDeviceToHost));
    return ABNN_OK;
}

abnn_status abnn_debug_wave_clock(abnn_brain* b, uint64_t* out, uint64_t n)
{
    REQUIRE(b, "null argument");
    // a fused pass p writes slot p % kWaveClockPasses, the two-kernel gate slot 0
    const uint32_t slot = b->last_pass_fused && b->pass_host ? (uint32_t)((b->pass_host - 1) % kWaveClockPasses) : 0u;
    return abnn_debug_wave_clock_slot(b, slot, out, n);
}

// Diagnostics (not part of abnn.h): the last k_apply's per-workgroup timeline,
// 8 u64 per workgroup (see k_apply), 100 MHz ticks.
abnn_status abnn_debug_apply_clock(abnn_brain* b, uint64_t* out, uint64_t n)
{
    REQUIRE(b && out, "null argument");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(out, b->d.apply_clock, std::min<uint64_t>(n, 8ull * kWalkBlocks) * 8, hipMemcpyDeviceToHost));
    return ABNN_OK;
}

// Diagnostics (not part of abnn.h): the recent-spike bitmap of the last pass
// (n_bitmap_words u32; bit i = neuron i was recent at that pass's start) and
// whether k_apply built the next pass's (no k_bitmap launch).
abnn_status abnn_debug_bitmap(abnn_brain* b, uint32_t* out, uint64_t n, int* incremental_next)
{
    REQUIRE(b && out, "null argument");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(out, b->d.bitmap, std::min<uint64_t>(n, b->d.n_bitmap_words) * 4, hipMemcpyDeviceToHost));
    if (incremental_next) *incremental_next = b->next_built ? 1 : 0;
    return ABNN_OK;
}

// Diagnostics (not part of abnn.h): the current sweep partition, n_ranges + 1
// iteration bounds.
abnn_status abnn_debug_range_bounds(abnn_brain* b, uint32_t* out, uint64_t n)
{
    REQUIRE(b && out, "null argument");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(out, b->d.range_bounds, std::min<uint64_t>(n, b->d.n_ranges + 1ull) * 4, hipMemcpyDeviceToHost));
    return ABNN_OK;
}

abnn_status abnn_get_stats(abnn_brain* b, abnn_stats* out)
{
    REQUIRE(b && out, "null argument");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemcpy(out, &b->d.work->stats, sizeof(abnn_stats), hipMemcpyDeviceToHost));
    std::vector<abnn_stats> wg(kWalkBlocks);
    HIP_TRY(hipMemcpy(wg.data(), b->d.wg_stats, kWalkBlocks * sizeof(abnn_stats), hipMemcpyDeviceToHost));
    for (const abnn_stats& x : wg) {
        out->passes += x.passes;
        out->events += x.events;
        out->pre_gated += x.pre_gated;
        out->post_gated += x.post_gated;
        out->updated += x.updated;
        out->fired += x.fired;
        out->pruned += x.pruned;
        out->grown += x.grown;
    }
    return ABNN_OK;
}

abnn_status abnn_reset_stats(abnn_brain* b)
{
    REQUIRE(b, "null argument");
    ST_TRY(sync_all(b));
    HIP_TRY(hipMemset(&b->d.work->stats, 0, sizeof(abnn_stats)));
    HIP_TRY(hipMemset(b->d.wg_stats, 0, kWalkBlocks * sizeof(abnn_stats)));
    return ABNN_OK;
}

abnn_status abnn_enable_timing(abnn_brain* b, int every)
{
    REQUIRE(b && every >= 0, "bad argument");
    ST_TRY(sync_all(b));
    b->timing = every;
    b->timing_count = 0;
    b->events_used = 0;
    return ABNN_OK;
}

abnn_status abnn_get_kernel_time(abnn_brain* b, double* ms_total, uint64_t* launches)
{
    REQUIRE(b && ms_total && launches, "null argument");
    ST_TRY(sync_all(b));
    double tot = 0;
    for (size_t i = 0; i < b->events_used; ++i) {
        float ms = 0;
        HIP_TRY(hipEventElapsedTime(&ms, b->events[i].a, b->events[i].b));
        tot += ms;
    }
    *ms_total = tot;
    *launches = b->events_used;
    b->events_used = 0;
    return ABNN_OK;
}

abnn_status abnn_get_kernel_times(abnn_brain* b, float* out_ms, uint64_t cap, uint64_t* launches)
{
    REQUIRE(b && launches && (out_ms || cap == 0), "null argument");
    ST_TRY(sync_all(b));
    for (size_t i = 0; i < b->events_used && i < cap; ++i)
        HIP_TRY(hipEventElapsedTime(&out_ms[i], b->events[i].a, b->events[i].b));
    *launches = b->events_used;
    b->events_used = 0;
    return ABNN_OK;
}

// ---- persistence -----------------------------------------------------------

abnn_status abnn_save_bnn(abnn_brain* b, const char* path)
{
    REQUIRE(b && path, "null argument");
    REQUIRE(b->dims.n_syn <= 0xFFFFFFFFull && b->n_nrn <= 0xFFFFFFFFull,
            ".bnn header holds u32 sizes (brain.cpp:163-164)");
    ST_TRY(sync_all(b));
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        set_err(std::string("cannot open ") + path);
        return ABNN_ERR_IO;
    }
    const uint32_t hdr[2] = {(uint32_t)b->dims.n_syn, (uint32_t)b->n_nrn};  // brain.cpp:163-164
    bool ok = std::fwrite(hdr, 4, 2, f) == 2;
    std::vector<abnn_synapse> buf;
    for (uint64_t i = 0; ok && i < b->dims.n_syn; i += kIoRecs) {
        const uint64_t n = std::min<uint64_t>(kIoRecs, b->dims.n_syn - i);
        buf.resize(n);
        if (records_d2h(b->d.syn, i, n, buf.data()) != ABNN_OK) {
            std::fclose(f);
            return ABNN_ERR_HIP;
        }
        ok = std::fwrite(buf.data(), 16, n, f) == n;  // brain.cpp:165-166
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        set_err(std::string("write failed: ") + path);
        return ABNN_ERR_IO;
    }
    return ABNN_OK;
}

abnn_status abnn_load_bnn(abnn_brain* b, const char* path)
{
    REQUIRE(b && path, "null argument");
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        set_err(std::string("cannot open ") + path);
        return ABNN_ERR_IO;
    }
    uint32_t hdr[2] = {0, 0};
    if (std::fread(hdr, 4, 2, f) != 2) {
        std::fclose(f);
        set_err("short .bnn header");
        return ABNN_ERR_IO;
    }
    if (!(hdr[0] == b->dims.n_syn && hdr[1] == b->n_nrn)) {  // brain.cpp:174
        std::fclose(f);
        set_err(".bnn header does not match this brain");
        return ABNN_ERR_SIZE_MISMATCH;
    }
    abnn_status st = sync_all(b);
    if (st != ABNN_OK) {
        std::fclose(f);
        return st;
    }
    std::vector<abnn_synapse> buf;
    for (uint64_t i = 0; i < b->dims.n_syn; i += kIoRecs) {
        const uint64_t n = std::min<uint64_t>(kIoRecs, b->dims.n_syn - i);
        buf.resize(n);
        if (std::fread(buf.data(), 16, n, f) != n) {
            std::fclose(f);
            set_err("short .bnn body");
            return ABNN_ERR_IO;
        }
        st = validate_records(b, buf.data(), n);
        if (st == ABNN_OK) st = records_h2d(b->d.syn, i, n, buf.data());
        if (st != ABNN_OK) {
            std::fclose(f);
            return st;
        }
    }
    std::fclose(f);
    b->records_invalid = false;
    return retally(b, 0, b->dims.n_syn);
}

abnn_status abnn_save_flat(abnn_brain* b, const char* path)
{
    REQUIRE(b && path, "null argument");
    REQUIRE(b->dims.n_syn <= 0xFFFFFFFFull && b->n_nrn <= 0xFFFFFFFFull,
            "flat header holds u32 sizes (README §2.1)");
    ST_TRY(sync_all(b));
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        set_err(std::string("cannot open ") + path);
        return ABNN_ERR_IO;
    }
    uint32_t hdr[4] = {(uint32_t)b->dims.n_syn, (uint32_t)b->n_nrn, 0, 0};
    bool ok = std::fwrite(hdr, 4, 4, f) == 4;
    std::vector<abnn_synapse> buf;
    std::vector<uint32_t> pairs;
    std::vector<float> ws;
    // synapses (src, dst) pairs, then weights: two sweeps
    for (int sweep = 0; ok && sweep < 2; ++sweep) {
        for (uint64_t i = 0; ok && i < b->dims.n_syn; i += kIoRecs) {
            const uint64_t n = std::min<uint64_t>(kIoRecs, b->dims.n_syn - i);
            buf.resize(n);
            if (records_d2h(b->d.syn, i, n, buf.data()) != ABNN_OK) {
                ok = false;
                break;
            }
            if (sweep == 0) {
                pairs.resize(2 * n);
                for (uint64_t k = 0; k < n; ++k) {
                    pairs[2 * k] = buf[k].src;
                    pairs[2 * k + 1] = buf[k].dst;
                }
                ok = std::fwrite(pairs.data(), 8, n, f) == n;
            } else {
                ws.resize(n);
                for (uint64_t k = 0; k < n; ++k) ws[k] = buf[k].w;
                ok = std::fwrite(ws.data(), 4, n, f) == n;
            }
        }
    }
    std::vector<uint64_t> ts(b->n_nrn);
    for (int arr = 0; ok && arr < 2; ++arr) {
        uint64_t* src = arr == 0 ? b->d.last_fired : b->d.last_visited;
        if (b->n_nrn && hipMemcpy(ts.data(), src, b->n_nrn * 8, hipMemcpyDeviceToHost) != hipSuccess) {
            ok = false;
            break;
        }
        ok = std::fwrite(ts.data(), 8, b->n_nrn, f) == b->n_nrn;
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        set_err(std::string("flat save failed: ") + path);
        return ABNN_ERR_IO;
    }
    return ABNN_OK;
}

abnn_status abnn_load_flat(abnn_brain* b, const char* path)
{
    REQUIRE(b && path, "null argument");
    FILE* f = std::fopen(path, "rb");
    if (!f) {
        set_err(std::string("cannot open ") + path);
        return ABNN_ERR_IO;
    }
    uint32_t hdr[4] = {0, 0, 0, 0};
    if (std::fread(hdr, 4, 4, f) != 4) {
        std::fclose(f);
        set_err("short flat header");
        return ABNN_ERR_IO;
    }
    if (!(hdr[0] == b->dims.n_syn && hdr[1] == b->n_nrn)) {
        std::fclose(f);
        set_err("flat header does not match this brain");
        return ABNN_ERR_SIZE_MISMATCH;
    }
    abnn_status st = sync_all(b);
    if (st != ABNN_OK) {
        std::fclose(f);
        return st;
    }
    const uint64_t N = b->dims.n_syn;
    const long pairs_at = 16, weights_at = 16 + (long)(8 * N);
    std::vector<abnn_synapse> buf;
    std::vector<uint32_t> pairs;
    std::vector<float> ws;
    bool ok = true;
    for (uint64_t i = 0; ok && i < N; i += kIoRecs) {
        const uint64_t n = std::min<uint64_t>(kIoRecs, N - i);
        pairs.resize(2 * n);
        ws.resize(n);
        buf.resize(n);
        ok = std::fseek(f, pairs_at + (long)(8 * i), SEEK_SET) == 0 &&
             std::fread(pairs.data(), 8, n, f) == n &&
             std::fseek(f, weights_at + (long)(4 * i), SEEK_SET) == 0 &&
             std::fread(ws.data(), 4, n, f) == n;
        if (!ok) break;
        for (uint64_t k = 0; k < n; ++k) buf[k] = {pairs[2 * k], pairs[2 * k + 1], ws[k], 0.0f};
        st = validate_records(b, buf.data(), n);
        if (st != ABNN_OK) {
            std::fclose(f);
            return st;
        }
        ok = records_h2d(b->d.syn, i, n, buf.data()) == ABNN_OK;
    }
    std::vector<uint64_t> ts(b->n_nrn);
    if (ok) ok = std::fseek(f, weights_at + (long)(4 * N), SEEK_SET) == 0;
    for (int arr = 0; ok && arr < 2; ++arr) {
        ok = std::fread(ts.data(), 8, b->n_nrn, f) == b->n_nrn;
        uint64_t* dst = arr == 0 ? b->d.last_fired : b->d.last_visited;
        if (ok && b->n_nrn)
            ok = hipMemcpy(dst, ts.data(), b->n_nrn * 8, hipMemcpyHostToDevice) == hipSuccess;
        if (ok && arr == 0) state_written(b, b->n_nrn ? *std::max_element(ts.begin(), ts.end()) : 0);
    }
    std::fclose(f);
    if (!ok) {
        set_err(std::string("flat load failed: ") + path);
        return ABNN_ERR_IO;
    }
    b->records_invalid = false;
    if (b->d.visit_mark) {  // lastVisited replaced on every shard (replicated state)
        HIP_TRY(hipMemset(b->d.visit_mark, 0, b->n_nrn));
        b->marks_dirty = false;
    }
    return retally(b, 0, N);
}

}  // extern "C"
