/*
 * c1_oracle.c -- CPU restatement of the reference traversal pass under the
 * deterministic schedule C1.  TEST INFRASTRUCTURE ONLY (see c1_oracle.h):
 * the product never links, loads or calls this file.
 *
 * PARITY UNPINNED (no reference tests/fixtures exist and brain.metal cannot be
 * built or run in this image -- DESIGN.md §3).
 *
 * Build: gcc -O2 -std=c11 -ffp-contract=off -fPIC -shared -pthread
 * (-ffp-contract=off: every fp32 operation rounds on its own, exactly like the
 * HIP product which is compiled the same way.)
 *
 * Reference line citations are relative to /root/reference:
 *   MSL  = abnn/src/core/kernels/brain.metal
 *   BR   = abnn/src/core/brain/brain.cpp
 *   ENG  = abnn/src/core/brain-engine.cpp
 */
#define _GNU_SOURCE
#include "c1_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

void oracle_default_params(abnn_params* p)
{
    memset(p, 0, sizeof(*p));
    p->base_scale = 0.8f;        /* MSL:22 */
    p->refractory = 2u;          /* MSL:23 */
    p->window_pre = 5u;          /* MSL:24 */
    p->clock_inc = 1u;           /* MSL:26 */
    p->target_rate_hz = 1000.0f; /* MSL:28 */
    p->eta_home = 1.0e-6f;       /* MSL:29 */
    p->eta_reward = 1.0e-3f;     /* MSL:30 */
    p->alpha_rbar = 0.001f;      /* MSL:31 */
    p->a_ltp = 0.04f;            /* constants.h:16 */
    p->a_ltd = 0.02f;            /* constants.h:17 */
    p->w_min = 0.001f;           /* constants.h:18 */
    p->w_max = 1.0f;             /* constants.h:19 */
    p->max_spikes = 2560u;       /* brain.h:18 */
    p->tick_ns = 1000u;          /* brain.h:17 */
    p->tau_vis = 50000u;         /* BR:102 */
    p->tau_pre = 50000u;         /* BR:102 */
    p->renorm_thresh = 4000000u; /* brain.h:19 */
    p->track_visits = 0u;
    p->seed = 1u;
}

/* rand01, MSL:15-19: xorshift32 (<<13, >>17, <<5) then 24-bit mantissa. */
float oracle_rand01(uint32_t s)
{
    s ^= s << 13;
    s ^= s >> 17;
    s ^= s << 5;
    return (float)(s & 0xFFFFFFu) * (1.0f / 16777216.0f);
}

/* The k-th output (k >= 0) of SplitMix64 seeded with `seed`. */
uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1u) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Timestamp arithmetic of the reference: lastF and clock are `uint` (MSL:43,45;
 * BR:55-57), so every age `now - ts` (MSL:74,80,116) and the renormalisation
 * test (BR:127-128) are u32 wrap-around.  The build stores u64 timestamps
 * (README lastFiredNS) and takes every decision on their low 32 bits, so a
 * stamp ahead of the clock ages like the reference's (2^32 - k, not 2^64 - k). */
static inline uint32_t age32(uint64_t now, uint64_t ts) { return (uint32_t)now - (uint32_t)ts; }

static inline float clampf(float x, float lo, float hi)
{
    /* Metal clamp(x, lo, hi) = min(max(x, lo), hi) */
    float m = x > lo ? x : lo;
    return m < hi ? m : hi;
}

/* Visited events per pass.  Sweep: the grid is roundup(EVENTS,256) threads
 * and every tid >= nSyn returns at once (BR:116-118, MSL:60-61).  Random
 * mode (README §4): exactly EVENTS picks. */
uint64_t oracle_visited_events(const abnn_dims* d, uint32_t mode)
{
    if (mode == ABNN_MODE_RANDOM) return d->n_syn ? d->events_per_pass : 0;
    uint64_t grid = (d->events_per_pass + 255u) / 256u * 256u;
    return grid < d->n_syn ? grid : d->n_syn;
}

/* Philox4x32-10: ten rounds of two 32x32->64 multiplies; the key is bumped
 * by the Weyl constants between rounds. */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4])
{
    uint32_t x0 = ctr[0], x1 = ctr[1], x2 = ctr[2], x3 = ctr[3], k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * x0, p1 = (uint64_t)0xCD9E8D57u * x2;
        const uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ k0, y1 = (uint32_t)p1;
        const uint32_t y2 = (uint32_t)(p0 >> 32) ^ x3 ^ k1, y3 = (uint32_t)p0;
        x0 = y0; x1 = y1; x2 = y2; x3 = y3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = x0; out[1] = x1; out[2] = x2; out[3] = x3;
}

/* Random-mode record of local event t: Lemire multiply-shift of a 64-bit
 * Philox draw onto [0, n_syn). */
uint64_t oracle_pick(uint64_t seed, uint64_t stream, uint64_t pass, uint64_t t, uint64_t n_syn)
{
    const uint64_t k = seed ^ stream;
    const uint32_t c[4] = {(uint32_t)t, (uint32_t)(t >> 32), (uint32_t)pass, (uint32_t)(pass >> 32)};
    const uint32_t key[2] = {(uint32_t)k, (uint32_t)(k >> 32)};
    uint32_t o[4];
    oracle_philox4x32_10(c, key, o);
    const uint64_t x = ((uint64_t)o[1] << 32) | o[0];
    return (uint64_t)(((unsigned __int128)x * n_syn) >> 64);
}

/* Synthetic graph, recipe of build_random_graph (ENG:31-53) with a portable
 * counter-based RNG (the reference's mt19937 + std distributions are
 * implementation-defined, so its bytes are not reproducible anywhere else). */
static inline float unit24(uint64_t x) { return (float)(x >> 40) * (1.0f / 16777216.0f); }

void oracle_gen_synapse(uint64_t i, uint32_t n_in, uint32_t n_out, uint64_t n_nrn,
                        uint64_t seed, abnn_synapse* out)
{
    uint64_t n_io = (uint64_t)n_in * (uint64_t)n_out;
    uint64_t x2 = oracle_splitmix64_at(seed, 3u * i + 2u);
    if (i < n_io) { /* dense input -> output block, ENG:40-43 */
        out->src = (uint32_t)(i / n_out);
        out->dst = n_in + (uint32_t)(i % n_out);
        out->w = 0.4f + unit24(x2) * (0.8f - 0.4f);
    } else {        /* sparse hidden -> hidden, ENG:45-50 */
        uint64_t lo = (uint64_t)n_in + n_out;
        uint64_t range = n_nrn - lo;
        uint64_t x0 = oracle_splitmix64_at(seed, 3u * i + 0u);
        uint64_t x1 = oracle_splitmix64_at(seed, 3u * i + 1u);
        out->src = (uint32_t)(lo + (((x0 >> 32) * range) >> 32));
        out->dst = (uint32_t)(lo + (((x1 >> 32) * range) >> 32));
        out->w = 0.1f + unit24(x2) * (0.2f - 0.1f);
    }
    out->pad = 0.0f;
}

typedef struct gen_job {
    abnn_synapse* out;
    uint64_t first, n;
    uint32_t n_in, n_out;
    uint64_t n_nrn, seed;
} gen_job;

static void* gen_worker(void* arg)
{
    gen_job* j = (gen_job*)arg;
    for (uint64_t k = 0; k < j->n; ++k)
        oracle_gen_synapse(j->first + k, j->n_in, j->n_out, j->n_nrn, j->seed, &j->out[k]);
    return NULL;
}

void oracle_gen_synapses(abnn_synapse* out, uint64_t first_global, uint64_t n,
                         uint32_t n_in, uint32_t n_out, uint64_t n_nrn,
                         uint64_t seed, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    gen_job jobs[256];
    uint64_t per = (n + (uint64_t)nthreads - 1) / (uint64_t)nthreads;
    int started = 0;
    for (int k = 0; k < nthreads; ++k) {
        uint64_t a = per * (uint64_t)k;
        if (a >= n) break;
        uint64_t b = a + per < n ? a + per : n;
        jobs[k] = (gen_job){out + a, first_global + a, b - a, n_in, n_out, n_nrn, seed};
        if (nthreads == 1) { gen_worker(&jobs[k]); continue; }
        pthread_create(&th[k], NULL, gen_worker, &jobs[k]);
        started = k + 1;
    }
    for (int k = 0; k < started; ++k) pthread_join(th[k], NULL);
}

static inline uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Position-sensitive checksum: sum_i mix64(rec_i ^ mix64(i*golden + w)). */
uint64_t oracle_checksum_synapses(const abnn_synapse* s, uint64_t n, uint64_t first_global)
{
    uint64_t acc = 0;
    for (uint64_t k = 0; k < n; ++k) {
        uint32_t wb, pb;
        memcpy(&wb, &s[k].w, 4);
        memcpy(&pb, &s[k].pad, 4);
        uint64_t i = first_global + k;
        uint64_t a = ((uint64_t)s[k].src << 32) | s[k].dst;
        uint64_t b = ((uint64_t)wb << 32) | pb;
        acc += mix64(a ^ mix64(b + i * 0x9E3779B97F4A7C15ull));
    }
    return acc;
}

/* Host RNG of a handle: SplitMix64 stream, uni() in [0,1) with 24 bits. */
static inline float host_uni(uint64_t* state)
{
    *state += 0x9E3779B97F4A7C15ull;
    return unit24(mix64(*state));
}

/* Brain::inject_inputs, BR:73-83.  pTick = hz * kTickNS * NSEC_PER_SEC in
 * float arithmetic (kTickNS and NSEC_PER_SEC converted to float). */
void oracle_inject_inputs(oracle_state* s, const float* v, uint32_t n, float hz)
{
    float p_tick = hz * (float)s->p.tick_ns;
    p_tick = p_tick * (float)1000000000ull;
    uint64_t now = s->clock;
    for (uint32_t i = 0; i < n && i < s->dims.n_input; ++i)
        if (host_uni(&s->rng) < p_tick * v[i]) s->last_fired[i] = now;
}

/* Brain::read_outputs, BR:145-157. */
void oracle_read_outputs(const oracle_state* s, uint8_t* out, uint32_t n)
{
    uint32_t now = (uint32_t)s->clock;          /* u32 (BR:149-153) */
    uint32_t start = now > 1 ? now - 1 : 0;
    for (uint32_t o = 0; o < n && o < s->dims.n_output; ++o) {
        uint32_t ts = (uint32_t)s->last_fired[s->dims.n_input + o];
        out[o] = (ts != 0 && ts >= start && ts < now) ? 1 : 0;
    }
}

/* The weight update of one event that reached it (MSL:91-122). */
static inline float updated_weight(const abnn_params* p, float w, int fired,
                                   float R, float rb, float isi)
{
    float dW = fired ? p->a_ltp * (1.0f - w) : (-p->a_ltd) * w;      /* MSL:101-102 */
    dW = dW + (p->eta_reward * (R - rb)) * (fired ? 1.0f : 0.0f);    /* MSL:105-107 */
    float est_hz = isi > 0.0f ? 1e6f / isi : 0.0f;                   /* MSL:116-117 */
    dW = dW + (p->eta_home * (p->target_rate_hz - est_hz)) * w;      /* MSL:118 */
    return clampf(w + dW, p->w_min, p->w_max);                       /* MSL:121 */
}

static inline int spike_candidate(const abnn_params* p, float w, uint64_t t_global, uint64_t now)
{
    float prob = clampf((w * w) * p->base_scale, 0.0f, 1.0f);         /* MSL:91 */
    return prob > oracle_rand01((uint32_t)t_global ^ (uint32_t)now);  /* MSL:92 */
}

/* ---- structural plasticity (README §5; contract in abnn.h) --------------- */
static const uint32_t kTomb = 0xFFFFFFFFu;

/* Store an updated weight, or remove the synapse if it fell below w_prune;
 * returns 1 if it was removed. */
static int store_weight(oracle_state* s, uint64_t e, float w)
{
    if (s->p.w_prune > 0.0f && w < s->p.w_prune) {
        s->syn[e].src = kTomb;
        s->syn[e].dst = kTomb;
        s->syn[e].w = w;
        s->syn[e].pad = 0.0f;
        return 1;
    }
    s->syn[e].w = w;
    return 0;
}

/* The spike in global budget slot k may grow a synapse from `src`. */
static void genesis(oracle_state* s, uint64_t k, uint32_t src)
{
    const abnn_params* p = &s->p;
    if (!(p->p_new > 0.0f) || p->compact_every == 0 || !s->grown) return;
    const uint64_t x = oracle_splitmix64_at(p->seed ^ ABNN_GENESIS_KEY, (s->pass_index << 32) | k);
    if (!((float)(x >> 40) * (1.0f / 16777216.0f) < p->p_new)) return;
    const uint64_t lo = s->dims.n_input, span = s->n_nrn - lo;
    abnn_synapse* g = &s->grown[(s->pass_index % p->compact_every) * p->max_spikes + k];
    g->src = src;
    g->dst = (uint32_t)(lo + (((x & 0xFFFFFFFFu) * span) >> 32));
    g->w = p->w_init;
    uint32_t one = 1u;
    memcpy(&g->pad, &one, 4);
}

/* After every compact_every-th pass: the tombstones removed (their holes filled
 * from the array's end), then the grown synapses in (pass, slot) order while
 * capacity lasts. */
static void structural_update(oracle_state* s)
{
    const abnn_params* p = &s->p;
    if (p->compact_every == 0 || s->pass_index % p->compact_every != 0) return;
    /* Removal (abnn.h contract, round 6): with D tombstones and m = n - D,
     * the k-th tombstone below m (in index order) takes the k-th live record
     * of the tail [m, n) (in index order), and the array ends at m.  Only the
     * filled holes' records move: O(D) -- a sweep prunes inside its visited
     * window, and the tail's live records (D of them at most) fill its holes. */
    uint64_t n = s->dims.n_syn, D = 0;
    for (uint64_t i = 0; i < n; ++i) D += s->syn[i].src == kTomb;
    if (D) {
        const uint64_t m = n - D;
        uint64_t from = m;  /* the next tail record to consider */
        for (uint64_t i = 0; i < m; ++i) {
            if (s->syn[i].src != kTomb) continue;
            while (s->syn[from].src == kTomb) ++from;  /* tail live records = holes below m */
            s->syn[i] = s->syn[from++];
        }
        n = m;
    }
    const uint64_t slots = (uint64_t)p->compact_every * p->max_spikes;
    for (uint64_t j = 0; s->grown && j < slots; ++j) {
        uint32_t flag;
        memcpy(&flag, &s->grown[j].pad, 4);
        if (flag == 1u && n < s->dims.syn_capacity) {
            s->syn[n] = s->grown[j];
            s->syn[n].pad = 0.0f;
            n++;
            s->stats.grown++;
        }
        memset(&s->grown[j], 0, sizeof(abnn_synapse));
    }
    s->dims.n_syn = n;
}

/* Random mode: weight stores collected in event order, resolved per record
 * (the highest event wins) at the end of the pass. */
typedef struct pend_w {
    uint64_t e, order;
    float w;
} pend_w;
typedef struct pend_list {
    pend_w* v;
    uint64_t n, cap;
} pend_list;

static void pend_push(pend_list* l, uint64_t e, float w)
{
    if (l->n == l->cap) {
        l->cap = l->cap ? 2 * l->cap : 1024;
        l->v = (pend_w*)realloc(l->v, l->cap * sizeof(pend_w));
    }
    l->v[l->n].e = e;
    l->v[l->n].order = l->n;
    l->v[l->n].w = w;
    l->n++;
}

static int pend_cmp(const void* a, const void* b)
{
    const pend_w *x = (const pend_w*)a, *y = (const pend_w*)b;
    if (x->e != y->e) return x->e < y->e ? -1 : 1;
    return x->order < y->order ? -1 : (x->order > y->order);
}

static void pend_resolve(oracle_state* s, pend_list* l)
{
    qsort(l->v, l->n, sizeof(pend_w), pend_cmp);
    for (uint64_t i = 0; i < l->n; ++i)
        if (i + 1 == l->n || l->v[i + 1].e != l->v[i].e) s->stats.pruned += store_weight(s, l->v[i].e, l->v[i].w);
    free(l->v);
    l->v = NULL;
    l->n = l->cap = 0;
}

/* Record visited by local event t (sweep: t itself). */
static inline uint64_t rec_index(const oracle_state* s, uint64_t t)
{
    if (s->p.mode != ABNN_MODE_RANDOM) return t;
    return oracle_pick(s->p.seed, s->dims.syn_offset, s->pass_index, t, s->dims.n_syn);
}

static uint64_t events_of(const oracle_state* s) { return oracle_visited_events(&s->dims, s->p.mode); }

/* Pass start: auto-stimulus (the bench's "all inputs fire") and the host's
 * renormalisation decision, taken on the pass-start clock (BR:127-128). */
static int pass_begin(oracle_state* s)
{
    uint64_t now = s->clock;
    for (uint64_t i = 0; i < s->stim_count; ++i)
        if (s->stim_first + i < s->n_nrn) s->last_fired[s->stim_first + i] = now;
    return (uint64_t)(uint32_t)now > s->p.renorm_thresh;  /* u32 clock, BR:127-128 */
}

/* Pass end: deferred stamps, rBar, clock tick (MSL:110-113,125-129), then the
 * renormalisation kernel (MSL:135-145) with base = the ticked clock. */
static void pass_end(oracle_state* s, const uint32_t* fired, uint64_t n_fired,
                     int t0_updated, uint64_t global_events, int renorm)
{
    uint64_t now = s->clock;
    for (uint64_t i = 0; i < n_fired; ++i) s->last_fired[fired[i]] = now;
    if (t0_updated && s->p.max_spikes > 0)
        s->rbar = s->rbar + s->p.alpha_rbar * (s->reward - s->rbar);
    if (global_events > 0) s->clock = now + s->p.clock_inc;
    if (renorm) {
        uint64_t base = s->clock;
        for (uint64_t i = 0; i < s->n_nrn; ++i) s->last_fired[i] -= base;
        s->clock = 0;
        s->renorms += 1;
    }
    s->stats.passes += 1;
    s->pass_index += 1;
    structural_update(s);
}

/* ---- the oracle of record: literal serial C1 loop ------------------------ */
void oracle_pass_serial(oracle_state* s)
{
    const abnn_params* p = &s->p;
    int renorm = pass_begin(s);
    const uint64_t now = s->clock;                 /* per-TG clock cache, MSL:63-68 */
    const uint64_t E = events_of(s);
    const uint64_t* L = s->last_fired;             /* pass-start snapshot (C1)       */
    const float R = s->reward, rb = s->rbar;        /* MSL:105-106                    */
    uint32_t budget = p->max_spikes;               /* reset per pass, BR:90          */
    uint32_t* fired = (uint32_t*)malloc(sizeof(uint32_t) * (p->max_spikes + 1u));
    uint64_t n_fired = 0;
    int t0_updated = 0;
    const int random = p->mode == ABNN_MODE_RANDOM;
    /* random mode: weights are written after the sweep, so every event reads
     * the pass-start record; of several stores to one record the last wins */
    pend_list pend = {NULL, 0, 0};

    for (uint64_t t = 0; t < E; ++t) {
        const uint64_t e = rec_index(s, t);
        abnn_synapse sy = s->syn[e];               /* MSL:70 */
        uint64_t tg = s->dims.syn_offset + t;
        if (p->track_visits && sy.dst < s->n_nrn) {  /* README §4 */
            s->last_visited[sy.dst] = now;
            if (s->visit_mark) s->visit_mark[sy.dst] = 1;
        }
        if (sy.src >= s->n_nrn) continue;                       /* removed synapse (README §5) */
        if (age32(now, L[sy.src]) > p->window_pre) continue;    /* MSL:73-77 */
        s->stats.pre_gated++;
        uint64_t ld = L[sy.dst];                                /* MSL:79 */
        if (age32(now, ld) <= p->refractory) continue;          /* MSL:80-83 */
        s->stats.post_gated++;
        if (budget == 0) continue;                              /* MSL:85-88 */
        s->stats.updated++;
        int f = spike_candidate(p, sy.w, tg, now);              /* MSL:91-92 */
        if (f) budget -= 1;                                     /* MSL:95-98 (C1: never loses) */
        if (tg == 0) t0_updated = 1;                            /* MSL:110-113 */
        float isi = (float)age32(now, ld);                      /* MSL:116 (u32) */
        float w = updated_weight(p, sy.w, f, R, rb, isi);       /* MSL:101-121 */
        if (!random) s->stats.pruned += store_weight(s, t, w);  /* MSL:122 (+ pruning) */
        else pend_push(&pend, e, w);
        if (f) {
            genesis(s, n_fired, sy.src);                        /* README §5 */
            fired[n_fired++] = sy.dst;                          /* MSL:125-126 (deferred) */
        }
    }
    pend_resolve(s, &pend);
    s->stats.events += E;
    s->stats.fired += n_fired;
    pass_end(s, fired, n_fired, t0_updated,
             s->dims.global_events ? s->dims.global_events : E, renorm);
    free(fired);
}

/* ---- sharded / threaded phases -------------------------------------------- */
typedef struct g2vec {
    oracle_g2* v;
    uint64_t n, cap;
    int owned;
    int overflow;
} g2vec;

static int g2_push(g2vec* g, const oracle_g2* e)
{
    if (g->n == g->cap) {
        if (!g->owned) { g->overflow = 1; return 0; }
        uint64_t nc = g->cap ? g->cap * 2 : 1024;
        oracle_g2* nv = (oracle_g2*)realloc(g->v, nc * sizeof(oracle_g2));
        if (!nv) { g->overflow = 1; return 0; }
        g->v = nv;
        g->cap = nc;
    }
    g->v[g->n++] = *e;
    return 1;
}

typedef struct gate_counts {
    uint64_t g1, g2, cand;
    int t0;
} gate_counts;

/* Gate events [t0, t1) of the local sweep: both gates and the spike-candidate
 * test; entries whose local candidate prefix already reaches the budget can
 * never be updated (offsets only add) and are counted but not stored. */
static void gate_range(const oracle_state* s, uint64_t t0, uint64_t t1, g2vec* out,
                       gate_counts* c)
{
    const abnn_params* p = &s->p;
    const uint64_t now = s->clock;
    const uint64_t* L = s->last_fired;
    memset(c, 0, sizeof(*c));
    for (uint64_t t = t0; t < t1; ++t) {
        abnn_synapse sy = s->syn[rec_index(s, t)];
        /* lastVisited is never read by a decision: written as visited, with
         * the same value `now` from every thread */
        if (p->track_visits && sy.dst < s->n_nrn) {
            s->last_visited[sy.dst] = now;
            if (s->visit_mark) s->visit_mark[sy.dst] = 1;  /* the shard merge's marks (abnn.h) */
        }
        if (sy.src >= s->n_nrn) continue;  /* removed synapse */
        if (age32(now, L[sy.src]) > p->window_pre) continue;
        c->g1++;
        uint64_t ld = L[sy.dst];
        if (age32(now, ld) <= p->refractory) continue;
        c->g2++;
        uint64_t tg = s->dims.syn_offset + t;
        if (tg == 0) c->t0 = 1;
        if (c->cand >= p->max_spikes) continue;
        oracle_g2 e;
        e.t = t;
        e.isi = (float)age32(now, ld);
        e.pre = (uint32_t)c->cand;
        e.cand = (uint32_t)spike_candidate(p, sy.w, tg, now);
        e.w = sy.w;
        c->cand += e.cand;
        g2_push(out, &e);
    }
}

/* Apply stored entries with global budget offset `off` (exclusive count of
 * candidates in all earlier shards, capped); returns spikes emitted. */
static uint64_t apply_range(oracle_state* s, const oracle_g2* g, uint64_t n, uint64_t off,
                            int32_t* fired, uint64_t* updated, pend_list* pend, uint64_t* pruned)
{
    const abnn_params* p = &s->p;
    const float R = s->reward, rb = s->rbar;
    uint64_t nf = 0, nu = 0;
    for (uint64_t j = 0; j < n; ++j) {
        uint64_t pre = off + g[j].pre;
        if (pre >= p->max_spikes) break; /* entries are in order: the rest are inactive */
        const uint64_t e = rec_index(s, g[j].t);
        const abnn_synapse sy = s->syn[e];  /* pass-start src/dst (stores below) */
        const float w = updated_weight(p, g[j].w, (int)g[j].cand, R, rb, g[j].isi);  /* pass-start w */
        if (pend) pend_push(pend, e, w);
        else *pruned += (uint64_t)store_weight(s, e, w);
        nu++;
        if (g[j].cand) {
            genesis(s, pre, sy.src);
            fired[pre] = (int32_t)sy.dst;
            nf++;
        }
    }
    *updated = nu;
    return nf;
}

uint32_t oracle_exchange_words(uint32_t max_spikes)
{
    return 2u * ABNN_SUMMARY_WORDS + ((max_spikes + 1u) & ~1u);
}

int64_t oracle_shard_gate(oracle_state* s, oracle_g2* out, uint64_t cap, int32_t* xchg)
{
    (void)pass_begin(s); /* stimulus; the renorm decision is re-taken in commit */
    uint64_t E = events_of(s);
    g2vec g = {out, 0, cap, 0, 0};
    gate_counts c;
    gate_range(s, 0, E, &g, &c);
    s->stats.pre_gated += c.g1;
    s->stats.post_gated += c.g2;
    s->stats.events += E;
    int64_t* summary = (int64_t*)xchg;
    int32_t* spikes = xchg + 2 * ABNN_SUMMARY_WORDS;
    summary[0] = (int64_t)(c.cand < s->p.max_spikes ? c.cand : s->p.max_spikes);
    summary[1] = c.t0;
    summary[2] = (int64_t)E;
    summary[3] = (int64_t)c.g2;
    memset(spikes, 0, sizeof(int32_t) * ((s->p.max_spikes + 1u) & ~1u));
    for (uint64_t j = 0; j < g.n; ++j)  /* local spikes in local budget order */
        if (g.v[j].cand) spikes[g.v[j].pre] = (int32_t)s->syn[rec_index(s, g.v[j].t)].dst;
    return g.overflow ? -1 : (int64_t)g.n;
}

static uint64_t shard_offset(const int32_t* gathered, uint32_t rank, uint32_t budget)
{
    const uint32_t words = oracle_exchange_words(budget);
    uint64_t off = 0;
    for (uint32_t r = 0; r < rank; ++r) off += (uint64_t) * (const int64_t*)(gathered + r * words);
    return off < budget ? off : budget;
}

void oracle_shard_apply(oracle_state* s, const oracle_g2* g2, int64_t n_g2,
                        const int32_t* gathered, uint32_t world, uint32_t rank)
{
    (void)world;
    int32_t* fired = (int32_t*)calloc(s->p.max_spikes + 1u, sizeof(int32_t)); /* unused: stamps come from the records */
    uint64_t off = shard_offset(gathered, rank, s->p.max_spikes);
    uint64_t nu = 0;
    pend_list pend = {NULL, 0, 0};
    const int random = s->p.mode == ABNN_MODE_RANDOM;
    uint64_t np = 0;
    uint64_t nf = apply_range(s, g2, (uint64_t)n_g2, off, fired, &nu, random ? &pend : NULL, &np);
    if (random) pend_resolve(s, &pend);
    s->stats.pruned += np;
    s->stats.updated += nu;
    s->stats.fired += nf;
    free(fired);
}

void oracle_shard_commit(oracle_state* s, const int32_t* gathered, uint32_t world)
{
    const uint32_t words = oracle_exchange_words(s->p.max_spikes);
    const uint64_t budget = s->p.max_spikes;
    uint64_t events = 0, off = 0;
    int64_t t0 = 0;
    int renorm = (uint64_t)(uint32_t)s->clock > s->p.renorm_thresh;
    uint64_t now = s->clock;
    for (uint32_t r = 0; r < world; ++r) {
        const int64_t* sm = (const int64_t*)(gathered + r * words);
        const int32_t* sp = gathered + r * words + 2 * ABNN_SUMMARY_WORDS;
        events += (uint64_t)sm[2];
        t0 |= sm[1];
        uint64_t room = budget - off, n = (uint64_t)sm[0] < room ? (uint64_t)sm[0] : room;
        for (uint64_t i = 0; i < n; ++i) s->last_fired[(uint32_t)sp[i]] = now;  /* rank order = budget order */
        off += n;
    }
    if (t0 && s->p.max_spikes > 0)
        s->rbar = s->rbar + s->p.alpha_rbar * (s->reward - s->rbar);
    if (events > 0) s->clock = now + s->p.clock_inc;
    if (renorm) {
        uint64_t base = s->clock;
        for (uint64_t i = 0; i < s->n_nrn; ++i) s->last_fired[i] -= base;
        s->clock = 0;
        s->renorms += 1;
    }
    s->stats.passes += 1;
    s->pass_index += 1;
    structural_update(s);
}

/* ---- threaded pass: nthreads contiguous virtual shards ------------------- */
typedef struct thr_job {
    oracle_state* s;
    uint64_t t0, t1, off;
    g2vec g;
    gate_counts c;
    int32_t* fired;
    uint64_t nf, nu, np;
    int phase;
    pend_list* pend;  /* random mode: shared, the apply phase runs serially */
} thr_job;

static void* thr_worker(void* arg)
{
    thr_job* j = (thr_job*)arg;
    if (j->phase == 0)
        gate_range(j->s, j->t0, j->t1, &j->g, &j->c);
    else
        j->nf = apply_range(j->s, j->g.v, j->g.n, j->off, j->fired, &j->nu, j->pend, &j->np);
    return NULL;
}

void oracle_pass_threaded(oracle_state* s, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    const abnn_params* p = &s->p;
    int renorm = pass_begin(s);
    uint64_t E = events_of(s);
    thr_job* jobs = (thr_job*)calloc((size_t)nthreads, sizeof(thr_job));
    pthread_t th[256];
    uint64_t per = (E + (uint64_t)nthreads - 1) / (uint64_t)nthreads;
    int32_t* fired = (int32_t*)calloc(p->max_spikes + 1u, sizeof(int32_t));
    pend_list pend = {NULL, 0, 0};
    for (int k = 0; k < nthreads; ++k) {
        jobs[k].pend = p->mode == ABNN_MODE_RANDOM ? &pend : NULL;
        jobs[k].s = s;
        jobs[k].t0 = per * (uint64_t)k < E ? per * (uint64_t)k : E;
        jobs[k].t1 = jobs[k].t0 + per < E ? jobs[k].t0 + per : E;
        jobs[k].g.owned = 1;
        jobs[k].fired = fired;
    }
    for (int phase = 0; phase < 2; ++phase) {
        if (phase == 1) { /* serial prefix over the shards' candidate counts */
            uint64_t off = 0;
            for (int k = 0; k < nthreads; ++k) {
                jobs[k].off = off < p->max_spikes ? off : p->max_spikes;
                off += jobs[k].c.cand;
            }
        }
        /* random mode: shards may pick the same synapse, so the writes go in
         * event order (shard order) on one thread; the gate phase is parallel */
        const int serial = nthreads == 1 || (phase == 1 && p->mode == ABNN_MODE_RANDOM);
        for (int k = 0; k < nthreads; ++k) {
            jobs[k].phase = phase;
            if (serial) thr_worker(&jobs[k]);
            else pthread_create(&th[k], NULL, thr_worker, &jobs[k]);
        }
        if (!serial)
            for (int k = 0; k < nthreads; ++k) pthread_join(th[k], NULL);
    }
    pend_resolve(s, &pend);
    uint64_t total = 0, nf = 0;
    int t0 = 0;
    for (int k = 0; k < nthreads; ++k) {
        s->stats.pre_gated += jobs[k].c.g1;
        s->stats.post_gated += jobs[k].c.g2;
        s->stats.updated += jobs[k].nu;
        s->stats.pruned += jobs[k].np;
        total += jobs[k].c.cand;
        nf += jobs[k].nf;
        t0 |= jobs[k].c.t0;
        free(jobs[k].g.v);
    }
    uint64_t n_fired = total < p->max_spikes ? total : p->max_spikes;
    (void)nf;
    s->stats.events += E;
    s->stats.fired += n_fired;
    uint32_t* fu = (uint32_t*)fired;
    pass_end(s, fu, n_fired, t0, s->dims.global_events ? s->dims.global_events : E, renorm);
    free(fired);
    free(jobs);
}
