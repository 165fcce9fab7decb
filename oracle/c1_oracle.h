/*
 * c1_oracle.h -- CPU restatement of the reference hot path.  TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, never by the product (abnn_amd/).
 *
 * PARITY UNPINNED: the reference (tjamescouch/abnn) ships no tests, golden
 * vectors or fixtures for this path, and its kernel (brain.metal) needs the
 * Metal toolchain and <metal_stdlib>, neither of which exists in this image,
 * so it cannot be run here.  This file restates the algorithm
 * of abnn/src/core/kernels/brain.metal:15-19,41-145 and
 * abnn/src/core/brain/brain.cpp:73-178 under the deterministic legal schedule
 * C1; it is cross-checked against an independent pure-Python
 * restatement and hand-derived known answers in tests/.
 */
#ifndef ABNN_C1_ORACLE_H
#define ABNN_C1_ORACLE_H

#include <stdint.h>
#include "../include/abnn/abnn.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Oracle state: all arrays owned by the caller (numpy in tests). */
typedef struct oracle_state {
    abnn_dims dims;
    abnn_params p;
    uint64_t n_nrn;
    abnn_synapse* syn;          /* dims.n_syn records (local shard)        */
    uint64_t* last_fired;       /* n_nrn                                   */
    uint64_t* last_visited;     /* n_nrn                                   */
    uint64_t clock;
    float reward;
    float rbar;
    uint64_t rng;               /* host RNG state (inject_inputs)          */
    uint64_t stim_first, stim_count;
    abnn_stats stats;
    uint64_t pass_index;        /* passes run (keys the random-mode picks)   */
    abnn_synapse* grown;        /* structural plasticity: compact_every *
                                   max_spikes slots, zeroed by the caller;
                                   a grown synapse has pad bits = 1          */
    uint8_t* visit_mark;        /* shard with track_visits: n_nrn, 1 = visited
                                   since the last lastVisited merge (the
                                   caller merges, abnn.h); NULL = none       */
    uint64_t renorms;           /* renormalisations run                     */
} oracle_state;

/* One G2 entry (event that passed both gates) of a shard, in event order. */
typedef struct oracle_g2 {
    uint64_t t;                 /* local event index                       */
    float isi;                  /* (float)(now - lastFired[dst])           */
    uint32_t pre;               /* local exclusive count of spike candidates */
    uint32_t cand;              /* 1 if p > rand01                         */
    float w;                    /* pass-start weight of the visited record */
} oracle_g2;

void oracle_default_params(abnn_params* p);
float oracle_rand01(uint32_t s);
uint64_t oracle_splitmix64_at(uint64_t seed, uint64_t k);
uint64_t oracle_visited_events(const abnn_dims* d, uint32_t mode);
/* Philox4x32-10 (Salmon et al., SC'11; the Random123 constants) and the
 * random-mode pick of abnn.h: record visited by local event t. */
void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
uint64_t oracle_pick(uint64_t seed, uint64_t stream, uint64_t pass, uint64_t t, uint64_t n_syn);
void oracle_gen_synapse(uint64_t i, uint32_t n_in, uint32_t n_out, uint64_t n_nrn,
                        uint64_t seed, abnn_synapse* out);
void oracle_gen_synapses(abnn_synapse* out, uint64_t first_global, uint64_t n,
                         uint32_t n_in, uint32_t n_out, uint64_t n_nrn,
                         uint64_t seed, int nthreads);
uint64_t oracle_checksum_synapses(const abnn_synapse* s, uint64_t n, uint64_t first_global);

void oracle_inject_inputs(oracle_state* s, const float* v, uint32_t n, float hz);
void oracle_read_outputs(const oracle_state* s, uint8_t* out, uint32_t n);

/* One whole pass, literal serial C1 loop (the oracle of record). */
void oracle_pass_serial(oracle_state* s);
/* One whole pass as nthreads virtual shards (3 phases, bit-exact to serial);
 * the CPU baseline timed by bench.py. */
void oracle_pass_threaded(oracle_state* s, int nthreads);

/* Sharded phases with one exchange (abnn.h): gate writes this shard's
 * record (summary + local spike list, oracle_exchange_words int32), the
 * caller all-gathers the W records in rank order, apply and commit read
 * them.  Returns the number of stored G2 entries (-1: `out` overflowed). */
uint32_t oracle_exchange_words(uint32_t max_spikes);
int64_t oracle_shard_gate(oracle_state* s, oracle_g2* out, uint64_t cap, int32_t* xchg);
void oracle_shard_apply(oracle_state* s, const oracle_g2* g2, int64_t n_g2,
                        const int32_t* gathered, uint32_t world, uint32_t rank);
void oracle_shard_commit(oracle_state* s, const int32_t* gathered, uint32_t world);

#ifdef __cplusplus
}
#endif
#endif
