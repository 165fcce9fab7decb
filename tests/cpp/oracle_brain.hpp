// oracle_brain.hpp -- TEST INFRASTRUCTURE: the CPU oracle (oracle/c1_oracle.c)
// behind the pass-boundary surface abnn::BrainEngine drives, so the same
// driver code runs over the GPU brain and over the oracle.
#pragma once

#include <cstdint>
#include <stdexcept>
#include <vector>

#include "../../oracle/c1_oracle.h"

struct OracleBrain {
    OracleBrain(uint32_t n_in, uint32_t n_out, uint64_t n_hid, uint64_t n_syn, uint64_t events,
                const abnn_params* params = nullptr)
    {
        s_ = oracle_state{};
        if (params) s_.p = *params;
        else oracle_default_params(&s_.p);
        s_.dims = abnn_dims{n_in, n_out, n_hid, n_syn, events, 0, 0};
        s_.n_nrn = (uint64_t)n_in + n_out + n_hid;
        syn_.resize(n_syn);
        lf_.assign(s_.n_nrn, 0);
        lv_.assign(s_.n_nrn, 0);
        s_.syn = syn_.data();
        s_.last_fired = lf_.data();
        s_.last_visited = lv_.data();
        s_.rng = s_.p.seed;
    }
    void build_random_graph(uint64_t seed = 1)
    {
        oracle_gen_synapses(syn_.data(), 0, syn_.size(), s_.dims.n_input, s_.dims.n_output, s_.n_nrn, seed, 4);
    }
    uint32_t n_input() const { return s_.dims.n_input; }
    uint32_t n_output() const { return s_.dims.n_output; }
    void inject_inputs(const std::vector<float>& v, float hz)
    {
        oracle_inject_inputs(&s_, v.data(), (uint32_t)v.size(), hz);
    }
    abnn_scalars scalars() const { return abnn_scalars{s_.clock, s_.reward, s_.rbar}; }
    std::vector<uint64_t> last_fired(uint64_t first, uint64_t n) const
    {
        return std::vector<uint64_t>(lf_.begin() + first, lf_.begin() + first + n);
    }
    void set_timestamps(const std::vector<uint32_t>& idx, uint64_t v)
    {
        for (uint32_t i : idx)
            if (i < s_.n_nrn) lf_[i] = v;
    }
    void encode_traversal(void* = nullptr, uint32_t passes = 1)
    {
        for (uint32_t k = 0; k < passes; ++k) oracle_pass_serial(&s_);
    }
    void synchronize(void* = nullptr) {}
    std::vector<bool> read_outputs() const
    {
        std::vector<uint8_t> o(s_.dims.n_output);
        oracle_read_outputs(&s_, o.data(), (uint32_t)o.size());
        return std::vector<bool>(o.begin(), o.end());
    }
    void set_reward(float r) { s_.reward = r; }
    template <class OS> void save(OS&) const { throw std::runtime_error("not used"); }
    template <class IS> void load(IS&) { throw std::runtime_error("not used"); }

    const std::vector<abnn_synapse>& synapses() const { return syn_; }
    const std::vector<uint64_t>& all_last_fired() const { return lf_; }
    float rbar() const { return s_.rbar; }

    oracle_state s_;
    std::vector<abnn_synapse> syn_;
    std::vector<uint64_t> lf_, lv_;
};
