// brain_cpp_test.cpp -- drives the C++ Brain API (include/abnn/brain.hpp) the
// way BrainEngine::run_one_pass drives the reference (brain-engine.cpp:108-190,
// minus stimulus files and GUI): inject inputs, one pass, read outputs, reward.
// Prints a JSON line that tests/test_cpp_api.py compares against the oracle.
#include <abnn/brain.hpp>

#include <cinttypes>
#include <cstdio>
#include <sstream>

int main()
{
    try {
        abnn::Brain brain(256, 256, 488, 10'000, 100'000);
        brain.build_pipeline();
        brain.build_buffers();
        brain.build_random_graph(1);
        std::vector<float> in(256);
        for (int i = 0; i < 256; ++i) in[i] = (i % 3 == 0) ? 0.5f : 0.0f;
        uint64_t outputs_fired = 0;
        for (int pass = 0; pass < 24; ++pass) {
            brain.inject_inputs(in, 1000.0f);
            if (pass == 12) brain.set_reward(0.5f);
            brain.encode_traversal();
            brain.synchronize();
            for (bool b : brain.read_outputs()) outputs_fired += b ? 1 : 0;
        }
        // .bnn round trip through an in-memory stream (brain.cpp:161-178)
        std::stringstream ss;
        brain.save(ss);
        abnn::Brain copy(256, 256, 488, 10'000, 100'000);
        copy.load(ss);
        bool mismatch_thrown = false;
        try {
            abnn::Brain other(256, 256, 489, 10'000, 100'000);
            std::stringstream s2(ss.str());
            other.load(s2);
        } catch (const abnn::size_mismatch&) {
            mismatch_thrown = true;
        }
        // The reference caller's own code shapes (brain-engine.cpp:31-53,
        // 119-134, 180-182) through the MTL::Buffer-like views: records
        // written into synapse_buffer()->contents() + didModifyRange,
        // teacher spikes poked into the u32 lastFired view, the reward through
        // its view, the budget read after every pass (brain.h:54-58).
        uint64_t views_checksum = 0, budget_sum = 0, views_outputs = 0;
        {
            abnn::Brain vb(256, 256, 488, 10'000, 100'000);
            vb.build_pipeline();
            vb.build_buffers();
            auto* syn = reinterpret_cast<abnn::SynapsePacked*>(vb.synapse_buffer()->contents());
            const uint32_t max = vb.n_syn();
            for (uint32_t i = 0; i < max; ++i)  // a reproducible graph (tests/test_cpp_api.py restates it)
                syn[i] = {(i * 7919u) % vb.n_neuron(), (i * 104729u + 13u) % vb.n_neuron(),
                          0.1f + (float)(i % 1000) / 1000.0f, 0.0f};
            vb.synapse_buffer()->didModifyRange(abnn::Range(0, (uint64_t)max * sizeof(abnn::SynapsePacked)));
            for (int pass = 0; pass < 24; ++pass) {
                vb.inject_inputs(in, 1000.0f);
                uint32_t* lf = (uint32_t*)vb.last_fired_buffer()->contents();
                const uint32_t now = *(uint32_t*)vb.clock_buffer()->contents();
                if (pass % 2 == 0)
                    for (uint32_t o = 0; o < vb.n_output(); ++o)
                        if (o % 5 == (uint32_t)pass % 5 && now - lf[vb.n_input() + o] > 1) lf[vb.n_input() + o] = now;
                if (pass == 12) {
                    float* r = (float*)vb.reward_buffer()->contents();
                    *r = 0.25f;
                    vb.reward_buffer()->didModifyRange(abnn::Range(0, 4));
                }
                vb.encode_traversal();
                vb.synchronize();
                budget_sum += *(uint32_t*)vb.budget_buffer()->contents();
                for (bool b : vb.read_outputs()) views_outputs += b ? 1 : 0;
            }
            views_checksum = vb.checksum();
            bool threw = false;
            try {
                *(uint32_t*)vb.budget_buffer()->contents() = 7;
                vb.budget_buffer()->didModifyRange(abnn::Range(0, 4));
            } catch (const std::logic_error&) {
                threw = true;
            }
            if (!threw) throw std::runtime_error("budget_buffer() accepted a write");
        }
        // Both Shared views (lastFired and the clock) written before the next
        // device operation: both writes reach the device (brain.cpp:55-57).
        bool shared_both_ok = false;
        {
            abnn::Brain sb(256, 256, 488, 10'000, 100'000);
            sb.build_random_graph(1);
            uint32_t* lf = (uint32_t*)sb.last_fired_buffer()->contents();
            uint32_t* clk = (uint32_t*)sb.clock_buffer()->contents();
            lf[300] = 4242u;
            *clk = 5000u;
            const abnn_scalars s0 = sb.scalars();            // a device operation flushes both
            const uint64_t lf300 = sb.last_fired(300, 1)[0];
            const uint32_t seen_clk = *(uint32_t*)sb.clock_buffer()->contents();
            const uint32_t seen_lf = ((uint32_t*)sb.last_fired_buffer()->contents())[300];
            lf = (uint32_t*)sb.last_fired_buffer()->contents();
            clk = (uint32_t*)sb.clock_buffer()->contents();
            lf[301] = 4999u;
            *clk = 6000u;
            sb.encode_traversal();                           // ... and so does a pass
            sb.synchronize();
            const abnn_scalars s1 = sb.scalars();
            const uint64_t lf301 = sb.last_fired(301, 1)[0];
            shared_both_ok = s0.clock == 5000u && lf300 == 4242u && seen_clk == 5000u && seen_lf == 4242u &&
                             s1.clock == 6001u && (lf301 == 4999u || lf301 == 6000u);
        }
        const abnn_scalars sc = brain.scalars();
        uint64_t lf_sum = 0;
        for (uint64_t v : brain.last_fired()) lf_sum += v;
        std::printf("{\"clock\": %" PRIu64 ", \"rbar\": %.9g, \"checksum\": %" PRIu64
                    ", \"copy_checksum\": %" PRIu64 ", \"last_fired_sum\": %" PRIu64
                    ", \"outputs_fired\": %" PRIu64 ", \"mismatch_thrown\": %s, \"views_checksum\": %" PRIu64
                    ", \"budget_sum\": %" PRIu64 ", \"views_outputs\": %" PRIu64 ", \"shared_both_ok\": %s}\n",
                    sc.clock, (double)sc.rbar, brain.checksum(), copy.checksum(), lf_sum,
                    outputs_fired, mismatch_thrown ? "true" : "false", views_checksum, budget_sum, views_outputs,
                    shared_both_ok ? "true" : "false");
        return 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
}
