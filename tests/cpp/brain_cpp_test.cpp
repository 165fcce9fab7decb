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
        const abnn_scalars sc = brain.scalars();
        uint64_t lf_sum = 0;
        for (uint64_t v : brain.last_fired()) lf_sum += v;
        std::printf("{\"clock\": %" PRIu64 ", \"rbar\": %.9g, \"checksum\": %" PRIu64
                    ", \"copy_checksum\": %" PRIu64 ", \"last_fired_sum\": %" PRIu64
                    ", \"outputs_fired\": %" PRIu64 ", \"mismatch_thrown\": %s}\n",
                    sc.clock, (double)sc.rbar, brain.checksum(), copy.checksum(), lf_sum,
                    outputs_fired, mismatch_thrown ? "true" : "false");
        return 0;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 2;
    }
}
