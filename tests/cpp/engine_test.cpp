// engine_test.cpp -- TEST PROGRAM: the learning driver (include/abnn/engine.hpp,
// BrainEngine::run_one_pass of brain-engine.cpp:108-190) run over the GPU
// brain and over the CPU oracle with the same stimulus; every pass's output
// spikes and normalised rates, every window's loss and reward, and the final
// weights / lastFired / clock / rBar must agree bit for bit.
//   usage: engine_test PASSES WIN_SIZE   (prints one JSON line)
#include <abnn/brain.hpp>
#include <abnn/engine.hpp>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "oracle_brain.hpp"

static std::shared_ptr<abnn::FunctionalDataset> dataset()
{
    // the app's stimulus (view-delegate.cpp:32-42): cos^2 input, 0.5 sin + 0.5 target
    return std::make_shared<abnn::FunctionalDataset>(256, 256, 0.0009, 0.5, abnn::FunctionalDataset::cos_squared,
                                                     abnn::FunctionalDataset::half_sine);
}

int main(int argc, char** argv)
{
    const int passes = argc > 1 ? std::atoi(argv[1]) : 300;
    const std::size_t win = argc > 2 ? (std::size_t)std::atoll(argv[2]) : 50;
    const uint32_t n_in = 256, n_out = 256;
    const uint64_t n_hid = 488, n_syn = 10000, events = 100000;  // config 1

    abnn::Brain gpu(n_in, n_out, n_hid, n_syn, events);
    gpu.build_random_graph(1);
    OracleBrain cpu(n_in, n_out, n_hid, n_syn, events);
    cpu.build_random_graph(1);

    abnn::EngineConfig cfg;
    cfg.win_size = win;
    abnn::BrainEngine<abnn::Brain> eg(gpu, cfg);
    abnn::BrainEngine<OracleBrain> ec(cpu, cfg);
    eg.set_stimulus(dataset());
    ec.set_stimulus(dataset());

    uint64_t spikes = 0;
    for (int k = 0; k < passes; ++k) {
        const std::vector<bool> og = eg.run_one_pass(), oc = ec.run_one_pass();
        if (og != oc) {
            std::printf("{\"ok\": false, \"pass\": %d, \"what\": \"outputs\"}\n", k);
            return 1;
        }
        if (std::memcmp(eg.smooth_rates().data(), ec.smooth_rates().data(), n_out * sizeof(float)) != 0) {
            std::printf("{\"ok\": false, \"pass\": %d, \"what\": \"rates\"}\n", k);
            return 1;
        }
        if (eg.last_loss() != ec.last_loss() || eg.last_reward() != ec.last_reward()) {
            std::printf("{\"ok\": false, \"pass\": %d, \"what\": \"loss\"}\n", k);
            return 1;
        }
        for (bool b : og) spikes += b ? 1 : 0;
    }
    std::vector<abnn::SynapsePacked> w(n_syn);
    abnn::check(abnn_download_synapses(gpu.handle(), 0, reinterpret_cast<abnn_synapse*>(w.data()), n_syn),
                "download");
    const bool syn_ok = std::memcmp(w.data(), cpu.synapses().data(), n_syn * sizeof(abnn_synapse)) == 0;
    const bool lf_ok = gpu.last_fired() == cpu.all_last_fired();
    const abnn_scalars sg = gpu.scalars(), sc = cpu.scalars();
    const bool sc_ok = sg.clock == sc.clock && std::memcmp(&sg.rbar, &sc.rbar, 4) == 0 &&
                       std::memcmp(&sg.reward, &sc.reward, 4) == 0;
    std::printf("{\"ok\": %s, \"passes\": %d, \"windows\": %llu, \"spikes\": %llu, \"loss\": %.17g, "
                "\"reward\": %.9g, \"clock\": %llu, \"synapses\": %s, \"last_fired\": %s, \"scalars\": %s}\n",
                (syn_ok && lf_ok && sc_ok) ? "true" : "false", passes, (unsigned long long)eg.windows(),
                (unsigned long long)spikes, eg.last_loss(), eg.last_reward(), (unsigned long long)sg.clock,
                syn_ok ? "true" : "false", lf_ok ? "true" : "false", sc_ok ? "true" : "false");
    return (syn_ok && lf_ok && sc_ok) ? 0 : 1;
}
