// brain.hpp -- header-only C++ `Brain` over the C-ABI (abnn.h).
//
// Mirrors the reference host class abnn/src/core/brain/brain.h:24-83 so that a
// BrainEngine-style caller changes only what Metal forced on it (see
// INTEGRATION.md):
//   Brain(nInput, nOutput, nHidden, nSynapses, eventsPerPass)   brain.h:27-31
//   build_pipeline / build_buffers                               brain.h:35-36
//   encode_traversal                                             brain.h:39
//   inject_inputs / read_outputs                                 brain.h:40-41
//   save(ostream&) / load(istream&)                              brain.h:44-45
//   n_input() ... n_syn()                                        brain.h:48-52
//   synapse_buffer() ... reward_buffer()  (device pointers)      brain.h:54-58
// Errors throw std::runtime_error (the reference threw a pointer,
// brain.cpp:174); a .bnn size mismatch throws abnn::size_mismatch.
#pragma once

#include <cstdint>
#include <istream>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "abnn.h"

namespace abnn {

using SynapsePacked = abnn_synapse;  // {u32 src, u32 dst, f32 w, f32 pad}, brain.h:21

static constexpr uint32_t kTickNS = 1000;             // brain.h:17
static constexpr uint32_t kMaxSpikes = 2560;          // brain.h:18
static constexpr uint32_t kRenormThresh = 4'000'000;  // brain.h:19

struct size_mismatch : std::runtime_error {
    using std::runtime_error::runtime_error;
};

inline void check(abnn_status s, const char* what)
{
    if (s == ABNN_OK) return;
    std::string m = std::string(what) + ": " + abnn_status_string(s) + " (" + abnn_last_error() + ")";
    if (s == ABNN_ERR_SIZE_MISMATCH) throw size_mismatch(m);
    throw std::runtime_error(m);
}

class Brain {
public:
    Brain(uint32_t nInput, uint32_t nOutput, uint32_t nHidden, uint32_t nSynapses,
          uint32_t eventsPerPass, int device = 0, const abnn_params* params = nullptr)
    {
        abnn_dims d{};
        d.n_input = nInput;
        d.n_output = nOutput;
        d.n_hidden = nHidden;
        d.n_syn = nSynapses;
        d.events_per_pass = eventsPerPass;
        check(abnn_brain_create(&d, params, device, &h_), "abnn_brain_create");
    }
    ~Brain() { abnn_brain_destroy(h_); }
    Brain(const Brain&) = delete;
    Brain& operator=(const Brain&) = delete;

    // brain.h:35-36.  Kernels are compiled into the library and buffers are
    // allocated (zeroed) by the constructor; build_buffers re-zeroes the state.
    void build_pipeline() {}
    void build_buffers()
    {
        std::vector<uint64_t> z(n_neuron(), 0);
        check(abnn_set_last_fired(h_, 0, z.data(), z.size()), "abnn_set_last_fired");
        check(abnn_set_last_visited(h_, 0, z.data(), z.size()), "abnn_set_last_visited");
        abnn_scalars s{0, 0.0f, 0.0f};
        check(abnn_set_scalars(h_, &s), "abnn_set_scalars");
    }

    // One C1 pass: traversal + clock tick + renormalisation when due
    // (brain.cpp:87-141).  Enqueued on `stream` (a hipStream_t, NULL =
    // default); synchronize() is the reference's waitUntilCompleted.
    void encode_traversal(void* stream = nullptr, uint32_t passes = 1)
    {
        check(abnn_traverse(h_, passes, stream), "abnn_traverse");
    }
    void synchronize(void* stream = nullptr) { check(abnn_synchronize(h_, stream), "abnn_synchronize"); }

    void inject_inputs(const std::vector<float>& vals, float hz)  // brain.cpp:73-83
    {
        check(abnn_inject_inputs(h_, vals.data(), (uint32_t)vals.size(), hz), "abnn_inject_inputs");
    }
    std::vector<bool> read_outputs() const  // brain.cpp:145-157
    {
        std::vector<uint8_t> o(n_output());
        check(abnn_read_outputs(h_, o.data(), (uint32_t)o.size()), "abnn_read_outputs");
        return std::vector<bool>(o.begin(), o.end());
    }

    // .bnn persistence, byte-compatible with brain.cpp:161-178.
    void save(std::ostream& os) const
    {
        const uint32_t hdr[2] = {n_syn(), n_neuron()};
        os.write(reinterpret_cast<const char*>(hdr), sizeof(hdr));
        std::vector<SynapsePacked> buf;
        for (uint64_t i = 0; i < n_syn(); i += kPiece) {
            const uint64_t n = std::min<uint64_t>(kPiece, n_syn() - i);
            buf.resize(n);
            check(abnn_download_synapses(h_, i, buf.data(), n), "abnn_download_synapses");
            os.write(reinterpret_cast<const char*>(buf.data()), (std::streamsize)(n * sizeof(SynapsePacked)));
        }
    }
    void load(std::istream& is)
    {
        uint32_t s = 0, n = 0;
        is.read(reinterpret_cast<char*>(&s), 4);
        is.read(reinterpret_cast<char*>(&n), 4);
        if (!(s == n_syn() && n == n_neuron())) throw size_mismatch(".bnn header does not match");
        std::vector<SynapsePacked> buf;
        for (uint64_t i = 0; i < n_syn(); i += kPiece) {
            const uint64_t k = std::min<uint64_t>(kPiece, n_syn() - i);
            buf.resize(k);
            is.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)(k * sizeof(SynapsePacked)));
            if (!is) throw std::runtime_error("short .bnn body");
            check(abnn_upload_synapses(h_, i, buf.data(), k), "abnn_upload_synapses");
        }
    }

    uint32_t n_input() const { return dims().n_input; }
    uint32_t n_output() const { return dims().n_output; }
    uint32_t n_hidden() const { return (uint32_t)dims().n_hidden; }
    uint32_t n_neuron() const { return (uint32_t)abnn_n_neuron(h_); }
    uint32_t n_syn() const { return (uint32_t)dims().n_syn; }

    // Borrowed device pointers (brain.h:54-58).  The reference's budget buffer
    // has no equivalent: the budget is the max_spikes parameter.
    // bufSyn_ as device arrays (abnn.h abnn_state: src in two streams);
    // SynapsePacked is the upload/download/.bnn format.
    struct SynapseArrays {
        uint16_t* src_lo;
        uint8_t* src_hi;
        abnn_dst_w* dst_w;  // {dst, w} of each record
    };
    SynapseArrays synapse_buffer() const
    {
        const abnn_state s = state();
        return {s.syn_src_lo, s.syn_src_hi, s.syn_dst_w};
    }
    uint64_t* last_fired_buffer() const { return state().last_fired; }
    uint64_t* clock_buffer() const { return state().clock; }
    float* reward_buffer() const { return state().reward; }

    // Additions used by the engine-side driver.
    void build_random_graph(uint64_t seed = 1)  // brain-engine.cpp:31-53 recipe
    {
        check(abnn_generate_synapses(h_, seed), "abnn_generate_synapses");
    }
    void set_auto_stimulus(uint64_t first, uint64_t count)
    {
        check(abnn_set_auto_stimulus(h_, first, count), "abnn_set_auto_stimulus");
    }
    void set_reward(float r) { check(abnn_set_reward(h_, r), "abnn_set_reward"); }
    void set_timestamps(const std::vector<uint32_t>& idx, uint64_t value)
    {
        check(abnn_set_timestamps(h_, idx.data(), idx.size(), value), "abnn_set_timestamps");
    }
    abnn_scalars scalars() const
    {
        abnn_scalars s{};
        check(abnn_get_scalars(h_, &s), "abnn_get_scalars");
        return s;
    }
    std::vector<uint64_t> last_fired() const { return last_fired(0, n_neuron()); }
    std::vector<uint64_t> last_fired(uint64_t first, uint64_t n) const
    {
        std::vector<uint64_t> v(n);
        check(abnn_get_last_fired(h_, first, v.data(), n), "abnn_get_last_fired");
        return v;
    }
    uint64_t checksum() const
    {
        uint64_t c = 0;
        check(abnn_checksum_synapses(h_, &c), "abnn_checksum_synapses");
        return c;
    }
    abnn_brain* handle() const { return h_; }

private:
    static constexpr uint64_t kPiece = 1u << 20;
    abnn_dims dims() const
    {
        abnn_dims d{};
        abnn_get_dims(h_, &d);
        return d;
    }
    abnn_state state() const
    {
        abnn_state s{};
        abnn_state_ptrs(h_, &s);
        return s;
    }
    abnn_brain* h_ = nullptr;
};

}  // namespace abnn
