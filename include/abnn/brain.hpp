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
//   synapse_buffer() ... budget_buffer()  (MTL::Buffer-like views) brain.h:54-58
// Errors throw std::runtime_error (the reference threw a pointer,
// brain.cpp:174); a .bnn size mismatch throws abnn::size_mismatch.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <istream>
#include <memory>
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

// NS::Range(location, length) of the reference's didModifyRange calls (ENG:52,181).
struct Range {
    uint64_t location, length;
    Range(uint64_t loc, uint64_t len) : location(loc), length(len) {}
};

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
        touch();
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
        touch();
        check(abnn_traverse(h_, passes, stream), "abnn_traverse");
    }
    void synchronize(void* stream = nullptr) { check(abnn_synchronize(h_, stream), "abnn_synchronize"); }

    void inject_inputs(const std::vector<float>& vals, float hz)  // brain.cpp:73-83
    {
        touch();
        check(abnn_inject_inputs(h_, vals.data(), (uint32_t)vals.size(), hz), "abnn_inject_inputs");
    }
    std::vector<bool> read_outputs() const  // brain.cpp:145-157
    {
        flush_shared();
        std::vector<uint8_t> o(n_output());
        check(abnn_read_outputs(h_, o.data(), (uint32_t)o.size()), "abnn_read_outputs");
        return std::vector<bool>(o.begin(), o.end());
    }

    // .bnn persistence, byte-compatible with brain.cpp:161-178.
    void save(std::ostream& os) const
    {
        flush_shared();
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
        touch();
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

    // The buffer getters (brain.h:54-58): host views standing in for the
    // MTL::Buffer objects, so the reference's callers keep their code:
    //   auto* syn = (SynapsePacked*)b.synapse_buffer()->contents();   ENG:37
    //   ... syn[idx++] = {...};  b.synapse_buffer()->didModifyRange(Range(0, n*16));  ENG:52
    //   uint32_t* lf = (uint32_t*)b.last_fired_buffer()->contents();  ENG:123
    //   uint32_t now = *(uint32_t*)b.clock_buffer()->contents();      ENG:124
    //   lf[nIn + o] = now;                                            ENG:131
    //   float* r = (float*)b.reward_buffer()->contents(); *r = x; didModifyRange   ENG:180-182
    // contents() is a host copy, downloaded when the device state changed
    // since it was taken.  Managed buffers (synapses, reward, budget;
    // brain.cpp:54,58-59) send host writes with didModifyRange.  Shared ones
    // (lastFired, clock; brain.cpp:55-57) need no call: the writes are sent
    // before the next device operation of this Brain (encode_traversal, ...).
    // lastFired and the clock are presented as the reference's u32 (the low
    // 32 bits of the u64 state, on which every decision is taken).  The
    // budget view reads the budget left by the last pass (writing it is an
    // error: the reference's host resets it to kMaxSpikes every pass,
    // brain.cpp:90; the knob is abnn_params.max_spikes).
    class Buffer {
    public:
        void* contents()
        {
            if (!mapped_ || version_ != owner_->version_) refresh();
            return host_.data();
        }
        uint64_t length() const { return bytes(); }
        void didModifyRange(Range r)  // Managed: upload [location, location + length)
        {
            if (!mapped_) return;
            const uint64_t es = elem_bytes(), i0 = r.location / es, i1 = (r.location + r.length + es - 1) / es;
            upload(i0, std::min<uint64_t>(i1, count()));
        }

    private:
        friend class Brain;
        enum Kind { kSynapses, kLastFired, kClock, kReward, kBudget };
        Buffer(Brain* owner, Kind k) : owner_(owner), kind_(k) {}
        uint64_t count() const
        {
            switch (kind_) {
                case kSynapses: return owner_->n_syn();
                case kLastFired: return owner_->n_neuron();
                default: return 1;
            }
        }
        uint64_t elem_bytes() const { return kind_ == kSynapses ? sizeof(SynapsePacked) : 4; }
        uint64_t bytes() const { return count() * elem_bytes(); }
        bool shared() const { return kind_ == kLastFired || kind_ == kClock; }
        void refresh()
        {
            owner_->flush_shared();
            host_.assign(bytes(), 0);
            abnn_brain* h = owner_->h_;
            switch (kind_) {
                case kSynapses:
                    for (uint64_t i = 0; i < count(); i += kPiece)
                        check(abnn_download_synapses(h, i, reinterpret_cast<SynapsePacked*>(host_.data()) + i,
                                                     std::min<uint64_t>(kPiece, count() - i)),
                              "abnn_download_synapses");
                    break;
                case kLastFired: {
                    const std::vector<uint64_t> v = owner_->last_fired();
                    uint32_t* o = reinterpret_cast<uint32_t*>(host_.data());
                    for (uint64_t i = 0; i < v.size(); ++i) o[i] = (uint32_t)v[i];
                    break;
                }
                case kClock: {
                    const uint32_t c = (uint32_t)owner_->scalars().clock;
                    std::memcpy(host_.data(), &c, 4);
                    break;
                }
                case kReward: {
                    const float r = owner_->scalars().reward;
                    std::memcpy(host_.data(), &r, 4);
                    break;
                }
                case kBudget: {
                    uint32_t left = 0;
                    check(abnn_get_budget(h, &left), "abnn_get_budget");
                    std::memcpy(host_.data(), &left, 4);
                    break;
                }
            }
            pristine_ = host_;
            mapped_ = true;
            version_ = owner_->version_;
        }
        void upload(uint64_t i0, uint64_t i1)  // elements [i0, i1) host -> device
        {
            if (i1 <= i0) return;
            abnn_brain* h = owner_->h_;
            switch (kind_) {
                case kSynapses:
                    for (uint64_t i = i0; i < i1; i += kPiece)
                        check(abnn_upload_synapses(h, i, reinterpret_cast<const SynapsePacked*>(host_.data()) + i,
                                                   std::min<uint64_t>(kPiece, i1 - i)),
                              "abnn_upload_synapses");
                    break;
                case kLastFired: {  // changed entries, grouped by value (the teacher writes one value)
                    const uint32_t* v = reinterpret_cast<const uint32_t*>(host_.data());
                    const uint32_t* p = reinterpret_cast<const uint32_t*>(pristine_.data());
                    std::vector<std::pair<uint32_t, uint32_t>> ch;
                    for (uint64_t i = i0; i < i1; ++i)
                        if (v[i] != p[i]) ch.push_back({v[i], (uint32_t)i});
                    std::sort(ch.begin(), ch.end());
                    for (size_t a = 0; a < ch.size();) {
                        size_t e = a;
                        std::vector<uint32_t> idx;
                        while (e < ch.size() && ch[e].first == ch[a].first) idx.push_back(ch[e++].second);
                        check(abnn_set_timestamps(h, idx.data(), idx.size(), ch[a].first), "abnn_set_timestamps");
                        a = e;
                    }
                    break;
                }
                case kClock: {
                    abnn_scalars sc{};
                    check(abnn_get_scalars(h, &sc), "abnn_get_scalars");
                    uint32_t c;
                    std::memcpy(&c, host_.data(), 4);
                    sc.clock = c;
                    check(abnn_set_scalars(h, &sc), "abnn_set_scalars");
                    break;
                }
                case kReward: {
                    float r;
                    std::memcpy(&r, host_.data(), 4);
                    check(abnn_set_reward(h, r), "abnn_set_reward");
                    break;
                }
                case kBudget:
                    if (std::memcmp(host_.data(), pristine_.data(), 4) != 0)
                        throw std::logic_error("budget_buffer() is read-only: the budget resets to max_spikes every "
                                               "pass (brain.cpp:90)");
                    break;
            }
            std::copy(host_.begin() + i0 * elem_bytes(), host_.begin() + i1 * elem_bytes(),
                      pristine_.begin() + i0 * elem_bytes());
            ++owner_->version_;  // the device changed: other views refresh
            version_ = owner_->version_;
        }
        Brain* owner_;
        Kind kind_;
        bool mapped_ = false;
        uint64_t version_ = 0;
        std::vector<uint8_t> host_, pristine_;
    };

    Buffer* synapse_buffer() const { return view(Buffer::kSynapses); }
    Buffer* last_fired_buffer() const { return view(Buffer::kLastFired); }
    Buffer* clock_buffer() const { return view(Buffer::kClock); }
    Buffer* reward_buffer() const { return view(Buffer::kReward); }
    Buffer* budget_buffer() const { return view(Buffer::kBudget); }

    // Borrowed device pointers (abnn_state; the synapse records are opaque).
    abnn_state device_state() const { return state(); }

    // Additions used by the engine-side driver.
    void build_random_graph(uint64_t seed = 1)  // brain-engine.cpp:31-53 recipe
    {
        touch();
        check(abnn_generate_synapses(h_, seed), "abnn_generate_synapses");
    }
    void set_auto_stimulus(uint64_t first, uint64_t count)
    {
        check(abnn_set_auto_stimulus(h_, first, count), "abnn_set_auto_stimulus");
    }
    void set_reward(float r)
    {
        touch();
        check(abnn_set_reward(h_, r), "abnn_set_reward");
    }
    void set_timestamps(const std::vector<uint32_t>& idx, uint64_t value)
    {
        touch();
        check(abnn_set_timestamps(h_, idx.data(), idx.size(), value), "abnn_set_timestamps");
    }
    abnn_scalars scalars() const
    {
        flush_shared();
        abnn_scalars s{};
        check(abnn_get_scalars(h_, &s), "abnn_get_scalars");
        return s;
    }
    std::vector<uint64_t> last_fired() const { return last_fired(0, n_neuron()); }
    std::vector<uint64_t> last_fired(uint64_t first, uint64_t n) const
    {
        flush_shared();
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
    Buffer* view(int k) const
    {
        if (!views_[k]) views_[k].reset(new Buffer(const_cast<Brain*>(this), (Buffer::Kind)k));
        return views_[k].get();
    }
    // Host writes into the current Shared views (lastFired, clock) go to the
    // device before any other operation of this Brain (brain.cpp:55-57 are
    // StorageModeShared: the reference's host writes are seen by the next pass).
    // The dirty views are collected against the version seen on entry: an
    // upload bumps the version, so checking inside the loop would skip (and a
    // later contents() would overwrite) the second view's write.  After the
    // uploads every flushed view equals the device again.
    void flush_shared() const
    {
        Buffer* dirty[2];
        int n = 0;
        for (int k : {(int)Buffer::kLastFired, (int)Buffer::kClock}) {
            Buffer* v = views_[k].get();
            if (v && v->mapped_ && v->version_ == version_ && v->host_ != v->pristine_) dirty[n++] = v;
        }
        for (int i = 0; i < n; ++i) dirty[i]->upload(0, dirty[i]->count());
        for (int i = 0; i < n; ++i) dirty[i]->version_ = version_;
    }
    void touch() const  // before an operation that changes device state
    {
        flush_shared();
        ++version_;
    }
    abnn_brain* h_ = nullptr;
    mutable uint64_t version_ = 1;
    mutable std::unique_ptr<Buffer> views_[5];
};

}  // namespace abnn
