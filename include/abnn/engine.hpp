// engine.hpp -- the reference's per-pass learning driver over abnn::Brain.
//
// BrainEngine::run_one_pass (abnn/src/core/brain-engine.cpp:108-190) with its
// collaborators: the rate filter (core/output-filter/rate-filter.h:7-68), the
// sinusoid stimulus (stimulus/functional-dataset.cpp:6-52) and the engine
// constants (core/constants.h:7-14, brain-engine.h:54,81-84).  One pass:
//
//   input / expected frame  -> Brain::inject_inputs           (ENG:114-117)
//   Poisson teacher spikes on every other pass                (ENG:119-134)
//   traversal (the GPU pass) and the output spikes            (ENG:136-143)
//   rate EWMA -> RateFilter -> peak-normalised rates          (ENG:145-164)
//   every win_size passes: MSE(rates, expected) -> reward = previous loss - loss
//                                                             (ENG:170-186)
//
// Host code, as in the reference: per pass it moves 256 + 256 timestamps and
// a few KB of floats.  Differences, all deliberate:
//   * the teacher-forcing RNG is seeded (EngineConfig::teacher_seed, SplitMix64,
//     24-bit uniforms) instead of random_device-seeded (ENG:120);
//   * the rate / window state is per engine, not function-static (ENG:126,145);
//   * the logger (ENG:166-168, logger.cpp) is out of scope.
// The arithmetic keeps the reference's types and order (float EWMA, double
// filter coefficient, double loss), so a run is reproducible bit for bit and
// BrainEngine<OracleBrain> over the CPU oracle matches BrainEngine<Brain>
// (tests/cpp/engine_test.cpp).
#pragma once

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <fstream>
#include <functional>
#include <memory>
#include <string>
#include <thread>
#include <vector>

namespace abnn {

struct EngineConfig {
    float input_rate_hz = 1000.0f;  // INPUT_RATE_HZ, constants.h:9
    float peak_decay = 0.999f;      // PEAK_DECAY, constants.h:10
    double filter_tau = 0.02;       // FILTER_TAU, constants.h:12
    bool use_fir = true;            // USE_FIR, constants.h:13
    std::size_t fir_size = 20;      // RateFilter default window, rate-filter.h:14
    double dt_sec = 0.0009;         // dT_SEC, constants.h:14
    float rate_alpha = 0.5f;        // EWMA of the output spikes, ENG:146
    float max_observed = 0.5f;      // initial peak, brain-engine.h:54
    std::size_t win_size = 1000;    // WIN_SIZE_, brain-engine.h:81
    double last_loss = 0.25;        // graded-reward baseline, brain-engine.h:83
    uint64_t teacher_seed = 1;
};

// Continuous-time low-pass filter with an optional trailing moving average
// (rate-filter.h:7-68): r += float(a * (raw - r)), a = dt / (tau + dt) in
// double; the FIR output is the float mean of the last fir_size filtered
// frames, summed oldest first.
class RateFilter {
public:
    explicit RateFilter(double tau_sec, bool use_fir = true, std::size_t fir_size = 20)
        : tau_(tau_sec), fir_(use_fir), fir_size_(fir_size) {}

    std::vector<float> process(const std::vector<float>& raw, double dt_sec)
    {
        if (state_.empty()) state_ = raw;  // first frame initialises the state
        const double a = dt_sec / (tau_ + dt_sec);
        for (std::size_t i = 0; i < raw.size(); ++i) state_[i] += float(a * (raw[i] - state_[i]));
        if (!fir_) return state_;
        if (hist_.size() < fir_size_) {
            hist_.push_back(state_);
        } else {  // ring: overwrite the oldest frame
            hist_[head_] = state_;
            head_ = (head_ + 1) % fir_size_;
        }
        std::vector<float> mean(raw.size(), 0.0f);
        const std::size_t n = hist_.size();
        for (std::size_t f = 0; f < n; ++f) {
            const std::vector<float>& frame = hist_[(head_ + f) % n];  // oldest first
            for (std::size_t i = 0; i < mean.size(); ++i) mean[i] += frame[i];
        }
        const float inv = 1.0f / float(n);
        for (float& v : mean) v *= inv;
        return mean;
    }

private:
    double tau_;
    bool fir_;
    std::size_t fir_size_;
    std::vector<float> state_;
    std::vector<std::vector<float>> hist_;
    std::size_t head_ = 0;  // index of the oldest frame once the ring is full
};

// stimulus/stimulus-provider.h: one input and one expected frame per pass.
class StimulusProvider {
public:
    virtual ~StimulusProvider() = default;
    virtual std::vector<float> nextInput() = 0;
    virtual std::vector<float> nextExpected() = 0;
    virtual double time() const = 0;
};

// Phase-shifted functions of 2*pi*(i/n + phase), the phase advancing by
// freq * dt per input frame (functional-dataset.cpp:24-52).  The input
// argument is rounded to float before the call; the expected argument is
// computed in double and converted by the float(float) function type, as in
// the reference.
class FunctionalDataset : public StimulusProvider {
public:
    FunctionalDataset(uint32_t n_input, uint32_t n_output, double dt_sec, double freq_hz,
                      std::function<float(float)> f_input, std::function<float(float)> f_expected)
        : n_in_(n_input), n_out_(n_output), dt_(dt_sec), f_hz_(freq_hz),
          f_in_(std::move(f_input)), f_exp_(std::move(f_expected)) {}

    std::vector<float> nextInput() override
    {
        phase_ += f_hz_ * dt_;
        if (phase_ > 1.0) phase_ -= 1.0;
        t_ += dt_;
        std::vector<float> v(n_in_);
        for (uint32_t i = 0; i < n_in_; ++i) {
            const double x = static_cast<double>(i) / n_in_;
            v[i] = f_in_(static_cast<float>(kTwoPi * (x + phase_)));
        }
        return v;
    }
    std::vector<float> nextExpected() override
    {
        std::vector<float> v(n_out_);
        for (uint32_t i = 0; i < n_out_; ++i) {
            const double x = static_cast<double>(i) / n_out_;
            v[i] = f_exp_(static_cast<float>(kTwoPi * (x + phase_)));
        }
        return v;
    }
    double time() const override { return t_; }

    // The functions the app wires in (view-delegate.cpp:32-42).
    static float cos_squared(float x) { return std::cos(x) * std::cos(x); }
    static float half_sine(float x) { return 0.5f * std::sin(x) + 0.5f; }

private:
    static constexpr double kTwoPi = 6.283185307179586;  // 2.0 * M_PI
    uint32_t n_in_, n_out_;
    double dt_, f_hz_;
    std::function<float(float)> f_in_, f_exp_;
    double phase_ = 0.0, t_ = 0.0;
};

// BrainT: abnn::Brain, or any type with the same pass-boundary surface
// (n_input, n_output, inject_inputs, scalars, last_fired(first, n),
// set_timestamps, encode_traversal, synchronize, read_outputs, set_reward,
// save, load) -- the CPU oracle adapter in tests/cpp is one.
template <class BrainT>
class BrainEngine {
public:
    explicit BrainEngine(BrainT& brain, EngineConfig cfg = {})
        : brain_(brain), cfg_(cfg), n_in_(brain.n_input()), n_out_(brain.n_output()),
          rate_(n_out_, 0.0f), spike_window_(n_out_, 0u),
          filter_(cfg.filter_tau, cfg.use_fir, cfg.fir_size),
          max_observed_(cfg.max_observed), last_loss_(cfg.last_loss), rng_(cfg.teacher_seed)
    {
    }
    ~BrainEngine() { stop_async(); }
    BrainEngine(const BrainEngine&) = delete;
    BrainEngine& operator=(const BrainEngine&) = delete;

    void set_stimulus(std::shared_ptr<StimulusProvider> s) { stim_ = std::move(s); }

    // One synchronous pass (ENG:108-190); returns the output spikes.
    std::vector<bool> run_one_pass()
    {
        if (!stim_) return {};
        const std::vector<float> in = stim_->nextInput();
        const std::vector<float> expected = stim_->nextExpected();
        brain_.inject_inputs(in, cfg_.input_rate_hz);

        // Poisson teacher forcing on every other pass (ENG:119-134): output o
        // is stamped with p = expected[o] unless it fired within the last tick.
        const uint64_t now = brain_.scalars().clock;
        const float teacher_rate = teach_ ? 1.0f : 0.0f;
        const std::vector<uint64_t> lf = brain_.last_fired(n_in_, n_out_);
        std::vector<uint32_t> teach;
        for (uint32_t o = 0; o < n_out_; ++o) {
            const float p = expected[o] * teacher_rate;
            const float u = uni();  // drawn for every output, as in the reference
            if (u < p && (uint32_t)now - (uint32_t)lf[o] > 1u) teach.push_back(n_in_ + o);  // u32 ages (ENG:123-130)
        }
        if (!teach.empty()) brain_.set_timestamps(teach, now);
        teach_ = !teach_;

        brain_.encode_traversal();
        brain_.synchronize();
        const std::vector<bool> out = brain_.read_outputs();

        const float a = cfg_.rate_alpha;
        for (uint32_t i = 0; i < n_out_; ++i) rate_[i] = (1 - a) * rate_[i] + a * (out[i] ? 1.f : 0.f);
        std::vector<float> smooth = filter_.process(rate_, cfg_.dt_sec);
        for (float r : smooth) max_observed_ = std::max(max_observed_, r);
        max_observed_ *= cfg_.peak_decay;  // slowly forget old peaks
        for (float& r : smooth) r = std::min(r / max_observed_, 1.0f);
        ++step_;

        for (uint32_t i = 0; i < n_out_; ++i) spike_window_[i] += out[i] ? 1u : 0u;
        if (++win_pos_ == cfg_.win_size) {
            double loss = 0.0;
            for (uint32_t i = 0; i < n_out_; ++i) {
                const double err = smooth[i] - expected[i];
                loss += err * err;
            }
            loss /= n_out_;
            last_reward_ = float(last_loss_ - loss);
            brain_.set_reward(last_reward_);
            last_loss_ = loss;
            win_pos_ = 0;
            ++windows_;
        }
        smooth_ = std::move(smooth);
        return out;
    }

    // Background loop on one worker thread (ENG:193-209).
    void start_async()
    {
        if (running_.load() || !stim_) return;
        running_.store(true);
        worker_ = std::thread([this] {
            while (running_.load()) run_one_pass();
        });
    }
    void stop_async()
    {
        if (!running_.load()) return;
        running_.store(false);
        if (worker_.joinable()) worker_.join();
    }

    // Model persistence in the reference's .bnn format (ENG:85-102).
    bool load_model(const std::string& path)
    {
        std::ifstream is(path, std::ios::binary);
        if (!is) return false;
        try {
            brain_.load(is);
        } catch (const std::exception&) {
            return false;
        }
        return true;
    }
    bool save_model(const std::string& path) const
    {
        std::ofstream os(path, std::ios::binary);
        if (!os) return false;
        brain_.save(os);
        return static_cast<bool>(os);
    }

    double last_loss() const { return last_loss_; }
    float last_reward() const { return last_reward_; }
    float max_observed() const { return max_observed_; }
    uint64_t step() const { return step_; }
    uint64_t windows() const { return windows_; }
    const std::vector<float>& rates() const { return rate_; }
    const std::vector<float>& smooth_rates() const { return smooth_; }
    const std::vector<uint32_t>& spike_window() const { return spike_window_; }

private:
    float uni()  // SplitMix64 -> 24-bit uniform in [0, 1)
    {
        uint64_t z = (rng_ += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        return (float)(z >> 40) * (1.0f / 16777216.0f);
    }

    BrainT& brain_;
    EngineConfig cfg_;
    uint32_t n_in_, n_out_;
    std::shared_ptr<StimulusProvider> stim_;
    std::vector<float> rate_, smooth_;
    std::vector<uint32_t> spike_window_;
    RateFilter filter_;
    float max_observed_;
    double last_loss_;
    float last_reward_ = 0.0f;
    uint64_t rng_;
    bool teach_ = false;  // the reference's `even`, false on the first pass
    std::size_t win_pos_ = 0;
    uint64_t step_ = 0, windows_ = 0;
    std::thread worker_;
    std::atomic<bool> running_{false};
};

}  // namespace abnn
