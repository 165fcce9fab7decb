// engine_host_test.cpp -- TEST PROGRAM (CPU only): RateFilter and
// FunctionalDataset of include/abnn/engine.hpp on fixed inputs; the output is
// compared with an independent numpy restatement in tests/test_engine.py.
#include <abnn/engine.hpp>

#include <cstdio>

int main()
{
    abnn::FunctionalDataset ds(8, 8, 0.0009, 0.5, abnn::FunctionalDataset::cos_squared,
                               abnn::FunctionalDataset::half_sine);
    abnn::RateFilter iir(0.02, false), fir(0.02, true, 5);
    std::printf("{\"frames\": [");
    for (int f = 0; f < 12; ++f) {
        const std::vector<float> in = ds.nextInput(), ex = ds.nextExpected();
        std::vector<float> raw(8);
        for (int i = 0; i < 8; ++i) raw[i] = ((f * 7 + i * 3) % 5) * 0.25f;
        const std::vector<float> a = iir.process(raw, 0.0009), b = fir.process(raw, 0.0009);
        std::printf("%s{\"in\": [", f ? ", " : "");
        for (int i = 0; i < 8; ++i) std::printf("%s%.9g", i ? ", " : "", in[i]);
        std::printf("], \"ex\": [");
        for (int i = 0; i < 8; ++i) std::printf("%s%.9g", i ? ", " : "", ex[i]);
        std::printf("], \"iir\": [");
        for (int i = 0; i < 8; ++i) std::printf("%s%.9g", i ? ", " : "", a[i]);
        std::printf("], \"fir\": [");
        for (int i = 0; i < 8; ++i) std::printf("%s%.9g", i ? ", " : "", b[i]);
        std::printf("]}");
    }
    std::printf("], \"time\": %.17g}\n", ds.time());
    return 0;
}
