// gossip_protocol_amd/csrc/glibc_stream.hpp -- the reference's rand() stream, by draw index.
//
// The reference seeds glibc with srand(time(NULL)) (Application.cpp:50/96) and then
// draws rand() once per EmulNet::ENsend call (EmulNet.cpp:89) and once in
// Application::fail (Application.cpp:182/189).  glibc's default generator is TYPE_3
// random_r: an additive lagged-Fibonacci sequence s[i] = s[i-3] + s[i-31] (mod 2^32)
// whose first 31 words come from the minimal-standard LCG 16807 x mod (2^31 - 1); the
// first 310 sums are discarded and rand() returns s >> 1.  Materialising a window of
// the sequence makes "value of draw g" an index lookup, which is what lets the device
// send builder draw for a whole batch of messages in parallel.
#pragma once
#include <cstdint>
#include <vector>

namespace gsp {

class GlibcStream {
public:
    explicit GlibcStream(uint32_t seed = 1) { reseed(seed); }

    void reseed(uint32_t seed) {
        int64_t w = seed == 0 ? 1 : int32_t(seed);
        uint32_t init[34];
        init[0] = uint32_t(w);
        for (int i = 1; i < 31; ++i) {
            // Park-Miller step via Schrage's decomposition, signed as in glibc
            const int64_t prev = int32_t(init[i - 1]);
            w = 16807 * (prev % 127773) - 2836 * (prev / 127773);
            if (w < 0) w += 2147483647;
            init[i] = uint32_t(w);
        }
        for (int i = 31; i < 34; ++i) init[i] = init[i - 31];
        for (int i = 0; i < 34; ++i) lag_[i] = init[i];
        produced_ = 34;
        for (int i = 0; i < 310; ++i) next_word();
        base_ = 0;
        window_.clear();
    }

    // srand(seed) issued after g draws: draw g is the first value of seed's stream
    void reseed_at(uint32_t seed, int64_t g) {
        reseed(seed);
        base_ = g;
    }

    // rand() value of draw index g (g = 0 is the first rand() after srand); g >= base().
    int32_t at(int64_t g) {
        fill_to(g + 1);
        return window_[size_t(g - base_)];
    }
    // contiguous values of draws [g, g + n); g >= base()
    const int32_t *span(int64_t g, int64_t n) {
        fill_to(g + (n > 0 ? n : 1));
        return window_.data() + (g - base_);
    }
    // forget draws below g (they will never be asked for again)
    void trim(int64_t g) {
        if (g <= base_) return;
        const int64_t have = base_ + int64_t(window_.size());
        if (g >= have) {
            while (base_ + int64_t(window_.size()) < g) window_.push_back(int32_t(next_word() >> 1));
            window_.clear();
            base_ = g;
            return;
        }
        window_.erase(window_.begin(), window_.begin() + (g - base_));
        base_ = g;
    }
    int64_t base() const { return base_; }

private:
    void fill_to(int64_t end) {
        while (base_ + int64_t(window_.size()) < end) window_.push_back(int32_t(next_word() >> 1));
    }
    uint32_t next_word() {
        // lag_ holds the last 34 words; slot of word i is i % 34
        const uint32_t v = lag_[(produced_ - 31) % 34] + lag_[(produced_ - 3) % 34];
        lag_[produced_ % 34] = v;
        ++produced_;
        return v;
    }
    uint32_t lag_[34];
    uint64_t produced_ = 0;
    int64_t base_ = 0;
    std::vector<int32_t> window_;
};

}  // namespace gsp
