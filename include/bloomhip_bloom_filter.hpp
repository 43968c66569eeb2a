// bloomhip_bloom_filter.hpp — header-only C++ drop-in for the reference's
// `class BloomFilter` (jackdent/cs265-lsm-tree src/bloom_filter.h:6-15).
//
// With the reference's src/bloom_filter.h reduced to include/dropin/bloom_filter.h
//     #include <cstdint>
//     #include "types.h"
//     #include <bloomhip_bloom_filter.hpp>
// src/run.cpp compiles unchanged: Run::Run constructs it from
// `max_size * bf_bits_per_entry` (src/run.cpp:15), Run::put calls set()
// (src/run.cpp:162) and Run::get calls is_set() (src/run.cpp:93).
// tests/test_dropin.py compiles the reference's own src/*.cpp this way.
//
// set() is buffered on the host and flushed to the GPU as one batch (the
// reference calls it once per entry of a flush/compaction loop); is_set()
// flushes pending keys first, so results are exactly the reference's.  The
// batch methods are the fast path for batched callers.
#pragma once

// <algorithm> and <cstring>: src/run.cpp uses std::upper_bound (:97, :130,
// :137) and strdup (:22) without including them; boost/dynamic_bitset.hpp
// used to bring both in through src/bloom_filter.h.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "bloomhip.h"

namespace bloomhip_detail {
inline void check(int rc, const char *what) {
    if (rc != BLOOMHIP_OK)
        throw std::runtime_error(std::string(what) + ": " + bloomhip_strerror(rc) + " " +
                                 bloomhip_last_error());
}
inline int default_device() {
    static int dev = 0;  // one process per GPU: the process's device 0
    return dev;
}
}  // namespace bloomhip_detail

class BloomFilter {
   public:
    // BloomFilter(long length) : table(length) {}   src/bloom_filter.h:12
    BloomFilter(long length) { create((uint64_t)length); }

    BloomFilter(const BloomFilter &o) {
        o.flush();
        create(o.m_);
        std::vector<uint64_t> w = o.words();
        bloomhip_detail::check(bloomhip_upload(h_, w.data(), w.size(), nullptr), "bloomhip_upload");
    }
    BloomFilter(BloomFilter &&o) noexcept : h_(o.h_), m_(o.m_), pending_(std::move(o.pending_)) {
        o.h_ = nullptr;
    }
    BloomFilter &operator=(const BloomFilter &o) {
        if (this != &o) {
            BloomFilter tmp(o);
            *this = std::move(tmp);
        }
        return *this;
    }
    BloomFilter &operator=(BloomFilter &&o) noexcept {
        if (this != &o) {
            release();
            h_ = o.h_;
            m_ = o.m_;
            pending_ = std::move(o.pending_);
            o.h_ = nullptr;
        }
        return *this;
    }
    ~BloomFilter() { release(); }

    // void set(KEY_t)             src/bloom_filter.cpp:49-53
    void set(int32_t key) {
        pending_.push_back(key);
        if (pending_.size() >= kFlushKeys) flush();
    }

    // bool is_set(KEY_t) const    src/bloom_filter.cpp:55-59
    bool is_set(int32_t key) const {
        flush();
        int hit = 0;
        bloomhip_detail::check(bloomhip_is_set(h_, key, &hit), "bloomhip_is_set");
        return hit != 0;
    }

    // ---- batch surface -------------------------------------------------
    void set_batch(const int32_t *keys, size_t n, size_t stride_bytes = 4, bool on_device = false,
                   void *stream = nullptr) {
        flush();
        bloomhip_detail::check(
            bloomhip_set_batch(h_, keys, n, stride_bytes, on_device ? 1 : 0, stream),
            "bloomhip_set_batch");
    }
    // packed: ceil(n/64) words, bit i%64 of word i/64 = is_set(keys[i]).
    void is_set_batch(const int32_t *keys, size_t n, uint64_t *packed, size_t stride_bytes = 4,
                      bool on_device = false, void *stream = nullptr) const {
        flush();
        const bloomhip_filter *f = h_;
        bloomhip_detail::check(bloomhip_test_batch(&f, 1, keys, n, stride_bytes, on_device ? 1 : 0,
                                                   packed, on_device ? 1 : 0, stream),
                               "bloomhip_test_batch");
    }
    // The bitmap in the reference's dynamic_bitset block layout.
    std::vector<uint64_t> words() const {
        flush();
        uint64_t nw = 0;
        bloomhip_detail::check(bloomhip_nwords(h_, &nw), "bloomhip_nwords");
        std::vector<uint64_t> w(nw);
        bloomhip_detail::check(bloomhip_download(h_, w.data(), w.size(), nullptr),
                               "bloomhip_download");
        return w;
    }
    uint64_t size() const { return m_; }
    bloomhip_filter *handle() const {
        flush();
        return h_;
    }

   private:
    static constexpr size_t kFlushKeys = 1u << 20;

    void create(uint64_t m) {
        m_ = m;
        bloomhip_detail::check(bloomhip_create(bloomhip_detail::default_device(), m, &h_),
                               "bloomhip_create");
    }
    void release() {
        if (h_) {
            bloomhip_destroy(h_);
            h_ = nullptr;
        }
    }
    void flush() const {
        std::lock_guard<std::mutex> lk(mu_);
        if (pending_.empty()) return;
        bloomhip_detail::check(
            bloomhip_set_batch(h_, pending_.data(), pending_.size(), sizeof(int32_t), 0, nullptr),
            "bloomhip_set_batch");
        pending_.clear();
    }

    bloomhip_filter *h_ = nullptr;
    uint64_t m_ = 0;
    mutable std::vector<int32_t> pending_;
    mutable std::mutex mu_;
};
