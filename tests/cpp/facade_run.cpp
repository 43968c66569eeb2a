// Exercises include/bloomhip_bloom_filter.hpp the way the reference's Run
// uses BloomFilter (src/run.cpp:15, :93, :162): construct from
// max_size * bf_bits_per_entry (long * float), set() every entry of a run,
// is_set() per GET.  Prints the bitmap popcount, the hit count and a
// checksum so tests/test_facade.py can compare against the oracle.
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <vector>

#include "bloomhip_bloom_filter.hpp"

int main(int argc, char **argv) {
    const long max_size = argc > 1 ? atol(argv[1]) : 512;
    const float bpe = argc > 2 ? (float)atof(argv[2]) : 0.5f;
    try {
        BloomFilter bloom_filter(max_size * bpe);  // as Run::Run, src/run.cpp:15
        for (long i = 0; i < max_size; i++) bloom_filter.set((int32_t)(i * 2654435761u));
        long hits = 0;
        for (long i = 0; i < 2 * max_size; i++) hits += bloom_filter.is_set((int32_t)(i * 2654435761u));
        // batch surface on the same filter
        std::vector<int32_t> probe(2 * max_size);
        for (long i = 0; i < 2 * max_size; i++) probe[i] = (int32_t)(i * 2654435761u);
        std::vector<uint64_t> packed((probe.size() + 63) / 64);
        bloom_filter.is_set_batch(probe.data(), probe.size(), packed.data());
        long bhits = 0;
        for (uint64_t w : packed) bhits += __builtin_popcountll(w);
        BloomFilter copy = bloom_filter;  // deep copy (Run is copied into its level deque)
        std::vector<uint64_t> w = copy.words();
        long pop = 0;
        uint64_t sum = 0;
        for (size_t i = 0; i < w.size(); i++) {
            pop += __builtin_popcountll(w[i]);
            sum = sum * 1099511628211ull + w[i];
        }
        printf("m=%llu pop=%ld hits=%ld batch_hits=%ld sum=%llu\n",
               (unsigned long long)copy.size(), pop, hits, bhits, (unsigned long long)sum);
    } catch (const std::exception &e) {
        printf("error: %s\n", e.what());
        return 3;
    }
    return 0;
}
