// The reference's only filter-dependent golden test, test/test-6 (params
// `-b 1`, out line 2 `1535`), replayed through include/bloomhip_bloom_filter.hpp
// the way LSMTree drives it: `-b 1` gives a 512-entry buffer
// (src/main.cpp:89), so the 1537 puts flush three runs of capacity 512 at the
// default 0.5 bits/entry (src/lsm_tree.cpp:124-129), each filter
// BloomFilter(512 * 0.5f) = 256 bits (src/run.cpp:15), set() once per entry
// (src/run.cpp:162).  `g 1535` reaches the newest run and needs is_set(1535)
// (src/run.cpp:93).  Keys come from stdin as "run key" lines; prints each
// run's bitmap words and the newest run's is_set answers for argv keys.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <stdexcept>
#include <vector>

#include "bloomhip_bloom_filter.hpp"

int main(int argc, char **argv) {
    const long max_size = 512;
    const float bf = 0.5f;
    try {
        std::deque<BloomFilter> runs;  // newest first, as Level::runs
        long cur = -1, r = 0, k = 0;
        while (scanf("%ld %ld", &r, &k) == 2) {
            if (r != cur) {
                runs.emplace_front(max_size * bf);
                cur = r;
            }
            runs.front().set((int32_t)k);
        }
        for (size_t i = 0; i < runs.size(); i++) {
            std::vector<uint64_t> w = runs[i].words();
            printf("run%zu m=%llu", i, (unsigned long long)runs[i].size());
            for (uint64_t x : w) printf(" %016llx", (unsigned long long)x);
            printf("\n");
        }
        for (int a = 1; a < argc; a++) {
            const int32_t key = (int32_t)atol(argv[a]);
            printf("is_set %d %d\n", key, runs.empty() ? 0 : (int)runs.front().is_set(key));
        }
    } catch (const std::exception &e) {
        printf("error: %s\n", e.what());
        return 3;
    }
    return 0;
}
