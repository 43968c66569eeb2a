// workload.cpp — host restatement of the CS265 workload generator's key
// streams (jackdent/cs265-lsm-tree generator/generator.c), so the benchmark
// feeds the filter exactly the keys the configs name.  See
// include/bloomhip_workload.h for the RNG provenance.
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/bloomhip.h"
#include "../../include/bloomhip_workload.h"

namespace {

// MT19937 with GSL's seeding (gsl_rng_mt19937: seed 0 -> 4357), identical
// to std::mt19937's init_genrand.
class Mt19937 {
   public:
    explicit Mt19937(uint32_t seed) {
        if (seed == 0) seed = 4357;
        mt_[0] = seed;
        for (int i = 1; i < 624; i++)
            mt_[i] = 1812433253u * (mt_[i - 1] ^ (mt_[i - 1] >> 30)) + (uint32_t)i;
        idx_ = 624;
    }
    uint32_t next() {
        if (idx_ >= 624) twist();
        uint32_t y = mt_[idx_++];
        y ^= y >> 11;
        y ^= (y << 7) & 0x9d2c5680u;
        y ^= (y << 15) & 0xefc60000u;
        y ^= y >> 18;
        return y;
    }

   private:
    void twist() {
        for (int i = 0; i < 624; i++) {
            const uint32_t y = (mt_[i] & 0x80000000u) | (mt_[(i + 1) % 624] & 0x7fffffffu);
            mt_[i] = mt_[(i + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        idx_ = 0;
    }
    uint32_t mt_[624];
    int idx_;
};

// glibc random()/rand(): the TYPE_3 additive feedback generator
// r[i] = r[i-3] + r[i-31] (mod 2^32), output r >> 1, seeded through the
// 16807 Lehmer sequence and warmed up by 310 draws.
class GlibcRand {
   public:
    explicit GlibcRand(uint32_t seed) {
        int32_t word = (int32_t)(seed == 0 ? 1u : seed);
        r_[0] = (uint32_t)word;
        for (int i = 1; i < 31; i++) {
            const int64_t hi = word / 127773, lo = word % 127773;
            int64_t w = 16807 * lo - 2836 * hi;
            if (w < 0) w += 2147483647;
            word = (int32_t)w;
            r_[i] = (uint32_t)word;
        }
        f_ = 3;
        b_ = 0;
        for (int i = 0; i < 310; i++) next();
    }
    int32_t next() {
        r_[f_] += r_[b_];
        const int32_t out = (int32_t)(r_[f_] >> 1);
        f_ = (f_ + 1) % 31;
        b_ = (b_ + 1) % 31;
        return out;
    }

   private:
    uint32_t r_[31];
    int f_, b_;
};

}  // namespace

extern "C" {

int bloomhip_gen_mt19937(uint32_t seed, size_t n, uint32_t *out) {
    if (n && !out) return BLOOMHIP_EINVAL;
    Mt19937 mt(seed);
    for (size_t i = 0; i < n; i++) out[i] = mt.next();
    return BLOOMHIP_OK;
}

int bloomhip_gen_glibc_rand(uint32_t seed, size_t n, int32_t *out) {
    if (n && !out) return BLOOMHIP_EINVAL;
    GlibcRand r(seed);
    for (size_t i = 0; i < n; i++) out[i] = r.next();
    return BLOOMHIP_OK;
}

int bloomhip_gen_puts(uint32_t seed, size_t n_puts, int32_t *keys_out, int32_t *vals_out) {
    if (n_puts && !keys_out) return BLOOMHIP_EINVAL;
    Mt19937 mt(seed);
    for (size_t i = 0; i < n_puts; i++) {
        keys_out[i] = (int32_t)mt.next();  // KEY_t k = gsl_rng_get(r)   generator.c:353
        const int32_t v = (int32_t)mt.next();  // VAL_t v = gsl_rng_get(r) generator.c:354
        if (vals_out) vals_out[i] = v;
    }
    return BLOOMHIP_OK;
}

int bloomhip_gen_workload(uint32_t seed, size_t n_puts, size_t n_gets, float gets_skewness,
                          float gets_misses_ratio, int32_t *put_keys_out, int32_t *get_keys_out) {
    if ((n_puts && !put_keys_out) || (n_gets && !get_keys_out)) return BLOOMHIP_EINVAL;
    if (n_puts == 0) return BLOOMHIP_EINVAL;  // generator.c: "0 puts not allowed"
    if (n_puts > 0x7fffffff || n_gets > 0x7fffffff) return BLOOMHIP_ERANGE;
    Mt19937 mt(seed);
    GlibcRand crand(1);  // rand() is never seeded by the generator
    // Pool sizes as generator.c:270-292 computes them (a count times
    // sizeof(KEY_t), capped at 10M * sizeof(KEY_t)).
    const size_t puts_cap = (n_puts < 10000000 ? n_puts : 10000000) * sizeof(int32_t);
    const size_t gets_cap = (n_gets < 10000000 ? n_gets : 10000000) * sizeof(int32_t);
    std::vector<int32_t> puts_pool, gets_pool;
    puts_pool.reserve(n_puts < puts_cap ? n_puts : puts_cap);
    gets_pool.reserve(n_gets < gets_cap ? n_gets : gets_cap);
    // `s->gets_skewness*10` and `s->gets_misses_ratio*10` are float products
    // compared against an int (generator.c:384,388).
    const float skew10 = gets_skewness * 10;
    const float miss10 = gets_misses_ratio * 10;
    size_t cp = 0, cg = 0;
    while (cp < n_puts || cg < n_gets) {
        const int op = crand.next() % 4;  // generator.c:310
        if (op == 0) {  // PUT, generator.c:350-375
            if (cp >= n_puts) continue;
            const int32_t k = (int32_t)mt.next();
            (void)mt.next();  // value
            put_keys_out[cp] = k;
            if (puts_pool.size() >= puts_cap)
                puts_pool[(size_t)(crand.next() % (int32_t)puts_pool.size())] = k;
            else
                puts_pool.push_back(k);
            cp++;
        } else if (op == 1) {  // GET, generator.c:376-414
            if (cg >= n_gets) continue;
            if (cp == 0) continue;
            int32_t k;
            if ((float)(crand.next() % 10) > skew10 || gets_pool.empty()) {
                if ((float)(crand.next() % 10) > miss10)
                    k = puts_pool[(size_t)(crand.next() % (int32_t)puts_pool.size())];
                else
                    k = (int32_t)mt.next();
                if (gets_pool.size() >= gets_cap)
                    gets_pool[(size_t)(crand.next() % (int32_t)gets_pool.size())] = k;
                else
                    gets_pool.push_back(k);
            } else {
                k = gets_pool[(size_t)(crand.next() % (int32_t)gets_pool.size())];
            }
            get_keys_out[cg++] = k;
        }
        // RANGE / DELETE: none requested; the loop re-draws (generator.c:314-323)
    }
    return BLOOMHIP_OK;
}

}  // extern "C"
