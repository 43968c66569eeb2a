/*
 * bloomhip_workload.h — host C++ restatement of the CS265 workload
 * generator's key streams (jackdent/cs265-lsm-tree generator/generator.c),
 * used to produce the exact key vectors the benchmark configs name.
 *
 * The generator draws keys with GSL's gsl_rng_mt19937 (seeded with
 * gsl_rng_default_seed = --seed, generator.c:258-263; keys are
 * (int32_t) gsl_rng_get, data_types.h:26) and picks operations and pool
 * entries with glibc rand() from its default (unseeded) state
 * (generator.c:310,358-367,384-407).  GSL is absent from this image: the
 * MT19937 here follows GSL's documented seeding (seed 0 -> 4357), which
 * equals std::mt19937; glibc's rand() is restated as its TYPE_3 additive
 * feedback generator.  Both are checked against independent
 * implementations in tests/test_workload.py.
 */
#ifndef BLOOMHIP_WORKLOAD_H
#define BLOOMHIP_WORKLOAD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Raw MT19937 outputs (GSL seeding) — n values. */
int bloomhip_gen_mt19937(uint32_t seed, size_t n, uint32_t *out);
/* glibc rand() outputs after srand(seed) (seed 1 = the unseeded state). */
int bloomhip_gen_glibc_rand(uint32_t seed, size_t n, int32_t *out);

/* `generator --puts n --seed s` (no gets): the PUT keys in stream order.
 * Each PUT draws its key then its value (generator.c:353-354), so keys are
 * the MT outputs at even indices.  vals_out may be NULL. */
int bloomhip_gen_puts(uint32_t seed, size_t n_puts, int32_t *keys_out, int32_t *vals_out);

/* `generator --puts P --gets G --gets-skewness S --gets-misses-ratio R
 * --seed s` restricted to PUT and GET operations (generator.c:300-414):
 * writes the P put keys and the G get keys, each in stream order. */
int bloomhip_gen_workload(uint32_t seed, size_t n_puts, size_t n_gets, float gets_skewness,
                          float gets_misses_ratio, int32_t *put_keys_out, int32_t *get_keys_out);

#ifdef __cplusplus
}
#endif

#endif /* BLOOMHIP_WORKLOAD_H */
