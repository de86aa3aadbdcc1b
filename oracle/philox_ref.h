/*
 * philox_ref.h -- ORACLE / TEST INFRASTRUCTURE ONLY.
 *
 * Per-pixel random stream used by the oracle.  The reference seeds cuRAND XORWOW
 * with clock64() (ACMMP.cu:684), so its random numbers are not reproducible by
 * construction.  The rebuild replaces that with a seeded counter-based stream:
 * Philox4x32-10 (Salmon et al., SC'11; the algorithm behind cuRAND's
 * curandStatePhilox4_32_10_t), keyed by the 64-bit run seed, with
 * subsequence = row-major pixel index and the draw counter as the block counter,
 * i.e. exactly what curand_init(seed, subsequence=pixel, offset=0, &philox)
 * followed by curand() would produce.  curand_uniform's (0,1] mapping
 * x*2^-32 + 2^-33 is kept.  Pinned by the Random123 known-answer vectors in
 * tests/test_oracle_rng.py.
 */
#ifndef ACMMP_ORACLE_PHILOX_REF_H
#define ACMMP_ORACLE_PHILOX_REF_H
#include <stdint.h>
#include <math.h>

static inline void or_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * (uint64_t)c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * (uint64_t)c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* One pixel's stream: draw n of subsequence `sub` under `seed`. */
typedef struct {
    uint32_t key[2];
    uint32_t sub_lo, sub_hi;
    uint32_t n;          /* draws consumed so far */
} or_rng;

static inline void or_rng_init(or_rng *s, uint64_t seed, uint64_t subsequence)
{
    s->key[0] = (uint32_t)seed;
    s->key[1] = (uint32_t)(seed >> 32);
    s->sub_lo = (uint32_t)subsequence;
    s->sub_hi = (uint32_t)(subsequence >> 32);
    s->n = 0;
}

static inline uint32_t or_rng_next_u32(or_rng *s)
{
    const uint32_t ctr[4] = { s->n >> 2, 0u, s->sub_lo, s->sub_hi };
    uint32_t out[4];
    or_philox4x32_10(ctr, s->key, out);
    const uint32_t v = out[s->n & 3u];
    s->n++;
    return v;
}

/* curand_uniform(): (0, 1] */
static inline float or_rng_uniform(or_rng *s)
{
    const uint32_t x = or_rng_next_u32(s);
    return fmaf((float)x, 2.3283064365386963e-10f, 1.1641532182693481e-10f);
}

#endif
