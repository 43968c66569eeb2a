// bloom_math.h — the position arithmetic of the reference filter, written once
// for both the gfx950 kernels and the host self-test hook.
//
// Reference (jackdent/cs265-lsm-tree):
//   hash_1  src/bloom_filter.cpp:8-20    hash_2  :22-34    hash_3  :36-47
//   input  `uint64_t key; key = k;`  — the int32 key SIGN-EXTENDED to 64 bits
//   output `key % table.size()`      — full 64-bit unsigned remainder by m
//
// The remainder is the expensive part on a GPU (no integer divide).  For
// m < 2^32 (every filter up to 512 MiB) it is computed exactly with two
// multiplies and no division:
//   1. fold the high word:   y = xh * (2^32 mod m) + xl        (y ≡ x mod m, y < m * 2^32)
//   2. one 2-by-1 word division by the normalised divisor d = m << l using the
//      precomputed reciprocal v = floor((2^64-1)/d) - 2^32 (Möller & Granlund,
//      "Improved division by invariant integers", IEEE TC 2011, Alg. 4),
//      keeping only the remainder.
// For 2^32 <= m <= 2^46 (bloomhip_create's bound) mod_wide estimates the
// quotient in double precision and corrects it with one exact 64-bit
// multiply-subtract (see there); no integer division either.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bloomhip {

#define BH_HD __host__ __device__ __forceinline__

// ---- the three reference hashes, before the modulo --------------------------
// Each chain is the reference's, rewritten only where an identity on the
// sign-extended key saves gfx950 instructions (same value mod 2^64):
//   ~x + (x << 15)            == x * 32767 - 1        (one v_mad_i64_i32 on the
//   (x + c) + (x << 12)       == x * 4097 + c          int32 key)
//   x + (x << s)              == lshl_add(x, s, x)    (one v_lshl_add_u64; the
//   x * 2057                  == (x << 11) + lshl_add(x, 3, x)   (the compiler
//                                                          emits a 64-bit multiply)
// tests/test_host.py fuzzes the host build of these against the oracle.

// (a << S) + b in 64 bits.  v_lshl_add_u64 takes shifts 0..4 only (a larger
// immediate is silently truncated: it broke parity when this was tried with 11).
template <int S>
BH_HD uint64_t lshl_add64(uint64_t a, uint64_t b) {
    static_assert(S >= 0 && S <= 4, "v_lshl_add_u64 shifts by 0..4");
#if defined(__HIP_DEVICE_COMPILE__)
    uint64_t r;
    asm("v_lshl_add_u64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "i"(S), "v"(b));
    return r;
#else
    return (a << S) + b;
#endif
}

BH_HD uint64_t raw_hash1(int32_t k) {  // src/bloom_filter.cpp:8-20
    uint64_t x = (uint64_t)((int64_t)k * 32767 - 1);  // x = ~x + (x << 15)
    x = x ^ (x >> 12);
    x = lshl_add64<2>(x, x);                            // x = x + (x << 2)
    x = x ^ (x >> 4);
    x = (x << 11) + lshl_add64<3>(x, x);                // x = x * 2057
    x = x ^ (x >> 16);
    return x;
}

// (x ^ c) ^ (x >> S) for a 32-bit constant c: on gfx950 one 64-bit shift, one
// xor of the high words and one three-input xor of the low words (gfx950
// v_bitop3_b32 with truth table 0x96 = a ^ b ^ c; the compiler
// splits the shift into an alignbit + a second shift and xors c separately:
// 4 instructions against 3).
template <int S>
BH_HD uint64_t xor_shr_c(uint64_t x, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
    uint64_t t;
    asm("v_lshrrev_b64 %0, %2, %1" : "=v"(t) : "v"(x), "i"(S));
    uint32_t lo;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(lo) : "v"((uint32_t)x), "v"((uint32_t)t), "s"(c));
    const uint32_t hi = (uint32_t)(x >> 32) ^ (uint32_t)(t >> 32);
    return ((uint64_t)hi << 32) | lo;
#else
    return (x ^ c) ^ (x >> S);
#endif
}

BH_HD uint64_t raw_hash2(int32_t k) {  // src/bloom_filter.cpp:22-34
    uint64_t x = (uint64_t)((int64_t)k * 4097 + 0x7ed55d16);  // (x + 0x7ed55d16) + (x << 12)
    x = xor_shr_c<19>(x, 0xc761c23cu);                          // (x ^ 0xc761c23c) ^ (x >> 19)
    x = (x + 0x165667b1u) + (x << 5);
    x = (x + 0xd3a2646cu) ^ (x << 9);
    x = (x + 0xfd7046c5u) + (x << 3);
    x = xor_shr_c<16>(x, 0xb55a4f09u);                          // (x ^ 0xb55a4f09) ^ (x >> 16)
    return x;
}

BH_HD uint64_t raw_hash3(int32_t k) {  // src/bloom_filter.cpp:36-47
#if defined(__HIP_DEVICE_COMPILE__)
    // (x ^ 61) ^ (x >> 16) on the sign-extended key, by halves: the high word
    // of x is s = 0 or ~0 (the sign), so the result's high word is
    // s ^ (s >> 16) = s & 0xFFFF0000 and its low word k ^ 61 ^ alignbit(s, k, 16)
    // (one v_bitop3_b32 xor3; 61 is an inline constant).
    const uint32_t xl = (uint32_t)k, xh = (uint32_t)(k >> 31);
    uint32_t lo;
    asm("v_bitop3_b32 %0, %1, %2, 61 bitop3:0x96" : "=v"(lo) : "v"(xl), "v"(__builtin_amdgcn_alignbit(xh, xl, 16)));
    uint64_t x = ((uint64_t)(xh & 0xFFFF0000u) << 32) | lo;
#else
    uint64_t x = (uint64_t)(int64_t)k;
    x = (x ^ 61u) ^ (x >> 16);
#endif
    x = lshl_add64<3>(x, x);                            // x = x + (x << 3)
    x = x ^ (x >> 4);
    // x * 0x27d4eb2d mod 2^64 as lo32 * c (one v_mad_u64_u32) plus hi32 * c in
    // the high word (v_mul_lo_u32): the compiler's 64-bit multiply takes two
    // v_mad_u64_u32 and two moves
    x = (uint64_t)(uint32_t)x * 0x27d4eb2du + ((uint64_t)((uint32_t)(x >> 32) * 0x27d4eb2du) << 32);
    x = x ^ (x >> 15);
    return x;
}

// ---- exact x % m -------------------------------------------------------------
struct ModParams {
    uint64_t m;   // table.size()
    uint32_t R;   // 2^32 mod m                      (fast path)
    uint32_t dn;  // m << l, top bit set             (fast path)
    uint32_t v;   // floor((2^64-1)/dn) - 2^32       (fast path)
    uint32_t l;   // leading zeros of m as a u32     (fast path)
    uint32_t fast;  // 1 when m <= 0xFFFFFFFF
    uint32_t p2;    // 1 when m = d << t with d | 255, d >= 3, 12 <= t < 32 (p2 path)
    double minv;  // 1.0 / m                         (wide path)
    uint32_t p2t;   // t                             (p2 path)
    uint32_t p2d;   // d
    uint32_t p2M;   // ceil(2^32 / d)
    uint32_t p2pad;
};

// m = d << t with d | 255 (d in 3, 5, 15, 17, 51, 85, 255) and 12 <= t < 32:
// the form every LSM filter of the reference's configs takes (Run::Run sizes
// m = capacity * bits/entry, a power-of-two page count times 5 at 10 bits per
// entry, times 3 at 12: C2 5<<25, C3 5<<(17+2i), C4 3<<30, C5 5<<27).
inline bool p2_form(uint64_t m, uint32_t *d_out, uint32_t *t_out) {
    if (m == 0 || m > 0xFFFFFFFFull) return false;
    uint32_t t = (uint32_t)__builtin_ctzll(m);
    const uint64_t d = m >> t;
    if (t < 12 || t >= 32 || d < 3 || 255 % d != 0) return false;
    *d_out = (uint32_t)d;
    *t_out = t;
    return true;
}

// Host-side precomputation (m >= 1).
inline ModParams make_mod_params(uint64_t m) {
    ModParams p{};
    p.m = m;
    if (m >= 1 && m <= 0xFFFFFFFFull) {
        uint32_t m32 = (uint32_t)m;
        uint32_t l = (uint32_t)__builtin_clz(m32);
        uint32_t dn = m32 << l;
        p.fast = 1;
        p.l = l;
        p.dn = dn;
        p.v = (uint32_t)(~0ull / dn - (1ull << 32));
        p.R = (uint32_t)((1ull << 32) % m);
        uint32_t d = 0, t = 0;
        if (p2_form(m, &d, &t)) {
            p.p2 = 1;
            p.p2t = t;
            p.p2d = d;
            p.p2M = (uint32_t)(((1ull << 32) + d - 1) / d);
        }
    }
    p.minv = m ? 1.0 / (double)m : 0.0;
    return p;
}

// (x >> t) % d for m = d << t (p.p2).  d | 255 makes 2^8 = 1 (mod d), so a
// number is congruent mod d to the sum of its bytes: y = x >> t is
// yh * 2^32 + yl with yh = xh >> t < 2^20, and
//   y = yh + (sum of yl's four bytes)   (mod d),
// a sum s < 2^21 that gfx950 forms in ONE v_sad_u8 (|yl.b_i - 0| summed,
// plus yh).  Then q = mulhi(s, M) with M = ceil(2^32/d) = (2^32 + e)/d,
// e < d, is floor(s/d) exactly: s*M/2^32 = s/d + s*e/(d*2^32), and the excess
// stays below the 1/d gap to the next integer because s*e < 2^21 * 255 < 2^32.
// r = s - q*d is one v_mad_i32_i24 (q < 2^20, d < 2^8).
// 5 instructions (alignbit, shift, sad, mulhi, mad) against the general
// remainder's 10; tests/test_host.py fuzzes it against the oracle.
BH_HD uint32_t mod_p2_hi(uint64_t x, const ModParams &p) {
    const uint32_t xh = (uint32_t)(x >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t yl = __builtin_amdgcn_alignbit(xh, (uint32_t)x, p.p2t);
    const uint32_t s = __builtin_amdgcn_sad_u8(yl, 0u, xh >> p.p2t);
    const uint32_t q = __umulhi(s, p.p2M);
    return (uint32_t)((int)s + __mul24((int)q, -(int)p.p2d));  // one v_mad_i32_i24
#else
    const uint32_t yl = (uint32_t)(x >> p.p2t);
    const uint32_t s = (yl & 0xFFu) + ((yl >> 8) & 0xFFu) + ((yl >> 16) & 0xFFu) + (yl >> 24) +
                       (xh >> p.p2t);
    const uint32_t q = (uint32_t)(((uint64_t)s * p.p2M) >> 32);
    return s - q * p.p2d;
#endif
}

// (x >> 24) % d for the p2 form (d | 255): x >> 24 = xh * 2^8 + (xl >> 24)
// and 2^8 = 1 (mod d), so it is congruent to the sum of xh's four bytes plus
// xl's top byte: one shift and ONE v_sad_u8 (s <= 5 * 255), then the same
// mulhi / mad as mod_p2_hi -- 4 instructions against 5, the alignbit gone.
// plan_build's one-member ladder takes it when 24 lies in [s, t] (the hash
// bits [24, t) are then bin bits): a' = (x >> 24) % d = (2^(t-24) a + c) % d
// with a = (x >> t) % d and c = bits [24, t) of x, so a' is a relabelling of
// a for every bin, which pass 2 undoes block by block (ladder0_block).
BH_HD uint32_t mod_p2_hi24(uint64_t x, const ModParams &p) {
    const uint32_t xh = (uint32_t)(x >> 32);
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t s = __builtin_amdgcn_sad_u8(xh, 0u, (uint32_t)x >> 24);
    const uint32_t q = __umulhi(s, p.p2M);
    return (uint32_t)((int)s + __mul24((int)q, -(int)p.p2d));
#else
    const uint32_t s = (xh & 0xFFu) + ((xh >> 8) & 0xFFu) + ((xh >> 16) & 0xFFu) + (xh >> 24) +
                       ((uint32_t)x >> 24);
    const uint32_t q = (uint32_t)(((uint64_t)s * p.p2M) >> 32);
    return s - q * p.p2d;
#endif
}

// The bitmap block a = (x >> t) % d of image block a' = (x >> 24) % d in bin
// b of plan_build's one-member ladder with the relabelled pass 1 (s <= 24 <=
// t): c = bits [24, t) of x = b >> (24 - s), and a' = (2^(t-24) a + c) % d,
// so a = (a' - c) * 2^-(t-24) mod d (d odd).  inv = 2^-(t-24) mod d.
BH_HD uint32_t ladder0_block(uint32_t ap, uint32_t b, uint32_t s, uint32_t d, uint32_t inv) {
    const uint32_t c = (b >> (24 - s)) % d;
    return ((ap + d - c) * inv) % d;
}

// x % m for m = d << t (p.p2): ((x >> t) % d) << t | (x mod 2^t).
BH_HD uint32_t mod_p2(uint64_t x, const ModParams &p) {
    const uint32_t r = mod_p2_hi(x, p);
    return (r << p.p2t) | ((uint32_t)x & ((1u << p.p2t) - 1u));
}

// (x % m) << l for m < 2^32 (p.fast): the remainder before the final
// normalisation shift (callers that take bit-fields of it save that shift).
BH_HD uint32_t mod_fast_scaled(uint64_t x, const ModParams &p) {
    const uint32_t xh = (uint32_t)(x >> 32), xl = (uint32_t)x;
    const uint64_t y = (uint64_t)xh * p.R + xl;   // < m * 2^32, so u below < dn * 2^32
    const uint64_t u = y << p.l;
    const uint32_t u1 = (uint32_t)(u >> 32), u0 = (uint32_t)u;
    const uint64_t q = (uint64_t)p.v * u1 + u;    // (q1, q0) = v*u1 + (u1, u0); < 2^64
    const uint32_t q1 = (uint32_t)(q >> 32) + 1u;
    const uint32_t q0 = (uint32_t)q;
    uint32_t r = u0 - q1 * p.dn;
    if (r > q0) r += p.dn;
    if (r >= p.dn) r -= p.dn;
    return r;
}

// x % m for m < 2^32 (p.fast).  Returns the remainder as u32.
BH_HD uint32_t mod_fast(uint64_t x, const ModParams &p) { return mod_fast_scaled(x, p) >> p.l; }

// x % m for 2^32 <= m <= 2^46.  q = trunc(double(x) * (1/m)): x < 2^64 and
// m >= 2^32 make x/m < 2^32, and the three roundings (x to double, 1/m, the
// product) err by under 2^-50 relative, i.e. under 2^-18 absolute, so q is
// floor(x/m) or one off either way.  r = x - q*m in wrapping 64-bit
// arithmetic is then r_true - m (negative as int64: r < m < 2^46), r_true, or
// r_true + m (in [m, 2m)), fixed by one conditional add or subtract.
// tests/test_host.py fuzzes it against the oracle's exact remainder.
BH_HD uint64_t mod_wide(uint64_t x, const ModParams &p) {
    const uint64_t q = (uint64_t)((double)x * p.minv);
    uint64_t r = x - q * p.m;
    if ((int64_t)r < 0) r += p.m;
    else if (r >= p.m) r -= p.m;
    return r;
}

// x % m for m < 2^32: the p2 form when m has it, else the general remainder.
BH_HD uint32_t mod_32(uint64_t x, const ModParams &p) {
    return p.p2 ? mod_p2(x, p) : mod_fast(x, p);
}

BH_HD uint64_t mod_any(uint64_t x, const ModParams &p) {
    return p.fast ? (uint64_t)mod_32(x, p) : mod_wide(x, p);
}

// ---- exact q = x / S for 32-bit x, runtime S >= 2 (Granlund–Montgomery,
// "Division by invariant integers using multiplication", PLDI 1994, Fig 4.1):
// l = ceil(log2 S), M = floor(2^32 (2^l - S) / S) + 1,
// q = (t + ((x - t) >> 1)) >> (l - 1) with t = mulhi(M, x).
struct DivParams {
    uint32_t S;
    uint32_t M;
    uint32_t sh;  // l - 1
    uint32_t pad;
};

inline DivParams make_div_params(uint32_t S) {
    DivParams d{};
    d.S = S;
    uint32_t l = 0;
    while (l < 32 && (1ull << l) < S) l++;
    d.M = (uint32_t)(((1ull << 32) * ((1ull << l) - S)) / S + 1);
    d.sh = l - 1;
    return d;
}

BH_HD uint32_t div_fast(uint32_t x, const DivParams &d) {
    const uint32_t t = (uint32_t)(((uint64_t)d.M * x) >> 32);
    return (t + ((x - t) >> 1)) >> d.sh;
}

BH_HD void positions3(int32_t k, const ModParams &p, uint64_t out[3]) {
    out[0] = mod_any(raw_hash1(k), p);
    out[1] = mod_any(raw_hash2(k), p);
    out[2] = mod_any(raw_hash3(k), p);
}

}  // namespace bloomhip
