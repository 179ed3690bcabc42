// cg_glibc_rand.h -- glibc's rand() (random_r TYPE_3, the generator the
// reference's colour modes 1-2 consume, rasteriser/Source/skeleton.cpp:649-659),
// restated with jump-ahead so a frame's stream can start at any call index.
//
// glibc, seeded with 1 (the reference never calls srand):
//   r[0] = 1; r[i] = 16807 r[i-1] mod (2^31 - 1), i = 1..30 (Schrage's method);
//   r[i] = r[i-31], i = 31..33;  r[i] = r[i-31] + r[i-3] (mod 2^32), i >= 34;
//   call k (k = 0, 1, ...) returns r[k + 344] >> 1.
// For i >= 3 the sequence obeys r[i+31] = r[i+28] + r[i], characteristic
// polynomial P(x) = x^31 - x^28 - 1 over Z/2^32, so r[n] = sum_j c_j r[3+j]
// with sum_j c_j x^j = x^(n-3) mod P (and shifting the window shifts n).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace cg {

constexpr int kRandDeg = 31;

// c = a * b mod P (degree < 31 polynomials, coefficients mod 2^32)
inline void rand_poly_mulmod(const uint32_t *a, const uint32_t *b, uint32_t *c)
{
    uint32_t t[2 * kRandDeg - 1] = {};
    for (int i = 0; i < kRandDeg; ++i)
        for (int j = 0; j < kRandDeg; ++j) t[i + j] += a[i] * b[j];
    for (int k = 2 * kRandDeg - 2; k >= kRandDeg; --k) {   // x^k = x^(k-31) (x^28 + 1)
        t[k - 3] += t[k];
        t[k - kRandDeg] += t[k];
    }
    for (int i = 0; i < kRandDeg; ++i) c[i] = t[i];
}

// x^e mod P
inline void rand_poly_xpow(uint64_t e, uint32_t *out)
{
    uint32_t res[kRandDeg] = {}, base[kRandDeg] = {}, tmp[kRandDeg];
    res[0] = 1;
    base[1] = 1;
    for (; e; e >>= 1) {
        if (e & 1) {
            rand_poly_mulmod(res, base, tmp);
            for (int i = 0; i < kRandDeg; ++i) res[i] = tmp[i];
        }
        rand_poly_mulmod(base, base, tmp);
        for (int i = 0; i < kRandDeg; ++i) base[i] = tmp[i];
    }
    for (int i = 0; i < kRandDeg; ++i) out[i] = res[i];
}

// r[0 .. n) of the seed-1 state sequence (n >= 34)
inline std::vector<uint32_t> rand_state_prefix(int n)
{
    std::vector<uint32_t> r((size_t)n);
    int32_t w = 1;
    r[0] = 1;
    for (int i = 1; i < 31; ++i) {
        const int32_t hi = w / 127773, lo = w % 127773;
        w = 16807 * lo - 2836 * hi;
        if (w < 0) w += 2147483647;
        r[i] = (uint32_t)w;
    }
    for (int i = 31; i < 34; ++i) r[i] = r[i - 31];
    for (int i = 34; i < n; ++i) r[i] = r[i - 31] + r[i - 3];
    return r;
}

// The 61 state words r[idx .. idx + 61) with idx = 344 + call_index: the
// window of the stream's first value plus the 30 after it (a jump of J
// positions then needs only these and the coefficients of x^J mod P).
inline void rand_window(uint64_t call_index, uint32_t out[61])
{
    static const std::vector<uint32_t> r = rand_state_prefix(3 + kRandDeg + 61);
    uint32_t c[kRandDeg];
    rand_poly_xpow(call_index + 344 - 3, c);
    for (int j = 0; j < 61; ++j) {
        uint32_t v = 0;
        for (int i = 0; i < kRandDeg; ++i) v += c[i] * r[3 + i + j];
        out[j] = v;
    }
}

}  // namespace cg
