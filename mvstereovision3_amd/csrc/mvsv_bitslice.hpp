// mvsv_bitslice.hpp — bit-sliced SGM arithmetic (round 5).
//
// In the headline regime (configs/sgbm.yml: P1 = 2, P2 = 5 after OpenCV's
// defaulting, the no-wrap bound) every quantity a direction pass
// carries is a small integer: the clamped cost residual C' = min(C - min_d C,
// 2 P2) <= 10, the path state s(d) = min(L(d) - min_d L, P2) <= 5 and the
// delta = min(s(d), s(d -+ 1) + P1, P2) <= 5 (the
// residual's exactness argument is DESIGN.md §4b).  So the passes run
// bit-sliced: one 32-bit word holds bit b of 32 disparities, a 3-input
// boolean function of three such words is one v_bitop3_b32, and a lane
// updates 32 disparities of one bit plane per instruction instead of two
// (packed int16).  Disparity order inside a pixel's 64-disparity half h:
// word (h, e, b) bit p <-> d = 64 h + 2 p + e (E = even-d word, O = odd-d word).
//
// These helpers are per lane and per word and compile for the host too (the
// CPU check tests/cpp/bitslice_check.cpp runs the same functions against a
// scalar recurrence); the cross-lane steps live in the kernels.
#pragma once

#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define MVSV_BS_HD __host__ __device__ __forceinline__
#else
#define MVSV_BS_HD inline
#endif

namespace mvsv {
namespace bs {

// truth-table operands of v_bitop3_b32: result bit = TT[(a << 2) | (b << 1) | c]
constexpr unsigned kA = 0xF0u, kB = 0xCCu, kC = 0xAAu;

template <unsigned TT>
MVSV_BS_HD uint32_t lop3(uint32_t a, uint32_t b, uint32_t c)
{
    static_assert(TT < 256u, "3-input truth table");
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_bitop3_b32(a, b, c, TT);
#else
    uint32_t r = 0;
    for (int i = 0; i < 8; i++)
        if (TT & (1u << i)) r |= ((i & 4) ? a : ~a) & ((i & 2) ? b : ~b) & ((i & 1) ? c : ~c);
    return r;
#endif
}

// {hi:lo} >> s (v_alignbit_b32), 0 <= s < 32
MVSV_BS_HD uint32_t fshr(uint32_t hi, uint32_t lo, unsigned s)
{
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
}

// truth tables used below
constexpr unsigned kAndNotAB = (~kA & kB) & 0xFFu;                  // ~a & b
constexpr unsigned kLtChain = ((~kA & kB) | (~(kA ^ kB) & kC)) & 0xFFu;  // [a < b] with carry-in c; also the borrow of a - b - c
constexpr unsigned kMux = ((kA & kB) | (~kA & kC)) & 0xFFu;        // a ? b : c
constexpr unsigned kXor3 = (kA ^ kB ^ kC) & 0xFFu;
constexpr unsigned kMaj = ((kA & kB) | (kA & kC) | (kB & kC)) & 0xFFu;
static_assert(kAndNotAB == 0x0C && kLtChain == 0x8E && kMux == 0xCA && kXor3 == 0x96 && kMaj == 0xE8,
              "bitop3 truth tables");

// r = min(a, b) of two 3-bit sliced values (6 instructions)
MVSV_BS_HD void min3b(const uint32_t (&a)[3], const uint32_t (&b)[3], uint32_t (&r)[3])
{
    const uint32_t l0 = lop3<kAndNotAB>(a[0], b[0], a[0]);
    const uint32_t l1 = lop3<kLtChain>(a[1], b[1], l0);
    const uint32_t lt = lop3<kLtChain>(a[2], b[2], l1);  // a < b
    r[0] = lop3<kMux>(lt, a[0], b[0]);
    r[1] = lop3<kMux>(lt, a[1], b[1]);
    r[2] = lop3<kMux>(lt, a[2], b[2]);
}

// truth table of output bit k of u = min(t + P1, P2) over the 3-bit t (all 8
// codes: a neighbour outside [0, D) is the code 7 and maps to P2)
template <int P1, int P2>
constexpr unsigned g_table(int k)
{
    unsigned tt = 0;
    for (int t = 0; t < 8; t++) {
        const int u = t + P1 < P2 ? t + P1 : P2;
        if ((u >> k) & 1) tt |= 1u << t;
    }
    return tt;
}
template <int P1, int P2>
MVSV_BS_HD void gmap(const uint32_t (&t)[3], uint32_t (&u)[3])
{
    u[0] = lop3<g_table<P1, P2>(0)>(t[2], t[1], t[0]);
    u[1] = lop3<g_table<P1, P2>(1)>(t[2], t[1], t[0]);
    u[2] = lop3<g_table<P1, P2>(2)>(t[2], t[1], t[0]);
}

// the path delta of one word: min(s, min(s(d-1), s(d+1)) + P1, P2) with the
// neighbour words sl / sr already aligned to s (15 instructions)
template <int P1, int P2>
MVSV_BS_HD void delta3(const uint32_t (&s)[3], const uint32_t (&sl)[3],
                                                const uint32_t (&sr)[3], uint32_t (&dl)[3])
{
    uint32_t t[3], u[3];
    min3b(sl, sr, t);
    gmap<P1, P2>(t, u);
    min3b(s, u, dl);
}

// v = c + d, c 4-bit, d 3-bit, the sum known to be <= 15 (7 instructions)
MVSV_BS_HD void add43(const uint32_t (&c)[4], const uint32_t (&d)[3], uint32_t (&v)[4])
{
    const uint32_t k0 = c[0] & d[0];
    v[0] = c[0] ^ d[0];
    v[1] = lop3<kXor3>(c[1], d[1], k0);
    const uint32_t k1 = lop3<kMaj>(c[1], d[1], k0);
    v[2] = lop3<kXor3>(c[2], d[2], k1);
    const uint32_t k2 = lop3<kMaj>(c[2], d[2], k1);
    v[3] = c[3] ^ k2;
}

// v = a + b, both 3-bit, 4-bit result (6 instructions)
MVSV_BS_HD void add33(const uint32_t (&a)[3], const uint32_t (&b)[3], uint32_t (&v)[4])
{
    const uint32_t k0 = a[0] & b[0];
    v[0] = a[0] ^ b[0];
    v[1] = lop3<kXor3>(a[1], b[1], k0);
    const uint32_t k1 = lop3<kMaj>(a[1], b[1], k0);
    v[2] = lop3<kXor3>(a[2], b[2], k1);
    v[3] = lop3<kMaj>(a[2], b[2], k1);
}

// v = a + b, both 4-bit, 5-bit result (8 instructions)
MVSV_BS_HD void add44(const uint32_t (&a)[4], const uint32_t (&b)[4], uint32_t (&v)[5])
{
    const uint32_t k0 = a[0] & b[0];
    v[0] = a[0] ^ b[0];
    v[1] = lop3<kXor3>(a[1], b[1], k0);
    const uint32_t k1 = lop3<kMaj>(a[1], b[1], k0);
    v[2] = lop3<kXor3>(a[2], b[2], k1);
    const uint32_t k2 = lop3<kMaj>(a[2], b[2], k1);
    v[3] = lop3<kXor3>(a[3], b[3], k2);
    v[4] = lop3<kMaj>(a[3], b[3], k2);
}

// v = a + b, a 5-bit, b 4-bit, the sum known to be < 64 (6-bit result, 9 instructions)
MVSV_BS_HD void add54(const uint32_t (&a)[5], const uint32_t (&b)[4], uint32_t (&v)[6])
{
    const uint32_t k0 = a[0] & b[0];
    v[0] = a[0] ^ b[0];
    v[1] = lop3<kXor3>(a[1], b[1], k0);
    const uint32_t k1 = lop3<kMaj>(a[1], b[1], k0);
    v[2] = lop3<kXor3>(a[2], b[2], k1);
    const uint32_t k2 = lop3<kMaj>(a[2], b[2], k1);
    v[3] = lop3<kXor3>(a[3], b[3], k2);
    const uint32_t k3 = lop3<kMaj>(a[3], b[3], k2);
    v[4] = a[4] ^ k3;
    v[5] = a[4] & k3;
}

// v = a + b, both 5-bit, the sum known to be < 64 (6-bit result, 10 instructions)
MVSV_BS_HD void add55(const uint32_t (&a)[5], const uint32_t (&b)[5], uint32_t (&v)[6])
{
    const uint32_t k0 = a[0] & b[0];
    v[0] = a[0] ^ b[0];
    v[1] = lop3<kXor3>(a[1], b[1], k0);
    const uint32_t k1 = lop3<kMaj>(a[1], b[1], k0);
    v[2] = lop3<kXor3>(a[2], b[2], k1);
    const uint32_t k2 = lop3<kMaj>(a[2], b[2], k1);
    v[3] = lop3<kXor3>(a[3], b[3], k2);
    const uint32_t k3 = lop3<kMaj>(a[3], b[3], k2);
    v[4] = lop3<kXor3>(a[4], b[4], k3);
    v[5] = lop3<kMaj>(a[4], b[4], k3);
}

// The WTA's S'' = n C' + (sum of the n deltas), 7 bits.
// MODE_HH (n = 8): s6 = the eight deltas (<= 40), S'' = s6 + 8 C' <= 120 --
// the low 3 bits of s6 stay, C' adds to the rest (7 instructions).
MVSV_BS_HD void total8(const uint32_t (&c)[4], const uint32_t (&s6)[6], uint32_t (&S)[7])
{
    const uint32_t top[3] = {s6[3], s6[4], s6[5]};
    uint32_t hi[4];
    add43(c, top, hi);
    S[0] = s6[0], S[1] = s6[1], S[2] = s6[2];
    S[3] = hi[0], S[4] = hi[1], S[5] = hi[2], S[6] = hi[3];
}
// MODE_SGBM (n = 5): s5 = the five deltas (<= 25), S'' = (s5 + C') + 4 C' <= 75:
// t = s5 + C' <= 35, its low 2 bits stay, C' adds to t >> 2 (<= 8; 17 instructions)
MVSV_BS_HD void total5(const uint32_t (&c)[4], const uint32_t (&s5)[5], uint32_t (&S)[7])
{
    uint32_t t[6];
    add54(s5, c, t);
    const uint32_t a[4] = {t[2], t[3], t[4], t[5]};
    uint32_t hi[5];
    add44(a, c, hi);
    S[0] = t[0], S[1] = t[1];
    S[2] = hi[0], S[3] = hi[1], S[4] = hi[2], S[5] = hi[3], S[6] = hi[4];
}

// Tie rules of the WTA among the d that attain min S (d = 64 h + 2 p + e on
// word bit p of parity e, half h): OpenCV 3.4's MODE_HH loop and later
// releases take the smallest d; 3.4's MODE_SGBM SSE2 loop keeps one minimum
// per SIMD lane d mod 8 (the first d of that lane) and takes the lowest lane
// that holds the overall minimum -- the smallest (d mod 8, d).  Key of the
// winner among the set bits `mask` of one word (smaller key wins; d in the low
// 7 bits; 1 << 20 for an empty mask).  d mod 8 = 2 (p mod 4) + e.
MVSV_BS_HD int wta_key(uint32_t mask, int h, int e, bool lane_rule)
{
    if (!mask) return 1 << 20;
    uint32_t sel = mask;
    if (lane_rule) {
        const uint32_t m0 = mask & 0x11111111u, m1 = mask & 0x22222222u, m2 = mask & 0x44444444u;
        sel = m0 ? m0 : m1 ? m1 : m2 ? m2 : mask;
    }
#if defined(__HIP_DEVICE_COMPILE__)
    const int p = __builtin_ctz(sel);
#else
    int p = 0;
    while (!((sel >> p) & 1u)) p++;
#endif
    const int d = 64 * h + 2 * p + e;
    return lane_rule ? ((2 * (p & 3) + e) << 7) | d : d;
}

// s = min(v - m, P2) for a 4-bit v >= m and a lane-uniform 3-bit m given as
// all-ones / all-zero masks m0..m2 (13 instructions)
template <int P2>
MVSV_BS_HD void subclamp(const uint32_t (&v)[4], uint32_t m0, uint32_t m1, uint32_t m2,
                                                  uint32_t (&s)[3])
{
    static_assert(P2 >= 2 && P2 <= 5, "3-bit states: P2 in [2, 5]");
    const uint32_t r0 = v[0] ^ m0;
    const uint32_t b0 = lop3<kAndNotAB>(v[0], m0, m0);
    const uint32_t r1 = lop3<kXor3>(v[1], m1, b0);
    const uint32_t b1 = lop3<kLtChain>(v[1], m1, b0);
    const uint32_t r2 = lop3<kXor3>(v[2], m2, b1);
    const uint32_t b2 = lop3<kLtChain>(v[2], m2, b1);
    // r3 = v3 ^ b2; ge = [r >= P2] = r3 | y
    uint32_t y;
    if constexpr (P2 == 2)
        y = r2 | r1;
    else if constexpr (P2 == 3)
        y = lop3<(kA | (kB & kC)) & 0xFFu>(r2, r1, r0);
    else if constexpr (P2 == 4)
        y = r2;
    else
        y = lop3<(kA & (kB | kC)) & 0xFFu>(r2, r1, r0);
    const uint32_t ge = lop3<((kA ^ kB) | kC) & 0xFFu>(v[3], b2, y);
    s[0] = (P2 & 1) ? (r0 | ge) : lop3<(kA & ~kB) & 0xFFu>(r0, ge, ge);
    s[1] = (P2 & 2) ? (r1 | ge) : lop3<(kA & ~kB) & 0xFFu>(r1, ge, ge);
    s[2] = (P2 & 4) ? (r2 | ge) : lop3<(kA & ~kB) & 0xFFu>(r2, ge, ge);
}

// Plane layouts of the pipeline (rows padded to W1q = W1 rounded up to 4
// pixels; rowq = (frame * H + y) * W1q).  The C' plane groups four pixels:
// [x / 4][q][x % 4][bit b] with q = 2 h + e, so a lane that owns one (h, e)
// word set of a row reads 64 contiguous bytes per four pixels; the line delta
// planes likewise [x / 4][q][x % 4][b < 3].
MVSV_BS_HD size_t cq_word(size_t rowq, int x, int q) { return (rowq + (size_t)(x & ~3)) * 16 + q * 16 + (x & 3) * 4; }
MVSV_BS_HD size_t dl_word(size_t rowq, int x, int q) { return (rowq + (size_t)(x & ~3)) * 12 + q * 12 + (x & 3) * 3; }
MVSV_BS_HD int padq(int w) { return (w + 3) & ~3; }

// scalar value of a sliced number at word bit p (host checks, sub-pixel reads)
template <int NB>
MVSV_BS_HD int bits_at(const uint32_t (&w)[NB], int p)
{
    int v = 0;
    for (int k = 0; k < NB; k++) v |= (int)((w[k] >> p) & 1u) << k;
    return v;
}

}  // namespace bs
}  // namespace mvsv
