// Host check of the bit-sliced SGM arithmetic (mvsv_bitslice.hpp) and of the
// lane-pair step the bit-sliced kernels run (mvsv_bsgm.hip): every helper
// against its scalar definition, then whole scanlines of the direction
// recurrence -- two lanes per pixel (64-disparity halves), E / O parity words,
// the neighbour words through the partner lane, the bit-serial row minimum --
// against OpenCV 3.4's recurrence on unclamped costs, the
// lane-quad form of the step (the line kernel's), the grouped plane layouts,
// the cost kernel's 32 x 32 lane transpose against its definition, and the WTA
// sum / argmin / neighbour extraction of the bit-sliced final pass.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../../mvstereovision3_amd/csrc/mvsv_bitslice.hpp"

using namespace mvsv::bs;

static int fails = 0;
#define CHECK(c, ...)                          \
    do {                                       \
        if (!(c)) {                            \
            if (fails++ < 20) {                \
                std::printf("FAIL %s: ", #c);  \
                std::printf(__VA_ARGS__);      \
                std::printf("\n");             \
            }                                  \
        }                                      \
    } while (0)

constexpr int P1 = 2, P2 = 5;
constexpr uint32_t ONES = 0xffffffffu;

template <int NB>
static void put(uint32_t (&w)[NB], int p, int v)
{
    for (int k = 0; k < NB; k++) w[k] = (w[k] & ~(1u << p)) | ((uint32_t)((v >> k) & 1) << p);
}

static void check_helpers(std::mt19937& rng)
{
    for (int it = 0; it < 2000; it++) {
        uint32_t a[3] = {0, 0, 0}, b[3] = {0, 0, 0}, s[3] = {0, 0, 0}, c4[4] = {0, 0, 0, 0}, a4[4] = {0, 0, 0, 0};
        uint32_t a5[5] = {0, 0, 0, 0, 0};
        int va[32], vb[32], vs[32], vc[32], v4[32], v5[32];
        for (int p = 0; p < 32; p++) {
            va[p] = rng() % 8;
            vb[p] = rng() % 8;
            vs[p] = rng() % (P2 + 1);
            vc[p] = rng() % (2 * P2 + 1);
            v4[p] = rng() % 16;
            v5[p] = rng() % 32;
            put(a, p, va[p]);
            put(b, p, vb[p]);
            put(s, p, vs[p]);
            put(c4, p, vc[p]);
            put(a4, p, v4[p]);
            put(a5, p, v5[p]);
        }
        uint32_t r[3], u[3], d[3], v[4], w4[4], w5[5], w6[6];
        min3b(a, b, r);
        gmap<P1, P2>(a, u);
        delta3<P1, P2>(s, a, b, d);
        add33(a, b, w4);
        add44(a4, a4, w5);
        uint32_t sm[3] = {s[0], s[1], s[2]};
        add43(c4, sm, v);
        add54(a5, a4, w6);
        uint32_t w6b[6];
        add55(a5, a5, w6b);
        for (int p = 0; p < 32; p++) {
            CHECK(bits_at<3>(r, p) == std::min(va[p], vb[p]), "min3b");
            CHECK(bits_at<3>(u, p) == std::min(va[p] + P1, P2), "gmap");
            const int t = std::min(va[p], vb[p]);
            CHECK(bits_at<3>(d, p) == std::min(vs[p], std::min(t + P1, P2)), "delta3 %d %d %d", vs[p], va[p], vb[p]);
            CHECK(bits_at<4>(w4, p) == va[p] + vb[p], "add33");
            CHECK(bits_at<5>(w5, p) == 2 * v4[p], "add44");
            CHECK(bits_at<4>(v, p) == vc[p] + vs[p], "add43");
            CHECK(bits_at<6>(w6, p) == v5[p] + v4[p], "add54");
            CHECK(bits_at<6>(w6b, p) == 2 * v5[p], "add55");
        }
        // subclamp: v >= m, m lane-uniform in [0, P2]
        const int m = rng() % (P2 + 1);
        uint32_t vv[4] = {0, 0, 0, 0};
        int vvs[32];
        for (int p = 0; p < 32; p++) {
            vvs[p] = m + rng() % (16 - m);
            put(vv, p, vvs[p]);
        }
        uint32_t so[3];
        subclamp<P2>(vv, (m & 1) ? ONES : 0u, (m & 2) ? ONES : 0u, (m & 4) ? ONES : 0u, so);
        for (int p = 0; p < 32; p++) CHECK(bits_at<3>(so, p) == std::min(vvs[p] - m, P2), "subclamp");
    }
    // subclamp for every P2 the header allows, exhaustively
    auto sc = [&](auto tag) {
        constexpr int Q = decltype(tag)::value;
        for (int m = 0; m <= Q; m++)
            for (int vbase = 0; vbase < 16; vbase += 1) {
                uint32_t vv[4] = {0, 0, 0, 0};
                int vs[32];
                for (int p = 0; p < 32; p++) {
                    vs[p] = std::max(m, (vbase + p) % 16);
                    put(vv, p, vs[p]);
                }
                uint32_t so[3];
                subclamp<Q>(vv, (m & 1) ? ONES : 0u, (m & 2) ? ONES : 0u, (m & 4) ? ONES : 0u, so);
                for (int p = 0; p < 32; p++) CHECK(bits_at<3>(so, p) == std::min(vs[p] - m, Q), "subclamp P2=%d", Q);
            }
    };
    sc(std::integral_constant<int, 2>());
    sc(std::integral_constant<int, 3>());
    sc(std::integral_constant<int, 4>());
    sc(std::integral_constant<int, 5>());

    // the WTA totals: S'' = 8 C' + s (s <= 40) and 5 C' + s (s <= 25)
    for (int it = 0; it < 2000; it++) {
        uint32_t c[4] = {0, 0, 0, 0}, s6[6] = {0, 0, 0, 0, 0, 0}, s5[5] = {0, 0, 0, 0, 0}, S8[7], S5[7];
        int vc[32], v8[32], v5[32];
        for (int p = 0; p < 32; p++) {
            vc[p] = rng() % (2 * P2 + 1);
            v8[p] = rng() % (8 * P2 + 1);
            v5[p] = rng() % (5 * P2 + 1);
            put(c, p, vc[p]);
            put(s6, p, v8[p]);
            put(s5, p, v5[p]);
        }
        total8(c, s6, S8);
        total5(c, s5, S5);
        for (int p = 0; p < 32; p++) {
            CHECK(bits_at<7>(S8, p) == 8 * vc[p] + v8[p], "total8");
            CHECK(bits_at<7>(S5, p) == 5 * vc[p] + v5[p], "total5");
        }
    }
    // wta_key: the smallest d, or the smallest (d mod 8, d) (MODE_SGBM lane rule)
    for (int it = 0; it < 4000; it++) {
        const uint32_t mask = it < 8 ? (1u << (rng() % 32)) : (uint32_t)rng() & (uint32_t)rng();
        const int h = rng() % 2, e = rng() % 2;
        int bd = -1, bl = -1;
        for (int p = 0; p < 32; p++)
            if ((mask >> p) & 1u) {
                const int d = 64 * h + 2 * p + e;
                if (bd < 0) bd = d;
                if (bl < 0 || (d & 7) < (bl & 7)) bl = d;
            }
        const int k0 = wta_key(mask, h, e, false), k1 = wta_key(mask, h, e, true);
        if (!mask) {
            CHECK(k0 == (1 << 20) && k1 == (1 << 20), "wta_key empty");
        } else {
            CHECK(k0 == bd, "wta_key min d");
            CHECK((k1 & 127) == bl && (k1 >> 7) == (bl & 7), "wta_key lane rule %08x", mask);
        }
    }
}

// One pixel's 128 disparities on two lanes (h = 0, 1), each with E / O words.
struct Lane {
    uint32_t sE[3], sO[3];
};

// the kernels' step for one direction: new state and delta of a pixel
// (mirrors bs_dir_step in mvsv_bsgm.hip; `partner` = the other lane's value)
static void pair_step(Lane (&ln)[2], const uint32_t (&cE)[2][4], const uint32_t (&cO)[2][4], uint32_t (&dEo)[2][3],
                      uint32_t (&dOo)[2][3])
{
    uint32_t vE[2][4], vO[2][4];
    for (int h = 0; h < 2; h++) {
        const Lane& o = ln[h ^ 1];
        uint32_t slE[3], srO[3];
        for (int k = 0; k < 3; k++) {
            const uint32_t prevO = (h == 1 ? o.sO[k] : 0u) | (h == 0 ? ONES : 0u);
            const uint32_t nextE = (h == 0 ? o.sE[k] : 0u) | (h == 1 ? ONES : 0u);
            slE[k] = fshr(ln[h].sO[k], prevO, 31);
            srO[k] = fshr(nextE, ln[h].sE[k], 1);
        }
        delta3<P1, P2>(ln[h].sE, slE, ln[h].sO, dEo[h]);
        delta3<P1, P2>(ln[h].sO, ln[h].sE, srO, dOo[h]);
        add43(cE[h], dEo[h], vE[h]);
        add43(cO[h], dOo[h], vO[h]);
    }
    // bit-serial minimum over both lanes (min <= P2 < 8: bit 3 is 0)
    uint32_t cdE[2], cdO[2], M[3][2];
    for (int h = 0; h < 2; h++) {
        cdE[h] = ~vE[h][3];
        cdO[h] = ~vO[h][3];
    }
    for (int b = 2; b >= 0; b--) {
        uint32_t zE[2], zO[2], any[2];
        for (int h = 0; h < 2; h++) {
            zE[h] = cdE[h] & ~vE[h][b];
            zO[h] = cdO[h] & ~vO[h][b];
            any[h] = zE[h] | zO[h];
        }
        const uint32_t a0 = any[0] | any[1], a1 = any[1] | any[0];
        for (int h = 0; h < 2; h++) {
            const bool f = (h ? a1 : a0) != 0;
            cdE[h] = f ? zE[h] : cdE[h];
            cdO[h] = f ? zO[h] : cdO[h];
            M[b][h] = f ? 0u : ONES;
        }
    }
    for (int h = 0; h < 2; h++) {
        subclamp<P2>(vE[h], M[0][h], M[1][h], M[2][h], ln[h].sE);
        subclamp<P2>(vO[h], M[0][h], M[1][h], M[2][h], ln[h].sO);
    }
}

// The lane-quad step (bs_quad_step in mvsv_bsgm.hip): lane q = 2 h + e holds
// the parity-e words of half h; the shifted neighbour is alignbit(hi = quad
// lane q + 1, lo = q - 1) by 1 (odd) / 31 (even), all-ones past the quad's
// ends, the partner word is lo (odd) / hi (even), the minimum ORs the quad.
static void quad_step(uint32_t (&s)[4][3], const uint32_t (&c)[4][4], uint32_t (&d)[4][3])
{
    uint32_t v[4][4];
    for (int q = 0; q < 4; q++) {
        const bool odd = (q & 1) != 0;
        uint32_t nb[3], pt[3];
        for (int k = 0; k < 3; k++) {
            const uint32_t hi = q < 3 ? s[q + 1][k] : ONES;
            const uint32_t lo = q > 0 ? s[q - 1][k] : ONES;
            nb[k] = fshr(hi, lo, odd ? 1 : 31);
            pt[k] = odd ? lo : hi;
        }
        delta3<P1, P2>(s[q], nb, pt, d[q]);
        add43(c[q], d[q], v[q]);
    }
    uint32_t kk[4], M[3];
    for (int q = 0; q < 4; q++) kk[q] = ~v[q][3];
    for (int b = 2; b >= 0; b--) {
        uint32_t z[4], any = 0;
        for (int q = 0; q < 4; q++) {
            z[q] = kk[q] & ~v[q][b];
            any |= z[q];
        }
        const bool f = any != 0u;
        if (b > 0 && f)
            for (int q = 0; q < 4; q++) kk[q] = z[q];
        M[b] = f ? 0u : ONES;
    }
    for (int q = 0; q < 4; q++) subclamp<P2>(v[q], M[0], M[1], M[2], s[q]);
}

static int dof(int h, int e, int p) { return 64 * h + 2 * p + e; }

static void check_recurrence(std::mt19937& rng)
{
    constexpr int D = 128;
    for (int line = 0; line < 300; line++) {
        const int N = 40 + rng() % 60;
        // scalar state (OpenCV's L - the unbiased cost of the first step)
        std::vector<int> Lp(D, 0);
        Lane ln[2] = {};
        uint32_t sq[4][3] = {};  // the lane-quad form of the same scanline
        const int mode = line % 4;  // cost distributions: wide, narrow, flat, spiky
        for (int i = 0; i < N; i++) {
            int C[D];
            for (int d = 0; d < D; d++) {
                switch (mode) {
                case 0: C[d] = rng() % 3000; break;
                case 1: C[d] = 100 + rng() % 12; break;
                case 2: C[d] = 50 + (rng() % 7 == 0 ? rng() % 3 : 0); break;
                default: C[d] = (rng() % 9 == 0) ? rng() % 20 : 200 + rng() % 40; break;
                }
            }
            if (i % 17 == 16) {  // a path restart: state of an out-of-image predecessor is 0
                std::fill(Lp.begin(), Lp.end(), 0);
                ln[0] = ln[1] = Lane{};
                for (auto& w : sq) w[0] = w[1] = w[2] = 0u;
            }
            int minLp = 1 << 30;
            for (int d = 0; d < D; d++) minLp = std::min(minLp, Lp[d]);
            int delta[D], L[D];
            for (int d = 0; d < D; d++) {
                const int lm = d > 0 ? Lp[d - 1] : 1 << 29, lpp = d < D - 1 ? Lp[d + 1] : 1 << 29;
                const int t = std::min(std::min(Lp[d], std::min(lm, lpp) + P1), minLp + P2);
                delta[d] = t - minLp;
                L[d] = C[d] + delta[d];
            }
            Lp.assign(L, L + D);
            // bit-sliced: C' = min(C - m, 2 P2)
            int m = 1 << 30;
            for (int d = 0; d < D; d++) m = std::min(m, C[d]);
            uint32_t cE[2][4] = {}, cO[2][4] = {};
            for (int h = 0; h < 2; h++)
                for (int p = 0; p < 32; p++) {
                    put(cE[h], p, std::min(C[dof(h, 0, p)] - m, 2 * P2));
                    put(cO[h], p, std::min(C[dof(h, 1, p)] - m, 2 * P2));
                }
            uint32_t dE[2][3], dO[2][3];
            pair_step(ln, cE, cO, dE, dO);
            {
                uint32_t cq[4][4], dq[4][3];
                for (int q = 0; q < 4; q++)
                    for (int b = 0; b < 4; b++) cq[q][b] = (q & 1) ? cO[q >> 1][b] : cE[q >> 1][b];
                quad_step(sq, cq, dq);
                for (int q = 0; q < 4; q++)
                    for (int p = 0; p < 32; p++) {
                        const int d = dof(q >> 1, q & 1, p);
                        CHECK(bits_at<3>(dq[q], p) == delta[d], "quad delta line %d step %d d %d", line, i, d);
                    }
            }
            for (int h = 0; h < 2; h++)
                for (int p = 0; p < 32; p++) {
                    CHECK(bits_at<3>(dE[h], p) == delta[dof(h, 0, p)], "delta line %d step %d d %d", line, i, dof(h, 0, p));
                    CHECK(bits_at<3>(dO[h], p) == delta[dof(h, 1, p)], "delta line %d step %d d %d", line, i, dof(h, 1, p));
                }
            int minL = 1 << 30;
            for (int d = 0; d < D; d++) minL = std::min(minL, L[d]);
            for (int h = 0; h < 2; h++)
                for (int p = 0; p < 32; p++) {
                    CHECK(bits_at<3>(ln[h].sE, p) == std::min(L[dof(h, 0, p)] - minL, P2), "state");
                    CHECK(bits_at<3>(ln[h].sO, p) == std::min(L[dof(h, 1, p)] - minL, P2), "state");
                    for (int e = 0; e < 2; e++)
                        CHECK(bits_at<3>(sq[2 * h + e], p) == std::min(L[dof(h, e, p)] - minL, P2), "quad state");
                }
        }
    }
}

// The cost kernel's transpose: lane p (of a 32-lane half) holds bytes for
// columns k = 0..3, byte k = C'(col(k), 2p) | C'(col(k), 2p + 1) << 4; after
// five delta-swap stages lane q holds word (k, e, b) = q's bits k = q >> 3,
// e = (q >> 2) & 1, b = q & 3: bit p = bit b of C'(col(k), 2p + e).
static void check_transpose(std::mt19937& rng)
{
    for (int it = 0; it < 200; it++) {
        uint32_t X[32], ref[32];
        int cv[4][64];
        for (int k = 0; k < 4; k++)
            for (int d = 0; d < 64; d++) cv[k][d] = rng() % 11;
        for (int p = 0; p < 32; p++) {
            X[p] = 0;
            for (int k = 0; k < 4; k++) X[p] |= (uint32_t)(cv[k][2 * p] | (cv[k][2 * p + 1] << 4)) << (8 * k);
        }
        for (int q = 0; q < 32; q++) {
            const int k = q >> 3, e = (q >> 2) & 1, b = q & 3;
            ref[q] = 0;
            for (int p = 0; p < 32; p++) ref[q] |= (uint32_t)((cv[k][2 * p + e] >> b) & 1) << p;
        }
        // stages s = 16, 8, 4, 2, 1 (mirrors bs_transpose32 in mvsv_sgbm.hip)
        static const uint32_t Mk[5] = {0x55555555u, 0x33333333u, 0x0F0F0F0Fu, 0x00FF00FFu, 0x0000FFFFu};
        for (int j = 4; j >= 0; j--) {
            const int s = 1 << j;
            uint32_t Y[32];
            for (int l = 0; l < 32; l++) {
                const uint32_t partner = X[l ^ s];
                const bool upper = (l & s) != 0;
                const uint32_t sh = upper ? fshr(partner, partner, s) : fshr(partner, partner, 32 - s);
                const uint32_t K = upper ? ~Mk[j] : Mk[j];
                Y[l] = (K & X[l]) | (~K & sh);
            }
            for (int l = 0; l < 32; l++) X[l] = Y[l];
        }
        for (int q = 0; q < 32; q++) CHECK(X[q] == ref[q], "transpose word %d", q);
    }
}

// The grouped plane layouts: the cost kernel's store word for transpose lane
// p of the wave's four columns (mvsv_sgbm.hip) is cq_word's (column c, q =
// 2 h + e) word + bit b, and both layouts tile a row of groups exactly.
static void check_layouts()
{
    for (int p = 0; p < 64; p++) {
        const int q = p & 31, kq = q >> 3;
        const int c = ((kq & 1) << 1) | (kq >> 1);
        const int h = p >> 5, e = (q & 7) >> 2, b = q & 3;
        const int qw = (2 * (p >> 5) + ((q & 7) >> 2)) * 16 + c * 4 + (q & 3);
        CHECK((size_t)qw == cq_word(0, c, 2 * h + e) + b, "cost kernel C' word p %d", p);
    }
    for (int W1 : {1, 5, 8, 131, 1151}) {
        const int Wq = padq(W1);
        std::vector<int> seen16((size_t)Wq * 16, 0), seen12((size_t)Wq * 12, 0);
        for (int x = 0; x < Wq; x++)
            for (int q = 0; q < 4; q++) {
                for (int b = 0; b < 4; b++) seen16[cq_word(0, x, q) + b]++;
                for (int b = 0; b < 3; b++) seen12[dl_word(0, x, q) + b]++;
            }
        for (int v : seen16) CHECK(v == 1, "cq_word tiling W1 %d", W1);
        for (int v : seen12) CHECK(v == 1, "dl_word tiling W1 %d", W1);
        CHECK(cq_word((size_t)Wq, 0, 0) == (size_t)Wq * 16, "cq_word row stride");
        CHECK(dl_word((size_t)Wq, 0, 0) == (size_t)Wq * 12, "dl_word row stride");
    }
}

int main()
{
    std::mt19937 rng(12345);
    check_helpers(rng);
    check_recurrence(rng);
    check_transpose(rng);
    check_layouts();
    std::printf("bitslice checks: %d failures\n", fails);
    return fails ? 1 : 0;
}
