/*
 * mvsv_oracle.c — CPU restatement of OpenCV 3.4 StereoSGBM / StereoBM as
 * called by the reference's Disparity::sgbm / Disparity::bm
 * (src/disparity.cpp:6-22).  TEST INFRASTRUCTURE ONLY — see mvsv_oracle.h.
 *
 * The SGBM core deliberately keeps OpenCV's buffer discipline (rolling
 * horizontal-sum ring, running cost rows, double-buffered per-direction path
 * costs with zeroed borders, saturating int16 arithmetic of the CV_SIMD128
 * path) so that its quirks are reproduced by construction rather than by
 * special cases.  oracle/twin.py restates the same semantics in closed form
 * and the two are cross-checked in tests/test_oracle_cross.py.
 */
#include "mvsv_oracle.h"

#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int iabs(int a) { return a < 0 ? -a : a; }
static inline int sat16(int v) { return v > 32767 ? 32767 : (v < -32768 ? -32768 : v); }

#define MAX_COST 32767
#define DISP_SHIFT 4
#define DISP_SCALE 16

/* ------------------------------------------------------------------------ */
/* SGBM: effective parameters ([OpenCV] computeDisparitySGBM prologue)       */
/* ------------------------------------------------------------------------ */
typedef struct {
    int minD, maxD, D, SW2, SH2, ftzero, uniq, disp12, P1, P2;
    int minX1, maxX1, W1, INVALID;
    int fullDP;
} sgbm_eff;

static int sgbm_resolve(const orc_sgbm_params* p, int W, sgbm_eff* e)
{
    int bs = p->block_size > 0 ? p->block_size : 5;
    e->minD = p->min_disparity;
    e->D = p->num_disparities;
    e->maxD = e->minD + e->D;
    e->SW2 = bs / 2;
    e->SH2 = bs / 2;
    e->ftzero = imax(p->pre_filter_cap, 15) | 1;
    e->uniq = p->uniqueness_ratio >= 0 ? p->uniqueness_ratio : 10;
    e->disp12 = p->disp12_max_diff > 0 ? p->disp12_max_diff : 1;
    e->P1 = p->p1 > 0 ? p->p1 : 2;
    e->P2 = imax(p->p2 > 0 ? p->p2 : 5, e->P1 + 1);
    e->minX1 = imax(e->maxD, 0);
    e->maxX1 = W + imin(e->minD, 0);
    e->W1 = e->maxX1 - e->minX1;
    e->INVALID = (e->minD - 1) * DISP_SCALE;
    e->fullDP = p->mode == 1;
    return 0;
}

/* clipTab[k] = (uchar)(clip(k - 1024, -ftzero, ftzero) + ftzero) */
#define TAB_OFS 1024
#define TAB_SIZE (256 + TAB_OFS * 2)

static void make_cliptab(int ftzero, uint8_t* tab)
{
    for (int k = 0; k < TAB_SIZE; k++)
        tab[k] = (uint8_t)(imin(imax(k - TAB_OFS, -ftzero), ftzero) + ftzero);
}

/* [OpenCV] calcPixelCostBT for one image row y, single channel.
 * cost is W1*D int16, indexed [x - minX1][d - minD]; it is overwritten. */
static void pixel_cost_bt(const uint8_t* L, ptrdiff_t ls, const uint8_t* R,
                          ptrdiff_t rs, int W, int H, int y, const sgbm_eff* e,
                          const uint8_t* tab, int16_t* cost, uint8_t* work)
{
    const int minD = e->minD, maxD = e->maxD, D = e->D;
    const int minX1 = e->minX1, maxX1 = e->maxX1;
    const int minX2 = imax(minX1 - maxD, 0), maxX2 = imin(maxX1 - minD, W);
    /* prow1[c][x]: left, prow2[c][W-1-x]: right (x-reversed); c=0 sobel, 1 raw */
    uint8_t* prow1 = work;
    uint8_t* prow2 = work + 2 * W;
    uint8_t* v0buf = work + 4 * W;
    uint8_t* v1buf = work + 5 * W;
    const uint8_t* r1 = L + (ptrdiff_t)y * ls;
    const uint8_t* r2 = R + (ptrdiff_t)y * rs;
    ptrdiff_t n1 = y > 0 ? -ls : 0, s1 = y < H - 1 ? ls : 0;
    ptrdiff_t n2 = y > 0 ? -rs : 0, s2 = y < H - 1 ? rs : 0;
    const uint8_t* t = tab + TAB_OFS;

    for (int c = 0; c < 2; c++) {
        prow1[W * c] = prow1[W * c + W - 1] = t[0];
        prow2[W * c] = prow2[W * c + W - 1] = t[0];
    }
    int xa = imax(imin(minX1, minX2) - 1, 1);
    int xb = imin(imax(maxX1, maxX2) + 1, W - 1);
    for (int x = xa; x < xb; x++) {
        prow1[x] = t[(r1[x + 1] - r1[x - 1]) * 2 + r1[x + n1 + 1] - r1[x + n1 - 1] +
                     r1[x + s1 + 1] - r1[x + s1 - 1]];
        prow2[W - 1 - x] = t[(r2[x + 1] - r2[x - 1]) * 2 + r2[x + n2 + 1] - r2[x + n2 - 1] +
                             r2[x + s2 + 1] - r2[x + s2 - 1]];
        prow1[x + W] = r1[x];
        prow2[W - 1 - x + W] = r2[x];
    }

    memset(cost, 0, sizeof(int16_t) * (size_t)e->W1 * D);

    for (int c = 0; c < 2; c++) {
        const uint8_t* p1 = prow1 + W * c;
        const uint8_t* p2 = prow2 + W * c;
        int diff_scale = c == 0 ? 0 : 2;
        /* Birchfield-Tomasi half-pixel interval of the reversed right row.
         * Computed for every index; only [W-maxX2, W-1-minX2] is read. */
        for (int j = 0; j < W; j++) {
            int v = p2[j];
            int vl = j > 0 ? (v + p2[j - 1]) / 2 : v;
            int vr = j < W - 1 ? (v + p2[j + 1]) / 2 : v;
            v0buf[j] = (uint8_t)imin(imin(vl, vr), v);
            v1buf[j] = (uint8_t)imax(imax(vl, vr), v);
        }
        for (int x = minX1; x < maxX1; x++) {
            int u = p1[x];
            int ul = x > 0 ? (u + p1[x - 1]) / 2 : u;
            int ur = x < W - 1 ? (u + p1[x + 1]) / 2 : u;
            int u0 = imin(imin(ul, ur), u), u1 = imax(imax(ul, ur), u);
            int16_t* cp = cost + (size_t)(x - minX1) * D - minD;
            for (int d = minD; d < maxD; d++) {
                int j = W - 1 - x + d;
                int v = p2[j], v0 = v0buf[j], v1 = v1buf[j];
                int c0 = imax(imax(0, u - v1), v0 - u);
                int c1 = imax(imax(0, v - u1), u0 - v);
                cp[d] = (int16_t)(cp[d] + (imin(c0, c1) >> diff_scale));
            }
        }
    }
}

/* Shared by orc_sgbm_core (mode 0: run; mode 1: only dump C). */
static int sgbm_run(const uint8_t* L, ptrdiff_t ls, const uint8_t* R, ptrdiff_t rs,
                    int W, int H, const orc_sgbm_params* p, unsigned flags,
                    int16_t* disp, ptrdiff_t ds, int16_t* Cdump)
{
    sgbm_eff e;
    if (!L || !R || W <= 0 || H <= 0 || !p) return -1;
    sgbm_resolve(p, W, &e);
    if (e.D <= 0 || e.D % 16 != 0) return -2;

    if (e.minX1 >= e.maxX1) {
        if (disp)
            for (int y = 0; y < H; y++)
                for (int x = 0; x < W; x++) disp[(ptrdiff_t)y * ds + x] = (int16_t)e.INVALID;
        return Cdump ? 0 : 0;
    }

    const int D = e.D, W1 = e.W1, minD = e.minD, SW2 = e.SW2, SH2 = e.SH2;
    const int P1 = e.P1, P2 = e.P2;
    const int npasses = e.fullDP ? 2 : 1;
    const size_t row = (size_t)W1 * D;
    const size_t CSsize = row * (e.fullDP ? (size_t)H : 1);
    const int nrows = SH2 * 2 + 2;
    const int D2 = D + 2;                 /* d = -1 .. D padded */
    const int XS = W1 + 2;                /* x = -1 .. W1 padded */

    uint8_t tab[TAB_SIZE];
    make_cliptab(e.ftzero, tab);

    int16_t* Cbuf = (int16_t*)malloc(sizeof(int16_t) * CSsize);
    int16_t* Sbuf = (int16_t*)malloc(sizeof(int16_t) * CSsize);
    int16_t* hsum = (int16_t*)malloc(sizeof(int16_t) * row * nrows);
    int16_t* pix = (int16_t*)malloc(sizeof(int16_t) * row);
    uint8_t* work = (uint8_t*)malloc((size_t)W * 6);
    /* Lr[buf][x+1][dir][d+1] ; minLr[buf][x+1][dir] */
    int16_t* Lr[2];
    int16_t* minLr[2];
    int16_t* disp2cost = (int16_t*)malloc(sizeof(int16_t) * W);
    int16_t* disp2 = (int16_t*)malloc(sizeof(int16_t) * W);
    for (int k = 0; k < 2; k++) {
        Lr[k] = (int16_t*)malloc(sizeof(int16_t) * (size_t)XS * 4 * D2);
        minLr[k] = (int16_t*)malloc(sizeof(int16_t) * (size_t)XS * 4);
    }
    if (!Cbuf || !Sbuf || !hsum || !pix || !work || !Lr[0] || !Lr[1] || !minLr[0] ||
        !minLr[1] || !disp2cost || !disp2) {
        free(Cbuf); free(Sbuf); free(hsum); free(pix); free(work);
        free(Lr[0]); free(Lr[1]); free(minLr[0]); free(minLr[1]);
        free(disp2cost); free(disp2);
        return -3;
    }
#define LR(buf, x, k, d) Lr[buf][(((size_t)((x) + 1) * 4 + (k)) * D2) + (d) + 1]
#define MINLR(buf, x, k) minLr[buf][(size_t)((x) + 1) * 4 + (k)]

    /* add P2 to every C(x,y): the bias cancels in the recurrence */
    for (size_t k = 0; k < CSsize; k++) Cbuf[k] = (int16_t)P2;

    for (int pass = 1; pass <= npasses; pass++) {
        int y1, y2, dy, x1, x2, dx;
        if (pass == 1) { y1 = 0; y2 = H; dy = 1; x1 = 0; x2 = W1; dx = 1; }
        else { y1 = H - 1; y2 = -1; dy = -1; x1 = W1 - 1; x2 = -1; dx = -1; }
        int cur = 0, prv = 1;
        /* zero both path buffers; the d = -1 / D pads hold MAX_COST */
        for (int b = 0; b < 2; b++) {
            for (int x = -1; x <= W1; x++)
                for (int k = 0; k < 4; k++) {
                    LR(b, x, k, -1) = MAX_COST;
                    LR(b, x, k, D) = MAX_COST;
                    for (int d = 0; d < D; d++) LR(b, x, k, d) = 0;
                    MINLR(b, x, k) = 0;
                }
        }

        for (int y = y1; y != y2; y += dy) {
            int16_t* C = Cbuf + (e.fullDP ? (size_t)y * row : 0);
            int16_t* S = Sbuf + (e.fullDP ? (size_t)y * row : 0);

            if (pass == 1) {
                int dya = y == 0 ? 0 : y + SH2, dyb = y == 0 ? SH2 : dya;
                for (int k = dya; k <= dyb; k++) {
                    int16_t* hadd = hsum + (size_t)(imin(k, H - 1) % nrows) * row;
                    if (k < H) {
                        pixel_cost_bt(L, ls, R, rs, W, H, k, &e, tab, pix, work);
                        for (int d = 0; d < D; d++) {
                            int s = 0;
                            /* OpenCV reads pix[0..SW2] unclamped; identical for W1 > SW2 */
                            for (int x = 0; x <= SW2; x++)
                                s += pix[(size_t)imin(x, W1 - 1) * D + d] * (x == 0 ? SW2 + 1 : 1);
                            hadd[d] = (int16_t)s;
                        }
                        if (y > 0) {
                            const int16_t* hsub = hsum + (size_t)(imax(y - SH2 - 1, 0) % nrows) * row;
                            const int16_t* Cprev = (!e.fullDP) ? C : C - row;
                            if (flags & ORC_F_FIRSTCOL_FIX)
                                for (int d = 0; d < D; d++)
                                    C[d] = (int16_t)sat16(sat16(Cprev[d] - hsub[d]) + hadd[d]);
                            for (int x = 1; x < W1; x++) {
                                const int16_t* padd = pix + (size_t)imin(x + SW2, W1 - 1) * D;
                                const int16_t* psub = pix + (size_t)imax(x - SW2 - 1, 0) * D;
                                for (int d = 0; d < D; d++) {
                                    int hv = (int16_t)(hadd[(size_t)(x - 1) * D + d] + padd[d] - psub[d]);
                                    hadd[(size_t)x * D + d] = (int16_t)hv;
                                    size_t i = (size_t)x * D + d;
                                    C[i] = (int16_t)sat16(sat16(Cprev[i] - hsub[i]) + hv);
                                }
                            }
                        } else {
                            for (int x = 1; x < W1; x++) {
                                const int16_t* padd = pix + (size_t)imin(x + SW2, W1 - 1) * D;
                                const int16_t* psub = pix + (size_t)imax(x - SW2 - 1, 0) * D;
                                for (int d = 0; d < D; d++)
                                    hadd[(size_t)x * D + d] =
                                        (int16_t)(hadd[(size_t)(x - 1) * D + d] + padd[d] - psub[d]);
                            }
                        }
                    }
                    if (y == 0) {
                        int scale = k == 0 ? SH2 + 1 : 1;
                        for (size_t i = 0; i < row; i++)
                            C[i] = (int16_t)(C[i] + hadd[i] * scale);
                    }
                }
                for (size_t i = 0; i < row; i++) S[i] = 0;
            }

            if (Cdump) {
                if (pass == 1) memcpy(Cdump + (size_t)y * row, C, sizeof(int16_t) * row);
                continue;
            }

            /* clear the left / right borders of the current path row */
            for (int k = 0; k < 4; k++) {
                for (int d = 0; d < D; d++) { LR(cur, -1, k, d) = 0; LR(cur, W1, k, d) = 0; }
                MINLR(cur, -1, k) = 0;
                MINLR(cur, W1, k) = 0;
            }

            for (int x = x1; x != x2; x += dx) {
                /* predecessors: 0:(x-dx, y) 1:(x-1, y-dy) 2:(x, y-dy) 3:(x+1, y-dy) */
                const int px[4] = {x - dx, x - 1, x, x + 1};
                const int pb[4] = {cur, prv, prv, prv};
                const int16_t* Cp = C + (size_t)x * D;
                int16_t* Sp = S + (size_t)x * D;
                int minL[4] = {MAX_COST, MAX_COST, MAX_COST, MAX_COST};
                int16_t Lnew[4][512 + 2];
                int16_t* Lnp[4];
                int16_t* Lbig = NULL;
                if (D > 512) {
                    Lbig = (int16_t*)malloc(sizeof(int16_t) * 4 * D);
                    for (int k = 0; k < 4; k++) Lnp[k] = Lbig + (size_t)k * D;
                } else {
                    for (int k = 0; k < 4; k++) Lnp[k] = Lnew[k];
                }
                for (int k = 0; k < 4; k++) {
                    int delta = (int16_t)(MINLR(pb[k], px[k], k) + P2);
                    for (int d = 0; d < D; d++) {
                        int lp = LR(pb[k], px[k], k, d);
                        int lm = sat16(LR(pb[k], px[k], k, d - 1) + P1);
                        int lq = sat16(LR(pb[k], px[k], k, d + 1) + P1);
                        int m = imin(imin(imin(lp, lm), lq), delta);
                        int v = sat16(sat16(m - delta) + Cp[d]);
                        Lnp[k][d] = (int16_t)v;
                        if (v < minL[k]) minL[k] = v;
                    }
                }
                for (int k = 0; k < 4; k++) {
                    for (int d = 0; d < D; d++) LR(cur, x, k, d) = Lnp[k][d];
                    MINLR(cur, x, k) = (int16_t)minL[k];
                }
                /* S = sat(sat(S + sat(L0+L1)) + sat(L2+L3))  (CV_SIMD128 order) */
                for (int d = 0; d < D; d++) {
                    int a = sat16(Lnp[0][d] + Lnp[1][d]);
                    int b = sat16(Lnp[2][d] + Lnp[3][d]);
                    Sp[d] = (int16_t)sat16(sat16(Sp[d] + a) + b);
                }
                free(Lbig);
            }

            if (pass == npasses) {
                int16_t* dptr = disp + (ptrdiff_t)y * ds;
                for (int x = 0; x < W; x++) {
                    dptr[x] = disp2[x] = (int16_t)e.INVALID;
                    disp2cost[x] = MAX_COST;
                }
                for (int x = W1 - 1; x >= 0; x--) {
                    int16_t* Sp = S + (size_t)x * D;
                    int minS = MAX_COST, bestDisp = -1;
                    if (npasses == 1) {
                        /* 5th direction (R->L) of MODE_SGBM, fused with WTA */
                        int delta = (int16_t)(MINLR(cur, x + 1, 0) + P2);
                        const int16_t* Cp = C + (size_t)x * D;
                        int minL0 = MAX_COST;
                        int laneMin[8], laneBest[8];
                        for (int l = 0; l < 8; l++) { laneMin[l] = MAX_COST; laneBest[l] = -1; }
                        /* values of x+1 are read before x is written: buffer the row */
                        int16_t Ltmp[512];
                        int16_t* Lt = D > 512 ? (int16_t*)malloc(sizeof(int16_t) * D) : Ltmp;
                        for (int d = 0; d < D; d++) {
                            int lp = LR(cur, x + 1, 0, d);
                            int lm = sat16(LR(cur, x + 1, 0, d - 1) + P1);
                            int lq = sat16(LR(cur, x + 1, 0, d + 1) + P1);
                            int m = imin(imin(imin(lp, lm), lq), delta);
                            int v = sat16(sat16(m - delta) + Cp[d]);
                            Lt[d] = (int16_t)v;
                            if (v < minL0) minL0 = v;
                            int sv = sat16(v + Sp[d]);
                            Sp[d] = (int16_t)sv;
                            int l = d & 7;
                            if (laneMin[l] > sv) laneBest[l] = d;
                            laneMin[l] = imin(laneMin[l], sv);
                        }
                        for (int d = 0; d < D; d++) LR(cur, x, 0, d) = Lt[d];
                        if (Lt != Ltmp) free(Lt);
                        MINLR(cur, x, 0) = (int16_t)minL0;
                        if (flags & ORC_F_WTA_MIN_D) {
                            for (int d = 0; d < D; d++)
                                if (Sp[d] < minS) { minS = Sp[d]; bestDisp = d; }
                        } else {
                            for (int l = 0; l < 8; l++) minS = imin(minS, laneMin[l]);
                            for (int l = 0; l < 8; l++)
                                if (laneMin[l] == minS) { bestDisp = laneBest[l]; break; }
                        }
                    } else {
                        for (int d = 0; d < D; d++)
                            if (Sp[d] < minS) { minS = Sp[d]; bestDisp = d; }
                    }

                    int d;
                    for (d = 0; d < D; d++)
                        if (Sp[d] * (100 - e.uniq) < minS * 100 && iabs(bestDisp - d) > 1) break;
                    if (d < D) continue;
                    d = bestDisp;
                    int x2i = x + e.minX1 - d - minD;
                    if (x2i >= 0 && x2i < W && disp2cost[x2i] > minS) {
                        disp2cost[x2i] = (int16_t)minS;
                        disp2[x2i] = (int16_t)(d + minD);
                    }
                    if (0 < d && d < D - 1) {
                        int denom2 = imax(Sp[d - 1] + Sp[d + 1] - 2 * Sp[d], 1);
                        d = d * DISP_SCALE + ((Sp[d - 1] - Sp[d + 1]) * DISP_SCALE + denom2) / (denom2 * 2);
                    } else {
                        d *= DISP_SCALE;
                    }
                    dptr[x + e.minX1] = (int16_t)(d + minD * DISP_SCALE);
                }
                for (int x = e.minX1; x < e.maxX1; x++) {
                    int d1 = dptr[x];
                    if (d1 == e.INVALID) continue;
                    int dl = d1 >> DISP_SHIFT;
                    int dh = (d1 + DISP_SCALE - 1) >> DISP_SHIFT;
                    int xl = x - dl, xh = x - dh;
                    if (0 <= xl && xl < W && disp2[xl] >= minD && iabs(disp2[xl] - dl) > e.disp12 &&
                        0 <= xh && xh < W && disp2[xh] >= minD && iabs(disp2[xh] - dh) > e.disp12)
                        dptr[x] = (int16_t)e.INVALID;
                }
            }
            /* shift the cyclic path buffers */
            int t = cur; cur = prv; prv = t;
        }
        if (Cdump) break;
    }
#undef LR
#undef MINLR
    free(Cbuf); free(Sbuf); free(hsum); free(pix); free(work);
    free(Lr[0]); free(Lr[1]); free(minLr[0]); free(minLr[1]);
    free(disp2cost); free(disp2);
    return Cdump ? e.W1 : 0;
}

int orc_sgbm_core(const uint8_t* L, ptrdiff_t ls, const uint8_t* R, ptrdiff_t rs, int W,
                  int H, const orc_sgbm_params* p, unsigned flags, int16_t* out,
                  ptrdiff_t os)
{
    if (!out) return -1;
    return sgbm_run(L, ls, R, rs, W, H, p, flags, out, os, NULL);
}

int orc_sgbm_cost_volume(const uint8_t* L, ptrdiff_t ls, const uint8_t* R, ptrdiff_t rs,
                         int W, int H, const orc_sgbm_params* p, unsigned flags,
                         int16_t* C)
{
    sgbm_eff e;
    if (!p || !C) return -1;
    sgbm_resolve(p, W, &e);
    if (e.minX1 >= e.maxX1) return 0;
    return sgbm_run(L, ls, R, rs, W, H, p, flags, NULL, 0, C);
}

int orc_sgbm_compute(const uint8_t* L, ptrdiff_t ls, const uint8_t* R, ptrdiff_t rs,
                     int W, int H, const orc_sgbm_params* p, unsigned flags,
                     int16_t* out, ptrdiff_t os)
{
    int rc = orc_sgbm_core(L, ls, R, rs, W, H, p, flags, out, os);
    if (rc < 0) return rc;
    orc_median3x3_s16(out, os, W, H, out, os);
    if (p->speckle_window_size > 0)
        rc = orc_filter_speckles_s16(out, os, W, H, (p->min_disparity - 1) * DISP_SCALE,
                                     p->speckle_window_size, DISP_SCALE * p->speckle_range);
    return rc < 0 ? rc : 0;
}

/* ------------------------------------------------------------------------ */
/* medianBlur(3x3), CV_16S, replicate border                                 */
/* ------------------------------------------------------------------------ */
static int cmp_s16(const void* a, const void* b)
{
    return (int)*(const int16_t*)a - (int)*(const int16_t*)b;
}

void orc_median3x3_s16(const int16_t* src, ptrdiff_t ss, int W, int H, int16_t* dst,
                       ptrdiff_t dstr)
{
    int16_t* tmp = (int16_t*)malloc(sizeof(int16_t) * (size_t)W * H);
    for (int y = 0; y < H; y++)
        memcpy(tmp + (size_t)y * W, src + (ptrdiff_t)y * ss, sizeof(int16_t) * W);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            int16_t v[9];
            int n = 0;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    int yy = imin(imax(y + dy, 0), H - 1), xx = imin(imax(x + dx, 0), W - 1);
                    v[n++] = tmp[(size_t)yy * W + xx];
                }
            qsort(v, 9, sizeof(int16_t), cmp_s16);
            dst[(ptrdiff_t)y * dstr + x] = v[4];
        }
    free(tmp);
}

/* ------------------------------------------------------------------------ */
/* filterSpeckles (CV_16S): 4-connected regions of pixels != newVal whose    */
/* neighbours differ by <= maxDiff; regions of size <= maxSpeckleSize are    */
/* overwritten with newVal.  Raster-order seeds, explicit DFS stack.         */
/* ------------------------------------------------------------------------ */
int orc_filter_speckles_s16(int16_t* img, ptrdiff_t st, int W, int H, int newVal,
                            int maxSpeckleSize, int maxDiff)
{
    size_t np = (size_t)W * H;
    int* labels = (int*)calloc(np, sizeof(int));
    int* stack = (int*)malloc(sizeof(int) * (np + 1));
    unsigned char* rtype = (unsigned char*)calloc(np + 1, 1);
    if (!labels || !stack || !rtype) { free(labels); free(stack); free(rtype); return -3; }
    int curlabel = 0;
    for (int i = 0; i < H; i++) {
        int16_t* ds = img + (ptrdiff_t)i * st;
        int* ls = labels + (size_t)W * i;
        for (int j = 0; j < W; j++) {
            if (ds[j] == newVal) continue;
            if (ls[j]) {
                if (rtype[ls[j]]) ds[j] = (int16_t)newVal;
                continue;
            }
            int sp = 0;
            int px = j, py = i;
            curlabel++;
            int count = 0;
            ls[j] = curlabel;
            for (;;) {
                count++;
                int16_t* dpp = img + (ptrdiff_t)py * st + px;
                int dp = *dpp;
                int* lpp = labels + (size_t)W * py + px;
                if (py < H - 1 && !lpp[W] && dpp[st] != newVal && iabs(dp - dpp[st]) <= maxDiff) {
                    lpp[W] = curlabel; stack[sp++] = (py + 1) * W + px;
                }
                if (py > 0 && !lpp[-W] && dpp[-st] != newVal && iabs(dp - dpp[-st]) <= maxDiff) {
                    lpp[-W] = curlabel; stack[sp++] = (py - 1) * W + px;
                }
                if (px < W - 1 && !lpp[1] && dpp[1] != newVal && iabs(dp - dpp[1]) <= maxDiff) {
                    lpp[1] = curlabel; stack[sp++] = py * W + px + 1;
                }
                if (px > 0 && !lpp[-1] && dpp[-1] != newVal && iabs(dp - dpp[-1]) <= maxDiff) {
                    lpp[-1] = curlabel; stack[sp++] = py * W + px - 1;
                }
                if (sp == 0) break;
                int q = stack[--sp];
                py = q / W; px = q % W;
            }
            if (count <= maxSpeckleSize) {
                rtype[ls[j]] = 1;
                ds[j] = (int16_t)newVal;
            } else {
                rtype[ls[j]] = 0;
            }
        }
    }
    free(labels); free(stack); free(rtype);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* StereoBM                                                                  */
/* ------------------------------------------------------------------------ */
void orc_prefilter_xsobel(const uint8_t* src, ptrdiff_t ss, int W, int H, int ftzero,
                          uint8_t* dst)
{
    const int OFS = 256 * 4, TABSZ = OFS * 2 + 256;
    uint8_t tab[OFS * 2 + 256];
    for (int x = 0; x < TABSZ; x++)
        tab[x] = (uint8_t)(x - OFS < -ftzero ? 0 : x - OFS > ftzero ? ftzero * 2 : x - OFS + ftzero);
    uint8_t val0 = tab[OFS];
    int y;
    for (y = 0; y < H - 1; y += 2) {
        const uint8_t* srow1 = src + (ptrdiff_t)y * ss;
        const uint8_t* srow0 = y > 0 ? srow1 - ss : (H > 1 ? srow1 + ss : srow1);
        const uint8_t* srow2 = y < H - 1 ? srow1 + ss : (H > 1 ? srow1 - ss : srow1);
        const uint8_t* srow3 = y < H - 2 ? srow1 + ss * 2 : srow1;
        uint8_t* d0 = dst + (size_t)y * W;
        uint8_t* d1 = d0 + W;
        d0[0] = d0[W - 1] = d1[0] = d1[W - 1] = val0;
        for (int x = 1; x < W - 1; x++) {
            int a0 = srow0[x + 1] - srow0[x - 1], a1 = srow1[x + 1] - srow1[x - 1];
            int a2 = srow2[x + 1] - srow2[x - 1], a3 = srow3[x + 1] - srow3[x - 1];
            d0[x] = tab[a0 + a1 * 2 + a2 + OFS];
            d1[x] = tab[a1 + a2 * 2 + a3 + OFS];
        }
    }
    for (; y < H; y++)
        for (int x = 0; x < W; x++) dst[(size_t)y * W + x] = val0;
}

/* [OpenCV] prefilterNorm (PREFILTER_NORMALIZED_RESPONSE) */
static void prefilter_norm(const uint8_t* src, ptrdiff_t ss, int W, int H, int winsize,
                           int ftzero, uint8_t* dst)
{
    int wsz2 = winsize / 2;
    int* vsumbuf = (int*)malloc(sizeof(int) * (size_t)(W + 2 * wsz2 + 4));
    int* vsum = vsumbuf + wsz2 + 1;
    int scale_g = winsize * winsize / 8, scale_s = (1024 + scale_g) / (scale_g * 2);
    const int OFS = 256 * 5, TABSZ = OFS * 2 + 256;
    uint8_t* tab = (uint8_t*)malloc(TABSZ);
    scale_g *= scale_s;
    for (int x = 0; x < TABSZ; x++)
        tab[x] = (uint8_t)(x - OFS < -ftzero ? 0 : x - OFS > ftzero ? ftzero * 2 : x - OFS + ftzero);
    for (int x = 0; x < W; x++) vsum[x] = (uint16_t)(src[x] * (wsz2 + 2));
    for (int y = 1; y < wsz2; y++)
        for (int x = 0; x < W; x++) vsum[x] = (uint16_t)(vsum[x] + src[(ptrdiff_t)ss * y + x]);
    for (int y = 0; y < H; y++) {
        const uint8_t* top = src + ss * imax(y - wsz2 - 1, 0);
        const uint8_t* bottom = src + ss * imin(y + wsz2, H - 1);
        const uint8_t* prev = src + ss * imax(y - 1, 0);
        const uint8_t* curr = src + ss * y;
        const uint8_t* next = src + ss * imin(y + 1, H - 1);
        uint8_t* dptr = dst + (size_t)y * W;
        int x;
        for (x = 0; x < W; x++) vsum[x] = (uint16_t)(vsum[x] + bottom[x] - top[x]);
        for (x = 0; x <= wsz2; x++) {
            vsum[-x - 1] = vsum[0];
            vsum[W + x] = vsum[W - 1];
        }
        int sum = vsum[0] * (wsz2 + 1);
        for (x = 1; x <= wsz2; x++) sum += vsum[x];
        int val = ((curr[0] * 5 + curr[1] + prev[0] + next[0]) * scale_g - sum * scale_s) >> 10;
        dptr[0] = tab[val + OFS];
        for (x = 1; x < W - 1; x++) {
            sum += vsum[x + wsz2] - vsum[x - wsz2 - 1];
            val = ((curr[x] * 4 + curr[x - 1] + curr[x + 1] + prev[x] + next[x]) * scale_g -
                   sum * scale_s) >> 10;
            dptr[x] = tab[val + OFS];
        }
        sum += vsum[x + wsz2] - vsum[x - wsz2 - 1];
        val = ((curr[x] * 5 + curr[x - 1] + prev[x] + next[x]) * scale_g - sum * scale_s) >> 10;
        dptr[x] = tab[val + OFS];
    }
    free(vsumbuf);
    free(tab);
}

static inline int16_t disp_descale(int v1, int v2, int d)
{
    return (int16_t)((v1 * 256 + (d != 0 ? v2 * 256 / d : 0) + 15) >> 4);
}

/* [OpenCV] findStereoCorrespondenceBM on one stripe = rows [row0,row1) of
 * the full images (dy0 = row0, dy1 = H - row1 rows available outside). */
static void bm_stripe(const uint8_t* Lf, const uint8_t* Rf, int W, int H, int row0, int row1,
                      const orc_bm_params* p, int16_t* disp, ptrdiff_t ds, int* costmap)
{
    const int wsz = p->block_size, wsz2 = wsz / 2;
    const int dy0 = imin(row0, wsz2 + 1), dy1 = imin(H - row1, wsz2 + 1);
    const int ndisp = p->num_disparities, mindisp = p->min_disparity;
    const int lofs = imax(ndisp - 1 + mindisp, 0), rofs = -imin(ndisp - 1 + mindisp, 0);
    const int width = W, height = row1 - row0;
    const int width1 = width - rofs - ndisp + 1;
    const int ftzero = p->pre_filter_cap;
    const int16_t FILTERED = (int16_t)((mindisp - 1) * (1 << DISP_SHIFT));  /* no UB shift of a negative value */
    const int nrow = height + dy0 + dy1;
    /* hsad[y + dy0][d], cbuf[ring][y + dy0][d], htext[y + wsz2 + 1] */
    int* hsad0 = (int*)calloc((size_t)nrow * ndisp, sizeof(int));
    unsigned char* cbuf0 = (unsigned char*)calloc((size_t)(wsz + 1) * nrow * ndisp, 1);
    int* htextb = (int*)calloc((size_t)(height + 2 * wsz2 + 4), sizeof(int));
    int* htext = htextb + wsz2 + 1;
    int* sadb = (int*)calloc((size_t)ndisp + 2, sizeof(int));
    int* sad = sadb + 1;
    uint8_t tab[256];
    for (int x = 0; x < 256; x++) tab[x] = (uint8_t)iabs(x - ftzero);
    const uint8_t* lptr0 = Lf + (size_t)row0 * W + lofs;
    const uint8_t* rptr0 = Rf + (size_t)row0 * W + rofs;
#define HSAD(y) (hsad0 + (size_t)((y) + dy0) * ndisp)
#define CBUF(slot, y) (cbuf0 + ((size_t)(slot) * nrow + (size_t)((y) + dy0)) * ndisp)

    for (int x = -wsz2 - 1; x < wsz2; x++) {
        int lc = imin(imax(x, -lofs), width - lofs - 1);
        int rc = imin(imax(x, -rofs), width - rofs - ndisp);
        for (int y = -dy0; y < height + dy1; y++) {
            const uint8_t* lp = lptr0 + (ptrdiff_t)y * W + lc;
            const uint8_t* rp = rptr0 + (ptrdiff_t)y * W + rc;
            int lval = lp[0];
            int* hs = HSAD(y);
            unsigned char* cb = CBUF(x + wsz2 + 1, y);
            for (int d = 0; d < ndisp; d++) {
                int diff = iabs(lval - rp[d]);
                cb[d] = (unsigned char)diff;
                hs[d] += diff;
            }
            htext[y] += tab[lval];
        }
    }
    for (int y = 0; y < height; y++) {
        int16_t* dr = disp + (ptrdiff_t)(row0 + y) * ds;
        for (int x = 0; x < lofs; x++) dr[x] = FILTERED;
        for (int x = lofs + width1; x < width; x++) dr[x] = FILTERED;
    }
    /* OpenCV runs x to width1 even when lofs + width1 > W (minDisparity > 0)
     * and spills the tail into the next row (a data race between stripes);
     * the restatement stops at the row end, see DESIGN.md. */
    const int xend = imin(width1, width - lofs);
    for (int x = 0; x < xend; x++) {
        int x0 = x - wsz2 - 1, x1 = x + wsz2;
        int slot_sub = (x0 + wsz2 + 1) % (wsz + 1);
        int slot_add = (x1 + wsz2 + 1) % (wsz + 1);
        int lcs = imin(imax(x0, -lofs), width - 1 - lofs);
        int lca = imin(imax(x1, -lofs), width - 1 - lofs);
        int rca = imin(imax(x1, -rofs), width - ndisp - rofs);
        for (int y = -dy0; y < height + dy1; y++) {
            const uint8_t* lp = lptr0 + (ptrdiff_t)y * W + lca;
            const uint8_t* lps = lptr0 + (ptrdiff_t)y * W + lcs;
            const uint8_t* rp = rptr0 + (ptrdiff_t)y * W + rca;
            int lval = lp[0];
            int* hs = HSAD(y);
            unsigned char* cb = CBUF(slot_add, y);
            const unsigned char* cbs = CBUF(slot_sub, y);
            for (int d = 0; d < ndisp; d++) {
                int diff = iabs(lval - rp[d]);
                int sub = cbs[d];
                cb[d] = (unsigned char)diff;
                hs[d] = hs[d] + diff - sub;
            }
            htext[y] += tab[lval] - tab[lps[0]];
        }
        for (int y = dy1; y <= wsz2; y++) htext[height + y] = htext[height + dy1 - 1];
        for (int y = -wsz2 - 1; y < -dy0; y++) htext[y] = htext[-dy0];

        int tsum = 0;
        for (int d = 0; d < ndisp; d++) sad[d] = HSAD(-dy0)[d] * (wsz2 + 2 - dy0);
        for (int y = 1 - dy0; y < wsz2; y++)
            for (int d = 0; d < ndisp; d++) sad[d] += HSAD(y)[d];
        for (int y = -wsz2 - 1; y < wsz2; y++) tsum += htext[y];

        for (int y = 0; y < height; y++) {
            int minsad = INT_MAX, mind = -1;
            const int* hs = HSAD(imin(y + wsz2, height + dy1 - 1));
            const int* hsub = HSAD(imax(y - wsz2 - 1, -dy0));
            for (int d = 0; d < ndisp; d++) {
                int cur = sad[d] + hs[d] - hsub[d];
                sad[d] = cur;
                if (cur < minsad) { minsad = cur; mind = d; }
            }
            int16_t* dp = disp + (ptrdiff_t)(row0 + y) * ds + lofs + x;
            tsum += htext[y + wsz2] - htext[y - wsz2 - 1];
            if (tsum < p->texture_threshold) { *dp = FILTERED; continue; }
            if (p->uniqueness_ratio > 0) {
                int thresh = minsad + (minsad * p->uniqueness_ratio / 100);
                int d;
                for (d = 0; d < ndisp; d++)
                    if ((d < mind - 1 || d > mind + 1) && sad[d] <= thresh) break;
                if (d < ndisp) { *dp = FILTERED; continue; }
            }
            sad[-1] = sad[1];
            sad[ndisp] = sad[ndisp - 2];
            int pp = sad[mind + 1], nn = sad[mind - 1];
            int dd = pp + nn - 2 * sad[mind] + iabs(pp - nn);
            *dp = disp_descale(ndisp - mind - 1 + mindisp, pp - nn, dd);
            if (costmap) costmap[(size_t)(row0 + y) * W + lofs + x] = sad[mind];
        }
    }
#undef HSAD
#undef CBUF
    free(hsad0); free(cbuf0); free(htextb); free(sadb);
}

/* [OpenCV] validateDisparity with an int cost map, restricted to rows [r0,r1) */
static void bm_validate(int16_t* disp, ptrdiff_t ds, const int* cost, int W, int r0, int r1,
                        int minD, int ndisp, int disp12MaxDiff)
{
    int maxD = minD + ndisp;
    int minX1 = imax(maxD, 0), maxX1 = W + imin(minD, 0);
    int INV = (minD - 1) * DISP_SCALE;
    int* d2 = (int*)malloc(sizeof(int) * W);
    int* c2 = (int*)malloc(sizeof(int) * W);
    disp12MaxDiff *= DISP_SCALE;
    for (int y = r0; y < r1; y++) {
        int16_t* dp = disp + (ptrdiff_t)y * ds;
        const int* cp = cost + (size_t)y * W;
        for (int x = 0; x < W; x++) { d2[x] = INV; c2[x] = INT_MAX; }
        for (int x = minX1; x < maxX1; x++) {
            int d = dp[x], c = cp[x];
            if (d == INV) continue;
            int x2 = x - ((d + DISP_SCALE / 2) >> DISP_SHIFT);
            if (x2 >= 0 && x2 < W && c2[x2] > c) { c2[x2] = c; d2[x2] = d; }
        }
        for (int x = minX1; x < maxX1; x++) {
            int d = dp[x];
            if (d == INV) continue;
            int dl = d >> DISP_SHIFT, dh = (d + DISP_SCALE - 1) >> DISP_SHIFT;
            int xl = x - dl, xh = x - dh;
            if ((0 <= xl && xl < W && d2[xl] > INV && iabs(d2[xl] - d) > disp12MaxDiff) &&
                (0 <= xh && xh < W && d2[xh] > INV && iabs(d2[xh] - d) > disp12MaxDiff))
                dp[x] = (int16_t)INV;
        }
    }
    free(d2); free(c2);
}

int orc_bm_compute(const uint8_t* L, ptrdiff_t ls, const uint8_t* R, ptrdiff_t rs, int W,
                   int H, const orc_bm_params* p, int16_t* out, ptrdiff_t os)
{
    if (!L || !R || !out || !p || W <= 0 || H <= 0) return -1;
    if (p->pre_filter_type != 0 && p->pre_filter_type != 1) return -2;
    if (p->pre_filter_size < 5 || p->pre_filter_size > 255 || p->pre_filter_size % 2 == 0) return -2;
    if (p->pre_filter_cap < 1 || p->pre_filter_cap > 63) return -2;
    if (p->block_size < 5 || p->block_size > 255 || p->block_size % 2 == 0 ||
        p->block_size >= imin(W, H))
        return -2;
    if (p->num_disparities <= 0 || p->num_disparities % 16 != 0) return -2;
    if (p->texture_threshold < 0 || p->uniqueness_ratio < 0) return -2;

    const int ndisp = p->num_disparities, mindisp = p->min_disparity;
    const int16_t FILTERED = (int16_t)((mindisp - 1) * (1 << DISP_SHIFT));  /* no UB shift of a negative value */
    int lofs = imax(ndisp - 1 + mindisp, 0), rofs = -imin(ndisp - 1 + mindisp, 0);
    int width1 = W - rofs - ndisp + 1;
    if (lofs >= W || rofs >= W || width1 < 1) {
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) out[(ptrdiff_t)y * os + x] = FILTERED;
        return 0;
    }
    uint8_t* Lf = (uint8_t*)malloc((size_t)W * H);
    uint8_t* Rf = (uint8_t*)malloc((size_t)W * H);
    if (p->pre_filter_type == 0) {
        prefilter_norm(L, ls, W, H, p->pre_filter_size, p->pre_filter_cap, Lf);
        prefilter_norm(R, rs, W, H, p->pre_filter_size, p->pre_filter_cap, Rf);
    } else {
        orc_prefilter_xsobel(L, ls, W, H, p->pre_filter_cap, Lf);
        orc_prefilter_xsobel(R, rs, W, H, p->pre_filter_cap, Rf);
    }
    /* getValidDisparityROI with empty roi1/roi2 */
    int SW2 = p->block_size / 2;
    int maxDm1 = mindisp + ndisp - 1;
    int xmin = imax(0, maxDm1) + SW2, xmax = W - SW2, ymin = SW2, ymax = H - SW2;
    int vw = xmax - xmin, vh = ymax - ymin;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) out[(ptrdiff_t)y * os + x] = FILTERED;
    if (vw > 0 && vh > 0) {
        int* cost = p->disp12_max_diff >= 0 ? (int*)calloc((size_t)W * H, sizeof(int)) : NULL;
        bm_stripe(Lf, Rf, W, H, ymin, ymax, p, out, os, cost);
        if (cost) {
            bm_validate(out, os, cost, W, ymin, ymax, mindisp, ndisp, p->disp12_max_diff);
            free(cost);
        }
        for (int y = ymin; y < ymax; y++) {
            int16_t* dr = out + (ptrdiff_t)y * os;
            for (int x = 0; x < xmin; x++) dr[x] = FILTERED;
            for (int x = xmax; x < W; x++) dr[x] = FILTERED;
        }
    }
    free(Lf);
    free(Rf);
    if (p->speckle_range >= 0 && p->speckle_window_size > 0)
        return orc_filter_speckles_s16(out, os, W, H, FILTERED, p->speckle_window_size,
                                       p->speckle_range);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* MeanDisparityDetection::build(MEAN_VALUE)                                 */
/* ------------------------------------------------------------------------ */
void orc_mean_disparity_grid(const int16_t* dmap, ptrdiff_t st, int W, int H, float* means)
{
    int dx = W / 9, dy = H / 9;
    for (int r = 0; r < 9; r++)
        for (int c = 0; c < 9; c++) {
            int total = 0, n = 0;
            for (int y = r * dy; y < r * dy + dy; y++)
                for (int x = c * dx; x < c * dx + dx; x++) {
                    int v = dmap[(ptrdiff_t)y * st + x];
                    if (v > 1) { total += v; n++; }
                }
            means[r * 9 + c] = (total == 0 || n == 0) ? 0.0f : (float)(total / iabs(n));
        }
}

/* [Utility::calcCoordinate] src/utility.cpp:176-198, applied per pixel as in
 * Utility::dmap2pcl src/utility.cpp:242-262 */
void orc_reproject(const int16_t* dmap, ptrdiff_t st, int W, int H, const float* Q, float* out)
{
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float v = (float)dmap[(ptrdiff_t)y * st + x];
            float c[4] = {(float)x, (float)y, v / 16, 1.0f};
            float r[4];
            for (int i = 0; i < 4; i++) {
                double acc = 0.0;
                for (int k = 0; k < 4; k++) acc += (double)Q[4 * i + k] * (double)c[k];
                r[i] = (float)acc;
            }
            float alpha = (float)(1.0 / (double)r[3]);
            float* o = out + ((size_t)y * W + x) * 4;
            o[0] = r[0] * alpha;
            o[1] = r[1] * alpha;
            o[2] = r[2] * alpha;
            if (isinf(o[2] / 1000)) o[2] = 0.0f;
            o[3] = v > 0 ? 1.0f : 0.0f;
        }
}

/* [OpenCV 3.4 imgproc/src/imgwarp.cpp] RemapInvoker (CV_32FC1 maps -> fixed point:
 * X = saturate_cast<int>(mapx * INTER_TAB_SIZE), XY = X >> INTER_BITS, A = low bits)
 * and remapBilinear<FixedPtCast<int, uchar, 15>> with initInterTab2D's integer
 * bilinear table (exact for INTER_LINEAR: weights * 32768 are integers). */
static int orc_round_f(float v)
{
    if (v != v) return INT_MIN;
    if (v >= 2147483648.0f) return INT_MAX;
    if (v < -2147483648.0f) return INT_MIN;
    return (int)lrintf(v); /* cvRound: round half to even */
}

void orc_remap_linear(const uint8_t* src, ptrdiff_t ss, int sw, int sh, const float* mapx,
                      const float* mapy, uint8_t* dst, int dw, int dh)
{
    for (int y = 0; y < dh; y++)
        for (int x = 0; x < dw; x++) {
            int X = orc_round_f(mapx[(size_t)y * dw + x] * 32);
            int Y = orc_round_f(mapy[(size_t)y * dw + x] * 32);
            int sx = X >> 5, sy = Y >> 5;
            if (sx < -32768) sx = -32768;
            if (sx > 32767) sx = 32767;
            if (sy < -32768) sy = -32768;
            if (sy > 32767) sy = 32767;
            int ax = X & 31, ay = Y & 31;
            int v;
            if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
                v = 0;
            } else {
                int w[4] = {(32 - ay) * (32 - ax) * 32, (32 - ay) * ax * 32, ay * (32 - ax) * 32,
                            ay * ax * 32};
                int xs[4] = {sx, sx + 1, sx, sx + 1}, ys[4] = {sy, sy, sy + 1, sy + 1};
                int acc = 0;
                for (int t = 0; t < 4; t++) {
                    int inside = xs[t] >= 0 && xs[t] < sw && ys[t] >= 0 && ys[t] < sh;
                    acc += (inside ? src[(ptrdiff_t)ys[t] * ss + xs[t]] : 0) * w[t];
                }
                v = (acc + (1 << 14)) >> 15;
                if (v < 0) v = 0;
                if (v > 255) v = 255;
            }
            dst[(size_t)y * dw + x] = (uint8_t)v;
        }
}

/* [OpenCV 3.4 imgproc/src/resize.cpp] cv::resize(src, dst, Size(0, 0), fx, fy,
 * INTER_LINEAR) for CV_8UC1 -- the resize of Stereosystem::getRectifiedImagepair
 * (Stereopair&, float) (src/Stereosystem.cpp:279-315).  TEST INFRASTRUCTURE.
 *   dsize = (saturate_cast<int>(sw * fx), saturate_cast<int>(sh * fy)) (cvRound);
 *   scale = 1 / inv_scale; a scale of exactly 2 x 2 runs INTER_AREA's fast path
 *   (resizeAreaFast_: (a + b + c + d + 2) >> 2 over full 2x2 blocks -- the SIMD
 *   op and its scalar tail agree -- and a float mean rounded half to even over
 *   the clipped blocks of an odd edge);
 *   otherwise resizeGeneric_ with HResizeLinear (exact integer taps, 11-bit
 *   coefficients saturate_cast<short>(cbuf * 2048), x clamped with fx = 0) and
 *   VResizeLinear<.., FixedPtCast<int, uchar, 22>>: the CV_SIMD128 op
 *   (VResizeLinearVec_32s8u) covers x < width - 8 (16- and 8-wide loops) with
 *   16-bit arithmetic -- s = (S >> 4) per row, mulhi by beta, saturating add,
 *   (+2) >> 2 -- and the scalar tail x >= width - 8 rounds (sum + 2^21) >> 22.
 *   Rows clamp to [0, sh - 1] (beta from the unclamped fy). */
static int orc_round_d(double v) { return (int)lrint(v); }

void orc_resize_linear(const uint8_t* src, ptrdiff_t ss, int sw, int sh, double fx, double fy,
                       uint8_t* dst, ptrdiff_t ds, int* out_w, int* out_h)
{
    const int dw = orc_round_d(sw * fx), dh = orc_round_d(sh * fy);
    *out_w = dw;
    *out_h = dh;
    if (!dst) return;
    if (dw == sw && dh == sh) { /* dsize == ssize: src.copyTo(dst) */
        for (int y = 0; y < sh; y++) memcpy(dst + (ptrdiff_t)y * ds, src + (ptrdiff_t)y * ss, (size_t)sw);
        return;
    }
    const double scale_x = 1.0 / fx, scale_y = 1.0 / fy;
    const int isx = orc_round_d(scale_x), isy = orc_round_d(scale_y);
    const int area_fast = fabs(scale_x - isx) < DBL_EPSILON && fabs(scale_y - isy) < DBL_EPSILON;
    if (area_fast && isx == 2 && isy == 2) {
        const int w1 = sw / 2;
        for (int dy = 0; dy < dh; dy++) {
            uint8_t* D = dst + (ptrdiff_t)dy * ds;
            const int sy0 = dy * 2;
            if (sy0 >= sh) {
                for (int dx = 0; dx < dw; dx++) D[dx] = 0;
                continue;
            }
            const int w = sy0 + 2 <= sh ? w1 : 0;
            const uint8_t* S0 = src + (ptrdiff_t)sy0 * ss;
            int dx = 0;
            for (; dx < w; dx++) {
                const int i = 2 * dx;
                D[dx] = (uint8_t)((S0[i] + S0[i + 1] + S0[ss + i] + S0[ss + i + 1] + 2) >> 2);
            }
            for (; dx < dw; dx++) {
                int sum = 0, count = 0;
                const int sx0 = 2 * dx;
                if (sx0 >= sw) {
                    D[dx] = 0;
                    continue;
                }
                for (int sy = 0; sy < 2 && sy0 + sy < sh; sy++)
                    for (int sx = 0; sx < 2 && sx0 + sx < sw; sx++) {
                        sum += src[(ptrdiff_t)(sy0 + sy) * ss + sx0 + sx];
                        count++;
                    }
                int v = (int)lrintf((float)sum / (float)count);
                D[dx] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
            }
        }
        return;
    }
    int* xofs = (int*)malloc(sizeof(int) * (size_t)dw);
    short* ialpha = (short*)malloc(sizeof(short) * 2 * (size_t)dw);
    int* rows = (int*)malloc(sizeof(int) * 2 * (size_t)dw);
    for (int dx = 0; dx < dw; dx++) {
        float f = (float)((dx + 0.5) * scale_x - 0.5);
        int sx = (int)floorf(f);
        f -= (float)sx;
        if (sx < 0) f = 0.f, sx = 0;
        if (sx >= sw - 1) f = 0.f, sx = sw - 1;
        xofs[dx] = sx;
        ialpha[2 * dx] = (short)lrintf((1.f - f) * 2048.f);
        ialpha[2 * dx + 1] = (short)lrintf(f * 2048.f);
    }
    for (int dy = 0; dy < dh; dy++) {
        float f = (float)((dy + 0.5) * scale_y - 0.5);
        const int sy = (int)floorf(f);
        f -= (float)sy;
        const int b0 = (short)lrintf((1.f - f) * 2048.f), b1 = (short)lrintf(f * 2048.f);
        for (int k = 0; k < 2; k++) {
            int r = sy + k;
            r = r < 0 ? 0 : r >= sh ? sh - 1 : r;
            const uint8_t* S = src + (ptrdiff_t)r * ss;
            int* o = rows + (size_t)k * dw;
            for (int dx = 0; dx < dw; dx++) {
                const int sx = xofs[dx];
                const int a1 = ialpha[2 * dx + 1];
                o[dx] = S[sx] * ialpha[2 * dx] + (a1 ? S[sx + 1] * a1 : 0);
            }
        }
        uint8_t* D = dst + (ptrdiff_t)dy * ds;
        /* columns the SIMD op covers: its 16-wide loop (x <= width - 16), then
         * its 8-wide loop (x < width - 8) */
        int simd_end = 0;
        while (simd_end <= dw - 16) simd_end += 16;
        while (simd_end < dw - 8) simd_end += 8;
        for (int x = 0; x < dw; x++) {
            const int s0 = rows[x], s1 = rows[dw + x];
            int v;
            if (x < simd_end) {
                int h0 = s0 >> 4, h1 = s1 >> 4;
                h0 = h0 > 32767 ? 32767 : h0 < -32768 ? -32768 : h0;
                h1 = h1 > 32767 ? 32767 : h1 < -32768 ? -32768 : h1;
                int r = ((h0 * b0) >> 16) + ((h1 * b1) >> 16);
                r = r > 32767 ? 32767 : r < -32768 ? -32768 : r;
                r += 2;
                r = r > 32767 ? 32767 : r;
                v = r >> 2;
            } else {
                v = (s0 * b0 + s1 * b1 + (1 << 21)) >> 22;
            }
            D[x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
        }
    }
    free(xofs);
    free(ialpha);
    free(rows);
}
