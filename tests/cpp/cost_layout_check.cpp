// cost_layout_check.cpp — exhaustive bounds check of the register-ring cost
// kernel's addresses (sgbm_cost2_kernel, mvsv_sgbm.hip) on the host.
//
// The kernel takes its tile geometry, global staging offsets and LDS slots from
// mvsv_cost_layout.hpp; this program runs the same functions for every tile,
// thread and staging item of every shape the launcher (launch_cost) can pick,
// and checks:
//   * the staging loads (issued by every thread, even for unused items) stay
//     inside the frame's two BT-interval planes, i.e. inside ctx->pre;
//   * the LDS stores / loads of the staging, pixel-cost and window phases stay
//     inside the launch's dynamic LDS (lay.bytes <= 160 KiB);
//   * the cost stores stay inside the frame's [H][W1][D] slab of ctx->cost.
// Prints the extreme addresses of the shape of the recorded round-1 fault
// (D = 64, blockSize 13, minD 1, 360 x 80, MODE_SGBM) and exits 1 on a violation.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <iterator>
#include <vector>

#include "../../mvstereovision3_amd/csrc/mvsv_cost_layout.hpp"

using namespace mvsv;

struct Stats {
    long long gmin = 1LL << 62, gmax = -1, cmin = 1LL << 62, cmax = -1, lmax = -1;
    long long violations = 0;
};

// Mirrors launch_cost's choice: the register-ring kernel when SW2 = SH2 <= 7,
// the staging items fit two per thread and the LDS image fits 160 KiB.
static bool cost2_selected(int D, int SW2, int TY)
{
    const Cost2Layout l = cost2_layout(D, SW2, TY);
    const int items = 2 * l.NX + D - 1;
    return SW2 <= 7 && l.CL >= 1 && items <= kCost2Threads * 2 && l.bytes <= 160 * 1024;
}

static void check_shape(int D, int SW2, int TY, int W, int H, int minD, int n, Stats& st,
                        bool verbose)
{
    const int maxD = minD + D;
    const int minX1 = std::max(maxD, 0);
    const int W1 = W + std::min(minD, 0) - minX1;
    if (W1 <= SW2) return;  // resolve_sgbm rejects these
    const Cost2Layout lay = cost2_layout(D, SW2, TY);
    const int PP = lay.PP, CL = lay.CL, TX = lay.TX, NX = lay.NX, NR = 2 * SW2 + 1, SH2 = SW2;
    const int STG = 2 * lay.NX + D - 1 > kCost2Threads ? 2 : 1;
    const long long plane = (long long)W * H;
    const long long pre_elems = (long long)n * 2 * plane;      // u64 elements of ctx->pre
    const long long c_dwords = (long long)n * H * W1 * PP;       // int16 pairs of ctx->cost
    auto viol = [&](const char* what, long long v, long long lim) {
        if (st.violations < 10)
            std::fprintf(stderr, "VIOLATION %s: %lld not in [0,%lld)  D=%d SW2=%d TY=%d W=%d H=%d minD=%d\n",
                         what, v, lim, D, SW2, TY, W, H, minD);
        st.violations++;
    };
    const int gx = (W1 + TX - 1) / TX, gy = (H + TY - 1) / TY;
    // every column tile; the row tiles and frames at the extremes (the staging
    // offsets do not depend on the row tile: rows are clamped into [0, H-1];
    // the cost stores are affine in the row tile and the frame)
    for (int f : {0, n - 1})
        for (int by : {0, gy - 1})
            for (int bx = 0; bx < gx; bx++) {
                const Cost2Tile t = cost2_tile(TX, TY, SW2, bx, by, W1, H, minX1, minD, D);
                // staging loads: rows clamped to [0, H-1], every thread and item
                for (int tid = 0; tid < kCost2Threads; tid++)
                    for (int k = 0; k < STG; k++) {
                        const int i = kCost2Threads - 1 - tid + kCost2Threads * k;
                        const Cost2Item it = cost2_item(t, i, W, (int)plane);
                        for (int r : {0, H - 1})
                            for (int o : {it.oa, it.ob}) {
                                const long long g = (long long)f * 2 * plane + (long long)r * W + o;
                                st.gmin = std::min(st.gmin, g);
                                st.gmax = std::max(st.gmax, g);
                                if (g < 0 || g >= pre_elems) viol("staging load", g, pre_elems);
                            }
                        // staging LDS stores
                        if (i < t.nL) {
                            const long long b4 = (long long)lay.off_l4 + lay.lstride4 + 16LL * i + 15;
                            const long long b2 = (long long)lay.off_l2 + lay.lstride2 + 8LL * i + 7;
                            if (i >= NX) viol("left slot", i, NX);
                            st.lmax = std::max({st.lmax, b4, b2});
                        } else if (i < t.nItems) {
                            const int q = cost2_qslot(lay, i - t.nL);
                            if (q < 0 || q >= 2 * lay.qhalf) viol("right slot", q, 2 * lay.qhalf);
                            st.lmax = std::max(st.lmax, (long long)lay.off_q2 + (long long)lay.qstride2 + 8LL * q + 7);
                        }
                    }
                // pixel-cost phase: LDS operand slots and pix-row stores
                for (int tid = 0; tid < kCost2Threads; tid++) {
                    const int cl = tid / PP, p = tid - cl * PP;
                    if (cl >= CL) continue;
                    for (int xv = 2 * cl; xv < NX; xv += 2 * CL) {
                        for (int dx = 0; dx < 2; dx++) {
                            const int xc = t.linear ? xv + dx
                                                    : cost2_clampi(t.x0 - SW2 + xv + dx, 0, W1 - 1) - t.xclo;
                            if (xc < 0 || xc >= t.nL) viol("pix left slot", xc, t.nL);
                            const int q = cost2_qslot(lay, t.nL - 1 - xc + 2 * p);
                            if (q < 0 || q >= 2 * lay.qhalf) viol("pix right slot", q, 2 * lay.qhalf);
                        }
                        const long long pw = (long long)p * lay.PS + xv + 1;
                        if (pw >= (long long)lay.PP * lay.PS) viol("pix store", pw, (long long)lay.PP * lay.PS);
                        st.lmax = std::max(st.lmax, (long long)lay.off_pix + (long long)lay.pstride + 4 * pw + 3);
                    }
                    // window loads of the horizontal sum
                    const int tx0 = cl * kCost2Run;
                    const long long wl = (long long)p * lay.PS + tx0 + NR + kCost2Run - 2;
                    if (wl >= (long long)lay.PP * lay.PS) viol("window load", wl, (long long)lay.PP * lay.PS);
                    // cost stores of the emitted rows
                    const int nrows = (t.y1 - t.y0) + 2 * SH2;
                    const int nout = std::min(kCost2Run, W1 - (t.x0 + tx0));
                    const long long ostride = (long long)W1 * PP;
                    const long long obase = (((long long)f * H + t.y0) * W1 + t.x0 + tx0) * PP + p -
                                            (long long)(2 * SH2) * ostride;
                    for (int kk : {NR - 1, nrows - 1}) {
                        if (kk < NR - 1 || kk >= nrows) continue;
                        for (int i = 0; i < nout; i++) {
                            const long long c = obase + (long long)kk * ostride + (long long)i * PP;
                            st.cmin = std::min(st.cmin, c);
                            st.cmax = std::max(st.cmax, c);
                            if (c < 0 || c >= c_dwords) viol("cost store", c, c_dwords);
                        }
                    }
                }
            }
    if (st.lmax >= (long long)lay.bytes) viol("LDS extent", st.lmax, (long long)lay.bytes);
    if (verbose)
        std::printf("shape D=%d bs=%d TY=%d %dx%d minD=%d n=%d: staging u64 [%lld, %lld] of %lld, "
                    "cost pairs [%lld, %lld] of %lld, LDS bytes <= %lld of %zu\n",
                    D, 2 * SW2 + 1, TY, W, H, minD, n, st.gmin, st.gmax, pre_elems, st.cmin, st.cmax,
                    c_dwords, st.lmax, lay.bytes);
}

int main()
{
    long long shapes = 0, violations = 0;
    {  // the shape of the recorded round-1 fault (test_sgbm_block_sizes[64-13])
        Stats st;
        check_shape(64, 6, 16, 360, 80, 1, 1, st, true);
        violations += st.violations;
    }
    const int widths[] = {23, 360, 641, 1280};
    const int heights[] = {1, 5, 80, 960};
    const int mins[] = {-3, 0, 1};
    // every height the launcher picks (kCostTileHeights) plus 1 (a forced
    // MVSV_COST_TY extreme)
    std::vector<int> tys(std::begin(kCostTileHeights), std::end(kCostTileHeights));
    tys.push_back(1);
    for (int D = 16; D <= 512; D += 16)
        for (int SW2 = 0; SW2 <= 7; SW2++)
            for (int TY : tys) {
                if (!cost2_selected(D, SW2, TY)) continue;
                for (int W : widths)
                    for (int H : heights)
                        for (int minD : mins) {
                            if (W > 400 && (D % 64 || SW2 % 3)) continue;  // keep it fast
                            Stats st;
                            check_shape(D, SW2, TY, W, H, minD, 2, st, false);
                            violations += st.violations;
                            shapes++;
                        }
            }
    // the register-ring kernel (and with it the bit-sliced planes and the
    // residual plane) must launch for every window of D = 128 / 256 at every
    // tile height: its LDS -- layout + the LDS ring slots -- fits a CU (a
    // shape that did not would fall back to the LDS-ring kernel silently;
    // ADVICE r05).  Mirrors launch_cost / cost2_runs in mvsv_cost.hip.
    for (int D : {128, 256})
        for (int SW2 = 0; SW2 <= 7; SW2++)
            for (int TY : tys) {
                const Cost2Layout l2 = cost2_layout(D, SW2, TY);
                const int items = 2 * l2.NX + D - 1;
                const int ppc = l2.PP == 64 ? 64 : (l2.PP == 128 ? 128 : 0);
                const size_t lbytes = cost2_total_bytes(l2, 2 * SW2 + 1, items > kCost2Threads ? 2 : 1, ppc);
                if (!(l2.CL >= 1 && items <= 2 * kCost2Threads && lbytes <= 160 * 1024)) {
                    std::printf("register-ring cost kernel does not fit: D %d blockSize %d TY %d (%zu B)\n", D,
                                2 * SW2 + 1, TY, lbytes);
                    violations++;
                }
            }
    std::printf("cost_layout_check: %lld shapes, %lld violations\n", shapes, violations);
    return violations ? 1 : 0;
}
