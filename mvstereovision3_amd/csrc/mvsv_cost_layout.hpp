// mvsv_cost_layout.hpp — tile geometry and staging address arithmetic of the
// register-ring cost-volume kernel (sgbm_cost2_kernel, mvsv_sgbm.hip).  The
// kernel computes every global staging offset and LDS slot through these
// functions, and tests/cpp/cost_layout_check.cpp runs the same functions on the
// host over every tile of every (D, blockSize, tile height, image) shape the
// launcher can pick, checking each address against its buffer's bounds.
#pragma once

#include <cstddef>

#if defined(__HIPCC__)
#define MVSV_HD __host__ __device__
#else
#define MVSV_HD
#endif

namespace mvsv {

constexpr int kCost2Threads = 512;
constexpr int kCost2Run = 4;
// tile heights sgbm_device picks from (images >= 256 rows; 16 below that);
// tests/cpp/cost_layout_check.cpp bounds-checks every one of them
constexpr int kCostTileHeights[] = {120, 96, 64, 48, 32, 24, 16};

struct Cost2Layout {
    int PP, CL, TX, TY, NX, PS, nQmax, qhalf;
    size_t off_l4, off_l2, off_q4, off_q2, off_pix, bytes;
    size_t lstride4, lstride2, qstride4, qstride2, pstride;  // bytes per buffer (x2 each)
};

// A column's BT operands for both channels are six u16-pair dwords
// {a.v, a.lo, a.hi, b.v, b.lo, b.hi}: dwords 0-3 in a 16-byte slot (ds_read_b128,
// 4 LDS cycles), dwords 4-5 in an 8-byte slot (ds_read_b64, 2 cycles).  Right
// pairs j are stored by parity so the lanes of a wave (j = t + 2p) read
// consecutive, conflict-free slots.
MVSV_HD inline Cost2Layout cost2_layout(int D, int SW2, int TY)
{
    Cost2Layout c;
    c.PP = D / 2;
    c.CL = kCost2Threads / c.PP;
    c.TX = c.CL * kCost2Run;
    c.TY = TY;
    c.NX = c.TX + 2 * SW2;  // even
    // pix row: [pair p][column], PS dwords per pair with PS/2 odd: the b64
    // column-pair stores (16-lane groups, 32 banks) and the b64 window loads
    // (32-lane groups, 64 banks) of a wave are conflict-free
    c.PS = c.NX + ((2 - c.NX) % 4 + 4) % 4;
    c.nQmax = c.NX + D - 1;
    c.qhalf = (c.nQmax + 1) / 2;  // slots per parity half
    c.lstride4 = (size_t)c.NX * 16;
    c.lstride2 = (size_t)c.NX * 8;
    c.qstride4 = (size_t)2 * c.qhalf * 16;
    c.qstride2 = (size_t)2 * c.qhalf * 8;
    c.pstride = (size_t)c.PS * c.PP * 4;
#if MVSV_COST2_ONE_STRIDE
    // both double buffers as one block each: every region of buffer 1 sits one
    // buffer stride BS after buffer 0's (one select per row instead of five)
    c.off_l4 = 0;
    c.off_q4 = c.off_l4 + c.lstride4;
    c.off_l2 = c.off_q4 + c.qstride4;
    c.off_q2 = c.off_l2 + c.lstride2;
    c.off_pix = (c.off_q2 + c.qstride2 + 15) & ~(size_t)15;
    const size_t BS = (c.off_pix + c.pstride + 15) & ~(size_t)15;
    c.lstride4 = c.lstride2 = c.qstride4 = c.qstride2 = c.pstride = BS;
    c.bytes = 2 * BS;
#else
    c.off_l4 = 0;
    c.off_q4 = c.off_l4 + 2 * c.lstride4;
    c.off_l2 = c.off_q4 + 2 * c.qstride4;
    c.off_q2 = c.off_l2 + 2 * c.lstride2;
    c.off_pix = ((c.off_q2 + 2 * c.qstride2) + 15) & ~(size_t)15;
    c.bytes = c.off_pix + 2 * c.pstride;
#endif
    return c;
}

// Ring slots of the vertical window kept in LDS instead of registers (slots
// RR .. NR - 1, RR = NR - this; one uint4 per thread and slot after the
// layout's buffers).  Large windows of the D = 128 / 256 kernels otherwise
// exceed 128 VGPRs (4 waves per SIMD) and the compiler spills ring slots to
// scratch, whose evicted lines reach HBM (tools/kernel_resources.py audits it).
MVSV_HD constexpr int cost2_lds_ring_slots(int nr, int stg, int ppc)
{
    // (register slots 8 for D = 128 up to blockSize 13, 10 at 15 so that two
    // blocks still fit a CU's LDS; 12 for D = 256 -- tools/kernel_resources.py)
    return stg != 1 ? 0
           : ppc == 64  ? (nr > 13 ? nr - 10 : nr > 8 ? nr - 8 : 0)
           : ppc == 128 ? (nr > 12 ? nr - 12 : 0)
                        : 0;
}
MVSV_HD inline size_t cost2_ring_offset(const Cost2Layout& l) { return (l.bytes + 15) & ~(size_t)15; }
MVSV_HD inline size_t cost2_total_bytes(const Cost2Layout& l, int nr, int stg, int ppc)
{
    return cost2_ring_offset(l) + (size_t)cost2_lds_ring_slots(nr, stg, ppc) * kCost2Threads * 16;
}

MVSV_HD inline int cost2_clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// One TX x TY tile of cost columns [x0, x0+TX) x rows [y0, y1): the left image
// columns it stages (with the SW2 halo, clamped to the cost space) and the
// reversed right columns (rtop - j) of its disparity range.
struct Cost2Tile {
    int x0, y0, y1, xclo, xchi, nL, nQ, nItems, ilo, rtop;
    bool linear;  // no clamped column in the tile's window
};

MVSV_HD inline Cost2Tile cost2_tile(int TX, int TY, int SW2, int bx, int by, int W1, int H,
                                    int minX1, int minD, int D)
{
    Cost2Tile t;
    t.x0 = bx * TX;
    t.y0 = by * TY;
    t.y1 = t.y0 + TY < H ? t.y0 + TY : H;
    t.xclo = t.x0 - SW2 > 0 ? t.x0 - SW2 : 0;
    t.xchi = t.x0 + TX + SW2 - 1 < W1 - 1 ? t.x0 + TX + SW2 - 1 : W1 - 1;
    t.nL = t.xchi - t.xclo + 1;
    t.nQ = t.nL + D - 1;
    t.nItems = t.nL + t.nQ;
    t.ilo = minX1 + t.xclo;
    t.rtop = minX1 + t.xchi - minD;
    t.linear = t.x0 - SW2 >= 0 && t.x0 + TX + SW2 <= W1;
    return t;
}

// Staging item i of a tile: item i < nL is left column ilo + i; else right pair
// j = i - nL (reversed columns rtop - j and rtop - j - 1, zero outside the
// image).  oa / ob: element offsets of the two loaded columns from the start
// of the staged row in the LEFT plane (the right plane follows at + plane),
// always clamped into the row; ma / mb: the loaded values are used.
struct Cost2Item {
    int oa, ob;
    bool ma, mb, left;
};

MVSV_HD inline Cost2Item cost2_item(const Cost2Tile& t, int i, int W, int plane)
{
    Cost2Item it;
    it.left = i < t.nL;
    const int xa = it.left ? t.ilo + i : t.rtop - (i - t.nL);
    const int xb = xa - 1;
    it.ma = i < t.nItems && xa >= 0 && xa < W;
    it.mb = !it.left && i < t.nItems && xb >= 0 && xb < W;
    const int pofs = it.left ? 0 : plane;
    it.oa = pofs + cost2_clampi(xa, 0, W - 1);
    it.ob = pofs + cost2_clampi(xb, 0, W - 1);
    return it;
}

// LDS slot of right pair j (both parity halves descend with j)
MVSV_HD inline int cost2_qslot(const Cost2Layout& l, int j) { return (j & 1) * l.qhalf + l.qhalf - 1 - (j >> 1); }

}  // namespace mvsv
