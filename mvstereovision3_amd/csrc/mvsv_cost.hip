// mvsv_cost.hip — StereoSGBM prefilter and cost volume on MI355X (gfx950).
//
// Stages 1-3 of the SGBM pipeline (mvsv_sgbm.hip drives them): the clipped
// x-Sobel + raw BT interval planes, the Birchfield-Tomasi pixel cost summed over
// the blockSize x blockSize window (OpenCV 3.4 computeDisparitySGBM / calcPixelCostBT,
// reached through Disparity::sgbm, /root/reference/src/disparity.cpp:6-10; SURVEY
// Appendix A.3), the cost residual / bit-sliced C' emission of the later
// stages, and OpenCV 3.4's cost-row quirks.  Its own translation unit so the
// cost kernels rebuild without the path kernels.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "mvsv_cost_layout.hpp"
#include "mvsv_device.hpp"
#include "mvsv_bitslice.hpp"
#include "mvsv_internal.hpp"

#ifndef MVSV_COST2_FETCH_DEPTH
#define MVSV_COST2_FETCH_DEPTH 1  // staged rows in flight in the cost kernel (A/B knob)
#endif

namespace mvsv {
namespace {

using namespace dev;

// ---------------------------------------------------------------------------
// 1. prefilter: per pixel one u64 = BT interval of the clipped x-Sobel channel
//    (bits 0-23: val | lo << 8 | hi << 16) and of the raw channel (bits
//    32-55), planes [frame][2][H][W] (left, right).
// [OpenCV] calcPixelCostBT: tab[(r[x+1]-r[x-1])*2 + rn[x+1]-rn[x-1] + rs[x+1]-rs[x-1]],
// columns 0 and W-1 of both channels = tab[0] = ftzero; the BT interval of a
// value v is min/max of {v, (v + left)/2, (v + right)/2} inside the row.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bt_interval(int v, int l, int r, bool has_l, bool has_r)
{
    int a = has_l ? (v + l) >> 1 : v;
    int b = has_r ? (v + r) >> 1 : v;
    int lo = min(min(a, b), v), hi = max(max(a, b), v);
    return (uint32_t)v | ((uint32_t)lo << 8) | ((uint32_t)hi << 16);
}

__global__ __launch_bounds__(256) void sgbm_prefilter_kernel(
    const uint8_t* __restrict__ L, size_t ls, size_t lfs, const uint8_t* __restrict__ R,
    size_t rs, size_t rfs, int W, int H, int ftzero, uint64_t* __restrict__ pre)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint8_t* ch = smem;  // [4][W]: L sobel, L raw, R sobel, R raw
    const int y = blockIdx.x;
    const int img = blockIdx.y;  // 0 = left, 1 = right
    const int f = blockIdx.z;
    const uint8_t* base = img == 0 ? L + f * lfs : R + f * rfs;
    const size_t st = img == 0 ? ls : rs;
    const int yn = y > 0 ? y - 1 : y, ys = y < H - 1 ? y + 1 : y;
    const uint8_t* r0 = base + (size_t)y * st;
    const uint8_t* rn = base + (size_t)yn * st;
    const uint8_t* rsr = base + (size_t)ys * st;
    const uint8_t fz = (uint8_t)ftzero;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        uint8_t a = fz, b = fz;
        if (x > 0 && x < W - 1) {
            int g = (r0[x + 1] - r0[x - 1]) * 2 + rn[x + 1] - rn[x - 1] + rsr[x + 1] - rsr[x - 1];
            a = (uint8_t)(clampi(g, -ftzero, ftzero) + ftzero);
            b = r0[x];
        }
        ch[x] = a;
        ch[W + x] = b;
    }
    __syncthreads();
    uint64_t* o = pre + (((size_t)f * 2 + img) * H + y) * W;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        const bool hl = x > 0, hr = x < W - 1;
        const int xl = hl ? x - 1 : x, xr = hr ? x + 1 : x;
        uint32_t s0 = bt_interval(ch[x], ch[xl], ch[xr], hl, hr);
        uint32_t s1 = bt_interval(ch[W + x], ch[W + xl], ch[W + xr], hl, hr);
        o[x] = (uint64_t)s0 | ((uint64_t)s1 << 32);
    }
}

// ---------------------------------------------------------------------------
// 2. cost volume.
// Block = 256 threads owns cost columns [x0, x0+TX) x rows [y0, y0+TY) x all d.
// Thread (cl, p) works on the disparity pair (2p, 2p+1) packed in one VGPR
// (v_pk_*_u16) and on column lane cl.  For each clamped source row:
//   stage  BT intervals of the needed left columns and (x-reversed, twice,
//          with a one-column shift so every pair is one aligned 16-byte LDS
//          read) right columns in LDS;
//   pix    Birchfield-Tomasi cost of TX + 2*SW2 columns, two disparities per
//          instruction (bytes -> u16 halves with v_perm_b32);
//   hsum   horizontal box sum, sliding along the thread's run of RUN columns;
//   vsum   vertical window sum kept in registers, the last 2*SH2+1 horizontal
//          sums in an LDS ring; emit C = P2 + window sum (u16 wrap = int16 cast).
// ---------------------------------------------------------------------------
constexpr int kCostRun = 4;  // output columns per thread

struct CostLayout {
    int PP, CL, TX, TY, NX, NR, nLmax, nRmax;
    size_t off_ra, off_rb, off_pix, off_ring, bytes;
};

__host__ __device__ inline CostLayout cost_layout(int D, int SW2, int SH2, int TY)
{
    CostLayout c;
    c.PP = D / 2;
    c.CL = 256 / c.PP;
    if (c.CL < 1) c.CL = 1;
    c.TX = c.CL * kCostRun;
    c.TY = TY;
    c.NX = c.TX + 2 * SW2;
    c.NR = 2 * SH2 + 1;
    c.nLmax = c.NX;
    c.nRmax = c.NX + D + 2;
    c.off_ra = ((size_t)c.nLmax * 8 + 15) & ~(size_t)15;
    c.off_rb = c.off_ra + (((size_t)c.nRmax * 8 + 15) & ~(size_t)15);
    c.off_pix = c.off_rb + (((size_t)c.nRmax * 8 + 15) & ~(size_t)15);
    c.off_ring = c.off_pix + (((size_t)c.NX * c.PP * 4 + 15) & ~(size_t)15);
    c.bytes = c.off_ring + (size_t)c.NR * c.TX * c.PP * 4;
    return c;
}
// ---------------------------------------------------------------------------
// Residual cost plane R (the "cost residual"): for every pixel p and disparity
//     R(p, d) = min(C(p, d) - min_k C(p, k), 2*P2) + P2        in [P2, 3*P2]
// stored as nibbles (byte k of a pixel = R(2k) | R(2k+1) << 4; 3*P2 <= 15).
// Why the direction passes may read R instead of C (exactly, bit for bit):
//  * offset: a path step subtracts min_k L(prev, k) and only uses
//    L(prev, .) - min L(prev, .), so adding a constant to C(p, .) for all d
//    changes no path delta (and every L stays an exact non-negative int16 in
//    the no-wrap regime the launcher requires, sgbm_no_wrap);
//  * clamp: a step only sees min(L(prev, d) - min L(prev, .), P2) (the P2
//    candidate caps every term), and with C' = C - min_k C, min L(prev, .) <=
//    P2 (the d with C' = 0 has L <= C' + P2), so any C'(d) >= 2*P2 gives
//    L(d) - min L >= P2 whatever its exact value -- and never attains min L.
// The path-delta planes computed from R are therefore identical to those from
// C; the final kernel (WTA, uniqueness ratio, sub-pixel fit) still reads C.
// ---------------------------------------------------------------------------

// BT cost of one channel for a disparity pair: u* broadcast, v* per half.
// The distance of u to the interval [v0, v1] is max(u - v1, v0 - u, 0); with
// v0 <= v1 at most one of the two saturated differences is non-zero, so their
// sum (bytes: no half carries -- a full-rate 32-bit add) is that maximum.
__device__ __forceinline__ uint32_t bt_pair(uint32_t u, uint32_t u0, uint32_t u1, uint32_t v,
                                           uint32_t v0, uint32_t v1)
{
    uint32_t c0 = add2_nc(pk_subsat_u16(u, v1), pk_subsat_u16(v0, u));
    uint32_t c1 = add2_nc(pk_subsat_u16(v, u1), pk_subsat_u16(u0, v));
    return pk_min_u16(c0, c1);
}

constexpr int kStageRegs = 3;  // staging loads per thread per row (nL + nR + 1 <= 768)

__global__ __launch_bounds__(256) void sgbm_cost_kernel(const uint64_t* __restrict__ pre, int W,
                                                        int H, SgbmEff e, int TY,
                                                        int16_t* __restrict__ C)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int D = e.D, W1 = e.W1, SW2 = e.SW2, SH2 = e.SH2;
    const CostLayout lay = cost_layout(D, SW2, SH2, TY);
    const int PP = lay.PP, CL = lay.CL, TX = lay.TX, NX = lay.NX, NR = lay.NR;
    const int f = blockIdx.z;
    const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
    const int y1 = min(y0 + TY, H);
    const int xclo = max(x0 - SW2, 0), xchi = min(x0 + TX + SW2 - 1, W1 - 1);
    const int nL = xchi - xclo + 1;
    const int ilo = e.minX1 + xclo;  // first left image column
    // right columns, x-reversed: j = rtop - xr, rtop = right column of d = 0 at xc = xchi
    const int rtop = e.minX1 + xchi - e.minD;
    const int nR = nL + D;  // covers j in [0, nL - 1 + D - 1] (+1 slack for copy B)
    uint64_t* lpk = (uint64_t*)smem;
    uint64_t* ra = (uint64_t*)(smem + lay.off_ra);
    uint64_t* rb = (uint64_t*)(smem + lay.off_rb);
    uint32_t* pixrow = (uint32_t*)(smem + lay.off_pix);
    uint32_t* ring = (uint32_t*)(smem + lay.off_ring);
    const size_t plane = (size_t)W * H;
    const uint64_t* PL = pre + (size_t)f * 2 * plane;
    const uint64_t* PR = PL + plane;
    const int tid = threadIdx.x;
    const int cl = tid / PP, p = tid - (tid / PP) * PP;
    const bool worker = cl < CL;
    const int tx0 = cl * kCostRun;
    const uint32_t p2x2 = (uint32_t)(e.P2 & 0xffff) * 0x10001u;
    // staging item i: i < nL -> left column ilo + i; else right j = i - nL (0..nR)
    const int nItems = nL + nR + 1;

    uint32_t csum[kCostRun];
#pragma unroll
    for (int i = 0; i < kCostRun; i++) csum[i] = 0;
    uint64_t pf[kStageRegs];

    auto fetch_row = [&](int v) {
        const int r = clampi(v, 0, H - 1);
        const uint64_t* lrow = PL + (size_t)r * W;
        const uint64_t* rrow = PR + (size_t)r * W;
#pragma unroll
        for (int k = 0; k < kStageRegs; k++) {
            const int i = tid + 256 * k;
            uint64_t val = 0;
            if (i < nL) {
                val = lrow[ilo + i];
            } else if (i < nItems) {
                const int x = rtop - (i - nL);
                if (x >= 0 && x < W) val = rrow[x];
            }
            pf[k] = val;
        }
    };
    auto stage_row = [&]() {
#pragma unroll
        for (int k = 0; k < kStageRegs; k++) {
            const int i = tid + 256 * k;
            if (i < nL) {
                lpk[i] = pf[k];
            } else if (i < nItems) {
                const int j = i - nL;
                if (j < nR) ra[j] = pf[k];
                if (j > 0) rb[j - 1] = pf[k];
            }
        }
    };

    const int vstart = y0 - SH2, vend = y1 + SH2;
    fetch_row(vstart);
    stage_row();
    for (int v = vstart; v < vend; v++) {
        __syncthreads();  // staging of row v visible; hsum of row v-1 done with pixrow
        if (v + 1 < vend) fetch_row(v + 1);  // in flight during the pixel-cost phase
        if (worker) {
            for (int xv = cl; xv < NX; xv += CL) {
                const int xc = clampi(x0 - SW2 + xv, 0, W1 - 1);
                const uint64_t lw = lpk[xc - xclo];
                const uint32_t l0 = (uint32_t)lw, l1 = (uint32_t)(lw >> 32);
                // j of d = 2p at this column
                const int j0 = (xchi - xc) + 2 * p;
                const uint64_t* src = (j0 & 1) ? (rb + (j0 - 1)) : (ra + j0);
                const uint4 rr = *(const uint4*)src;  // cols j0, j0+1 (both channels)
                uint32_t acc;
                {
                    const uint32_t a = rr.x, b = rr.z;  // channel 0 of d, d+1
                    uint32_t U = __builtin_amdgcn_perm(l0, l0, 0x0c040c00u);
                    uint32_t U0 = __builtin_amdgcn_perm(l0, l0, 0x0c050c01u);
                    uint32_t U1 = __builtin_amdgcn_perm(l0, l0, 0x0c060c02u);
                    uint32_t V = __builtin_amdgcn_perm(b, a, 0x0c040c00u);
                    uint32_t V0 = __builtin_amdgcn_perm(b, a, 0x0c050c01u);
                    uint32_t V1 = __builtin_amdgcn_perm(b, a, 0x0c060c02u);
                    acc = bt_pair(U, U0, U1, V, V0, V1);
                }
                {
                    const uint32_t a = rr.y, b = rr.w;  // channel 1 (raw) of d, d+1
                    uint32_t U = __builtin_amdgcn_perm(l1, l1, 0x0c040c00u);
                    uint32_t U0 = __builtin_amdgcn_perm(l1, l1, 0x0c050c01u);
                    uint32_t U1 = __builtin_amdgcn_perm(l1, l1, 0x0c060c02u);
                    uint32_t V = __builtin_amdgcn_perm(b, a, 0x0c040c00u);
                    uint32_t V0 = __builtin_amdgcn_perm(b, a, 0x0c050c01u);
                    uint32_t V1 = __builtin_amdgcn_perm(b, a, 0x0c060c02u);
                    uint32_t c = bt_pair(U, U0, U1, V, V0, V1);
                    acc = pk_add_u16(acc, (c >> 2) & 0x3fff3fffu);
                }
                pixrow[xv * PP + p] = acc;
            }
        }
        __syncthreads();  // pixrow complete; staging buffers free
        if (v + 1 < vend) stage_row();
        if (worker) {
            const int k = v - vstart;
            const int slot = k % NR;
            const bool emit = k >= NR - 1;
            const int y = v - SH2;
            uint32_t h = 0;
            const uint32_t* pr = pixrow + tx0 * PP + p;
            for (int q = 0; q <= 2 * SW2; q++) h = pk_add_u16(h, pr[q * PP]);
#pragma unroll
            for (int i = 0; i < kCostRun; i++) {
                if (i > 0)
                    h = pk_sub_u16(pk_add_u16(h, pr[(i + 2 * SW2) * PP]), pr[(i - 1) * PP]);
                uint32_t* rs = ring + (slot * TX + tx0 + i) * PP + p;
                if (k >= NR) csum[i] = pk_sub_u16(csum[i], *rs);
                csum[i] = pk_add_u16(csum[i], h);
                *rs = h;
                const int xo = x0 + tx0 + i;
                if (emit && xo < W1)
                    *(uint32_t*)(C + (((size_t)f * H + y) * W1 + xo) * D + 2 * p) =
                        pk_add_u16(p2x2, csum[i]);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// 2b. cost volume, register-ring variant (NR = blockSize rows, 1..15).
// Block = 512 threads; thread (cl, p) owns disparity pair p and the RUN output
// columns [cl*RUN, cl*RUN + RUN) of a TX = CL*RUN wide tile.  Per source row:
//   stage  left columns as broadcast u16-pair forms {v, lo, hi} x 2 channels and
//          right columns as (j, j+1) u16-pair forms, so one lane reads the BT
//          operands of two disparities with two aligned 16-byte LDS reads and
//          no byte shuffles (double-buffered: row k+1 is staged while row k is
//          matched);
//   pix    BT cost of TX + 2*SW2 columns;
//   hsum   sliding horizontal box sum over the thread's RUN columns;
//   vsum   the last NR horizontal sums live in registers (ring slot = row mod
//          NR, resolved at compile time by unrolling the row loop by NR).
// One workgroup barrier per row.
// ---------------------------------------------------------------------------
// broadcast form of one channel dword (bytes v, lo, hi): {v|v<<16, lo|lo<<16, hi|hi<<16}
__device__ __forceinline__ uint3 bt_bcast(uint32_t w)
{
    return make_uint3(__builtin_amdgcn_perm(w, w, 0x0c040c00u), __builtin_amdgcn_perm(w, w, 0x0c050c01u),
                      __builtin_amdgcn_perm(w, w, 0x0c060c02u));
}
// pair form of one channel: low halves from column a (disparity d), high from b (d+1)
__device__ __forceinline__ uint3 bt_pairform(uint32_t a, uint32_t b)
{
    return make_uint3(__builtin_amdgcn_perm(b, a, 0x0c040c00u), __builtin_amdgcn_perm(b, a, 0x0c050c01u),
                      __builtin_amdgcn_perm(b, a, 0x0c060c02u));
}
__device__ __forceinline__ uint32_t bt_cost2(uint4 u4, uint2 u2, uint4 v4, uint2 v2)
{
    const uint32_t ca = bt_pair(u4.x, u4.y, u4.z, v4.x, v4.y, v4.z);
    const uint32_t cb = bt_pair(u4.w, u2.x, u2.y, v4.w, v2.x, v2.y);
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    const u16x2 two = {2, 2};
    // ca <= 2 ftzero <= 126, cb >> 2 <= 63: the halves never carry (full-rate add)
    return add2_nc(ca, __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, cb) >> two));
}

// 32 x 32 bit transpose inside each 32-lane half of the wave: afterwards lane q
// (of its half) holds bit q of every lane p's input word, as bit p.  Five
// delta-swap stages, lane distance s = 16 .. 1 against word-bit distance s
// (the host mirror in tests/cpp/bitslice_check.cpp checks the same stages):
// 16- and 8-bit fields move as bytes (v_permlane16_swap / DPP row_ror:8 + one
// v_perm_b32), 4-, 2- and 1-bit fields by rotating the partner's word and one
// v_bfi_b32 with the lane's keep mask.
__device__ __forceinline__ uint32_t bs_rotmix(uint32_t own, uint32_t pt, bool upper, int s, uint32_t M)
{
    const uint32_t sh = bs::fshr(pt, pt, upper ? s : 32 - s);
    const uint32_t K = upper ? ~M : M;
    return (K & own) | (~K & sh);
}
__device__ __forceinline__ uint32_t bs_transpose32(uint32_t x, int lane)
{
    {
        // rows (0, 1) and (2, 3) of the wave swap halves: r[0] keeps even rows
        // and receives the odd rows' words, r[1] the reverse
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        x = __builtin_amdgcn_perm(r[1], r[0], (lane & 16) ? 0x07060302u : 0x05040100u);
    }
    {
        const uint32_t pt = (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x128, 0xf, 0xf, true);  // row_ror:8 = lane ^ 8
        x = __builtin_amdgcn_perm(pt, x, (lane & 8) ? 0x03070105u : 0x06020400u);
    }
    {
        // lane ^ 4: row_shl:4 into banks 0 and 2, row_shr:4 into banks 1 and 3
        int pt = __builtin_amdgcn_update_dpp(0, (int)x, 0x104, 0xf, 0x5, false);
        pt = __builtin_amdgcn_update_dpp(pt, (int)x, 0x114, 0xf, 0xa, false);
        x = bs_rotmix(x, (uint32_t)pt, (lane & 4) != 0, 4, 0x0F0F0F0Fu);
    }
    x = bs_rotmix(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xf, 0xf, true), (lane & 2) != 0, 2, 0x33333333u);
    x = bs_rotmix(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xf, 0xf, true), (lane & 1) != 0, 1, 0x55555555u);
    return x;
}

// BSE: the bit-sliced pipeline's emission (C' planes, pixel-quad C, m; PPC 64
// only) compiled in place of the int16 C rows and the residual nibbles
template <int NR, int STG, int PPC, bool BSE>
__global__ __launch_bounds__(kCost2Threads) __attribute__((amdgpu_waves_per_eu(4))) void sgbm_cost2_kernel(const uint64_t* __restrict__ pre,
                                                                   int W, int H, SgbmEff e, int TY,
                                                                   int16_t* __restrict__ C,
                                                                   uint8_t* __restrict__ Rv,
                                                                   uint16_t* __restrict__ Mv,
                                                                   uint32_t* __restrict__ Bv, int xcd_bands)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int SH2 = NR / 2;
    constexpr int SW2 = SH2;  // StereoSGBM's window is square (SW = SH = blockSize)
    const int D = e.D, W1 = e.W1;
    const Cost2Layout lay = cost2_layout(D, SW2, TY);
    // PPC > 0: the disparity-pair count is known at compile time (PPC == D / 2),
    // so the interior pixel-cost loop unrolls with every LDS address an
    // immediate offset from one base per operand
    const int PP = PPC > 0 ? PPC : lay.PP, CL = PPC > 0 ? kCost2Threads / PPC : lay.CL;
    const int TX = CL * kCost2Run, NX = lay.NX;
    // XCD-aware tiles: workgroups go to the 8 XCDs round-robin by linear id
    // (tools/ubench/xcc_map.hip), so a row band's tiles -- which stage the same
    // input rows -- land on every XCD and each XCD's L2 fetches the band again.
    // When the bands divide evenly, XCD x runs whole bands x, x + 8, ... in
    // order instead (a bijection of the grid: linear id = 8 l + x).
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    {
        const int GX = gridDim.x, NB = gridDim.y * gridDim.z;
        if ((NB & 7) == 0 && xcd_bands) {
            const int id = bx + GX * (by + gridDim.y * bz);
            const int l = id >> 3, band = (l / GX) * 8 + (id & 7);
            bx = l % GX;
            by = band % gridDim.y;
            bz = band / gridDim.y;
        }
    }
    const int f = bz;
    const Cost2Tile tile = cost2_tile(TX, TY, SW2, bx, by, W1, H, e.minX1, e.minD, D);
    const int x0 = tile.x0, y0 = tile.y0, y1 = tile.y1, xclo = tile.xclo;
    const int nL = tile.nL;
    const size_t plane = (size_t)W * H;
    const uint64_t* PL = pre + (size_t)f * 2 * plane;
    const int tid = threadIdx.x;
    const int cl = tid / PP, p = tid - cl * PP;
    const bool worker = cl < CL;
    const int tx0 = cl * kCost2Run;
    const uint32_t p2x2 = (uint32_t)(e.P2 & 0xffff) * 0x10001u;
    const int nItems = tile.nItems;
    const bool linear = tile.linear;  // no clamped columns in this tile

    // staging: item i < nL -> left column ilo + i; else right pair j = i - nL
    // (reversed columns rtop - j and rtop - j - 1, zero outside the image).
    // Which items exist and where they sit in a row does not depend on the
    // row: the column offsets and validity masks are fixed here, fetch_row
    // only issues loads, and the loaded words are first touched by the next
    // row's stage_row -- so each row's loads stay in flight for a whole row
    // interval instead of being waited for where they are issued.
    // staged rows in flight: row r's loads sit in register set r % FD and are
    // first used FD - 1 rows after the row that issued them
    constexpr int FD = MVSV_COST2_FETCH_DEPTH;
    uint64_t pa[FD][STG], pb[FD][STG];
    int oa[STG], ob[STG];
    bool ma[STG], mb[STG];
#pragma unroll
    for (int k = 0; k < STG; k++) {
        const int i = kCost2Threads - 1 - tid + kCost2Threads * k;  // high waves: fewer pix columns
        const Cost2Item it = cost2_item(tile, i, W, (int)plane);
        ma[k] = it.ma;
        mb[k] = it.mb;
        oa[k] = it.oa;
        ob[k] = it.ob;
    }
    auto fetch_row = [&](int v, int set) {
        const uint64_t* row = PL + (size_t)clampi(v, 0, H - 1) * W;
#pragma unroll
        for (int k = 0; k < STG; k++) {
            pa[set][k] = row[oa[k]];
            pb[set][k] = row[ob[k]];
        }
    };
    auto stage_row = [&](int buf, int set) {
        uint4* l4 = (uint4*)(smem + lay.off_l4 + (buf ? lay.lstride4 : 0));
        uint2* l2 = (uint2*)(smem + lay.off_l2 + (buf ? lay.lstride2 : 0));
        uint4* q4 = (uint4*)(smem + lay.off_q4 + (buf ? lay.qstride4 : 0));
        uint2* q2 = (uint2*)(smem + lay.off_q2 + (buf ? lay.qstride2 : 0));
#pragma unroll
        for (int k = 0; k < STG; k++) {
            const int i = kCost2Threads - 1 - tid + kCost2Threads * k;  // high waves: fewer pix columns
            const uint64_t va = ma[k] ? pa[set][k] : 0ull, vb = mb[k] ? pb[set][k] : 0ull;
            if (i < nL) {
                const uint3 fa = bt_bcast((uint32_t)va), fb = bt_bcast((uint32_t)(va >> 32));
                l4[i] = make_uint4(fa.x, fa.y, fa.z, fb.x);
                l2[i] = make_uint2(fb.y, fb.z);
            } else if (i < nItems) {
                const int q = cost2_qslot(lay, i - nL);  // descending
                const uint3 fa = bt_pairform((uint32_t)va, (uint32_t)vb);
                const uint3 fb = bt_pairform((uint32_t)(va >> 32), (uint32_t)(vb >> 32));
                q4[q] = make_uint4(fa.x, fa.y, fa.z, fb.x);
                q2[q] = make_uint2(fb.y, fb.z);
            }
        }
    };
    auto pix_row = [&](int buf) {
        const uint4* l4 = (const uint4*)(smem + lay.off_l4 + (buf ? lay.lstride4 : 0));
        const uint2* l2 = (const uint2*)(smem + lay.off_l2 + (buf ? lay.lstride2 : 0));
        const uint4* q4 = (const uint4*)(smem + lay.off_q4 + (buf ? lay.qstride4 : 0));
        const uint2* q2 = (const uint2*)(smem + lay.off_q2 + (buf ? lay.qstride2 : 0));
        uint32_t* prow = (uint32_t*)(smem + lay.off_pix + (buf ? lay.pstride : 0)) + p * lay.PS;
        if (!worker) return;
        // slot of right pair j = t + 2p (t = xchi - xc); slots descend with j, so
        // a column lane's slot ascends as its column xv does
        auto qslot = [&](int t) { return cost2_qslot(lay, t + 2 * p); };
        // column lane cl computes column pairs (xv, xv + 1), xv = 2 cl + 2 CL k,
        // and stores each pair with one b64 write
        if (linear) {
            // interior tile: column xv reads left slot xv and right slot
            // qslot(nL - 1 - xv); both step by a fixed amount per iteration
            const int xa = 2 * cl;
            const int ta = nL - 1 - xa;
            if constexpr (PPC > 0) {
                constexpr int CLC = kCost2Threads / PPC;
                constexpr int KMAX = 2 + (SW2 + CLC - 1) / CLC;  // ceil((TX + 2 SW2) / (2 CL))
                const uint4* pl4 = l4 + xa;
                const uint2* pl2 = l2 + xa;
                const uint4* qa4 = q4 + qslot(ta);
                const uint2* qa2 = q2 + qslot(ta);
                const uint4* qb4 = q4 + qslot(ta - 1);
                const uint2* qb2 = q2 + qslot(ta - 1);
                uint2* pp = (uint2*)(prow + xa);
#pragma unroll
                for (int k = 0; k < KMAX; k++) {
                    if (xa + 2 * CLC * k >= NX) break;
                    const uint32_t c0 = bt_cost2(pl4[2 * CLC * k], pl2[2 * CLC * k], qa4[CLC * k], qa2[CLC * k]);
                    const uint32_t c1 =
                        bt_cost2(pl4[2 * CLC * k + 1], pl2[2 * CLC * k + 1], qb4[CLC * k], qb2[CLC * k]);
                    pp[CLC * k] = make_uint2(c0, c1);
                }
                return;
            }
            const uint4* pl4 = l4 + xa;
            const uint2* pl2 = l2 + xa;
            const uint4* qa4 = q4 + qslot(ta);
            const uint2* qa2 = q2 + qslot(ta);
            const uint4* qb4 = q4 + qslot(ta - 1);
            const uint2* qb2 = q2 + qslot(ta - 1);
            uint2* pp = (uint2*)(prow + xa);
#pragma unroll 1
            for (int xv = xa; xv < NX; xv += 2 * CL) {
                const uint32_t c0 = bt_cost2(pl4[0], pl2[0], *qa4, *qa2);
                const uint32_t c1 = bt_cost2(pl4[1], pl2[1], *qb4, *qb2);
                *pp = make_uint2(c0, c1);
                pl4 += 2 * CL;
                pl2 += 2 * CL;
                qa4 += CL;
                qa2 += CL;
                qb4 += CL;
                qb2 += CL;
                pp += CL;
            }
            return;
        }
#pragma unroll 1
        for (int xv = 2 * cl; xv < NX; xv += 2 * CL) {
            const int xca = clampi(x0 - SW2 + xv, 0, W1 - 1) - xclo;
            const int xcb = clampi(x0 - SW2 + xv + 1, 0, W1 - 1) - xclo;
            const int ja = qslot(nL - 1 - xca), jb = qslot(nL - 1 - xcb);
            *(uint2*)(prow + xv) = make_uint2(bt_cost2(l4[xca], l2[xca], q4[ja], q2[ja]),
                                              bt_cost2(l4[xcb], l2[xcb], q4[jb], q2[jb]));
        }
    };

    // the vertical window's ring of horizontal sums: slots 0 .. RR - 1 in
    // registers, RR .. NR - 1 in LDS (cost2_lds_ring_slots; this thread's own
    // words, so no barrier)
    constexpr int RL = cost2_lds_ring_slots(NR, STG, PPC), RR = NR - RL;
    uint4* ringl = (uint4*)(smem + cost2_ring_offset(lay)) + tid;
    uint32_t csum[kCost2Run], ring[RR][kCost2Run];
#pragma unroll
    for (int i = 0; i < kCost2Run; i++) {
        csum[i] = 0;
#pragma unroll
        for (int s = 0; s < RR; s++) ring[s][i] = 0;
    }
#pragma unroll
    for (int s = 0; s < RL; s++) ringl[s * kCost2Threads] = make_uint4(0, 0, 0, 0);

    const int vstart = y0 - SH2;
    const int nrows = (y1 - y0) + 2 * SH2;
    // row k of the sweep emits cost row y = y0 - 2*SH2 + k (once k >= NR - 1)
    const size_t ostride = (size_t)W1 * PP;  // dwords per cost row
    uint32_t* obase = (uint32_t*)C + (((size_t)f * H + y0) * W1 + x0 + tx0) * PP + p -
                      (size_t)(2 * SH2) * ostride;
    const int nout = min(kCost2Run, W1 - (x0 + tx0));
    // the bit-sliced pipeline's pixel-quad-major C (D = 128: 16 uint4 per pixel)
    const int W1q = (W1 + 3) & ~3;
    uint4* cq = (uint4*)C + ((ptrdiff_t)((size_t)f * H + y0 - 2 * SH2) * W1q + x0 + tx0) * 16 + p;
    // ... and the C' bit planes' four-pixel group of the wave's columns
    uint32_t* bq = Bv ? Bv + ((ptrdiff_t)((size_t)f * H + y0 - 2 * SH2) * W1q + x0 + tx0) * 16 : nullptr;
    static_assert(!BSE || PPC == 64, "bit-sliced emission: D = 128");
    // every column of the wave inside the image (all but the last tile column):
    // unpredicated stores
    const bool full = __all(nout == kCost2Run);
    const bool hh_pin = e.fullDP != 0;  // the fix-up kernel's MODE_HH cases, done here
    const bool fix_x0 = (e.variant & MVSV_VARIANT_FIRSTCOL_FIX) != 0;
    const int ybot = max(H - SH2, 1);
    fetch_row(vstart, 0);
    stage_row(0, 0);
#pragma unroll
    for (int r = 1; r <= FD; r++)
        if (r < nrows) fetch_row(vstart + r, r % FD);
    __syncthreads();
    // unrolled by NR * FD: the ring slot (k mod NR) and the register set of
    // every staged row are compile-time constants
    for (int base = 0; base < nrows; base += NR * FD) {
#pragma unroll
        for (int su = 0; su < NR * FD; su++) {
            const int k = base + su;
            const int s = su % NR;
            if (k >= nrows) break;
            const int buf = k & 1;
            if (k + 1 < nrows) {
                stage_row(buf ^ 1, (su + 1) % FD);
                if (k + 1 + FD < nrows) fetch_row(vstart + k + 1 + FD, (su + 1) % FD);
            }
            pix_row(buf);
            __syncthreads();  // pix[buf] complete; staging of row k+1 visible
            if (worker) {
                const bool lslot = s >= RR;
                const int sr = lslot ? 0 : s;
                uint4 lold = make_uint4(0, 0, 0, 0);
                if (lslot) lold = ringl[(s - RR) * kCost2Threads];
                // the thread's NR + RUN - 1 window columns: b64 loads, all in flight
                constexpr int NV = NR + kCost2Run - 1;  // even
                const uint2* pr = (const uint2*)((const uint32_t*)(smem + lay.off_pix + (buf ? lay.pstride : 0)) +
                                                 p * lay.PS + tx0);
                uint32_t wv[NV];
#pragma unroll
                for (int q = 0; q < NV / 2; q++) {
                    const uint2 t2 = pr[q];
                    wv[2 * q] = t2.x;
                    wv[2 * q + 1] = t2.y;
                }
                uint32_t h = 0;
#pragma unroll
                // packed sums as 32-bit words (full rate): a pixel cost is <= 189,
                // so a horizontal sum h <= 15 * 189 and a window sum <= 15 * 15 * 189
                // = 42525 < 2^16 -- no half ever carries or borrows (the slide
                // subtracts a term the sum holds)
                for (int q = 0; q < NR; q++) h = add2_nc(h, wv[q]);
                const bool emit = k >= NR - 1;
                uint32_t* orow = obase + (size_t)k * ostride;
                // MODE_HH: OpenCV 3.4 leaves P2 in the rows it never recomputes
                // (y >= H - SH2) and in column x = 0 of rows y >= 1
                const int yo = y0 - 2 * SH2 + k;
                const bool pin_row = hh_pin && yo >= ybot;
                const bool pin_x0 = hh_pin && !fix_x0 && yo >= 1 && x0 + tx0 == 0;
                uint32_t ov[kCost2Run], hv[kCost2Run];
#pragma unroll
                for (int i = 0; i < kCost2Run; i++) {
                    if (i > 0) h = sub2_nb(add2_nc(h, wv[i + NR - 1]), wv[i - 1]);
                    const uint32_t lo_i = i == 0 ? lold.x : i == 1 ? lold.y : i == 2 ? lold.z : lold.w;
                    csum[i] = add2_nc(sub2_nb(csum[i], lslot ? lo_i : ring[sr][i]), h);
                    if (lslot)
                        hv[i] = h;
                    else
                        ring[sr][i] = h;
                    const bool pin = pin_row || (i == 0 && pin_x0);
                    ov[i] = pin ? p2x2 : pk_add_u16(p2x2, csum[i]);
                }
                if (lslot) ringl[(s - RR) * kCost2Threads] = make_uint4(hv[0], hv[1], hv[2], hv[3]);
                // (bit-sliced pipeline: C is stored pixel-quad major by the C'
                // block below, one 16-byte store per lane)
                if constexpr (!BSE) {
                    if (emit) {
#pragma unroll
                        for (int i = 0; i < kCost2Run; i++)
                            if (full || i < nout) orow[i * PP] = ov[i];
                    }
                }
                // residual plane + per-pixel minimum: the lanes of a column
                // lane hold its pixel's D costs (PP <= 64 lanes, an aligned
                // segment of the wave).  Columns are paired (0, 1), (2, 3):
                // Plo = (c0[2p], c1[2p]), Phi = (c0[2p+1], c1[2p+1]); their
                // minima per lane, then one transposing step (even lanes keep
                // reducing columns (0, 1), odd lanes (2, 3)) and five
                // parity-preserving butterfly steps on a single dword.
                if ((BSE || Rv) && emit) {
                    const uint32_t Plo01 = __builtin_amdgcn_perm(ov[1], ov[0], 0x05040100u);
                    const uint32_t Phi01 = __builtin_amdgcn_perm(ov[1], ov[0], 0x07060302u);
                    const uint32_t Plo23 = __builtin_amdgcn_perm(ov[3], ov[2], 0x05040100u);
                    const uint32_t Phi23 = __builtin_amdgcn_perm(ov[3], ov[2], 0x07060302u);
                    uint32_t A = pk_min_u16(Plo01, Phi01), B = pk_min_u16(Plo23, Phi23);
                    const bool odd = (p & 1) != 0;
                    uint32_t X = pk_min_u16(odd ? B : A,
                                            (uint32_t)__builtin_amdgcn_mov_dpp((int)(odd ? A : B), 0xB1, 0xf, 0xf, false));
                    X = pk_min_u16(X, (uint32_t)__builtin_amdgcn_mov_dpp((int)X, 0x4E, 0xf, 0xf, false));   // lane ^ 2
                    X = pk_min_u16(X, (uint32_t)__builtin_amdgcn_mov_dpp((int)X, 0x124, 0xf, 0xf, false));  // row_ror:4
                    X = pk_min_u16(X, (uint32_t)__builtin_amdgcn_mov_dpp((int)X, 0x128, 0xf, 0xf, false));  // row_ror:8
                    if (PP >= 32) {
                        const auto sw = __builtin_amdgcn_permlane16_swap(X, X, false, false);
                        X = pk_min_u16(sw[0], sw[1]);
                    }
                    if (PP >= 64) {
                        const auto sw = __builtin_amdgcn_permlane32_swap(X, X, false, false);
                        X = pk_min_u16(sw[0], sw[1]);
                    }
                    const uint32_t Y = (uint32_t)__builtin_amdgcn_mov_dpp((int)X, 0xB1, 0xf, 0xf, false);
                    A = odd ? Y : X;  // (m0, m1) in every lane
                    B = odd ? X : Y;  // (m2, m3)
                    // per-pixel minimum (the final kernel's absolute cost base):
                    // lane p < 4 stores column p's
                    if (p < kCost2Run && p < nout) {
                        const uint32_t ab = p < 2 ? A : B;
                        Mv[(size_t)(orow - (uint32_t*)C) / PP + p] = (uint16_t)(p & 1 ? ab >> 16 : ab);
                    }
                    if constexpr (BSE) {
                        {
                            // bit-sliced C' = min(C - m, 2 P2) (round 5, mvsv_bitslice.hpp):
                            // nibble bytes as below but without the + P2 bias, columns in
                            // byte order (0, 2, 1, 3), then a 32 x 32 bit transpose inside
                            // each 32-lane half: lane l ends with word (h, e, b) of column
                            // c, bit p = bit b of C'(c, 64 h + 2 p + e) -- one dword store
                            // per lane, the wave's four pixels as one 256-byte record run
                            // (C' <= 2 P2 <= 10: the subtractions never borrow, m <= C)
                            const uint32_t p2x4 = add2_nc(p2x2, p2x2);
                            const uint32_t r01 = pk_min_u16(sub2_nb(Plo01, A), p2x4) |
                                                 (pk_min_u16(sub2_nb(Phi01, A), p2x4) << 4);
                            const uint32_t r23 = pk_min_u16(sub2_nb(Plo23, B), p2x4) |
                                                 (pk_min_u16(sub2_nb(Phi23, B), p2x4) << 4);
                            const uint32_t tw = bs_transpose32(r01 | (r23 << 8), p);
                            const int q = p & 31, kq = q >> 3;
                            const int c = ((kq & 1) << 1) | (kq >> 1);
                            // the four-pixel group of the wave's columns (mvsv_bitslice.hpp
                            // cq_word): word (q' = 2 h + e) * 16 + c * 4 + b
                            const int qw = (2 * (p >> 5) + ((q & 7) >> 2)) * 16 + c * 4 + (q & 3);
                            if (full || c < nout) bq[(ptrdiff_t)k * W1q * 16 + qw] = tw;
                            // C is read only for the WTA's C(best -+ 1) gathers, so it
                            // is stored [frame][y][x / 4][d][x % 4] (rows padded to
                            // a multiple of 4 pixels, read by mvsv_bsgm.hip bsgm_wta_kernel):
                            // the four pixels' C(d -+ 1) share a line; lane p writes
                            // d = 2 p, 2 p + 1 of the wave's four columns -- the
                            // wave's 1 KiB as one run
                            // (a wave wholly right of W1 -- nout <= 0 -- would land in
                            // the next row)
                            if (nout > 0) cq[(ptrdiff_t)k * W1q * 16] = make_uint4(Plo01, Plo23, Phi01, Phi23);
                        }
                    }
                    if (!BSE && Rv) {
                    // R = min(C - m, 2 P2) + P2 = min(C - (m - P2), 3 P2) on the
                    // column pairs; one word holds columns 0 and 1's residual
                    // bytes R[2p] | R[2p+1] << 4 in bits 0-7 and 16-23
                    const uint32_t p2x3 = pk_add_u16(pk_add_u16(p2x2, p2x2), p2x2);
                    // (residual runs are no-wrap: P2 <= m <= C, so the 32-bit
                    // subtractions never borrow)
                    const uint32_t Am = sub2_nb(A, p2x2), Bm = sub2_nb(B, p2x2);
                    const uint32_t r01 = pk_min_u16(sub2_nb(Plo01, Am), p2x3) |
                                         (pk_min_u16(sub2_nb(Phi01, Am), p2x3) << 4);
                    const uint32_t r23 = pk_min_u16(sub2_nb(Plo23, Bm), p2x3) |
                                         (pk_min_u16(sub2_nb(Phi23, Bm), p2x3) << 4);
                    uint8_t* rrow = Rv + (orow - (uint32_t*)C);  // byte (pixel, pair) = dword (pixel, pair) of C
                    const uint32_t rw[kCost2Run] = {r01, r01 >> 16, r23, r23 >> 16};
#pragma unroll
                    for (int i = 0; i < kCost2Run; i++)
                        if (full || i < nout) rrow[i * PP] = (uint8_t)rw[i];
                    }
                }
            }
        }
    }
}

// 3. OpenCV 3.4 cost-row quirks (see oracle/twin.py sgbm_cost_volume):
//    rows y >= 1 never refresh column x = 0; rows with y + SH2 >= H are never
//    recomputed (MODE_SGBM keeps the last computed row, MODE_HH keeps P2).
// Column x = 0 of rows 1 .. ybot - 1 (block per row; not launched with
// FIRSTCOL_FIX): C(0, 0, d), or P2 in MODE_HH.
// A pixel's residual (when Rv != nullptr) depends only on its own D costs, so
// a copied cost vector carries its residual bytes along (P2 everywhere: P2).
__global__ __launch_bounds__(256) void sgbm_cost_fixup_col0_kernel(int16_t* __restrict__ C, int H,
                                                                   SgbmEff e, uint8_t* __restrict__ Rv,
                                                                   uint16_t* __restrict__ Mv)
{
    const int y = 1 + blockIdx.x;
    const int f = blockIdx.y;
    const int D = e.D, W1 = e.W1;
    int16_t* Cf = C + (size_t)f * H * W1 * D;
    int16_t* row = Cf + (size_t)y * W1 * D;
    for (int d = threadIdx.x; d < D; d += blockDim.x) row[d] = e.fullDP ? (int16_t)e.P2 : Cf[d];
    if (Rv) {
        uint8_t* Rf = Rv + (size_t)f * H * W1 * (D / 2);
        uint8_t* rrow = Rf + (size_t)y * W1 * (D / 2);
        for (int k = threadIdx.x; k < D / 2; k += blockDim.x)
            rrow[k] = e.fullDP ? (uint8_t)(e.P2 * 0x11) : Rf[k];
        uint16_t* Mf = Mv + (size_t)f * H * W1;
        if (threadIdx.x == 0) Mf[(size_t)y * W1] = e.fullDP ? (uint16_t)e.P2 : Mf[0];
    }
}

// Rows ybot .. H - 1, all columns (grid: 8-element chunks x rows x frames):
// row ylast (column 0: C(0, 0, d) unless FIRSTCOL_FIX) or P2 (MODE_HH).  D is a
// multiple of 16, so a 16-byte chunk never straddles two columns.
__global__ __launch_bounds__(256) void sgbm_cost_fixup_bottom_kernel(int16_t* __restrict__ C, int H,
                                                                     SgbmEff e, int ylast, int ybot,
                                                                     uint8_t* __restrict__ Rv,
                                                                     uint16_t* __restrict__ Mv)
{
    const int D = e.D, W1 = e.W1;
    const size_t chunk = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // 8 elements each
    const size_t rowlen = (size_t)W1 * D;
    if (chunk * 8 >= rowlen) return;
    const int y = ybot + blockIdx.y;
    const int f = blockIdx.z;
    int16_t* Cf = C + (size_t)f * H * rowlen;
    uint4* dst = (uint4*)(Cf + (size_t)y * rowlen) + chunk;
    uint4 v;
    const bool fix = (e.variant & MVSV_VARIANT_FIRSTCOL_FIX) != 0;
    const bool col0 = chunk * 8 < (size_t)D && !fix;
    if (e.fullDP) {
        const uint32_t p2 = (uint32_t)(e.P2 & 0xffff) * 0x10001u;
        v = make_uint4(p2, p2, p2, p2);
    } else {
        v = *((const uint4*)(Cf + (col0 ? 0 : (size_t)ylast * rowlen)) + chunk);
    }
    *dst = v;
    if (Rv) {  // the chunk's 8 residual nibbles: one dword
        uint32_t* Rf = (uint32_t*)(Rv + (size_t)f * H * (rowlen / 2));
        Rf[(size_t)y * (rowlen / 8) + chunk] =
            e.fullDP ? (uint32_t)e.P2 * 0x11111111u : Rf[(col0 ? 0 : (size_t)ylast * (rowlen / 8)) + chunk];
        if (chunk * 8 % D == 0) {  // the first chunk of a pixel carries its minimum
            uint16_t* Mf = Mv + (size_t)f * H * W1;
            const size_t x = chunk * 8 / D;
            Mf[(size_t)y * W1 + x] = e.fullDP ? (uint16_t)e.P2 : Mf[col0 ? 0 : (size_t)ylast * W1 + x];
        }
    }
}

}  // namespace

using Cost2Kern = void (*)(const uint64_t*, int, int, SgbmEff, int, int16_t*, uint8_t*, uint16_t*, uint32_t*, int);
template <int STG, int PPC, bool BSE>
static Cost2Kern cost2_pick_nr(int nr)
{
    switch (nr) {
    case 1: return sgbm_cost2_kernel<1, STG, PPC, BSE>;
    case 3: return sgbm_cost2_kernel<3, STG, PPC, BSE>;
    case 5: return sgbm_cost2_kernel<5, STG, PPC, BSE>;
    case 7: return sgbm_cost2_kernel<7, STG, PPC, BSE>;
    case 9: return sgbm_cost2_kernel<9, STG, PPC, BSE>;
    case 11: return sgbm_cost2_kernel<11, STG, PPC, BSE>;
    case 13: return sgbm_cost2_kernel<13, STG, PPC, BSE>;
    default: return sgbm_cost2_kernel<15, STG, PPC, BSE>;
    }
}
// kernel for blockSize nr, STG staged items per thread (1 / 2), PPC pairs (64 /
// 128 fixed, 0 = from the layout); bse: the bit-sliced emission (PPC 64)
static Cost2Kern cost2_pick(int nr, int stg, int ppc, bool bse)
{
    if (bse)
        return stg == 1 ? cost2_pick_nr<1, 64, true>(nr) : cost2_pick_nr<2, 64, true>(nr);
    if (stg == 1)
        return ppc == 64    ? cost2_pick_nr<1, 64, false>(nr)
               : ppc == 128 ? cost2_pick_nr<1, 128, false>(nr)
                            : cost2_pick_nr<1, 0, false>(nr);
    return ppc == 64 ? cost2_pick_nr<2, 64, false>(nr)
           : ppc == 128 ? cost2_pick_nr<2, 128, false>(nr)
                        : cost2_pick_nr<2, 0, false>(nr);
}

// Cost-volume launch: the register-ring kernel when blockSize <= 15 and the
// tile fits, else the LDS-ring kernel.  *Rv (residual plane, may be nullptr)
// is written by the register-ring kernel only: the LDS-ring fallback sets it
// to nullptr, and the direction passes then read C.
int launch_cost(mvsv_ctx* ctx, int n, int W, int H, const SgbmEff& e, int TY,
                       const uint64_t* pre, int16_t* Cv, uint8_t** Rv, uint16_t* Mv, bool* pinned_hh,
                       uint32_t** Bv)
{
    *pinned_hh = false;
    hipStream_t s = ctx->stream;
    int rc;
    if (ctx->cost2 && e.SH2 <= 7 && e.SW2 == e.SH2) {
        const Cost2Layout l2 = cost2_layout(e.D, e.SW2, TY);
        const int items = 2 * l2.NX + e.D - 1;
        const bool two = items > kCost2Threads;
        // numDisparities 128 / 256: the pair count is a compile-time
        // constant (unrolled pixel-cost loop, immediate LDS offsets)
        const int ppc = !ctx->cost_fixed_pp ? 0 : l2.PP == 64 ? 64 : (l2.PP == 128 ? 128 : 0);
        const size_t lbytes = cost2_total_bytes(l2, 2 * e.SH2 + 1, two ? 2 : 1, ppc);
        if (l2.CL >= 1 && items <= kCost2Threads * 2 && lbytes <= 160 * 1024) {
            dim3 grid2((e.W1 + l2.TX - 1) / l2.TX, (H + TY - 1) / TY, n);
            Cost2Kern kern = nullptr;
            if (ppc != 64) *Bv = nullptr;  // the bit-sliced plane: D = 128 kernels only
            kern = cost2_pick(2 * e.SH2 + 1, two ? 2 : 1, ppc, *Bv != nullptr);
            if (lbytes > 65536 &&
                (rc = check_hip(ctx, hipFuncSetAttribute((const void*)kern,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize,
                                                         (int)lbytes),
                                "sgbm cost LDS attribute")))
                return rc;
            {
                StageTimer tm(ctx, kStageCost);
                hipLaunchKernelGGL(kern, grid2, dim3(kCost2Threads), lbytes, s, pre, W, H, e, TY,
                                   Cv, *Bv ? nullptr : *Rv, Mv, *Bv, ctx->cost_xcd ? 1 : 0);
            }
            *pinned_hh = e.fullDP != 0;  // MODE_HH fix-up rows/column written by the kernel
            return check_hip(ctx, hipGetLastError(), "sgbm cost kernel");
        }
    }
    *Rv = nullptr;
    *Bv = nullptr;
    CostLayout lay = cost_layout(e.D, e.SW2, e.SH2, TY);
    if (lay.nLmax + lay.nRmax + 1 > 256 * kStageRegs)
        return set_error(ctx, MVSV_E_INVALID_ARG, "numDisparities too large for the GPU cost kernel");
    if (lay.bytes > 160 * 1024)
        return set_error(ctx, MVSV_E_INVALID_ARG, "blockSize too large for the GPU cost kernel");
    dim3 cgrid((e.W1 + lay.TX - 1) / lay.TX, (H + TY - 1) / TY, n);
    if (lay.bytes > 65536 &&
        (rc = check_hip(ctx, hipFuncSetAttribute((const void*)sgbm_cost_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)lay.bytes),
                        "sgbm cost LDS attribute")))
        return rc;
    {
        StageTimer tm(ctx, kStageCost);
        hipLaunchKernelGGL(sgbm_cost_kernel, cgrid, dim3(256), lay.bytes, s, pre, W, H, e, TY, Cv);
    }
    return check_hip(ctx, hipGetLastError(), "sgbm cost kernel");
}

bool cost2_runs(const mvsv_ctx* ctx, const SgbmEff& e)
{
    if (!ctx->cost2 || e.SH2 > 7 || e.SW2 != e.SH2) return false;
    const Cost2Layout l2 = cost2_layout(e.D, e.SW2, 120);  // (the layout does not depend on the tile height)
    const int items = 2 * l2.NX + e.D - 1;
    const int ppc = !ctx->cost_fixed_pp ? 0 : l2.PP == 64 ? 64 : (l2.PP == 128 ? 128 : 0);
    const size_t lbytes = cost2_total_bytes(l2, 2 * e.SH2 + 1, items > kCost2Threads ? 2 : 1, ppc);
    return l2.CL >= 1 && items <= kCost2Threads * 2 && lbytes <= 160 * 1024;
}

int launch_prefilter(mvsv_ctx* ctx, int n, const uint8_t* L, size_t ls, size_t lfs, const uint8_t* R, size_t rs,
                     size_t rfs, int W, int H, int ftzero, uint64_t* pre)
{
    StageTimer tm(ctx, kStagePre);
    hipLaunchKernelGGL(sgbm_prefilter_kernel, dim3(H, 2, n), dim3(256), (size_t)W * 2, ctx->stream, L, ls, lfs, R,
                       rs, rfs, W, H, ftzero, pre);
    return check_hip(ctx, hipGetLastError(), "sgbm prefilter");
}

int launch_cost_fixup(mvsv_ctx* ctx, int n, int H, const SgbmEff& e, int16_t* Cv, uint8_t* Rv, uint16_t* Mv)
{
    hipStream_t s = ctx->stream;
    const int ybot = std::max(H - e.SH2, 1);     // first row that is never recomputed
    const int ylast = std::max(H - e.SH2 - 1, 0);  // last recomputed row
    StageTimer tm(ctx, kStageFixup);
    // OpenCV 3.4 quirks: rows >= 1 never refresh column 0; rows with
    // y + SH2 >= H are never recomputed (MODE_SGBM keeps the last computed
    // row, MODE_HH keeps P2).  Column 0 of the bottom rows is written by the
    // bottom kernel (the rows are disjoint).
    const bool fix = (e.variant & MVSV_VARIANT_FIRSTCOL_FIX) != 0;
    if (ybot > 1 && !fix)
        hipLaunchKernelGGL(sgbm_cost_fixup_col0_kernel, dim3(ybot - 1, n), dim3(256), 0, s, Cv, H, e, Rv, Mv);
    if (ybot < H) {
        const size_t chunks = ((size_t)e.W1 * e.D + 7) / 8;
        hipLaunchKernelGGL(sgbm_cost_fixup_bottom_kernel, dim3((unsigned)((chunks + 255) / 256), H - ybot, n),
                           dim3(256), 0, s, Cv, H, e, ylast, ybot, Rv, Mv);
    }
    return check_hip(ctx, hipGetLastError(), "sgbm cost fixup");
}

}  // namespace mvsv
