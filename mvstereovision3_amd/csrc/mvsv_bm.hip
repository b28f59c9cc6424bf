// mvsv_bm.hip — StereoBM on MI355X (gfx950).
//
// Replaces Disparity::bm (src/disparity.cpp:18-22) -> cv::StereoBM::compute
// with a CV_16S output.  Pipeline:
//   1. bm_xsobel_kernel     [OpenCV] prefilterXSobel: clipped x-Sobel on row pairs
//      (bm_prefilter_norm_kernel for PREFILTER_NORMALIZED_RESPONSE: prefilterNorm)
//   2. fill_kernel          everything FILTERED = (minDisparity - 1) * 16
//   3. bm_match_kernel      16x16 output tile per 256-thread block: the left /
//                           right prefiltered tiles are staged in LDS, column
//                           sums of |L - R| are built per disparity with
//                           running sums, the window SAD of every pixel of
//                           every disparity is kept in LDS for the
//                           uniqueness test and the parabola fit; texture
//                           test, uniqueness, sub-pixel as OpenCV 3.4
//   4. bm_validate_kernel   (disp12MaxDiff >= 0) validateDisparity per row
//   5. bm_roi_kernel        validDisparityRect -> FILTERED outside
//   6. speckle filter       (speckleWindowSize > 0 and speckleRange >= 0)
// Window semantics: every computed pixel uses the virtual column
// j = x - lofs with OpenCV's separate left / right column clamps
// (left: lofs + clamp(j, -lofs, W-1-lofs), right: rofs + clamp(j, -rofs,
// W-ndisp-rofs) + k), so the border columns that validateDisparity sees
// match OpenCV's sliding-sum implementation bit for bit.
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "mvsv_device.hpp"
#include "mvsv_internal.hpp"

namespace mvsv {
namespace {

using namespace dev;

__global__ __launch_bounds__(256) void bm_xsobel_kernel(const uint8_t* __restrict__ src, size_t ss,
                                                        size_t sfs, int W, int H, int cap,
                                                        uint8_t* __restrict__ dst)
{
    const int y = blockIdx.x;
    const int f = blockIdx.y;
    const uint8_t* s = src + f * sfs;
    uint8_t* o = dst + ((size_t)f * H + y) * W;
    const uint8_t c8 = (uint8_t)cap;
    if ((H & 1) && y == H - 1) {
        for (int x = threadIdx.x; x < W; x += blockDim.x) o[x] = c8;
        return;
    }
    const int yb = y & ~1;
    const int k = y - yb;
    const int r0 = yb > 0 ? yb - 1 : (H > 1 ? yb + 1 : yb);
    const int r1 = yb;
    const int r2 = yb < H - 1 ? yb + 1 : (H > 1 ? yb - 1 : yb);
    const int r3 = yb < H - 2 ? yb + 2 : yb;
    const uint8_t* a = s + (size_t)(k == 0 ? r0 : r1) * ss;
    const uint8_t* b = s + (size_t)(k == 0 ? r1 : r2) * ss;
    const uint8_t* c = s + (size_t)(k == 0 ? r2 : r3) * ss;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        uint8_t v = c8;
        if (x > 0 && x < W - 1) {
            int g = (a[x + 1] - a[x - 1]) + 2 * (b[x + 1] - b[x - 1]) + (c[x + 1] - c[x - 1]);
            v = (uint8_t)(clampi(g, -cap, cap) + cap);
        }
        o[x] = v;
    }
}

// [OpenCV] prefilterNorm (PREFILTER_NORMALIZED_RESPONSE), one block per row:
// vsum[x] = sum of the winsize rows around y (replicated borders, exact in 16
// bits: <= 255 * 255), sum(x) = sum of vsum over the winsize columns around x
// (replicated), val = ((4 c[x] + c[x-1] + c[x+1] + p[x] + n[x]) * scale_g -
// sum * scale_s) >> 10 with c/p/n the current / previous / next row
// (replicated), out = clamp(val, -ftzero, ftzero) + ftzero.  The row's vsum
// lives in LDS with wsz2 replicated cells on either side.
__global__ __launch_bounds__(256) void bm_prefilter_norm_kernel(const uint8_t* __restrict__ src,
                                                                size_t ss, size_t sfs, int W, int H,
                                                                int winsize, int ftzero,
                                                                uint8_t* __restrict__ dst)
{
    extern __shared__ int vs[];  // W + 2 * wsz2 cells
    const int y = blockIdx.x;
    const int f = blockIdx.y;
    const int wsz2 = winsize / 2;
    const uint8_t* s = src + f * sfs;
    uint8_t* o = dst + ((size_t)f * H + y) * W;
    const int scale_g0 = winsize * winsize / 8;
    const int scale_s = (1024 + scale_g0) / (scale_g0 * 2);
    const int scale_g = scale_g0 * scale_s;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        int v = 0;
        for (int r = y - wsz2; r <= y + wsz2; r++) v += s[(size_t)clampi(r, 0, H - 1) * ss + x];
        vs[wsz2 + x] = v;
    }
    __syncthreads();
    for (int k = threadIdx.x; k < wsz2; k += blockDim.x) {
        vs[k] = vs[wsz2];
        vs[wsz2 + W + k] = vs[wsz2 + W - 1];
    }
    __syncthreads();
    const uint8_t* prev = s + (size_t)max(y - 1, 0) * ss;
    const uint8_t* curr = s + (size_t)y * ss;
    const uint8_t* next = s + (size_t)min(y + 1, H - 1) * ss;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        int sum = 0;
        for (int k = 0; k <= 2 * wsz2; k++) sum += vs[x + k];
        const int c4 = curr[x] * 4 + curr[max(x - 1, 0)] + curr[min(x + 1, W - 1)];
        const int val = ((c4 + prev[x] + next[x]) * scale_g - sum * scale_s) >> 10;
        o[x] = (uint8_t)(clampi(val, -ftzero, ftzero) + ftzero);
    }
}

__global__ void bm_fill_kernel(int16_t* __restrict__ out, size_t os, size_t ofs, int W, int H,
                               int16_t v)
{
    const int y = blockIdx.x, f = blockIdx.y;
    int16_t* o = out + f * ofs + (size_t)y * os;
    for (int x = threadIdx.x; x < W; x += blockDim.x) o[x] = v;
}

struct BmLayout {
    int NJ, NRW, NRC;
    size_t off_r, off_v, off_sad, bytes;
};

__host__ __device__ inline BmLayout bm_layout(int nd, int w2, int sad_bytes)
{
    BmLayout l;
    l.NJ = 16 + 2 * w2;
    l.NRW = 16 + 2 * w2;
    l.NRC = l.NJ + nd;
    l.off_r = (((size_t)l.NRW * l.NJ) + 15) & ~(size_t)15;
    l.off_v = (l.off_r + (size_t)l.NRW * l.NRC + 15) & ~(size_t)15;
    l.off_sad = l.off_v + (size_t)16 * l.NJ * 4;
    l.bytes = l.off_sad + (size_t)nd * 256 * sad_bytes;
    return l;
}

// bound on the general kernel's global window-sum scratch (per launch)
constexpr size_t kBmScratchBytes = (size_t)64 << 20;

// gsad != nullptr: the per-disparity window sums live in a global scratch slab
// of this block ([numDisparities][256]) instead of LDS (large numDisparities x
// blockSize whose LDS image would not fit).  The slab is indexed by the block
// of this launch; the host splits such grids into launches of a bounded block
// count (row-tile offset by0, frame f0), so the scratch stays bounded.
template <typename SadT>
__global__ __launch_bounds__(256) void bm_match_kernel(const uint8_t* __restrict__ Lf,
                                                       const uint8_t* __restrict__ Rf, int W,
                                                       int H, BmEff e, int keep_border,
                                                       int16_t* __restrict__ out, size_t os,
                                                       size_t ofs, int* __restrict__ cost,
                                                       SadT* __restrict__ gsad, int by0, int f0)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nd = e.ndisp, w2 = e.wsz2, win = 2 * w2 + 1;
    const BmLayout lay = bm_layout(nd, w2, (int)sizeof(SadT));
    uint8_t* Lt = smem;
    uint8_t* Rt = smem + lay.off_r;
    uint32_t* V = (uint32_t*)(smem + lay.off_v);
    const size_t blk = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    SadT* sadbuf = gsad ? gsad + blk * (size_t)e.ndisp * 256 : (SadT*)(smem + lay.off_sad);
    const int NJ = lay.NJ, NRW = lay.NRW, NRC = lay.NRC;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int f = f0 + (int)blockIdx.z;
    const int xl0 = blockIdx.x * 16;
    const int yr0 = e.ymin + (by0 + (int)blockIdx.y) * 16;
    const int lofs = e.lofs, rofs = e.rofs;
    const uint8_t* Lfr = Lf + (size_t)f * W * H;
    const uint8_t* Rfr = Rf + (size_t)f * W * H;
    const int jmin = xl0 - w2;
    auto clampL = [&](int j) { return lofs + clampi(j, -lofs, W - 1 - lofs); };
    auto clampR = [&](int j) { return clampi(j, -rofs, W - nd - rofs); };
    const int rbase = clampR(jmin);

    // stage the tiles (rows clamped to the image; only valid rows are used)
    for (int i = tid; i < NRW * NJ; i += 256) {
        int r = i / NJ, c = i - r * NJ;
        int yy = clampi(yr0 - w2 + r, 0, H - 1);
        Lt[i] = Lfr[(size_t)yy * W + clampL(jmin + c)];
    }
    for (int i = tid; i < NRW * NRC; i += 256) {
        int r = i / NRC, c = i - r * NRC;
        int yy = clampi(yr0 - w2 + r, 0, H - 1);
        int xx = min(rofs + rbase + c, W - 1);
        Rt[i] = Rfr[(size_t)yy * W + xx];
    }
    __syncthreads();

    const int xl = xl0 + tx, y = yr0 + ty;
    const bool active = xl < e.ncol && y < e.ymax;
    uint32_t minsad = 0xffffffffu;
    int mind = -1;
    for (int k = 0; k < nd; k++) {
        // column sums: thread -> (column c, 4-row chunk)
        for (int item = tid; item < NJ * 4; item += 256) {
            int c = item % NJ, chunk = item / NJ;
            int rc = clampR(jmin + c) - rbase + k;
            int t0 = chunk * 4;
            const uint8_t* lcol = Lt + c;
            const uint8_t* rcol = Rt + rc;
            uint32_t sum = 0;
            for (int r = t0; r < t0 + win; r++) sum += abs((int)lcol[r * NJ] - (int)rcol[r * NRC]);
            V[t0 * NJ + c] = sum;
            for (int t = t0 + 1; t < t0 + 4; t++) {
                int ra = t + win - 1, rs = t - 1;
                sum += abs((int)lcol[ra * NJ] - (int)rcol[ra * NRC]);
                sum -= abs((int)lcol[rs * NJ] - (int)rcol[rs * NRC]);
                V[t * NJ + c] = sum;
            }
        }
        __syncthreads();
        uint32_t sad = 0;
        const uint32_t* vr = V + ty * NJ + tx;
        for (int q = 0; q < win; q++) sad += vr[q];
        sadbuf[k * 256 + tid] = (SadT)sad;
        if (sad < minsad) {
            minsad = sad;
            mind = k;
        }
        __syncthreads();
    }
    if (!active) return;
    const int ximg = lofs + xl;
    int16_t* op = out + f * ofs + (size_t)y * os + ximg;
    if (!keep_border && (ximg < e.xmin || ximg >= e.xmax)) {
        *op = (int16_t)e.filtered;
        return;
    }
    int tsum = 0;
    for (int r = ty; r < ty + win; r++)
        for (int q = tx; q < tx + win; q++) tsum += abs((int)Lt[r * NJ + q] - e.cap);
    if (tsum < e.tex) {
        *op = (int16_t)e.filtered;
        return;
    }
    if (e.uniq > 0) {
        const int ms = (int)minsad;
        const int thresh = ms + (ms * e.uniq / 100);
        for (int k = 0; k < nd; k++) {
            if ((k < mind - 1 || k > mind + 1) && (int)sadbuf[k * 256 + tid] <= thresh) {
                *op = (int16_t)e.filtered;
                return;
            }
        }
    }
    const int v1 = nd - mind - 1 + e.mindisp;
    int val;
    if (0 < mind && mind < nd - 1) {
        int p = (int)sadbuf[(mind + 1) * 256 + tid], n = (int)sadbuf[(mind - 1) * 256 + tid];
        int d = p + n - 2 * (int)minsad + abs(p - n);
        val = (v1 * 256 + (d != 0 ? (p - n) * 256 / d : 0) + 15) >> 4;
    } else {
        val = (v1 * 256 + 15) >> 4;
    }
    *op = (int16_t)val;
    if (cost) cost[((size_t)f * H + y) * W + ximg] = (int)minsad;
}

// ---------------------------------------------------------------------------
// bm_match2_kernel: disparities on the lanes.  A 256-thread block stages the
// prefiltered rows of a (64 / NR)-column x TY-row tile (plus the window halo)
// in LDS.  The block's four waves form 4 / NR column groups of 16 output
// columns; the NR waves of a group hold the disparity indices
// kk = lane + 64 g (g = the wave's rank in its group) and walk down the tile's
// rows together:
//   * column sums of |L - R| over the window's rows per virtual column, kept in
//     registers and slid down one row per step: one masked byte SAD
//     (v_msad_u8) adds the new row, one subtracts the old.  Both views are
//     staged as value + 1 (never 0, so the byte mask of v_msad_u8 selects one
//     byte; differences are unchanged): the left view as one dword per pixel
//     with the byte in lane (column & 3), read as wave-uniform b128 broadcasts,
//     the right view as four byte-shifted dword copies, so lane kk reads the
//     four right pixels of four consecutive columns with one ds_read_b32;
//   * the window SAD of the 16 output columns by a sliding sum over the
//     virtual columns, written to the group's [column][disparity] LDS slab
//     (disparity indices >= numDisparities carry a +0x10000 offset per column
//     sum, so they never win and never fail the uniqueness test);
//   * the slab is re-read with 4 NR lanes per output column (each wave of the
//     group takes 16 / NR of the columns), each lane scanning 16 disparity
//     indices: argmin (ties -> smallest index, as OpenCV's ascending scan with
//     '<') with keys (sad << 8 | index) and v_min3, DPP reductions; the
//     uniqueness test masks the winner and its two neighbours in the slab and
//     takes a second minimum; texture sums (column sums of |L - cap| slid the
//     same way) and the parabola neighbours as bm_match_kernel.
// Same virtual-column clamps and the same per-pixel decisions as
// bm_match_kernel (which remains for blockSize > 21 or numDisparities > 128).
// ---------------------------------------------------------------------------
constexpr int kBm2Cols = 16;   // output columns per column group
constexpr int kBm2Waves = 4;   // waves per block
constexpr uint32_t kBm2Pad = 0x10000u;  // per-column offset of the unused disparity lanes

struct Bm2Layout {
    int NJ, NJP, NRW, NRC;
    size_t copy, off_r, off_sad, off_tc, off_rec, bytes;
};

__host__ __device__ inline Bm2Layout bm2_layout(int w2, int TY, int NR)
{
    Bm2Layout l;
    l.NJ = kBm2Waves / NR * kBm2Cols + 2 * w2;
    l.NJP = (l.NJ + 3) & ~3;
    l.NRW = TY + 2 * w2;
    l.NRC = (l.NJ + 64 * NR + 4 + 3) & ~3;  // right-view bytes per row
    // four byte-shifted copies of the right view; copy stride = 32 mod 128
    // bytes: a ds_read_b32 half-wave (32 lanes, banks = dword mod 32) reads 8
    // consecutive dwords of each copy, at bank offsets 0 / 8 / 16 / 24
    l.copy = (((size_t)l.NRW * l.NRC + 127) & ~(size_t)127) + 32;
    l.off_r = (size_t)l.NRW * l.NJP * 4;
    l.off_sad = l.off_r + 4 * l.copy;
    // slabs of all groups: [column][NR * 64 + 4] -- the 16-byte pad puts the
    // four columns of a ds_read_b128 lane group on different banks
    l.off_tc = l.off_sad + (size_t)(kBm2Waves / NR) * kBm2Cols * (NR * 64 + 4) * 4;
    l.off_rec = l.off_tc + (size_t)kBm2Waves * 64 * 4;  // texture sums per wave
    l.bytes = l.off_rec + (size_t)kBm2Waves * 64 * 8;   // per-wave output records
    return l;
}

template <int NR, int W2>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) void bm_match2_kernel(
    const uint8_t* __restrict__ Lf, const uint8_t* __restrict__ Rf, int W, int H, BmEff e,
    int keep_border, int TY, int16_t* __restrict__ out, size_t os, size_t ofs,
    int* __restrict__ cost)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int win = 2 * W2 + 1;
    constexpr int BC = kBm2Waves / NR * kBm2Cols;  // output columns per block
    constexpr int NC = kBm2Cols + 2 * W2;          // virtual columns of a column group
    const int nd = e.ndisp;
    const Bm2Layout lay = bm2_layout(W2, TY, NR);
    const int NJP = lay.NJP, NRW = lay.NRW, NRC = lay.NRC;
    uint32_t* Lt = (uint32_t*)smem;         // [NRW][NJP] (L + 1) << 8 (c & 3)
    uint8_t* Rp = smem + lay.off_r;         // copy 0: [NRW][NRC] bytes R + 1
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int cg = wv / NR, g = wv % NR;  // column group, disparity block of this wave
    constexpr int SS = NR * 64 + 4;  // slab column stride (dwords)
    uint32_t* sadx = (uint32_t*)(smem + lay.off_sad) + (size_t)cg * kBm2Cols * SS;
    int* tcb = (int*)(smem + lay.off_tc) + wv * 64;
    uint2* recs = (uint2*)(smem + lay.off_rec) + wv * 64;
    const int f = blockIdx.z;
    const int xl0 = blockIdx.x * BC;
    const int yr0 = e.ymin + blockIdx.y * TY;
    const int lofs = e.lofs, rofs = e.rofs;
    const uint8_t* Lfr = Lf + (size_t)f * W * H;
    const uint8_t* Rfr = Rf + (size_t)f * W * H;
    const int jmin = xl0 - W2;
    // left tile column c <- image column clamp(lofs + jmin + c, 0, W - 1)
    // (OpenCV's left clamp); right: clampR below, the tile starting at rbase
    auto clampR = [&](int j) { return clampi(j, -rofs, W - nd - rofs); };
    const int rbase = clampR(jmin);

    // staging: dword loads (two aligned dwords funnel-shifted per four bytes;
    // the prefilter buffers carry 64 bytes of tail padding), byte loads only
    // where a clamp falls inside the four / eight bytes.  One item = four left
    // pixels (-> four shifted dwords, one b128 store) or four right-view
    // dwords (bytes [4 i, 4 i + 8) of the row -> dword i of the four copies).
    auto load4 = [](const uint8_t* p) -> uint32_t {
        const uintptr_t a = (uintptr_t)p;
        const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
        return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
    };
    {
        const int NJ4 = NJP / 4;
        const int items = NRW * NJ4;
        int r = tid / NJ4, q = tid - r * NJ4;
        const int dr = 256 / NJ4, dq = 256 - dr * NJ4;
        for (int it = tid; it < items; it += 256) {
            const int yy = clampi(yr0 - W2 + r, 0, H - 1);
            const uint8_t* row = Lfr + (size_t)yy * W;
            const int x0 = lofs + jmin + 4 * q;
            uint32_t w;
            if (x0 >= 0 && x0 + 3 <= W - 1) {
                w = load4(row + x0);
            } else {
                w = 0;
                for (int b = 0; b < 4; b++) w |= (uint32_t)row[clampi(x0 + b, 0, W - 1)] << (8 * b);
            }
            w += 0x01010101u;  // prefiltered values <= 126: no carries
            *(uint4*)(Lt + r * NJP + 4 * q) =
                make_uint4(w & 0xffu, w & 0xff00u, w & 0xff0000u, w & 0xff000000u);
            q += dq;
            r += dr;
            if (q >= NJ4) {
                q -= NJ4;
                r++;
            }
        }
    }
    {
        const int NR4 = NRC / 4;
        const int items = NRW * NR4;
        int r = tid / NR4, i = tid - r * NR4;
        const int dr = 256 / NR4, di = 256 - dr * NR4;
        for (int it = tid; it < items; it += 256) {
            const int yy = clampi(yr0 - W2 + r, 0, H - 1);
            const uint8_t* row = Rfr + (size_t)yy * W;
            const int x0 = rofs + rbase + 4 * i;  // >= 0
            uint32_t lo, hi;
            if (x0 + 7 <= W - 1) {
                lo = load4(row + x0);
                hi = load4(row + x0 + 4);
            } else {
                lo = hi = 0;
                for (int b = 0; b < 4; b++) {
                    lo |= (uint32_t)row[min(x0 + b, W - 1)] << (8 * b);
                    hi |= (uint32_t)row[min(x0 + 4 + b, W - 1)] << (8 * b);
                }
            }
            lo += 0x01010101u;
            hi += 0x01010101u;
            uint32_t* d = (uint32_t*)Rp + r * NR4 + i;
            d[0] = lo;
            d[lay.copy / 4] = __builtin_amdgcn_alignbyte(hi, lo, 1);
            d[2 * (lay.copy / 4)] = __builtin_amdgcn_alignbyte(hi, lo, 2);
            d[3 * (lay.copy / 4)] = __builtin_amdgcn_alignbyte(hi, lo, 3);
            i += di;
            r += dr;
            if (i >= NR4) {
                i -= NR4;
                r++;
            }
        }
    }

    const int c0 = cg * kBm2Cols;  // the group's first virtual column in the tile
    const int rows = min(TY, e.ymax - yr0);
    // right-tile column of virtual column v: rcol(v) = clampR(jmin + c0 + v) - rbase
    // (wave-uniform).  Groups without a clamp inside their NC columns address
    // it as rcol(0) + v through the shifted copies; the others read rcol(v)
    // byte by byte.
    const int cr0 = clampR(jmin + c0) - rbase;
    const bool lin = clampR(jmin + c0 + NC - 1) - rbase == cr0 + NC - 1;
    const int kl = lane + 64 * g;  // this lane's disparity index in the column-sum phase
    const uint32_t pad = kl < nd ? 0u : kBm2Pad;
    const int rb = cr0 + kl;  // lin: right byte of virtual column v = rb + v
    const uint32_t* Rq = (const uint32_t*)(Rp + (rb & 3) * lay.copy) + (rb >> 2);
    const uint32_t capsh = (uint32_t)(e.cap + 1) << (8 * ((c0 + lane) & 3));
    __syncthreads();

    // argmin phase: output column qx of the group (LPC lanes each), sub-lane h
    // scans the disparity indices [16 h, 16 h + 16)
    constexpr int LPC = 4 * NR, CPW = kBm2Cols / NR;
    const int qx = g * CPW + lane / LPC, h = lane % LPC;

    uint32_t cs[NC];
    uint32_t tc = 0;  // texture column sum of virtual column `lane` (lanes < NC)
    auto colsums = [&](auto LIN, auto INIT, int t) {
        constexpr bool kLin = decltype(LIN)::value;
        // |L - R| of row r, virtual column v, added to acc
        auto absd = [&](int r, int v, uint32_t lw, uint32_t acc) -> uint32_t {
            if constexpr (kLin) {
                return __builtin_amdgcn_msad_u8(Rq[r * (NRC / 4) + (v >> 2)], lw, acc);
            } else {
                // opaque row base: keeps the compiler from hoisting one
                // address register per column out of the row loop
                uint32_t rowo = (uint32_t)(lay.off_r + kl + r * NRC);  // byte offset in smem
                asm volatile("" : "+v"(rowo));
                const uint32_t rbyte = smem[rowo + (uint32_t)(clampR(jmin + c0 + v) - rbase)];
                return __builtin_amdgcn_msad_u8(rbyte << (8 * (v & 3)), lw, acc);
            }
        };
        if constexpr (decltype(INIT)::value) {
#pragma unroll
            for (int v = 0; v < NC; v++) cs[v] = pad;
#pragma unroll 1
            for (int r = 0; r < win; r++) {
                const uint32_t* Lr = Lt + r * NJP + c0;
#pragma unroll
                for (int v = 0; v < NC; v++) cs[v] = absd(r, v, Lr[v], cs[v]);
                tc = __builtin_amdgcn_sad_u8(Lr[lane], capsh, tc);
            }
        } else {
            const int rn = t + win - 1, ro = t - 1;
            const uint32_t* Ln = Lt + rn * NJP + c0;
            const uint32_t* Lo = Lt + ro * NJP + c0;
            tc = __builtin_amdgcn_sad_u8(Ln[lane], capsh, tc) - __builtin_amdgcn_sad_u8(Lo[lane], capsh, 0u);
#pragma unroll
            for (int v = 0; v < NC; v++) {
                const uint32_t add = absd(rn, v, Ln[v], cs[v]);
                cs[v] = add - absd(ro, v, Lo[v], 0u);
                // bound the LDS loads the scheduler hoists (registers)
                if ((v & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        }
    };
    auto group_sync = [&]() {
        if constexpr (NR == 1) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        } else {
            __syncthreads();
        }
    };
    auto wave_sync = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // output records: rows t0 .. t0 + cnt - 1 of the wave's CPW columns; lane
    // (slot, column) = (lane / CPW, lane % CPW)
    constexpr int RB = LPC;  // rows per flush: RB * CPW = 64
    auto flush = [&](int t0, int cnt) {
        wave_sync();  // the h == 0 lanes' records
        const int slot = lane / CPW, qf = g * CPW + lane % CPW;
        const int xf = xl0 + c0 + qf, xi = lofs + xf;
        if (slot < cnt && xf < e.ncol) {
            const uint2 r = recs[lane];
            const int y = yr0 + t0 + slot;
            const int mind = (int)(r.x & 0xffu);
            const int minsad = (int)((r.x & 0x3fffffffu) >> 8);
            int16_t res = (int16_t)e.filtered;
            const bool fail = (!keep_border && (xi < e.xmin || xi >= e.xmax)) || (r.x >> 30) != 0;
            if (!fail) {
                const int pp = (int)(r.y & 0xffffu), nn = (int)(r.y >> 16);
                const int v1 = nd - mind - 1 + e.mindisp;
                int val;
                if (0 < mind && mind < nd - 1) {
                    const int d = pp + nn - 2 * minsad + abs(pp - nn);
                    val = (v1 * 256 + (d != 0 ? (pp - nn) * 256 / d : 0) + 15) >> 4;
                } else {
                    val = (v1 * 256 + 15) >> 4;
                }
                res = (int16_t)val;
                if (cost) cost[((size_t)f * H + y) * W + xi] = minsad;
            }
            out[f * ofs + (size_t)y * os + xi] = res;
        }
    };
    // one row's window SADs, argmin, tests and output
    auto row_out = [&](int t) {
        // window SADs of the group's 16 output columns -> slab [column][disparity]
        {
            uint32_t sum = 0;
#pragma unroll
            for (int v = 0; v < win; v++) sum += cs[v];
            sadx[g * 64 + lane] = sum;
#pragma unroll
            for (int x = 1; x < kBm2Cols; x++) {
                sum += cs[x + win - 1];
                sum -= cs[x - 1];
                sadx[x * SS + g * 64 + lane] = sum;
            }
        }
        tcb[lane] = (int)tc;
        group_sync();
        uint32_t* srow = sadx + qx * SS;
        const int k0 = h * 16;
        // argmin over this lane's 16 slab entries, keys (sad << 8) | index
        uint32_t best;
        {
            uint32_t key[16];
#pragma unroll
            for (int i = 0; i < 16; i += 4) {
                const uint4 w = *(const uint4*)(srow + k0 + i);
                key[i] = (w.x << 8) | (uint32_t)i;
                key[i + 1] = (w.y << 8) | (uint32_t)(i + 1);
                key[i + 2] = (w.z << 8) | (uint32_t)(i + 2);
                key[i + 3] = (w.w << 8) | (uint32_t)(i + 3);
            }
            best = min(key[0], key[1]);
#pragma unroll
            for (int i = 2; i < 16; i += 2) best = min(min(best, key[i]), key[i + 1]);
            best |= (uint32_t)k0;
        }
        best = min(best, (uint32_t)__builtin_amdgcn_mov_dpp((int)best, 0xB1, 0xf, 0xf, false));
        best = min(best, (uint32_t)__builtin_amdgcn_mov_dpp((int)best, 0x4E, 0xf, 0xf, false));
        if constexpr (NR == 2)  // row_half_mirror: quad 0 <-> quad 1 of each 8 lanes
            best = min(best, (uint32_t)__builtin_amdgcn_mov_dpp((int)best, 0x141, 0xf, 0xf, false));
        const int mind = (int)(best & 0xff);
        const uint32_t minsad = best >> 8;
        // parabola neighbours (read before the uniqueness pass masks them)
        const int pp = (int)srow[min(mind + 1, 64 * NR - 1)];
        const int nn = (int)srow[max(mind - 1, 0)];
        bool bad = false;
        if (e.uniq > 0) {
            const uint32_t ms = minsad;
            const uint32_t thresh = ms + (uint32_t)((int)ms * e.uniq / 100);
            wave_sync();  // every lane of the column has read the slab row
            if (h == 0) {
                srow[mind] = 0xffffffffu;
                if (mind > 0) srow[mind - 1] = 0xffffffffu;
                if (mind + 1 < 64 * NR) srow[mind + 1] = 0xffffffffu;
            }
            wave_sync();
            uint32_t m2 = 0xffffffffu;
#pragma unroll
            for (int i = 0; i < 16; i += 4) {
                const uint4 w = *(const uint4*)(srow + k0 + i);
                m2 = min(min(m2, w.x), w.y);
                m2 = min(min(m2, w.z), w.w);
            }
            m2 = min(m2, (uint32_t)__builtin_amdgcn_mov_dpp((int)m2, 0xB1, 0xf, 0xf, false));
            m2 = min(m2, (uint32_t)__builtin_amdgcn_mov_dpp((int)m2, 0x4E, 0xf, 0xf, false));
            if constexpr (NR == 2)
                m2 = min(m2, (uint32_t)__builtin_amdgcn_mov_dpp((int)m2, 0x141, 0xf, 0xf, false));
            bad = m2 <= thresh;
        }
        int tsum = 0;
#pragma unroll
        for (int qq = 0; qq < win; qq++) tsum += tcb[qx + qq];
        // park the column's verdict; every RB rows the wave's 64 lanes finish
        // RB x CPW pixels at once (division, stores) instead of 16 / NR lanes
        // per row
        if (h == 0)
            recs[(t & (RB - 1)) * CPW + lane / LPC] =
                make_uint2(best | (bad ? 1u << 31 : 0u) | (tsum < e.tex ? 1u << 30 : 0u),
                           ((uint32_t)pp & 0xffffu) | ((uint32_t)nn << 16));
        if ((t & (RB - 1)) == RB - 1 || t == rows - 1) flush(t & ~(RB - 1), (t & (RB - 1)) + 1);
        group_sync();
    };
    // the whole row walk per addressing variant (no register copies between
    // variants at the loop back edge); row 0 builds the column sums
    auto walk = [&](auto LIN) {
        colsums(LIN, std::true_type(), 0);
        row_out(0);
        for (int t = 1; t < rows; t++) {
            colsums(LIN, std::false_type(), t);
            row_out(t);
        }
    };
    if (lin)
        walk(std::true_type());
    else
        walk(std::false_type());
}

// [OpenCV] validateDisparity, one block per valid row: the right-view winner
// per x2 is the smallest cost, ties -> the smallest x (first in the scan).
__global__ __launch_bounds__(256) void bm_validate_kernel(int16_t* __restrict__ out, size_t os,
                                                          size_t ofs, const int* __restrict__ cost,
                                                          int W, int H, BmEff e)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned long long* key = (unsigned long long*)smem;
    int16_t* d2 = (int16_t*)(key + W);
    const int y = e.ymin + blockIdx.x;
    const int f = blockIdx.y;
    int16_t* row = out + f * ofs + (size_t)y * os;
    const int* crow = cost + ((size_t)f * H + y) * W;
    const int minD = e.mindisp, maxD = minD + e.ndisp;
    const int minX1 = max(maxD, 0), maxX1 = W + min(minD, 0);
    const int INV = (minD - 1) * kDispScale;
    const int d12 = e.disp12 * kDispScale;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        key[x] = ~0ull;
        d2[x] = (int16_t)INV;
    }
    __syncthreads();
    for (int x = minX1 + threadIdx.x; x < maxX1; x += blockDim.x) {
        int d = row[x];
        if (d == INV) continue;
        int x2 = x - ((d + kDispScale / 2) >> kDispShift);
        if (x2 < 0 || x2 >= W) continue;
        unsigned long long k = ((unsigned long long)(unsigned)crow[x] << 32) | (unsigned)x;
        atomicMin(key + x2, k);
    }
    __syncthreads();
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        unsigned long long k = key[x];
        if (k != ~0ull) d2[x] = row[(int)(k & 0xffffffffu)];
    }
    __syncthreads();
    // every thread reads the pre-validation values of its own x only
    for (int x = minX1 + threadIdx.x; x < maxX1; x += blockDim.x) {
        int d = row[x];
        if (d == INV) continue;
        int dl = d >> kDispShift, dh = (d + kDispScale - 1) >> kDispShift;
        int xl = x - dl, xh = x - dh;
        if ((0 <= xl && xl < W && d2[xl] > INV && abs(d2[xl] - d) > d12) &&
            (0 <= xh && xh < W && d2[xh] > INV && abs(d2[xh] - d) > d12))
            row[x] = (int16_t)INV;
    }
}

__global__ void bm_roi_kernel(int16_t* __restrict__ out, size_t os, size_t ofs, int W, BmEff e)
{
    const int y = e.ymin + blockIdx.x, f = blockIdx.y;
    int16_t* row = out + f * ofs + (size_t)y * os;
    for (int x = threadIdx.x; x < W; x += blockDim.x)
        if (x < e.xmin || x >= e.xmax) row[x] = (int16_t)e.filtered;
}

}  // namespace

static int bm_finish(mvsv_ctx* ctx, int n, int W, int H, const BmEff& e, int16_t* out, size_t os,
                     size_t ofs, int* cost);

int bm_device(mvsv_ctx* ctx, int n, const uint8_t* L, size_t ls, size_t lfs, const uint8_t* R,
              size_t rs, size_t rfs, int W, int H, const BmEff& e, int16_t* out, size_t os,
              size_t ofs)
{
    hipStream_t s = ctx->stream;
    int rc;
    hipLaunchKernelGGL(bm_fill_kernel, dim3(H, n), dim3(256), 0, s, out, os, ofs, W, H,
                       (int16_t)e.filtered);
    if ((rc = check_hip(ctx, hipGetLastError(), "bm fill"))) return rc;
    if (e.lofs >= W || e.rofs >= W || e.width1 < 1) return MVSV_OK;
    if (e.xmax - e.xmin <= 0 || e.ymax - e.ymin <= 0 || e.ncol <= 0) return MVSV_OK;
    const size_t plane = (size_t)W * H;
    // + 64: the match kernel's staging reads whole aligned dwords past a row end
    if ((rc = ensure(ctx, ctx->bm_lf, (size_t)n * plane + 64, "bm left prefilter"))) return rc;
    if ((rc = ensure(ctx, ctx->bm_rf, (size_t)n * plane + 64, "bm right prefilter"))) return rc;
    uint8_t* Lf = (uint8_t*)ctx->bm_lf.ptr;
    uint8_t* Rf = (uint8_t*)ctx->bm_rf.ptr;
    if (e.prefilter_type == MVSV_PREFILTER_XSOBEL) {
        hipLaunchKernelGGL(bm_xsobel_kernel, dim3(H, n), dim3(256), 0, s, L, ls, lfs, W, H, e.cap, Lf);
        hipLaunchKernelGGL(bm_xsobel_kernel, dim3(H, n), dim3(256), 0, s, R, rs, rfs, W, H, e.cap, Rf);
    } else {
        const size_t lds = (size_t)(W + e.prefilter_size) * sizeof(int);
        if (lds > 160 * 1024) return set_error(ctx, MVSV_E_INVALID_ARG, "image too wide for the prefilter");
        if (lds > 65536 &&
            (rc = check_hip(ctx, hipFuncSetAttribute((const void*)bm_prefilter_norm_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                            "bm prefilter LDS attribute")))
            return rc;
        hipLaunchKernelGGL(bm_prefilter_norm_kernel, dim3(H, n), dim3(256), lds, s, L, ls, lfs, W, H,
                           e.prefilter_size, e.cap, Lf);
        hipLaunchKernelGGL(bm_prefilter_norm_kernel, dim3(H, n), dim3(256), lds, s, R, rs, rfs, W, H,
                           e.prefilter_size, e.cap, Rf);
    }

    const bool validate = e.disp12 >= 0;
    int* cost = nullptr;
    if (validate) {
        if ((rc = ensure(ctx, ctx->bm_cost, (size_t)n * plane * 4, "bm cost map"))) return rc;
        cost = (int*)ctx->bm_cost.ptr;
    }
    const int win = 2 * e.wsz2 + 1;
    // disparities on the lanes (bm_match2_kernel) for blockSize <= 21 and
    // numDisparities <= 128; the 16x16-tile kernel otherwise
    if (ctx->bm2 && e.wsz2 >= 2 && e.wsz2 <= 10 && e.ndisp <= 128) {
        const int NR = e.ndisp > 64 ? 2 : 1;
        const int BC = kBm2Waves / NR * kBm2Cols;
        const int gx = (e.ncol + BC - 1) / BC, nrows = e.ymax - e.ymin;
        typedef void (*Bm2Fn)(const uint8_t*, const uint8_t*, int, int, BmEff, int, int, int16_t*,
                              size_t, size_t, int*);
        static const Bm2Fn fns[2][9] = {
            {bm_match2_kernel<1, 2>, bm_match2_kernel<1, 3>, bm_match2_kernel<1, 4>,
             bm_match2_kernel<1, 5>, bm_match2_kernel<1, 6>, bm_match2_kernel<1, 7>,
             bm_match2_kernel<1, 8>, bm_match2_kernel<1, 9>, bm_match2_kernel<1, 10>},
            {bm_match2_kernel<2, 2>, bm_match2_kernel<2, 3>, bm_match2_kernel<2, 4>,
             bm_match2_kernel<2, 5>, bm_match2_kernel<2, 6>, bm_match2_kernel<2, 7>,
             bm_match2_kernel<2, 8>, bm_match2_kernel<2, 9>, bm_match2_kernel<2, 10>}};
        const Bm2Fn kern = fns[NR - 1][e.wsz2 - 2];
        // resident blocks per CU from the kernel's registers (4 waves per
        // block, one per SIMD; 512 VGPRs per SIMD lane)
        static int vgpr_blocks_of[2][9];  // 0 = not queried yet (same value on every gfx950)
        int vgpr_blocks = vgpr_blocks_of[NR - 1][e.wsz2 - 2];
        if (vgpr_blocks <= 0) {
            hipFuncAttributes fa;
            vgpr_blocks = 4;
            if (hipFuncGetAttributes(&fa, (const void*)kern) == hipSuccess && fa.numRegs > 0)
                vgpr_blocks = std::max(1, std::min(8, 512 / ((fa.numRegs + 7) & ~7)));
            else
                (void)hipGetLastError();
            vgpr_blocks_of[NR - 1][e.wsz2 - 2] = vgpr_blocks;
        }
        // tile height: rounds of resident blocks x (rows + start-up of the
        // window, ~win / 4 + 1 rows), with a penalty for fewer than four
        // resident blocks per CU (the kernel hides LDS latency with waves);
        // fitted to configs 1 / 2 at batch 1 and 8 (tools/bm_time.py sweep)
        int TY = ctx->bm_ty;
        if (TY <= 0) {
            double best = 1e30;
            for (int ty = 4; ty <= 64; ty += 4) {
                const size_t bytes = bm2_layout(e.wsz2, ty, NR).bytes;
                if (bytes > 160 * 1024) break;
                // LDS is handed out in 2 KiB steps (measured: 54 208 B per block
                // gives two resident blocks, not three)
                const long long k =
                    std::min<long long>(vgpr_blocks, (160 * 1024) / (long long)((bytes + 2047) & ~(size_t)2047));
                const long long blocks = (long long)gx * ((nrows + ty - 1) / ty) * n;
                const long long rounds = (blocks + ctx->cus * k - 1) / (ctx->cus * k);
                const double c = rounds * (ty + win * 0.25 + 1) * std::pow(4.0 / std::min<long long>(k, 4), 0.6);
                if (c < best - 1e-9) {
                    best = c;
                    TY = ty;
                }
            }
        }
        const Bm2Layout l2 = bm2_layout(e.wsz2, TY, NR);
        if (l2.bytes > 160 * 1024)
            return set_error(ctx, MVSV_E_INVALID_ARG, "BM tile height too large for LDS");
        if (l2.bytes > 65536 &&
            (rc = check_hip(ctx, hipFuncSetAttribute((const void*)kern,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)l2.bytes),
                            "bm LDS attribute")))
            return rc;
        dim3 grid2(gx,
                   (e.ymax - e.ymin + TY - 1) / TY, n);
        {
            StageTimer tm(ctx, kStageBm);
            hipLaunchKernelGGL(kern, grid2, dim3(256), l2.bytes, s, Lf, Rf, W, H, e, validate ? 1 : 0, TY,
                               out, os, ofs, cost);
        }
        if ((rc = check_hip(ctx, hipGetLastError(), "bm match"))) return rc;
        return bm_finish(ctx, n, W, H, e, out, os, ofs, cost);
    }
    const bool small = (long long)win * win * 2 * e.cap <= 65535;
    BmLayout lay = bm_layout(e.ndisp, e.wsz2, small ? 2 : 4);
    dim3 grid((e.ncol + 15) / 16, (e.ymax - e.ymin + 15) / 16, n);
    void* gsad = nullptr;
    size_t lds = lay.bytes;
    // row tiles per launch (all of them unless the window sums go to scratch)
    int rows_per_launch = (int)grid.y;
    if (lay.bytes > 160 * 1024) {
        // window sums in a global scratch slab per block (the LDS keeps the
        // tiles); launches of at most kBmScratchBytes of slab, one frame and a
        // band of row tiles each, reuse the slab in stream order
        lds = lay.off_sad;
        const size_t per_block = (size_t)e.ndisp * 256 * (small ? 2 : 4);
        const size_t per_row = per_block * grid.x;
        rows_per_launch = (int)std::max<size_t>(1, std::min<size_t>(grid.y, kBmScratchBytes / per_row));
        if ((rc = ensure(ctx, ctx->bm_sad, per_row * rows_per_launch, "bm window-sum scratch"))) return rc;
        gsad = ctx->bm_sad.ptr;
    }
    if (lds > 160 * 1024)
        return set_error(ctx, MVSV_E_INVALID_ARG, "blockSize too large for the GPU BM kernel");
    if (lds > 65536) {
        const void* fn = small ? (const void*)bm_match_kernel<uint16_t>
                               : (const void*)bm_match_kernel<uint32_t>;
        if ((rc = check_hip(ctx, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)lds),
                            "bm LDS attribute")))
            return rc;
    }
    StageTimer tm(ctx, kStageBm);
    if (!gsad) {
        if (small)
            hipLaunchKernelGGL(bm_match_kernel<uint16_t>, grid, dim3(256), lds, s, Lf, Rf, W, H,
                               e, validate ? 1 : 0, out, os, ofs, cost, (uint16_t*)nullptr, 0, 0);
        else
            hipLaunchKernelGGL(bm_match_kernel<uint32_t>, grid, dim3(256), lds, s, Lf, Rf, W, H,
                               e, validate ? 1 : 0, out, os, ofs, cost, (uint32_t*)nullptr, 0, 0);
    } else {
        for (int f = 0; f < n; f++)
            for (int by = 0; by < (int)grid.y; by += rows_per_launch) {
                const dim3 g(grid.x, std::min(rows_per_launch, (int)grid.y - by), 1);
                if (small)
                    hipLaunchKernelGGL(bm_match_kernel<uint16_t>, g, dim3(256), lds, s, Lf, Rf, W, H, e,
                                       validate ? 1 : 0, out, os, ofs, cost, (uint16_t*)gsad, by, f);
                else
                    hipLaunchKernelGGL(bm_match_kernel<uint32_t>, g, dim3(256), lds, s, Lf, Rf, W, H, e,
                                       validate ? 1 : 0, out, os, ofs, cost, (uint32_t*)gsad, by, f);
            }
    }
    if ((rc = check_hip(ctx, hipGetLastError(), "bm match"))) return rc;
    return bm_finish(ctx, n, W, H, e, out, os, ofs, cost);
}

// validateDisparity + ROI + speckle after either match kernel
static int bm_finish(mvsv_ctx* ctx, int n, int W, int H, const BmEff& e, int16_t* out, size_t os,
                     size_t ofs, int* cost)
{
    hipStream_t s = ctx->stream;
    int rc;
    const bool validate = e.disp12 >= 0;
    if (validate) {
        size_t lds = (size_t)W * 8 + (size_t)W * 2;
        hipLaunchKernelGGL(bm_validate_kernel, dim3(e.ymax - e.ymin, n), dim3(256), lds, s, out, os,
                           ofs, cost, W, H, e);
        hipLaunchKernelGGL(bm_roi_kernel, dim3(e.ymax - e.ymin, n), dim3(256), 0, s, out, os, ofs,
                           W, e);
        if ((rc = check_hip(ctx, hipGetLastError(), "bm validate"))) return rc;
    }
    if (e.speckle_range >= 0 && e.speckle_window > 0)
        return speckle_device(ctx, n, out, os, ofs, W, H, e.filtered, e.speckle_window,
                              e.speckle_range);
    return MVSV_OK;
}

}  // namespace mvsv
