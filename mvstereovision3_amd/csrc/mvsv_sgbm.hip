// mvsv_sgbm.hip — StereoSGBM on MI355X (gfx950).
//
// Replaces Disparity::sgbm (src/disparity.cpp:6-10) -> cv::StereoSGBM::compute.
// Pipeline per batch of frames (all launches on the context stream):
//   1. sgbm_prefilter_kernel   clipped x-Sobel + raw channel per row    (u8 planes)
//   2. sgbm_cost_kernel        Birchfield-Tomasi pixel cost + bs x bs box
//                              sum -> C[y][x][d] int16 (+P2 bias), LDS-staged
//                              rows, running vertical sums in registers
//   3. sgbm_cost_fixup_kernel  OpenCV 3.4's cost-row quirks (column x=0 and
//                              the bottom SH2 rows are not refreshed)
//   4. sgbm_path_kernel        one wave per scanline of one direction: the
//                              SGM recurrence on packed int16 pairs
//                              (v_pk_*_i16), d+-1 neighbours via DPP
//                              wave_shr/shl, per-step min over d via a DPP
//                              butterfly; S += L with int16 saturation
//   5. sgbm_final_kernel       the last direction (R->L) fused with WTA,
//                              uniqueness, sub-pixel fit, right-view map and
//                              the left-right check (one wave per row)
//   6. median 3x3 + optional speckle filter (mvsv_post.hip)
// Data layout in HBM: C and S are [frame][y][x][d] int16 with d contiguous,
// so one cost column (D = 128 -> 256 B) is one coalesced wave access.
#include <algorithm>

#include "mvsv_device.hpp"
#include "mvsv_internal.hpp"

namespace mvsv {
namespace {

using namespace dev;

// ---------------------------------------------------------------------------
// 1. prefilter: planes [frame][4][H][W] = L sobel, L raw, R sobel, R raw.
// [OpenCV] calcPixelCostBT: tab[(r[x+1]-r[x-1])*2 + rn[x+1]-rn[x-1] + rs[x+1]-rs[x-1]],
// columns 0 and W-1 of both channels = tab[0] = ftzero.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sgbm_prefilter_kernel(
    const uint8_t* __restrict__ L, size_t ls, size_t lfs, const uint8_t* __restrict__ R,
    size_t rs, size_t rfs, int W, int H, int ftzero, uint8_t* __restrict__ pre)
{
    const int y = blockIdx.x;
    const int f = blockIdx.y;
    const uint8_t* l = L + f * lfs;
    const uint8_t* r = R + f * rfs;
    const size_t plane = (size_t)W * H;
    uint8_t* o = pre + (size_t)f * 4 * plane + (size_t)y * W;
    const int yn = y > 0 ? y - 1 : y, ys = y < H - 1 ? y + 1 : y;
    const uint8_t* l0 = l + (size_t)y * ls;
    const uint8_t* ln = l + (size_t)yn * ls;
    const uint8_t* lsr = l + (size_t)ys * ls;
    const uint8_t* r0 = r + (size_t)y * rs;
    const uint8_t* rn = r + (size_t)yn * rs;
    const uint8_t* rsr = r + (size_t)ys * rs;
    const uint8_t fz = (uint8_t)ftzero;
    for (int x = threadIdx.x; x < W; x += blockDim.x) {
        uint8_t a = fz, b = fz, c = fz, d = fz;
        if (x > 0 && x < W - 1) {
            int gl = (l0[x + 1] - l0[x - 1]) * 2 + ln[x + 1] - ln[x - 1] + lsr[x + 1] - lsr[x - 1];
            int gr = (r0[x + 1] - r0[x - 1]) * 2 + rn[x + 1] - rn[x - 1] + rsr[x + 1] - rsr[x - 1];
            a = (uint8_t)(clampi(gl, -ftzero, ftzero) + ftzero);
            b = l0[x];
            c = (uint8_t)(clampi(gr, -ftzero, ftzero) + ftzero);
            d = r0[x];
        }
        o[x] = a;
        o[plane + x] = b;
        o[2 * plane + x] = c;
        o[3 * plane + x] = d;
    }
}

// ---------------------------------------------------------------------------
// 2. cost volume.
// Block = 256 threads owns cost columns [x0, x0+TX) x rows [y0, y0+TY) x all d.
// For each (clamped) source row it stages the BT intervals of the needed left /
// right columns in LDS, computes the pixel cost of TX + 2*SW2 columns, the
// horizontal box sum of its cells, and keeps the vertical window sum of its
// cells in registers (ring of the last 2*SH2+1 horizontal sums in LDS).
// ---------------------------------------------------------------------------
struct CostLayout {
    int TX, TY, NX, NR, nLmax, nRmax;
    size_t off_r, off_pix, off_ring, bytes;
};

__host__ __device__ inline CostLayout cost_layout(int D, int SW2, int SH2, int CPT, int TY)
{
    CostLayout c;
    c.TX = (256 * CPT) / D;
    if (c.TX < 1) c.TX = 1;
    c.TY = TY;
    c.NX = c.TX + 2 * SW2;
    c.NR = 2 * SH2 + 1;
    c.nLmax = c.NX;
    c.nRmax = c.NX + D;
    c.off_r = (size_t)c.nLmax * 8;
    c.off_pix = c.off_r + (size_t)c.nRmax * 8;
    size_t pix = (size_t)c.NX * D * 2;
    c.off_ring = (c.off_pix + pix + 15) & ~(size_t)15;
    c.bytes = c.off_ring + (size_t)c.NR * c.TX * D * 2;
    return c;
}

// BT interval of one column of one channel: val | lo << 8 | hi << 16.
__device__ __forceinline__ uint32_t bt_pack(const uint8_t* row, int x, int W)
{
    int v = row[x];
    int l = x > 0 ? (v + row[x - 1]) >> 1 : v;
    int r = x < W - 1 ? (v + row[x + 1]) >> 1 : v;
    int lo = min(min(l, r), v), hi = max(max(l, r), v);
    return (uint32_t)v | ((uint32_t)lo << 8) | ((uint32_t)hi << 16);
}

__device__ __forceinline__ int bt_cost(uint32_t a, uint32_t b)
{
    int u = a & 255, u0 = (a >> 8) & 255, u1 = (a >> 16) & 255;
    int v = b & 255, v0 = (b >> 8) & 255, v1 = (b >> 16) & 255;
    int c0 = max(max(0, u - v1), v0 - u);
    int c1 = max(max(0, v - u1), u0 - v);
    return min(c0, c1);
}

template <int CPT>
__global__ __launch_bounds__(256) void sgbm_cost_kernel(const uint8_t* __restrict__ pre, int W,
                                                        int H, SgbmEff e, int TY,
                                                        int16_t* __restrict__ C)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int D = e.D, W1 = e.W1, SW2 = e.SW2, SH2 = e.SH2;
    const CostLayout lay = cost_layout(D, SW2, SH2, CPT, TY);
    const int TX = lay.TX, NX = lay.NX, NR = lay.NR;
    const int f = blockIdx.z;
    const int x0 = blockIdx.x * TX, y0 = blockIdx.y * TY;
    const int y1 = min(y0 + TY, H);
    const int xclo = max(x0 - SW2, 0), xchi = min(x0 + TX + SW2 - 1, W1 - 1);
    const int nL = xchi - xclo + 1;
    const int ilo = e.minX1 + xclo;                  // first left image column
    const int rlo = ilo - (e.maxD - 1);              // first right image column
    const int nR = (e.minX1 + xchi - e.minD) - rlo + 1;
    uint64_t* lpk = (uint64_t*)smem;
    uint64_t* rpk = (uint64_t*)(smem + lay.off_r);
    int16_t* pixrow = (int16_t*)(smem + lay.off_pix);
    int16_t* ring = (int16_t*)(smem + lay.off_ring);
    const size_t plane = (size_t)W * H;
    const uint8_t* P = pre + (size_t)f * 4 * plane;
    const int tid = threadIdx.x;
    const int ncell = TX * D;

    int csum[CPT];
#pragma unroll
    for (int i = 0; i < CPT; i++) csum[i] = 0;

    const int vstart = y0 - SH2, vend = y1 + SH2;
    for (int v = vstart; v < vend; v++) {
        const int r = clampi(v, 0, H - 1);
        const uint8_t* Ls = P + (size_t)r * W;
        const uint8_t* Lr = Ls + plane;
        const uint8_t* Rs = Ls + 2 * plane;
        const uint8_t* Rr = Ls + 3 * plane;
        for (int i = tid; i < nL; i += 256) {
            int x = ilo + i;
            lpk[i] = (uint64_t)bt_pack(Ls, x, W) | ((uint64_t)bt_pack(Lr, x, W) << 32);
        }
        for (int i = tid; i < nR; i += 256) {
            int x = rlo + i;
            uint64_t val = 0;
            if (x >= 0 && x < W)
                val = (uint64_t)bt_pack(Rs, x, W) | ((uint64_t)bt_pack(Rr, x, W) << 32);
            rpk[i] = val;
        }
        __syncthreads();
        for (int idx = tid; idx < NX * D; idx += 256) {
            int xv = idx / D;
            int d = idx - xv * D;
            int xc = clampi(x0 - SW2 + xv, 0, W1 - 1);
            int li = xc - xclo;
            int rj = (e.minX1 + xc - (d + e.minD)) - rlo;
            uint64_t a = lpk[li], b = rpk[rj];
            int pc = bt_cost((uint32_t)a, (uint32_t)b) +
                     (bt_cost((uint32_t)(a >> 32), (uint32_t)(b >> 32)) >> 2);
            pixrow[idx] = (int16_t)pc;
        }
        __syncthreads();
        const int k = v - vstart;
        const int slot = k % NR;
        const bool emit = k >= NR - 1;
        const int y = v - SH2;
#pragma unroll
        for (int i = 0; i < CPT; i++) {
            int cell = tid + 256 * i;
            if (cell < ncell) {
                int tx = cell / D;
                int d = cell - tx * D;
                int h = 0;
                const int16_t* pr = pixrow + tx * D + d;
                for (int q = 0; q <= 2 * SW2; q++) h += pr[q * D];
                int16_t* rs = ring + slot * ncell + cell;
                if (k >= NR) csum[i] -= *rs;
                csum[i] += h;
                *rs = (int16_t)h;
                if (emit && x0 + tx < W1)
                    C[(((size_t)f * H + y) * W1 + x0 + tx) * D + d] = (int16_t)(e.P2 + csum[i]);
            }
        }
        __syncthreads();
    }
}

// 3. OpenCV 3.4 cost-row quirks (see oracle/twin.py sgbm_cost_volume):
//    rows y >= 1 never refresh column x = 0; rows with y + SH2 >= H are never
//    recomputed (MODE_SGBM keeps the last computed row, MODE_HH keeps P2).
__global__ __launch_bounds__(256) void sgbm_cost_fixup_kernel(int16_t* __restrict__ C, int H,
                                                              SgbmEff e, int ylast, int ybot)
{
    // blockIdx.x enumerates (row y >= 1), threads sweep x*D + d.
    const int y = 1 + blockIdx.x;
    const int f = blockIdx.y;
    const int D = e.D, W1 = e.W1;
    const bool fix = (e.variant & MVSV_VARIANT_FIRSTCOL_FIX) != 0;
    const bool bottom = y >= ybot;
    if (!bottom && fix) return;
    int16_t* Cf = C + (size_t)f * H * W1 * D;
    int16_t* row = Cf + (size_t)y * W1 * D;
    const int n = bottom ? W1 * D : D;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int x = i / D;
        int16_t val;
        if (e.fullDP) {
            val = (int16_t)e.P2;
        } else if (x == 0 && !fix) {
            val = Cf[i];  // C(0, 0, d)
        } else {
            val = Cf[(size_t)ylast * W1 * D + i];
        }
        row[i] = val;
    }
}

// ---------------------------------------------------------------------------
// 4. path aggregation along one direction (predecessor (x-dx, y-dy)).
// ---------------------------------------------------------------------------
struct Line {
    int xs, ys, len;
};

__device__ __forceinline__ Line line_geometry(int line, int dx, int dy, int W1, int H)
{
    Line g;
    if (dy == 0) {
        g.ys = line;
        g.xs = dx > 0 ? 0 : W1 - 1;
        g.len = W1;
    } else if (dx == 0) {
        g.xs = line;
        g.ys = dy > 0 ? 0 : H - 1;
        g.len = H;
    } else {
        const int ye = dy > 0 ? 0 : H - 1, xe = dx > 0 ? 0 : W1 - 1;
        if (line < W1) {
            g.xs = line;
            g.ys = ye;
        } else {
            g.xs = xe;
            g.ys = ye + dy * (line - W1 + 1);
        }
        int nx = dx > 0 ? W1 - g.xs : g.xs + 1;
        int ny = dy > 0 ? H - g.ys : g.ys + 1;
        g.len = min(nx, ny);
    }
    return g;
}

__host__ __device__ inline int num_lines(int dx, int dy, int W1, int H)
{
    return dy == 0 ? H : (dx == 0 ? W1 : W1 + H - 1);
}

template <int NP>
struct Vec;
template <>
struct Vec<1> {
    uint32_t v[1];
    __device__ __forceinline__ void load(const int16_t* p) { v[0] = *(const uint32_t*)p; }
    __device__ __forceinline__ void store(int16_t* p) const { *(uint32_t*)p = v[0]; }
};
template <>
struct Vec<2> {
    uint32_t v[2];
    __device__ __forceinline__ void load(const int16_t* p)
    {
        uint2 t = *(const uint2*)p;
        v[0] = t.x;
        v[1] = t.y;
    }
    __device__ __forceinline__ void store(int16_t* p) const { *(uint2*)p = make_uint2(v[0], v[1]); }
};
template <>
struct Vec<4> {
    uint32_t v[4];
    __device__ __forceinline__ void load(const int16_t* p)
    {
        uint4 t = *(const uint4*)p;
        v[0] = t.x;
        v[1] = t.y;
        v[2] = t.z;
        v[3] = t.w;
    }
    __device__ __forceinline__ void store(int16_t* p) const
    {
        *(uint4*)p = make_uint4(v[0], v[1], v[2], v[3]);
    }
};

// One SGM step for the NP packed pairs a lane owns.  lp: previous L (MAX in
// padded slots), delta = (int16)(minLp + P2) packed twice, c: cost C.
template <int NP>
__device__ __forceinline__ void sgm_step(const uint32_t (&lp)[NP], uint32_t delta2, uint32_t p1x2,
                                         const uint32_t (&c)[NP], const bool (&valid)[NP],
                                         uint32_t (&ln)[NP])
{
    const uint32_t MAXP = 0x7fff7fffu;
    const uint32_t prev_hi = wave_shr1(lp[NP - 1], MAXP);  // lane-1's last pair
    const uint32_t next_lo = wave_shl1(lp[0], MAXP);       // lane+1's first pair
#pragma unroll
    for (int p = 0; p < NP; p++) {
        uint32_t ph = p == 0 ? prev_hi : lp[p - 1];
        uint32_t nl = p == NP - 1 ? next_lo : lp[p + 1];
        uint32_t lm = __builtin_amdgcn_alignbit(lp[p], ph, 16);  // (L[d-1], L[d])
        uint32_t lq = __builtin_amdgcn_alignbit(nl, lp[p], 16);  // (L[d+1], L[d+2])
        uint32_t m = pk_min(lp[p], pk_add_sat(lm, p1x2));
        m = pk_min(m, pk_add_sat(lq, p1x2));
        m = pk_min(m, delta2);
        uint32_t r = pk_add_sat(pk_sub_sat(m, delta2), c[p]);
        ln[p] = valid[p] ? r : MAXP;
    }
}

template <int NP>
__device__ __forceinline__ int lane_min(const uint32_t (&ln)[NP])
{
    int m = 32767;
#pragma unroll
    for (int p = 0; p < NP; p++) m = min(m, min(lo16(ln[p]), hi16(ln[p])));
    return m;
}

constexpr int kPF = 4;  // software prefetch depth (steps)

template <int NP, bool ACC>
__global__ __launch_bounds__(256) void sgbm_path_kernel(const int16_t* __restrict__ C,
                                                        int16_t* __restrict__ S, int H, int W1,
                                                        int D, int dx, int dy, int P1, int P2)
{
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane keeps the line walk scalar
    const int line = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int f = blockIdx.y;
    if (line >= num_lines(dx, dy, W1, H)) return;
    const Line g = line_geometry(line, dx, dy, W1, H);
    const size_t frame = (size_t)H * W1 * D;
    const ptrdiff_t step = ((ptrdiff_t)dy * W1 + dx) * D;
    const int d0 = lane * 2 * NP;
    const size_t off = f * frame + ((size_t)g.ys * W1 + g.xs) * D + (d0 < D ? d0 : 0);
    const int16_t* cp = C + off;
    int16_t* sp = S + off;
    bool valid[NP];
    uint32_t lp[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        valid[p] = d0 + 2 * p < D;
        lp[p] = valid[p] ? 0u : 0x7fff7fffu;
    }
    const bool lane_on = d0 < D;
    const uint32_t p1x2 = (uint32_t)(P1 & 0xffff) * 0x10001u;
    int minp = 0;
    const int len = g.len;

    Vec<NP> cb[kPF], sb[kPF];
#pragma unroll
    for (int j = 0; j < kPF; j++) {
        if (j < len && lane_on) {
            cb[j].load(cp + j * step);
            if (ACC) sb[j].load(sp + j * step);
        }
    }
    for (int base = 0; base < len; base += kPF) {
#pragma unroll
        for (int j = 0; j < kPF; j++) {
            const int s = base + j;
            if (s >= len) break;
            const int dl = (int16_t)(minp + P2);
            const uint32_t delta2 = (uint32_t)(dl & 0xffff) * 0x10001u;
            uint32_t c[NP], ln[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) c[p] = cb[j].v[p];
            sgm_step<NP>(lp, delta2, p1x2, c, valid, ln);
            minp = wave_min_i32(lane_min<NP>(ln));
            if (lane_on) {
                Vec<NP> o;
#pragma unroll
                for (int p = 0; p < NP; p++) o.v[p] = ACC ? pk_add_sat(sb[j].v[p], ln[p]) : ln[p];
                o.store(sp + (ptrdiff_t)s * step);
                if (s + kPF < len) {
                    cb[j].load(cp + (ptrdiff_t)(s + kPF) * step);
                    if (ACC) sb[j].load(sp + (ptrdiff_t)(s + kPF) * step);
                }
            }
#pragma unroll
            for (int p = 0; p < NP; p++) lp[p] = ln[p];
        }
    }
}

// ---------------------------------------------------------------------------
// 5. last direction (R->L) + WTA + uniqueness + sub-pixel + LR check.
// ---------------------------------------------------------------------------
template <int NP>
__global__ __launch_bounds__(64) void sgbm_final_kernel(const int16_t* __restrict__ C,
                                                       const int16_t* __restrict__ S, int H,
                                                       int W, SgbmEff e,
                                                       int16_t* __restrict__ raw)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    int16_t* disp1 = (int16_t*)smem;
    int16_t* d2 = disp1 + W;
    int16_t* d2c = d2 + W;
    const int lane = threadIdx.x;
    const int y = blockIdx.x;
    const int f = blockIdx.y;
    const int D = e.D, W1 = e.W1, minD = e.minD, minX1 = e.minX1;
    const int INV = e.invalid;
    for (int x = lane; x < W; x += 64) {
        disp1[x] = (int16_t)INV;
        d2[x] = (int16_t)INV;
        d2c[x] = (int16_t)kMaxCost;
    }
    __syncthreads();

    const bool lane_rule = !e.fullDP && !(e.variant & MVSV_VARIANT_WTA_MIN_D);
    const size_t frame = (size_t)H * W1 * D;
    const int d0 = lane * 2 * NP;
    const bool lane_on = d0 < D;
    const size_t off = f * frame + ((size_t)y * W1 + (W1 - 1)) * D + (lane_on ? d0 : 0);
    const int16_t* cp = C + off;
    const int16_t* sp = S + off;
    bool valid[NP];
    uint32_t lp[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        valid[p] = d0 + 2 * p < D;
        lp[p] = valid[p] ? 0u : 0x7fff7fffu;
    }
    const uint32_t p1x2 = (uint32_t)(e.P1 & 0xffff) * 0x10001u;
    int minp = 0;
    const int uq = e.uniq;

    Vec<NP> cb[kPF], sb[kPF];
#pragma unroll
    for (int j = 0; j < kPF; j++) {
        if (j < W1 && lane_on) {
            cb[j].load(cp - (ptrdiff_t)j * D);
            sb[j].load(sp - (ptrdiff_t)j * D);
        }
    }
    for (int base = 0; base < W1; base += kPF) {
#pragma unroll
        for (int j = 0; j < kPF; j++) {
            const int s = base + j;
            if (s >= W1) break;
            const int x = W1 - 1 - s;
            const int dl = (int16_t)(minp + e.P2);
            const uint32_t delta2 = (uint32_t)(dl & 0xffff) * 0x10001u;
            uint32_t c[NP], ln[NP], st[NP];
#pragma unroll
            for (int p = 0; p < NP; p++) c[p] = cb[j].v[p];
            sgm_step<NP>(lp, delta2, p1x2, c, valid, ln);
            minp = wave_min_i32(lane_min<NP>(ln));
            // total aggregated cost and the WTA key of this lane
            int key = 0x7fffffff;
#pragma unroll
            for (int p = 0; p < NP; p++) {
                st[p] = valid[p] ? pk_add_sat(sb[j].v[p], ln[p]) : 0x7fff7fffu;
                if (valid[p]) {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        int d = d0 + 2 * p + h;
                        int sv = h ? hi16(st[p]) : lo16(st[p]);
                        int sub = lane_rule ? (((d & 7) << 12) | (d >> 3)) : d;
                        key = min(key, (sv << 16) | sub);
                    }
                }
            }
            if (lane_on && s + kPF < W1) {
                cb[j].load(cp - (ptrdiff_t)(s + kPF) * D);
                sb[j].load(sp - (ptrdiff_t)(s + kPF) * D);
            }
#pragma unroll
            for (int p = 0; p < NP; p++) lp[p] = ln[p];

            const int K = wave_min_i32(key);
            const int minS = K >> 16;
            const int sub = K & 0xffff;
            int best = lane_rule ? (((sub & 0xfff) << 3) | (sub >> 12)) : sub;
            if (minS >= kMaxCost) best = -1;  // no strict minimum below MAX_COST
            // uniqueness: some d with S[d]*(100-u) < minS*100 and |d-best| > 1
            bool rej = false;
#pragma unroll
            for (int p = 0; p < NP; p++) {
                if (valid[p]) {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        int d = d0 + 2 * p + h;
                        int sv = h ? hi16(st[p]) : lo16(st[p]);
                        rej |= (sv * (100 - uq) < minS * 100) && (abs(best - d) > 1);
                    }
                }
            }
            if (__ballot(rej) != 0ull) continue;
            // right-view map (x descending: the larger x wins ties)
            const int x2 = x + minX1 - best - minD;
            if (lane == 0 && x2 >= 0 && x2 < W && d2c[x2] > minS) {
                d2c[x2] = (int16_t)minS;
                d2[x2] = (int16_t)(best + minD);
            }
            int d16;
            if (0 < best && best < D - 1) {
                auto fetch = [&](int d) -> int {
                    int ln_ = d / (2 * NP), el = d - ln_ * 2 * NP;
                    uint32_t v = st[0];
#pragma unroll
                    for (int p = 1; p < NP; p++)
                        if ((el >> 1) == p) v = st[p];
                    uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)v, ln_);
                    return (el & 1) ? hi16(w) : lo16(w);
                };
                int Sm = fetch(best - 1), Sp = fetch(best + 1);
                int den = max(Sm + Sp - 2 * minS, 1);
                d16 = best * kDispScale + ((Sm - Sp) * kDispScale + den) / (den * 2);
            } else {
                d16 = best * kDispScale;
            }
            if (lane == 0) disp1[x + minX1] = (int16_t)(d16 + minD * kDispScale);
        }
    }
    __syncthreads();
    int16_t* out = raw + ((size_t)f * H + y) * W;
    for (int x = lane; x < W; x += 64) {
        int v = disp1[x];
        if (x >= minX1 && x < e.maxX1 && v != INV) {
            int dl = v >> kDispShift, dh = (v + kDispScale - 1) >> kDispShift;
            int xl = x - dl, xh = x - dh;
            if (0 <= xl && xl < W && d2[xl] >= minD && abs(d2[xl] - dl) > e.disp12 && 0 <= xh &&
                xh < W && d2[xh] >= minD && abs(d2[xh] - dh) > e.disp12)
                v = INV;
        }
        out[x] = (int16_t)v;
    }
}

__global__ void fill_s16_kernel(int16_t* __restrict__ out, size_t os, size_t ofs, int W, int H,
                                int16_t v)
{
    const int y = blockIdx.x, f = blockIdx.y;
    int16_t* o = out + f * ofs + (size_t)y * os;
    for (int x = threadIdx.x; x < W; x += blockDim.x) o[x] = v;
}

template <int NP>
int launch_paths(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, int16_t* Cv,
                 int16_t* Sv, int16_t* raw)
{
    hipStream_t s = ctx->stream;
    static const int dirs_sgbm[4][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}};
    static const int dirs_hh[7][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {1, -1}, {0, -1}, {-1, -1}};
    const int ndir = e.fullDP ? 7 : 4;
    for (int k = 0; k < ndir; k++) {
        int dx = e.fullDP ? dirs_hh[k][0] : dirs_sgbm[k][0];
        int dy = e.fullDP ? dirs_hh[k][1] : dirs_sgbm[k][1];
        int nl = num_lines(dx, dy, e.W1, H);
        dim3 grid((nl + 3) / 4, n);
        if (k == 0)
            hipLaunchKernelGGL((sgbm_path_kernel<NP, false>), grid, dim3(256), 0, s, Cv, Sv, H,
                               e.W1, e.D, dx, dy, e.P1, e.P2);
        else
            hipLaunchKernelGGL((sgbm_path_kernel<NP, true>), grid, dim3(256), 0, s, Cv, Sv, H,
                               e.W1, e.D, dx, dy, e.P1, e.P2);
    }
    size_t lds = (size_t)W * 3 * sizeof(int16_t);
    hipLaunchKernelGGL((sgbm_final_kernel<NP>), dim3(H, n), dim3(64), lds, s, Cv, Sv, H, W, e,
                       raw);
    return check_hip(ctx, hipGetLastError(), "sgbm path kernels");
}

}  // namespace

int sgbm_device(mvsv_ctx* ctx, int n, const uint8_t* L, size_t ls, size_t lfs, const uint8_t* R,
                size_t rs, size_t rfs, int W, int H, const SgbmEff& e, int16_t* out, size_t os,
                size_t ofs)
{
    hipStream_t s = ctx->stream;
    int rc;
    if (e.minX1 >= e.maxX1) {
        hipLaunchKernelGGL(fill_s16_kernel, dim3(H, n), dim3(256), 0, s, out, os, ofs, W, H,
                           (int16_t)e.invalid);
        return check_hip(ctx, hipGetLastError(), "sgbm fill");
    }
    if (e.D > 512) return set_error(ctx, MVSV_E_INVALID_ARG, "numDisparities > 512 not supported");
    const size_t plane = (size_t)W * H;
    const size_t vol = (size_t)e.W1 * H * e.D;
    if ((rc = ensure(ctx, ctx->pre, (size_t)n * 4 * plane, "sgbm prefilter planes"))) return rc;
    if ((rc = ensure(ctx, ctx->cost, (size_t)n * vol * 2, "sgbm cost volume"))) return rc;
    if ((rc = ensure(ctx, ctx->agg, (size_t)n * vol * 2, "sgbm aggregated cost"))) return rc;
    if ((rc = ensure(ctx, ctx->raw, (size_t)n * plane * 2, "sgbm raw disparity"))) return rc;
    uint8_t* pre = (uint8_t*)ctx->pre.ptr;
    int16_t* Cv = (int16_t*)ctx->cost.ptr;
    int16_t* Sv = (int16_t*)ctx->agg.ptr;
    int16_t* raw = (int16_t*)ctx->raw.ptr;

    hipLaunchKernelGGL(sgbm_prefilter_kernel, dim3(H, n), dim3(256), 0, s, L, ls, lfs, R, rs, rfs,
                       W, H, e.ftzero, pre);

    // cost volume: pick cells-per-thread so the LDS image stays <= 64 KiB
    const int TY = H >= 256 ? 48 : 16;
    int cpt = 8;
    CostLayout lay = cost_layout(e.D, e.SW2, e.SH2, cpt, TY);
    while (lay.bytes > 65536 && cpt > 1) {
        cpt >>= 1;
        lay = cost_layout(e.D, e.SW2, e.SH2, cpt, TY);
    }
    if (lay.bytes > 160 * 1024)
        return set_error(ctx, MVSV_E_INVALID_ARG, "blockSize too large for the GPU cost kernel");
    dim3 cgrid((e.W1 + lay.TX - 1) / lay.TX, (H + TY - 1) / TY, n);
    if (lay.bytes > 65536) {
        const void* fn = cpt == 8 ? (const void*)sgbm_cost_kernel<8>
                       : cpt == 4 ? (const void*)sgbm_cost_kernel<4>
                       : cpt == 2 ? (const void*)sgbm_cost_kernel<2>
                                  : (const void*)sgbm_cost_kernel<1>;
        if ((rc = check_hip(ctx, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)lay.bytes),
                            "sgbm cost LDS attribute")))
            return rc;
    }
    switch (cpt) {
    case 8: hipLaunchKernelGGL(sgbm_cost_kernel<8>, cgrid, dim3(256), lay.bytes, s, pre, W, H, e, TY, Cv); break;
    case 4: hipLaunchKernelGGL(sgbm_cost_kernel<4>, cgrid, dim3(256), lay.bytes, s, pre, W, H, e, TY, Cv); break;
    case 2: hipLaunchKernelGGL(sgbm_cost_kernel<2>, cgrid, dim3(256), lay.bytes, s, pre, W, H, e, TY, Cv); break;
    default: hipLaunchKernelGGL(sgbm_cost_kernel<1>, cgrid, dim3(256), lay.bytes, s, pre, W, H, e, TY, Cv); break;
    }
    if ((rc = check_hip(ctx, hipGetLastError(), "sgbm cost kernel"))) return rc;

    const int ybot = std::max(H - e.SH2, 1);     // first row that is never recomputed
    const int ylast = std::max(H - e.SH2 - 1, 0);  // last recomputed row
    if (H > 1) {
        hipLaunchKernelGGL(sgbm_cost_fixup_kernel, dim3(H - 1, n), dim3(256), 0, s, Cv, H, e,
                           ylast, ybot);
        if ((rc = check_hip(ctx, hipGetLastError(), "sgbm cost fixup"))) return rc;
    }

    const int np = (e.D + 127) / 128;
    if (np == 1) rc = launch_paths<1>(ctx, n, H, W, e, Cv, Sv, raw);
    else if (np == 2) rc = launch_paths<2>(ctx, n, H, W, e, Cv, Sv, raw);
    else rc = launch_paths<4>(ctx, n, H, W, e, Cv, Sv, raw);
    if (rc) return rc;

    if ((rc = median3x3_device(ctx, n, raw, W, plane, out, os, ofs, W, H))) return rc;
    if (e.speckle_window > 0)
        return speckle_device(ctx, n, out, os, ofs, W, H, e.invalid, e.speckle_window,
                              e.speckle_diff);
    return MVSV_OK;
}

}  // namespace mvsv
