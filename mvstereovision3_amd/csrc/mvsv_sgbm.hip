// mvsv_sgbm.hip — StereoSGBM on MI355X (gfx950).
//
// Replaces Disparity::sgbm (src/disparity.cpp:6-10) -> cv::StereoSGBM::compute.
// Pipeline per batch of frames (all launches on the context stream):
//   1. sgbm_prefilter_kernel   clipped x-Sobel + raw channel per row    (u8 planes)
//      (stages 1-3 live in mvsv_cost.hip)
//   2. sgbm_cost_kernel        Birchfield-Tomasi pixel cost + bs x bs box
//                              sum -> C[y][x][d] int16 (+P2 bias), LDS-staged
//                              rows, running vertical sums in registers
//   3. sgbm_cost_fixup_*_kernel OpenCV 3.4's cost-row quirks (column x=0 and
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
#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "mvsv_cost_layout.hpp"
#include "mvsv_device.hpp"
#include "mvsv_bitslice.hpp"
#include "mvsv_internal.hpp"


namespace mvsv {
namespace {

using namespace dev;

// ---------------------------------------------------------------------------
// 4. path aggregation along one direction (predecessor (x-dx, y-dy)).
// ---------------------------------------------------------------------------
struct Line {
    int xs, ys, len;
};

// u8 accumulator when the summed path deltas (each <= P2) fit a byte
__host__ __device__ inline bool acc_is_u8(const SgbmEff& e)
{
    return (e.fullDP ? 8 : 5) * e.P2 <= 255;
}

// 4-bit accumulator planes: the sheared-strip schedule writes one plane per
// group of at most three directions (3 strip directions, or the L->R line),
// so each plane holds sums <= 3 * P2; with P2 <= 5 (OpenCV's default P2 = 5,
// which configs/sgbm.yml gets because it leaves P1/P2 at 0) they fit a nibble.
// Element offsets stay in disparity units; a byte holds two of them.
struct nib2_t {
    uint8_t v;
};
__host__ __device__ inline bool acc_is_nib(const SgbmEff& e) { return 3 * e.P2 <= 15; }
template <typename T>
struct AccEpu {
    static constexpr int v = 1;  // accumulator elements per storage unit
};
template <>
struct AccEpu<nib2_t> {
    static constexpr int v = 2;
};
template <>
struct AccEpu<const nib2_t> {
    static constexpr int v = 2;
};
template <typename T>
__host__ __device__ __forceinline__ T* acc_add(T* p, ptrdiff_t e)
{
    return p + e / AccEpu<T>::v;  // e is even for nib2_t (d0 and D are even)
}
static_assert(AccEpu<const nib2_t>::v == 2 && AccEpu<const uint8_t>::v == 1, "accumulator units");
// non-negative 32-bit offsets: the unit division is a shift and the 64-bit
// address add needs no sign extension
template <typename T>
__device__ __forceinline__ T* acc_addu(T* p, uint32_t e)
{
    return p + e / (uint32_t)AccEpu<T>::v;
}

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

template <>
struct Vec<8> {
    uint32_t v[8];
    __device__ __forceinline__ void load(const int16_t* p)
    {
        uint4 a = *(const uint4*)p, b = *(const uint4*)(p + 8);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    }
    __device__ __forceinline__ void store(int16_t* p) const
    {
        *(uint4*)p = make_uint4(v[0], v[1], v[2], v[3]);
        *(uint4*)(p + 8) = make_uint4(v[4], v[5], v[6], v[7]);
    }
};

// Cost input of the direction passes: the int16 cost volume C (RES = false)
// or the residual plane R (RES = true, two nibbles per byte, see above).
// Offsets are in cost elements (disparity units) either way; get() returns the
// lane's NP packed (d, d+1) u16 pairs.
template <int NP, bool RES>
struct CostIn;
template <int NP>
struct CostIn<NP, false> {
    Vec<NP> b;
    static __device__ __forceinline__ const void* at(const void* base, ptrdiff_t e)
    {
        return (const int16_t*)base + e;
    }
    __device__ __forceinline__ void load(const void* p) { b.load((const int16_t*)p); }
    __device__ __forceinline__ void get(uint32_t (&c)[NP]) const
    {
#pragma unroll
        for (int i = 0; i < NP; i++) c[i] = b.v[i];
    }
};
template <int NP>
struct CostIn<NP, true> {
    static constexpr int NWD = NP >= 8 ? 2 : 1;
    uint32_t w[NWD];
    static __device__ __forceinline__ const void* at(const void* base, ptrdiff_t e)
    {
        return (const uint8_t*)base + e / 2;  // e is even (D and the lane offsets are)
    }
    __device__ __forceinline__ void load(const void* p)
    {
        if constexpr (NP == 1) {
            w[0] = *(const uint8_t*)p;
        } else if constexpr (NP == 2) {
            w[0] = *(const uint16_t*)p;
        } else if constexpr (NP == 4) {
            w[0] = *(const uint32_t*)p;
        } else {
            const uint2 t = *(const uint2*)p;
            w[0] = t.x;
            w[1] = t.y;
        }
    }
    // byte k = (R(2k), R(2k+1)) nibbles -> pair k = R(2k) | R(2k+1) << 16:
    // low nibbles E and high nibbles O as bytes, then one v_perm_b32 per pair
    __device__ __forceinline__ void get(uint32_t (&c)[NP]) const
    {
#pragma unroll
        for (int q = 0; q < NWD; q++) {
            const uint32_t E = w[q] & 0x0f0f0f0fu, O = (w[q] >> 4) & 0x0f0f0f0fu;
#pragma unroll
            for (int k = 0; k < (NP < 4 ? NP : 4); k++)
                c[4 * q + k] = __builtin_amdgcn_perm(O, E, 0x0c000c00u | (uint32_t)k | ((uint32_t)(4 + k) << 16));
        }
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


// Cross-direction accumulator.  With cb = C - P2 (the unbiased box cost) every
// path cost is L_r = cb + delta_r with delta_r in [0, P2] (the min() term of
// the recurrence minus min_k L_r(p-r,k) lies in [0, P2]); hence
//     S = min(sum_r L_r, MAX_COST) = min(ndir*cb + sum_r delta_r, MAX_COST)
// and only sum_r delta_r has to travel between the direction kernels: one byte
// per (pixel, disparity) when ndir*P2 <= 255 (sgbm.yml: P2 = 5), else a
// saturating u16 (saturation above MAX_COST cannot change the min()).
template <int NP, typename AccT>
struct AccVec;

template <int NP>
struct AccVec<NP, uint16_t> {  // packed u16 pairs, one dword per pair
    static __device__ __forceinline__ void load(const uint16_t* p, uint32_t (&v)[NP])
    {
        Vec<NP> t;
        t.load((const int16_t*)p);
#pragma unroll
        for (int i = 0; i < NP; i++) v[i] = t.v[i];
    }
    static __device__ __forceinline__ void store(uint16_t* p, const uint32_t (&v)[NP])
    {
        Vec<NP> t;
#pragma unroll
        for (int i = 0; i < NP; i++) t.v[i] = v[i];
        t.store((int16_t*)p);
    }
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b)
    {
        typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
        return __builtin_bit_cast(uint32_t, __builtin_elementwise_add_sat(
                                                __builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
    }
};

// u8 storage: byte pair <-> u16 pair with v_perm_b32
__device__ __forceinline__ uint32_t u8x2_to_u16x2(uint32_t w, int half)
{
    return __builtin_amdgcn_perm(0u, w, half ? 0x0c030c02u : 0x0c010c00u);
}

template <>
struct AccVec<1, uint8_t> {
    static __device__ __forceinline__ void load(const uint8_t* p, uint32_t (&v)[1])
    {
        v[0] = u8x2_to_u16x2(*(const uint16_t*)p, 0);
    }
    static __device__ __forceinline__ void store(uint8_t* p, const uint32_t (&v)[1])
    {
        *(uint16_t*)p = (uint16_t)__builtin_amdgcn_perm(0u, v[0], 0x0c0c0200u);
    }
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return a + b; }
};
template <>
struct AccVec<2, uint8_t> {
    static __device__ __forceinline__ void load(const uint8_t* p, uint32_t (&v)[2])
    {
        uint32_t w = *(const uint32_t*)p;
        v[0] = u8x2_to_u16x2(w, 0);
        v[1] = u8x2_to_u16x2(w, 1);
    }
    static __device__ __forceinline__ void store(uint8_t* p, const uint32_t (&v)[2])
    {
        *(uint32_t*)p = __builtin_amdgcn_perm(v[1], v[0], 0x06040200u);
    }
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return a + b; }
};
template <>
struct AccVec<4, uint8_t> {
    static __device__ __forceinline__ void load(const uint8_t* p, uint32_t (&v)[4])
    {
        uint2 w = *(const uint2*)p;
        v[0] = u8x2_to_u16x2(w.x, 0);
        v[1] = u8x2_to_u16x2(w.x, 1);
        v[2] = u8x2_to_u16x2(w.y, 0);
        v[3] = u8x2_to_u16x2(w.y, 1);
    }
    static __device__ __forceinline__ void store(uint8_t* p, const uint32_t (&v)[4])
    {
        *(uint2*)p = make_uint2(__builtin_amdgcn_perm(v[1], v[0], 0x06040200u),
                                __builtin_amdgcn_perm(v[3], v[2], 0x06040200u));
    }
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return a + b; }
};

template <>
struct AccVec<8, uint8_t> {
    static __device__ __forceinline__ void load(const uint8_t* p, uint32_t (&v)[8])
    {
        uint4 w = *(const uint4*)p;
        v[0] = u8x2_to_u16x2(w.x, 0);
        v[1] = u8x2_to_u16x2(w.x, 1);
        v[2] = u8x2_to_u16x2(w.y, 0);
        v[3] = u8x2_to_u16x2(w.y, 1);
        v[4] = u8x2_to_u16x2(w.z, 0);
        v[5] = u8x2_to_u16x2(w.z, 1);
        v[6] = u8x2_to_u16x2(w.w, 0);
        v[7] = u8x2_to_u16x2(w.w, 1);
    }
    static __device__ __forceinline__ void store(uint8_t* p, const uint32_t (&v)[8])
    {
        *(uint4*)p = make_uint4(__builtin_amdgcn_perm(v[1], v[0], 0x06040200u),
                                __builtin_amdgcn_perm(v[3], v[2], 0x06040200u),
                                __builtin_amdgcn_perm(v[5], v[4], 0x06040200u),
                                __builtin_amdgcn_perm(v[7], v[6], 0x06040200u));
    }
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return a + b; }
};

// nibble storage of the sums (each <= 15): every 4 consecutive disparities
// d..d+3 = pairs (d, d+1), (d+2, d+3) form one u16 with d, d+2, d+1, d+3 in
// nibbles 0..3 -- independent of how many pairs a lane holds, so writers with
// 16 lanes per row and the final kernel's 32 lanes per row agree.  (One pair
// per lane, D = 32 only: nibbles 0, 1 of a byte.)
template <int NP>
struct AccVec<NP, nib2_t> {
    static __device__ __forceinline__ uint32_t pack4(uint32_t a, uint32_t b, uint32_t c, uint32_t d)
    {
        const uint32_t h0 = a | (b << 4), h1 = c | (d << 4);  // bytes 0 and 2 carry the groups
        return __builtin_amdgcn_perm(h1, h0, 0x06040200u);
    }
    static __device__ __forceinline__ void store(nib2_t* p, const uint32_t (&v)[NP])
    {
        if constexpr (NP == 1) {
            *(uint8_t*)p = (uint8_t)(v[0] | (v[0] >> 12));
        } else if constexpr (NP == 2) {
            const uint32_t w = v[0] | (v[1] << 4);
            *(uint16_t*)p = (uint16_t)(w | (w >> 8));
        } else if constexpr (NP == 4) {
            *(uint32_t*)p = pack4(v[0], v[1], v[2], v[3]);
        } else {
            *(uint2*)p = make_uint2(pack4(v[0], v[1], v[2], v[3]), pack4(v[4], v[5], v[6], v[7]));
        }
    }
};

// delta = L - C + P2 (exact, in [0, P2]) for a packed pair
__device__ __forceinline__ uint32_t path_delta(uint32_t ln, uint32_t c, uint32_t p2x2)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    u16x2 r = __builtin_bit_cast(u16x2, ln) - __builtin_bit_cast(u16x2, c) + __builtin_bit_cast(u16x2, p2x2);
    return __builtin_bit_cast(uint32_t, r);
}

// One wave per scanline.  The loop is branch-free around memory: every
// prefetch address is clamped into the line (duplicates are never consumed),
// so the compiler can count outstanding loads exactly and keep kPathPF steps
// of C / accumulator loads in flight.  FULL = every lane owns real
// disparities (D == 128 * NP); otherwise stores are lane-predicated.
constexpr int kPathPF = 8;

template <int NP, bool FIRST, bool FULL, typename AccT>
__global__ __launch_bounds__(256) void sgbm_path_kernel(const int16_t* __restrict__ C,
                                                        AccT* __restrict__ A, int H, int W1,
                                                        int D, int dx, int dy, int P1, int P2)
{
    using AV = AccVec<NP, AccT>;
    constexpr int PF = kPathPF;
    const int lane = threadIdx.x & 63;
    // wave-uniform by construction; readfirstlane keeps the line walk scalar
    const int line = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));
    const int f = blockIdx.y;
    if (line >= num_lines(dx, dy, W1, H)) return;
    const Line g = line_geometry(line, dx, dy, W1, H);
    const size_t frame = (size_t)H * W1 * D;
    const ptrdiff_t step = ((ptrdiff_t)dy * W1 + dx) * D;
    const int d0 = lane * 2 * NP;
    const bool lane_on = FULL || d0 < D;
    const size_t off = f * frame + ((size_t)g.ys * W1 + g.xs) * D + (lane_on ? d0 : 0);
    const int16_t* cp = C + off;
    AccT* ap = A + off;
    bool valid[NP];
    uint32_t lp[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        valid[p] = FULL || d0 + 2 * p < D;
        lp[p] = valid[p] ? 0u : 0x7fff7fffu;
    }
    const uint32_t p1x2 = (uint32_t)(P1 & 0xffff) * 0x10001u;
    const uint32_t p2x2 = (uint32_t)(P2 & 0xffff) * 0x10001u;
    int minp = 0;
    const int len = g.len;

    Vec<NP> cb[PF];
    uint32_t ab[PF][NP];
#pragma unroll
    for (int j = 0; j < PF; j++) {
        const ptrdiff_t t = min(j, len - 1);
        cb[j].load(cp + t * step);
        if (!FIRST) AV::load(ap + t * step, ab[j]);
    }
    auto body = [&](int s, int j) {
        const int dl = (int16_t)(minp + P2);
        const uint32_t delta2 = (uint32_t)(dl & 0xffff) * 0x10001u;
        uint32_t c[NP], ln[NP], o[NP];
#pragma unroll
        for (int p = 0; p < NP; p++) c[p] = cb[j].v[p];
        sgm_step<NP>(lp, delta2, p1x2, c, valid, ln);
        minp = wave_min_i32(lane_min<NP>(ln));
#pragma unroll
        for (int p = 0; p < NP; p++) {
            uint32_t dv = path_delta(ln[p], c[p], p2x2);
            o[p] = FIRST ? dv : AV::add(ab[j][p], dv);
            lp[p] = ln[p];
        }
        if (FULL || lane_on) AV::store(ap + (ptrdiff_t)s * step, o);
    };
    int s = 0;
    for (; s + PF <= len; s += PF) {
#pragma unroll
        for (int j = 0; j < PF; j++) {
            body(s + j, j);
            const ptrdiff_t t = min(s + j + PF, len - 1);
            cb[j].load(cp + t * step);
            if (!FIRST) AV::load(ap + t * step, ab[j]);
        }
    }
    const int rem = len - s;
#pragma unroll
    for (int j = 0; j < PF; j++)
        if (j < rem) body(s + j, j);
}

// ---------------------------------------------------------------------------
// 4b. path aggregation, 16 lanes per scanline (D = 32 * NP, NP in {1,2,4,8}).
// A wave walks four scanlines at once, one per 16-lane DPP row: every lane
// owns 2*NP consecutive disparities (16 B of C per lane for D = 128), the d+-1
// neighbours cross lanes with row_shr/row_shl, the per-step min over d is a
// four-step DPP butterfly inside the row (no readlane / SGPR round trip).
// Rows whose scanline is shorter than the wave's longest one keep running on
// clamped loads and store into a private dummy slot (branch-free memory).
// ---------------------------------------------------------------------------
template <int NP>
__device__ __forceinline__ void sgm_step_row(const uint32_t (&lp)[NP], uint32_t delta2,
                                             uint32_t p1x2, const uint32_t (&c)[NP],
                                             uint32_t (&ln)[NP])
{
    const uint32_t MAXP = 0x7fff7fffu;
    const uint32_t prev_hi = row_shr1(lp[NP - 1], MAXP);
    const uint32_t next_lo = row_shl1(lp[0], MAXP);
#pragma unroll
    for (int p = 0; p < NP; p++) {
        uint32_t ph = p == 0 ? prev_hi : lp[p - 1];
        uint32_t nl = p == NP - 1 ? next_lo : lp[p + 1];
        uint32_t lm = __builtin_amdgcn_alignbit(lp[p], ph, 16);
        uint32_t lq = __builtin_amdgcn_alignbit(nl, lp[p], 16);
        // min(L[d-1] + P1, L[d+1] + P1) == min(L[d-1], L[d+1]) + P1 (saturating add is monotone)
        uint32_t m = pk_min(lp[p], pk_add_sat(pk_min(lm, lq), p1x2));
        m = pk_min(m, delta2);
        ln[p] = pk_add_sat(pk_sub_sat(m, delta2), c[p]);
    }
}

// sgm_step_row that also returns t = sat(m - delta) = delta_r - P2 in [-P2, 0]
// (delta_r = the path's increment over cb, exact: every candidate of m lies
// in [minLp, minLp + P2]).  The neighbour minima min(L[d-1], L[d+1]) of the
// NP pairs come from NP + 1 pairwise minima X_q = min(pair q, pair q + 1):
// pair p's is (X_{p-1}.hi, X_p.lo) -- one v_pk_min + one v_alignbit per pair.
//
// NW ("no wrap", chosen by the host when P2 + blockSize^2 * (2*ftzero + 63) +
// P2 <= 32767, sgbm_no_wrap): every C, L and delta = minLp + P2 is then a
// non-negative int16, so with u = delta - min(m, delta) = max(delta - m, 0)
// (one unsigned saturating subtract) L = C - u, and the path's increment over
// cb is P2 - u: five VALU per pair instead of six.  tu[] returns u (NW) or the
// signed t = -u (the general form, exact for wrapped costs too).
template <bool NW>
__device__ __forceinline__ void sgm_pair(uint32_t lp, uint32_t nb, uint32_t delta2, uint32_t p1x2,
                                         uint32_t c, uint32_t& ln, uint32_t& tu)
{
    if constexpr (NW) {
        // full-rate 32-bit forms, exact here: nb <= 0x7fff and P1 < 0x8000, so
        // nb + P1 never carries out of its half (the unsigned min then equals
        // min(L, sat(nb + P1)) because L <= 0x7fff); u <= P2 <= C (every cost
        // of the no-wrap regime is P2 + a window sum, every residual is in
        // [P2, 3 P2]), so C - u never borrows
        const uint32_t m = pk_min_u16(lp, add2_nc(nb, p1x2));
        tu = pk_subsat_u16(delta2, m);
        ln = sub2_nb(c, tu);
    } else {
        const uint32_t m = pk_min(lp, pk_add_sat(nb, p1x2));
        tu = pk_sub_sat(pk_min(m, delta2), delta2);
        ln = pk_add_sat(tu, c);
    }
}
// delta = t + P2 (general) = P2 - u (NW, u <= P2: no borrow), in [0, P2]
template <bool NW>
__device__ __forceinline__ uint32_t sgm_delta(uint32_t tu, uint32_t p2x2)
{
    return NW ? sub2_nb(p2x2, tu) : pk_add_u16(tu, p2x2);
}
// the packed delta = (short)(minLp + P2) of the next step
template <bool NW>
__device__ __forceinline__ uint32_t sgm_delta2(int minp, int P2)
{
    return NW ? (uint32_t)(minp + P2) * 0x10001u : (uint32_t)((minp + P2) & 0xffff) * 0x10001u;
}
template <int NP, bool NW = false, int LPC = 16>
__device__ __forceinline__ void sgm_step_row_t(const uint32_t (&lp)[NP], uint32_t delta2,
                                               uint32_t p1x2, const uint32_t (&c)[NP],
                                               uint32_t (&ln)[NP], uint32_t (&t)[NP])
{
    static_assert(LPC == 8 || LPC == 16, "row-DPP segments of 8 or 16 lanes");
    const uint32_t MAXP = 0x7fff7fffu;
    // d-1 / d+1 neighbours across the lane boundary: zero-filled DPP shifts
    // (bound_ctrl) OR'ed with MAX at the segment ends fold into v_or_b32_dpp
    // (an 8-lane segment's first lane receives the previous segment's last
    // lane; the OR with MAX discards it: L values are in [0, 0x7fff])
    const uint32_t rls = __lane_id() % LPC;
    const uint32_t prev_hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)lp[NP - 1], 0x111, 0xf, 0xf, true) |
                             (rls == 0 ? MAXP : 0u);
    const uint32_t next_lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)lp[0], 0x101, 0xf, 0xf, true) |
                             (rls == LPC - 1 ? MAXP : 0u);
    uint32_t X[NP + 1];  // X[q + 1] = X_q, X[0] = X_{-1}
    X[0] = pk_min(prev_hi, lp[0]);
#pragma unroll
    for (int q = 0; q + 1 < NP; q++) X[q + 1] = pk_min(lp[q], lp[q + 1]);
    X[NP] = pk_min(lp[NP - 1], next_lo);
#pragma unroll
    for (int p = 0; p < NP; p++)
        sgm_pair<NW>(lp[p], __builtin_amdgcn_alignbit(X[p + 1], X[p], 16), delta2, p1x2, c[p], ln[p], t[p]);
}

// Minimum over an LPC-lane segment (8: one half of a DPP row, 16: a row);
// every lane of the segment gets it.
template <int LPC>
__device__ __forceinline__ int seg_lane_min(int v)
{
    static_assert(LPC == 8 || LPC == 16, "row-DPP segments of 8 or 16 lanes");
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true));   // quad_perm [1,0,3,2]
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true));   // quad_perm [2,3,0,1]
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, true));  // row_half_mirror
    if constexpr (LPC == 16) v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, true));  // row_mirror
    return v;
}

// Lane segments of the final kernel: LPR lanes own one image row (16: a DPP
// row; 32: two DPP rows joined by v_permlane16_swap).
template <int LPR>
__device__ __forceinline__ int seg_min_i32(int v)
{
    if constexpr (LPR == 8) return seg_lane_min<8>(v);
    v = row_min_i32(v);
    if constexpr (LPR == 32) {
        const auto sw = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
        v = min((int)sw[0], (int)sw[1]);
    }
    return v;
}
// sgm_step_row_t over an LPR-lane segment: the d-1 / d+1 neighbours of a lane's
// first / last pair come from the adjacent lane of the segment (MAX at the
// segment ends).
template <int NP, int LPR, bool NW>
__device__ __forceinline__ void sgm_step_seg_t(const uint32_t (&lp)[NP], uint32_t delta2,
                                               uint32_t p1x2, const uint32_t (&c)[NP],
                                               uint32_t (&ln)[NP], uint32_t (&t)[NP], bool seg_first,
                                               bool seg_last)
{
    if constexpr (LPR <= 16) {
        sgm_step_row_t<NP, NW, LPR>(lp, delta2, p1x2, c, ln, t);
    } else {
        const uint32_t MAXP = 0x7fff7fffu;
        // zero-filled wave shifts (bound_ctrl) OR'ed with MAX at the segment
        // ends (L values are in [0, 0x7fff], so x | MAXP == MAXP): one
        // v_or_b32_dpp per neighbour
        const uint32_t prev_hi =
            (uint32_t)__builtin_amdgcn_mov_dpp((int)lp[NP - 1], 0x138, 0xf, 0xf, true) | (seg_first ? MAXP : 0u);
        const uint32_t next_lo =
            (uint32_t)__builtin_amdgcn_mov_dpp((int)lp[0], 0x130, 0xf, 0xf, true) | (seg_last ? MAXP : 0u);
        uint32_t X[NP + 1];  // X[q + 1] = X_q, X[0] = X_{-1}
        X[0] = pk_min(prev_hi, lp[0]);
#pragma unroll
        for (int q = 0; q + 1 < NP; q++) X[q + 1] = pk_min(lp[q], lp[q + 1]);
        X[NP] = pk_min(lp[NP - 1], next_lo);
#pragma unroll
        for (int p = 0; p < NP; p++)
            sgm_pair<NW>(lp[p], __builtin_amdgcn_alignbit(X[p + 1], X[p], 16), delta2, p1x2, c[p], ln[p],
                         t[p]);
    }
}

// The lane's minimum over its NP pairs in BOTH halves (the swap is a VOP3P
// op_sel, no extra instruction): for L in [0, 0x7fff] the packed (m, m) orders
// like m as an int32, so the segment butterfly runs on it unchanged and the
// next step's packed delta = (minLp + P2) x 2 is one v_add_u32 (no-wrap form).
template <int NP>
__device__ __forceinline__ uint32_t lane_min_pk(const uint32_t (&ln)[NP])
{
    uint32_t m = ln[0];
#pragma unroll
    for (int p = 1; p < NP; p++) m = pk_min(m, ln[p]);
    const s16x2 v = as_s2(m);
    return as_u(__builtin_elementwise_min(v, __builtin_shufflevector(v, v, 1, 0)));
}

template <int NP>
__device__ __forceinline__ int lane_min_row(const uint32_t (&ln)[NP])
{
    uint32_t m = ln[0];
#pragma unroll
    for (int p = 1; p < NP; p++) m = pk_min(m, ln[p]);
    return min(lo16(m), hi16(m));
}

__device__ __forceinline__ uint32_t pk_mad_u16(uint32_t a, uint32_t b, uint32_t c)
{
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) * __builtin_bit_cast(u16x2, b) +
                                            __builtin_bit_cast(u16x2, c));
}

constexpr int kPath16PF = 12;

// LPC lanes per line (2*NP disparities each, D = 2*NP*LPC): 16 (a DPP row),
// or 8 for D = 16 (captureDisparity's create(0, 16, 5, 200, 800)), eight lines
// per wave
template <int LPC>
constexpr int path16_lines_per_block() { return 4 * (64 / LPC); }

template <int NP, bool FIRST, typename AccT, bool NW = false, bool RES = false, int LPC = 16>
__device__ __forceinline__ void path16_lines(const void* __restrict__ C, AccT* __restrict__ A,
                                             AccT* __restrict__ dummy, int H, int W1, int D, int dx,
                                             int dy, int P1, int P2, int bx, int f)
{
    static_assert(LPC == 8 || LPC == 16, "row-DPP segments of 8 or 16 lanes");
    using AV = AccVec<NP, AccT>;
    using CI = CostIn<NP, RES>;
    constexpr int PF = kPath16PF;
    constexpr int LPW = 64 / LPC;  // lines per wave
    const int lane = threadIdx.x & 63;
    const int row = lane / LPC, rl = lane % LPC;
    const int nl = num_lines(dx, dy, W1, H);
    const int line0 = __builtin_amdgcn_readfirstlane((bx * 4 + (int)(threadIdx.x >> 6)) * LPW);
    if (line0 >= nl) return;
    const int line = min(line0 + row, nl - 1);
    const Line g = line_geometry(line, dx, dy, W1, H);
    const int len = line0 + row < nl ? g.len : 0;
    int maxlen = __builtin_amdgcn_readlane(len, 0);
#pragma unroll
    for (int r = 1; r < LPW; r++) maxlen = max(maxlen, __builtin_amdgcn_readlane(len, r * LPC));
    const size_t frame = (size_t)H * W1 * D;
    const ptrdiff_t step = ((ptrdiff_t)dy * W1 + dx) * D;
    const int d0 = rl * 2 * NP;
    const size_t off = f * frame + ((size_t)g.ys * W1 + g.xs) * D + d0;
    const void* cp = CI::at(C, (ptrdiff_t)off);
    AccT* ap = acc_add(A, (ptrdiff_t)off);
    AccT* dp = acc_add(dummy, (ptrdiff_t)threadIdx.x * 2 * NP);
    const int last = max(len - 1, 0);
    uint32_t lp[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) lp[p] = 0u;
    const uint32_t p1x2 = (uint32_t)(P1 & 0xffff) * 0x10001u;
    const uint32_t p2x2 = (uint32_t)(P2 & 0xffff) * 0x10001u;
    int minp = 0;

    CI cb[PF];
    uint32_t ab[PF][NP];
#pragma unroll
    for (int j = 0; j < PF; j++) {
        const ptrdiff_t t = min(j, last);
        cb[j].load(CI::at(cp, t * step));
        if constexpr (!FIRST) AV::load(acc_add(ap, t * step), ab[j]);
    }
    auto body = [&](int s, int j) {
        const uint32_t delta2 = sgm_delta2<NW>(minp, P2);
        uint32_t c[NP], ln[NP], o[NP], tt[NP];
        cb[j].get(c);
        sgm_step_row_t<NP, NW, LPC>(lp, delta2, p1x2, c, ln, tt);
        minp = seg_lane_min<LPC>(lane_min_row<NP>(ln));
#pragma unroll
        for (int p = 0; p < NP; p++) {
            const uint32_t dv = sgm_delta<NW>(tt[p], p2x2);  // delta = t + P2 = P2 - u
            if constexpr (FIRST)
                o[p] = dv;
            else
                o[p] = AV::add(ab[j][p], dv);
            lp[p] = ln[p];
        }
        AccT* dst = s < len ? acc_add(ap, (ptrdiff_t)s * step) : dp;
        AV::store(dst, o);
    };
    int s = 0;
    for (; s + PF <= maxlen; s += PF) {
#pragma unroll
        for (int j = 0; j < PF; j++) {
            body(s + j, j);
            const ptrdiff_t t = min(s + j + PF, last);
            cb[j].load(CI::at(cp, t * step));
            if constexpr (!FIRST) AV::load(acc_add(ap, t * step), ab[j]);
        }
    }
    const int rem = maxlen - s;
#pragma unroll
    for (int j = 0; j < PF; j++)
        if (j < rem) body(s + j, j);
}


template <int NP, bool FIRST, typename AccT, bool NW = false, bool RES = false>
__global__ __launch_bounds__(256) void sgbm_path16_kernel(const void* __restrict__ C,
                                                          AccT* __restrict__ A,
                                                          AccT* __restrict__ dummy, int H, int W1,
                                                          int D, int dx, int dy, int P1, int P2)
{
    path16_lines<NP, FIRST, AccT, NW, RES>(C, A, dummy, H, W1, D, dx, dy, P1, P2, blockIdx.x, blockIdx.y);
}

// All directions of a small launch at once (blockIdx.z = direction k, its
// deltas into plane k): one frame's 4 or 7 line directions run side by side
// instead of as sheared strips, whose 480-step chain is the single-frame
// critical path.
struct PathDirs {
    int dx[8], dy[8];
};
template <int NP, typename AccT, bool NW, bool RES = false, int LPC = 16>
__global__ __launch_bounds__(256) void sgbm_pathdirs16_kernel(const void* __restrict__ C,
                                                              AccT* __restrict__ A, size_t plane,
                                                              AccT* __restrict__ dummy, int H, int W1,
                                                              int D, PathDirs dirs, int P1, int P2)
{
    const int k = blockIdx.z;
    path16_lines<NP, true, AccT, NW, RES, LPC>(C, acc_add(A, (ptrdiff_t)k * (ptrdiff_t)plane), dummy, H, W1, D,
                                          dirs.dx[k], dirs.dy[k], P1, P2, blockIdx.x, blockIdx.y);
}

// ---------------------------------------------------------------------------
// 4c. three vertical-ish directions in one sweep over sheared strips.
// With U = x - t + (H - 1) for step t (row y = t top-down, y = H-1-t
// bottom-up), the cell (x, y) at step t has its predecessors at step t-1 in
// U-column U (dir (1, sy)), U+1 (dir (0, sy)) and U+2 (dir (-1, sy)), sy = +1
// (down) or -1 (up).  So one block owning U-columns [U0, U0+SW) walks its
// strip one step per row -- every step is SW contiguous x-columns of C and of
// the accumulator -- and needs only the two U-columns right of it from the
// previous step: the strip to its right (lower block index) publishes them as
// tagged 8-byte granules with write-through stores, this strip polls them
// (bounded spin).  C is read once for three directions instead of three
// times.  Cells outside the image carry L = 0, min 0: exactly the zero start
// state of every path at the image border.
// Lanes: 16 per U-column (2*NP disparities each), 4 columns per compute wave;
// one extra wave per block does all strip-to-strip traffic, so the compute
// waves' memory counters only ever wait for their own C loads.
// ---------------------------------------------------------------------------
// compute waves per block (WV): wide strips, 15 (+ the exchange wave = 1024
// threads, <= 128 VGPRs) for up to 8 disparities per lane, 7 for D = 256 (16
// per lane, ~200 VGPRs) -- the throughput shape for frame batches; narrow
// strips, 8 (4 for D = 256) compute waves -- the latency shape for one or two
// frames, where wide strips leave most CUs idle and each step of a strip is
// the serial work of its CU (see launch_tri)
// LPC = lanes per U-column (2*NP disparities each, D = 2*NP*LPC): 16 (one DPP
// row per column) or 8 (half a DPP row, twice the disparities per lane: the
// per-column minimum is a 3-step butterfly, and the lane-boundary neighbours,
// the step's row minima and its bookkeeping are shared by twice the work --
// the throughput shape for D = 128 batches, two 512-thread blocks per CU).
// LPC = 32 (round 6, D = 256 launches too small for wide strips: config 5's
// one or two frames): two DPP rows per U-column, 4 disparity pairs per lane --
// half the per-wave work of a strip step at the same strip width (8 compute
// waves x 2 columns); the three boundary items then need 96 exchange lanes,
// so such a block has two exchange waves.
template <int NP, int LPC = 16>
constexpr int tri_wide_waves() { return LPC == 8 ? 7 : (NP >= 8 ? 7 : 15); }
template <int NP, int LPC = 16>
constexpr int tri_narrow_waves() { return LPC == 8 ? 4 : LPC == 32 ? 8 : (NP >= 8 ? 4 : 8); }
template <int NP, int WV, int LPC = 16>
struct TriCfg {
    static constexpr int kWaves = WV;
    static constexpr int kCPW = 64 / LPC;   // U-columns per compute wave
    static constexpr int kSW = kCPW * kWaves;  // U-columns per strip
    static constexpr int kComm = LPC == 32 ? 2 : 1;  // exchange waves: 3 items x LPC lanes
    static constexpr int kThreads = 64 * (kWaves + kComm);
    // blocks per CU the register budget aims at: one 1024-thread block, or two
    // 512-thread ones (4 waves per SIMD either way); D = 256 on 16 lanes: 2.
    // (Narrow strips reading the cost residual aim at 5: two 9-wave blocks
    // per CU, each filling the other's step-barrier and hand-off waits.)
    static constexpr int kWavesPerEU = (NP >= 8 && LPC == 16) ? 2 : 4;
};
#ifndef MVSV_TRI_PF
#define MVSV_TRI_PF 4
#endif
#ifndef MVSV_FINAL32_PF
#define MVSV_FINAL32_PF 8  // steps of prefetch in the 32-lanes-per-row final kernel
#endif
#ifndef MVSV_FINAL_LPR
#define MVSV_FINAL_LPR 32  // lanes per row of the final kernel for D >= 128 (16: A/B)
#endif
#ifndef MVSV_TRI_STEP_SEQ
#define MVSV_TRI_STEP_SEQ 0  // 1: the three recurrences of a step one after the other (A/B)
#endif
constexpr int kTriPF = MVSV_TRI_PF;     // steps of C prefetch (compute waves)
constexpr int kTriBF = 4;               // steps of boundary prefetch (comm wave)
constexpr int kTriUnroll = 4;           // lcm(kTriPF, kTriBF, 2)

template <int NP, int WV, int LPC = 16>
struct TriLayout {
    static constexpr int kCols = TriCfg<NP, WV, LPC>::kSW + 2;  // + two columns of the right strip
    // Element-major columns: lane (column c, rl) keeps element p of its 2*NP
    // disparities at c*kColDw + p*LPC + rl.  A b32 access (ds_read2_b32 /
    // ds_write2_b32) is served per 32-lane half-wave on 32 banks ((a/4) mod 32,
    // MI355X_MICROARCH.md §LDS); the half-wave holds 32/LPC columns, and with
    // kColDw = LPC (mod 32) they land on disjoint bank ranges: conflict-free.
    // (The former lane-major layout, c*kColDw + rl*NP + p with an odd stride,
    // mapped lanes rl and rl + 32/NP of a column onto one bank: 2-way
    // conflicts, SQ_LDS_BANK_CONFLICT 44 % of the LDS cycles.)
    static constexpr int kColDw = ((NP * LPC + 31) / 32) * 32 + LPC % 32;
    static constexpr int kBufDw = 2 * kCols * kColDw;   // dirs b and c
    static constexpr int kLDw = 2 * kBufDw;             // double-buffered
    static constexpr int kMinInts = 2 * 2 * kCols;      // [buf][dir][col]
    static constexpr size_t kBytes = (size_t)(kLDw + kMinInts) * 4;
};

// Boundary granules of one strip and step: [NG][4 item rows][LPC lanes] u64
// (the 4th item row is never written: the comm wave's spare lanes repeat
// item 2).  Item 0 = L of dir
// (0, sy) at the strip's first column, 1 = dir (-1, sy) at the first column,
// 2 = dir (-1, sy) at the second column.  A lane's item is its 2*NP int16
// costs + the column min, three int16 per granule under a 16-bit launch tag
// (bits 48-63): the tag is the data-ready flag.
template <int NP>
struct TriGran {
    static constexpr int NG = (2 * NP + 1 + 2) / 3;
    static __device__ __forceinline__ void pack(const uint32_t (&v)[NP], int mn, unsigned long long tag,
                                                unsigned long long (&g)[NG])
    {
        uint32_t s[3 * NG];
#pragma unroll
        for (int i = 0; i < 3 * NG; i++) s[i] = 0u;
#pragma unroll
        for (int p = 0; p < NP; p++) {
            s[2 * p] = v[p] & 0xffffu;
            s[2 * p + 1] = v[p] >> 16;
        }
        s[2 * NP] = (uint32_t)mn & 0xffffu;
#pragma unroll
        for (int i = 0; i < NG; i++)
            g[i] = tag | ((unsigned long long)s[3 * i + 2] << 32) | (s[3 * i + 1] << 16) | s[3 * i];
    }
    static __device__ __forceinline__ void unpack(const unsigned long long (&g)[NG], uint32_t (&v)[NP],
                                                  int& mn)
    {
        uint32_t s[3 * NG];
#pragma unroll
        for (int i = 0; i < NG; i++) {
            s[3 * i] = (uint32_t)g[i] & 0xffffu;
            s[3 * i + 1] = (uint32_t)g[i] >> 16;
            s[3 * i + 2] = (uint32_t)(g[i] >> 32) & 0xffffu;
        }
#pragma unroll
        for (int p = 0; p < NP; p++) v[p] = s[2 * p] | (s[2 * p + 1] << 16);
        mn = (int)(int16_t)s[2 * NP];
    }
};

template <int NP, int LPC = 16>
__device__ __forceinline__ size_t tri_slot(int chain, int k, int t, int nchains, int H)
{
    return ((((size_t)k * nchains + chain) * H + t) * 4) * LPC * TriGran<NP>::NG;
}

template <int NP, int WV, int LPC, typename AccT, bool NW = false, bool RES = false>
__global__ __launch_bounds__((TriCfg<NP, WV, LPC>::kThreads))
__attribute__((amdgpu_waves_per_eu(TriCfg<NP, WV, LPC>::kWavesPerEU + (RES && WV <= 8 && NP <= 4 ? 1 : 0)))) void sgbm_tri_kernel(
    const void* __restrict__ C, AccT* __restrict__ A, size_t plane, AccT* __restrict__ dummy,
    int H, int W1, int D, int npass, int P1, int P2, unsigned long long* __restrict__ bnd,
    unsigned epoch, int nframes, int nstrips, int* __restrict__ status, unsigned spin_limit,
    int* __restrict__ report, unsigned long long* __restrict__ stats, int trace_h, long long ticket0)
{
    using AV = AccVec<NP, AccT>;
    using CI = CostIn<NP, RES>;
    using TL = TriLayout<NP, WV, LPC>;
    using TG = TriGran<NP>;
    constexpr int NG = TG::NG;
    constexpr int kTriWaves = TriCfg<NP, WV, LPC>::kWaves;
    constexpr int kTriSW = TriCfg<NP, WV, LPC>::kSW;
    constexpr int kCPW = TriCfg<NP, WV, LPC>::kCPW;
    constexpr int PF = NP >= 8 ? 2 : kTriPF;  // 16 disparities per lane: registers
    constexpr int BF = kTriBF;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    uint32_t* lds = (uint32_t*)smem;
    int* lmin = (int*)(lds + TL::kLDw);
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool comm = w >= kTriWaves;
    const int cw = comm ? w - kTriWaves : 0;  // exchange wave rank (LPC = 32: 0 or 1)
    const bool comm0 = comm && cw == 0;     // the one that records statistics / traces
    const int r = lane / LPC, rl = lane % LPC;
    // strips counted from the right; pass 0 sweeps down (sy = +1), pass 1 up
    // (sy = -1), each into its own accumulator plane; every strip's producer
    // is strip k - 1 of its chain (same pass and frame).  Which strip a block
    // runs is the ticket it draws on arrival (status[2] counts the context's
    // strip blocks, ticket0 = this launch's first), not its blockIdx: a strip
    // only ever waits on a strip whose block arrived before it and is running
    // or done, so the chain progresses whatever order and placement the
    // dispatcher picks (ticket0 < 0: blockIdx order, which relies on in-order
    // dispatch -- measured on gfx950, tools/ubench/xcc_map.hip -- and keeps a
    // chain on one XCD under round-robin placement: strips 1.60 vs 1.68 ms).
    __shared__ int s_ticket;
    if (threadIdx.x == 0)
        s_ticket = ticket0 < 0 ? (int)blockIdx.x
                               : (int)(__hip_atomic_fetch_add((unsigned*)status + 2, 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT) - (unsigned)ticket0);
    __syncthreads();
    const int bx = s_ticket;
    if ((unsigned)bx >= gridDim.x) {  // ticket count out of step with the host: drain, report
        if (threadIdx.x == 0) {
            __hip_atomic_store(status, (int)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(report, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    const int nchains = npass * nframes;
    const int k = bx / nchains;
    const int chain = bx - k * nchains;
    const int pass = chain / nframes;
    const int f = chain - pass * nframes;
    const int sy = pass == 0 ? 1 : -1;
    A = acc_add(A, (ptrdiff_t)pass * (ptrdiff_t)plane);
    const int Utot = W1 + H - 1;
    const int U0 = Utot - kTriSW * (k + 1);
    const int col = kCPW * w + r;  // compute waves
    const int U = U0 + col;
    // active steps: some column of the strip has 0 <= x = U - (H-1) + t < W1
    const int tb = max(0, (H - 1) - (U0 + kTriSW - 1));
    const int te = min(H, W1 + (H - 1) - U0);
    if (tb >= te) return;
    unsigned long long st_t0 = stats ? __builtin_amdgcn_s_memtime() : 0ull, st_spin = 0, st_n = 0;
    const int d0 = rl * 2 * NP;
    const size_t frame = (size_t)H * W1 * D;
    const void* Cf = CI::at(C, (ptrdiff_t)(f * frame + d0));
    AccT* Af = acc_add(A, (ptrdiff_t)(f * frame + d0));
    AccT* dp = acc_add(dummy, (ptrdiff_t)threadIdx.x * 2 * NP);
    const uint32_t p1x2 = (uint32_t)(P1 & 0xffff) * 0x10001u;
    const uint32_t p2x3 = (uint32_t)((3 * P2) & 0xffff) * 0x10001u;
    const unsigned tag16 = epoch & 0xffffu;
    const unsigned long long tag = (unsigned long long)tag16 << 48;

    auto lcol = [&](int buf, int dir, int c) -> uint32_t* {
        return lds + (size_t)((buf * 2 + dir) * TL::kCols + c) * TL::kColDw + rl;  // element p at [p * LPC]
    };
    auto mcol = [&](int buf, int dir, int c) -> int* { return lmin + (buf * 2 + dir) * TL::kCols + c; };

    // zero both LDS rows (cells outside the image / before the first step)
    for (int i = threadIdx.x; i < TL::kLDw + TL::kMinInts; i += TriCfg<NP, WV, LPC>::kThreads) lds[i] = 0u;

    // ---- comm wave: lanes (item j = min(r, 2), rl); row 3 repeats item 2's
    // loads and stores at item 2's own addresses (same values: the duplicate
    // lanes cost no extra traffic), so every comm-wave memory instruction is
    // unpredicated and its wait counts are exact.  A step's granules are laid
    // out [granule i][item row][lane]: each of the NG store / load
    // instructions covers 512 contiguous bytes.
    const int ir = cw * (64 / LPC) + r;  // item row of this exchange lane
    const int jj = min(ir, 2);
    const bool jlive = ir < 3;
    const int bcol = kTriSW + (jj == 2 ? 1 : 0);  // LDS column the consumed item lands in
    const int bdir = jj == 0 ? 0 : 1;
    const int pcol = jj == 2 ? 1 : 0;              // own column published as item jj
    const size_t bstep = (size_t)4 * LPC * NG;
    const unsigned long long* bsrc =
        bnd + tri_slot<NP, LPC>(chain, k > 0 ? k - 1 : k, 0, nchains, H) + (size_t)jj * LPC + rl;
    unsigned long long* pdst = bnd + tri_slot<NP, LPC>(chain, k, 0, nchains, H) + (size_t)jj * LPC + rl;
    auto bvalid = [&](int t) {
        const int xx = U0 + bcol - (H - 1) + t;
        return k > 0 && t >= 0 && xx >= 0 && xx < W1;
    };
    auto bload = [&](int t, unsigned long long (&g)[NG]) {
        const unsigned long long* q = bsrc + (size_t)clampi(t, 0, H - 1) * bstep;
#pragma unroll
        for (int i = 0; i < NG; i++) g[i] = __hip_atomic_load(q + 4 * LPC * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // item t into LDS row buf, spinning until the producer's tag shows
    auto bconsume = [&](int t, int buf, unsigned long long (&g)[NG]) {
        const bool need = jlive && bvalid(t);
        bool ok = true;
#pragma unroll
        for (int i = 0; i < NG; i++) ok &= !need || (unsigned)(g[i] >> 48) == tag16;
        if (!__all(ok)) {
            const unsigned long long sp0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
            unsigned spins = 0;
            while (!__all(ok)) {
                // give up after spin_limit polls, or soon after any block of
                // this launch gave up (status = this launch's epoch): the
                // launch then drains, the median kernel writes its maps as
                // INVALID and the host reports MVSV_E_TIMEOUT
                if (++spins > spin_limit) {
                    if (lane == 0) {
                        __hip_atomic_store(status, (int)epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        __hip_atomic_store(report, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    }
                    break;
                }
                if ((spins & 63) == 0 &&
                    __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (int)epoch)
                    break;
                __builtin_amdgcn_s_sleep(1);
                const unsigned long long* q = bsrc + (size_t)clampi(t, 0, H - 1) * bstep;
                ok = true;
#pragma unroll
                for (int i = 0; i < NG; i++) {
                    g[i] = __hip_atomic_load(q + 4 * LPC * i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok &= !need || (unsigned)(g[i] >> 48) == tag16;
                }
            }
            if (stats) {
                st_spin += __builtin_amdgcn_s_memtime() - sp0;
                st_n += spins;
            }
        }
        uint32_t v[NP];
        int mn;
        TG::unpack(g, v, mn);
        if (jlive) {
            uint32_t* dst = lcol(buf, bdir, bcol);
#pragma unroll
            for (int i = 0; i < NP; i++) dst[i * LPC] = need ? v[i] : 0u;
            // the compute waves keep column minima packed (m, m) in the no-wrap form
            if (rl == 0) *mcol(buf, bdir, bcol) = need ? (NW ? (int)((uint32_t)mn * 0x10001u) : mn) : 0;
        }
    };
    // publish step t of this strip's columns 0 and 1 (LDS row buf) for the left
    // strip; unconditional stores (idle lanes and unused steps hit unread slots)
    auto publish = [&](int t, int buf) {
        uint32_t v[NP];
        const uint32_t* src = lcol(buf, bdir, pcol);
#pragma unroll
        for (int i = 0; i < NP; i++) v[i] = src[i * LPC];
        const int mn = *mcol(buf, bdir, pcol);
        unsigned long long g[NG];
        TG::pack(v, mn, tag, g);
        unsigned long long* q = pdst + (size_t)clampi(t, 0, H - 1) * bstep;
#pragma unroll
        for (int i = 0; i < NG; i++) __hip_atomic_store(q + 4 * LPC * i, g[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (trace_h && comm0 && lane == 0)  // MVSV_TRI_TRACE: when step t went out (100 MHz clock)
            stats[(size_t)bx * (8 + 2 * trace_h) + 8 + t] = __builtin_amdgcn_s_memrealtime();
    };

    // ---- compute waves ----
    // cell (x, y) of step t: y*W1 + x = c0 + t*(sy*W1 + 1), element offsets in
    // int32 (the launcher checks H*W1*D < 2^31); cells outside the image read
    // the frame's first cell and store into the lane's dummy slot
    auto cell_x = [&](int t) { return U - (H - 1) + t; };
    const int c0D = ((sy > 0 ? 0 : (H - 1) * W1) + U - (H - 1)) * D;
    const int cstepD = (sy * W1 + 1) * D;
    auto cell_off = [&](int t) -> uint32_t {  // >= 0: in-image cells only
        return (unsigned)cell_x(t) < (unsigned)W1 ? (uint32_t)(c0D + t * cstepD) : 0u;
    };
    uint32_t la[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) la[p] = 0u;
    int ma = 0;
    CI cb[PF];
    unsigned long long bg[BF][NG];

    __syncthreads();  // LDS zeroed
    if (comm) __builtin_amdgcn_s_setprio(1);  // the exchange wave gates every step's barrier
    if (comm) {
        bload(tb - 1, bg[0]);
        bconsume(tb - 1, 1, bg[0]);  // the right strip's cells the first step reads
#pragma unroll
        for (int j = 0; j < BF; j++) bload(tb + j, bg[j]);
    } else {
#pragma unroll
        for (int j = 0; j < PF; j++) cb[j].load(CI::at(Cf, cell_off(min(tb + j, te - 1))));
    }
    __syncthreads();

    // The exchange wave and the compute waves run separate loops with the same
    // number of block barriers (one per step): the register allocator then
    // gives each path its own registers (the exchange wave's granule prefetch
    // no longer competes with the compute waves' C prefetch).
    auto comm_step = [&](int i, int j) {
        const int t = tb + i;
        const int cur = i & 1, prv = cur ^ 1;
        if (i > 0) publish(t - 1, prv);
        bconsume(t, cur, bg[j % BF]);
        if (trace_h && comm0 && lane == 0)  // when the producer's step t was in
            stats[(size_t)bx * (8 + 2 * trace_h) + 8 + trace_h + t] = __builtin_amdgcn_s_memrealtime();
        bload(t + BF, bg[j % BF]);
        __syncthreads();
    };
    // One step: the three recurrences one after the other (each direction's
    // neighbours, update, column minimum and LDS hand-over before the next
    // starts, so only one direction's temporaries are live); the output word
    // accumulates the deltas as they come.
    const uint32_t p2x2 = (uint32_t)(P2 & 0xffff) * 0x10001u;
    auto step = [&](int i, int j) {
        const int t = tb + i;
        const int cur = i & 1, prv = cur ^ 1;
        const int x = cell_x(t);
        const bool valid = x >= 0 && x < W1;
        const bool allv = __all(valid);
        uint32_t c[NP];
        cb[j % PF].get(c);
        cb[j % PF].load(CI::at(Cf, cell_off(min(t + PF, te - 1))));
        // the column minimum of one direction (packed (m, m) in the no-wrap
        // form) and the next step's delta from it
        auto dmin = [&](const uint32_t (&n)[NP]) -> int {
            if constexpr (LPC == 32)
                return seg_min_i32<32>(NW ? (int)lane_min_pk<NP>(n) : lane_min_row<NP>(n));
            else if constexpr (NW)
                return seg_lane_min<LPC>((int)lane_min_pk<NP>(n));
            else
                return seg_lane_min<LPC>(lane_min_row<NP>(n));
        };
        // one recurrence step over the column's LPC lanes
        auto rstep = [&](const uint32_t (&lp)[NP], uint32_t delta2, uint32_t (&n)[NP], uint32_t (&u)[NP]) {
            if constexpr (LPC == 32)
                sgm_step_seg_t<NP, 32, NW>(lp, delta2, p1x2, c, n, u, rl == 0, rl == LPC - 1);
            else
                sgm_step_row_t<NP, NW, LPC>(lp, delta2, p1x2, c, n, u);
        };
        auto dl2 = [&](int m) -> uint32_t {
            if constexpr (NW)
                return (uint32_t)m + p2x2;  // (minLp + P2) x 2, no carry between halves
            else
                return sgm_delta2<false>(m, P2);
        };
        // sum of the three deltas t_r + P2 = 3 P2 - (u_a + u_b + u_c) (no-wrap)
        // or t_a + t_b + t_c + 3 P2, exact in u16 wrap arithmetic
        // (no-wrap: 3 P2 minus three u <= P2 each never borrows -> one full-rate v_sub_u32)
        auto acc = [&](uint32_t o, uint32_t u) -> uint32_t { return NW ? sub2_nb(o, u) : pk_add_u16(o, u); };
        uint32_t o[NP];
#if MVSV_TRI_STEP_SEQ
        {  // (1, sy): the strip's own column, state in registers
            uint32_t n[NP], u[NP];
            rstep(la, dl2(ma), n, u);
#pragma unroll
            for (int p = 0; p < NP; p++) o[p] = acc(p2x3, u[p]);
            const int mn = dmin(n);
            if (__builtin_expect(!allv, 0)) {
#pragma unroll
                for (int p = 0; p < NP; p++) n[p] = valid ? n[p] : 0u;
            }
#pragma unroll
            for (int p = 0; p < NP; p++) la[p] = n[p];
            ma = valid ? mn : 0;
        }
#pragma unroll
        for (int dir = 0; dir < 2; dir++) {  // (0, sy) from column col + 1, (-1, sy) from col + 2
            uint32_t pv[NP];
            const uint32_t* src = lcol(prv, dir, col + 1 + dir);
#pragma unroll
            for (int p = 0; p < NP; p++) pv[p] = src[p * LPC];
            const int mp = *mcol(prv, dir, col + 1 + dir);
            uint32_t n[NP], u[NP];
            rstep(pv, dl2(mp), n, u);
#pragma unroll
            for (int p = 0; p < NP; p++) o[p] = acc(o[p], u[p]);
            const int mn = dmin(n);
            if (__builtin_expect(!allv, 0)) {
#pragma unroll
                for (int p = 0; p < NP; p++) n[p] = valid ? n[p] : 0u;
            }
            uint32_t* dst = lcol(cur, dir, col);
#pragma unroll
            for (int p = 0; p < NP; p++) dst[p * LPC] = n[p];
            if (rl == 0) *mcol(cur, dir, col) = valid ? mn : 0;
        }
#else
        // the three recurrences side by side (the compiler interleaves their
        // independent chains; measured faster than one after the other)
        uint32_t pb[NP], pc[NP];
        {
            const uint32_t* sb = lcol(prv, 0, col + 1);
            const uint32_t* sc = lcol(prv, 1, col + 2);
#pragma unroll
            for (int p = 0; p < NP; p++) {
                pb[p] = sb[p * LPC];
                pc[p] = sc[p * LPC];
            }
        }
        const int mb = *mcol(prv, 0, col + 1), mc = *mcol(prv, 1, col + 2);
        uint32_t na[NP], nb[NP], nc[NP], ta[NP], tb_[NP], tc[NP];
        rstep(la, dl2(ma), na, ta);
        rstep(pb, dl2(mb), nb, tb_);
        rstep(pc, dl2(mc), nc, tc);
        const int mna = dmin(na), mnb = dmin(nb), mnc = dmin(nc);
#pragma unroll
        for (int p = 0; p < NP; p++) o[p] = acc(acc(acc(p2x3, ta[p]), tb_[p]), tc[p]);
        if (__builtin_expect(!allv, 0)) {
#pragma unroll
            for (int p = 0; p < NP; p++) {
                na[p] = valid ? na[p] : 0u;
                nb[p] = valid ? nb[p] : 0u;
                nc[p] = valid ? nc[p] : 0u;
            }
        }
#pragma unroll
        for (int p = 0; p < NP; p++) la[p] = na[p];
        ma = valid ? mna : 0;
        {
            uint32_t* db = lcol(cur, 0, col);
            uint32_t* dc = lcol(cur, 1, col);
#pragma unroll
            for (int p = 0; p < NP; p++) {
                db[p * LPC] = nb[p];
                dc[p * LPC] = nc[p];
            }
            if (rl == 0) {
                *mcol(cur, 0, col) = valid ? mnb : 0;
                *mcol(cur, 1, col) = valid ? mnc : 0;
            }
        }
#endif
        AV::store(valid ? acc_addu(Af, cell_off(t)) : dp, o);
        __syncthreads();
    };
    const int len = te - tb;
    int i = 0;
    if (comm) {
        for (; i + kTriUnroll <= len; i += kTriUnroll) {
#pragma unroll
            for (int j = 0; j < kTriUnroll; j++) comm_step(i + j, j);
        }
#pragma unroll
        for (int j = 0; j < kTriUnroll; j++)
            if (i + j < len) comm_step(i + j, j);
    } else {
        for (; i + kTriUnroll <= len; i += kTriUnroll) {
#pragma unroll
            for (int j = 0; j < kTriUnroll; j++) step(i + j, j);
        }
#pragma unroll
        for (int j = 0; j < kTriUnroll; j++)
            if (i + j < len) step(i + j, j);
    }
    if (comm) {
        publish(te - 1, (len - 1) & 1);
        if (stats && comm0 && lane == 0) {
            unsigned long long* q = stats + (size_t)bx * (8 + 2 * trace_h);
            q[0] = st_t0;
            q[1] = __builtin_amdgcn_s_memtime();
            q[2] = st_spin;
            q[3] = st_n;
            q[4] = (unsigned long long)len;
            q[5] = (unsigned long long)k;
            q[6] = (unsigned long long)pass;
            q[7] = (unsigned long long)tb;
        }
    }
}

// ---------------------------------------------------------------------------
// 5b. last direction (R->L) + WTA + uniqueness + sub-pixel + LR check with 16
// lanes per image row (4 rows per wave).  The right-view map is built with
// order-independent atomicMin on keys (minS << 16 | 0xFFFF - x): smallest cost,
// then the largest x -- exactly OpenCV's descending scan with a strict '>'.
// ---------------------------------------------------------------------------

// Raw accumulator words of one lane (2*NP disparities): the NACC planes are
// summed in storage format -- u8 bytes never carry because the total over all
// directions is <= ndir*P2 <= 255 (acc_is_u8) -- and unpacked to u16 pairs once.
template <int NP, typename AccT>
struct AccRaw;
template <int NP>
struct AccRaw<NP, uint8_t> {
    static constexpr int NW = NP >= 2 ? NP / 2 : 1;
    static __device__ __forceinline__ void load(const uint8_t* p, uint32_t (&w)[NW])
    {
        if constexpr (NP == 1) {
            w[0] = *(const uint16_t*)p;
        } else if constexpr (NP == 2) {
            w[0] = *(const uint32_t*)p;
        } else if constexpr (NP == 4) {
            const uint2 t = *(const uint2*)p;
            w[0] = t.x;
            w[1] = t.y;
        } else {
            const uint4 t = *(const uint4*)p;
            w[0] = t.x;
            w[1] = t.y;
            w[2] = t.z;
            w[3] = t.w;
        }
    }
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return a + b; }
    static __device__ __forceinline__ void unpack(const uint32_t (&w)[NW], uint32_t (&v)[NP])
    {
#pragma unroll
        for (int p = 0; p < NP; p++) v[p] = u8x2_to_u16x2(w[p >> 1], p & 1);
    }
    template <int NACC>
    static __device__ __forceinline__ void combine(const uint32_t (&w)[NACC][NW], uint32_t (&v)[NP])
    {
        uint32_t s[NW];
#pragma unroll
        for (int k = 0; k < NW; k++) {
            s[k] = w[0][k];
#pragma unroll
            for (int i = 1; i < NACC; i++) s[k] = add(s[k], w[i][k]);
        }
        unpack(s, v);
    }
};
template <int NP>
struct AccRaw<NP, uint16_t> {
    static constexpr int NW = NP;
    static __device__ __forceinline__ void load(const uint16_t* p, uint32_t (&w)[NW])
    {
        AccVec<NP, uint16_t>::load(p, w);
    }
    static __device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b)
    {
        return AccVec<NP, uint16_t>::add(a, b);
    }
    static __device__ __forceinline__ void unpack(const uint32_t (&w)[NW], uint32_t (&v)[NP])
    {
#pragma unroll
        for (int p = 0; p < NP; p++) v[p] = w[p];
    }
    template <int NACC>
    static __device__ __forceinline__ void combine(const uint32_t (&w)[NACC][NW], uint32_t (&v)[NP])
    {
        uint32_t s[NW];
#pragma unroll
        for (int k = 0; k < NW; k++) {
            s[k] = w[0][k];
#pragma unroll
            for (int i = 1; i < NACC; i++) s[k] = add(s[k], w[i][k]);
        }
        unpack(s, v);
    }
};
// Nibble planes (AccVec<NP, nib2_t> layout): the planes' sums exceed a
// nibble, so each word is split into its even and odd nibbles as bytes
// (E, O), the planes are added bytewise (<= NACC * 15), then spread to pairs.
template <int NP>
struct AccRaw<NP, nib2_t> {
    static constexpr int NW = NP >= 4 ? NP / 4 : 1;
    static __device__ __forceinline__ void load(const nib2_t* p, uint32_t (&w)[NW])
    {
        if constexpr (NP == 1) {
            w[0] = *(const uint8_t*)p;
        } else if constexpr (NP == 2) {
            w[0] = *(const uint16_t*)p;
        } else if constexpr (NP == 4) {
            w[0] = *(const uint32_t*)p;
        } else {
            const uint2 t = *(const uint2*)p;
            w[0] = t.x;
            w[1] = t.y;
        }
    }
    template <int NACC>
    static __device__ __forceinline__ void combine(const uint32_t (&w)[NACC][NW], uint32_t (&v)[NP])
    {
        constexpr uint32_t M = 0x0f0f0f0fu;
#pragma unroll
        for (int k = 0; k < NW; k++) {
            uint32_t E = w[0][k] & M, O = (w[0][k] >> 4) & M;
#pragma unroll
            for (int i = 1; i < NACC; i++) {
                E += w[i][k] & M;
                O += (w[i][k] >> 4) & M;
            }
            if constexpr (NP >= 4) {
                // E bytes: d0 d1 d4 d5, O bytes: d2 d3 d6 d7
                v[4 * k + 0] = __builtin_amdgcn_perm(0u, E, 0x0c010c00u);
                v[4 * k + 1] = __builtin_amdgcn_perm(0u, O, 0x0c010c00u);
                v[4 * k + 2] = __builtin_amdgcn_perm(0u, E, 0x0c030c02u);
                v[4 * k + 3] = __builtin_amdgcn_perm(0u, O, 0x0c030c02u);
            } else if constexpr (NP == 2) {
                // E bytes: lo0 hi0, O bytes: lo1 hi1
                v[0] = __builtin_amdgcn_perm(0u, E, 0x0c010c00u);
                v[1] = __builtin_amdgcn_perm(0u, O, 0x0c010c00u);
            } else {
                v[0] = (E & 0xffu) | ((O & 0xffu) << 16);
            }
        }
    }
};

// Steps of C / accumulator prefetch: as deep as ~160 VGPRs of buffers allow
// (a power of two dividing the 16-step flush period).  The kernel is bound by
// load latency at ~2 waves per SIMD, so depth is what buys bandwidth.
template <int NP, int NACC, typename AccT, bool UQ>
constexpr int final16_pf()
{
    constexpr int words = NP + NACC * AccRaw<NP, AccT>::NW;  // VGPRs per step
    // three or more planes (MODE_HH, side by side) unpack more per step: at
    // 160 buffer VGPRs those instances spilled 36-105 VGPRs (round 6 audit)
    constexpr int budget = UQ ? 96 : (NACC >= 3 ? 80 : 160);
    return budget / words >= 16 ? 16 : (budget / words >= 8 ? 8 : 4);
}

// raw buffer loads of BYTES bytes into little-endian words (zero-extended)
constexpr int kBufWord3 = 0x00020000;  // buffer descriptor word 3: 32-bit data format
template <int BYTES, int NWD>
__device__ __forceinline__ void buf_words(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff,
                                          uint32_t (&w)[NWD])
{
    if constexpr (BYTES == 1) {
        w[0] = __builtin_amdgcn_raw_buffer_load_b8(r, voff, soff, 0);
    } else if constexpr (BYTES == 2) {
        w[0] = __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, 0);
    } else if constexpr (BYTES == 4) {
        w[0] = __builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, 0);
    } else if constexpr (BYTES == 8) {
        const auto t = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
        w[0] = t[0];
        w[1] = t[1];
    } else {
        static_assert(BYTES % 16 == 0 && NWD == BYTES / 4, "buffer load size");
#pragma unroll
        for (int q = 0; q < BYTES / 16; q++) {
            const auto t = __builtin_amdgcn_raw_buffer_load_b128(r, voff + 16 * q, soff, 0);
#pragma unroll
            for (int k = 0; k < 4; k++) w[4 * q + k] = t[k];
        }
    }
}

// a * b + c per u16 half, saturated at 0xffff (VOP3P clamp)
__device__ __forceinline__ uint32_t pk_mad_u16_clamp(uint32_t a, uint32_t b, uint32_t c)
{
    uint32_t r;
    asm("v_pk_mad_u16 %0, %1, %2, %3 clamp" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// NACC accumulator planes (A + i * plane) hold the summed deltas of disjoint
// direction groups written by concurrent passes; their sum is the S input.
// UQ: uniquenessRatio > 0.
// RESF (round 4; uniquenessRatio == 0 only, no-wrap regime): the recurrence
// and the WTA run on the residual plane R instead of C.  With C' = C - m
// (m = the pixel's minimum cost, Mv) and C'' = min(C', 2 P2) = R - P2, the
// step computes S'' = n C'' + sum of deltas (n = 8 or 5 directions);
// S = min(n (m - P2) + S', MAX_COST) has the same argmin and ties as S'' (the
// minimum of S' is <= n P2 < 2 n P2 <= S'' of any clamped d), and with
// uniquenessRatio 0 no d is ever rejected.  Only the sub-pixel fit needs
// exact S(best -+ 1): where S'' >= 2 n P2 the residual
// may be clamped and the flush loads C(best -+ 1) from the cost volume (one
// 2-byte gather per pixel, issued one flush ahead of its use so the prefetch
// loads are never waited for).
template <int NP, int NACC, typename AccT, bool UQ, int LPR, bool NOWRAP = false, bool RESF = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NP >= 8 ? 1 : 2))) void sgbm_final16_kernel(const int16_t* __restrict__ C,
                                                         const AccT* __restrict__ A, size_t plane,
                                                         int H, int W, SgbmEff e,
                                                         int16_t* __restrict__ raw,
                                                         uint32_t* __restrict__ keys,
                                                         int16_t* __restrict__ dummy,
                                                         const uint8_t* __restrict__ Rv,
                                                         const uint16_t* __restrict__ Mv)
{
    static_assert(!(RESF && UQ), "the residual final kernel needs uniquenessRatio 0");
    using AR = AccRaw<NP, AccT>;
    constexpr int NW = AR::NW;
    // 32 lanes per row: twice the waves, so a shallower prefetch keeps the
    // kernel at <= 128 VGPRs (4 waves per SIMD); wide slots (u16 planes of D =
    // 256, config 5: 12 words per step) take 4 steps -- 8 spilled 14 VGPRs
    // into scratch (round 6 dispatch census, tests/test_kernel_scratch.py).
    // The step loop is unrolled by LPR, so PF must divide it.
    constexpr int kF32Words = (RESF ? 1 : NP) + NACC * AccRaw<NP, AccT>::NW;
    constexpr int PF = LPR == 32 ? (kF32Words > 24 ? 2 : kF32Words > 10 ? 4 : MVSV_FINAL32_PF)
                                 : (final16_pf<NP, NACC, AccT, UQ>() < LPR ? final16_pf<NP, NACC, AccT, UQ>() : LPR);
    static_assert(LPR % PF == 0, "prefetch slots must divide the unrolled step loop");
    constexpr int RPW = 64 / LPR;     // image rows per wave
    constexpr int DR = 2 * NP * LPR;  // disparities of a row (D)
    // S of the current step, one D-vector per row: S[best -+ 1] come back
    // through LDS instead of lane shuffles.
    __shared__ __attribute__((aligned(16))) uint16_t srow[RPW * DR];
    const int lane = threadIdx.x;
    const int row = lane / LPR, rl = lane % LPR;
    const bool seg_first = rl == 0, seg_last = rl == LPR - 1;
    const int yr = blockIdx.x * RPW + row;
    const bool exists = yr < H;
    const int y = min(yr, H - 1);
    const int f = blockIdx.y;
    const int D = e.D, W1 = e.W1, minD = e.minD, minX1 = e.minX1;
    const int INV = e.invalid;
    int16_t* orow = raw + ((size_t)f * H + y) * W;
    uint32_t* krow = keys + ((size_t)f * H + y) * W;
    if (exists)
        for (int x = rl; x < W; x += LPR) {
            orow[x] = (int16_t)INV;
            krow[x] = 0xffffffffu;
        }
    __threadfence_block();
    __syncthreads();

    const bool lane_rule = !e.fullDP && !(e.variant & MVSV_VARIANT_WTA_MIN_D);
    const size_t frame = (size_t)H * W1 * D;
    const int d0 = rl * 2 * NP;
    uint16_t* ms = srow + row * DR;
    uint32_t lp[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) lp[p] = 0u;
    const uint32_t p1x2 = (uint32_t)(e.P1 & 0xffff) * 0x10001u;
    const uint32_t p2x2 = (uint32_t)(e.P2 & 0xffff) * 0x10001u;
    // S = min(ndir*(C - P2) + sum of deltas, MAX_COST) = min((ndir-1)*cb + L + acc, MAX_COST)
    // with cb = C - P2, L = cb + delta of the R->L direction computed here
    const uint32_t ndm1 = (uint32_t)(e.fullDP ? 7 : 4) * 0x10001u;
    const int uq = e.uniq;
    // tie order of the WTA key: d, or OpenCV's SIMD lane order for MODE_SGBM
    uint32_t subk[2 * NP];
#pragma unroll
    for (int i = 0; i < 2 * NP; i++) {
        const int d = d0 + i;
        subk[i] = lane_rule ? (uint32_t)(((d & 7) << 12) | (d >> 3)) : (uint32_t)d;
    }
    uint32_t dpair[NP];  // (d, d + 1) of each packed pair
#pragma unroll
    for (int p = 0; p < NP; p++) dpair[p] = (uint32_t)(d0 + 2 * p) | ((uint32_t)(d0 + 2 * p + 1) << 16);
    int minp = 0;

    // cost words per prefetch slot: NP packed pairs of C, or the lane's 2 NP
    // residual nibbles (NP bytes, one word)
    constexpr int NCW = RESF ? 1 : NP;
    uint32_t cw[PF][NCW];
    uint32_t ab[PF][NACC][NW];
    // Buffer loads: one descriptor per volume over the wave's RPW rows, the
    // lane's row/disparity offset in a VGPR and the column (x = W1 - 1 - t)
    // in the scalar offset, so the per-step address update is SALU work.
    const int ybase = (int)blockIdx.x * RPW;  // <= y
    const size_t rbase = f * frame + (size_t)ybase * W1 * D;
    const uint32_t loff = (uint32_t)((y - ybase) * W1 * D + d0);  // elements, even
    constexpr uint32_t kAccNum = (uint32_t)sizeof(AccT), kAccDen = AccEpu<AccT>::v;  // bytes per element
    constexpr uint32_t kCNum = RESF ? 1u : 4u, kCDen = 2u;  // cost input bytes per element: 1/2 or 2
    const int nrec_c = (int)((uint32_t)(RPW * W1 * D) * kCNum / kCDen);
    const int nrec_a = (int)((uint32_t)(RPW * W1 * D) * kAccNum / kAccDen);
    const void* cbase = RESF ? (const void*)(Rv + rbase / 2) : (const void*)(C + rbase);
    const __amdgpu_buffer_rsrc_t rc_c =
        __builtin_amdgcn_make_buffer_rsrc((void*)cbase, (short)0, nrec_c, kBufWord3);
    __amdgpu_buffer_rsrc_t rc_a[NACC];
#pragma unroll
    for (int i = 0; i < NACC; i++)
        rc_a[i] = __builtin_amdgcn_make_buffer_rsrc(
            (void*)acc_add(A, (ptrdiff_t)(rbase + (size_t)i * plane)), (short)0, nrec_a, kBufWord3);
    const uint32_t vo_c = loff * kCNum / kCDen, vo_a = loff * kAccNum / kAccDen;
    auto prefetch = [&](int j, ptrdiff_t t) {
        const uint32_t xd = (uint32_t)((W1 - 1 - (int)t) * D);
        buf_words<(int)(2 * NP * kCNum / kCDen)>(rc_c, vo_c, xd * kCNum / kCDen, cw[j]);
#pragma unroll
        for (int i = 0; i < NACC; i++)
            buf_words<2 * NP * kAccNum / kAccDen>(rc_a[i], vo_a, xd * kAccNum / kAccDen, ab[j][i]);
    };
#pragma unroll
    for (int j = 0; j < PF; j++) prefetch(j, min(j, W1 - 1));
    // Per step the row's 16 lanes agree on K = (minS << 16 | tie-order sub),
    // S[best-1], S[best+1] and the uniqueness verdict; they park that record in
    // LDS slot (s & 15) of the row, and every 16 steps lane rl picks up record
    // rl and the 16 lanes finish 16 columns at once (sub-pixel division, raw
    // store, right-view atomicMin) -- the per-step path stays branch-free so
    // consecutive steps overlap.
    __shared__ uint2 srec[RPW * LPR];
    uint2* recs = srec + row * LPR;
    auto body = [&](int s, int j) {
        const uint32_t delta2 = sgm_delta2<NOWRAP>(minp, e.P2);
        uint32_t c[NP], ln[NP], st[NP], acc[NP], tt[NP];
        if constexpr (RESF) {
            CostIn<NP, true> ci;
            ci.w[0] = cw[j][0];
            ci.get(c);
        } else {
#pragma unroll
            for (int p = 0; p < NP; p++) c[p] = cw[j][p];
        }
        sgm_step_seg_t<NP, LPR, NOWRAP>(lp, delta2, p1x2, c, ln, tt, seg_first, seg_last);
        minp = seg_min_i32<LPR>(lane_min_row<NP>(ln));
        AR::template combine<NACC>(ab[j], acc);
        uint32_t key = 0x7fffffffu;
#pragma unroll
        for (int p = 0; p < NP; p++) {
            // residual form (RESF): R >= P2, L + deltas <= 4 P2 + 7 P2 -- the
            // full-rate 32-bit sub / add never borrow or carry
            const uint32_t cbv = RESF ? sub2_nb(c[p], p2x2) : pk_sub_u16(c[p], p2x2);
            const uint32_t sv = pk_mad_u16_clamp(cbv, ndm1, RESF ? add2_nc(ln[p], acc[p]) : pk_add_u16(ln[p], acc[p]));
            st[p] = pk_min_u16(sv, 0x7fff7fffu);
            lp[p] = ln[p];
            const uint32_t klo = (st[p] << 16) | subk[2 * p];
            const uint32_t khi = (st[p] & 0xffff0000u) | subk[2 * p + 1];
            key = min(key, min(klo, khi));
        }
        const int K = seg_min_i32<LPR>((int)key);
        const int minS = K >> 16;
        const int sub = K & 0xffff;
        const int best = lane_rule ? (((sub & 0xfff) << 3) | (sub >> 12)) : sub;
        // S[best -+ 1] (clamped into [0, D)) through the row's LDS vector
        {
            Vec<NP> o;
#pragma unroll
            for (int p = 0; p < NP; p++) o.v[p] = st[p];
            o.store((int16_t*)(ms + d0));
        }
        // the wave barriers order the lanes' LDS hand-over for the compiler
        // (without them it moved accesses across lanes' writes: wrong maps)
        __builtin_amdgcn_wave_barrier();
        const int bm = max(best - 1, 0), bp = min(best + 1, DR - 1);
        const int Sm = ms[bm], Sp = ms[bp];
        int rej = 0;
        if constexpr (UQ) {
            // min of S outside [best-1, best+1]: y = best + 1 - d is <= 2
            // (unsigned) exactly there; those cells are lifted to >= 0xfffd
            const uint32_t b2 = (uint32_t)(best + 1) * 0x10001u;
            uint32_t m2 = 0xffffffffu;
#pragma unroll
            for (int p = 0; p < NP; p++) {
                const uint32_t yv = pk_sub_u16(b2, dpair[p]);
                const uint32_t lift = pk_sub_u16(pk_min_u16(yv, 0x00030003u), 0x00030003u);
                m2 = pk_min_u16(m2, pk_max_u16(st[p], lift));
            }
            const int m2r = seg_min_i32<LPR>((int)min(m2 & 0xffffu, m2 >> 16));
            rej = m2r < 0xfffd && m2r * (100 - uq) < minS * 100;
        }
        recs[s & (LPR - 1)] = make_uint2((uint32_t)K | ((uint32_t)rej << 31),
                                  ((uint32_t)Sp << 16) | ((uint32_t)Sm & 0xffffu));
        __builtin_amdgcn_wave_barrier();
    };
    // lane rl finishes column s0 + rl of the sweep (x = W1 - 1 - s)
    // Branch-free around memory (so the prefetch loads keep their exact
    // vmcnt accounting across the flush): a lane without a column stores to
    // its dummy slot, a rejected column rewrites INVALID, and an atomicMin
    // that must not count carries the all-ones key (a no-op).
    int16_t* dslot = dummy + (blockIdx.x & 63) * 64 + lane;
    // store + right-view key of one finished column (x, exact minS, Sm, Sp)
    auto finish = [&](bool own, int x, int best, int minS, int Sm, int Sp, int kRej) {
        if (minS >= kMaxCost) best = -1;  // no strict minimum below MAX_COST
        const int den = max(Sm + Sp - 2 * minS, 1);
        const int frac = ((Sm - Sp) * kDispScale + den) / (den * 2);
        // arithmetic mask, not a select: the division stays unconditional (no
        // branch inside the loop body)
        const int d16 = best * kDispScale + (frac & -(int)(0 < best && best < D - 1));
        const int16_t v = kRej ? (int16_t)INV : (int16_t)(d16 + minD * kDispScale);
        *(own ? orow + x + minX1 : dslot) = v;
        const int x2 = x + minX1 - best - minD;
        const bool hit = own && !kRej && minS < kMaxCost && x2 >= 0 && x2 < W;
        atomicMin(krow + clampi(x2, 0, W - 1),
                  hit ? (((uint32_t)minS << 16) | (uint32_t)(0xffff - x)) : 0xffffffffu);
    };
    auto flush = [&](int s0, int cnt) {
        const int s = s0 + rl;
        const bool own = exists && rl < cnt;
        const uint2 rec = recs[rl];
        const uint32_t kK = rec.x & 0x7fffffffu, kS = rec.y;
        const int kRej = (int)(rec.x >> 31);
        const int minS = (int)(kK >> 16);
        const int sub = (int)(kK & 0xffffu);
        const int best = lane_rule ? (((sub & 0xfff) << 3) | (sub >> 12)) : sub;
        const int Sm = (int)(int16_t)(kS & 0xffffu), Sp = (int)(int16_t)(kS >> 16);
        finish(own, W1 - 1 - s, best, minS, Sm, Sp, kRej);
    };
    // RESF: a flush reads its columns' records and issues their loads (the
    // pixel minimum, C(best -+ 1) where the residual may be clamped); the next
    // flush (or the row end) finishes them.  Pending state per lane: the
    // record and three loaded values (the column and ownership follow from
    // the pending flush's first step and count, wave-uniform).
    struct Pend {
        uint2 rec;
        int mC;
        uint2 cw;  // C[base .. base + 3] of the column, base = min((best - 1) & ~1, D - 4)
    } pend{};
    int pend_s0 = 0, pend_cnt = 0;
    const int16_t* crow = C + f * frame + (size_t)y * W1 * D;
    const uint16_t* mrowp = RESF ? Mv + ((size_t)f * H + y) * W1 : nullptr;
    const int ndir = e.fullDP ? 8 : 5;
    const int clampS = ndir * 2 * e.P2;  // S'' >= this: C'' may be the clamp value
    auto rec_best = [&](uint32_t kK) {
        const int sub = (int)(kK & 0xffffu);
        return lane_rule ? (((sub & 0xfff) << 3) | (sub >> 12)) : sub;
    };
    auto finish_res = [&](const Pend& q, int s0, int cnt) {
        const uint32_t kK = q.rec.x & 0x7fffffffu;
        const int base = ndir * (q.mC - e.P2);  // S = min(base + S', MAX_COST)
        auto exact = [&](int Spp, int cv) -> int {
            // S'' = ndir C'' + deltas; where the flush loaded C(d) (S'' >=
            // clampS: cv is exact, else a placeholder) replace C'' = min(C', 2 P2)
            // by C'
            const int c1 = Spp >= clampS ? cv - q.mC : 0;
            return min(base + Spp + ndir * (c1 - min(c1, 2 * e.P2)), kMaxCost);
        };
        const int best = rec_best(kK);
        const int bm = max(best - 1, 0), bp = min(best + 1, D - 1);
        const int cb0 = min(bm & ~1, D - 4);
        auto cword = [&](int d) -> int {  // C(d) out of the loaded 4-element window
            const int i = d - cb0;
            const uint32_t w = (i & 2) ? q.cw.y : q.cw.x;
            return (int)((i & 1) ? (w >> 16) : (w & 0xffffu));
        };
        const int Sm = exact((int)(q.rec.y & 0xffffu), cword(bm)), Sp = exact((int)(q.rec.y >> 16), cword(bp));
        finish(exists && rl < cnt, W1 - 1 - (s0 + rl), best, min(base + (int)(kK >> 16), kMaxCost), Sm, Sp, 0);
    };
    auto flush_res = [&](int s0, int cnt) {
        Pend q;
        const bool own = exists && rl < cnt;
        q.rec = recs[rl];
        const int best = rec_best(q.rec.x & 0x7fffffffu);
        const int xc = own ? W1 - 1 - (s0 + rl) : 0;
        q.mC = mrowp[xc];
        // C(best - 1) and C(best + 1) in one 8-byte load (4-byte aligned, inside
        // the pixel's D costs); one shared address for the lanes that need no
        // exact cost
        const int cb0 = min(max(best - 1, 0) & ~1, D - 4);
        const bool need = own && ((int)(q.rec.y & 0xffffu) >= clampS || (int)(q.rec.y >> 16) >= clampS);
        q.cw = *(const uint2*)(crow + (need ? (size_t)xc * D + cb0 : 0));
        finish_res(pend, pend_s0, pend_cnt);  // the previous flush's columns (none the first time)
        pend = q;
        pend_s0 = s0;
        pend_cnt = cnt;
    };
    int s = 0;
    for (; s + LPR <= W1; s += LPR) {
#pragma unroll
        for (int j = 0; j < LPR; j++) {
            body(s + j, j % PF);
            prefetch(j % PF, min(s + j + PF, W1 - 1));
        }
        if constexpr (RESF)
            flush_res(s, LPR);
        else
            flush(s, LPR);
    }
    const int rem = W1 - s;
#pragma unroll
    for (int j = 0; j < LPR; j++) {
        if (j < rem) {
            body(s + j, j % PF);
            prefetch(j % PF, min(s + j + PF, W1 - 1));
        }
    }
    if constexpr (RESF) {
        if (rem > 0) flush_res(s, rem);
        finish_res(pend, pend_s0, pend_cnt);
    } else {
        if (rem > 0) flush(s, rem);
    }
    __threadfence_block();
    __syncthreads();
    if (!exists) return;
    // left-right check (src: OpenCV 3.4 final loop) -- reads the finished row
    for (int x = minX1 + rl; x < e.maxX1; x += LPR) {
        const int v = orow[x];
        if (v == INV) continue;
        const int dlo = v >> kDispShift, dhi = (v + kDispScale - 1) >> kDispShift;
        const int xl = x - dlo, xh = x - dhi;
        auto d2at = [&](int xx) -> int {
            const uint32_t k = __hip_atomic_load(krow + xx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // untouched entries keep OpenCV's INVALID_DISP_SCALED (compared as a disparity)
            if (k == 0xffffffffu) return INV;
            const int xc = 0xffff - (int)(k & 0xffffu);
            return xc + minX1 - xx;  // best + minD of the winning cost column
        };
        if (0 <= xl && xl < W && 0 <= xh && xh < W) {
            const int a = d2at(xl), b = d2at(xh);
            if (a >= minD && abs(a - dlo) > e.disp12 && b >= minD && abs(b - dhi) > e.disp12)
                orow[x] = (int16_t)INV;
        }
    }
}

// ---------------------------------------------------------------------------
// 5. last direction (R->L) + WTA + uniqueness + sub-pixel + LR check.
// ---------------------------------------------------------------------------
constexpr int kFinalPF = 4;

template <int NP, bool FULL, typename AccT>
__global__ __launch_bounds__(64) void sgbm_final_kernel(const int16_t* __restrict__ C,
                                                       const AccT* __restrict__ A, int H,
                                                       int W, SgbmEff e,
                                                       int16_t* __restrict__ raw)
{
    using AV = AccVec<NP, AccT>;
    typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
    constexpr int PF = kFinalPF;
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
    const bool lane_on = FULL || d0 < D;
    const size_t off = f * frame + ((size_t)y * W1 + (W1 - 1)) * D + (lane_on ? d0 : 0);
    const int16_t* cp = C + off;
    const AccT* sp = A + off;
    bool valid[NP];
    uint32_t lp[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        valid[p] = FULL || d0 + 2 * p < D;
        lp[p] = valid[p] ? 0u : 0x7fff7fffu;
    }
    const uint32_t p1x2 = (uint32_t)(e.P1 & 0xffff) * 0x10001u;
    const uint32_t p2x2 = (uint32_t)(e.P2 & 0xffff) * 0x10001u;
    const bool eight = e.fullDP != 0;
    int minp = 0;
    const int uq = e.uniq;

    Vec<NP> cb[PF];
    uint32_t sb[PF][NP];
#pragma unroll
    for (int j = 0; j < PF; j++) {
        const ptrdiff_t t = min(j, W1 - 1);
        cb[j].load(cp - t * D);
        AV::load(sp - t * D, sb[j]);
    }
    // phase A of one step: recurrence, total cost, WTA reductions (no LDS, no
    // branches); results per step: minS, best, rejected, Sm, Sp (wave-uniform)
    int rMin[PF], rBest[PF], rRej[PF], rSm[PF], rSp[PF];
    auto phaseA = [&](int j) {
        const int dl = (int16_t)(minp + e.P2);
        const uint32_t delta2 = (uint32_t)(dl & 0xffff) * 0x10001u;
        uint32_t c[NP], ln[NP], st[NP];
#pragma unroll
        for (int p = 0; p < NP; p++) c[p] = cb[j].v[p];
        sgm_step<NP>(lp, delta2, p1x2, c, valid, ln);
        minp = wave_min_i32(lane_min<NP>(ln));
        int key = 0x7fffffff;
#pragma unroll
        for (int p = 0; p < NP; p++) {
            // S = min(ndir*(C - P2) + sum of deltas, MAX_COST), saturating u16
            u16x2 cbv = __builtin_bit_cast(u16x2, c[p]) - __builtin_bit_cast(u16x2, p2x2);
            u16x2 x2 = __builtin_elementwise_add_sat(cbv, cbv);
            u16x2 x4 = __builtin_elementwise_add_sat(x2, x2);
            u16x2 t = eight ? __builtin_elementwise_add_sat(x4, x4)
                            : __builtin_elementwise_add_sat(x4, cbv);
            u16x2 acc = __builtin_elementwise_add_sat(
                __builtin_bit_cast(u16x2, sb[j][p]),
                __builtin_bit_cast(u16x2, path_delta(ln[p], c[p], p2x2)));
            u16x2 sv = __builtin_elementwise_min(__builtin_elementwise_add_sat(t, acc),
                                                 (u16x2){32767, 32767});
            st[p] = valid[p] ? __builtin_bit_cast(uint32_t, sv) : 0x7fff7fffu;
            lp[p] = ln[p];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                int d = d0 + 2 * p + h;
                int v = h ? hi16(st[p]) : lo16(st[p]);
                int sub = lane_rule ? (((d & 7) << 12) | (d >> 3)) : d;
                key = min(key, valid[p] ? ((v << 16) | sub) : 0x7fffffff);
            }
        }
        const int K = wave_min_i32(key);
        const int minS = K >> 16;
        const int sub = K & 0xffff;
        int best = lane_rule ? (((sub & 0xfff) << 3) | (sub >> 12)) : sub;
        if (minS >= kMaxCost) best = -1;  // no strict minimum below MAX_COST
        bool rej = false;
#pragma unroll
        for (int p = 0; p < NP; p++) {
#pragma unroll
            for (int h = 0; h < 2; h++) {
                int d = d0 + 2 * p + h;
                int v = h ? hi16(st[p]) : lo16(st[p]);
                rej |= valid[p] && (v * (100 - uq) < minS * 100) && (abs(best - d) > 1);
            }
        }
        auto fetch = [&](int d) -> int {
            d = clampi(d, 0, D - 1);
            int ln_ = d / (2 * NP), el = d - ln_ * 2 * NP;
            uint32_t v = st[0];
#pragma unroll
            for (int p = 1; p < NP; p++) v = ((el >> 1) == p) ? st[p] : v;
            uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)v, ln_);
            return (el & 1) ? hi16(w) : lo16(w);
        };
        rMin[j] = minS;
        rBest[j] = best;
        rRej[j] = __ballot(rej) != 0ull;
        rSm[j] = fetch(best - 1);
        rSp[j] = fetch(best + 1);
    };
    // phase B of one step (x descending, sequential semantics of the scan)
    auto phaseB = [&](int s, int j) {
        if (rRej[j]) return;
        const int x = W1 - 1 - s;
        const int minS = rMin[j], best = rBest[j];
        const int x2 = x + minX1 - best - minD;
        if (lane == 0 && x2 >= 0 && x2 < W && d2c[x2] > minS) {
            d2c[x2] = (int16_t)minS;
            d2[x2] = (int16_t)(best + minD);
        }
        int d16;
        if (0 < best && best < D - 1) {
            const int Sm = rSm[j], Sp = rSp[j];
            const int den = max(Sm + Sp - 2 * minS, 1);
            d16 = best * kDispScale + ((Sm - Sp) * kDispScale + den) / (den * 2);
        } else {
            d16 = best * kDispScale;
        }
        if (lane == 0) disp1[x + minX1] = (int16_t)(d16 + minD * kDispScale);
    };
    int s = 0;
    for (; s + PF <= W1; s += PF) {
#pragma unroll
        for (int j = 0; j < PF; j++) {
            phaseA(j);
            const ptrdiff_t t = min(s + j + PF, W1 - 1);
            cb[j].load(cp - t * D);
            AV::load(sp - t * D, sb[j]);
        }
#pragma unroll
        for (int j = 0; j < PF; j++) phaseB(s + j, j);
    }
    const int rem = W1 - s;
#pragma unroll
    for (int j = 0; j < PF; j++)
        if (j < rem) phaseA(j);
#pragma unroll
    for (int j = 0; j < PF; j++)
        if (j < rem) phaseB(s + j, j);
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

// ---------------------------------------------------------------------------
// 5b. WTA of the split side-by-side form (round 6): the R->L direction ran as
// one more side-by-side chain set, so every pixel's S is a sum of planes --
// S = min(ndir (C - P2) + sum of the ndir deltas, MAX_COST), exact in int32 --
// and the WTA, uniqueness ratio, sub-pixel fit and right-view keys run on a
// thread per pixel with no chain along the row; a row's block then runs the
// left-right check (as sgbm_final16_kernel).  Byte / u16 planes, element order
// d within a pixel.
// ---------------------------------------------------------------------------
constexpr int kWtaThreads = 256;

template <typename AccT>
__device__ __forceinline__ void load8_planes(const AccT* p, uint32_t (&v)[8])
{
    if constexpr (sizeof(AccT) == 2) {
        const uint4 t = *(const uint4*)p;
        const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int i = 0; i < 4; i++) {
            v[2 * i] = w[i] & 0xffffu;
            v[2 * i + 1] = w[i] >> 16;
        }
    } else {
        const uint2 t = *(const uint2*)p;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            v[i] = (t.x >> (8 * i)) & 0xffu;
            v[4 + i] = (t.y >> (8 * i)) & 0xffu;
        }
    }
}

// LPP = D / 8 lanes per pixel, 8 disparities per lane (coalesced 16-byte
// loads of C and of every plane); the lanes of a pixel reduce the key, the
// uniqueness minimum and S(best -+ 1) with lane shuffles, and the pixel's first
// lane finishes it.
template <typename AccT, bool UQ, int LPP>
__global__ __launch_bounds__(kWtaThreads) void sgbm_wta_planes_kernel(const int16_t* __restrict__ C,
                                                                     const AccT* __restrict__ A, size_t plane,
                                                                     int nplanes, int H, int W, SgbmEff e,
                                                                     int16_t* __restrict__ raw,
                                                                     uint32_t* __restrict__ keys)
{
    static_assert(LPP >= 2 && LPP <= 32 && (LPP & (LPP - 1)) == 0, "8 disparities per lane, D = 16 .. 256");
    constexpr int PPB = kWtaThreads / LPP;  // pixels per block iteration
    const int y = blockIdx.x, f = blockIdx.y;
    const int D = 8 * LPP, W1 = e.W1, INV = e.invalid, minD = e.minD, minX1 = e.minX1;
    int16_t* orow = raw + ((size_t)f * H + y) * W;
    uint32_t* krow = keys + ((size_t)f * H + y) * W;
    for (int x = threadIdx.x; x < W; x += kWtaThreads) {
        orow[x] = (int16_t)INV;
        krow[x] = 0xffffffffu;
    }
    __threadfence_block();
    __syncthreads();
    const bool lane_rule = !e.fullDP && !(e.variant & MVSV_VARIANT_WTA_MIN_D);
    const int ndir = e.fullDP ? 8 : 5;
    const size_t row0 = ((size_t)f * H + y) * W1;
    const int sl = threadIdx.x % LPP, gbase = (int)(threadIdx.x & 63) - sl;  // lane in the pixel, its first lane
    const int d0 = 8 * sl;
    for (int xb = 0; xb < W1; xb += PPB) {
        const int xr = xb + (int)threadIdx.x / LPP;
        const int x = min(xr, W1 - 1);
        const size_t off = (row0 + x) * D + d0;
        int S[8];
        {
            const uint4 cw = *(const uint4*)(C + off);
            const uint32_t cv[4] = {cw.x, cw.y, cw.z, cw.w};
            int acc[8];
#pragma unroll
            for (int i = 0; i < 4; i++) {
                acc[2 * i] = ndir * ((int)(cv[i] & 0xffffu) - e.P2);
                acc[2 * i + 1] = ndir * ((int)(cv[i] >> 16) - e.P2);
            }
            for (int k = 0; k < nplanes; k++) {
                uint32_t dv[8];
                load8_planes<AccT>(A + (size_t)k * plane + off, dv);
#pragma unroll
                for (int i = 0; i < 8; i++) acc[i] += (int)dv[i];
            }
#pragma unroll
            for (int i = 0; i < 8; i++) S[i] = min(acc[i], kMaxCost);
        }
        // argmin, ties in OpenCV's order (d, or MODE_SGBM's SIMD lane d mod 8 first)
        uint32_t key = 0xffffffffu;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const int d = d0 + i;
            const uint32_t sub = lane_rule ? (uint32_t)((i << 12) | (d >> 3)) : (uint32_t)d;
            key = min(key, ((uint32_t)S[i] << 16) | sub);
        }
#pragma unroll
        for (int m = 1; m < LPP; m <<= 1) key = min(key, (uint32_t)__shfl_xor((int)key, m, 64));
        const int minS = (int)(key >> 16), sub = (int)(key & 0xffffu);
        const int best = lane_rule ? (((sub & 0xfff) << 3) | (sub >> 12)) : sub;
        const int bm = max(best - 1, 0), bp = min(best + 1, D - 1);
        auto elem = [&](int d) -> int {  // S[d & 7] of this lane
            int v = S[0];
#pragma unroll
            for (int i = 1; i < 8; i++) v = (d & 7) == i ? S[i] : v;
            return v;
        };
        const int Sm = __shfl(elem(bm), gbase + (bm >> 3), 64);
        const int Sp = __shfl(elem(bp), gbase + (bp >> 3), 64);
        bool rej = false;
        if constexpr (UQ) {
            int m2 = 0x7fffffff;
#pragma unroll
            for (int i = 0; i < 8; i++) {
                const int d = d0 + i;
                if (d < best - 1 || d > best + 1) m2 = min(m2, S[i]);
            }
#pragma unroll
            for (int m = 1; m < LPP; m <<= 1) m2 = min(m2, __shfl_xor(m2, m, 64));
            rej = m2 != 0x7fffffff && m2 * (100 - e.uniq) < minS * 100;
        }
        if (sl == 0 && xr < W1) {
            const int bst = minS >= kMaxCost ? -1 : best;  // no strict minimum below MAX_COST
            const int den = max(Sm + Sp - 2 * minS, 1);
            const int frac = ((Sm - Sp) * kDispScale + den) / (den * 2);
            const int d16 = bst * kDispScale + (frac & -(int)(0 < bst && bst < D - 1));
            orow[x + minX1] = rej ? (int16_t)INV : (int16_t)(d16 + minD * kDispScale);
            const int x2 = x + minX1 - bst - minD;
            if (!rej && minS < kMaxCost && x2 >= 0 && x2 < W)
                atomicMin(krow + x2, ((uint32_t)minS << 16) | (uint32_t)(0xffff - x));
        }
    }
    __threadfence_block();
    __syncthreads();
    // left-right check (src: OpenCV 3.4 final loop) -- reads the finished row
    for (int x = minX1 + threadIdx.x; x < e.maxX1; x += kWtaThreads) {
        const int v = orow[x];
        if (v == INV) continue;
        const int dlo = v >> kDispShift, dhi = (v + kDispScale - 1) >> kDispShift;
        const int xl = x - dlo, xh = x - dhi;
        auto d2at = [&](int xx) -> int {
            const uint32_t k = __hip_atomic_load(krow + xx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (k == 0xffffffffu) return INV;  // untouched: OpenCV's INVALID_DISP_SCALED
            return 0xffff - (int)(k & 0xffffu) + minX1 - xx;
        };
        if (0 <= xl && xl < W && 0 <= xh && xh < W) {
            const int a = d2at(xl), b = d2at(xh);
            if (a >= minD && abs(a - dlo) > e.disp12 && b >= minD && abs(b - dhi) > e.disp12)
                orow[x] = (int16_t)INV;
        }
    }
}

__global__ void fill_s16_kernel(int16_t* __restrict__ out, size_t os, size_t ofs, int W, int H,
                                int16_t v)
{
    const int y = blockIdx.x, f = blockIdx.y;
    int16_t* o = out + f * ofs + (size_t)y * os;
    for (int x = threadIdx.x; x < W; x += blockDim.x) o[x] = v;
}

// sheared-strip schedule: enabled, and int32 element offsets cover a frame
template <int NP, int NACC, typename AccT, bool NW = false, bool RES = false, int LPC = 16>
void launch_final16(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, const int16_t* Cv,
                    const AccT* Av, size_t plane, int16_t* raw, const void* Rv = nullptr,
                    const uint16_t* Mv = nullptr)
{
    // NP: disparity pairs per lane at LPC lanes per row (LPC = 8: D = 16, eight
    // rows per wave).  D >= 128: 32 lanes per row (half the pairs per lane,
    // twice the rows in flight per SIMD); a lane keeps >= 2 pairs, so it reads
    // whole 4-disparity nibble groups.
    constexpr int LPR = LPC == 8 ? 8 : (NP >= 4 ? MVSV_FINAL_LPR : 16);
    constexpr int NPL = LPC == 8 ? NP : NP * 16 / LPR;
    constexpr int RPW = 64 / LPR;
    const dim3 grid((H + RPW - 1) / RPW, n);
    uint32_t* keys = (uint32_t*)ctx->keys.ptr;
    int16_t* dummy = (int16_t*)ctx->dummy.ptr;
    if constexpr (RES) {
        // residual plane: WTA on R, exact costs gathered for the sub-pixel fit
        // (uniquenessRatio 0 only: a ratio test needs every exact cost)
        if (e.uniq == 0) {
            hipLaunchKernelGGL((sgbm_final16_kernel<NPL, NACC, AccT, false, LPR, NW, true>), grid, dim3(64), 0,
                               ctx->stream, Cv, Av, plane, H, W, e, raw, keys, dummy, (const uint8_t*)Rv, Mv);
            return;
        }
    }
    if (e.uniq > 0)
        hipLaunchKernelGGL((sgbm_final16_kernel<NPL, NACC, AccT, true, LPR, NW>), grid, dim3(64), 0,
                           ctx->stream, Cv, Av, plane, H, W, e, raw, keys, dummy, nullptr, nullptr);
    else
        hipLaunchKernelGGL((sgbm_final16_kernel<NPL, NACC, AccT, false, LPR, NW>), grid, dim3(64), 0,
                           ctx->stream, Cv, Av, plane, H, W, e, raw, keys, dummy, nullptr, nullptr);
}

// Every cost C = P2 + (box sum of blockSize^2 BT costs, each <= 2*ftzero + 63),
// every L <= C and delta = minLp + P2: when that bound stays <= 32767 nothing
// wraps in int16 and the path kernels may use the NW recurrence (sgm_pair).
// The split side-by-side form (sgbm_wta_planes_kernel): byte / u16 planes,
// D <= 32.  Measured (MI355X r06 sp2, split vs fused R->L + WTA): D 16 640x480
// x 1 / 2 / 8 frames 0.278 -> 0.196, 0.297 -> 0.220, 0.515 -> 0.477 ms; D 32
// 1280x960 0.522 -> 0.491; D 64 x 1 / 2 0.746 -> 0.802, 1.125 -> 1.282 and D 128
// 1.083 -> 1.370 (the fifth chain set lengthens the direction pass more than
// the chain-free WTA saves); MODE_HH D 64 1.01 either way
static bool wta_split(const mvsv_ctx* ctx, const SgbmEff& e)
{
    return ctx->final_split && e.P2 > 15 && e.D <= 32;
}

static bool sgbm_no_wrap(const SgbmEff& e)
{
    const long bs = 2L * e.SW2 + 1;
    return (long)e.P2 + bs * bs * (2L * e.ftzero + 63) + e.P2 <= 32767;
}

// The direction passes read the residual plane (see its definition above)
// when it is exact and smaller: no-wrap regime, residuals <= 3 * P2 in a
// nibble, a 16-lane path schedule (1 = strips + lines, 2 = side by side) and
// D <= 128 (one cost kernel wave segment holds a pixel's D costs).
static bool use_residual(const mvsv_ctx* ctx, const SgbmEff& e, int sched)
{
    return ctx->cost_res && (sched == 1 || sched == 2) && sgbm_no_wrap(e) && 3 * e.P2 <= 15 &&
           (e.D == 32 || e.D == 64 || e.D == 128);
}

static bool use_strips(const mvsv_ctx* ctx, const SgbmEff& e, int H)
{
    return ctx->tri && (size_t)H * e.W1 * e.D < ((size_t)1 << 31);
}

// Path schedule of the 16-lane kernels (D = 32 / 64 / 128 / 256):
// 2 = all line directions side by side (sgbm_pathdirs16_kernel, one 4-bit plane
// per direction, P2 <= 15) -- the latency shape for launches too small to fill
// the chip with strips (one camera frame); 1 = sheared strips (batches).
// ctx->path_sched: 0 = by launch size, 1 / 2 force (tests, A/B).
static int path_schedule(const mvsv_ctx* ctx, const SgbmEff& e, int H, int n)
{
    if (e.D == 16 && ctx->path16 && ctx->path_sched != 1) return 2;  // launch_paths_d16
    if (!ctx->path16 || !(e.D == 32 || e.D == 64 || e.D == 128 || e.D == 256)) return 0;
    const bool dirs_ok = e.P2 <= 15 || ctx->path_sched == 2;  // nibble planes; wider planes when forced
    if (ctx->path_sched == 2) return 2;
    if (ctx->path_sched == 0 && bsgm_eligible(ctx, e, n, H) && e.SH2 <= 7 && e.SW2 == e.SH2) {
        // bit-sliced regime (round 6): the side-by-side chains' work grows with
        // the direction-pixels, the strips' time with the chain length; measured
        // (8 frames, MI355X r06e): 640x480 5 paths 0.90 side vs 1.11 ms strips,
        // 8 paths 1.10 vs 1.06; 1280x960 5 paths 3.49 vs 3.07, 8 paths 4.53 vs
        // 3.20; one 1280x960 frame, 8 paths 0.73 vs 1.03 (round 5)
        const long long dirpix = (long long)n * e.W1 * H * (e.fullDP ? 8 : 5);
        if (dirpix <= 12000000LL) return 2;
        return use_strips(ctx, e, H) ? 1 : 0;
    }
    if (ctx->path_sched == 0 && dirs_ok) {
        const int wide = e.D > 128 ? 7 : 15;
        const long long blocks = (long long)(e.fullDP ? 2 : 1) * n * ((e.W1 + H - 1 + 4 * wide - 1) / (4 * wide));
        // measured: one 640x480 or 1280x960 frame and two 640x480 frames gain
        // (0.76 -> 0.43, 1.62 -> 1.11, 0.83 -> 0.60 ms); two 1280x960 frames
        // lose (1.87 -> 1.95 ms: seven planes into the final kernel)
        if (2 * blocks <= ctx->cus) return 2;
    }
    if (ctx->path_sched == 0 && e.P2 > 15) {
        // byte / u16 planes (liveDisparity's create(0, 64, 9, 648, 2592)): side by
        // side while the planes stay small -- their bytes against the strip
        // chain's latency.  Measured (1280x960, MI355X r06 s2a / d16a): MODE_SGBM
        // D 32 x 1-3 frames 0.91 -> 0.53, 1.20 -> 1.07 ms; D 64 x 1, 2 frames
        // 1.16 -> 0.71, 1.34 -> 1.12 ms, x 4 1.98 -> 2.14 (strips kept); D 128 x 1
        // 1.50 -> 1.08, x 2 1.86 -> 1.90; D 256 x 1 2.08 -> 2.16; MODE_HH D 64 x 1
        // 1.18 -> 0.90, x 2 1.52 -> 1.59
        const double bytes = (double)n * e.W1 * H * e.D * (e.fullDP ? 7 : 4) * (acc_is_u8(e) ? 1 : 2);
        if (bytes <= 1.4e9) return 2;
    }
    return use_strips(ctx, e, H) ? 1 : 0;
}

template <int NP, int WV, int LPC, typename AccT, bool NW, bool RES>
int launch_tri_wv(mvsv_ctx* ctx, int n, int H, const SgbmEff& e, const void* Cv, AccT* Av, size_t plane,
                  int npass)
{
    using TL = TriLayout<NP, WV, LPC>;
    constexpr int kTriSW = TriCfg<NP, WV, LPC>::kSW;
    const int nstrips = (e.W1 + H - 1 + kTriSW - 1) / kTriSW;
    const size_t bytes = (size_t)npass * n * nstrips * H * 4 * LPC * TriGran<NP>::NG * 8;
    int rc;
    if (ctx->tri_bnd.bytes < bytes) {
        if ((rc = ensure(ctx, ctx->tri_bnd, bytes, "sgbm strip boundary granules"))) return rc;
        // fresh granules carry tag 0, which no launch uses
        if ((rc = check_hip(ctx, hipMemsetAsync(ctx->tri_bnd.ptr, 0, ctx->tri_bnd.bytes, ctx->stream),
                            "sgbm boundary reset")))
            return rc;
    }
    if (!ctx->status.ptr) {
        // [0] give-up epoch, [2] strip tickets drawn
        if ((rc = ensure(ctx, ctx->status, 16, "device status words"))) return rc;
        if ((rc = check_hip(ctx, hipMemsetAsync(ctx->status.ptr, 0, 16, ctx->stream), "status reset")))
            return rc;
        ctx->tri_tickets = 0;
    }
    // Launch epochs never repeat between two zeroings of the granules: tag 0
    // means "never written", and when the 16-bit tag wraps every slot is
    // zeroed again, so a slot carrying this launch's tag was written by it.
    if ((++ctx->tri_epoch & 0xffffu) == 0) {
        ++ctx->tri_epoch;
        if ((rc = check_hip(ctx, hipMemsetAsync(ctx->tri_bnd.ptr, 0, ctx->tri_bnd.bytes, ctx->stream),
                            "sgbm boundary reset")))
            return rc;
    }
    const unsigned epoch = ctx->tri_epoch;
    dim3 grid(nstrips * npass * n);
    unsigned long long* stats = nullptr;
    // MVSV_TRI_STATS: per-strip summary on stderr; MVSV_TRI_TRACE=path: also
    // every step's publish / consume time (100 MHz) of every strip, to a file
    const char* trace_path = std::getenv("MVSV_TRI_TRACE");
    const bool want_stats = std::getenv("MVSV_TRI_STATS") != nullptr || trace_path;
    const int trace_h = trace_path ? H : 0;
    const size_t sb = 8 + 2 * (size_t)trace_h;  // u64 per block
    if (want_stats) {
        (void)hipMalloc(&stats, (size_t)grid.x * sb * 8);
        (void)hipMemset(stats, 0, (size_t)grid.x * sb * 8);
    }
    // Strip tickets for every launch (round 4): a launch of at most one block
    // per CU is not resident all at once when other work shares the GPU
    // (stream lanes, batches in flight), so blockIdx order would rest on
    // in-order dispatch; tickets never do.  MVSV_OPT_STRIP_TICKETS = 0 keeps
    // blockIdx order for A/B runs.
    const bool tickets = ctx->strip_tickets != 0;
    if (TL::kBytes > 65536 &&
        (rc = check_hip(ctx, hipFuncSetAttribute((const void*)sgbm_tri_kernel<NP, WV, LPC, AccT, NW, RES>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)TL::kBytes),
                        "sgbm strip LDS attribute")))
        return rc;
    hipLaunchKernelGGL((sgbm_tri_kernel<NP, WV, LPC, AccT, NW, RES>), grid, dim3(TriCfg<NP, WV, LPC>::kThreads), TL::kBytes,
                       ctx->stream, Cv, Av, plane, (AccT*)ctx->dummy.ptr, H, e.W1, e.D, npass, e.P1,
                       e.P2, (unsigned long long*)ctx->tri_bnd.ptr, epoch, n, nstrips,
                       (int*)ctx->status.ptr, ctx->spin_limit, ctx->report_target, stats, trace_h,
                       tickets ? (long long)ctx->tri_tickets : -1ll);
    rc = check_hip(ctx, hipGetLastError(), "sgbm sheared-strip path kernel");
    if (rc == MVSV_OK && tickets) ctx->tri_tickets += grid.x;  // one ticket per block (u32 wrap is harmless)
    if (want_stats) {
        (void)hipStreamSynchronize(ctx->stream);
        std::vector<unsigned long long> h((size_t)grid.x * sb);
        (void)hipMemcpy(h.data(), stats, h.size() * 8, hipMemcpyDeviceToHost);
        (void)hipFree(stats);
        if (trace_path) {
            if (FILE* fp = std::fopen(trace_path, "wb")) {
                const unsigned long long hdr[8] = {grid.x, sb, (unsigned long long)H, (unsigned long long)nstrips,
                                                   (unsigned long long)npass, (unsigned long long)n,
                                                   (unsigned long long)kTriSW, (unsigned long long)e.W1};
                std::fwrite(hdr, 8, 8, fp);
                std::fwrite(h.data(), 8, h.size(), fp);
                std::fclose(fp);
            }
        }
        unsigned long long t0 = ~0ull, t1 = 0, spin = 0, busy = 0, steps = 0, longest = 0, lst = 0;
        for (size_t b = 0; b < grid.x; b++) {
            const unsigned long long* q = &h[b * sb];
            if (!q[1]) continue;
            t0 = std::min(t0, q[0]);
            t1 = std::max(t1, q[1]);
            spin += q[2];
            busy += q[1] - q[0];
            steps += q[4];
            if (q[4] > longest) { longest = q[4]; lst = q[1] - q[0]; }
        }
        std::fprintf(stderr, "[tri] span %llu ticks, blocks %u, block-ticks %llu, spin-ticks %llu (%.1f%%), "
                     "ticks/step %.1f, longest strip %llu steps in %llu ticks\n",
                     t1 - t0, grid.x, busy, spin, 100.0 * spin / std::max(busy, 1ull),
                     (double)busy / std::max(steps, 1ull), longest, lst);
        for (size_t b = 0; b < grid.x; b += grid.x / 24 + 1) {
            const unsigned long long* q = &h[b * sb];
            std::fprintf(stderr, "[tri]  blk %zu k %llu pass %llu tb %llu len %llu start %llu dur %llu spin %llu n %llu\n",
                         b, q[5], q[6], q[7], q[4], q[0] - t0, q[1] - q[0], q[2], q[3]);
        }
    }
    return rc;
}

// Strip width: wide strips while the launch has at least one block per CU
// (frame batches: the kernel is VALU-bound and wide strips share the step
// barrier and the exchange wave among 15 compute waves); narrow strips when it
// would not (one 640x480 frame: 34 wide blocks on 256 CUs, each strip step the
// serial VALU work of 15 waves on one CU) -- the chain of strips then spreads
// over more CUs at about half the per-step work (640x480, one frame: strips
// 0.62 -> 0.41 ms; 4 waves per strip: 0.42 ms, its longer chain of strips
// eats the shorter steps).  MVSV_OPT_STRIP_WAVES forces either shape.
// (Round 3's 8-lanes-per-column variant, LPC = 8, measured slower and is no
// longer instantiated; the kernel keeps the LPC parameter.)
template <int NP, int LPC, typename AccT, bool NW, bool RES>
int launch_tri_lpc(mvsv_ctx* ctx, int n, int H, const SgbmEff& e, const void* Cv, AccT* Av, size_t plane,
                   int npass)
{
    constexpr int wide = tri_wide_waves<NP, LPC>(), narrow = tri_narrow_waves<NP, LPC>();
    constexpr int cpw = 64 / LPC;
    int wv = ctx->strip_waves;
    if (wv != wide && wv != narrow) {
        const long long blocks = (long long)npass * n * ((e.W1 + H - 1 + cpw * wide - 1) / (cpw * wide));
        wv = blocks < ctx->cus ? narrow : wide;
    }
    if (wv == narrow) return launch_tri_wv<NP, narrow, LPC, AccT, NW, RES>(ctx, n, H, e, Cv, Av, plane, npass);
    return launch_tri_wv<NP, wide, LPC, AccT, NW, RES>(ctx, n, H, e, Cv, Av, plane, npass);
}

template <int NP, typename AccT, bool NW, bool RES>
int launch_tri(mvsv_ctx* ctx, int n, int H, const SgbmEff& e, const void* Cv, AccT* Av, size_t plane,
               int npass)
{
    if constexpr (NP == 8 && !RES) {
        // D = 256 launches that would run narrow strips (one or two frames):
        // 32 lanes per column (MVSV_TRI32 = 0: the 16-lane narrow strips)
        constexpr int wide = tri_wide_waves<NP, 16>();
        const long long blocks = (long long)npass * n * ((e.W1 + H - 1 + 4 * wide - 1) / (4 * wide));
        if (ctx->tri32 && ctx->strip_waves == 0 && blocks < ctx->cus)
            return launch_tri_wv<NP / 2, tri_narrow_waves<NP / 2, 32>(), 32, AccT, NW, RES>(ctx, n, H, e, Cv, Av,
                                                                                           plane, npass);
    }
    return launch_tri_lpc<NP, 16, AccT, NW, RES>(ctx, n, H, e, Cv, Av, plane, npass);
}

// Sheared-strip schedule: the down pass ((1,1) (0,1) (-1,1)), the up pass
// ((1,-1) (0,-1) (-1,-1), MODE_HH) and the L->R lines each write their own
// accumulator plane; the L->R lines run on a second stream beside the strip
// kernel, and the final kernel (R->L + WTA) sums the planes.  The direction
// passes read Cin -- the cost volume, or (RES) its residual plane -- and the
// final kernel the cost volume Cv.
template <int NP, typename AccT, bool NW, bool RES = false>
int launch_paths_tri(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, int16_t* Cv, const void* Cin,
                     AccT* Av, size_t plane, int16_t* raw, const uint16_t* Mv = nullptr)
{
    hipStream_t s = ctx->stream;
    int rc;
    if (!ctx->aux) {
        if ((rc = check_hip(ctx, hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking), "aux stream")) ||
            (rc = check_hip(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming), "event")) ||
            (rc = check_hip(ctx, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming), "event")))
            return rc;
    }
    const int npass = e.fullDP ? 2 : 1;
    AccT* dummy = (AccT*)ctx->dummy.ptr;
    {
        StageTimer tm(ctx, kStagePath);
        if ((rc = check_hip(ctx, hipEventRecord(ctx->ev_fork, s), "fork")) ||
            (rc = check_hip(ctx, hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0), "fork wait")))
            return rc;
        // lines_aux < 0 (default): beside the strips when the launch is small
        // (the strips then occupy a fraction of the CUs -- one frame: ~60 of
        // 256 -- and the L->R lines fill idle ones); after them for batches,
        // where both kernels saturate the GPU and running them together was
        // measured slower
        // Round 4: with the residual input the line kernel needs 53 VGPRs and
        // the wide strip kernel 103, so a line wave fits beside a strip block
        // on every SIMD -- launched after the strips on the second stream, the
        // lines fill the strips' step-barrier and hand-off waits (one batch of
        // 8 frames: 4.49 -> 4.37-4.40 ms, MI355X r04d A/B)
        // Round 6: "small" counts the strip blocks the launch will really have
        // (launch_tri_lpc picks narrow strips -- 1.7x the blocks -- whenever the
        // wide ones would not fill the CUs): beside the strips only while those
        // occupy at most 60 % of the CUs (one 1280x960 frame: 125 narrow D = 256
        // blocks, 132 narrow D = 128 MODE_HH blocks).  Two config-5 frames (D 256,
        // 248 narrow blocks) had the lines beside them at 2.68 ms instead of
        // 0.66 for one frame (r04g c5_frame.jsonl): every CU held a strip.
        int aux_mode = ctx->lines_aux;
        if (aux_mode < 0) {
            constexpr int wide = tri_wide_waves<NP>(), narrow = tri_narrow_waves<NP>();
            auto nblocks = [&](int wv) {
                return (long long)npass * n * ((e.W1 + H - 1 + 4 * wv - 1) / (4 * wv));
            };
            const int wv = ctx->strip_waves == wide || ctx->strip_waves == narrow
                               ? ctx->strip_waves
                               : (nblocks(wide) < ctx->cus ? narrow : wide);
            // Round 6: byte / u16 planes at D <= 64 run the lines beside the
            // strips in batches too (liveDisparity default, 1280x960 x 4 / x 8:
            // 1.97 -> 1.87, 3.13 -> 2.88 ms); D = 256 keeps them after the
            // strips (x 4: 4.90 -> 5.7 ms beside, x 8: 8.60 -> 8.50;
            // profiles/r06/aux/lines_aux_ab.txt)
            aux_mode = 5 * nblocks(wv) <= 3 * ctx->cus ? 1 : ((RES || NP <= 2) ? 2 : 0);
        }
        hipStream_t ls = aux_mode ? ctx->aux : s;
        auto lines = [&]() {
            StageTimer tl(ctx, kStageLines, ls);
            dim3 grid((num_lines(1, 0, e.W1, H) + 15) / 16, n);
            hipLaunchKernelGGL((sgbm_path16_kernel<NP, true, AccT, NW, RES>), grid, dim3(256), 0, ls, Cin,
                               acc_add(Av, (ptrdiff_t)npass * (ptrdiff_t)plane), dummy, H, e.W1,
                               e.D, 1, 0, e.P1, e.P2);
        };
        // lines_aux: 0 = after the strip kernel on the same stream, 1 = on the
        // second stream launched before it, 2 = on the second stream after it
        if (aux_mode == 1) lines();
        if ((rc = check_hip(ctx, hipGetLastError(), "sgbm L->R lines"))) return rc;
        {
            StageTimer ts(ctx, kStageStrips);
            if ((rc = launch_tri<NP, AccT, NW, RES>(ctx, n, H, e, Cin, Av, plane, npass))) return rc;
        }
        if (aux_mode != 1) lines();
        if ((rc = check_hip(ctx, hipEventRecord(ctx->ev_join, ctx->aux), "join")) ||
            (rc = check_hip(ctx, hipStreamWaitEvent(s, ctx->ev_join, 0), "join wait")))
            return rc;
    }
    StageTimer tm(ctx, kStageFinal);
    if (npass == 2)
        launch_final16<NP, 3, AccT, NW, RES>(ctx, n, H, W, e, Cv, Av, plane, raw, Cin, Mv);
    else
        launch_final16<NP, 2, AccT, NW, RES>(ctx, n, H, W, e, Cv, Av, plane, raw, Cin, Mv);
    return check_hip(ctx, hipGetLastError(), "sgbm path kernels (sheared strips)");
}

template <int NP, typename AccT>
int launch_paths16(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, int16_t* Cv, AccT* Av,
                   int16_t* raw)
{
    hipStream_t s = ctx->stream;
    static const int dirs_sgbm[4][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}};
    static const int dirs_hh[7][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {1, -1}, {0, -1}, {-1, -1}};
    int rc;
    if ((rc = ensure(ctx, ctx->dummy, 512 * 16 * 2 * NP, "sgbm dummy slots"))) return rc;
    if ((rc = ensure(ctx, ctx->keys, (size_t)n * H * W * 4, "sgbm right-view keys"))) return rc;
    AccT* dummy = (AccT*)ctx->dummy.ptr;
    const size_t plane = (size_t)n * H * e.W1 * e.D;
    // u8 / u16 planes (P2 > 5) at D = 256 (liveDisparity, config 5): the
    // no-wrap recurrence wherever no int16 can wrap -- its adds / subtracts
    // run at the full 32-bit rate, so it is the cheaper form here too (one
    // frame 2.04 -> 1.99 ms, profiles/r04/c5ab04); other D keep the general
    // form (compile time)
    if (use_strips(ctx, e, H)) {
        if constexpr (NP == 8)
            if (sgbm_no_wrap(e)) return launch_paths_tri<NP, AccT, true>(ctx, n, H, W, e, Cv, Cv, Av, plane, raw);
        return launch_paths_tri<NP, AccT, false>(ctx, n, H, W, e, Cv, Cv, Av, plane, raw);
    }
    const int ndir = e.fullDP ? 7 : 4;
    for (int k = 0; k < ndir; k++) {
        int dx = e.fullDP ? dirs_hh[k][0] : dirs_sgbm[k][0];
        int dy = e.fullDP ? dirs_hh[k][1] : dirs_sgbm[k][1];
        int nl = num_lines(dx, dy, e.W1, H);
        dim3 grid((nl + 15) / 16, n);
        StageTimer tm(ctx, kStagePath);
        if (k == 0)
            hipLaunchKernelGGL((sgbm_path16_kernel<NP, true, AccT>), grid, dim3(256), 0, s, Cv, Av,
                               dummy, H, e.W1, e.D, dx, dy, e.P1, e.P2);
        else
            hipLaunchKernelGGL((sgbm_path16_kernel<NP, false, AccT>), grid, dim3(256), 0, s, Cv,
                               Av, dummy, H, e.W1, e.D, dx, dy, e.P1, e.P2);
    }
    StageTimer tm(ctx, kStageFinal);
    launch_final16<NP, 1, AccT>(ctx, n, H, W, e, Cv, Av, plane, raw);
    return check_hip(ctx, hipGetLastError(), "sgbm path kernels (16-lane)");
}

template <int NP, typename AccT>
int launch_paths(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, int16_t* Cv, AccT* Av,
                 int16_t* raw)
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
        StageTimer tm(ctx, kStagePath);
        const bool full = e.D == 128 * NP;
        if (k == 0 && full)
            hipLaunchKernelGGL((sgbm_path_kernel<NP, true, true, AccT>), grid, dim3(256), 0, s,
                               Cv, Av, H, e.W1, e.D, dx, dy, e.P1, e.P2);
        else if (k == 0)
            hipLaunchKernelGGL((sgbm_path_kernel<NP, true, false, AccT>), grid, dim3(256), 0, s,
                               Cv, Av, H, e.W1, e.D, dx, dy, e.P1, e.P2);
        else if (full)
            hipLaunchKernelGGL((sgbm_path_kernel<NP, false, true, AccT>), grid, dim3(256), 0, s,
                               Cv, Av, H, e.W1, e.D, dx, dy, e.P1, e.P2);
        else
            hipLaunchKernelGGL((sgbm_path_kernel<NP, false, false, AccT>), grid, dim3(256), 0, s,
                               Cv, Av, H, e.W1, e.D, dx, dy, e.P1, e.P2);
    }
    size_t lds = (size_t)W * 3 * sizeof(int16_t);
    StageTimer tm(ctx, kStageFinal);
    if (e.D == 128 * NP)
        hipLaunchKernelGGL((sgbm_final_kernel<NP, true, AccT>), dim3(H, n), dim3(64), lds, s, Cv,
                           Av, H, W, e, raw);
    else
        hipLaunchKernelGGL((sgbm_final_kernel<NP, false, AccT>), dim3(H, n), dim3(64), lds, s, Cv,
                           Av, H, W, e, raw);
    return check_hip(ctx, hipGetLastError(), "sgbm path kernels");
}

template <int NP, typename AccT, bool NW, bool RES = false, int LPC = 16>
int launch_paths_dirs(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, int16_t* Cv, const void* Cin,
                      AccT* Av, int16_t* raw, const uint16_t* Mv = nullptr)
{
    static const int dirs_sgbm[4][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}};
    static const int dirs_hh[7][2] = {{1, 0}, {1, 1}, {0, 1}, {-1, 1}, {1, -1}, {0, -1}, {-1, -1}};
    // split form: the R->L direction as one more chain set, the WTA on its own
    constexpr bool kPlainPlanes = std::is_same<AccT, uint16_t>::value || std::is_same<AccT, uint8_t>::value;
    const bool split = !RES && kPlainPlanes && wta_split(ctx, e);
    const int ndir = (e.fullDP ? 7 : 4) + (split ? 1 : 0);
    PathDirs pd{};
    int maxnl = 0;
    for (int k = 0; k < ndir; k++) {
        const bool rl = split && k == ndir - 1;
        pd.dx[k] = rl ? -1 : e.fullDP ? dirs_hh[k][0] : dirs_sgbm[k][0];
        pd.dy[k] = rl ? 0 : e.fullDP ? dirs_hh[k][1] : dirs_sgbm[k][1];
        maxnl = std::max(maxnl, num_lines(pd.dx[k], pd.dy[k], e.W1, H));
    }
    const size_t plane = (size_t)n * H * e.W1 * e.D;
    {
        StageTimer tm(ctx, kStagePath);
        constexpr int lpb = path16_lines_per_block<LPC>();
        hipLaunchKernelGGL((sgbm_pathdirs16_kernel<NP, AccT, NW, RES, LPC>), dim3((maxnl + lpb - 1) / lpb, n, ndir),
                           dim3(256), 0, ctx->stream, Cin, Av, plane, (AccT*)ctx->dummy.ptr, H, e.W1, e.D, pd,
                           e.P1, e.P2);
    }
    StageTimer tm(ctx, kStageFinal);
    if constexpr (kPlainPlanes) {
        if (split) {
            constexpr int LPP = 2 * NP * LPC / 8;  // D / 8
            if (e.uniq > 0)
                hipLaunchKernelGGL((sgbm_wta_planes_kernel<AccT, true, LPP>), dim3(H, n), dim3(kWtaThreads), 0,
                                   ctx->stream, Cv, Av, plane, ndir, H, W, e, raw, (uint32_t*)ctx->keys.ptr);
            else
                hipLaunchKernelGGL((sgbm_wta_planes_kernel<AccT, false, LPP>), dim3(H, n), dim3(kWtaThreads), 0,
                                   ctx->stream, Cv, Av, plane, ndir, H, W, e, raw, (uint32_t*)ctx->keys.ptr);
            return check_hip(ctx, hipGetLastError(), "sgbm path kernels (directions side by side, split WTA)");
        }
    }
    if (ndir == 7)
        launch_final16<NP, 7, AccT, NW, RES, LPC>(ctx, n, H, W, e, Cv, Av, plane, raw, Cin, Mv);
    else
        launch_final16<NP, 4, AccT, NW, RES, LPC>(ctx, n, H, W, e, Cv, Av, plane, raw, Cin, Mv);
    return check_hip(ctx, hipGetLastError(), "sgbm path kernels (directions side by side)");
}

// Rv: the residual plane written by the cost kernel (nullptr: none; only ever
// set in the no-wrap regime with 3 * P2 <= 15, use_residual)
template <int NP>
int launch_paths16_acc(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, int16_t* Cv,
                       const uint8_t* Rv, const uint16_t* Mv, void* Av, int16_t* raw)
{
    if (path_schedule(ctx, e, H, n) == 2) {
        int rc;
        if ((rc = ensure(ctx, ctx->dummy, 512 * 16 * 2 * NP, "sgbm dummy slots"))) return rc;
        if ((rc = ensure(ctx, ctx->keys, (size_t)n * H * W * 4, "sgbm right-view keys"))) return rc;
        // one plane per direction: a delta <= P2 in a nibble (4 or 7 of them <= 105
    // per byte lane), a byte (when all directions' sum fits) or a u16
        if (e.P2 <= 15) {
            if (sgbm_no_wrap(e)) {
                if constexpr (NP <= 4)
                    if (Rv) return launch_paths_dirs<NP, nib2_t, true, true>(ctx, n, H, W, e, Cv, Rv, (nib2_t*)Av, raw, Mv);
                return launch_paths_dirs<NP, nib2_t, true>(ctx, n, H, W, e, Cv, Cv, (nib2_t*)Av, raw);
            }
            return launch_paths_dirs<NP, nib2_t, false>(ctx, n, H, W, e, Cv, Cv, (nib2_t*)Av, raw);
        }
        // the final kernel sums the planes in the plane's element type
        if (acc_is_u8(e)) return launch_paths_dirs<NP, uint8_t, false>(ctx, n, H, W, e, Cv, Cv, (uint8_t*)Av, raw);
        return launch_paths_dirs<NP, uint16_t, false>(ctx, n, H, W, e, Cv, Cv, (uint16_t*)Av, raw);
    }
    if (use_strips(ctx, e, H) && acc_is_nib(e)) {
        int rc;
        if ((rc = ensure(ctx, ctx->dummy, 512 * 16 * 2 * NP, "sgbm dummy slots"))) return rc;
        if ((rc = ensure(ctx, ctx->keys, (size_t)n * H * W * 4, "sgbm right-view keys"))) return rc;
        const size_t plane = (size_t)n * H * e.W1 * e.D;
        if (sgbm_no_wrap(e)) {
            if constexpr (NP <= 4)
                if (Rv) return launch_paths_tri<NP, nib2_t, true, true>(ctx, n, H, W, e, Cv, Rv, (nib2_t*)Av, plane, raw, Mv);
            return launch_paths_tri<NP, nib2_t, true>(ctx, n, H, W, e, Cv, Cv, (nib2_t*)Av, plane, raw);
        }
        return launch_paths_tri<NP, nib2_t, false>(ctx, n, H, W, e, Cv, Cv, (nib2_t*)Av, plane, raw);
    }
    if (acc_is_u8(e)) return launch_paths16<NP, uint8_t>(ctx, n, H, W, e, Cv, (uint8_t*)Av, raw);
    return launch_paths16<NP, uint16_t>(ctx, n, H, W, e, Cv, (uint16_t*)Av, raw);
}

// D = 16 (captureDisparity's create(0, 16, 5, 200, 800)): the directions side
// by side at 8 lanes per line / row (one disparity pair per lane), in every
// launch shape -- the per-pixel work is small enough that the planes' traffic
// never outweighs the single-frame latency of a strip chain.  Planes as in
// launch_paths16_acc's side-by-side branch: nibbles (P2 <= 15), else bytes or
// u16.
int launch_paths_d16(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, int16_t* Cv, void* Av,
                     int16_t* raw)
{
    int rc;
    if ((rc = ensure(ctx, ctx->dummy, 512 * 16 * 2, "sgbm dummy slots"))) return rc;
    if ((rc = ensure(ctx, ctx->keys, (size_t)n * H * W * 4, "sgbm right-view keys"))) return rc;
    if (e.P2 <= 15) {
        if (sgbm_no_wrap(e)) return launch_paths_dirs<1, nib2_t, true, false, 8>(ctx, n, H, W, e, Cv, Cv, (nib2_t*)Av, raw);
        return launch_paths_dirs<1, nib2_t, false, false, 8>(ctx, n, H, W, e, Cv, Cv, (nib2_t*)Av, raw);
    }
    if (acc_is_u8(e)) return launch_paths_dirs<1, uint8_t, false, false, 8>(ctx, n, H, W, e, Cv, Cv, (uint8_t*)Av, raw);
    return launch_paths_dirs<1, uint16_t, false, false, 8>(ctx, n, H, W, e, Cv, Cv, (uint16_t*)Av, raw);
}

template <int NP>
int launch_paths_acc(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, int16_t* Cv,
                     void* Av, int16_t* raw)
{
    if (acc_is_u8(e)) return launch_paths<NP, uint8_t>(ctx, n, H, W, e, Cv, (uint8_t*)Av, raw);
    return launch_paths<NP, uint16_t>(ctx, n, H, W, e, Cv, (uint16_t*)Av, raw);
}

}  // namespace

int sgbm_plan(const mvsv_ctx* ctx, const SgbmEff& e, int n, int H)
{
    if (e.minX1 >= e.maxX1) return 0;
    const int sched = path_schedule(ctx, e, H, n);
    const bool bs = bsgm_eligible(ctx, e, n, H) && (sched == 1 || sched == 2) && ctx->path16 && ctx->tri &&
                    ctx->cost_fixed_pp && e.SH2 <= 7 && e.SW2 == e.SH2 && cost2_runs(ctx, e);
    int plan = (bs ? MVSV_PLAN_BITSLICE : 0) | (sched == 2 ? MVSV_PLAN_SIDE : 0) | (sched == 1 ? MVSV_PLAN_STRIPS : 0);
    if (!bs && use_residual(ctx, e, sched) && cost2_runs(ctx, e)) plan |= MVSV_PLAN_RESIDUAL;
    return plan;
}

bool sgbm_graphable(const mvsv_ctx* ctx, const SgbmEff& e, int n, int H)
{
    return e.minX1 < e.maxX1 && e.D <= 512 && path_schedule(ctx, e, H, n) == 2;
}

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
    if ((rc = ensure(ctx, ctx->pre, (size_t)n * 2 * plane * 8, "sgbm BT interval planes"))) return rc;
    // (rows padded to a multiple of 4 pixels: the bit-sliced pipeline's layout)
    if ((rc = ensure(ctx, ctx->cost, (size_t)n * H * ((e.W1 + 3) & ~3) * e.D * 2, "sgbm cost volume"))) return rc;
    // bit-sliced MODE_HH paths (round 5, mvsv_bsgm.hip): the cost kernel writes
    // the C' bit planes instead of the residual nibbles; the planes of the
    // direction passes are sized by bsgm_paths
    // accumulator planes: one per concurrently written direction group
    const int sched = path_schedule(ctx, e, H, n);
    // (frame batches: the bit-sliced strips; launches too small to fill the
    // GPU with strips -- one camera frame, schedule 2 -- the bit-sliced
    // directions side by side, each on its own chains: bsgm_paths)
    const bool bs = bsgm_eligible(ctx, e, n, H) && (sched == 1 || sched == 2) && ctx->path16 && ctx->tri &&
                    ctx->cost2 && ctx->cost_fixed_pp && e.SH2 <= 7 && e.SW2 == e.SH2;
    uint32_t* Bv = nullptr;
    const int nplanes = sched == 2 ? (e.fullDP ? 7 : 4) + (wta_split(ctx, e) ? 1 : 0)
                                   : sched == 1 ? (e.fullDP ? 3 : 2) : 1;
    // 4-bit planes: one per direction (side by side, P2 <= 15) or per strip
    // pass + lines; bytes / u16 otherwise (side by side: one delta <= P2 each)
    const bool nib = (sched == 2 && e.P2 <= 15) || (sched == 1 && nplanes > 1 && acc_is_nib(e));
    const bool u8 = acc_is_u8(e);
    if (!bs && (rc = ensure(ctx, ctx->agg, nib ? (size_t)nplanes * n * vol / 2
                                               : (size_t)nplanes * n * vol * (u8 ? 1 : 2),
                            "sgbm path-delta accumulator")))
        return rc;
    if ((rc = ensure(ctx, ctx->raw, (size_t)n * plane * 2, "sgbm raw disparity"))) return rc;
    // residual plane for the direction passes (0.5 byte per cost instead of 2)
    // + the per-pixel cost minimum (u16 per cost column) behind it
    uint8_t* Rv = nullptr;
    uint16_t* Mv = nullptr;
    if (bs) {
        const size_t bbytes = (bsgm_plane_bytes(n, H, e.W1) + 255) & ~(size_t)255;
        if ((rc = ensure(ctx, ctx->cres, bbytes + (size_t)n * e.W1 * H * 2, "sgbm bit-sliced cost planes")))
            return rc;
        Bv = (uint32_t*)ctx->cres.ptr;
        Mv = (uint16_t*)((uint8_t*)ctx->cres.ptr + bbytes);
    } else if (use_residual(ctx, e, sched)) {
        const size_t rbytes = (n * vol / 2 + 255) & ~(size_t)255;
        if ((rc = ensure(ctx, ctx->cres, rbytes + (size_t)n * e.W1 * H * 2, "sgbm cost residual plane"))) return rc;
        Rv = (uint8_t*)ctx->cres.ptr;
        Mv = (uint16_t*)(Rv + rbytes);
    }
    uint64_t* pre = (uint64_t*)ctx->pre.ptr;
    int16_t* Cv = (int16_t*)ctx->cost.ptr;
    void* Sv = ctx->agg.ptr;
    int16_t* raw = (int16_t*)ctx->raw.ptr;
    const unsigned epoch0 = ctx->tri_epoch;

    if ((rc = launch_prefilter(ctx, n, L, ls, lfs, R, rs, rfs, W, H, e.ftzero, pre))) return rc;

    // cost volume: one block per TX x TY tile; keep the LDS image <= 160 KiB
    // Taller tiles re-read fewer halo rows (2*SH2 per tile); shorter ones give
    // small batches enough blocks (>= 2 per CU) to fill the chip.
    int TY = 16;
    if (ctx->cost_ty > 0) {
        TY = ctx->cost_ty;
    } else if (H >= 256) {
        const int TX = cost2_layout(e.D, e.SW2, 120).TX;
        const long tiles_x = (e.W1 + TX - 1) / TX;
        auto tiles = [&](int ty) { return tiles_x * ((H + ty - 1) / ty) * n; };
        TY = 120;
        if (tiles(120) < 1024) {
            // small launches: least per-CU work, tiles per CU x rows per tile
            // incl. the 2*SH2 halo, a lone tile on a CU counted 1.5x (8 waves
            // hide less latency than 16); measured against forced heights: one
            // 640x480 frame 0.097 -> 0.073 ms, two 0.124 -> 0.110 ms, one
            // 1280x960 frame 0.227 -> 0.187 ms
            long best = -1;
            for (int ty : kCostTileHeights) {
                const long per_cu = (tiles(ty) + ctx->cus - 1) / ctx->cus;
                const long c = per_cu * (ty + 2 * e.SH2) * (per_cu == 1 ? 3 : 2);
                if (best < 0 || c < best) {
                    best = c;
                    TY = ty;
                }
            }
        }
    }
    bool pinned_hh = false;
    if ((rc = launch_cost(ctx, n, W, H, e, TY, pre, Cv, &Rv, Mv, &pinned_hh, &Bv))) return rc;
    if (bs && !Bv) {
        // the cost kernel could not write the planes (a launch shape without
        // the D = 128 register-ring kernel): the packed kernels on C
        if ((rc = ensure(ctx, ctx->agg, nib ? (size_t)nplanes * n * vol / 2
                                            : (size_t)nplanes * n * vol * (u8 ? 1 : 2),
                         "sgbm path-delta accumulator")))
            return rc;
        Sv = ctx->agg.ptr;
    }

    if (Bv) {
        // bit-sliced layouts (MODE_SGBM: copied rows / column 0; MODE_HH: pinned
        // by the cost kernel)
        if ((rc = bsgm_cost_fixup(ctx, n, H, e, Cv, Bv, Mv))) return rc;
    } else if (H > 1 && !pinned_hh) {
        // OpenCV 3.4's never-recomputed rows and column 0 (mvsv_cost.hip)
        if ((rc = launch_cost_fixup(ctx, n, H, e, Cv, Rv, Mv))) return rc;
    }

    const int np = (e.D + 127) / 128;
    const bool wide = ctx->path16 && (e.D == 32 || e.D == 64 || e.D == 128 || e.D == 256);
    if (Bv) {
        rc = bsgm_paths(ctx, n, H, W, e, Cv, Bv, Mv, raw, sched == 2);
    } else if (e.D == 16 && sched == 2) {
        rc = launch_paths_d16(ctx, n, H, W, e, Cv, Sv, raw);
    } else if (wide) {
        switch (e.D) {
        case 32: rc = launch_paths16_acc<1>(ctx, n, H, W, e, Cv, Rv, Mv, Sv, raw); break;
        case 64: rc = launch_paths16_acc<2>(ctx, n, H, W, e, Cv, Rv, Mv, Sv, raw); break;
        case 128: rc = launch_paths16_acc<4>(ctx, n, H, W, e, Cv, Rv, Mv, Sv, raw); break;
        default: rc = launch_paths16_acc<8>(ctx, n, H, W, e, Cv, nullptr, nullptr, Sv, raw); break;
        }
    } else if (np == 1) rc = launch_paths_acc<1>(ctx, n, H, W, e, Cv, Sv, raw);
    else if (np == 2) rc = launch_paths_acc<2>(ctx, n, H, W, e, Cv, Sv, raw);
    else rc = launch_paths_acc<4>(ctx, n, H, W, e, Cv, Sv, raw);
    if (rc) return rc;

    // a strip launch of this call that gave up a wait poisons the median's output
    const bool strips_ran = ctx->tri_epoch != epoch0;
    StageTimer tm(ctx, kStagePost);
    const int* poison = strips_ran ? (const int*)ctx->status.ptr : nullptr;
    if ((rc = median3x3_device(ctx, n, raw, W, plane, out, os, ofs, W, H, poison, ctx->tri_epoch, e.invalid)))
        return rc;
    if (e.speckle_window > 0)
        return speckle_device(ctx, n, out, os, ofs, W, H, e.invalid, e.speckle_window, e.speckle_diff);
    return MVSV_OK;
}

}  // namespace mvsv
