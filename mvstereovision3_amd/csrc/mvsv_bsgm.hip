// mvsv_bsgm.hip — bit-sliced MODE_HH path aggregation (round 5).
//
// The same eight SGM directions as the packed-int16 kernels of mvsv_sgbm.hip
// (OpenCV 3.4 computeDisparitySGBM, reached through Disparity::sgbm /
// loadSGBMParameters, /root/reference/src/disparity.cpp:6-10,92-95; semantics in
// SURVEY.md Appendix A.4-A.5), restated on bit planes (mvsv_bitslice.hpp): in
// the headline regime (P1 = 2, P2 = 5, no-wrap, D = 128, uniquenessRatio 0)
// a direction's state s(d) = min(L(d) - min L, P2), its delta and the clamped
// cost residual C' are 3- and 4-bit numbers, so one v_bitop3_b32 updates 32
// disparities of one bit.  A pixel's 128 disparities live on two lanes (h = 0,
// 1: d in [64 h, 64 h + 64)) as parity words E (even d) / O (odd d), one per
// bit; d -+ 1 neighbours are the other parity word, shifted by one where the
// pair crosses into the partner lane (one DPP swap).
//
//   bsgm_strip_kernel  the six vertical / diagonal directions of both passes on
//                      sheared strips (the strip chain, tickets and boundary
//                      hand-off of sgbm_tri_kernel), one wave per direction
//   bsgm_lines4_kernel L->R and R->L along the rows (a pixel on a lane quad)
//   bsgm_wta_kernel    S'' = 8 C' + sum of deltas, argmin (smallest d), exact
//                      S(best -+ 1) for the parabola, right-view keys, LR check
//
// Data (per frame, W1 cost columns): C' planes and each strip pass's delta-sum
// planes [H][W1][16 words] (64 B per pixel: word h*8 + e*4 + b); line delta
// planes [H][W1][12 words] (h*6 + e*3 + b).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "mvsv_bitslice.hpp"
#include "mvsv_device.hpp"
#include "mvsv_internal.hpp"

namespace mvsv {

using namespace dev;

namespace {

constexpr uint32_t kOnes = 0xffffffffu;

// value of the partner lane (lane ^ 1: the pixel's other 64-disparity half)
__device__ __forceinline__ uint32_t xswap(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xf, 0xf, true);  // quad_perm [1,0,3,2]
}

// One direction step of one pixel on its lane pair (mirrored on the host by
// pair_step in tests/cpp/bitslice_check.cpp).  s: previous state (E / O words
// of 3 bits), c: C' of the cell (4 bits); fill0 / fill1 = all-ones on the h = 0
// / h = 1 lane (disparities -1 and 128 read the code 7, which maps to P2).
// Out: the new state n and the delta d.
template <int P1, int P2>
__device__ __forceinline__ void bs_dir_step(const uint32_t (&sE)[3], const uint32_t (&sO)[3],
                                            const uint32_t (&cE)[4], const uint32_t (&cO)[4], uint32_t fill0,
                                            uint32_t fill1, uint32_t (&nE)[3], uint32_t (&nO)[3],
                                            uint32_t (&dE)[3], uint32_t (&dO)[3])
{
    uint32_t slE[3], srO[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t prevO = xswap(sO[k]) | fill0;  // d = 64 h - 1: the h = 0 lane's last odd word
        const uint32_t nextE = xswap(sE[k]) | fill1;  // d = 64 h + 64: the h = 1 lane's first even word
        slE[k] = bs::fshr(sO[k], prevO, 31);
        srO[k] = bs::fshr(nextE, sE[k], 1);
    }
    bs::delta3<P1, P2>(sE, slE, sO, dE);
    bs::delta3<P1, P2>(sO, sE, srO, dO);
    uint32_t vE[4], vO[4];
    bs::add43(cE, dE, vE);
    bs::add43(cO, dO, vO);
    // min over the pixel's 128 v = C' + delta, bit-serial from bit 2: some d has
    // C' = 0, so the minimum is <= P2 < 8
    uint32_t kE = ~vE[3], kO = ~vO[3], M[3];
#pragma unroll
    for (int b = 2; b >= 0; b--) {
        const uint32_t zE = bs::lop3<bs::kAndNotAB>(vE[b], kE, kE);
        const uint32_t zO = bs::lop3<bs::kAndNotAB>(vO[b], kO, kO);
        uint32_t any = zE | zO;
        any |= xswap(any);
        const bool f = any != 0u;
        if (b > 0) {
            kE = f ? zE : kE;
            kO = f ? zO : kO;
        }
        M[b] = f ? 0u : kOnes;
    }
    bs::subclamp<P2>(vE, M[0], M[1], M[2], nE);
    bs::subclamp<P2>(vO, M[0], M[1], M[2], nO);
}

// The same step with a pixel on a lane quad, q = 2 h + e: the lane holds only
// the parity-e words of half h, so a step is half the instructions per lane
// (one delta, one add, one clamp) for twice the lanes -- the serial chains of a
// pass run at half the latency per step.  Neighbours: d -+ 1 of an even word
// is the partner word (lane q ^ 1) and, shifted in, the odd word of the lane
// below (q - 1); of an odd word the partner and the even word of q + 1.  One
// v_alignbit of (hi = quad lane q + 1, lo = q - 1) by 31 (even) / 1 (odd)
// gives the shifted neighbour, the partner is lo (odd) or hi (even).
// fill_hi / fill_lo: all-ones on q = 3 / q = 0 (d = 128 / -1: code 7 -> P2).
template <int P1, int P2>
__device__ __forceinline__ void bs_quad_step(const uint32_t (&s)[3], const uint32_t (&c)[4], uint32_t fill_hi,
                                             uint32_t fill_lo, bool odd, uint32_t sh, uint32_t (&n)[3],
                                             uint32_t (&d)[3])
{
    uint32_t nb[3], pt[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)s[k], 0xF9, 0xf, 0xf, true) | fill_hi;  // [1,2,3,3]
        const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)s[k], 0x90, 0xf, 0xf, true) | fill_lo;  // [0,0,1,2]
        nb[k] = __builtin_amdgcn_alignbit(hi, lo, sh);
        pt[k] = odd ? lo : hi;
    }
    bs::delta3<P1, P2>(s, nb, pt, d);
    uint32_t v[4];
    bs::add43(c, d, v);
    uint32_t kk = ~v[3], M[3];
#pragma unroll
    for (int b = 2; b >= 0; b--) {
        const uint32_t z = bs::lop3<bs::kAndNotAB>(v[b], kk, kk);
        uint32_t any = z | xswap(z);
        any |= (uint32_t)__builtin_amdgcn_mov_dpp((int)any, 0x4E, 0xf, 0xf, true);  // quad_perm [2,3,0,1]
        const bool f = any != 0u;
        if (b > 0) kk = f ? z : kk;
        M[b] = f ? 0u : kOnes;
    }
    bs::subclamp<P2>(v, M[0], M[1], M[2], n);
}

// ---------------------------------------------------------------------------
// Strips: the three directions of a pass on sheared U-columns (U = x - t + H - 1,
// t the step: y for the down pass, H - 1 - y for the up pass); the
// predecessors of U at step t are U (dir a = (1, sy)), U + 1 (b = (0, sy)) and
// U + 2 (c = (-1, sy)) of step t - 1 (the geometry of sgbm_tri_kernel).  A block
// owns 32 NG U-columns; wave 3 g + r runs direction r for columns 32 g .. 32 g +
// 31 of the strip (two lanes per column), the last wave moves the strip's
// boundary states to / from its neighbours.  Directions b and c hand their
// new states and deltas over through LDS; wave a sums the three deltas of a
// cell one step later and stores the pass's 4-bit plane.
// ---------------------------------------------------------------------------
template <int NG>
struct BsStripCfg {
    static constexpr int kSW = 32 * NG;          // U-columns per strip
    static constexpr int kCompute = 3 * NG;      // compute waves
    static constexpr int kThreads = 64 * (kCompute + 1);
    static constexpr int kCols = kSW + 2;        // + two columns of the right strip
    static constexpr int kSt = 2 * 2 * 6 * kCols * 2;  // states [buf][dir b, c][word][col][h]
    static constexpr int kDl = 2 * 2 * 6 * kSW * 2;    // deltas [buf][dir b, c][word][col][h]
    static constexpr size_t kBytes = (size_t)(kSt + kDl) * 4;
};
// boundary words per strip step: (dir b, column 0), (dir c, column 0), (dir c,
// column 1), each 2 lanes x 6 words; one u64 granule = 32-bit launch tag | word
constexpr int kBsGran = 36;
constexpr int kBsPF = 4;  // steps of C' prefetch (compute waves)
constexpr int kBsStripLds = 96 * 1024;  // strip block LDS allocation (launch_bs_strips)
constexpr int kBsBF = 4;  // steps of boundary prefetch (exchange wave)

template <int NG, int P1, int P2>
__global__ __launch_bounds__(BsStripCfg<NG>::kThreads) void bsgm_strip_kernel(
    const uint32_t* __restrict__ Bc, uint32_t* __restrict__ A, size_t plane_words, uint32_t* __restrict__ dummy,
    int H, int W1, int npass,
    unsigned long long* __restrict__ bnd, unsigned epoch, int nframes, int* __restrict__ status,
    unsigned spin_limit, int* __restrict__ report, long long ticket0, unsigned long long* __restrict__ stats,
    int)
{
    using Cfg = BsStripCfg<NG>;
    constexpr int SW = Cfg::kSW, NCOL = Cfg::kCols;
    extern __shared__ __attribute__((aligned(16))) uint32_t bs_lds[];
    uint32_t* st = bs_lds;
    uint32_t* dlt = bs_lds + Cfg::kSt;
    auto sti = [&](int buf, int d, int k, int c, int h) { return (((buf * 2 + d) * 6 + k) * NCOL + c) * 2 + h; };
    auto dli = [&](int buf, int d, int k, int c, int h) { return (((buf * 2 + d) * 6 + k) * SW + c) * 2 + h; };
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool comm = w == Cfg::kCompute;

    // strip ticket (sgbm_tri_kernel: a strip only ever waits on a strip whose
    // block arrived before it, whatever the dispatch order)
    __shared__ int s_ticket;
    if (threadIdx.x == 0)
        s_ticket = ticket0 < 0 ? (int)blockIdx.x
                               : (int)(__hip_atomic_fetch_add((unsigned*)status + 2, 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT) - (unsigned)ticket0);
    __syncthreads();
    const int bx = s_ticket;
    if ((unsigned)bx >= gridDim.x) {
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
    const int Utot = W1 + H - 1;
    const int U0 = Utot - SW * (k + 1);
    const int tb = max(0, (H - 1) - (U0 + SW - 1));
    const int te = min(H, W1 + (H - 1) - U0);
    if (tb >= te) return;

    for (int i = threadIdx.x; i < Cfg::kSt + Cfg::kDl; i += Cfg::kThreads) bs_lds[i] = 0u;

    // ---- exchange wave: lane j < 36 carries word (h, k) = (j % 12 / 6, j % 6)
    // of item j / 12; lanes 36..63 repeat lanes 0..27 (same addresses, same
    // values), so every memory instruction is unpredicated
    const int jj = lane < kBsGran ? lane : lane - kBsGran;
    const int item = jj / 12, wi = jj - 12 * item;
    const int ih = wi / 6, ik = wi - 6 * ih;
    const int idir = item == 0 ? 0 : 1;
    const int icol_in = SW + (item == 2 ? 1 : 0);  // LDS column the right strip's item lands in
    const int icol_out = item == 2 ? 1 : 0;        // own column published as item
    const size_t slot_step = kBsGran;
    const unsigned long long* bsrc =
        bnd + (((size_t)(k > 0 ? k - 1 : 0) * nchains + chain) * H) * slot_step + jj;
    unsigned long long* pdst = bnd + (((size_t)k * nchains + chain) * H) * slot_step + jj;
    const unsigned long long tag = (unsigned long long)epoch << 32;
    auto bvalid = [&](int t) {
        const int xx = U0 + icol_in - (H - 1) + t;
        return k > 0 && t >= 0 && xx >= 0 && xx < W1;
    };
    auto bload = [&](int t) -> unsigned long long {
        return __hip_atomic_load(bsrc + (size_t)clampi(t, 0, H - 1) * slot_step, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    };
    unsigned long long st_t0 = stats ? __builtin_amdgcn_s_memtime() : 0ull, st_spin = 0, st_n = 0;
    auto bconsume = [&](int t, int buf, unsigned long long g) {
        const bool need = bvalid(t);
        bool ok = !need || (unsigned)(g >> 32) == epoch;
        if (!__all(ok)) {
            const unsigned long long sp0 = stats ? __builtin_amdgcn_s_memtime() : 0ull;
            unsigned spins = 0;
            while (!__all(ok)) {
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
                g = bload(t);
                ok = !need || (unsigned)(g >> 32) == epoch;
            }
            if (stats) {
                st_spin += __builtin_amdgcn_s_memtime() - sp0;
                st_n += spins;
            }
        }
        st[sti(buf, idir, ik, icol_in, ih)] = need ? (uint32_t)g : 0u;
    };
    auto publish = [&](int t, int buf) {
        const uint32_t v = st[sti(buf, idir, ik, icol_out, ih)];
        __hip_atomic_store(pdst + (size_t)clampi(t, 0, H - 1) * slot_step, tag | v, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    };

    // ---- compute waves
    const int grp = comm ? 0 : w / 3;
    const int dir = comm ? 0 : w - 3 * grp;  // 0 = (1, sy), 1 = (0, sy), 2 = (-1, sy)
    const int u = lane >> 1, h = lane & 1;
    const int col = grp * 32 + u;
    const int U = U0 + col;
    const uint32_t fill0 = h == 0 ? kOnes : 0u, fill1 = h == 1 ? kOnes : 0u;
    auto cell_x = [&](int t) { return U - (H - 1) + t; };
    // word offset of the lane's half of cell (x(t), y(t)); cells outside the
    // image read the frame's first cell (their results are discarded)
    const int rowW = sy > 0 ? W1 : -W1;
    const int c0 = ((f * H + (sy > 0 ? 0 : H - 1)) * W1 + U - (H - 1)) * 16 + h * 8;
    const int cst = (rowW + 1) * 16;
    const int fbase = f * H * W1 * 16 + h * 8;
    auto cell_off = [&](int t) -> int { return (unsigned)cell_x(t) < (unsigned)W1 ? c0 + t * cst : fbase; };
    // the cell's E words in the grouped C' plane (bs::cq_word, q = 2 h); O at + 16
    const int W1q = bs::padq(W1);
    auto c_off = [&](int t) -> int {
        const int x = cell_x(t);
        if ((unsigned)x >= (unsigned)W1) return f * H * W1q * 16 + h * 32;
        return (int)bs::cq_word((size_t)(f * H + (sy > 0 ? t : H - 1 - t)) * W1q, x, 2 * h);
    };
    uint32_t* Ap = A + (size_t)pass * plane_words;
    uint4 cb[kBsPF][2];
    uint32_t sa[6];  // direction a's state (E words 0..2, O words 3..5)
#pragma unroll
    for (int q = 0; q < 6; q++) sa[q] = 0u;
    uint32_t pdl[6];  // direction a's delta of the previous step
    int pend_off = -1;
    unsigned long long bg[kBsBF];

    __syncthreads();  // LDS zeroed
    if (comm) {
        __builtin_amdgcn_s_setprio(1);  // the exchange wave gates every step's barrier
        bconsume(tb - 1, 1, bload(tb - 1));
#pragma unroll
        for (int j = 0; j < kBsBF; j++) bg[j] = bload(tb + j);
    } else {
#pragma unroll
        for (int j = 0; j < kBsPF; j++) {
            const uint4* q = (const uint4*)(Bc + c_off(min(tb + j, te - 1)));
            cb[j][0] = q[0];
            cb[j][1] = q[4];
        }
    }
    __syncthreads();

    auto comm_step = [&](int i, int j) {
        const int t = tb + i;
        const int cur = i & 1, prv = cur ^ 1;
        if (i > 0) publish(t - 1, prv);
        bconsume(t, cur, bg[j]);
        bg[j] = bload(t + kBsBF);
        __syncthreads();
    };
    // direction a: the three deltas of the previous step's cell -> the pass plane
    auto flush_a = [&](int prv) {
        uint32_t db[6], dc[6];
#pragma unroll
        for (int q = 0; q < 6; q++) {
            db[q] = dlt[dli(prv, 0, q, col, h)];
            dc[q] = dlt[dli(prv, 1, q, col, h)];
        }
        uint32_t o[2][4];
#pragma unroll
        for (int e = 0; e < 2; e++) {
            const uint32_t a3[3] = {pdl[3 * e], pdl[3 * e + 1], pdl[3 * e + 2]};
            const uint32_t b3[3] = {db[3 * e], db[3 * e + 1], db[3 * e + 2]};
            const uint32_t c3[3] = {dc[3 * e], dc[3 * e + 1], dc[3 * e + 2]};
            uint32_t ab[4];
            bs::add33(a3, b3, ab);
            bs::add43(ab, c3, o[e]);  // <= 3 P2 = 15
        }
        // unpredicated: a cell outside the image stores into the lane's dummy
        // slot, so the prefetch loads' wait counts stay exact
        uint4* q = pend_off >= 0 ? (uint4*)(Ap + pend_off) : (uint4*)(dummy + lane * 8);
        q[0] = make_uint4(o[0][0], o[0][1], o[0][2], o[0][3]);
        q[1] = make_uint4(o[1][0], o[1][1], o[1][2], o[1][3]);
    };
    // one step of direction DIR (compile time: each direction's loop has its
    // own LDS offsets and register allocation)
    auto step = [&](auto dtag, int i, int j) {
        constexpr int DIR = decltype(dtag)::value;
        const int t = tb + i;
        const int cur = i & 1, prv = cur ^ 1;
        const int x = cell_x(t);
        const bool valid = x >= 0 && x < W1;
        const uint32_t cE[4] = {cb[j][0].x, cb[j][0].y, cb[j][0].z, cb[j][0].w};
        const uint32_t cO[4] = {cb[j][1].x, cb[j][1].y, cb[j][1].z, cb[j][1].w};
        uint32_t sE[3], sO[3];
        if constexpr (DIR == 0) {
            if (i > 0) flush_a(prv);
#pragma unroll
            for (int q = 0; q < 3; q++) {
                sE[q] = sa[q];
                sO[q] = sa[3 + q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < 3; q++) {
                sE[q] = st[sti(prv, DIR - 1, q, col + DIR, h)];
                sO[q] = st[sti(prv, DIR - 1, 3 + q, col + DIR, h)];
            }
        }
        uint32_t nE[3], nO[3], dE[3], dO[3];
        bs_dir_step<P1, P2>(sE, sO, cE, cO, fill0, fill1, nE, nO, dE, dO);
        {
            // the slot's next load once its words are consumed (same registers)
            const uint4* q = (const uint4*)(Bc + c_off(min(t + kBsPF, te - 1)));
            cb[j][0] = q[0];
            cb[j][1] = q[4];
            __builtin_amdgcn_sched_barrier(0);
        }
        if (!valid) {
#pragma unroll
            for (int q = 0; q < 3; q++) nE[q] = nO[q] = 0u;
        }
        if constexpr (DIR == 0) {
#pragma unroll
            for (int q = 0; q < 3; q++) {
                sa[q] = nE[q];
                sa[3 + q] = nO[q];
                pdl[q] = dE[q];
                pdl[3 + q] = dO[q];
            }
            pend_off = valid ? cell_off(t) : -1;
        } else {
#pragma unroll
            for (int q = 0; q < 3; q++) {
                st[sti(cur, DIR - 1, q, col, h)] = nE[q];
                st[sti(cur, DIR - 1, 3 + q, col, h)] = nO[q];
                dlt[dli(cur, DIR - 1, q, col, h)] = dE[q];
                dlt[dli(cur, DIR - 1, 3 + q, col, h)] = dO[q];
            }
        }
        __syncthreads();
    };
    auto run = [&](auto dtag) {
        const int len = te - tb;
        int i = 0;
        for (; i + kBsPF <= len; i += kBsPF) {
#pragma unroll
            for (int j = 0; j < kBsPF; j++) step(dtag, i + j, j);
        }
#pragma unroll
        for (int j = 0; j < kBsPF; j++)
            if (i + j < len) step(dtag, i + j, j);
        __syncthreads();
        if constexpr (decltype(dtag)::value == 0) flush_a((len - 1) & 1);
    };
    if (comm) {
        const int len = te - tb;
        int i = 0;
        for (; i + kBsBF <= len; i += kBsBF) {
#pragma unroll
            for (int j = 0; j < kBsBF; j++) comm_step(i + j, j);
        }
#pragma unroll
        for (int j = 0; j < kBsBF; j++)
            if (i + j < len) comm_step(i + j, j);
        __syncthreads();
        publish(te - 1, (len - 1) & 1);
        if (stats && lane == 0) {
            unsigned long long* q = stats + (size_t)bx * 8;
            q[0] = st_t0;
            q[1] = __builtin_amdgcn_s_memtime();
            q[2] = st_spin;
            q[3] = st_n;
            q[4] = (unsigned long long)len;
            q[5] = (unsigned long long)k;
            q[6] = (unsigned long long)pass;
            q[7] = (unsigned long long)tb;
        }
    } else if (dir == 0) {
        run(std::integral_constant<int, 0>());
    } else if (dir == 1) {
        run(std::integral_constant<int, 1>());
    } else {
        run(std::integral_constant<int, 2>());
    }
}

// ---------------------------------------------------------------------------
// Lines: L->R (blockIdx.z = 0) and R->L (1); each writes its delta plane (3 bits).
// ---------------------------------------------------------------------------
// The lines on lane quads (bs_quad_step): 16 rows per wave, lane 4 r + q holds
// words (h, e) = (q >> 1, q & 1) of row r, so the grid has twice the waves of a
// lane-pair layout at two thirds of the instructions per step.  The planes are
// grouped by four pixels (bs::cq_word / dl_word): per four steps a lane loads 64
// contiguous bytes of C' (kBsLG groups ahead, in registers) and stores 48 of
// deltas -- with one 16-byte load and one 12-byte store per step (a load
// instruction then covering 16 rows x 64 bytes) the pass measured 0.50 ms of
// which 0.28 went to those loads and 0.14 to those stores (probes with the
// loads from one cached row / the stores to one slot, profiles/r05/README.md).
constexpr int kBsLG = 8;

template <int P1, int P2>
__device__ __forceinline__ void bs_line_chains(const uint32_t* __restrict__ Bc, uint32_t* __restrict__ Dl,
                                               size_t plane_words, int H, int W1, bool rl)
{
    const int lane = threadIdx.x;
    const int q = lane & 3, rr = lane >> 2;
    const int y = min((int)blockIdx.x * 16 + rr, H - 1);
    const int f = blockIdx.y;
    const bool odd = (q & 1) != 0;
    const uint32_t fill_hi = q == 3 ? kOnes : 0u, fill_lo = q == 0 ? kOnes : 0u, sh = odd ? 1u : 31u;
    const size_t rowq = (size_t)(f * H + y) * bs::padq(W1);
    // group g's 64 bytes of this lane / its 48 delta bytes
    const uint4* cgrp = (const uint4*)(Bc + bs::cq_word(rowq, 0, q));
    const int G = (W1 + 3) >> 2;
    const int part = W1 & 3;
    auto run = [&](auto rltag) __attribute__((always_inline)) {
        constexpr bool RL = decltype(rltag)::value;
        uint4* dgrp = (uint4*)(Dl + (RL ? plane_words : 0) + bs::dl_word(rowq, 0, q));
        // group of the i-th group step (clamped: loads past the row are issued, not used)
        auto grp = [&](int i) { return RL ? max(G - 1 - i, 0) : min(i, G - 1); };
        uint4 cr[kBsLG][4];
        auto load = [&](int j, int i) {
            const uint4* p = cgrp + (size_t)grp(i) * 16;
#pragma unroll
            for (int u = 0; u < 4; u++) cr[j][u] = p[u];
        };
        // R->L with a partial group: that group (step 0) first, from its own
        // registers; ring slot j then holds group steps ph + j + kBsLG m
        const int ph = (RL && part) ? 1 : 0;
        uint4 c0[4];
        if (ph) {
#pragma unroll
            for (int u = 0; u < 4; u++) c0[u] = cgrp[(size_t)grp(0) * 16 + u];
        }
        // (issued in slot order: the loop head's wait for slot 0 assumes it)
#pragma unroll
        for (int j = 0; j < kBsLG; j++) {
            load(j, ph + j);
            __builtin_amdgcn_sched_barrier(0);
        }
        uint32_t st[3] = {0u, 0u, 0u};
        // the pixels x = 4 g + u of group step i (u descending for R->L); n < 4:
        // the row's partial group (x >= W1 skipped: the state must not advance)
        auto group = [&](int i, uint4 (&cg)[4], int n) {
            uint32_t dv[12];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int u = RL ? 3 - k : k;
                if (u < n) {
                    const uint32_t cw[4] = {cg[u].x, cg[u].y, cg[u].z, cg[u].w};
                    uint32_t nw[3], dw[3];
                    bs_quad_step<P1, P2>(st, cw, fill_hi, fill_lo, odd, sh, nw, dw);
#pragma unroll
                    for (int b = 0; b < 3; b++) {
                        st[b] = nw[b];
                        dv[3 * u + b] = dw[b];
                    }
                } else {
#pragma unroll
                    for (int b = 0; b < 3; b++) dv[3 * u + b] = 0u;
                }
            }
            uint4* o = dgrp + (size_t)grp(i) * 12;
            o[0] = make_uint4(dv[0], dv[1], dv[2], dv[3]);
            o[1] = make_uint4(dv[4], dv[5], dv[6], dv[7]);
            o[2] = make_uint4(dv[8], dv[9], dv[10], dv[11]);
        };
        // a ring group: compute, then reload its slot kBsLG group steps ahead
        auto ring = [&](int i, int j, int n) {
            group(i, cr[j], n);
            load(j, i + kBsLG);
            __builtin_amdgcn_sched_barrier(0);
        };
        // the partial group (W1 % 4 pixels) is the last for L->R and the first
        // for R->L.  Whole blocks of kBsLG groups without exits in between (an
        // exit per group would make the loop head wait for every load in flight)
        if (ph) group(0, c0, part);
        const int full_end = (RL || !part) ? G : G - 1;
        int i = ph;
        for (; i + kBsLG <= full_end; i += kBsLG) {
#pragma unroll
            for (int j = 0; j < kBsLG; j++) ring(i + j, j, 4);
        }
        // tail: full groups, then L->R's partial group (slot full_end - i)
#pragma unroll
        for (int j = 0; j < kBsLG; j++) {
            if (i + j < full_end)
                ring(i + j, j, 4);
            else if (i + j == full_end && !RL && part)
                ring(i + j, j, part);
        }
    };
    if (rl)
        run(std::true_type());
    else
        run(std::false_type());
}

template <int P1, int P2>
__global__ __launch_bounds__(64) void bsgm_lines4_kernel(const uint32_t* __restrict__ Bc, uint32_t* __restrict__ Dl,
                                                          size_t plane_words, int H, int W1)
{
    bs_line_chains<P1, P2>(Bc, Dl, plane_words, H, W1, blockIdx.z != 0);
}

// ---------------------------------------------------------------------------
// Side by side (launches too small to fill the GPU with strip chains -- one or
// two camera frames, path_schedule 2): every direction on its own lane-quad
// chains, no strip hand-offs and no block barriers.  The vertical / diagonal
// directions step row by row (t; y = t down, H - 1 - t up), 16 chains per wave
// (lane 4 c + q: chain k0 + c, words (h, e) = (q >> 1, q & 1)), chain k on
// cell x = k + DX t; a chain outside the image carries the zero state (a path
// starts at the border).  Each direction writes its own grouped delta plane.
// A chain is as long as the image is tall, so a step costs the lane-quad
// step's latency (tools/ubench/bs_chain: 348 cycles) instead of a strip
// block's barrier-synchronised step.
// ---------------------------------------------------------------------------
constexpr int kBsDPF = 16;  // steps of C' prefetch

template <int DX, int P1, int P2>
__device__ __forceinline__ void bs_dir_chains(const uint32_t* __restrict__ Bc, uint32_t* __restrict__ Dp,
                                              size_t plane_words, int H, int W1, uint32_t* __restrict__ dummy,
                                              int pass)
{
    const int lane = threadIdx.x;
    const int c = lane >> 2, q = lane & 3;
    const int f = blockIdx.y;
    const bool odd = (q & 1) != 0;
    const uint32_t fill_hi = q == 3 ? kOnes : 0u, fill_lo = q == 0 ? kOnes : 0u, sh = odd ? 1u : 31u;
    const int kmin = DX > 0 ? -(H - 1) : 0;
    const int kend = DX < 0 ? W1 + H - 1 : W1;
    const int k0 = kmin + (int)blockIdx.x * 16;
    if (k0 >= kend) return;
    const int k = k0 + c;
    // the wave's steps with some cell inside the image
    const int tb = DX > 0 ? max(0, -(k0 + 15)) : DX < 0 ? max(0, k0 - W1 + 1) : 0;
    const int te = DX > 0 ? min(H, W1 - k0) : DX < 0 ? min(H, k0 + 16) : H;
    if (tb >= te) return;
    // 32-bit word offsets (bsgm_eligible bounds a plane below 2^31 words),
    // branch-free: the cell's column clamped into the row for the loads, the
    // validity only selects the state reset and the store slot
    const int W1q = bs::padq(W1);
    const int row0 = f * H + (pass == 0 ? 0 : H - 1), rs = pass == 0 ? 1 : -1;
    uint32_t* dplane = Dp + (size_t)(pass * 3 + (1 - DX)) * plane_words;  // slot: DX +1, 0, -1
    auto xrow = [&](int t, int& xc) -> uint32_t {
        xc = min(max(k + DX * t, 0), W1 - 1);
        return (uint32_t)(row0 + rs * t) * (uint32_t)W1q + (uint32_t)(xc & ~3);
    };
    auto coff = [&](int t) -> uint32_t {
        int xc;
        const uint32_t g = xrow(t, xc);
        return g * 16u + (uint32_t)(q * 16 + (xc & 3) * 4);
    };
    uint4 cr[kBsDPF];
#pragma unroll
    for (int j = 0; j < kBsDPF; j++) {
        cr[j] = *(const uint4*)(Bc + coff(min(tb + j, te - 1)));
        __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t st[3] = {0u, 0u, 0u};
    auto step = [&](int t, int j) {
        const bool valid = k < kend && (unsigned)(k + DX * t) < (unsigned)W1;
        const uint32_t cw[4] = {cr[j].x, cr[j].y, cr[j].z, cr[j].w};
        uint32_t nw[3], dw[3];
        bs_quad_step<P1, P2>(st, cw, fill_hi, fill_lo, odd, sh, nw, dw);
        cr[j] = *(const uint4*)(Bc + coff(min(t + kBsDPF, te - 1)));
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int b = 0; b < 3; b++) st[b] = valid ? nw[b] : 0u;
        // unpredicated: a cell outside the image stores into the lane's dummy slot
        int xc;
        const uint32_t g = xrow(t, xc);
        uint32_t* o = valid ? dplane + (g * 12u + (uint32_t)(q * 12 + (xc & 3) * 3)) : dummy + lane * 4;
        o[0] = dw[0];
        o[1] = dw[1];
        o[2] = dw[2];
    };
    int t = tb;
    for (; t + kBsDPF <= te; t += kBsDPF) {
#pragma unroll
        for (int j = 0; j < kBsDPF; j++) step(t + j, j);
    }
#pragma unroll
    for (int j = 0; j < kBsDPF; j++)
        if (t + j < te) step(t + j, j);
}

// blockIdx.z = pass * 3 + slot (slot 0, 1, 2: DX = +1, 0, -1); blockIdx.x: 16
// chains, as many as the longest direction has (W1 + H - 1).  z = 3 npass,
// 3 npass + 1: the two line directions (16 rows per block) into the planes
// after the vertical / diagonal ones -- one launch for all eight (MODE_HH,
// npass 2) or five (MODE_SGBM, npass 1) directions (a small launch pays no
// stream fork / join)
template <int P1, int P2>
__global__ __launch_bounds__(64) void bsgm_dir_kernel(const uint32_t* __restrict__ Bc, uint32_t* __restrict__ Dp,
                                                       size_t plane_words, int H, int W1,
                                                       uint32_t* __restrict__ dummy, int npass)
{
    const int zl = 3 * npass;
    if ((int)blockIdx.z >= zl) {
        if ((int)blockIdx.x * 16 < H)
            bs_line_chains<P1, P2>(Bc, Dp + (size_t)zl * plane_words, plane_words, H, W1, (int)blockIdx.z > zl);
        return;
    }
    const int pass = blockIdx.z / 3, slot = blockIdx.z - 3 * pass;
    if (slot == 0)
        bs_dir_chains<1, P1, P2>(Bc, Dp, plane_words, H, W1, dummy, pass);
    else if (slot == 1)
        bs_dir_chains<0, P1, P2>(Bc, Dp, plane_words, H, W1, dummy, pass);
    else
        bs_dir_chains<-1, P1, P2>(Bc, Dp, plane_words, H, W1, dummy, pass);
}

// ---------------------------------------------------------------------------
// WTA: one block per image row.  S'' = 8 C' + A_down + A_up + d_LR + d_RL (7
// bits; DESIGN.md §4b: same argmin and ties as S, exact minimum n (m - P2) +
// min S''), argmin with the smallest d on ties (MODE_HH), S''(best -+ 1) read
// off the bit planes, C(best -+ 1) gathered where the residual may be clamped,
// parabola, right-view keys (order-independent atomicMin), then the row's LR
// check (the final loop of OpenCV 3.4).
// ---------------------------------------------------------------------------
// The WTA's per-pixel tail (both WTA forms and bsgm_rl_final_kernel): exact
// S(best -+ 1) from S'' and, where the residual may be clamped, the C gathers;
// the parabola, the raw map, the right-view key.  best / mins / Sm / Sp: argmin,
// minimum S'' and S''(best -+ 1) of pixel pix (cost column x of its row).
// ndir = 8 (MODE_HH) or 5 (MODE_SGBM) directions: S = n (C - P2) + sum of deltas
__device__ __forceinline__ void bs_finish_pixel(const int16_t* __restrict__ C, const uint16_t* __restrict__ Mv,
                                                size_t pix, int W1, int W, int x, int best, int mins, int Sm,
                                                int Sp, const SgbmEff& e, int16_t* orow, uint32_t* krow)
{
    const int D = e.D;
    const int ndir = e.fullDP ? 8 : 5;
    const int clampS = ndir * 2 * e.P2;  // S'' >= this: C'' may be the clamp value
    const int mC = Mv[pix];
    const int base = ndir * (mC - e.P2);  // S = min(base + S', MAX_COST)
    const int bm = max(best - 1, 0), bp = min(best + 1, D - 1);
    const bool need = Sm >= clampS || Sp >= clampS;
    // C is stored [frame][y][x / 4][d][x % 4] on this pipeline (the cost
    // kernel's bit-sliced mode, rows padded to 4 pixels)
    const int prow = (int)(pix / W1), px = (int)(pix - (size_t)prow * W1);
    const size_t cbase = ((size_t)prow * ((W1 + 3) & ~3) + (px & ~3)) * D + (px & 3);
    auto cword = [&](int d) -> int { return need ? (int)(uint16_t)C[cbase + d * 4] : 0; };
    auto exact = [&](int Spp, int cv) -> int {
        const int c1 = Spp >= clampS ? cv - mC : 0;
        return min(base + Spp + ndir * (c1 - min(c1, 2 * e.P2)), kMaxCost);
    };
    const int minS = min(base + mins, kMaxCost);
    const int Smx = exact(Sm, cword(bm)), Spx = exact(Sp, cword(bp));
    int bst = best;
    if (minS >= kMaxCost) bst = -1;  // no strict minimum below MAX_COST
    const int den = max(Smx + Spx - 2 * minS, 1);
    const int frac = ((Smx - Spx) * kDispScale + den) / (den * 2);
    const int d16 = bst * kDispScale + (frac & -(int)(0 < bst && bst < D - 1));
    orow[x + e.minX1] = (int16_t)(d16 + e.minD * kDispScale);
    const int x2 = x + e.minX1 - bst - e.minD;
    if (minS < kMaxCost && x2 >= 0 && x2 < W)
        atomicMin(krow + x2, ((uint32_t)minS << 16) | (uint32_t)(0xffff - x));
}

// left-right check of a finished row (OpenCV 3.4 final loop), nthreads threads
__device__ __forceinline__ void bs_lr_check_row(int16_t* orow, const uint32_t* krow, int W, const SgbmEff& e,
                                                int nthreads)
{
    const int INV = e.invalid, minX1 = e.minX1, minD = e.minD;
    for (int x = minX1 + threadIdx.x; x < e.maxX1; x += nthreads) {
        const int v = orow[x];
        if (v == INV) continue;
        const int dlo = v >> kDispShift, dhi = (v + kDispScale - 1) >> kDispShift;
        const int xl = x - dlo, xh = x - dhi;
        auto d2at = [&](int xx) -> int {
            const uint32_t kk = __hip_atomic_load(krow + xx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (kk == 0xffffffffu) return INV;
            const int xc = 0xffff - (int)(kk & 0xffffu);
            return xc + minX1 - xx;
        };
        if (0 <= xl && xl < W && 0 <= xh && xh < W) {
            const int a = d2at(xl), b = d2at(xh);
            if (a >= minD && abs(a - dlo) > e.disp12 && b >= minD && abs(b - dhi) > e.disp12)
                orow[x] = (int16_t)INV;
        }
    }
}

constexpr int kBsWtaThreads = 512;

// NDIR = 8 (MODE_HH) / 5 (MODE_SGBM: the down pass's three directions and the
// two row directions).  SIDE: NDIR grouped delta planes (the side-by-side
// directions, then the two row directions); otherwise the strip passes' 4-bit
// planes (NDIR / 4 of them) and the two line planes.
template <bool SIDE, int NDIR>
__global__ __launch_bounds__(kBsWtaThreads) void bsgm_wta_kernel(const uint32_t* __restrict__ Bc,
                                                                 const uint32_t* __restrict__ A, size_t aplane,
                                                                 const uint32_t* __restrict__ Dl, size_t dplane,
                                                                 const int16_t* __restrict__ C,
                                                                 const uint16_t* __restrict__ Mv, int H, int W,
                                                                 SgbmEff e, int16_t* __restrict__ raw,
                                                                 uint32_t* __restrict__ keys)
{
    static_assert(NDIR == 8 || NDIR == 5, "8 or 5 directions");
    const int y = blockIdx.x, f = blockIdx.y;
    const int W1 = e.W1;
    const int INV = e.invalid;
    const bool lane_rule = NDIR == 5 && !(e.variant & MVSV_VARIANT_WTA_MIN_D);
    int16_t* orow = raw + ((size_t)f * H + y) * W;
    uint32_t* krow = keys + ((size_t)f * H + y) * W;
    for (int x = threadIdx.x; x < W; x += kBsWtaThreads) {
        orow[x] = (int16_t)INV;
        krow[x] = 0xffffffffu;
    }
    __threadfence_block();
    __syncthreads();
    const int h = threadIdx.x & 1;
    const size_t pix0 = ((size_t)f * H + y) * W1;
    for (int xb = 0; xb < W1; xb += kBsWtaThreads / 2) {
        const int xr = xb + (threadIdx.x >> 1);
        const bool own = xr < W1;
        const int x = min(xr, W1 - 1);
        const size_t pix = pix0 + x;
        uint32_t c[2][4];
        uint32_t S[2][7];
        const size_t rowq = (size_t)(f * H + y) * bs::padq(W1);
        const uint32_t* qc = Bc + bs::cq_word(rowq, x, 2 * h);
        if constexpr (SIDE) {
            // NDIR grouped delta planes: S'' = NDIR C' + the deltas
#pragma unroll
            for (int e2 = 0; e2 < 2; e2++) {
                const uint4 t = *(const uint4*)(qc + 16 * e2);
                c[e2][0] = t.x, c[e2][1] = t.y, c[e2][2] = t.z, c[e2][3] = t.w;
                uint32_t dd[NDIR][3];
#pragma unroll
                for (int i = 0; i < NDIR; i++) {
                    const uint32_t* qd = Dl + (size_t)i * dplane + bs::dl_word(rowq, x, 2 * h + e2);
#pragma unroll
                    for (int b = 0; b < 3; b++) dd[i][b] = qd[b];
                }
                uint32_t a4[4][4], a5[2][5], s6[6];
                bs::add33(dd[0], dd[1], a4[0]);
                bs::add33(dd[2], dd[3], a4[1]);
                bs::add44(a4[0], a4[1], a5[0]);  // <= 4 P2
                if constexpr (NDIR == 8) {
                    bs::add33(dd[4], dd[5], a4[2]);
                    bs::add33(dd[6], dd[7], a4[3]);
                    bs::add44(a4[2], a4[3], a5[1]);
                    bs::add55(a5[0], a5[1], s6);  // all deltas <= 8 P2 = 40
                    bs::total8(c[e2], s6, S[e2]);
                } else {
                    const uint32_t d4[4] = {dd[4][0], dd[4][1], dd[4][2], 0u};
                    bs::add54(a5[0], d4, s6);  // all deltas <= 5 P2 = 25 (bit 5 zero)
                    const uint32_t s5[5] = {s6[0], s6[1], s6[2], s6[3], s6[4]};
                    bs::total5(c[e2], s5, S[e2]);
                }
            }
        } else {
            // grouped C' and line planes (bs::cq_word / dl_word), E then O; the
            // strip planes per pixel (word h * 8 + e * 4 + b)
            const uint4* qd = (const uint4*)(A + pix * 16 + h * 8);
            const uint4* qu = (const uint4*)(A + aplane + pix * 16 + h * 8);
            const uint32_t* ql = Dl + bs::dl_word(rowq, x, 2 * h);
            const uint32_t* qr = Dl + dplane + bs::dl_word(rowq, x, 2 * h);
#pragma unroll
            for (int e2 = 0; e2 < 2; e2++) {
                uint4 t = *(const uint4*)(qc + 16 * e2);
                c[e2][0] = t.x, c[e2][1] = t.y, c[e2][2] = t.z, c[e2][3] = t.w;
                uint32_t ad[4], dl[3], dr[3];
                t = qd[e2];
                ad[0] = t.x, ad[1] = t.y, ad[2] = t.z, ad[3] = t.w;
#pragma unroll
                for (int b = 0; b < 3; b++) {
                    dl[b] = ql[12 * e2 + b];
                    dr[b] = qr[12 * e2 + b];
                }
                uint32_t d4[4];
                bs::add33(dl, dr, d4);  // lines <= 2 P2 = 10
                if constexpr (NDIR == 8) {
                    uint32_t au[4], s5[5], s6[6];
                    t = qu[e2];
                    au[0] = t.x, au[1] = t.y, au[2] = t.z, au[3] = t.w;
                    bs::add44(ad, au, s5);  // strips <= 2 * 3 P2 = 30
                    bs::add54(s5, d4, s6);  // all deltas <= 8 P2 = 40
                    bs::total8(c[e2], s6, S[e2]);
                } else {
                    uint32_t s5[5];
                    bs::add44(ad, d4, s5);  // all deltas <= 5 P2 = 25
                    bs::total5(c[e2], s5, S[e2]);
                }
            }
        }
        // argmin: the minimum is <= NDIR P2 (the d with C' = 0): < 64 (bit 6
        // zero) for 8 directions, < 32 (bits 5, 6 zero) for 5
        constexpr int TOP = NDIR == 8 ? 5 : 4;
        uint32_t kE = NDIR == 8 ? ~S[0][6] : ~(S[0][6] | S[0][5]);
        uint32_t kO = NDIR == 8 ? ~S[1][6] : ~(S[1][6] | S[1][5]);
        int mins = 0;
#pragma unroll
        for (int b = TOP; b >= 0; b--) {
            const uint32_t zE = bs::lop3<bs::kAndNotAB>(S[0][b], kE, kE);
            const uint32_t zO = bs::lop3<bs::kAndNotAB>(S[1][b], kO, kO);
            uint32_t any = zE | zO;
            any |= xswap(any);
            const bool fz = any != 0u;
            kE = fz ? zE : kE;
            kO = fz ? zO : kO;
            mins |= fz ? 0 : 1 << b;
        }
        // the tie rule among the minima (bs::wta_key): both parities of the
        // lane, then the partner lane
        int key = min(bs::wta_key(kE, h, 0, lane_rule), bs::wta_key(kO, h, 1, lane_rule));
        key = min(key, (int)xswap((uint32_t)key));
        const int best = key & 127;
        // S''(best -+ 1): both have the other parity; each lane reads its half
        const int eb = best & 1;
        int Sm = 0, Sp = 0;
        {
            const int pm = ((best - 1 - 64 * h) >> 1) & 31, pp = ((best + 1 - 64 * h) >> 1) & 31;
#pragma unroll
            for (int b = 0; b < 7; b++) {
                const uint32_t wv = eb ? S[0][b] : S[1][b];
                Sm |= (int)(__builtin_amdgcn_ubfe(wv, (uint32_t)pm, 1u) << b);
                Sp |= (int)(__builtin_amdgcn_ubfe(wv, (uint32_t)pp, 1u) << b);
            }
            const int Smo = (int)xswap((uint32_t)Sm), Spo = (int)xswap((uint32_t)Sp);
            if (((best - 1) >> 6) != h) Sm = Smo;
            if (((best + 1) >> 6) != h) Sp = Spo;
        }
        if (h == 0 && own) bs_finish_pixel(C, Mv, pix, W1, W, x, best, mins, Sm, Sp, e, orow, krow);
    }
    __threadfence_block();
    __syncthreads();
    bs_lr_check_row(orow, krow, W, e, kBsWtaThreads);
}

// ---------------------------------------------------------------------------
// R->L fused with the WTA (frame batches on the strip schedule): the R->L line
// direction's lane quads (bs_line_chains' layout) compute, right after each
// pixel's delta, S'' = 8 C' + A_down + A_up + d_LR + d_RL for their 32
// disparities, the argmin over the quad (bit-serial, smallest d), the minimum
// and S''(best -+ 1), and store one packed record per pixel (best | min << 8 |
// S''(best - 1) << 16 | S''(best + 1) << 24, grouped four pixels per 16-byte
// store); bsgm_rl_final_kernel finishes the pixels and the LR check.  Against
// lines + WTA this skips the R->L delta plane (written and read back) and the
// WTA's second read of C'.
// ---------------------------------------------------------------------------
constexpr int kBsRG = 3;  // groups (12 steps) of operands in the register ring

// NDIR = 8 (MODE_HH: both strip passes' planes) or 5 (MODE_SGBM: the down pass
// only); lane_rule: MODE_SGBM's lane tie rule (bs::wta_key)
template <int P1, int P2, int NDIR>
__global__ __launch_bounds__(64) void bsgm_rlwta_kernel(const uint32_t* __restrict__ Bc,
                                                         const uint32_t* __restrict__ A, size_t aplane,
                                                         const uint32_t* __restrict__ Dlr, int H, int W1,
                                                         uint32_t* __restrict__ rec, int lane_rule)
{
    static_assert(NDIR == 8 || NDIR == 5, "8 or 5 directions");
    const int lane = threadIdx.x;
    const int q = lane & 3, rr = lane >> 2;
    const int y = min((int)blockIdx.x * 16 + rr, H - 1);
    const int f = blockIdx.y;
    const int h = q >> 1, eo = q & 1;
    const bool odd = eo != 0;
    const uint32_t fill_hi = q == 3 ? kOnes : 0u, fill_lo = q == 0 ? kOnes : 0u, sh = odd ? 1u : 31u;
    const size_t rowq = (size_t)(f * H + y) * bs::padq(W1);
    const size_t pixrow = (size_t)(f * H + y) * W1;
    const uint4* cgrp = (const uint4*)(Bc + bs::cq_word(rowq, 0, q));
    const uint4* dgrp = (const uint4*)(Dlr + bs::dl_word(rowq, 0, q));
    const uint4* adn = (const uint4*)(A + pixrow * 16 + 4 * q);  // pixel x: + 4 x
    const uint4* aup = (const uint4*)(A + aplane + pixrow * 16 + 4 * q);
    uint4* rgrp = (uint4*)(rec + rowq);  // group g: + g
    const int G = (W1 + 3) >> 2;
    const int part = W1 & 3;
    // group of group step i (R->L, clamped: loads past the row are issued, not used)
    auto grp = [&](int i) { return max(G - 1 - i, 0); };
    struct Ops {
        uint4 c[4], d[3], a[4], b[4];
    };
    auto load = [&](Ops& o, int i) {
        const int g = grp(i);
#pragma unroll
        for (int u = 0; u < 4; u++) o.c[u] = cgrp[(size_t)g * 16 + u];
#pragma unroll
        for (int u = 0; u < 3; u++) o.d[u] = dgrp[(size_t)g * 12 + u];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int x = min(4 * g + u, W1 - 1);
            o.a[u] = adn[(size_t)x * 4];
            if constexpr (NDIR == 8) o.b[u] = aup[(size_t)x * 4];
        }
    };
    const int ph = part ? 1 : 0;
    Ops c0, ring[kBsRG];
    if (ph) load(c0, 0);
#pragma unroll
    for (int j = 0; j < kBsRG; j++) {
        load(ring[j], ph + j);
        __builtin_amdgcn_sched_barrier(0);
    }
    uint32_t st[3] = {0u, 0u, 0u};
    auto w4 = [](const uint4& v, int i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; };
    auto group = [&](int i, Ops& o, int n) {
        uint32_t rv[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int u = 3 - k;  // x = 4 g + u, descending
            if (u < n) {
                const uint32_t cw[4] = {o.c[u].x, o.c[u].y, o.c[u].z, o.c[u].w};
                uint32_t nw[3], dr[3];
                bs_quad_step<P1, P2>(st, cw, fill_hi, fill_lo, odd, sh, nw, dr);
#pragma unroll
                for (int b = 0; b < 3; b++) st[b] = nw[b];
                // S'' of this lane's 32 disparities
                const uint32_t ad[4] = {o.a[u].x, o.a[u].y, o.a[u].z, o.a[u].w};
                uint32_t dl[3];
#pragma unroll
                for (int b = 0; b < 3; b++) dl[b] = w4(o.d[(3 * u + b) >> 2], (3 * u + b) & 3);
                uint32_t d4[4], S[7];
                bs::add33(dl, dr, d4);  // lines <= 2 P2 = 10
                if constexpr (NDIR == 8) {
                    const uint32_t au[4] = {o.b[u].x, o.b[u].y, o.b[u].z, o.b[u].w};
                    uint32_t s5[5], s6[6];
                    bs::add44(ad, au, s5);  // strips <= 2 * 3 P2 = 30
                    bs::add54(s5, d4, s6);  // all deltas <= 8 P2 = 40
                    bs::total8(cw, s6, S);  // + 8 C'
                } else {
                    uint32_t s5[5];
                    bs::add44(ad, d4, s5);  // all deltas <= 5 P2 = 25
                    bs::total5(cw, s5, S);  // + 5 C'
                }
                // argmin over the quad: the minimum is <= NDIR P2, below 64 (8
                // directions: bit 6 zero) / 32 (5: bits 5 and 6 zero)
                constexpr int TOP = NDIR == 8 ? 5 : 4;
                uint32_t kk = NDIR == 8 ? ~S[6] : ~(S[6] | S[5]);
                int mins = 0;
#pragma unroll
                for (int b = TOP; b >= 0; b--) {
                    const uint32_t z = bs::lop3<bs::kAndNotAB>(S[b], kk, kk);
                    uint32_t any = z | xswap(z);
                    any |= (uint32_t)__builtin_amdgcn_mov_dpp((int)any, 0x4E, 0xf, 0xf, true);
                    const bool fz = any != 0u;
                    kk = fz ? z : kk;
                    mins |= fz ? 0 : 1 << b;
                }
                // the tie rule among the minima (bs::wta_key; d = 64 h + 2 p + e)
                int key = bs::wta_key(kk, h, eo, NDIR == 5 && lane_rule);
                key = min(key, (int)xswap((uint32_t)key));
                key = min(key, __builtin_amdgcn_mov_dpp(key, 0x4E, 0xf, 0xf, true));
                const int best = key & 127;
                // S''(best -+ 1) from the lane that holds it
                auto sat = [&](int d) -> uint32_t {
                    const int dq = 2 * ((d >> 6) & 1) + (d & 1), p = ((d & 63) >> 1);
                    uint32_t v = 0;
#pragma unroll
                    // one v_bfe + one v_lshl_or per bit
                    for (int b = 0; b < 7; b++) v |= __builtin_amdgcn_ubfe(S[b], (uint32_t)p, 1u) << b;
                    return dq == q ? v : 0u;
                };
                uint32_t sm = sat(best - 1) | (sat(best + 1) << 8);
                sm |= xswap(sm);
                sm |= (uint32_t)__builtin_amdgcn_mov_dpp((int)sm, 0x4E, 0xf, 0xf, true);
                rv[u] = (uint32_t)best | ((uint32_t)mins << 8) | (sm << 16);
            } else {
                rv[u] = 0u;
            }
        }
        // every lane of the quad stores the same record group (unpredicated)
        rgrp[grp(i)] = make_uint4(rv[0], rv[1], rv[2], rv[3]);
    };
    auto ringstep = [&](int i, int j, int n) {
        group(i, ring[j], n);
        load(ring[j], i + kBsRG);
        __builtin_amdgcn_sched_barrier(0);
    };
    if (ph) group(0, c0, part);
    int i = ph;
    for (; i + kBsRG <= G; i += kBsRG) {
#pragma unroll
        for (int j = 0; j < kBsRG; j++) ringstep(i + j, j, 4);
    }
#pragma unroll
    for (int j = 0; j < kBsRG; j++)
        if (i + j < G) ringstep(i + j, j, 4);
}

// the per-pixel tail and the LR check of rows computed by bsgm_rlwta_kernel
constexpr int kBsFinThreads = 256;
__global__ __launch_bounds__(kBsFinThreads) void bsgm_rl_final_kernel(const uint32_t* __restrict__ rec,
                                                                      const int16_t* __restrict__ C,
                                                                      const uint16_t* __restrict__ Mv, int H, int W,
                                                                      SgbmEff e, int16_t* __restrict__ raw,
                                                                      uint32_t* __restrict__ keys)
{
    const int y = blockIdx.x, f = blockIdx.y;
    const int W1 = e.W1;
    int16_t* orow = raw + ((size_t)f * H + y) * W;
    uint32_t* krow = keys + ((size_t)f * H + y) * W;
    for (int x = threadIdx.x; x < W; x += kBsFinThreads) {
        orow[x] = (int16_t)e.invalid;
        krow[x] = 0xffffffffu;
    }
    __threadfence_block();
    __syncthreads();
    const uint32_t* rrow = rec + (size_t)(f * H + y) * bs::padq(W1);
    const size_t pix0 = ((size_t)f * H + y) * W1;
    for (int x = threadIdx.x; x < W1; x += kBsFinThreads) {
        const uint32_t r = rrow[x];
        bs_finish_pixel(C, Mv, pix0 + x, W1, W, x, (int)(r & 0xffu), (int)((r >> 8) & 0xffu),
                        (int)((r >> 16) & 0xffu), (int)(r >> 24), e, orow, krow);
    }
    __threadfence_block();
    __syncthreads();
    bs_lr_check_row(orow, krow, W, e, kBsFinThreads);
}

// ---------------------------------------------------------------------------
// MODE_SGBM's cost-row quirks on the bit-sliced layouts (OpenCV 3.4, SURVEY
// Appendix A.3; the int16 form is sgbm_cost_fixup_*_kernel in mvsv_sgbm.hip):
// rows y >= ybot = H - SH2 are never recomputed and keep row ylast, and
// (without MVSV_VARIANT_FIRSTCOL_FIX) column 0 of every row y >= 1 keeps C(0, 0).
// A pixel's C' words, its pixel-quad C and its minimum m move together.  MODE_HH
// pins those cells to P2 inside the cost kernel instead.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void bsgm_fixup_bottom_kernel(uint32_t* __restrict__ Bc, int16_t* __restrict__ C,
                                                                uint16_t* __restrict__ Mv, int H, int W1, int ylast,
                                                                int ybot)
{
    const int y = ybot + blockIdx.y, f = blockIdx.z;
    const size_t W1q = (size_t)bs::padq(W1);
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t nb = W1q * 4, nc = W1q * 16;  // uint4 per row: C' (64 B / pixel), C (256 B / pixel)
    const size_t src = (size_t)f * H + ylast, dst = (size_t)f * H + y;
    if (i < nb) {
        ((uint4*)Bc)[dst * nb + i] = ((const uint4*)Bc)[src * nb + i];
    } else if (i < nb + nc) {
        const size_t j = i - nb;
        ((uint4*)C)[dst * nc + j] = ((const uint4*)C)[src * nc + j];
    }
    if (i < (size_t)W1) Mv[dst * W1 + i] = Mv[src * W1 + i];
}

// column 0 of rows 1 .. H - 1 <- pixel (0, 0) of the frame (D = 128)
__global__ __launch_bounds__(128) void bsgm_fixup_col0_kernel(uint32_t* __restrict__ Bc, int16_t* __restrict__ C,
                                                              uint16_t* __restrict__ Mv, int H, int W1)
{
    const int y = 1 + blockIdx.x, f = blockIdx.y;
    const size_t W1q = (size_t)bs::padq(W1);
    const size_t r0 = (size_t)f * H, r = r0 + y;
    const int t = threadIdx.x;
    if (t < 16) {
        // word (q, b) of pixel 0 in its group: q * 16 + b (bs::cq_word)
        const int o = (t >> 2) * 16 + (t & 3);
        Bc[bs::cq_word(r * W1q, 0, 0) + o] = Bc[bs::cq_word(r0 * W1q, 0, 0) + o];
    }
    // pixel-quad C: [row][x / 4][d][x % 4]
    C[(r * W1q) * 128 + t * 4] = C[(r0 * W1q) * 128 + t * 4];
    if (t == 0) Mv[r * W1] = Mv[r0 * W1];
}

}  // namespace

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
bool bsgm_eligible(const mvsv_ctx* ctx, const SgbmEff& e, int n, int H)
{
    const long bs = 2L * e.SW2 + 1;
    const bool no_wrap = (long)e.P2 + bs * bs * (2L * e.ftzero + 63) + e.P2 <= 32767;
    return ctx->bitslice && e.D == 128 && e.P1 == 2 && e.P2 == 5 && e.uniq == 0 && no_wrap &&
           e.W1 > 0 && (size_t)n * H * bs::padq(e.W1) * 16 < ((size_t)1 << 31);
}

size_t bsgm_plane_bytes(int n, int H, int W1) { return (size_t)n * H * bs::padq(W1) * 64; }

template <int NG>
static int launch_bs_strips(mvsv_ctx* ctx, int n, int H, const SgbmEff& e, const uint32_t* Bv, uint32_t* Av,
                            size_t aplane, uint32_t* dummy)
{
    using Cfg = BsStripCfg<NG>;
    const int npass = e.fullDP ? 2 : 1;  // MODE_SGBM: the down pass only
    const int nstrips = (e.W1 + H - 1 + Cfg::kSW - 1) / Cfg::kSW;
    const size_t bytes = (size_t)npass * n * nstrips * H * kBsGran * 8;
    int rc;
    if (ctx->bs_bnd.bytes < bytes) {
        if ((rc = ensure(ctx, ctx->bs_bnd, bytes, "bit-sliced strip boundary granules"))) return rc;
        // tag 0 (fresh memory) is never a launch epoch
        if ((rc = check_hip(ctx, hipMemsetAsync(ctx->bs_bnd.ptr, 0, ctx->bs_bnd.bytes, ctx->stream),
                            "bit-sliced boundary reset")))
            return rc;
    }
    if (!ctx->status.ptr) {
        if ((rc = ensure(ctx, ctx->status, 16, "device status words"))) return rc;
        if ((rc = check_hip(ctx, hipMemsetAsync(ctx->status.ptr, 0, 16, ctx->stream), "status reset"))) return rc;
        ctx->tri_tickets = 0;
    }
    // one epoch counter with the packed strip kernel: 32-bit tags here never repeat
    if ((++ctx->tri_epoch & 0xffffu) == 0) ++ctx->tri_epoch;
    const unsigned epoch = ctx->tri_epoch;
    const dim3 grid(nstrips * npass * n);
    const bool tickets = ctx->strip_tickets != 0;
    // MVSV_BS_STATS: per-strip spans and hand-off spin time on stderr
    // (diagnostics only: the buffer is cleared on the context stream, and any
    // failure turns the statistics off instead of touching a null buffer)
    unsigned long long* stats = nullptr;
    if (std::getenv("MVSV_BS_STATS")) {
        if (hipMalloc(&stats, (size_t)grid.x * 64) != hipSuccess) {
            (void)hipGetLastError();
            stats = nullptr;
        } else if (hipMemsetAsync(stats, 0, (size_t)grid.x * 64, ctx->stream) != hipSuccess) {
            (void)hipGetLastError();
            (void)hipFree(stats);
            stats = nullptr;
        }
    }
    // one strip block per CU: dynamic LDS past half the CU's 160 KiB (a second
    // strip block on the same CU makes that CU's strips, and every strip left of
    // them in the chain, step at half speed -- 2-group strips measured 1.17 ms
    // two to a CU, 0.88 ms one to a CU, 4-group strips 0.98 ms either way;
    // the lines / cost blocks of a concurrent batch still fit beside it).
    // MVSV_BS_LDSPAD overrides the size (A/B).
    size_t lds = std::max(Cfg::kBytes, (size_t)kBsStripLds);
    if (const char* pv = std::getenv("MVSV_BS_LDSPAD")) lds = std::max(Cfg::kBytes, (size_t)std::atol(pv));
    if (lds > 65536 &&
        (rc = check_hip(ctx, hipFuncSetAttribute((const void*)bsgm_strip_kernel<NG, 2, 5>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                        "bit-sliced strip LDS attribute")))
        return rc;
    hipLaunchKernelGGL((bsgm_strip_kernel<NG, 2, 5>), grid, dim3(Cfg::kThreads), lds, ctx->stream, Bv, Av,
                       aplane, dummy, H, e.W1, npass, (unsigned long long*)ctx->bs_bnd.ptr, epoch, n,
                       (int*)ctx->status.ptr, ctx->spin_limit, ctx->report_target,
                       tickets ? (long long)ctx->tri_tickets : -1ll, stats, 0);
    rc = check_hip(ctx, hipGetLastError(), "bit-sliced strip kernel");
    if (rc == MVSV_OK && tickets) ctx->tri_tickets += grid.x;
    if (stats) {
        std::vector<unsigned long long> hv((size_t)grid.x * 8);
        const bool ok = hipStreamSynchronize(ctx->stream) == hipSuccess &&
                        hipMemcpy(hv.data(), stats, hv.size() * 8, hipMemcpyDeviceToHost) == hipSuccess;
        (void)hipFree(stats);
        if (!ok) {
            (void)hipGetLastError();
            return rc;
        }
        unsigned long long t0 = ~0ull, t1 = 0, spin = 0, busy = 0, steps = 0;
        for (size_t b = 0; b < grid.x; b++) {
            const unsigned long long* q = &hv[b * 8];
            if (!q[1]) continue;
            t0 = std::min(t0, q[0]);
            t1 = std::max(t1, q[1]);
            spin += q[2];
            busy += q[1] - q[0];
            steps += q[4];
        }
        std::fprintf(stderr, "[bs] NG %d strips %d blocks %u span %llu ticks, block-ticks %llu, spin %.1f%%, ticks/step %.1f\n",
                     NG, nstrips, grid.x, t1 - t0, busy, 100.0 * spin / std::max(busy, 1ull),
                     (double)busy / std::max(steps, 1ull));
    }
    return rc;
}

// Small launches (path_schedule 2): all eight directions as independent
// lane-quad chains in one launch, eight delta planes, then the WTA over them.
static int bsgm_paths_side(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, const int16_t* Cv,
                           const uint32_t* Bv, const uint16_t* Mv, int16_t* raw)
{
    int rc;
    const int npass = e.fullDP ? 2 : 1, ndir = 3 * npass + 2;
    const size_t dplane = (size_t)n * H * bs::padq(e.W1) * 12;  // words per delta plane (grouped)
    // + 256 words: dummy store slots of cells outside the image
    if ((rc = ensure(ctx, ctx->agg, (ndir * dplane + 256) * 4, "bit-sliced delta planes"))) return rc;
    if ((rc = ensure(ctx, ctx->keys, (size_t)n * H * W * 4, "sgbm right-view keys"))) return rc;
    uint32_t* Dv = (uint32_t*)ctx->agg.ptr;
    hipStream_t s = ctx->stream;
    {
        StageTimer tm(ctx, kStagePath);
        hipLaunchKernelGGL((bsgm_dir_kernel<2, 5>), dim3((e.W1 + H - 1 + 15) / 16, n, ndir), dim3(64), 0, s, Bv,
                           Dv, dplane, H, e.W1, Dv + ndir * dplane, npass);
        if ((rc = check_hip(ctx, hipGetLastError(), "bit-sliced direction kernel"))) return rc;
    }
    StageTimer tm(ctx, kStageFinal);
    if (e.fullDP)
        hipLaunchKernelGGL((bsgm_wta_kernel<true, 8>), dim3(H, n), dim3(kBsWtaThreads), 0, s, Bv, nullptr, (size_t)0,
                           Dv, dplane, Cv, Mv, H, W, e, raw, (uint32_t*)ctx->keys.ptr);
    else
        hipLaunchKernelGGL((bsgm_wta_kernel<true, 5>), dim3(H, n), dim3(kBsWtaThreads), 0, s, Bv, nullptr, (size_t)0,
                           Dv, dplane, Cv, Mv, H, W, e, raw, (uint32_t*)ctx->keys.ptr);
    return check_hip(ctx, hipGetLastError(), "bit-sliced WTA kernel");
}

int bsgm_cost_fixup(mvsv_ctx* ctx, int n, int H, const SgbmEff& e, int16_t* Cv, uint32_t* Bv, uint16_t* Mv)
{
    if (e.fullDP || H <= 1) return MVSV_OK;  // MODE_HH: pinned inside the cost kernel
    hipStream_t s = ctx->stream;
    const int ybot = std::max(H - e.SH2, 1), ylast = std::max(H - e.SH2 - 1, 0);
    StageTimer tm(ctx, kStageFixup);
    if (ybot < H) {
        const size_t items = (size_t)bs::padq(e.W1) * 20;  // uint4 of C' and C per row
        hipLaunchKernelGGL(bsgm_fixup_bottom_kernel, dim3((unsigned)((items + 255) / 256), H - ybot, n), dim3(256),
                           0, s, Bv, Cv, Mv, H, e.W1, ylast, ybot);
    }
    // after the bottom rows: their column 0 is C(0, 0) too (unless FIRSTCOL_FIX)
    if (!(e.variant & MVSV_VARIANT_FIRSTCOL_FIX))
        hipLaunchKernelGGL(bsgm_fixup_col0_kernel, dim3(H - 1, n), dim3(128), 0, s, Bv, Cv, Mv, H, e.W1);
    return check_hip(ctx, hipGetLastError(), "bit-sliced cost fixup");
}

int bsgm_paths(mvsv_ctx* ctx, int n, int H, int W, const SgbmEff& e, const int16_t* Cv, const uint32_t* Bv,
               const uint16_t* Mv, int16_t* raw, bool side)
{
    int rc;
    if (side) return bsgm_paths_side(ctx, n, H, W, e, Cv, Bv, Mv, raw);
    const int npass = e.fullDP ? 2 : 1;  // strip passes (MODE_SGBM: down only)
    const size_t aplane = (size_t)n * H * e.W1 * 16;  // words per strip-pass plane
    const size_t dplane = (size_t)n * H * bs::padq(e.W1) * 12;  // words per line plane (grouped, padded rows)
    // + 512 words: the strip kernel's dummy store slots (cells outside the image)
    if ((rc = ensure(ctx, ctx->agg, (npass * aplane + 2 * dplane + 512) * 4, "bit-sliced delta planes")))
        return rc;
    if ((rc = ensure(ctx, ctx->keys, (size_t)n * H * W * 4, "sgbm right-view keys"))) return rc;
    uint32_t* Av = (uint32_t*)ctx->agg.ptr;
    uint32_t* Dv = Av + npass * aplane;
    hipStream_t s = ctx->stream;
    if (!ctx->aux) {
        if ((rc = check_hip(ctx, hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking), "aux stream")) ||
            (rc = check_hip(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming), "event")) ||
            (rc = check_hip(ctx, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming), "event")))
            return rc;
    }
    {
        StageTimer tm(ctx, kStagePath);
        // the row directions beside the strips on the aux stream (the strip
        // chain leaves CUs idle while it fills and drains, the line waves are
        // few and memory-bound): bench 2970 vs 2850 Mpix/s with the lines after
        // the strips on the context stream (MVSV_BS_SERIAL=1, same box, with
        // one-block-per-CU 2-group strips and the grouped planes)
        const bool side = !ctx->bs_serial;
        if (side && ((rc = check_hip(ctx, hipEventRecord(ctx->ev_fork, s), "fork")) ||
                     (rc = check_hip(ctx, hipStreamWaitEvent(ctx->aux, ctx->ev_fork, 0), "fork wait"))))
            return rc;
        hipStream_t ls = side ? ctx->aux : s;
        // fused: only L->R here, R->L runs with the WTA (bsgm_rlwta_kernel)
        const bool fuse = ctx->bs_fuse != 0;
        auto lines = [&]() -> int {
            StageTimer tl(ctx, kStageLines, ls);
            hipLaunchKernelGGL((bsgm_lines4_kernel<2, 5>), dim3((H + 15) / 16, n, fuse ? 1 : 2), dim3(64), 0, ls,
                               Bv, Dv, dplane, H, e.W1);
            return check_hip(ctx, hipGetLastError(), "bit-sliced line kernel");
        };
        if (side && (rc = lines())) return rc;
        {
            StageTimer ts(ctx, kStageStrips);
            // 3 column groups (96 U-columns, 10 waves) for MODE_HH batches: 352
            // strip blocks per 8-frame batch instead of 528 overlap better with
            // the other batch in flight (bench 3114-3120 -> 3164-3169 Mpix/s,
            // same box, r06n; one batch alone: strips 1.14 -> 1.15 ms); 4 groups
            // leave no room for the line waves beside them (lines 0.55 -> 2.0 ms)
            const int ng = ctx->bs_groups ? ctx->bs_groups : (e.fullDP ? 3 : 2);
            uint32_t* dummy = Dv + 2 * dplane;
            rc = ng == 1   ? launch_bs_strips<1>(ctx, n, H, e, Bv, Av, aplane, dummy)
                 : ng == 3 ? launch_bs_strips<3>(ctx, n, H, e, Bv, Av, aplane, dummy)
                 : ng == 4 ? launch_bs_strips<4>(ctx, n, H, e, Bv, Av, aplane, dummy)
                 : ng == 5 ? launch_bs_strips<5>(ctx, n, H, e, Bv, Av, aplane, dummy)
                           : launch_bs_strips<2>(ctx, n, H, e, Bv, Av, aplane, dummy);
            if (rc) return rc;
        }
        if (!side && (rc = lines())) return rc;
        if (side && ((rc = check_hip(ctx, hipEventRecord(ctx->ev_join, ctx->aux), "join")) ||
                     (rc = check_hip(ctx, hipStreamWaitEvent(s, ctx->ev_join, 0), "join wait"))))
            return rc;
    }
    StageTimer tm(ctx, kStageFinal);
    if (ctx->bs_fuse) {
        // per-pixel records in the (unused) R->L plane's space
        uint32_t* rec = Dv + dplane;
        const int lane_rule = !(e.variant & MVSV_VARIANT_WTA_MIN_D);
        if (e.fullDP)
            hipLaunchKernelGGL((bsgm_rlwta_kernel<2, 5, 8>), dim3((H + 15) / 16, n), dim3(64), 0, s, Bv, Av, aplane,
                               Dv, H, e.W1, rec, lane_rule);
        else
            hipLaunchKernelGGL((bsgm_rlwta_kernel<2, 5, 5>), dim3((H + 15) / 16, n), dim3(64), 0, s, Bv, Av, aplane,
                               Dv, H, e.W1, rec, lane_rule);
        if ((rc = check_hip(ctx, hipGetLastError(), "bit-sliced R->L + WTA kernel"))) return rc;
        hipLaunchKernelGGL(bsgm_rl_final_kernel, dim3(H, n), dim3(kBsFinThreads), 0, s, rec, Cv, Mv, H, W, e, raw,
                           (uint32_t*)ctx->keys.ptr);
        return check_hip(ctx, hipGetLastError(), "bit-sliced final kernel");
    }
    if (e.fullDP)
        hipLaunchKernelGGL((bsgm_wta_kernel<false, 8>), dim3(H, n), dim3(kBsWtaThreads), 0, s, Bv, Av, aplane, Dv,
                           dplane, Cv, Mv, H, W, e, raw, (uint32_t*)ctx->keys.ptr);
    else
        hipLaunchKernelGGL((bsgm_wta_kernel<false, 5>), dim3(H, n), dim3(kBsWtaThreads), 0, s, Bv, Av, aplane, Dv,
                           dplane, Cv, Mv, H, W, e, raw, (uint32_t*)ctx->keys.ptr);
    return check_hip(ctx, hipGetLastError(), "bit-sliced WTA kernel");
}

}  // namespace mvsv
