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

template <typename SadT>
__global__ __launch_bounds__(256) void bm_match_kernel(const uint8_t* __restrict__ Lf,
                                                       const uint8_t* __restrict__ Rf, int W,
                                                       int H, BmEff e, int keep_border,
                                                       int16_t* __restrict__ out, size_t os,
                                                       size_t ofs, int* __restrict__ cost)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int nd = e.ndisp, w2 = e.wsz2, win = 2 * w2 + 1;
    const BmLayout lay = bm_layout(nd, w2, (int)sizeof(SadT));
    uint8_t* Lt = smem;
    uint8_t* Rt = smem + lay.off_r;
    uint32_t* V = (uint32_t*)(smem + lay.off_v);
    SadT* sadbuf = (SadT*)(smem + lay.off_sad);
    const int NJ = lay.NJ, NRW = lay.NRW, NRC = lay.NRC;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int f = blockIdx.z;
    const int xl0 = blockIdx.x * 16;
    const int yr0 = e.ymin + blockIdx.y * 16;
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
    if ((rc = ensure(ctx, ctx->bm_lf, (size_t)n * plane, "bm left prefilter"))) return rc;
    if ((rc = ensure(ctx, ctx->bm_rf, (size_t)n * plane, "bm right prefilter"))) return rc;
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
    const bool small = (long long)win * win * 2 * e.cap <= 65535;
    BmLayout lay = bm_layout(e.ndisp, e.wsz2, small ? 2 : 4);
    if (lay.bytes > 160 * 1024)
        return set_error(ctx, MVSV_E_INVALID_ARG,
                         "numDisparities x blockSize too large for the GPU BM kernel");
    dim3 grid((e.ncol + 15) / 16, (e.ymax - e.ymin + 15) / 16, n);
    if (lay.bytes > 65536) {
        const void* fn = small ? (const void*)bm_match_kernel<uint16_t>
                               : (const void*)bm_match_kernel<uint32_t>;
        if ((rc = check_hip(ctx, hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)lay.bytes),
                            "bm LDS attribute")))
            return rc;
    }
    StageTimer tm(ctx, kStageBm);
    if (small)
        hipLaunchKernelGGL(bm_match_kernel<uint16_t>, grid, dim3(256), lay.bytes, s, Lf, Rf, W, H,
                           e, validate ? 1 : 0, out, os, ofs, cost);
    else
        hipLaunchKernelGGL(bm_match_kernel<uint32_t>, grid, dim3(256), lay.bytes, s, Lf, Rf, W, H,
                           e, validate ? 1 : 0, out, os, ofs, cost);
    if ((rc = check_hip(ctx, hipGetLastError(), "bm match"))) return rc;
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
