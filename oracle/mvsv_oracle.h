/*
 * mvsv_oracle.h — CPU restatement of the stereo-disparity hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (libmvsv, the
 * mvstereovision3_amd package) may link, load or call this code.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it,
 * and only as the checker / the timed CPU baseline.
 *
 * What it restates.  The reference (hG3n/mvStereoVision3) computes disparity
 * exclusively through OpenCV:
 *   Disparity::sgbm  src/disparity.cpp:6-10   -> cv::StereoSGBM::compute
 *   Disparity::bm    src/disparity.cpp:18-22  -> cv::StereoBM::compute
 *   Disparity::loadSGBMParameters src/disparity.cpp:60-108 (parameter mapping)
 * OpenCV is a third-party dependency that is NOT under /root/reference and
 * NOT installed in this image.  The pinned semantics are
 * OpenCV 3.4.x, x86-64 build with the CV_SIMD128 (SSE2) code paths, restated
 * from its published algorithm (calib3d/src/stereosgbm.cpp, stereobm.cpp,
 * imgproc/src/median_blur.cpp).  No golden vectors exist for this path in
 * the reference, so parity is UNPINNED: this oracle is cross-checked against
 * an independent numpy restatement (oracle/twin.py) instead.
 *
 * Two behaviours changed between OpenCV releases; they are switchable so the
 * oracle can be re-pinned if a real OpenCV ever becomes available:
 *   ORC_F_FIRSTCOL_FIX  C(x=0) of rows y>0 is updated (later releases); the
 *                       3.4 code leaves it at its row-0 value (MODE_SGBM) or
 *                       at the P2 pre-fill (MODE_HH).
 *   ORC_F_WTA_MIN_D     MODE_SGBM winner-take-all picks the smallest d among
 *                       ties (later releases); 3.4's SSE2 path picks the
 *                       lowest SIMD lane (d mod 8) among ties.
 * Default (flags = 0) is OpenCV 3.4 behaviour.
 */
#ifndef MVSV_ORACLE_H
#define MVSV_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_F_FIRSTCOL_FIX 1u
#define ORC_F_WTA_MIN_D    2u

/* Raw OpenCV StereoSGBM parameters (cv::StereoSGBM::create argument order). */
typedef struct {
    int min_disparity, num_disparities, block_size, p1, p2, disp12_max_diff,
        pre_filter_cap, uniqueness_ratio, speckle_window_size, speckle_range,
        mode; /* 0 = MODE_SGBM (5 paths), 1 = MODE_HH (8 paths) */
} orc_sgbm_params;

/* Raw OpenCV StereoBM parameters (defaults of StereoBM::create(D, bs)). */
typedef struct {
    int pre_filter_type; /* 0 = NORMALIZED_RESPONSE, 1 = XSOBEL */
    int pre_filter_size, pre_filter_cap, block_size, min_disparity,
        num_disparities, texture_threshold, uniqueness_ratio,
        speckle_window_size, speckle_range, disp12_max_diff;
} orc_bm_params;

/* Full StereoSGBM::compute: core + medianBlur(3) + filterSpeckles.
 * Returns 0 on success, <0 on invalid arguments. */
int orc_sgbm_compute(const uint8_t* L, ptrdiff_t lstride, const uint8_t* R,
                     ptrdiff_t rstride, int W, int H, const orc_sgbm_params* p,
                     unsigned flags, int16_t* out, ptrdiff_t ostride);

/* computeDisparitySGBM only (before the median / speckle post-filters). */
int orc_sgbm_core(const uint8_t* L, ptrdiff_t lstride, const uint8_t* R,
                  ptrdiff_t rstride, int W, int H, const orc_sgbm_params* p,
                  unsigned flags, int16_t* out, ptrdiff_t ostride);

/* Cost volume C (including the +P2 bias and the row/column quirks) of
 * computeDisparitySGBM, layout [H][W1][D] int16. Returns W1 (>0) or <=0. */
int orc_sgbm_cost_volume(const uint8_t* L, ptrdiff_t lstride, const uint8_t* R,
                         ptrdiff_t rstride, int W, int H,
                         const orc_sgbm_params* p, unsigned flags, int16_t* C);

/* Full StereoBM::compute with a CV_16S output. */
int orc_bm_compute(const uint8_t* L, ptrdiff_t lstride, const uint8_t* R,
                   ptrdiff_t rstride, int W, int H, const orc_bm_params* p,
                   int16_t* out, ptrdiff_t ostride);

/* StereoBM's prefilterXSobel (dst is W*H u8, contiguous). */
void orc_prefilter_xsobel(const uint8_t* src, ptrdiff_t sstride, int W, int H,
                          int ftzero, uint8_t* dst);

/* medianBlur(src, dst, 3) for CV_16S, replicate border. dst may equal src. */
void orc_median3x3_s16(const int16_t* src, ptrdiff_t sstride, int W, int H,
                       int16_t* dst, ptrdiff_t dstride);

/* filterSpeckles for CV_16S (in place). */
int orc_filter_speckles_s16(int16_t* img, ptrdiff_t stride, int W, int H,
                            int new_val, int max_speckle_size, int max_diff);

/* MeanDisparityDetection::build(MEAN_VALUE) post-pass: 81 tile means over a
 * CV_16S map (src/MeanDisparityDetection.cpp:159-206, Utility::
 * calcMeanDisparity src/utility.cpp:265-285). means[81] row-major tiles. */
/* cv::remap(src, dst, mapx, mapy, INTER_LINEAR, BORDER_CONSTANT, 0), CV_8UC1 with
 * CV_32FC1 maps (OpenCV 3.4 RemapInvoker map conversion + remapBilinear).
 * dst is dw x dh (stride dw), maps dw x dh (stride dw). */
void orc_remap_linear(const uint8_t* src, ptrdiff_t sstride, int sw, int sh, const float* mapx,
                      const float* mapy, uint8_t* dst, int dw, int dh);

/* Utility::calcCoordinate (src/utility.cpp:176-198) for every pixel:
 * out[y][x] = (X, Y, Z, v > 0), Q 4x4 CV_32F row-major.  OpenCV float Mat
 * product (double accumulation over k = 0..3, one rounding), then Mat /= W
 * (convertTo with float alpha = 1 / W), Z = 0 when Z / 1000 is infinite. */
void orc_reproject(const int16_t* dmap, ptrdiff_t stride, int W, int H, const float* Q,
                   float* out);

void orc_mean_disparity_grid(const int16_t* dmap, ptrdiff_t stride, int W,
                             int H, float* means);

/* cv::resize(src, dst, Size(0, 0), fx, fy, INTER_LINEAR), CV_8UC1 (OpenCV 3.4,
 * see mvsv_oracle.c): writes the output size to *out_w / *out_h and, when dst
 * is not NULL, the resized image (row stride ds). */
void orc_resize_linear(const uint8_t* src, ptrdiff_t ss, int sw, int sh, double fx, double fy,
                       uint8_t* dst, ptrdiff_t ds, int* out_w, int* out_h);

#ifdef __cplusplus
}
#endif
#endif
