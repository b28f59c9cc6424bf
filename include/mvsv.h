/*
 * mvsv.h — C ABI of the MI355X-native stereo disparity engine (libmvsv.so).
 *
 * This is the drop-in boundary for the reference's disparity hot path.  Every
 * entry point replaces one reference interface (hG3n/mvStereoVision3):
 *
 *   mvsv_sgbm / mvsv_sgbm_device      Disparity::sgbm        src/disparity.cpp:6-10,
 *                                     decl inc/disparity.h:29 (forwards to
 *                                     cv::StereoSGBM::compute, also called
 *                                     directly at trgt/liveDisparity.cpp:91)
 *   mvsv_bm / mvsv_bm_device          Disparity::bm          src/disparity.cpp:18-22,
 *                                     decl inc/disparity.h:31
 *   mvsv_load_sgbm_yaml               Disparity::loadSGBMParameters
 *                                     src/disparity.cpp:60-108, inc/disparity.h:34
 *   mvsv_load_bm_yaml                 (new) loader for configs/bm.yml:2-7, which
 *                                     the reference ships but never reads
 *   mvsv_sgbm_params / mvsv_bm_params cv::StereoSGBM / cv::StereoBM state set by
 *                                     create() + setters (src/disparity.cpp:83-95,
 *                                     trgt/liveDisparity.cpp:61); field meaning and
 *                                     defaults are OpenCV 3.4's
 *   mvsv_sgbm_yaml_values             struct Disparity::sgbmParameters
 *                                     inc/disparity.h:17-27
 *   mvsv_mean_disparity_grid_device   MeanDisparityDetection::build(MEAN_VALUE)
 *                                     src/MeanDisparityDetection.cpp:159-206 +
 *                                     Utility::calcMeanDisparity src/utility.cpp:265-285
 *   mvsv_mean_disparity_grid          same, host map (MeanDisparityDetection::build)
 *   mvsv_stream_*                     the disparity worker thread + main loop of
 *                                     trgt/mean_test.cpp:61-70,258-318 (condvar
 *                                     hand-off, Disparity::sgbm, build(MEAN_VALUE))
 *                                     as a double-buffered device pipeline
 *   mvsv_remap_device / mvsv_rectify  cv::remap(INTER_LINEAR) + ROI crop of
 *                                     Stereosystem::getRectifiedImagepair
 *                                     src/Stereosystem.cpp:243-262
 *   mvsv_init_undistort_rectify_map   cv::initUndistortRectifyMap (CV_32FC1) as
 *                                     called by Stereosystem::initRectification
 *                                     src/Stereosystem.cpp:193-237
 *   mvsv_reproject_device             Utility::calcCoordinate src/utility.cpp:176-198,
 *                                     per pixel (the loop of Utility::dmap2pcl :242-262)
 *   mvsv_calc_coordinate(s) / _distance  Utility::calcCoordinate / calcDistance
 *   / _dmap_values                    src/utility.cpp:176-240 (host, one point)
 *   mvsv_write_ply                    ply::write src/ply.cpp:37-133 (MODE PLAIN,
 *                                     WITH_COLOR, WITH_COLOR_SHADING)
 *   mvsv_dmap2pcl                     Utility::dmap2pcl src/utility.cpp:242-262
 *
 * Conventions
 *   - Plain C types only; no exceptions cross this boundary.
 *   - Every function returns MVSV_OK (0) or a negative MVSV_E_* code; the
 *     context's message is available through mvsv_last_error().
 *   - Parameter validation follows OpenCV's CV_Assert/CV_Error rules for the
 *     same call (invalid -> MVSV_E_INVALID_ARG instead of cv::Exception).
 *   - Output is CV_16S-compatible: int16 disparity * 16 (DISP_SHIFT = 4);
 *     invalid pixels are (minDisparity - 1) * 16.
 *   - A context owns one HIP stream and its cached device buffers; it is not
 *     thread-safe: use one context per host thread (the reference runs one
 *     matcher per worker thread, trgt/mean_test.cpp:61-70).
 *   - Host-pointer calls (mvsv_sgbm, mvsv_bm) are synchronous.  Device-pointer
 *     calls (*_device) enqueue on the context stream and return immediately;
 *     call mvsv_synchronize() before reading results on the host.
 */
#ifndef MVSV_H
#define MVSV_H

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define MVSV_API __attribute__((visibility("default")))
#else
#define MVSV_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define MVSV_VERSION 100 /* 1.0.0 */

enum {
    MVSV_OK = 0,
    MVSV_E_INVALID_ARG = -1, /* OpenCV would throw cv::Exception (StsOutOfRange / assert) */
    MVSV_E_HIP = -2,         /* HIP runtime error (launch, copy, device) */
    MVSV_E_OOM = -3,         /* device or host allocation failed */
    MVSV_E_IO = -4,          /* cannot open file */
    MVSV_E_PARSE = -5,       /* missing / malformed YAML key */
    MVSV_E_NODEV = -6,       /* no HIP device available */
    MVSV_E_TIMEOUT = -7      /* a strip-to-strip hand-off of the SGBM path kernel was
                                given up: the affected maps are all INVALID */
};

/* Context options (mvsv_set_option). */
enum {
    /* polls a strip-boundary wait of the SGBM path kernel makes before it gives
     * up (default 1 << 20, ~1 s); 0 gives up at the first poll that finds the
     * producer's data not yet written (fault injection for tests) */
    MVSV_OPT_STRIP_SPIN_LIMIT = 1,
    /* rows per block of the StereoBM disparities-on-lanes kernel (0 = chosen
     * per launch from the shape; 1..128 forces it -- tests, A/B runs) */
    MVSV_OPT_BM_TILE_ROWS = 2,
    /* compute waves per strip of the SGBM sheared-strip kernel: 0 = by launch
     * size (narrow strips when the wide ones would leave CUs idle), 8 (4 for
     * numDisparities > 128) = narrow, 15 (7) = wide; other values = 0 */
    MVSV_OPT_STRIP_WAVES = 3,
    /* SGBM path schedule (numDisparities 32 / 64 / 128 / 256): 0 = by launch
     * size -- all line directions side by side for launches that would fill
     * at most half the GPU with sheared strips (one camera frame; needs
     * P2 <= 15),
     * sheared strips otherwise; 1 = strips; 2 = directions side by side */
    MVSV_OPT_PATH_SCHEDULE = 4,
    /* which strip a block of the sheared-strip kernel runs: 1 (default) = a
     * ticket drawn on arrival, so a strip only waits on a strip already
     * running or done whatever the dispatch order and whatever else shares
     * the GPU (every launch size); 0 = its blockIdx (relies on in-order
     * dispatch, A/B runs only). */
    MVSV_OPT_STRIP_TICKETS = 5,
    /* SGBM direction passes read the cost residual plane
     * R = min(C - min_d C, 2*P2) + P2 (one nibble per cost, 4x fewer bytes
     * than C) instead of C where that is exact: no int16 wrap is possible,
     * 3*P2 <= 15 and numDisparities <= 128 (configs/sgbm.yml).  1 (default)
     * = on, 0 = always read C (A/B runs); results are identical either way. */
    MVSV_OPT_COST_RESIDUAL = 6,
    /* Bit-sliced MODE_HH path aggregation (round 5, mvsv_bsgm.hip): 1 (default)
     * = where it applies (MODE_HH, numDisparities 128, P1 2 / P2 5 -- the
     * sgbm.yml regime --, uniquenessRatio 0, no int16 wrap); 0 = the packed
     * int16 kernels.  Results are identical either way. */
    MVSV_OPT_BITSLICE = 7
};

/* StereoSGBM modes (cv::StereoSGBM::MODE_SGBM / MODE_HH). */
enum { MVSV_MODE_SGBM = 0, MVSV_MODE_HH = 1 };
/* StereoBM prefilter types (cv::StereoBM::PREFILTER_*). */
enum { MVSV_PREFILTER_NORMALIZED_RESPONSE = 0, MVSV_PREFILTER_XSOBEL = 1 };

/* Semantic variants of OpenCV releases (bit flags in mvsv_sgbm_params.variant).
 * 0 = OpenCV 3.4.x CV_SIMD128 behaviour (the pinned default). */
enum {
    MVSV_VARIANT_FIRSTCOL_FIX = 1, /* later releases refresh cost column x=0 */
    MVSV_VARIANT_WTA_MIN_D = 2     /* later releases: MODE_SGBM ties -> smallest d */
};

typedef struct {
    int min_disparity;       /* setMinDisparity */
    int num_disparities;     /* setNumDisparities, must be > 0 and % 16 == 0 */
    int block_size;          /* setBlockSize (<= 0 -> 5) */
    int p1, p2;              /* setP1 / setP2 (<= 0 -> 2 / 5, P2 = max(P2, P1+1)) */
    int disp12_max_diff;     /* setDisp12MaxDiff (<= 0 -> 1) */
    int pre_filter_cap;      /* setPreFilterCap (ftzero = max(cap,15)|1) */
    int uniqueness_ratio;    /* setUniquenessRatio (< 0 -> 10) */
    int speckle_window_size; /* setSpeckleWindowSize (0 disables speckle filter) */
    int speckle_range;       /* setSpeckleRange (multiplied by 16) */
    int mode;                /* MVSV_MODE_SGBM (5 paths) or MVSV_MODE_HH (8 paths) */
    int variant;             /* MVSV_VARIANT_* bits, 0 = OpenCV 3.4 */
} mvsv_sgbm_params;

typedef struct {
    int pre_filter_type;     /* MVSV_PREFILTER_XSOBEL (default) or _NORMALIZED_RESPONSE */
    int pre_filter_size;     /* odd, 5..255 */
    int pre_filter_cap;      /* 1..63 */
    int block_size;          /* odd, 5..255, < min(W, H) */
    int min_disparity;
    int num_disparities;     /* > 0, % 16 == 0 */
    int texture_threshold;   /* >= 0 */
    int uniqueness_ratio;    /* >= 0 */
    int speckle_window_size;
    int speckle_range;
    int disp12_max_diff;     /* < 0 disables the left-right check */
} mvsv_bm_params;

/* Disparity::sgbmParameters (inc/disparity.h:17-27): the raw YAML values. */
typedef struct {
    int minDisp, numDisp, blockSize, disp12MaxDiff, preFilterCap, uniquenessRatio,
        speckleWindowSize, speckleRange, disparityMode;
} mvsv_sgbm_yaml_values;

typedef struct mvsv_ctx mvsv_ctx;

MVSV_API int mvsv_version(void);

/* StereoSGBM::create() defaults: (0, 16, 3, 0, 0, 0, 0, 0, 0, 0, MODE_SGBM). */
MVSV_API void mvsv_sgbm_params_default(mvsv_sgbm_params* p);
/* StereoSGBM::create(minDisparity, numDisparities, blockSize, P1, P2, ...). */
MVSV_API void mvsv_sgbm_params_create(mvsv_sgbm_params* p, int min_disparity,
                                      int num_disparities, int block_size, int p1, int p2,
                                      int disp12_max_diff, int pre_filter_cap,
                                      int uniqueness_ratio, int speckle_window_size,
                                      int speckle_range, int mode);
/* StereoBM::create(numDisparities, blockSize) defaults. */
MVSV_API void mvsv_bm_params_default(mvsv_bm_params* p, int num_disparities, int block_size);

/* Validation only (no device needed): MVSV_OK or MVSV_E_INVALID_ARG. */
MVSV_API int mvsv_sgbm_validate(const mvsv_sgbm_params* p, int W, int H);
MVSV_API int mvsv_bm_validate(const mvsv_bm_params* p, int W, int H);

MVSV_API int mvsv_create(mvsv_ctx** out, int hip_device);
MVSV_API void mvsv_destroy(mvsv_ctx* ctx);
MVSV_API const char* mvsv_last_error(const mvsv_ctx* ctx);
/* Enqueue on an external hipStream_t (e.g. the caller's current stream).
 * NULL selects the HIP null (default) stream, which is what torch's default
 * current stream is; mvsv_use_own_stream() returns to the context's own
 * non-blocking stream. */
MVSV_API int mvsv_set_stream(mvsv_ctx* ctx, void* hip_stream);
MVSV_API int mvsv_use_own_stream(mvsv_ctx* ctx);
MVSV_API void* mvsv_get_stream(mvsv_ctx* ctx);
/* Waits for the context stream; MVSV_E_TIMEOUT if an SGBM launch since the last
 * check gave up a strip hand-off (its maps were written as all INVALID).  The
 * device calls also return MVSV_E_TIMEOUT, without enqueueing, when an earlier
 * launch that has completed by then gave up. */
MVSV_API int mvsv_synchronize(mvsv_ctx* ctx);
MVSV_API int mvsv_set_option(mvsv_ctx* ctx, int option, long long value);
/* Release cached device buffers. */
MVSV_API int mvsv_trim(mvsv_ctx* ctx);

/* Host pointers, synchronous.  Strides are in elements (bytes for u8, int16
 * elements for out); stride >= W allows ROI views (src/Stereosystem.cpp:255-256). */
MVSV_API int mvsv_sgbm(mvsv_ctx* ctx, const uint8_t* left, size_t left_stride,
                       const uint8_t* right, size_t right_stride, int width, int height,
                       const mvsv_sgbm_params* p, int16_t* out, size_t out_stride);
MVSV_API int mvsv_bm(mvsv_ctx* ctx, const uint8_t* left, size_t left_stride,
                     const uint8_t* right, size_t right_stride, int width, int height,
                     const mvsv_bm_params* p, int16_t* out, size_t out_stride);

/* Device pointers (HBM-resident), asynchronous on the context stream.
 * A batch of n frames: frame i starts at base + i * frame_stride (elements). */
MVSV_API int mvsv_sgbm_device(mvsv_ctx* ctx, int n, const uint8_t* left, size_t left_stride,
                              size_t left_frame_stride, const uint8_t* right,
                              size_t right_stride, size_t right_frame_stride, int width,
                              int height, const mvsv_sgbm_params* p, int16_t* out,
                              size_t out_stride, size_t out_frame_stride);
MVSV_API int mvsv_bm_device(mvsv_ctx* ctx, int n, const uint8_t* left, size_t left_stride,
                            size_t left_frame_stride, const uint8_t* right,
                            size_t right_stride, size_t right_frame_stride, int width,
                            int height, const mvsv_bm_params* p, int16_t* out,
                            size_t out_stride, size_t out_frame_stride);

/* Device bytes the context will cache for one SGBM / BM call of this shape. */
MVSV_API size_t mvsv_sgbm_workspace_bytes(int n, int width, int height,
                                          const mvsv_sgbm_params* p);

/* The pipeline this context would run for an SGBM call of this shape and these
   parameters (no reference counterpart: introspection for byte models and
   tests), as MVSV_PLAN_* bits in *plan. */
enum {
    MVSV_PLAN_BITSLICE = 1,  /* bit-sliced path aggregation (MODE_HH or MODE_SGBM, sgbm.yml regime) */
    MVSV_PLAN_SIDE = 2,      /* every direction on its own chains (small launches) */
    MVSV_PLAN_STRIPS = 4,    /* sheared strips + row directions (frame batches) */
    MVSV_PLAN_RESIDUAL = 8   /* packed passes read the nibble cost residual plane */
};
MVSV_API int mvsv_sgbm_plan(mvsv_ctx* ctx, int n, int width, int height, const mvsv_sgbm_params* p,
                            int* plan);

/* MeanDisparityDetection post-pass on device: 9x9 tile means of an int16 map
 * (tile = (W/9)x(H/9), remainder ignored; mean over values > 1 with integer
 * division, 0 for an empty tile).  means: 81 floats per frame (device ptr). */
MVSV_API int mvsv_mean_disparity_grid_device(mvsv_ctx* ctx, int n, const int16_t* dmap,
                                             size_t stride, size_t frame_stride, int width,
                                             int height, float* means);

/* Same grid for a host map (synchronous). means: 81 floats, row-major 9x9. */
MVSV_API int mvsv_mean_disparity_grid(mvsv_ctx* ctx, const int16_t* dmap, size_t stride,
                                      int width, int height, float* means);

/* ---- frame stream ------------------------------------------
 * A camera loop pushes rectified pairs from host memory and pops int16 maps in
 * push order.  Up to `depth` frames are in flight: the upload of one frame, the
 * SGBM of the previous one (on the context stream) and the download of the one
 * before overlap.  With grid_roi, each frame's 9x9 MeanDisparityDetection grid
 * over that ROI of the map (createDMapROIS, trgt/mean_test.cpp:80-106) is
 * computed on the device and returned by pop. */
typedef struct mvsv_stream mvsv_stream;
typedef struct { int x0, y0, x1, y1; } mvsv_rect; /* half-open [x0,x1) x [y0,y1) */
MVSV_API int mvsv_stream_create(mvsv_ctx* ctx, int width, int height, const mvsv_sgbm_params* p,
                                int depth, const mvsv_rect* grid_roi, mvsv_stream** out);
/* new parameters for frames pushed from now on (the reference's setters between frames) */
MVSV_API int mvsv_stream_set_params(mvsv_stream* s, const mvsv_sgbm_params* p);
/* compute pushed frames `batch` at a time (1..depth, default 1): one frame-batch
 * launch per group of consecutive frames -- the sustained rate of the batch
 * kernels for up to batch-1 frames of extra latency; pop / set_params launch a
 * partial group when they need its frames */
MVSV_API int mvsv_stream_set_batch(mvsv_stream* s, int batch);
/* up to n (1..4, default 1) frame-batch launches in flight at once: launches go
 * round-robin to the caller's context and n-1 contexts the stream creates on the
 * same device (own HIP stream and scratch each; kernel options copied from the
 * caller's context) -- one launch's latency-bound kernels overlap the next's */
MVSV_API int mvsv_stream_set_inflight(mvsv_stream* s, int n);
/* MVSV_E_INVALID_ARG when depth frames are already pending (pop first) */
MVSV_API int mvsv_stream_push(mvsv_stream* s, const uint8_t* left, size_t left_stride,
                              const uint8_t* right, size_t right_stride);
/* waits for the oldest pending frame; out (int16, stride in elements) and means
 * (81 floats) may be NULL */
MVSV_API int mvsv_stream_pop(mvsv_stream* s, int16_t* out, size_t out_stride, float* means);
/* pop without the map copy: *map points at the frame's int16 map in the stream's
 * pinned host slot (width elements per row, rows contiguous), valid until the
 * next push (which may reuse the slot); means (81 floats) may be NULL */
MVSV_API int mvsv_stream_pop_view(mvsv_stream* s, const int16_t** map, float* means);
MVSV_API int mvsv_stream_pending(const mvsv_stream* s);
MVSV_API void mvsv_stream_destroy(mvsv_stream* s);

/* ---- before the path: rectification ---------------------------
 * cv::remap(src, dst, map_x, map_y, INTER_LINEAR) with BORDER_CONSTANT 0 for CV_8UC1
 * images and CV_32FC1 maps, in OpenCV 3.4's fixed-point arithmetic (INTER_BITS 5,
 * 15-bit weights): bit-exact for given maps.  n frames (device pointers) share one
 * map pair (dst_width x dst_height floats each, map_stride floats per row). */
MVSV_API int mvsv_remap_device(mvsv_ctx* ctx, int n, const uint8_t* src, size_t src_stride,
                               size_t src_frame_stride, int src_width, int src_height,
                               const float* map_x, const float* map_y, size_t map_stride,
                               uint8_t* dst, size_t dst_stride, size_t dst_frame_stride,
                               int dst_width, int dst_height);

/* Stereosystem::getRectifiedImagepair on host buffers: remap both images of a
 * W x H pair with their map pairs (maps: left x, left y, right x, right y, host,
 * W x H floats each), then crop to roi (mDisplayROI) into out_left / out_right
 * ((roi.x1 - roi.x0) x (roi.y1 - roi.y0) bytes). */
MVSV_API int mvsv_rectify_pair(mvsv_ctx* ctx, const uint8_t* left, size_t left_stride,
                               const uint8_t* right, size_t right_stride, int width, int height,
                               const float* const* maps, const mvsv_rect* roi, uint8_t* out_left,
                               size_t out_left_stride, uint8_t* out_right, size_t out_right_stride);

/* cv::resize(src, dst, Size(0, 0), fx, fy, INTER_LINEAR) for CV_8UC1 -- the resize
 * step of Stereosystem::getRectifiedImagepair(Stereopair&, float)
 * (src/Stereosystem.cpp:279-315), in OpenCV 3.4's arithmetic (11-bit fixed-point
 * taps; a factor of exactly 0.5 takes INTER_AREA's fast 2x2 path).
 * mvsv_resize_size: the output size (cvRound(width * fx), cvRound(height * fy)).
 * mvsv_resize_device: n frames, device pointers, strides in bytes.
 * mvsv_resize: one host image (dst holds the mvsv_resize_size image). */
MVSV_API int mvsv_resize_size(int src_width, int src_height, double fx, double fy, int* dst_width,
                              int* dst_height);
MVSV_API int mvsv_resize_device(mvsv_ctx* ctx, int n, const uint8_t* src, size_t src_stride,
                                size_t src_frame_stride, int src_width, int src_height, double fx,
                                double fy, uint8_t* dst, size_t dst_stride, size_t dst_frame_stride);
MVSV_API int mvsv_resize(mvsv_ctx* ctx, const uint8_t* src, size_t src_stride, int src_width,
                         int src_height, double fx, double fy, uint8_t* dst, size_t dst_stride);

/* cv::initUndistortRectifyMap(K, dist, R, P, size, CV_32FC1): K 3x3, dist =
 * (k1, k2, p1, p2[, k3[, k4, k5, k6]]) with ndist in {0, 4, 5, 8}, R 3x3, P 3x3 or
 * the left 3x3 of a 3x4 projection (row-major doubles).  Double-precision
 * restatement (inverse of P*R by adjugate; OpenCV uses SVD, so maps may differ
 * in the last float bit); host only. */
MVSV_API int mvsv_init_undistort_rectify_map(const double* K, const double* dist, int ndist,
                                             const double* R, const double* P, int width,
                                             int height, float* map_x, float* map_y,
                                             size_t map_stride);

/* cv::stereoRectify(K1, D1, K2, D2, size, R, T, R1, R2, P1, P2, Q, flags, alpha,
 * size, &roi1, &roi2) as Stereosystem::initRectification calls it
 * (src/Stereosystem.cpp:209-212: flags = CALIB_ZERO_DISPARITY, alpha = 0).
 * K 3x3, D (k1, k2, p1, p2[, k3[, k4, k5, k6]]), R 3x3, T 3; outputs R1/R2 3x3,
 * P1/P2 3x4, Q 4x4 (may be NULL), valid-pixel ROIs (may be NULL); all row-major
 * doubles.  Double-precision restatement of OpenCV 3.4's cvStereoRectify (host). */
#define MVSV_CALIB_ZERO_DISPARITY 1024
MVSV_API int mvsv_stereo_rectify(const double* K1, const double* D1, int ndist1, const double* K2,
                                 const double* D2, int ndist2, int width, int height,
                                 const double* R, const double* T, int flags, double alpha,
                                 double* R1, double* R2, double* P1, double* P2, double* Q,
                                 mvsv_rect* roi1, mvsv_rect* roi2);

/* ---- calibration files -------------------------------------------
 * cv::FileStorage YAML matrices ("key: !!opencv-matrix", rows / cols / dt / data) in
 * the layout OpenCV 3.x writes (%YAML:1.0 header, data lists wrapped at column 71,
 * doubles "%.16e", floats "%.8e", integral values "%d."): the files of
 * parameters/<system>/{intrinsic,extrinsic}.yml and afterCalibrationParameters.yml.
 * Empty matrices are rows = cols = 0, dt 'u'. */
#define MVSV_MAT_MAX 16
typedef struct {
    int rows, cols;
    char dt; /* 'u' 'c' 'w' 's' 'i' 'f' 'd' (CV_8U ... CV_64F) */
    double data[MVSV_MAT_MAX];
} mvsv_mat;
/* Stereosystem's intrinsic state: the nodes saveIntrinsic writes, in order. */
typedef struct {
    mvsv_mat camera_matrix_left, camera_matrix_right, dist_coeffs_left, dist_coeffs_right,
        camera_matrix_left_new, camera_matrix_right_new, q_matrix;
} mvsv_intrinsics;
typedef struct { mvsv_mat R, T, E, F; } mvsv_extrinsics;
/* One matrix node: MVSV_E_IO (cannot open), MVSV_E_PARSE (absent / malformed / > 16). */
MVSV_API int mvsv_read_matrix_yaml(const char* path, const char* key, mvsv_mat* out);
/* n matrix nodes in order (a new file). */
MVSV_API int mvsv_write_matrices_yaml(const char* path, const char* const* keys,
                                      const mvsv_mat* mats, int n);
/* Stereosystem::loadIntrinsic (src/Stereosystem.cpp:356-386): cameraMatrixLeft,
 * cameraMatrixRight and distCoeffsRight must exist (the reference checks
 * distCoeffsRight twice, never distCoeffsLeft); the *_new and Q fields come back
 * empty (loadIntrinsic does not read them). */
MVSV_API int mvsv_load_intrinsic(const char* path, mvsv_intrinsics* out);
/* Stereosystem::loadExtrinisic (src/Stereosystem.cpp:326-354): R, T, E, F required. */
MVSV_API int mvsv_load_extrinsic(const char* path, mvsv_extrinsics* out);
/* Stereosystem::saveIntrinsic / saveExtrinsic (src/Stereosystem.cpp:388-446). */
MVSV_API int mvsv_save_intrinsic(const char* path, const mvsv_intrinsics* in);
MVSV_API int mvsv_save_extrinsic(const char* path, const mvsv_extrinsics* in);

/* ---- after the path: reprojection and point-cloud output ----
 * Q is the 4x4 CV_32F reprojection matrix of stereoRectify, 16 floats row-major
 * (e.g. afterCalibrationParameters.yml "Q"). */

/* Utility::calcCoordinate for every pixel of n int16 maps (device pointers):
 * (X, Y, Z, W) = Q * (x, y, v / 16, 1) in OpenCV's float GEMM arithmetic, divided
 * by W; Z = 0 where Z / 1000 is infinite.  xyzw[f][y][x] = (X, Y, Z, v > 0), i.e.
 * float4 per pixel, row stride / frame stride in float4 elements. */
MVSV_API int mvsv_reproject_device(mvsv_ctx* ctx, int n, const int16_t* dmap, size_t stride,
                                   size_t frame_stride, int width, int height, const float* Q,
                                   float* xyzw, size_t xyzw_stride, size_t xyzw_frame_stride);

/* Utility::calcCoordinate (one point, host): out = (X, Y, Z, 1). */
MVSV_API void mvsv_calc_coordinate(float image_x, float image_y, float d_value, const float* Q,
                                   float* out4);
/* calcCoordinate of n points at once (MeanDisparityDetection::detectObstacles'
 * per-tile loop, src/MeanDisparityDetection.cpp:228-240): xyd = n x (image x,
 * image y, disparity * 16), out = n x (X, Y, Z, 1); the same arithmetic as
 * mvsv_calc_coordinate, one call instead of one per found tile. */
MVSV_API void mvsv_calc_coordinates(int n, const float* xyd, const float* Q, float* out4);
/* Utility::calcDistance: Z / 1000 of calcCoordinate, 0 when infinite. */
MVSV_API float mvsv_calc_distance(float image_x, float image_y, float d_value, const float* Q);
/* Utility::calcDMapValues: metric point (x, y, z) -> image x, y and disparity * 16. */
MVSV_API void mvsv_calc_dmap_values(const float* c3, const float* Q, float* image_x,
                                    float* image_y, float* d_value);

enum { MVSV_PLY_PLAIN = 0, MVSV_PLY_WITH_COLOR = 1, MVSV_PLY_WITH_COLOR_SHADING = 2 };

/* ply::write: ASCII PLY of count vertices (x, y, z floats, vertex_stride floats
 * apart).  WITH_COLOR greys each vertex by (z - min) / (max - min) * 255 with the
 * min / max of the positive values of the int16 map dmap (the ply's mDMap);
 * WITH_COLOR_SHADING declares colour properties but writes none (as the
 * reference does).  Colour modes need dmap (returns MVSV_E_INVALID_ARG if it is
 * empty or has no positive value).  Host-only; MVSV_E_IO if the file cannot be
 * opened. */
MVSV_API int mvsv_write_ply(const char* path, const char* author, const char* object_name,
                            const float* xyz, size_t count, size_t vertex_stride, int mode,
                            const int16_t* dmap, size_t dmap_stride, int width, int height);

/* Utility::dmap2pcl: every pixel of the host int16 map with v > 0 reprojected
 * (on the device of ctx) and written as "Hagen Hiller" / "disparity pointcloud"
 * PLY in MODE WITH_COLOR, raster order. */
MVSV_API int mvsv_dmap2pcl(mvsv_ctx* ctx, const char* path, const int16_t* dmap, size_t stride,
                           int width, int height, const float* Q);

/* Disparity::loadSGBMParameters: reads configs/sgbm.yml keys minDisp, numDisp,
 * blockSize, disp12MaxDiff, preFilterCap, uniquenessRatio, speckleWindowSize,
 * speckleWindowRange, mode into *values and applies the 8 setters + mode to
 * *p (P1/P2 untouched, as in the reference).  Missing numDisp, blockSize,
 * speckleWindowSize or speckleWindowRange -> MVSV_E_PARSE; other keys missing
 * leave the value 0 (cv::FileNode >> int on an empty node). */
MVSV_API int mvsv_load_sgbm_yaml(const char* path, mvsv_sgbm_params* p,
                                 mvsv_sgbm_yaml_values* values);
/* configs/bm.yml keys: numDisp, blockSize, preFilterCap, preFilterSize,
 * uniquenessRatio, textureThreshold (+ optional minDisp, speckleWindowSize,
 * speckleWindowRange, disp12MaxDiff, preFilterType). numDisp and blockSize are
 * required. */
MVSV_API int mvsv_load_bm_yaml(const char* path, mvsv_bm_params* p);

/* Stage profiling with HIP events (used by bench.py to time the dominant kernel
 * live).  Stages: 0 prefilter, 1 cost volume, 2 cost fixup, 3 path aggregation
 * (span of all direction passes before the final one), 4 final direction +
 * WTA/LR, 5 post-filters (median + speckle), 6 BM match, 7 path strips (the
 * sheared-strip kernel alone, inside stage 3), 8 path lines (the L->R line
 * kernel on the second stream, overlapping stage 7). */
#define MVSV_NUM_STAGES 9
MVSV_API int mvsv_profile_enable(mvsv_ctx* ctx, int on);
MVSV_API int mvsv_profile_reset(mvsv_ctx* ctx);
/* Synchronizes, then writes accumulated milliseconds and launch counts per stage. */
MVSV_API int mvsv_profile_read(mvsv_ctx* ctx, double* stage_ms, int* stage_launches, int n);
MVSV_API const char* mvsv_profile_stage_name(int stage);

/* Deterministic synthetic rectified pair: PCG32 noise,
 * 3x3 box blur, slanted-plane + rectangle disparity field, +-1 noise.
 * Host buffers of width*height bytes each. */
MVSV_API int mvsv_synth_pair(uint32_t seed, int width, int height, int min_disparity,
                             int num_disparities, uint8_t* left, uint8_t* right);

#ifdef __cplusplus
}
#endif
#endif /* MVSV_H */
