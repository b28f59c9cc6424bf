// mvsv_cv.hpp — OpenCV glue for the reference's own types (cv::Mat,
// cv::Ptr<cv::StereoSGBM>, cv::Ptr<cv::StereoBM>).
//
// For a build of hG3n/mvStereoVision3 that keeps OpenCV for I/O and GUI but
// runs the disparity hot path on MI355X: src/disparity.cpp:6-10 and :18-22
// call mvsv_cv::compute() instead of dispCompute->compute().  The matcher
// object stays the reference's cv::StereoSGBM / cv::StereoBM: its state is
// read through the OpenCV 3.x getters on every call, so the setters the
// reference calls between frames (trgt/mean_test.cpp:348,355) keep working.
//
// Not compiled in this repository's tests: OpenCV is not installed in the
// build image; the cv-free path in mvsv_disparity.hpp is.
#ifndef MVSV_CV_HPP
#define MVSV_CV_HPP

#include <opencv2/calib3d.hpp>
#include <opencv2/core.hpp>

#include "mvsv_disparity.hpp"

namespace mvsv_cv {

inline mvsv_sgbm_params params_of(const cv::StereoSGBM& m)
{
    mvsv_sgbm_params p;
    mvsv_sgbm_params_create(&p, m.getMinDisparity(), m.getNumDisparities(), m.getBlockSize(),
                            m.getP1(), m.getP2(), m.getDisp12MaxDiff(), m.getPreFilterCap(),
                            m.getUniquenessRatio(), m.getSpeckleWindowSize(), m.getSpeckleRange(),
                            m.getMode() == cv::StereoSGBM::MODE_HH ? MVSV_MODE_HH : MVSV_MODE_SGBM);
    return p;
}

inline mvsv_bm_params params_of(const cv::StereoBM& m)
{
    mvsv_bm_params p;
    mvsv_bm_params_default(&p, m.getNumDisparities(), m.getBlockSize());
    p.pre_filter_type = m.getPreFilterType();
    p.pre_filter_size = m.getPreFilterSize();
    p.pre_filter_cap = m.getPreFilterCap();
    p.min_disparity = m.getMinDisparity();
    p.texture_threshold = m.getTextureThreshold();
    p.uniqueness_ratio = m.getUniquenessRatio();
    p.speckle_window_size = m.getSpeckleWindowSize();
    p.speckle_range = m.getSpeckleRange();
    p.disp12_max_diff = m.getDisp12MaxDiff();
    return p;
}

inline void check_inputs(const cv::Mat& L, const cv::Mat& R)
{
    CV_Assert(L.size() == R.size() && L.type() == R.type() && L.type() == CV_8UC1);
}

// Drop-in for dispCompute->compute(L, R, out) with a cv::StereoSGBM matcher.
inline void compute(const cv::Ptr<cv::StereoSGBM>& m, const cv::Mat& L, const cv::Mat& R,
                    cv::Mat& out)
{
    check_inputs(L, R);
    out.create(L.size(), CV_16S);
    mvsv_sgbm_params p = params_of(*m);
    mvsv_ctx* c = mvsv::thread_context();
    int rc = mvsv_sgbm(c, L.data, L.step, R.data, R.step, L.cols, L.rows, &p,
                       out.ptr<int16_t>(), out.step / sizeof(int16_t));
    if (rc < 0) CV_Error(cv::Error::StsError, mvsv_last_error(c));
}

inline void compute(const cv::Ptr<cv::StereoBM>& m, const cv::Mat& L, const cv::Mat& R,
                    cv::Mat& out)
{
    check_inputs(L, R);
    out.create(L.size(), CV_16S);
    mvsv_bm_params p = params_of(*m);
    mvsv_ctx* c = mvsv::thread_context();
    int rc = mvsv_bm(c, L.data, L.step, R.data, R.step, L.cols, L.rows, &p, out.ptr<int16_t>(),
                     out.step / sizeof(int16_t));
    if (rc < 0) CV_Error(cv::Error::StsOutOfRange, mvsv_last_error(c));
}

}  // namespace mvsv_cv

#endif  // MVSV_CV_HPP
