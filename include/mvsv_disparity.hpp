// mvsv_disparity.hpp — C++ drop-in for the reference's inc/disparity.h on libmvsv.
//
// Reference surface (hG3n/mvStereoVision3):
//   struct Stereopair                      inc/utility.h:31-41
//   Disparity::sgbmParameters              inc/disparity.h:17-27
//   Disparity::sgbm(Stereopair const&, cv::Mat&, cv::Ptr<cv::StereoSGBM>)   src/disparity.cpp:6-10
//   Disparity::bm  (Stereopair const&, cv::Mat&, cv::Ptr<cv::StereoBM>)     src/disparity.cpp:18-22
//   Disparity::loadSGBMParameters(std::string, cv::Ptr<cv::StereoSGBM>&, sgbmParameters&)
//                                                                          src/disparity.cpp:60-108
// This header keeps those names, argument meaning and error behaviour without
// OpenCV: mvsv::Mat is the subset of cv::Mat the path touches (rows, cols,
// step, CV_8UC1 / CV_16SC1 data, ROI views with step > cols) and
// mvsv::StereoSGBM / mvsv::StereoBM mirror cv::StereoSGBM / cv::StereoBM
// (create() defaults and setters of OpenCV 3.4).  Errors that OpenCV reports as
// cv::Exception throw mvsv::Error; the loaders return false.  Compute runs in
// the HIP kernels behind include/mvsv.h; for code that keeps cv::Mat and
// cv::Ptr<cv::StereoSGBM>, see include/mvsv_cv.hpp.
#ifndef MVSV_DISPARITY_HPP
#define MVSV_DISPARITY_HPP

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "mvsv.h"

namespace mvsv {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& msg)
        : std::runtime_error("mvsv error " + std::to_string(code) + ": " + msg), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void check(int rc, const mvsv_ctx* ctx)
{
    if (rc < 0) throw Error(rc, ctx ? mvsv_last_error(ctx) : "");
}

// One context (HIP stream + cached device buffers) per host thread, like the
// reference's one matcher per worker thread (trgt/mean_test.cpp:61-70).
inline mvsv_ctx* thread_context(int device = 0)
{
    struct Holder {
        mvsv_ctx* c = nullptr;
        ~Holder()
        {
            if (c) mvsv_destroy(c);
        }
    };
    thread_local Holder h;
    if (!h.c) check(mvsv_create(&h.c, device), nullptr);
    return h.c;
}

enum { MAT_8UC1 = 0, MAT_16SC1 = 3 };  // cv::Mat type codes CV_8UC1 / CV_16SC1

struct Rect {
    int x, y, width, height;
};

// The part of cv::Mat the disparity path uses.
struct Mat {
    int rows = 0, cols = 0, type = MAT_8UC1;
    size_t step = 0;  // bytes per row
    uint8_t* data = nullptr;
    std::shared_ptr<std::vector<uint8_t>> owner;

    Mat() = default;
    Mat(int r, int c, int t) { create(r, c, t); }
    static size_t elem(int t) { return t == MAT_16SC1 ? 2 : 1; }
    // non-owning view on user memory (step in bytes)
    static Mat wrap(void* p, int r, int c, int t, size_t step_bytes)
    {
        Mat m;
        m.rows = r;
        m.cols = c;
        m.type = t;
        m.step = step_bytes;
        m.data = static_cast<uint8_t*>(p);
        return m;
    }
    bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
    // cv::Mat::create: reallocate unless size and type already match
    void create(int r, int c, int t)
    {
        if (data && r == rows && c == cols && t == type) return;
        owner = std::make_shared<std::vector<uint8_t>>((size_t)r * c * elem(t));
        data = owner->data();
        rows = r;
        cols = c;
        type = t;
        step = (size_t)c * elem(t);
    }
    Mat operator()(const Rect& roi) const
    {
        if (roi.x < 0 || roi.y < 0 || roi.x + roi.width > cols || roi.y + roi.height > rows)
            throw Error(MVSV_E_INVALID_ARG, "ROI outside the image");
        Mat m = *this;
        m.data = data + (size_t)roi.y * step + (size_t)roi.x * elem(type);
        m.rows = roi.height;
        m.cols = roi.width;
        return m;
    }
    template <typename T>
    T* ptr(int y)
    {
        return reinterpret_cast<T*>(data + (size_t)y * step);
    }
    template <typename T>
    const T* ptr(int y) const
    {
        return reinterpret_cast<const T*>(data + (size_t)y * step);
    }
};

template <class T>
using Ptr = std::shared_ptr<T>;

inline void check_pair(const Mat& L, const Mat& R)
{
    if (L.empty() || L.type != MAT_8UC1 || R.type != MAT_8UC1 || L.rows != R.rows ||
        L.cols != R.cols)
        throw Error(MVSV_E_INVALID_ARG,
                    "left.size() == right.size() && left.type() == right.type() && CV_8UC1");
}

class StereoSGBM {
public:
    enum { MODE_SGBM = MVSV_MODE_SGBM, MODE_HH = MVSV_MODE_HH };
    static Ptr<StereoSGBM> create(int minDisparity = 0, int numDisparities = 16,
                                  int blockSize = 3, int P1 = 0, int P2 = 0,
                                  int disp12MaxDiff = 0, int preFilterCap = 0,
                                  int uniquenessRatio = 0, int speckleWindowSize = 0,
                                  int speckleRange = 0, int mode = MODE_SGBM)
    {
        auto m = std::make_shared<StereoSGBM>();
        mvsv_sgbm_params_create(&m->p, minDisparity, numDisparities, blockSize, P1, P2,
                                disp12MaxDiff, preFilterCap, uniquenessRatio, speckleWindowSize,
                                speckleRange, mode);
        return m;
    }
    void compute(const Mat& left, const Mat& right, Mat& disparity)
    {
        check_pair(left, right);
        disparity.create(left.rows, left.cols, MAT_16SC1);
        mvsv_ctx* c = thread_context();
        check(mvsv_sgbm(c, left.data, left.step, right.data, right.step, left.cols, left.rows, &p,
                        reinterpret_cast<int16_t*>(disparity.data), disparity.step / 2),
              c);
    }
    void setMinDisparity(int v) { p.min_disparity = v; }
    int getMinDisparity() const { return p.min_disparity; }
    void setNumDisparities(int v) { p.num_disparities = v; }
    int getNumDisparities() const { return p.num_disparities; }
    void setBlockSize(int v) { p.block_size = v; }
    int getBlockSize() const { return p.block_size; }
    void setSpeckleWindowSize(int v) { p.speckle_window_size = v; }
    int getSpeckleWindowSize() const { return p.speckle_window_size; }
    void setSpeckleRange(int v) { p.speckle_range = v; }
    int getSpeckleRange() const { return p.speckle_range; }
    void setDisp12MaxDiff(int v) { p.disp12_max_diff = v; }
    int getDisp12MaxDiff() const { return p.disp12_max_diff; }
    void setPreFilterCap(int v) { p.pre_filter_cap = v; }
    int getPreFilterCap() const { return p.pre_filter_cap; }
    void setUniquenessRatio(int v) { p.uniqueness_ratio = v; }
    int getUniquenessRatio() const { return p.uniqueness_ratio; }
    void setP1(int v) { p.p1 = v; }
    int getP1() const { return p.p1; }
    void setP2(int v) { p.p2 = v; }
    int getP2() const { return p.p2; }
    void setMode(int v) { p.mode = v; }
    int getMode() const { return p.mode; }
    const mvsv_sgbm_params& params() const { return p; }
    mvsv_sgbm_params p{};
};

class StereoBM {
public:
    enum {
        PREFILTER_NORMALIZED_RESPONSE = MVSV_PREFILTER_NORMALIZED_RESPONSE,
        PREFILTER_XSOBEL = MVSV_PREFILTER_XSOBEL
    };
    static Ptr<StereoBM> create(int numDisparities = 0, int blockSize = 21)
    {
        auto m = std::make_shared<StereoBM>();
        mvsv_bm_params_default(&m->p, numDisparities, blockSize);
        return m;
    }
    void compute(const Mat& left, const Mat& right, Mat& disparity)
    {
        check_pair(left, right);
        disparity.create(left.rows, left.cols, MAT_16SC1);
        mvsv_ctx* c = thread_context();
        check(mvsv_bm(c, left.data, left.step, right.data, right.step, left.cols, left.rows, &p,
                      reinterpret_cast<int16_t*>(disparity.data), disparity.step / 2),
              c);
    }
    void setMinDisparity(int v) { p.min_disparity = v; }
    int getMinDisparity() const { return p.min_disparity; }
    void setNumDisparities(int v) { p.num_disparities = v; }
    int getNumDisparities() const { return p.num_disparities; }
    void setBlockSize(int v) { p.block_size = v; }
    int getBlockSize() const { return p.block_size; }
    void setSpeckleWindowSize(int v) { p.speckle_window_size = v; }
    void setSpeckleRange(int v) { p.speckle_range = v; }
    void setDisp12MaxDiff(int v) { p.disp12_max_diff = v; }
    void setPreFilterType(int v) { p.pre_filter_type = v; }
    void setPreFilterSize(int v) { p.pre_filter_size = v; }
    void setPreFilterCap(int v) { p.pre_filter_cap = v; }
    int getPreFilterCap() const { return p.pre_filter_cap; }
    void setTextureThreshold(int v) { p.texture_threshold = v; }
    int getTextureThreshold() const { return p.texture_threshold; }
    void setUniquenessRatio(int v) { p.uniqueness_ratio = v; }
    int getUniquenessRatio() const { return p.uniqueness_ratio; }
    mvsv_bm_params p{};
};

}  // namespace mvsv

#ifndef MVSV_NO_STEREOPAIR
// inc/utility.h:31-41
struct Stereopair {
    Stereopair() : mTag("STEREOPAIR\t") {}
    Stereopair(mvsv::Mat& l, mvsv::Mat& r) : mLeft(l), mRight(r), mTag("STEREOPAIR\t") {}
    mvsv::Mat mLeft;
    mvsv::Mat mRight;
    std::string mTag;
};
#endif

namespace Disparity {

// inc/disparity.h:17-27
struct sgbmParameters {
    int minDisp;
    int numDisp;
    int blockSize;
    int disp12MaxDiff;
    int preFilterCap;
    int uniquenessRatio;
    int speckleWindowSize;
    int speckleRange;
    int disparityMode;
};

// src/disparity.cpp:6-10 — output (re)allocated CV_16S, disparity * 16
template <class Pair>
inline void sgbm(Pair const& inputImages, mvsv::Mat& output, mvsv::Ptr<mvsv::StereoSGBM> dispCompute)
{
    dispCompute->compute(inputImages.mLeft, inputImages.mRight, output);
}

// src/disparity.cpp:18-22
template <class Pair>
inline void bm(Pair const& inputImages, mvsv::Mat& output, mvsv::Ptr<mvsv::StereoBM> dispCompute)
{
    dispCompute->compute(inputImages.mLeft, inputImages.mRight, output);
}

// src/disparity.cpp:60-108 — eight setters + mode from configs/sgbm.yml; P1/P2 untouched
inline bool loadSGBMParameters(std::string const filename, mvsv::Ptr<mvsv::StereoSGBM>& disparityObj,
                               sgbmParameters& para)
{
    mvsv_sgbm_yaml_values v;
    int rc = mvsv_load_sgbm_yaml(filename.c_str(), &disparityObj->p, &v);
    if (rc == MVSV_E_PARSE) {
        std::fprintf(stderr, "ERROR: Node in %s is empty\n", filename.c_str());
        return false;
    }
    if (rc < 0) {
        std::fprintf(stderr, "ERROR: Unable to open disparity parameters\n");
        return false;
    }
    para = {v.minDisp,         v.numDisp,           v.blockSize,    v.disp12MaxDiff, v.preFilterCap,
            v.uniquenessRatio, v.speckleWindowSize, v.speckleRange, v.disparityMode};
    return true;
}

// new: configs/bm.yml:2-7 (shipped by the reference, read by nothing)
inline bool loadBMParameters(std::string const filename, mvsv::Ptr<mvsv::StereoBM>& disparityObj)
{
    return mvsv_load_bm_yaml(filename.c_str(), &disparityObj->p) == MVSV_OK;
}

}  // namespace Disparity

#endif  // MVSV_DISPARITY_HPP
