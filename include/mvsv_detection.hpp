// mvsv_detection.hpp — C++ mirror of the reference's code around the disparity
// path, on libmvsv:
//
//   struct dMapValues, namespace Utility        inc/utility.h:50-82, src/utility.cpp:176-303
//   class ply (MODE PLAIN / WITH_COLOR / ...)   inc/ply.h, src/ply.cpp:37-133
//   struct Subimage                             inc/Subimage.h:17-47
//   class MeanDisparityDetection                inc/MeanDisparityDetection.h,
//                                               src/MeanDisparityDetection.cpp:71-266
//   createDMapROIS                              trgt/mean_test.cpp:80-106
//   mvsv::DisparityStream                       replaces the worker thread +
//                                               condition variable of
//                                               trgt/mean_test.cpp:61-70,258-318
//
// Per-pixel work (the 9x9 tile means, reprojection) runs in the HIP kernels
// behind include/mvsv.h; the 81-element decisions stay on the host in the
// reference's order.  Matrices are the reference's CV_32F 4x4 Q (16 floats,
// row-major).
#ifndef MVSV_DETECTION_HPP
#define MVSV_DETECTION_HPP

#include <array>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "mvsv_disparity.hpp"

namespace mvsv {

using QMatrix = std::array<float, 16>;

struct dMapValues {  // inc/utility.h:50-55
    float dValue = 0, image_x = 0, image_y = 0;
};

struct Point {
    int x = 0, y = 0;
};

namespace Utility {

inline std::array<float, 4> calcCoordinate(dMapValues v, const QMatrix& Q)
{
    std::array<float, 4> c;
    mvsv_calc_coordinate(v.image_x, v.image_y, v.dValue, Q.data(), c.data());
    return c;
}
inline float calcDistance(dMapValues v, const QMatrix& Q, int /*binning*/)
{
    return mvsv_calc_distance(v.image_x, v.image_y, v.dValue, Q.data());
}
inline dMapValues calcDMapValues(const std::array<float, 3>& c, const QMatrix& Q)
{
    dMapValues v;
    mvsv_calc_dmap_values(c.data(), Q.data(), &v.image_x, &v.image_y, &v.dValue);
    return v;
}
// src/utility.cpp:242-262 (reprojection on the device, PLY WITH_COLOR)
inline void dmap2pcl(const std::string& filename, const Mat& dMap, const QMatrix& Q)
{
    if (dMap.type != MAT_16SC1) throw Error(MVSV_E_INVALID_ARG, "dmap2pcl: CV_16S map expected");
    mvsv_ctx* c = thread_context();
    check(mvsv_dmap2pcl(c, filename.c_str(), reinterpret_cast<const int16_t*>(dMap.data),
                        dMap.step / 2, dMap.cols, dMap.rows, Q.data()),
          c);
}
// src/utility.cpp:265-285 on the host: integer mean of the values > 1
inline float calcMeanDisparity(const Mat& m)
{
    int total = 0, n = 0;
    for (int r = 0; r < m.rows; r++)
        for (int c = 0; c < m.cols; c++) {
            short v = m.ptr<int16_t>(r)[c];
            if (v > 1) {
                total += v;
                ++n;
            }
        }
    if (total == 0 || n == 0) return 0.0f;
    return (float)(total / (n < 0 ? -n : n));
}

}  // namespace Utility

class ply {  // inc/ply.h
public:
    enum MODE { PLAIN = MVSV_PLY_PLAIN, WITH_COLOR = MVSV_PLY_WITH_COLOR,
                WITH_COLOR_SHADING = MVSV_PLY_WITH_COLOR_SHADING };
    ply() = default;
    ply(std::string author, std::string object) : mAuthor(std::move(author)), mObjectName(std::move(object)) {}
    ply(std::string author, std::string object, const Mat& dmap)
        : mAuthor(std::move(author)), mObjectName(std::move(object)), mDMap(dmap) {}
    bool write(const std::string& filename, const std::vector<std::array<float, 4>>& to_write, int mode)
    {
        if (mode != PLAIN && mDMap.empty()) return false;
        int rc = mvsv_write_ply(filename.c_str(), mAuthor.c_str(), mObjectName.c_str(),
                                to_write.empty() ? nullptr : to_write[0].data(), to_write.size(), 4,
                                mode, mDMap.empty() ? nullptr : reinterpret_cast<const int16_t*>(mDMap.data),
                                mDMap.step / 2, mDMap.cols, mDMap.rows);
        return rc == MVSV_OK;
    }

private:
    std::string mAuthor, mObjectName;
    Mat mDMap;
};

struct Subimage {  // inc/Subimage.h:17-47
    Subimage() = default;
    Subimage(Point tl_, Point br_) : tl(tl_), br(br_)
    {
        int tx = br.x - tl.x, ty = br.y - tl.y;
        roi_center = {tl.x + tx / 2, tl.y + ty / 2};
    }
    void calculateSubimageValue(const Mat& dMap)
    {
        value = Utility::calcMeanDisparity(dMap(Rect{tl.x, tl.y, br.x - tl.x, br.y - tl.y}));
    }
    Point tl, br, roi_center;
    float value = 0;
};

// trgt/mean_test.cpp:80-106 (the unbinned / binned work ROIs of the disparity map)
inline void createDMapROIS(int rows, int cols, int numDisp, Rect& roi_u, Rect& roi_b)
{
    int pixelShift = numDisp / 2;
    if (pixelShift % 2 == 1) {
        pixelShift = pixelShift + 1;
        if ((cols - pixelShift) % 8 != 0) pixelShift = pixelShift + (cols - pixelShift % 8);
    }
    roi_u = Rect{pixelShift, 0, cols - pixelShift, rows};
    roi_b = Rect{pixelShift / 2, 0, cols / 2 - pixelShift / 2, rows / 2};
}

class MeanDisparityDetection {  // src/MeanDisparityDetection.cpp
public:
    enum MODE { MEAN_DISTANCE, MEAN_VALUE };

    explicit MeanDisparityDetection(std::string pcl_dir = "pcl/subimage_detection")
        : mPclDir(std::move(pcl_dir))
    {
        for (int k = 0; k < 9; ++k) mPositions[k] = "TOP LEFT - " + std::to_string(k);
        mPositions[9] = "TOP - 0";  // the reference's table skips key 10
        for (int k = 1; k < 9; ++k) mPositions[10 + k] = "TOP - " + std::to_string(k);
        const char* groups[] = {"TOP RIGHT", "LEFT", "CENTER", "RIGHT", "BOTTOM LEFT", "BOTTOM",
                                "BOTTOM RIGHT"};
        for (int g = 0; g < 7; ++g)
            for (int k = 0; k < 9; ++k)
                mPositions[19 + 9 * g + k] = std::string(groups[g]) + " - " + std::to_string(k);
    }

    // :71-112
    void init(const Mat& reference, const QMatrix& Q, float min_distance, float max_distance)
    {
        mSubimageVec.clear();
        mQ = Q;
        int dx = reference.cols / 9, dy = reference.rows / 9;
        for (int r = 0; r < 9; ++r)
            for (int c = 0; c < 9; ++c) {
                Point tl{c * dx, r * dy}, br{c * dx + dx, r * dy + dy};
                mSubimageVec.emplace_back(tl, br);
                mFoundObstacles.emplace_back(tl, br);
            }
        dMapValues lo = Utility::calcDMapValues({0, 0, min_distance * 1000}, mQ);
        dMapValues hi = Utility::calcDMapValues({0, 0, max_distance * 1000}, mQ);
        mRangeDisparity = {lo.dValue, hi.dValue};
    }

    // :159-206; the 81 means come from the GPU (host map, or `means` from a stream pop)
    void build(const Mat& dMap, int /*binning*/, int mode, const float* means = nullptr)
    {
        mDMap = dMap;
        float m[81];
        if (!means) {
            if (dMap.type != MAT_16SC1) throw Error(MVSV_E_INVALID_ARG, "build: CV_16S map expected");
            mvsv_ctx* c = thread_context();
            check(mvsv_mean_disparity_grid(c, reinterpret_cast<const int16_t*>(dMap.data),
                                           dMap.step / 2, dMap.cols, dMap.rows, m),
                  c);
            means = m;
        }
        switch (mode) {
        case MEAN_DISTANCE:
            mDetectionMode = MEAN_DISTANCE;
            mMeanDistanceMap.clear();
            for (size_t i = 0; i < mSubimageVec.size(); ++i) {
                const Subimage& s = mSubimageVec[i];
                dMapValues v{means[i], (float)s.roi_center.x, (float)s.roi_center.y};
                mMeanDistanceMap.push_back(Utility::calcDistance(v, mQ, 0));
            }
            // falls through, as the reference's switch does
        case MEAN_VALUE:
            mDetectionMode = MEAN_VALUE;
            mMeanMap.clear();
            for (size_t i = 0; i < mSubimageVec.size(); ++i) {
                mSubimageVec[i].value = means[i];
                mMeanMap.push_back(means[i]);
            }
        }
    }

    // :211-266; returns the positions the reference prints in MEAN_DISTANCE mode
    std::vector<std::string> detectObstacles()
    {
        std::vector<std::string> printed;
        if (mDetectionMode == MEAN_DISTANCE) {
            for (size_t i = 0; i < mMeanDistanceMap.size(); ++i)
                if (mMeanDistanceMap[i] < mRange.second && mMeanDistanceMap[i] > mRange.first)
                    printed.push_back(mPositions[(int)i]);
            return printed;
        }
        if (mDetectionMode != MEAN_VALUE) return printed;
        mFoundObstacles.clear();
        std::vector<std::array<float, 4>> points;
        for (size_t i = 0; i < mMeanMap.size(); ++i) {
            if (mMeanMap[i] < mRangeDisparity.first && mMeanMap[i] > mRangeDisparity.second) {
                Subimage s = mSubimageVec[i];
                mFoundObstacles.push_back(s);
                dMapValues v{mMeanMap[i], (float)s.roi_center.x, (float)s.roi_center.y};
                points.push_back(Utility::calcCoordinate(v, mQ));
            }
        }
        if (!points.empty()) {
            ply p("Hagen Hiller", "obstacle pointcloud", mDMap);
            std::string prefix = mObstacleCounter < 10 ? "000" : (mObstacleCounter < 100 ? "00" : "0");
            p.write(mPclDir + "/pcl_" + prefix + std::to_string(mObstacleCounter) + ".ply", points,
                    ply::WITH_COLOR);
            ++mObstacleCounter;
        }
        return printed;
    }

    void setRange(float min_distance, float max_distance) { mRange = {min_distance, max_distance}; }
    std::pair<int, int> getRange() const { return {(int)mRange.first, (int)mRange.second}; }
    const std::vector<Subimage>& getSubimageVec() const { return mSubimageVec; }
    const std::vector<float>& getMeanMap() const { return mMeanMap; }
    const std::vector<float>& getMeanDistanceMap() const { return mMeanDistanceMap; }
    const std::vector<Subimage>& getFoundObstacles() const { return mFoundObstacles; }
    int getObstacleCounter() const { return mObstacleCounter; }
    std::pair<float, float> getRangeDisparity() const { return mRangeDisparity; }

private:
    std::string mPclDir;
    Mat mDMap;
    std::map<int, std::string> mPositions;
    std::vector<Subimage> mSubimageVec, mFoundObstacles;
    std::vector<float> mMeanMap, mMeanDistanceMap;
    QMatrix mQ{};
    int mDetectionMode = -1;
    int mObstacleCounter = 0;
    std::pair<float, float> mRange{0, 0}, mRangeDisparity{0, 0};
};

// Camera loop without the worker thread: push rectified pairs, pop maps (and the
// 9x9 means of the work ROI) in order; up to `depth` frames in flight.
class DisparityStream {
public:
    DisparityStream(const StereoSGBM& matcher, int width, int height, int depth = 3,
                    const Rect* grid_roi = nullptr)
        : ctx_(thread_context()), w_(width), h_(height)
    {
        mvsv_rect r{};
        if (grid_roi) r = {grid_roi->x, grid_roi->y, grid_roi->x + grid_roi->width, grid_roi->y + grid_roi->height};
        check(mvsv_stream_create(ctx_, width, height, &matcher.params(), depth, grid_roi ? &r : nullptr, &s_),
              ctx_);
    }
    ~DisparityStream()
    {
        if (s_) mvsv_stream_destroy(s_);
    }
    DisparityStream(const DisparityStream&) = delete;
    DisparityStream& operator=(const DisparityStream&) = delete;
    void setParams(const StereoSGBM& matcher) { check(mvsv_stream_set_params(s_, &matcher.params()), ctx_); }
    // frames computed `batch` at a time (frame-batch kernels, up to batch-1 frames of latency)
    void setBatch(int batch) { check(mvsv_stream_set_batch(s_, batch), ctx_); }
    // up to n frame-batch launches computed concurrently (1..4)
    void setInflight(int n) { check(mvsv_stream_set_inflight(s_, n), ctx_); }
    int pending() const { return mvsv_stream_pending(s_); }
    void push(const Stereopair& s)
    {
        check_pair(s.mLeft, s.mRight);
        check(mvsv_stream_push(s_, s.mLeft.data, s.mLeft.step, s.mRight.data, s.mRight.step), ctx_);
    }
    void pop(Mat& disparity, float* means81 = nullptr)
    {
        disparity.create(h_, w_, MAT_16SC1);
        check(mvsv_stream_pop(s_, reinterpret_cast<int16_t*>(disparity.data), disparity.step / 2, means81),
              ctx_);
    }
    // the oldest frame's map in the stream's pinned host slot (width x height
    // int16, no copy), valid until the next push
    const int16_t* popView(float* means81 = nullptr)
    {
        const int16_t* map = nullptr;
        check(mvsv_stream_pop_view(s_, &map, means81), ctx_);
        return map;
    }

private:
    mvsv_ctx* ctx_;
    mvsv_stream* s_ = nullptr;
    int w_, h_;
};

}  // namespace mvsv

#endif  // MVSV_DETECTION_HPP
