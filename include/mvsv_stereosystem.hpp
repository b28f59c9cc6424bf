// mvsv_stereosystem.hpp — C++ drop-in for the reference's class Stereosystem
// (inc/Stereosystem.h:16-86, src/Stereosystem.cpp) on libmvsv: calibration
// files, the rectification set-up and the rectified (optionally resized) pair.
//
// Reference surface kept (names, argument meaning, return values, quirks):
//   getFundamentalMatrix / getTranslationMatrix / getBaseline / getRotationMatrix /
//   getQMatrix / getNewKMats                         src/Stereosystem.cpp:47-80
//   initRectification                                src/Stereosystem.cpp:193-241
//   getRectifiedImagepair(Stereopair&)               src/Stereosystem.cpp:243-277
//   getRectifiedImagepair(Stereopair&, float)        src/Stereosystem.cpp:279-315
//   resetRectification                               src/Stereosystem.cpp:317-320
//   loadExtrinisic / loadIntrinsic / saveExtrinsic / saveIntrinsic
//                                                    src/Stereosystem.cpp:326-446
// What the reference gets from its two mvIMPACT cameras (image size, binning
// mode, the raw pair of getImagepair) is given here at construction / passed
// in: getRectifiedImagepair rectifies the raw pair the Stereopair holds, in
// place, like the reference does after Stereosystem::getImagepair filled it.
// Calibration (cv::stereoCalibrate) and getUndistortedImagepair stay out of
// scope.  Compute: the remap and resize run in HIP kernels
// (mvsv_rectify_pair, mvsv_resize, include/mvsv.h); stereoRectify and the
// undistort maps are host restatements (mvsv_stereo_rectify,
// mvsv_init_undistort_rectify_map).  LOG(INFO) / LOG(ERROR) lines of the
// reference go to stderr with the same mTag prefix.
#ifndef MVSV_STEREOSYSTEM_HPP
#define MVSV_STEREOSYSTEM_HPP

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

#include "mvsv.h"
#include "mvsv_disparity.hpp"

namespace mvsv {

// The small CV_64F / CV_32F matrices of the calibration state (cv::Mat subset:
// rows x cols doubles, the element type char of the file, empty = 0 x 0).
struct Matd {
    int rows = 0, cols = 0;
    char dt = 'u';
    std::vector<double> v;

    Matd() = default;
    Matd(int r, int c, char t = 'd') : rows(r), cols(c), dt(t), v((size_t)r * c, 0.0) {}
    bool empty() const { return rows == 0 || cols == 0; }
    double& at(int r, int c) { return v[(size_t)r * cols + c]; }
    double at(int r, int c) const { return v[(size_t)r * cols + c]; }
    const double* data() const { return v.data(); }
    static Matd from(const mvsv_mat& m)
    {
        Matd o(m.rows, m.cols, m.dt ? m.dt : 'u');
        for (int i = 0; i < m.rows * m.cols; i++) o.v[i] = m.data[i];
        return o;
    }
    mvsv_mat to() const
    {
        mvsv_mat m{};
        m.rows = rows;
        m.cols = cols;
        m.dt = empty() ? 'u' : dt;
        for (size_t i = 0; i < v.size() && i < MVSV_MAT_MAX; i++) m.data[i] = v[i];
        return m;
    }
    void copyTo(Matd& o) const { o = *this; }
};

class Stereosystem {
public:
    // width x height: the cameras' image size (halved by binning, like
    // Camera::getImageWidth / getImageHeight report it); binning: both cameras
    // in binning mode (the intrinsics are halved while the rectification is
    // initialised, src/Stereosystem.cpp:202-206, 232-236)
    Stereosystem(int width, int height, bool binning = false)
        : mWidth(width), mHeight(height), mBinning(binning), mTag("STEREOSYSTEM\t")
    {
        log_info("Stereosystem created\n");
    }
    ~Stereosystem() { log_info("Stereosystem destroyed\n"); }

    // --- getters (src/Stereosystem.cpp:47-80) --------------------------------
    void getFundamentalMatrix(Matd& fundamental) const { mF.copyTo(fundamental); }
    void getTranslationMatrix(Matd& translation) const { mT.copyTo(translation); }
    double getBaseline() const
    {
        return std::sqrt(std::pow(mT.at(0, 0), 2) + std::pow(mT.at(1, 0), 2) + std::pow(mT.at(2, 0), 2));
    }
    Matd getRotationMatrix() const { return mR; }
    Matd getQMatrix() const { return mQ; }
    std::vector<Matd> getNewKMats() const { return {mP0, mP1}; }

    // --- rectification (src/Stereosystem.cpp:193-320) --------------------------
    bool initRectification()
    {
        log_info("Called initRectifiaction()\n");
        if (mIntrinsicLeft.rows != 3 || mIntrinsicRight.rows != 3 || mR.rows != 3 || mT.empty()) {
            log_error("Unable to init rectification\n");
            return false;
        }
        Matd KL = mIntrinsicLeft, KR = mIntrinsicRight;
        if (mBinning)
            for (int i = 0; i < 9; i++) {
                KL.v[i] /= 2;
                KR.v[i] /= 2;
            }
        Matd R0(3, 3), R1(3, 3), P0(3, 4), P1(3, 4), Q(4, 4);
        mvsv_rect roi0{}, roi1{};
        if (mvsv_stereo_rectify(KL.data(), mDistCoeffsLeft.empty() ? nullptr : mDistCoeffsLeft.data(),
                                (int)mDistCoeffsLeft.v.size(), KR.data(),
                                mDistCoeffsRight.empty() ? nullptr : mDistCoeffsRight.data(),
                                (int)mDistCoeffsRight.v.size(), mWidth, mHeight, mR.data(), mT.data(),
                                MVSV_CALIB_ZERO_DISPARITY, 0.0, R0.v.data(), R1.v.data(), P0.v.data(),
                                P1.v.data(), Q.v.data(), &roi0, &roi1) != MVSV_OK) {
            log_error("Unable to init rectification\n");
            return false;
        }
        mR0 = R0;
        mR1 = R1;
        mP0 = P0;
        mP1 = P1;
        mQ = Q;
        mValidROI[0] = roi0;
        mValidROI[1] = roi1;
        const size_t px = (size_t)mWidth * mHeight;
        for (int c = 0; c < 2; c++) {
            mMap1[c].assign(px, 0.f);
            mMap2[c].assign(px, 0.f);
            const Matd& K = c ? KR : KL;
            const Matd& D = c ? mDistCoeffsRight : mDistCoeffsLeft;
            const Matd& R = c ? R1 : R0;
            const Matd& P = c ? P1 : P0;
            double P3[9];
            for (int r = 0; r < 3; r++)
                for (int k = 0; k < 3; k++) P3[r * 3 + k] = P.at(r, k);
            if (mvsv_init_undistort_rectify_map(K.data(), D.empty() ? nullptr : D.data(), (int)D.v.size(),
                                                R.data(), P3, mWidth, mHeight, mMap1[c].data(),
                                                mMap2[c].data(), mWidth) != MVSV_OK) {
                log_error("Unable to init rectification\n");
                return false;
            }
        }
        // mDisplayROI = mValidROI[0] & mValidROI[1]
        mDisplayROI = {std::max(roi0.x0, roi1.x0), std::max(roi0.y0, roi1.y0), std::min(roi0.x1, roi1.x1),
                       std::min(roi0.y1, roi1.y1)};
        if (mDisplayROI.x1 <= mDisplayROI.x0 || mDisplayROI.y1 <= mDisplayROI.y0) mDisplayROI = {0, 0, 0, 0};
        log_info("Rectification successfully initialized! [" + std::to_string(mDisplayROI.x1 - mDisplayROI.x0) +
                 " x " + std::to_string(mDisplayROI.y1 - mDisplayROI.y0) + " from (" +
                 std::to_string(mDisplayROI.x0) + ", " + std::to_string(mDisplayROI.y0) + ")]\n");
        mIsInit = true;
        return true;
    }

    // remap the raw pair in sip (mWidth x mHeight CV_8UC1) and crop it to the
    // display ROI
    bool getRectifiedImagepair(Stereopair& sip)
    {
        if (!mIsInit && !initRectification()) return false;
        return rectify(sip);
    }

    // ... and resize the crop by factor -- only when the rectification was
    // already initialised: the reference's initialising call returns the
    // unresized crop (src/Stereosystem.cpp:303-312)
    bool getRectifiedImagepair(Stereopair& sip, float factor)
    {
        if (mIsInit) {
            if (!rectify(sip)) return false;
            return resize_pair(sip, factor);
        }
        if (!initRectification()) return false;
        return rectify(sip);
    }

    void resetRectification() { mIsInit = false; }

    // --- load / save (src/Stereosystem.cpp:326-446) ---------------------------
    bool loadExtrinisic(std::string const& file)  // sic: the reference's spelling
    {
        mvsv_extrinsics v;
        const int rc = mvsv_load_extrinsic(file.c_str(), &v);
        if (rc == MVSV_E_PARSE) {
            log_error("Node in " + file + "is empty.\n");
            return false;
        }
        if (rc < 0) {
            log_error("Unable to open extrinsic file: " + file + "\n");
            return false;
        }
        mR = Matd::from(v.R);
        mT = Matd::from(v.T);
        mE = Matd::from(v.E);
        mF = Matd::from(v.F);
        log_info("Successfully loaded Extrinsics.\n");
        return true;
    }
    bool loadIntrinsic(std::string const& file)
    {
        mvsv_intrinsics v;
        const int rc = mvsv_load_intrinsic(file.c_str(), &v);
        if (rc == MVSV_E_PARSE) {
            log_error("Node in " + file + " is empty.\n");
            return false;
        }
        if (rc < 0) {
            log_error("Unable to open intrinsic file: " + file + "\n");
            return false;
        }
        mIntrinsicLeft = Matd::from(v.camera_matrix_left);
        mIntrinsicRight = Matd::from(v.camera_matrix_right);
        mDistCoeffsLeft = Matd::from(v.dist_coeffs_left);
        mDistCoeffsRight = Matd::from(v.dist_coeffs_right);
        log_info("Successfully loaded Intrinsics.\n");
        return true;
    }
    bool saveExtrinsic(std::string const& file)
    {
        mvsv_extrinsics v{mR.to(), mT.to(), mE.to(), mF.to()};
        if (mvsv_save_extrinsic(file.c_str(), &v) < 0) {
            log_error("Unable to open " + file + " for saving.\n");
            return false;
        }
        log_info("Successfully saved Extrinsics to " + file + "\n");
        return true;
    }
    bool saveIntrinsic(std::string const& file)
    {
        mvsv_intrinsics v{mIntrinsicLeft.to(),  mIntrinsicRight.to(), mDistCoeffsLeft.to(),
                          mDistCoeffsRight.to(), mP0.to(),           mP1.to(),
                          mQ.to()};
        if (mvsv_save_intrinsic(file.c_str(), &v) < 0) {
            log_error("Unable to open " + file + " for saving.\n");
            return false;
        }
        log_info("Successfully saved Intrinsics to " + file + "\n");
        return true;
    }

    // the state the reference keeps private, readable for tests / tools
    const mvsv_rect& displayROI() const { return mDisplayROI; }
    const std::vector<float>& map1(int c) const { return mMap1[c]; }
    const std::vector<float>& map2(int c) const { return mMap2[c]; }

private:
    void log_info(const std::string& m) const { std::fprintf(stderr, "%s%s", mTag.c_str(), m.c_str()); }
    void log_error(const std::string& m) const { std::fprintf(stderr, "%s%s", mTag.c_str(), m.c_str()); }

    bool rectify(Stereopair& sip)
    {
        const Mat& L = sip.mLeft;
        const Mat& R = sip.mRight;
        if (L.empty() || R.empty() || L.type != MAT_8UC1 || R.type != MAT_8UC1 || L.cols != mWidth ||
            L.rows != mHeight || R.cols != mWidth || R.rows != mHeight)
            return false;
        const int cw = mDisplayROI.x1 - mDisplayROI.x0, ch = mDisplayROI.y1 - mDisplayROI.y0;
        if (cw <= 0 || ch <= 0) return false;
        Mat oL(ch, cw, MAT_8UC1), oR(ch, cw, MAT_8UC1);
        const float* maps[4] = {mMap1[0].data(), mMap2[0].data(), mMap1[1].data(), mMap2[1].data()};
        mvsv_ctx* c = thread_context();
        check(mvsv_rectify_pair(c, L.data, L.step, R.data, R.step, mWidth, mHeight, maps, &mDisplayROI,
                                oL.data, oL.step, oR.data, oR.step),
              c);
        sip.mLeft = oL;
        sip.mRight = oR;
        return true;
    }
    bool resize_pair(Stereopair& sip, float factor)
    {
        Mat* im[2] = {&sip.mLeft, &sip.mRight};
        mvsv_ctx* c = thread_context();
        for (Mat* m : im) {
            int dw = 0, dh = 0;
            if (mvsv_resize_size(m->cols, m->rows, factor, factor, &dw, &dh) != MVSV_OK) return false;
            Mat o(dh, dw, MAT_8UC1);
            check(mvsv_resize(c, m->data, m->step, m->cols, m->rows, factor, factor, o.data, o.step), c);
            *m = o;
        }
        return true;
    }

    int mWidth, mHeight;
    bool mBinning;
    Matd mR, mT, mE, mF;
    bool mIsInit = false;
    std::vector<float> mMap1[2], mMap2[2];
    Matd mR0, mR1, mP0, mP1, mQ;
    mvsv_rect mValidROI[2] = {};
    mvsv_rect mDisplayROI = {};
    Matd mIntrinsicLeft, mIntrinsicRight, mDistCoeffsLeft, mDistCoeffsRight;
    std::string mTag;
};

}  // namespace mvsv

#endif  // MVSV_STEREOSYSTEM_HPP
