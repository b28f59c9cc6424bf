// Reference call pattern of the code around the path (trgt/mean_test.cpp:233-318,
// src/MeanDisparityDetection.cpp, src/utility.cpp:242-262) on include/mvsv_detection.hpp.
//   detection_check cpu OUT_DIR        host-only parts (ply, helpers, decisions)
//   detection_check gpu OUT_DIR        + stream, build() on the GPU grid, dmap2pcl
#include <cstdio>
#include <cstring>
#include <string>

#include "mvsv_detection.hpp"

static const mvsv::QMatrix Q = {1.f, 0.f, 0.f, -183.390320f, 0.f, 1.f, 0.f, -120.106110f,
                                0.f, 0.f, 0.f, 303.516571f,  0.f, 0.f, 0.00842495915f, 0.f};

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    const bool gpu = std::strcmp(argv[1], "gpu") == 0;
    const std::string dir = argv[2];
    try {
        // host parts
        mvsv::Mat dmap(96, 320, mvsv::MAT_16SC1);
        for (int y = 0; y < dmap.rows; y++)
            for (int x = 0; x < dmap.cols; x++) dmap.ptr<int16_t>(y)[x] = (int16_t)((x * 7 + y * 3) % 900 - 16);
        mvsv::Rect roi_u, roi_b;
        mvsv::createDMapROIS(dmap.rows, dmap.cols, 64, roi_u, roi_b);
        mvsv::Mat work = dmap(roi_u);
        mvsv::MeanDisparityDetection m(dir);
        m.init(work, Q, 0.1f, 1.5f);
        float means[81];
        for (int i = 0; i < 81; i++) means[i] = (float)(i * 80);
        m.build(work, 0, mvsv::MeanDisparityDetection::MEAN_VALUE, means);
        m.detectObstacles();
        std::printf("found %zu obstacles, counter %d\n", m.getFoundObstacles().size(), m.getObstacleCounter());
        mvsv::ply p("Hagen Hiller", "test", dmap);
        std::vector<std::array<float, 4>> pts = {{1.5f, -2.f, 3000.f, 1.f}, {0.f, 0.f, 100.f, 1.f}};
        if (!p.write(dir + "/two.ply", pts, mvsv::ply::WITH_COLOR)) return 3;
        std::printf("cpu ok\n");
        if (!gpu) return 0;
        // GPU parts: the camera loop as a stream, build() on the device grid, dmap2pcl
        auto sgbm = mvsv::StereoSGBM::create(0, 64, 9, 8 * 81, 32 * 81);
        std::vector<uint8_t> L(320 * 96), R(320 * 96);
        if (mvsv_synth_pair(0x5EED0000u + 90, 320, 96, 0, 64, L.data(), R.data()) != MVSV_OK) return 4;
        mvsv::Mat Lm = mvsv::Mat::wrap(L.data(), 96, 320, mvsv::MAT_8UC1, 320);
        mvsv::Mat Rm = mvsv::Mat::wrap(R.data(), 96, 320, mvsv::MAT_8UC1, 320);
        Stereopair s(Lm, Rm);
        mvsv::DisparityStream st(*sgbm, 320, 96, 2, &roi_u);
        st.setBatch(2);  // both frames in one frame-batch launch
        st.push(s);
        st.push(s);
        mvsv::Mat d1, d2;
        float g1[81], g2[81];
        st.pop(d1, g1);
        st.pop(d2, g2);
        mvsv::Mat direct;
        sgbm->compute(Lm, Rm, direct);
        for (int y = 0; y < 96; y++)
            if (std::memcmp(d1.ptr<int16_t>(y), direct.ptr<int16_t>(y), 640) ||
                std::memcmp(d2.ptr<int16_t>(y), direct.ptr<int16_t>(y), 640))
                return 5;
        // two frame-batch launches in flight on the stream's compute lanes
        {
            mvsv::DisparityStream st2(*sgbm, 320, 96, 4, &roi_u);
            st2.setInflight(2);
            for (int i = 0; i < 4; i++) st2.push(s);
            for (int i = 0; i < 4; i++) {
                mvsv::Mat di;
                float gi[81];
                st2.pop(di, gi);
                for (int y = 0; y < 96; y++)
                    if (std::memcmp(di.ptr<int16_t>(y), direct.ptr<int16_t>(y), 640)) return 7;
                if (std::memcmp(gi, g1, sizeof(gi))) return 8;
            }
        }
        mvsv::MeanDisparityDetection m2(dir);
        mvsv::Mat w2 = direct(roi_u);
        m2.init(w2, Q, 0.1f, 1.5f);
        m2.build(w2, 0, mvsv::MeanDisparityDetection::MEAN_VALUE);  // grid on the GPU
        for (int i = 0; i < 81; i++)
            if (m2.getMeanMap()[i] != g1[i]) return 6;
        mvsv::Utility::dmap2pcl(dir + "/cloud.ply", direct, Q);
        std::printf("gpu ok\n");
    } catch (const mvsv::Error& e) {
        std::printf("error: %s\n", e.what());
        return 1;
    }
    return 0;
}
