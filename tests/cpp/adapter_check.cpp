// C++ drop-in check: the reference's call pattern, compiled against
// include/mvsv_disparity.hpp and linked to libmvsv.so.
//   adapter_check cpu <configs dir>             loaders, defaults, errors (no GPU)
//   adapter_check gpu <configs dir> <out.bin>   Disparity::sgbm / ::bm on ROI views
#include <cstdio>
#include <cstring>
#include <string>

#include "mvsv_disparity.hpp"

#define REQUIRE(c)                                                              \
    do {                                                                        \
        if (!(c)) {                                                             \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

static int cpu_checks(const std::string& cfg)
{
    // trgt/mean_test.cpp:233-241 pattern
    auto sgbm = mvsv::StereoSGBM::create(0, 0, 0, 8 * 0 * 0, 32 * 0 * 0);
    Disparity::sgbmParameters para{};
    REQUIRE(Disparity::loadSGBMParameters(cfg + "/sgbm.yml", sgbm, para));
    REQUIRE(para.minDisp == 1 && para.numDisp == 128 && para.blockSize == 13);
    REQUIRE(para.speckleWindowSize == 150 && para.speckleRange == 2 && para.disparityMode == 0);
    REQUIRE(sgbm->getNumDisparities() == 128 && sgbm->getP1() == 0 && sgbm->getP2() == 0);
    REQUIRE(!Disparity::loadSGBMParameters(cfg + "/does_not_exist.yml", sgbm, para));
    auto bm = mvsv::StereoBM::create(64, 9);
    REQUIRE(bm->getPreFilterCap() == 31 && bm->getTextureThreshold() == 10);
    REQUIRE(Disparity::loadBMParameters(cfg + "/bm.yml", bm));
    REQUIRE(bm->getNumDisparities() == 80 && bm->getBlockSize() == 21);
    mvsv::Mat img(48, 64, mvsv::MAT_8UC1);
    mvsv::Mat roi = img(mvsv::Rect{4, 2, 40, 30});
    REQUIRE(roi.step == 64 && roi.cols == 40 && roi.data == img.data + 2 * 64 + 4);
    bool threw = false;
    try {
        (void)img(mvsv::Rect{40, 0, 40, 10});
    } catch (const mvsv::Error& e) {
        threw = e.code() == MVSV_E_INVALID_ARG;
    }
    REQUIRE(threw);
    std::printf("cpu ok\n");
    return 0;
}

static int gpu_run(const std::string& cfg, const std::string& out_path)
{
    const int W = 400, H = 200, X0 = 16, Y0 = 8, w = 320, h = 160;
    mvsv::Mat L(H, W, mvsv::MAT_8UC1), R(H, W, mvsv::MAT_8UC1);
    mvsv::check(mvsv_synth_pair(0x5EED0000u + 77, W, H, 1, 128, L.data, R.data), nullptr);
    Stereopair s(L, R);
    s.mLeft = L(mvsv::Rect{X0, Y0, w, h});  // cropped ROI views (src/Stereosystem.cpp:255-256)
    s.mRight = R(mvsv::Rect{X0, Y0, w, h});
    auto sgbm = mvsv::StereoSGBM::create(0, 0, 0, 0, 0);
    Disparity::sgbmParameters para{};
    REQUIRE(Disparity::loadSGBMParameters(cfg + "/sgbm.yml", sgbm, para));
    mvsv::Mat d1, d2;
    Disparity::sgbm(s, d1, sgbm);
    auto bm = mvsv::StereoBM::create(64, 9);
    Disparity::bm(s, d2, bm);
    REQUIRE(d1.rows == h && d1.cols == w && d1.type == mvsv::MAT_16SC1);
    FILE* f = std::fopen(out_path.c_str(), "wb");
    REQUIRE(f);
    std::fwrite(d1.data, 1, (size_t)w * h * 2, f);
    std::fwrite(d2.data, 1, (size_t)w * h * 2, f);
    std::fclose(f);
    // invalid parameters throw (OpenCV: cv::Exception)
    bool threw = false;
    try {
        auto bad = mvsv::StereoSGBM::create(0, 24, 5);
        Disparity::sgbm(s, d1, bad);
    } catch (const mvsv::Error& e) {
        threw = e.code() == MVSV_E_INVALID_ARG;
    }
    REQUIRE(threw);
    std::printf("gpu ok\n");
    return 0;
}

int main(int argc, char** argv)
{
    if (argc >= 3 && std::strcmp(argv[1], "cpu") == 0) return cpu_checks(argv[2]);
    if (argc >= 4 && std::strcmp(argv[1], "gpu") == 0) return gpu_run(argv[2], argv[3]);
    std::fprintf(stderr, "usage: adapter_check cpu|gpu <configs> [out]\n");
    return 2;
}
