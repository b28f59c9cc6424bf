// C++ Stereosystem mirror check (include/mvsv_stereosystem.hpp), linked to libmvsv.so.
//   stereosystem_check cpu <calib dir> <tmp dir>   calibration files + stereoRectify
//                                                  against the reference's own files (no GPU)
//   stereosystem_check gpu <calib dir> <tmp dir>   getRectifiedImagepair (both overloads):
//                                                  writes the raw pair and the outputs for
//                                                  the Python side to compare with the oracle
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>

#include "mvsv_stereosystem.hpp"

#define REQUIRE(c)                                                              \
    do {                                                                        \
        if (!(c)) {                                                             \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            return 1;                                                           \
        }                                                                       \
    } while (0)

static std::string slurp(const std::string& p)
{
    std::ifstream f(p, std::ios::binary);
    return std::string(std::istreambuf_iterator<char>(f), std::istreambuf_iterator<char>());
}

static bool same_mat(const mvsv::Matd& a, const mvsv_mat& b, bool as_float)
{
    if (a.rows != b.rows || a.cols != b.cols) return false;
    for (int i = 0; i < a.rows * a.cols; i++) {
        if (as_float ? ((float)a.v[i] != (float)b.data[i]) : (a.v[i] != b.data[i])) return false;
    }
    return true;
}

static int cpu_checks(const std::string& cal, const std::string& tmp)
{
    // trgt/obstacle.cpp:342-345: baseline_small, binning (376 x 240), initRectification
    mvsv::Stereosystem s(376, 240, true);
    REQUIRE(!s.loadIntrinsic(tmp + "/missing.yml"));
    REQUIRE(!s.loadExtrinisic(tmp + "/missing.yml"));
    REQUIRE(s.loadIntrinsic(cal + "/baseline_small/intrinsic.yml"));
    REQUIRE(s.loadExtrinisic(cal + "/baseline_small/extrinsic.yml"));
    mvsv::Matd T;
    s.getTranslationMatrix(T);
    REQUIRE(T.rows == 3 && T.cols == 1);
    REQUIRE(s.getBaseline() == std::sqrt(std::pow(T.at(0, 0), 2) + std::pow(T.at(1, 0), 2) +
                                         std::pow(T.at(2, 0), 2)));
    REQUIRE(s.getRotationMatrix().rows == 3);
    REQUIRE(s.initRectification());
    mvsv_mat q, kl, kr;
    const std::string after = cal + "/afterCalibrationParameters.yml";
    REQUIRE(mvsv_read_matrix_yaml(after.c_str(), "Q", &q) == MVSV_OK);
    REQUIRE(mvsv_read_matrix_yaml(after.c_str(), "K_L", &kl) == MVSV_OK);
    REQUIRE(mvsv_read_matrix_yaml(after.c_str(), "K_R", &kr) == MVSV_OK);
    REQUIRE(same_mat(s.getQMatrix(), q, true));       // Q is CV_32F in the file
    REQUIRE(same_mat(s.getNewKMats()[0], kl, false));  // %.16e: every bit
    REQUIRE(same_mat(s.getNewKMats()[1], kr, false));
    const mvsv_rect roi = s.displayROI();
    REQUIRE(0 <= roi.x0 && roi.x0 < roi.x1 && roi.x1 <= 376 && 0 <= roi.y0 && roi.y0 < roi.y1 && roi.y1 <= 240);
    // load + save gives the reference's bytes back (its saveIntrinsic wrote them)
    for (const char* sys : {"smallBL", "baseline_small", "foobar"}) {
        mvsv::Stereosystem t(752, 480);
        REQUIRE(t.loadIntrinsic(cal + "/" + sys + "/intrinsic.yml"));
        REQUIRE(t.loadExtrinisic(cal + "/" + sys + "/extrinsic.yml"));
        REQUIRE(t.saveIntrinsic(tmp + "/intrinsic.yml"));
        REQUIRE(t.saveExtrinsic(tmp + "/extrinsic.yml"));
        REQUIRE(slurp(tmp + "/intrinsic.yml") == slurp(cal + "/" + sys + "/intrinsic.yml"));
        REQUIRE(slurp(tmp + "/extrinsic.yml") == slurp(cal + "/" + sys + "/extrinsic.yml"));
    }
    REQUIRE(!s.saveIntrinsic(tmp + "/no/such/dir/x.yml"));
    std::printf("cpu ok\n");
    return 0;
}

static bool dump(const std::string& path, const mvsv::Mat& m)
{
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    std::fprintf(f, "%d %d\n", m.rows, m.cols);
    for (int y = 0; y < m.rows; y++) std::fwrite(m.ptr<uint8_t>(y), 1, (size_t)m.cols, f);
    std::fclose(f);
    return true;
}

static int gpu_run(const std::string& cal, const std::string& tmp)
{
    const int W = 376, H = 240;
    mvsv::Stereosystem s(W, H, true);
    REQUIRE(s.loadIntrinsic(cal + "/baseline_small/intrinsic.yml"));
    REQUIRE(s.loadExtrinisic(cal + "/baseline_small/extrinsic.yml"));
    mvsv::Mat L(H, W, mvsv::MAT_8UC1), R(H, W, mvsv::MAT_8UC1);
    mvsv::check(mvsv_synth_pair(0x5EED0000u + 31, W, H, 0, 64, L.data, R.data), nullptr);
    REQUIRE(dump(tmp + "/raw_l.bin", L) && dump(tmp + "/raw_r.bin", R));
    // first call initialises: the factor overload then returns the unresized crop
    Stereopair a(L, R);
    REQUIRE(s.getRectifiedImagepair(a, 0.5f));
    REQUIRE(dump(tmp + "/init_l.bin", a.mLeft) && dump(tmp + "/init_r.bin", a.mRight));
    Stereopair b(L, R);
    REQUIRE(s.getRectifiedImagepair(b));
    REQUIRE(dump(tmp + "/rect_l.bin", b.mLeft) && dump(tmp + "/rect_r.bin", b.mRight));
    const float factors[] = {0.5f, 0.75f, 1.5f, 0.3f};
    for (float f : factors) {
        Stereopair c(L, R);
        REQUIRE(s.getRectifiedImagepair(c, f));
        char name[64];
        std::snprintf(name, sizeof name, "/res_%g", (double)f);
        REQUIRE(dump(tmp + name + "_l.bin", c.mLeft) && dump(tmp + name + "_r.bin", c.mRight));
    }
    s.resetRectification();
    Stereopair d(L, R);
    REQUIRE(s.getRectifiedImagepair(d, 0.5f));  // re-initialises: unresized again
    REQUIRE(d.mLeft.cols == b.mLeft.cols && d.mLeft.rows == b.mLeft.rows);
    std::printf("gpu ok\n");
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s cpu|gpu <calib dir> <tmp dir>\n", argv[0]);
        return 2;
    }
    if (!std::strcmp(argv[1], "cpu")) return cpu_checks(argv[2], argv[3]);
    return gpu_run(argv[2], argv[3]);
}
