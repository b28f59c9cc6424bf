// sanitize_driver.cpp — host code of libmvsv and the oracle under
// AddressSanitizer + UBSan (SURVEY.md §5 "race detection / sanitizers").
// Built and run by tests/test_sanitizers.py from:
//   mvstereovision3_amd/csrc/mvsv_io.cpp   YAML readers, calibration files,
//                                           stereoRectify, undistort maps, PLY,
//                                           synthetic pairs
//   mvstereovision3_amd/csrc/mvsv_ring.hpp frame-stream slot bookkeeping
//   oracle/mvsv_oracle.c                   the CPU checker (test infrastructure)
// Exit status 0 = every check passed and no sanitizer report.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "../../include/mvsv.h"
#include "../../mvstereovision3_amd/csrc/mvsv_ring.hpp"
#include "../../oracle/mvsv_oracle.h"

static int g_fail = 0;
#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                     \
        }                                                                 \
    } while (0)

static std::string slurp(const std::string& p)
{
    FILE* f = std::fopen(p.c_str(), "rb");
    if (!f) return "";
    std::string s;
    char buf[4096];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, n);
    std::fclose(f);
    return s;
}

static void yaml_loaders(const std::string& golden, const std::string& tmp)
{
    mvsv_sgbm_params p;
    mvsv_sgbm_params_default(&p);
    mvsv_sgbm_yaml_values v;
    CHECK(mvsv_load_sgbm_yaml((golden + "/configs/sgbm.yml").c_str(), &p, &v) == MVSV_OK);
    CHECK(v.numDisp == 128 && v.blockSize == 13 && p.num_disparities == 128);
    CHECK(mvsv_load_sgbm_yaml((tmp + "/nope.yml").c_str(), &p, &v) == MVSV_E_IO);
    mvsv_bm_params b;
    std::memset(&b, 0, sizeof b);
    CHECK(mvsv_load_bm_yaml((golden + "/configs/bm.yml").c_str(), &b) == MVSV_OK);
    // malformed inputs: long lines, no colon, garbage numbers, CRLF
    const std::string bad = tmp + "/bad.yml";
    FILE* f = std::fopen(bad.c_str(), "wb");
    std::fprintf(f, "%%YAML:1.0\r\nnumDisp: 1e400\r\nblockSize: abc\r\n%s\r\n: 5\r\nx\r\n",
                 std::string(10000, 'k').c_str());
    std::fclose(f);
    CHECK(mvsv_load_sgbm_yaml(bad.c_str(), &p, &v) == MVSV_E_PARSE);
}

static void calibration(const std::string& golden, const std::string& tmp)
{
    for (const char* sys : {"smallBL", "baseline_small", "foobar"}) {
        const std::string d = golden + "/calib/" + sys;
        mvsv_intrinsics in;
        mvsv_extrinsics ex;
        CHECK(mvsv_load_intrinsic((d + "/intrinsic.yml").c_str(), &in) == MVSV_OK);
        CHECK(mvsv_load_extrinsic((d + "/extrinsic.yml").c_str(), &ex) == MVSV_OK);
        CHECK(mvsv_save_intrinsic((tmp + "/i.yml").c_str(), &in) == MVSV_OK);
        CHECK(mvsv_save_extrinsic((tmp + "/e.yml").c_str(), &ex) == MVSV_OK);
        CHECK(slurp(tmp + "/i.yml") == slurp(d + "/intrinsic.yml"));
        CHECK(slurp(tmp + "/e.yml") == slurp(d + "/extrinsic.yml"));
        // stereoRectify + both undistort maps at the binned size
        double K1[9], K2[9];
        for (int i = 0; i < 9; i++) {
            K1[i] = in.camera_matrix_left.data[i] / (i == 8 ? 1 : 2);
            K2[i] = in.camera_matrix_right.data[i] / (i == 8 ? 1 : 2);
        }
        double R1[9], R2[9], P1[12], P2[12], Q[16];
        mvsv_rect r1, r2;
        const int W = 376, H = 240;
        CHECK(mvsv_stereo_rectify(K1, in.dist_coeffs_left.data,
                                  in.dist_coeffs_left.rows * in.dist_coeffs_left.cols, K2,
                                  in.dist_coeffs_right.data,
                                  in.dist_coeffs_right.rows * in.dist_coeffs_right.cols, W, H,
                                  ex.R.data, ex.T.data, MVSV_CALIB_ZERO_DISPARITY, 0.0, R1, R2,
                                  P1, P2, Q, &r1, &r2) == MVSV_OK);
        std::vector<float> mx((size_t)W * H), my((size_t)W * H);
        const double P3[9] = {P1[0], P1[1], P1[2], P1[4], P1[5], P1[6], P1[8], P1[9], P1[10]};
        CHECK(mvsv_init_undistort_rectify_map(K1, in.dist_coeffs_left.data, 5, R1, P3, W, H,
                                              mx.data(), my.data(), W) == MVSV_OK);
        CHECK(std::isfinite(mx[(size_t)W * H - 1]) && r1.x1 > r1.x0);
    }
    // a matrix node that overflows the 16-element limit, a truncated list
    FILE* f = std::fopen((tmp + "/big.yml").c_str(), "wb");
    std::fprintf(f, "%%YAML:1.0\nA: !!opencv-matrix\n   rows: 5\n   cols: 5\n   dt: d\n   data: [ 1. ]\n"
                    "B: !!opencv-matrix\n   rows: 1\n   cols: 3\n   dt: d\n   data: [ 1., 2.");
    std::fclose(f);
    mvsv_mat m;
    CHECK(mvsv_read_matrix_yaml((tmp + "/big.yml").c_str(), "A", &m) == MVSV_E_PARSE);
    CHECK(mvsv_read_matrix_yaml((tmp + "/big.yml").c_str(), "B", &m) == MVSV_E_PARSE);
}

static void ply_and_points(const std::string& tmp)
{
    const int W = 37, H = 11;
    std::vector<int16_t> d((size_t)W * H);
    for (size_t i = 0; i < d.size(); i++) d[i] = (int16_t)((i * 37) % 900 - 100);
    std::vector<float> xyz(3 * 50);
    for (size_t i = 0; i < xyz.size(); i++) xyz[i] = (float)i * 0.25f;
    CHECK(mvsv_write_ply((tmp + "/a.ply").c_str(), "a", "b", xyz.data(), 50, 3, MVSV_PLY_WITH_COLOR,
                         d.data(), W, W, H) == MVSV_OK);
    CHECK(mvsv_write_ply((tmp + "/b.ply").c_str(), "a", "b", xyz.data(), 50, 3, MVSV_PLY_PLAIN,
                         nullptr, 0, 0, 0) == MVSV_OK);
    const float Q[16] = {1, 0, 0, -10, 0, 1, 0, -5, 0, 0, 0, 300, 0, 0, 0.01f, 0};
    float out[4];
    mvsv_calc_coordinate(3.f, 4.f, 160.f, Q, out);
    CHECK(std::isfinite(out[2]));
    std::vector<uint8_t> L((size_t)W * H), R((size_t)W * H);
    CHECK(mvsv_synth_pair(0x5EED0000u, W, H, 0, 16, L.data(), R.data()) == MVSV_OK);
}

static void oracle_small(void)
{
    const int W = 83, H = 29;
    std::vector<uint8_t> L((size_t)W * H), R((size_t)W * H);
    mvsv_synth_pair(0x5EED0001u, W, H, 0, 16, L.data(), R.data());
    std::vector<int16_t> out((size_t)W * H), out2((size_t)W * H);
    for (int mode = 0; mode < 2; mode++) {
        orc_sgbm_params p = {-3, 32, 5, 0, 0, 1, 0, 10, 20, 2, mode};
        CHECK(orc_sgbm_compute(L.data(), W, R.data(), W, W, H, &p, 0, out.data(), W) == 0);
        CHECK(orc_sgbm_compute(L.data(), W, R.data(), W, W, H, &p, ORC_F_FIRSTCOL_FIX | ORC_F_WTA_MIN_D,
                               out2.data(), W) == 0);
    }
    orc_bm_params b = {1, 9, 31, 9, 0, 16, 10, 15, 30, 2, 1};
    CHECK(orc_bm_compute(L.data(), W, R.data(), W, W, H, &b, out.data(), W) == 0);
    b.pre_filter_type = 0;
    CHECK(orc_bm_compute(L.data(), W, R.data(), W, W, H, &b, out.data(), W) == 0);
    orc_median3x3_s16(out.data(), W, W, H, out2.data(), W);
    CHECK(orc_filter_speckles_s16(out2.data(), W, W, H, -16, 15, 16) >= 0);
    float means[81];
    orc_mean_disparity_grid(out2.data(), W, W, H, means);
    std::vector<float> mapx((size_t)W * H), mapy((size_t)W * H);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            mapx[(size_t)y * W + x] = x * 1.1f - 3.f;
            mapy[(size_t)y * W + x] = y * 0.9f + 0.5f;
        }
    std::vector<uint8_t> dst((size_t)W * H);
    orc_remap_linear(L.data(), W, W, H, mapx.data(), mapy.data(), dst.data(), W, H);
}

// Random push / pop / set_batch sequences against the ring invariants.
static void ring_bookkeeping(void)
{
    std::mt19937 rng(7);
    for (int trial = 0; trial < 2000; trial++) {
        const long depth = 1 + rng() % 16;
        int batch = 1 + (int)(rng() % depth);
        long head = 0, tail = 0, launched = 0;
        std::vector<int> launches_of((size_t)4096, 0);
        auto launch_all = [&]() {
            mvsv::RingRun r;
            while (mvsv::ring_next_run(launched, head, depth, &r)) {
                CHECK(r.n >= 1 && r.i0 >= 0 && r.i0 + r.n <= depth);
                for (int k = 0; k < r.n; k++) {
                    CHECK((launched + k) % depth == r.i0 + k);
                    launches_of[(size_t)(launched + k)]++;
                }
                launched += r.n;
            }
        };
        for (int op = 0; op < 300 && head < 4000; op++) {
            const int what = (int)(rng() % 7);
            if (what < 4) {  // push
                if (mvsv::ring_full(head, tail, depth)) continue;
                head++;
                if (mvsv::ring_launch_after_push(head, launched, batch, depth)) launch_all();
                CHECK(head - launched < batch || head % depth == 0 || launched == head);
            } else if (what < 6) {  // pop
                if (head == tail) continue;
                if (tail >= launched) launch_all();
                CHECK(tail < launched);
                tail++;
            } else {  // set_batch: frames already pushed keep the old grouping
                launch_all();
                batch = 1 + (int)(rng() % depth);
            }
            CHECK(tail <= launched && launched <= head && head - tail <= depth);
        }
        launch_all();
        for (long fidx = 0; fidx < head; fidx++) CHECK(launches_of[(size_t)fidx] == 1);
    }
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s GOLDEN_DIR TMP_DIR\n", argv[0]);
        return 2;
    }
    yaml_loaders(argv[1], argv[2]);
    calibration(argv[1], argv[2]);
    ply_and_points(argv[2]);
    oracle_small();
    ring_bookkeeping();
    std::printf("sanitize_driver: %d failures\n", g_fail);
    return g_fail ? 1 : 0;
}
