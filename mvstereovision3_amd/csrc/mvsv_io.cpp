// mvsv_io.cpp — host-only parts of libmvsv (no HIP): the configs/*.yml
// readers, the synthetic pair generator, the per-point Utility helpers, the PLY
// writer, cv::FileStorage calibration matrices (Stereosystem::load/save
// Intrinsic/Extrinsic) and the rectification geometry (cv::stereoRectify,
// cv::initUndistortRectifyMap).  Kept free of HIP so the CPU suite can build it
// with AddressSanitizer + UBSan (tests/test_sanitizers.py).
#include <algorithm>
#include <cerrno>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/mvsv.h"

extern "C" {

int mvsv_version(void) { return MVSV_VERSION; }

void mvsv_sgbm_params_create(mvsv_sgbm_params* p, int min_disparity, int num_disparities,
                             int block_size, int p1, int p2, int disp12_max_diff,
                             int pre_filter_cap, int uniqueness_ratio, int speckle_window_size,
                             int speckle_range, int mode)
{
    if (!p) return;
    p->min_disparity = min_disparity;
    p->num_disparities = num_disparities;
    p->block_size = block_size;
    p->p1 = p1;
    p->p2 = p2;
    p->disp12_max_diff = disp12_max_diff;
    p->pre_filter_cap = pre_filter_cap;
    p->uniqueness_ratio = uniqueness_ratio;
    p->speckle_window_size = speckle_window_size;
    p->speckle_range = speckle_range;
    p->mode = mode;
    p->variant = 0;
}

void mvsv_sgbm_params_default(mvsv_sgbm_params* p)
{
    mvsv_sgbm_params_create(p, 0, 16, 3, 0, 0, 0, 0, 0, 0, 0, MVSV_MODE_SGBM);
}

void mvsv_bm_params_default(mvsv_bm_params* p, int num_disparities, int block_size)
{
    if (!p) return;
    p->pre_filter_type = MVSV_PREFILTER_XSOBEL;
    p->pre_filter_size = 9;
    p->pre_filter_cap = 31;
    p->block_size = block_size;
    p->min_disparity = 0;
    p->num_disparities = num_disparities > 0 ? num_disparities : 64;
    p->texture_threshold = 10;
    p->uniqueness_ratio = 15;
    p->speckle_window_size = 0;
    p->speckle_range = 0;
    p->disp12_max_diff = -1;
}

// ---------------------------------------------------------------------------
// Flat %YAML:1.0 "key: number" reader (the subset cv::FileStorage writes for
// configs/sgbm.yml and configs/bm.yml). Numbers are rounded like cvRound.
// ---------------------------------------------------------------------------
static int read_flat_yaml(const char* path, std::map<std::string, double>* kv)
{
    if (!path) return MVSV_E_INVALID_ARG;
    std::ifstream f(path);
    if (!f.is_open()) return MVSV_E_IO;
    std::string line;
    bool first = true;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (first) {
            first = false;
            if (line.rfind("%YAML", 0) == 0) continue;
        }
        size_t hash = line.find('#');
        if (hash != std::string::npos) line = line.substr(0, hash);
        if (line.find_first_not_of(" \t") == std::string::npos) continue;
        if (line == "---" || line == "...") continue;
        size_t colon = line.find(':');
        if (colon == std::string::npos) continue;
        std::string key = line.substr(0, colon);
        std::string val = line.substr(colon + 1);
        auto trim = [](std::string& s) {
            size_t a = s.find_first_not_of(" \t\"'");
            size_t b = s.find_last_not_of(" \t\"'");
            s = a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
        };
        trim(key);
        trim(val);
        if (key.empty() || val.empty()) continue;  // nested map / empty node
        char* end = nullptr;
        errno = 0;
        double d = std::strtod(val.c_str(), &end);
        if (end == val.c_str() || errno) continue;  // non-numeric: not an int node
        (*kv)[key] = d;
    }
    return MVSV_OK;
}

static int kv_int(const std::map<std::string, double>& kv, const char* key, int dflt)
{
    auto it = kv.find(key);
    return it == kv.end() ? dflt : (int)std::lrint(it->second);
}

int mvsv_load_sgbm_yaml(const char* path, mvsv_sgbm_params* p, mvsv_sgbm_yaml_values* v)
{
    std::map<std::string, double> kv;
    int rc = read_flat_yaml(path, &kv);
    if (rc) return rc;  // reference: LOG(ERROR) "Unable to open disparity parameters"
    // src/disparity.cpp:67 — required nodes
    for (const char* k : {"numDisp", "blockSize", "speckleWindowSize", "speckleWindowRange"})
        if (!kv.count(k)) return MVSV_E_PARSE;
    mvsv_sgbm_yaml_values tmp;
    tmp.minDisp = kv_int(kv, "minDisp", 0);
    tmp.numDisp = kv_int(kv, "numDisp", 0);
    tmp.blockSize = kv_int(kv, "blockSize", 0);
    tmp.disp12MaxDiff = kv_int(kv, "disp12MaxDiff", 0);
    tmp.preFilterCap = kv_int(kv, "preFilterCap", 0);
    tmp.uniquenessRatio = kv_int(kv, "uniquenessRatio", 0);
    tmp.speckleWindowSize = kv_int(kv, "speckleWindowSize", 0);
    tmp.speckleRange = kv_int(kv, "speckleWindowRange", 0);
    tmp.disparityMode = kv_int(kv, "mode", 0);
    if (v) *v = tmp;
    if (p) {  // src/disparity.cpp:83-95 — eight setters + mode, P1/P2 untouched
        p->min_disparity = tmp.minDisp;
        p->num_disparities = tmp.numDisp;
        p->block_size = tmp.blockSize;
        p->pre_filter_cap = tmp.preFilterCap;
        p->uniqueness_ratio = tmp.uniquenessRatio;
        p->disp12_max_diff = tmp.disp12MaxDiff;
        p->speckle_window_size = tmp.speckleWindowSize;
        p->speckle_range = tmp.speckleRange;
        p->mode = tmp.disparityMode == 1 ? MVSV_MODE_HH : MVSV_MODE_SGBM;
    }
    return MVSV_OK;
}

int mvsv_load_bm_yaml(const char* path, mvsv_bm_params* p)
{
    std::map<std::string, double> kv;
    int rc = read_flat_yaml(path, &kv);
    if (rc) return rc;
    for (const char* k : {"numDisp", "blockSize"})
        if (!kv.count(k)) return MVSV_E_PARSE;
    if (p) {
        p->num_disparities = kv_int(kv, "numDisp", p->num_disparities);
        p->block_size = kv_int(kv, "blockSize", p->block_size);
        p->pre_filter_cap = kv_int(kv, "preFilterCap", p->pre_filter_cap);
        p->pre_filter_size = kv_int(kv, "preFilterSize", p->pre_filter_size);
        p->uniqueness_ratio = kv_int(kv, "uniquenessRatio", p->uniqueness_ratio);
        p->texture_threshold = kv_int(kv, "textureThreshold", p->texture_threshold);
        p->min_disparity = kv_int(kv, "minDisp", p->min_disparity);
        p->speckle_window_size = kv_int(kv, "speckleWindowSize", p->speckle_window_size);
        p->speckle_range = kv_int(kv, "speckleWindowRange", p->speckle_range);
        p->disp12_max_diff = kv_int(kv, "disp12MaxDiff", p->disp12_max_diff);
        p->pre_filter_type = kv_int(kv, "preFilterType", p->pre_filter_type);
    }
    return MVSV_OK;
}

// ---------------------------------------------------------------------------
// Synthetic rectified pair.
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {
struct Pcg32 {
    uint64_t state;
    static constexpr uint64_t inc = 0xda3e39cb94b95bdbULL;
    explicit Pcg32(uint32_t seed) : state((uint64_t)seed * 2u + 1u) {}
    uint32_t next()
    {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((0u - rot) & 31u));
    }
};
}  // namespace

extern "C" {

int mvsv_synth_pair(uint32_t seed, int W, int H, int minD, int D, uint8_t* Lout, uint8_t* Rout)
{
    if (W <= 0 || H <= 0 || D <= 0 || !Lout || !Rout) return MVSV_E_INVALID_ARG;
    Pcg32 rng(seed);
    size_t np = (size_t)W * H;
    uint8_t* noise = (uint8_t*)std::malloc(np);
    if (!noise) return MVSV_E_OOM;
    for (size_t i = 0; i < np; i++) noise[i] = (uint8_t)(rng.next() >> 24);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            int s = 0;
            for (int dy = -1; dy <= 1; dy++)
                for (int dx = -1; dx <= 1; dx++) {
                    int yy = std::min(std::max(y + dy, 0), H - 1);
                    int xx = std::min(std::max(x + dx, 0), W - 1);
                    s += noise[(size_t)yy * W + xx];
                }
            Lout[(size_t)y * W + x] = (uint8_t)((2 * s + 9) / 18);  // round half up of s/9
        }
    std::free(noise);
    const int rect = (int)std::floor(0.6 * D + 0.5);
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            bool in = x >= W / 3 && x < 2 * W / 3 && y >= H / 3 && y < 2 * H / 3;
            int d = in ? rect : (int)std::floor(D / 8.0 + (D / 4.0) * y / H + 0.5);
            d = std::min(std::max(d, minD), minD + D - 1);
            int xs = std::min(std::max(x + d, 0), W - 1);
            int v = Lout[(size_t)y * W + xs] + (int)(rng.next() % 3u) - 1;
            Rout[(size_t)y * W + x] = (uint8_t)std::min(std::max(v, 0), 255);
        }
    return MVSV_OK;
}


// [Utility::calcCoordinate] src/utility.cpp:176-198 with OpenCV's float matrix
// product (double accumulation, one rounding) and Mat /= w (float scale).
void mvsv_calc_coordinate(float image_x, float image_y, float d_value, const float* Q, float* out)
{
    const float c[4] = {image_x, image_y, d_value / 16, 1.0f};
    float r[4];
    for (int i = 0; i < 4; i++) {
        double acc = 0.0;
        for (int k = 0; k < 4; k++) acc += (double)Q[4 * i + k] * (double)c[k];
        r[i] = (float)acc;
    }
    const float alpha = (float)(1.0 / (double)r[3]);
    for (int i = 0; i < 4; i++) out[i] = r[i] * alpha;
    if (std::isinf(out[2] / 1000)) out[2] = 0.0f;
}

void mvsv_calc_coordinates(int n, const float* xyd, const float* Q, float* out4)
{
    for (int i = 0; i < n; i++) mvsv_calc_coordinate(xyd[3 * i], xyd[3 * i + 1], xyd[3 * i + 2], Q, out4 + 4 * i);
}

// [Utility::calcDistance] src/utility.cpp:200-222
float mvsv_calc_distance(float image_x, float image_y, float d_value, const float* Q)
{
    const float c[4] = {image_x, image_y, d_value / 16, 1.0f};
    float r[4];
    for (int i = 0; i < 4; i++) {
        double acc = 0.0;
        for (int k = 0; k < 4; k++) acc += (double)Q[4 * i + k] * (double)c[k];
        r[i] = (float)acc;
    }
    const float alpha = (float)(1.0 / (double)r[3]);
    const float distance = (r[2] * alpha) / 1000;
    return std::isinf(distance) ? 0.0f : distance;
}

// [Utility::calcDMapValues] src/utility.cpp:224-240
void mvsv_calc_dmap_values(const float* c, const float* Q, float* image_x, float* image_y,
                           float* d_value)
{
    const float numerator = Q[2 * 4 + 3] - c[2] * Q[3 * 4 + 3];
    const float denominator = c[2] * Q[3 * 4 + 2];
    const float disparity_value = numerator / denominator;
    *image_x = c[0] * (disparity_value * Q[3 * 4 + 2] * Q[3 * 4 + 3]) + Q[0 * 4 + 3];
    *image_y = c[1] * (disparity_value * Q[3 * 4 + 2] * Q[3 * 4 + 3]) + Q[1 * 4 + 3];
    *d_value = disparity_value * 16;
}

// [Utility::calcMinMaxDisparity] src/utility.cpp:286-303 (positive values only)
static bool min_max_positive(const int16_t* d, size_t st, int W, int H, short* mn, short* mx)
{
    bool any = false;
    for (int r = 0; r < H; r++)
        for (int c = 0; c < W; c++) {
            const short v = d[(size_t)r * st + c];
            if (v > 0) {
                if (!any || v < *mn) *mn = v;
                if (!any || v > *mx) *mx = v;
                any = true;
            }
        }
    return any;
}

// [ply::write] src/ply.cpp:37-133: std::ofstream with default float formatting
int mvsv_write_ply(const char* path, const char* author, const char* object_name,
                   const float* xyz, size_t count, size_t vstride, int mode, const int16_t* dmap,
                   size_t dst, int W, int H)
{
    if (!path || (!xyz && count) || vstride < 3 || mode < MVSV_PLY_PLAIN ||
        mode > MVSV_PLY_WITH_COLOR_SHADING)
        return MVSV_E_INVALID_ARG;
    short mn = 0, mx = 0;
    if (mode != MVSV_PLY_PLAIN) {
        if (!dmap || W <= 0 || H <= 0) return MVSV_E_INVALID_ARG;  // "mDMap.rows == 0" -> false
        if (!min_max_positive(dmap, dst, W, H, &mn, &mx)) return MVSV_E_INVALID_ARG;
    }
    std::ofstream out(path);
    if (!out) return MVSV_E_IO;
    out << "ply\nformat ascii 1.0\ncomment author: " << (author ? author : "")
        << "\ncomment object:" << (object_name ? object_name : "") << "\n";
    out << "element vertex " << std::to_string(count) << "\n";
    out << "property float x\nproperty float y\nproperty float z\n";
    if (mode != MVSV_PLY_PLAIN) out << "property uchar red\nproperty uchar green\nproperty uchar blue\n";
    out << "end_header\n";
    for (size_t i = 0; i < count; i++) {
        const float* t = xyz + i * vstride;
        if (mode == MVSV_PLY_WITH_COLOR) {
            out << t[0] << " " << t[1] << " " << t[2] << " ";
            const int g = int((t[2] - mn) / (mx - mn) * 255.0);
            out << g << " " << g << " " << g << "\n";
        } else {
            out << t[0] << " " << t[1] << " " << t[2] << "\n";
        }
    }
    return out ? MVSV_OK : MVSV_E_IO;
}


// [cv::initUndistortRectifyMap] (OpenCV 3.4 undistort.cpp), CV_32FC1 output
int mvsv_init_undistort_rectify_map(const double* K, const double* dist, int ndist,
                                    const double* Rm, const double* P, int W, int H, float* mx,
                                    float* my, size_t ms)
{
    if (!K || !P || !mx || !my || W <= 0 || H <= 0 || ms < (size_t)W ||
        !(ndist == 0 || ndist == 4 || ndist == 5 || ndist == 8) || (ndist && !dist))
        return MVSV_E_INVALID_ARG;
    const double I3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    const double* R = Rm ? Rm : I3;
    // A = P[:, :3] * R; iR = A^-1
    double A[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double acc = 0;
            for (int k = 0; k < 3; k++) acc += P[i * 3 + k] * R[k * 3 + j];
            A[i * 3 + j] = acc;
        }
    const double det = A[0] * (A[4] * A[8] - A[5] * A[7]) - A[1] * (A[3] * A[8] - A[5] * A[6]) +
                       A[2] * (A[3] * A[7] - A[4] * A[6]);
    if (det == 0) return MVSV_E_INVALID_ARG;
    double ir[9] = {(A[4] * A[8] - A[5] * A[7]) / det, (A[2] * A[7] - A[1] * A[8]) / det,
                    (A[1] * A[5] - A[2] * A[4]) / det, (A[5] * A[6] - A[3] * A[8]) / det,
                    (A[0] * A[8] - A[2] * A[6]) / det, (A[2] * A[3] - A[0] * A[5]) / det,
                    (A[3] * A[7] - A[4] * A[6]) / det, (A[1] * A[6] - A[0] * A[7]) / det,
                    (A[0] * A[4] - A[1] * A[3]) / det};
    double k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < ndist; i++) k[i] = dist[i];
    const double k1 = k[0], k2 = k[1], p1 = k[2], p2 = k[3], k3 = k[4], k4 = k[5], k5 = k[6], k6 = k[7];
    const double u0 = K[2], v0 = K[5], fx = K[0], fy = K[4];
    for (int i = 0; i < H; i++) {
        float* m1 = mx + (size_t)i * ms;
        float* m2 = my + (size_t)i * ms;
        double _x = i * ir[1] + ir[2], _y = i * ir[4] + ir[5], _w = i * ir[7] + ir[8];
        for (int j = 0; j < W; j++, _x += ir[0], _y += ir[3], _w += ir[6]) {
            const double w = 1. / _w, x = _x * w, y = _y * w;
            const double x2 = x * x, y2 = y * y;
            const double r2 = x2 + y2, _2xy = 2 * x * y;
            const double kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2);
            const double u = fx * (x * kr + p1 * _2xy + p2 * (r2 + 2 * x2)) + u0;
            const double v = fy * (y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy) + v0;
            m1[j] = (float)u;
            m2[j] = (float)v;
        }
    }
    return MVSV_OK;
}

// ---------------------------------------------------------------------------
// cv::FileStorage YAML matrices, as Stereosystem::saveIntrinsic/saveExtrinsic
// write them (src/Stereosystem.cpp:388-446) and loadIntrinsic/loadExtrinisic
// read them back (:326-386).  The writer reproduces OpenCV 3.x persistence:
// "%YAML:1.0" header, "key: !!opencv-matrix" maps with rows / cols / dt, the
// elements as one flow list "data: [ ... ]" that breaks before an element
// which would end past column 71 (continuation indent 7), doubles as "%.16e"
// and floats as "%.8e" unless integral ("%d."), ".Nan" / ".Inf" / "-.Inf".
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

constexpr int kYmlWrap = 71;
constexpr int kYmlDataIndent = 7;  // CV_YML_INDENT (3) + map indent (3) + 1 (flow)

int round_half_even(double v) { return (int)std::lrint(v); }  // cvRound (SSE2 cvtsd2si)

std::string fmt_element(double v, char dt)
{
    char buf[64];
    if (dt == 'd' || dt == 'f') {
        const bool is_f = dt == 'f';
        const double x = is_f ? (double)(float)v : v;
        if (std::isnan(x)) return ".Nan";
        if (std::isinf(x)) return x < 0 ? "-.Inf" : ".Inf";
        if (std::fabs(x) < 2147483647.0 && (double)round_half_even(x) == x) {
            std::snprintf(buf, sizeof buf, "%d.", round_half_even(x));
        } else {
            std::snprintf(buf, sizeof buf, is_f ? "%.8e" : "%.16e", is_f ? (double)(float)x : x);
        }
        return buf;
    }
    std::snprintf(buf, sizeof buf, "%d", (int)v);
    return buf;
}

void write_matrix(std::string& out, const char* key, const mvsv_mat& m)
{
    out += key;
    out += ": !!opencv-matrix\n";
    out += "   rows: " + std::to_string(m.rows) + "\n";
    out += "   cols: " + std::to_string(m.cols) + "\n";
    out += "   dt: ";
    out += m.dt ? m.dt : 'u';
    out += "\n";
    std::string line = "   data: [";
    bool empty = true;
    const int n = m.rows * m.cols;
    for (int i = 0; i < n; i++) {
        const std::string d = fmt_element(m.data[i], m.dt);
        if (!empty) line += ',';
        const int new_offset = (int)(line.size() + d.size());
        if (new_offset > kYmlWrap && new_offset - kYmlDataIndent > 10) {
            out += line;
            out += '\n';
            line.assign(kYmlDataIndent, ' ');
        } else {
            line += ' ';
        }
        line += d;
        empty = false;
    }
    if (!empty && (int)line.size() > kYmlDataIndent) line += ' ';
    line += ']';
    out += line;
    out += '\n';
}

bool valid_dt(char c) { return std::strchr("ucwsifd", c) != nullptr && c; }

// All "key: !!opencv-matrix" nodes of a FileStorage YAML file.
int read_matrices(const char* path, std::map<std::string, mvsv_mat>* out)
{
    if (!path) return MVSV_E_INVALID_ARG;
    std::ifstream f(path);
    if (!f.is_open()) return MVSV_E_IO;
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    size_t pos = 0;
    const std::string tag = "!!opencv-matrix";
    while ((pos = text.find(tag, pos)) != std::string::npos) {
        size_t ls = text.rfind('\n', pos);
        ls = ls == std::string::npos ? 0 : ls + 1;
        std::string key = text.substr(ls, pos - ls);
        const size_t colon = key.rfind(':');
        pos += tag.size();
        if (colon == std::string::npos) continue;
        key = key.substr(0, colon);
        key.erase(0, key.find_first_not_of(" \t"));
        key.erase(key.find_last_not_of(" \t") + 1);
        mvsv_mat m;
        std::memset(&m, 0, sizeof m);
        auto field = [&](const char* name, std::string* val) -> bool {
            const size_t p = text.find(std::string(name) + ":", pos);
            if (p == std::string::npos) return false;
            const size_t e = text.find('\n', p);
            *val = text.substr(p + std::strlen(name) + 1, e == std::string::npos ? std::string::npos : e - p - std::strlen(name) - 1);
            val->erase(0, val->find_first_not_of(" \t"));
            val->erase(val->find_last_not_of(" \t\r") + 1);
            return true;
        };
        std::string rows, cols, dt;
        if (!field("rows", &rows) || !field("cols", &cols) || !field("dt", &dt)) return MVSV_E_PARSE;
        m.rows = std::atoi(rows.c_str());
        m.cols = std::atoi(cols.c_str());
        m.dt = dt.empty() ? 0 : dt[0];
        if (m.rows < 0 || m.cols < 0 || dt.size() != 1 || !valid_dt(m.dt) ||
            (long)m.rows * m.cols > MVSV_MAT_MAX)
            return MVSV_E_PARSE;
        const size_t lb = text.find('[', text.find("data:", pos));
        const size_t rb = lb == std::string::npos ? lb : text.find(']', lb);
        if (lb == std::string::npos || rb == std::string::npos) return MVSV_E_PARSE;
        std::string body = text.substr(lb + 1, rb - lb - 1);
        int n = 0;
        size_t q = 0;
        while (q <= body.size()) {
            size_t c = body.find(',', q);
            std::string tok = body.substr(q, c == std::string::npos ? std::string::npos : c - q);
            tok.erase(0, tok.find_first_not_of(" \t\r\n"));
            tok.erase(tok.find_last_not_of(" \t\r\n") + 1);
            if (!tok.empty()) {
                if (n >= m.rows * m.cols) return MVSV_E_PARSE;
                double v;
                if (tok == ".Nan" || tok == ".nan") v = NAN;
                else if (tok == ".Inf" || tok == ".inf") v = INFINITY;
                else if (tok == "-.Inf" || tok == "-.inf") v = -INFINITY;
                else {
                    char* end = nullptr;
                    v = std::strtod(tok.c_str(), &end);
                    if (end == tok.c_str()) return MVSV_E_PARSE;
                }
                m.data[n++] = v;
            }
            if (c == std::string::npos) break;
            q = c + 1;
        }
        if (n != m.rows * m.cols) return MVSV_E_PARSE;
        (*out)[key] = m;
        pos = rb;
    }
    return MVSV_OK;
}

int write_file(const char* path, const std::string& body)
{
    if (!path) return MVSV_E_INVALID_ARG;
    std::ofstream f(path, std::ios::binary);
    if (!f.is_open()) return MVSV_E_IO;
    f << "%YAML:1.0\n" << body;
    return f ? MVSV_OK : MVSV_E_IO;
}

void empty_mat(mvsv_mat* m)
{
    std::memset(m, 0, sizeof *m);
    m->dt = 'u';
}

}  // namespace

extern "C" {

int mvsv_read_matrix_yaml(const char* path, const char* key, mvsv_mat* out)
{
    if (!key || !out) return MVSV_E_INVALID_ARG;
    std::map<std::string, mvsv_mat> all;
    int rc = read_matrices(path, &all);
    if (rc) return rc;
    auto it = all.find(key);
    if (it == all.end()) return MVSV_E_PARSE;
    *out = it->second;
    return MVSV_OK;
}

int mvsv_write_matrices_yaml(const char* path, const char* const* keys, const mvsv_mat* mats, int n)
{
    if (n < 0 || (n && (!keys || !mats))) return MVSV_E_INVALID_ARG;
    std::string body;
    for (int i = 0; i < n; i++) {
        if (!keys[i] || mats[i].rows < 0 || mats[i].cols < 0 ||
            (long)mats[i].rows * mats[i].cols > MVSV_MAT_MAX)
            return MVSV_E_INVALID_ARG;
        write_matrix(body, keys[i], mats[i]);
    }
    return write_file(path, body);
}

// Stereosystem::loadIntrinsic (src/Stereosystem.cpp:356-386): the four nodes
// it checks must exist (it checks distCoeffsRight twice and never
// distCoeffsLeft, which then reads as an empty matrix when absent).
int mvsv_load_intrinsic(const char* path, mvsv_intrinsics* out)
{
    if (!out) return MVSV_E_INVALID_ARG;
    std::map<std::string, mvsv_mat> all;
    int rc = read_matrices(path, &all);
    if (rc) return rc;
    for (const char* k : {"cameraMatrixLeft", "cameraMatrixRight", "distCoeffsRight"})
        if (!all.count(k)) return MVSV_E_PARSE;
    mvsv_intrinsics v;
    for (mvsv_mat* m : {&v.camera_matrix_left, &v.camera_matrix_right, &v.dist_coeffs_left,
                        &v.dist_coeffs_right, &v.camera_matrix_left_new, &v.camera_matrix_right_new,
                        &v.q_matrix})
        empty_mat(m);
    v.camera_matrix_left = all["cameraMatrixLeft"];
    v.camera_matrix_right = all["cameraMatrixRight"];
    if (all.count("distCoeffsLeft")) v.dist_coeffs_left = all["distCoeffsLeft"];
    v.dist_coeffs_right = all["distCoeffsRight"];
    *out = v;
    return MVSV_OK;
}

// Stereosystem::loadExtrinisic (src/Stereosystem.cpp:326-354): R, T, E, F required.
int mvsv_load_extrinsic(const char* path, mvsv_extrinsics* out)
{
    if (!out) return MVSV_E_INVALID_ARG;
    std::map<std::string, mvsv_mat> all;
    int rc = read_matrices(path, &all);
    if (rc) return rc;
    for (const char* k : {"R", "T", "E", "F"})
        if (!all.count(k)) return MVSV_E_PARSE;
    out->R = all["R"];
    out->T = all["T"];
    out->E = all["E"];
    out->F = all["F"];
    return MVSV_OK;
}

// Stereosystem::saveIntrinsic (src/Stereosystem.cpp:418-446): seven nodes in this order.
int mvsv_save_intrinsic(const char* path, const mvsv_intrinsics* in)
{
    if (!in) return MVSV_E_INVALID_ARG;
    const char* keys[7] = {"cameraMatrixLeft", "cameraMatrixRight", "distCoeffsLeft",
                           "distCoeffsRight", "cameraMatrixLeftNew", "cameraMatrixRightNew",
                           "QMatrix"};
    const mvsv_mat mats[7] = {in->camera_matrix_left, in->camera_matrix_right,
                              in->dist_coeffs_left, in->dist_coeffs_right,
                              in->camera_matrix_left_new, in->camera_matrix_right_new,
                              in->q_matrix};
    return mvsv_write_matrices_yaml(path, keys, mats, 7);
}

// Stereosystem::saveExtrinsic (src/Stereosystem.cpp:388-416)
int mvsv_save_extrinsic(const char* path, const mvsv_extrinsics* in)
{
    if (!in) return MVSV_E_INVALID_ARG;
    const char* keys[4] = {"R", "T", "E", "F"};
    const mvsv_mat mats[4] = {in->R, in->T, in->E, in->F};
    return mvsv_write_matrices_yaml(path, keys, mats, 4);
}

// ---------------------------------------------------------------------------
// cv::stereoRectify (OpenCV 3.4 calibration.cpp, cvStereoRectify), as called by
// Stereosystem::initRectification (src/Stereosystem.cpp:209-212): rotate both
// cameras by half the relative rotation, then align the baseline with the x (or
// y) axis; common focal length from the smaller (distortion-corrected) f; with
// CALIB_ZERO_DISPARITY equal principal points; alpha scales between the
// inscribed (0) and the enclosing (1) rectangle of the undistorted images.
// Double-precision restatement: Rodrigues without OpenCV's SVD
// re-orthogonalisation of R, so results may differ in the last bits.
// ---------------------------------------------------------------------------
}  // extern "C"

namespace {

void mat3_mul(const double* A, const double* B, double* C, bool bt = false)
{
    double t[9];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += A[i * 3 + k] * (bt ? B[j * 3 + k] : B[k * 3 + j]);
            t[i * 3 + j] = s;
        }
    std::memcpy(C, t, sizeof t);
}

// cvRodrigues2, rotation vector -> matrix
void rodrigues_vec2mat(const double* r, double* R)
{
    const double theta = std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    if (theta < DBL_EPSILON) {
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        std::memcpy(R, I, sizeof I);
        return;
    }
    const double c = std::cos(theta), s = std::sin(theta), c1 = 1. - c;
    const double itheta = theta ? 1. / theta : 0.;
    const double x = r[0] * itheta, y = r[1] * itheta, z = r[2] * itheta;
    const double rrt[9] = {x * x, x * y, x * z, x * y, y * y, y * z, x * z, y * z, z * z};
    const double rx[9] = {0, -z, y, z, 0, -x, -y, x, 0};
    for (int k = 0; k < 9; k++) R[k] = c * (k % 4 == 0 ? 1. : 0.) + c1 * rrt[k] + s * rx[k];
}

// cvRodrigues2, matrix -> rotation vector
void rodrigues_mat2vec(const double* R, double* r)
{
    double rx = R[7] - R[5], ry = R[2] - R[6], rz = R[3] - R[1];
    double s = std::sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0] + R[4] + R[8] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = std::acos(c);
    if (s < 1e-5) {
        if (c > 0) {
            rx = ry = rz = 0;
        } else {
            double t;
            t = (R[0] + 1) * 0.5;
            rx = std::sqrt(std::max(t, 0.));
            t = (R[4] + 1) * 0.5;
            ry = std::sqrt(std::max(t, 0.)) * (R[1] < 0 ? -1. : 1.);
            t = (R[8] + 1) * 0.5;
            rz = std::sqrt(std::max(t, 0.)) * (R[2] < 0 ? -1. : 1.);
            if (std::fabs(rx) < std::fabs(ry) && std::fabs(rx) < std::fabs(rz) && (R[5] > 0) != (ry * rz > 0))
                rz = -rz;
            theta /= std::sqrt(rx * rx + ry * ry + rz * rz);
            rx *= theta;
            ry *= theta;
            rz *= theta;
        }
    } else {
        const double vth = 1 / (2 * s) * theta;
        rx *= vth;
        ry *= vth;
        rz *= vth;
    }
    r[0] = rx;
    r[1] = ry;
    r[2] = rz;
}

// cvUndistortPoints for one point (5 fixed-point iterations, OpenCV 3.4
// default criteria), then RR = P[:, :3] * R applied; P == nullptr -> identity.
void undistort_point(float& px, float& py, const double* K, const double* dist, int nd,
                     const double* R, const double* P)
{
    double k[14] = {0};
    for (int i = 0; i < nd && i < 14; i++) k[i] = dist[i];
    const double fx = K[0], fy = K[4], ifx = 1. / fx, ify = 1. / fy, cx = K[2], cy = K[5];
    double x = px, y = py;
    x = (x - cx) * ifx;
    y = (y - cy) * ify;
    if (nd > 0) {
        const double x0 = x, y0 = y;
        for (int j = 0; j < 5; j++) {
            const double r2 = x * x + y * y;
            const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                                  (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
            const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
            const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
            x = (x0 - deltaX) * icdist;
            y = (y0 - deltaY) * icdist;
        }
    }
    double RR[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    if (R) std::memcpy(RR, R, sizeof RR);
    if (P) {
        double P3[9] = {P[0], P[1], P[2], P[4], P[5], P[6], P[8], P[9], P[10]};
        mat3_mul(P3, RR, RR);
    }
    const double xx = RR[0] * x + RR[1] * y + RR[2];
    const double yy = RR[3] * x + RR[4] * y + RR[5];
    const double ww = 1. / (RR[6] * x + RR[7] * y + RR[8]);
    px = (float)(xx * ww);
    py = (float)(yy * ww);
}

struct RectF {
    float x, y, w, h;
};

// icvGetRectangles: inscribed / enclosing rectangles of the undistorted 9x9 grid
void get_rectangles(const double* K, const double* dist, int nd, const double* R, const double* P,
                    int W, int H, RectF& inner, RectF& outer)
{
    const int N = 9;
    float iX0 = -FLT_MAX, iX1 = FLT_MAX, iY0 = -FLT_MAX, iY1 = FLT_MAX;
    float oX0 = FLT_MAX, oX1 = -FLT_MAX, oY0 = FLT_MAX, oY1 = -FLT_MAX;
    for (int y = 0; y < N; y++)
        for (int x = 0; x < N; x++) {
            float px = (float)x * W / (N - 1), py = (float)y * H / (N - 1);
            undistort_point(px, py, K, dist, nd, R, P);
            oX0 = std::min(oX0, px);
            oX1 = std::max(oX1, px);
            oY0 = std::min(oY0, py);
            oY1 = std::max(oY1, py);
            if (x == 0) iX0 = std::max(iX0, px);
            if (x == N - 1) iX1 = std::min(iX1, px);
            if (y == 0) iY0 = std::max(iY0, py);
            if (y == N - 1) iY1 = std::min(iY1, py);
        }
    inner = {iX0, iY0, iX1 - iX0, iY1 - iY0};
    outer = {oX0, oY0, oX1 - oX0, oY1 - oY0};
}

mvsv_rect rect_and(mvsv_rect a, mvsv_rect b)  // cv::Rect & (as x0,y0,x1,y1)
{
    mvsv_rect r{std::max(a.x0, b.x0), std::max(a.y0, b.y0), std::min(a.x1, b.x1), std::min(a.y1, b.y1)};
    if (r.x1 <= r.x0 || r.y1 <= r.y0) r = {0, 0, 0, 0};
    return r;
}

}  // namespace

extern "C" {

int mvsv_stereo_rectify(const double* K1, const double* D1, int nd1, const double* K2,
                        const double* D2, int nd2, int W, int H, const double* Rm,
                        const double* T, int flags, double alpha, double* R1, double* R2,
                        double* P1, double* P2, double* Q, mvsv_rect* roi1, mvsv_rect* roi2)
{
    if (!K1 || !K2 || !Rm || !T || !R1 || !R2 || !P1 || !P2 || W <= 0 || H <= 0 || nd1 < 0 ||
        nd2 < 0 || nd1 > 14 || nd2 > 14 || (nd1 && !D1) || (nd2 && !D2))
        return MVSV_E_INVALID_ARG;
    // half rotation for each camera, then the baseline onto the x (or y) axis
    double om[3], r_r[9], t[3];
    rodrigues_mat2vec(Rm, om);
    for (double& v : om) v *= -0.5;
    rodrigues_vec2mat(om, r_r);
    for (int i = 0; i < 3; i++) t[i] = r_r[i * 3] * T[0] + r_r[i * 3 + 1] * T[1] + r_r[i * 3 + 2] * T[2];
    const int idx = std::fabs(t[0]) > std::fabs(t[1]) ? 0 : 1;
    const double c = t[idx], nt = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
    double uu[3] = {0, 0, 0};
    uu[idx] = c > 0 ? 1 : -1;
    double ww[3] = {t[1] * uu[2] - t[2] * uu[1], t[2] * uu[0] - t[0] * uu[2], t[0] * uu[1] - t[1] * uu[0]};
    const double nw = std::sqrt(ww[0] * ww[0] + ww[1] * ww[1] + ww[2] * ww[2]);
    if (nw > 0.0)
        for (double& v : ww) v *= std::acos(std::fabs(c) / nt) / nw;
    double wR[9];
    rodrigues_vec2mat(ww, wR);
    mat3_mul(wR, r_r, R1, true);  // Ri = wR * r_r^T
    mat3_mul(wR, r_r, R2);        // Ri = wR * r_r
    for (int i = 0; i < 3; i++) t[i] = R2[i * 3] * T[0] + R2[i * 3 + 1] * T[1] + R2[i * 3 + 2] * T[2];

    // common focal length
    double fc_new = DBL_MAX;
    const double* Ks[2] = {K1, K2};
    const double* Ds[2] = {D1, D2};
    const int nds[2] = {nd1, nd2};
    for (int k = 0; k < 2; k++) {
        const double dk1 = nds[k] > 0 ? Ds[k][0] : 0.;
        double fc = Ks[k][(idx ^ 1) * 3 + (idx ^ 1)];
        if (dk1 < 0) fc *= 1 + dk1 * ((double)W * W + (double)H * H) / (4 * fc * fc);
        fc_new = std::min(fc_new, fc);
    }
    // principal points: centre of the undistorted, rotated image corners
    double ccx[2], ccy[2];
    const double* Rs[2] = {R1, R2};
    for (int k = 0; k < 2; k++) {
        double sx = 0, sy = 0;
        for (int i = 0; i < 4; i++) {
            const int j = i < 2 ? 0 : 1;
            float px = (float)((i % 2) * (W - 1)), py = (float)(j * (H - 1));
            undistort_point(px, py, Ks[k], Ds[k], nds[k], nullptr, nullptr);
            // projectPoints of (px, py, 1) with R_k, t = 0, f = fc_new, c = 0
            const double X = px, Y = py, Z = 1.0;
            const double* R = Rs[k];
            const double xr = R[0] * X + R[1] * Y + R[2] * Z, yr = R[3] * X + R[4] * Y + R[5] * Z,
                         zr = R[6] * X + R[7] * Y + R[8] * Z;
            const double iz = zr ? 1. / zr : 1.;
            sx += (float)(fc_new * xr * iz);
            sy += (float)(fc_new * yr * iz);
        }
        ccx[k] = (W - 1) / 2. - sx / 4;
        ccy[k] = (H - 1) / 2. - sy / 4;
    }
    if (flags & MVSV_CALIB_ZERO_DISPARITY) {
        ccx[0] = ccx[1] = (ccx[0] + ccx[1]) * 0.5;
        ccy[0] = ccy[1] = (ccy[0] + ccy[1]) * 0.5;
    } else if (idx == 0) {
        ccy[0] = ccy[1] = (ccy[0] + ccy[1]) * 0.5;
    } else {
        ccx[0] = ccx[1] = (ccx[0] + ccx[1]) * 0.5;
    }
    for (int i = 0; i < 12; i++) P1[i] = P2[i] = 0;
    P1[0] = P1[5] = fc_new;
    P1[2] = ccx[0];
    P1[6] = ccy[0];
    P1[10] = 1;
    P2[0] = P2[5] = fc_new;
    P2[2] = ccx[1];
    P2[6] = ccy[1];
    P2[10] = 1;
    P2[idx * 4 + 3] = t[idx] * fc_new;

    alpha = std::min(alpha, 1.);
    RectF inner1, outer1, inner2, outer2;
    get_rectangles(K1, D1, nd1, R1, P1, W, H, inner1, outer1);
    get_rectangles(K2, D2, nd2, R2, P2, W, H, inner2, outer2);
    const double cx1_0 = ccx[0], cy1_0 = ccy[0], cx2_0 = ccx[1], cy2_0 = ccy[1];
    const double cx1 = W * cx1_0 / W, cy1 = H * cy1_0 / H, cx2 = W * cx2_0 / W, cy2 = H * cy2_0 / H;
    double s = 1.;
    if (alpha >= 0) {
        double s0 = std::max(std::max(std::max((double)cx1 / (cx1_0 - inner1.x), (double)cy1 / (cy1_0 - inner1.y)),
                                      (double)(W - cx1) / (inner1.x + inner1.w - cx1_0)),
                             (double)(H - cy1) / (inner1.y + inner1.h - cy1_0));
        s0 = std::max(std::max(std::max(std::max((double)cx2 / (cx2_0 - inner2.x), (double)cy2 / (cy2_0 - inner2.y)),
                                        (double)(W - cx2) / (inner2.x + inner2.w - cx2_0)),
                               (double)(H - cy2) / (inner2.y + inner2.h - cy2_0)),
                      s0);
        double s1 = std::min(std::min(std::min((double)cx1 / (cx1_0 - outer1.x), (double)cy1 / (cy1_0 - outer1.y)),
                                      (double)(W - cx1) / (outer1.x + outer1.w - cx1_0)),
                             (double)(H - cy1) / (outer1.y + outer1.h - cy1_0));
        s1 = std::min(std::min(std::min(std::min((double)cx2 / (cx2_0 - outer2.x), (double)cy2 / (cy2_0 - outer2.y)),
                                        (double)(W - cx2) / (outer2.x + outer2.w - cx2_0)),
                               (double)(H - cy2) / (outer2.y + outer2.h - cy2_0)),
                      s1);
        s = s0 * (1 - alpha) + s1 * alpha;
    }
    fc_new *= s;
    P1[0] = P1[5] = fc_new;
    P1[2] = cx1;
    P1[6] = cy1;
    P2[0] = P2[5] = fc_new;
    P2[2] = cx2;
    P2[6] = cy2;
    P2[idx * 4 + 3] *= s;
    const mvsv_rect full{0, 0, W, H};
    auto roi_of = [&](const RectF& in, double cx0, double cy0, double cx, double cy) {
        const int x = (int)std::ceil((in.x - cx0) * s + cx), y = (int)std::ceil((in.y - cy0) * s + cy);
        const int w = (int)std::floor(in.w * s), h = (int)std::floor(in.h * s);
        return rect_and(mvsv_rect{x, y, x + w, y + h}, full);
    };
    if (roi1) *roi1 = roi_of(inner1, cx1_0, cy1_0, cx1, cy1);
    if (roi2) *roi2 = roi_of(inner2, cx2_0, cy2_0, cx2, cy2);
    if (Q) {
        const double q[16] = {1, 0, 0, -cx1, 0, 1, 0, -cy1, 0, 0, 0, fc_new, 0, 0, -1. / t[idx],
                              (idx == 0 ? cx1 - cx2 : cy1 - cy2) / t[idx]};
        std::memcpy(Q, q, sizeof q);
    }
    return MVSV_OK;
}

}  // extern "C"
