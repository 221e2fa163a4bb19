// Fast text I/O for the reference-format output files.
//
// Grid dumps: same bytes as `os << std::setprecision(3) << std::setw(5) << v
// << " "` per value, rows top-down (hw/hw2/solution/2dHeat_solution.cu:247-258,
// 671-688), i.e. printf("%5.3g ").
// Vector dumps: `ofs << v << " "` (default 6 significant digits) as used for
// b.txt (hw/hw_final/programming/fp.cu:196-212), i.e. printf("%g ").
#include <cstdio>
#include <cstring>
#include <vector>

#include "cme213/cpu_common.h"

namespace {

template <typename T>
int write_grid(const char* path, const T* data, int pitch, int rows, int cols, int extra_endl) {
    FILE* f = std::fopen(path, "w");
    if (!f) return 1;
    std::vector<char> line;
    line.reserve((size_t)cols * 16 + 2);
    char tmp[64];
    for (int y = rows - 1; y >= 0; --y) {
        line.clear();
        const T* r = data + (size_t)y * pitch;
        for (int x = 0; x < cols; ++x) {
            int n = std::snprintf(tmp, sizeof(tmp), "%5.3g ", (double)r[x]);
            line.insert(line.end(), tmp, tmp + n);
        }
        line.push_back('\n');
        std::fwrite(line.data(), 1, line.size(), f);
    }
    std::fputc('\n', f);
    if (extra_endl) std::fputc('\n', f);
    return std::fclose(f) == 0 ? 0 : 1;
}

template <typename T>
int write_vec(const char* path, const T* data, long long n) {
    FILE* f = std::fopen(path, "w");
    if (!f) return 1;
    char tmp[64];
    std::vector<char> buf;
    buf.reserve(1 << 20);
    for (long long i = 0; i < n; ++i) {
        int k = std::snprintf(tmp, sizeof(tmp), "%g ", (double)data[i]);
        buf.insert(buf.end(), tmp, tmp + k);
        if (buf.size() > (1 << 20) - 64) {
            std::fwrite(buf.data(), 1, buf.size(), f);
            buf.clear();
        }
    }
    std::fwrite(buf.data(), 1, buf.size(), f);
    return std::fclose(f) == 0 ? 0 : 1;
}

}  // namespace

CME_CPU_EXPORT int cme_cpu_write_grid_f32(const char* path, const float* d, int pitch, int rows, int cols, int e) {
    return write_grid(path, d, pitch, rows, cols, e);
}
CME_CPU_EXPORT int cme_cpu_write_grid_f64(const char* path, const double* d, int pitch, int rows, int cols, int e) {
    return write_grid(path, d, pitch, rows, cols, e);
}
CME_CPU_EXPORT int cme_cpu_write_vec_f32(const char* path, const float* d, long long n) { return write_vec(path, d, n); }
CME_CPU_EXPORT int cme_cpu_write_vec_f64(const char* path, const double* d, long long n) { return write_vec(path, d, n); }
