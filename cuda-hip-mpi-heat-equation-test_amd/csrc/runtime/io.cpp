// Output writers.
//   * xyz: ASCII "x y T" triples, one point per line, x outer / y inner — the
//     int.dat / soln.dat / soln%05d.dat format of the reference
//     (fortran/serial/heat.f90:50-55,77-83; fortran/hip/heat.F90:308-319),
//     with gfortran list-directed style numbers (17 significant digits).
//     Rows are formatted in parallel and written in order.
//   * npy: binary NumPy array of the owned region (a 32768^2 ASCII dump is
//     ~1e9 lines; the binary dump is what large runs should use).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "heat2d/capi.h"
#include "heat2d/runtime.hpp"

namespace heat2d {
namespace io {

// gfortran-like list-directed REAL(8) item: F form with 17 significant digits
// for 0.1 <= |v| < 1e16 (and 0), E form with a 3-digit exponent otherwise.
inline int format_real(char* out, double v) {
  const double a = std::fabs(v);
  if (v == 0.0) return std::snprintf(out, 48, "   0.0000000000000000     ");
  // an unstable run (r > 1/4) overflows: gfortran writes these words, and
  // "%E" has no exponent to split (found by the UBSan build, tests/test_sanitizers.py)
  if (std::isnan(v)) return std::snprintf(out, 48, "%25s", "NaN");
  if (std::isinf(v)) return std::snprintf(out, 48, "%25s", v < 0 ? "-Infinity" : "Infinity");
  if (a >= 0.1 && a < 1e16) {
    const int d = (int)std::floor(std::log10(a)) + 1;  // digits left of the point (0 for [0.1,1))
    const int dec = std::max(0, 17 - std::max(d, 0));
    return std::snprintf(out, 64, "%*.*f     ", 20, dec, v);
  }
  char tmp[64];
  std::snprintf(tmp, sizeof(tmp), "%.16E", v);  // d.ddddE+xx
  char* e = std::strchr(tmp, 'E');
  const int ex = std::atoi(e + 1);
  *e = 0;
  return std::snprintf(out, 64, "  %sE%c%03d", tmp, ex < 0 ? '-' : '+', std::abs(ex));
}

template <typename T>
void write_xyz(const char* path, const T* data, int64_t nrows, int64_t ncols, int64_t ld, const double* x,
               const double* y, bool append) {
  FILE* f = std::fopen(path, append ? "ab" : "wb");
  HEAT2D_REQUIRE(f != nullptr, std::string("cannot open ") + path);
  const int nt = std::max(1, std::min(cpu::num_threads(), 32));
  const int64_t rows_per_chunk = std::max<int64_t>(1, (int64_t)(1 << 16) / std::max<int64_t>(ncols, 1));
  std::vector<std::string> bufs(nt);
  for (int64_t r0 = 0; r0 < nrows; r0 += rows_per_chunk * nt) {
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) {
      const int64_t b = r0 + t * rows_per_chunk, e = std::min(nrows, b + rows_per_chunk);
      bufs[t].clear();
      if (b >= e) continue;
      th.emplace_back([&, t, b, e] {
        std::string& s = bufs[t];
        s.reserve((size_t)((e - b) * ncols * 80));
        char line[256];
        for (int64_t i = b; i < e; ++i)
          for (int64_t j = 0; j < ncols; ++j) {
            int n = 0;
            n += format_real(line + n, x[i]);
            n += format_real(line + n, y[j]);
            n += format_real(line + n, (double)data[i * ld + j]);
            line[n++] = '\n';
            s.append(line, (size_t)n);
          }
      });
    }
    for (auto& x_ : th) x_.join();
    for (int t = 0; t < nt; ++t)
      if (!bufs[t].empty()) std::fwrite(bufs[t].data(), 1, bufs[t].size(), f);
  }
  std::fclose(f);
}

void write_npy(const char* path, DType dt, const void* data, int64_t nrows, int64_t ncols, int64_t ld) {
  FILE* f = std::fopen(path, "wb");
  HEAT2D_REQUIRE(f != nullptr, std::string("cannot open ") + path);
  std::string hdr = std::string("{'descr': '<") + (dt == DType::F32 ? "f4" : "f8") +
                    "', 'fortran_order': False, 'shape': (" + std::to_string(nrows) + ", " +
                    std::to_string(ncols) + "), }";
  const size_t pre = 10;  // magic(6) + version(2) + header len(2)
  size_t total = pre + hdr.size() + 1;
  const size_t pad = (64 - total % 64) % 64;
  hdr.append(pad, ' ');
  hdr.push_back('\n');
  const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
  std::fwrite(magic, 1, 8, f);
  const uint16_t hl = (uint16_t)hdr.size();
  std::fwrite(&hl, 2, 1, f);
  std::fwrite(hdr.data(), 1, hdr.size(), f);
  const size_t es = dtype_size(dt);
  for (int64_t i = 0; i < nrows; ++i)
    std::fwrite(static_cast<const char*>(data) + (size_t)(i * ld) * es, es, (size_t)ncols, f);
  std::fclose(f);
}

}  // namespace io
}  // namespace heat2d

extern "C" int heat2d_io_write_xyz_impl(const char* path, int dtype, const void* host, int64_t nrows,
                                        int64_t ncols, int64_t ld, const double* x, const double* y,
                                        int append) {
  using namespace heat2d;
  if (dtype == (int)DType::F32)
    io::write_xyz<float>(path, static_cast<const float*>(host), nrows, ncols, ld, x, y, append != 0);
  else
    io::write_xyz<double>(path, static_cast<const double*>(host), nrows, ncols, ld, x, y, append != 0);
  return 0;
}

extern "C" int heat2d_io_write_npy_impl(const char* path, int dtype, const void* host, int64_t nrows,
                                        int64_t ncols, int64_t ld) {
  heat2d::io::write_npy(path, (heat2d::DType)dtype, host, nrows, ncols, ld);
  return 0;
}
