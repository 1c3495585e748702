// CPU twins of the device kernels. They implement the same operations on the
// same SlabLayout with the same arithmetic order (built with
// -ffp-contract=off), so CPU, GPU, blocked and unblocked runs agree bitwise.
// This is also the native serial solver path that replaces
// fortran/serial/heat.f90 (whose k-inner loop over the strided index,
// :64-66, is cache-hostile; here the inner loop is the contiguous one).
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <thread>
#include <type_traits>
#include <vector>

#include "heat2d/runtime.hpp"

namespace heat2d {
namespace cpu {
namespace {

// Rows [begin, end) split over host threads; `row_cost` = elements per row.
// Below ~1M elements per call one thread is faster than spawning several
// (the 256^2 serial config runs ~3x faster that way).
template <typename F>
void parallel_rows(int64_t begin, int64_t end, F&& f, int64_t row_cost = 1 << 14) {
  const int64_t n = end - begin;
  if (n <= 0) return;
  int nt = num_threads();
  if (n < 64 || nt <= 1 || n * row_cost < (int64_t(1) << 20)) {
    f(begin, end);
    return;
  }
  nt = (int)std::min<int64_t>(nt, n / 32 > 0 ? n / 32 : 1);
  std::vector<std::thread> th;
  th.reserve(nt);
  const int64_t chunk = (n + nt - 1) / nt;
  for (int t = 0; t < nt; ++t) {
    const int64_t b = begin + t * chunk, e = std::min(end, b + chunk);
    if (b >= e) break;
    th.emplace_back([=, &f] { f(b, e); });
  }
  for (auto& x : th) x.join();
}

// One row of the FTCS update in the reference order
// T(x+1,y) + T(x,y+1) + T(x-1,y) + T(x,y-1) - 4*T(x,y), then C + r*(...) or
// its contracted form (the device kernel's arith 1, tb_impl.hpp). The fma form
// has a copy compiled for hosts with FMA3 (std::fma otherwise is a libm call
// per point: ~4x slower on the 256^2 serial config).
template <typename T>
void row_exact(const T* up, const T* mid, const T* dn, T* out, int64_t n, T r) {
  for (int64_t j = 0; j < n; ++j) {
    const T sum = ((dn[j] + mid[j + 1]) + up[j]) + mid[j - 1];
    out[j] = mid[j] + r * (sum - T(4) * mid[j]);
  }
}
template <typename T>
__attribute__((target("fma"))) void row_fma_hw(const T* up, const T* mid, const T* dn, T* out, int64_t n, T r) {
  for (int64_t j = 0; j < n; ++j) {
    const T sum = ((dn[j] + mid[j + 1]) + up[j]) + mid[j - 1];
    out[j] = std::fma(r, sum - T(4) * mid[j], mid[j]);
  }
}
template <typename T>
void row_fma_sw(const T* up, const T* mid, const T* dn, T* out, int64_t n, T r) {
  for (int64_t j = 0; j < n; ++j) {
    const T sum = ((dn[j] + mid[j + 1]) + up[j]) + mid[j - 1];
    out[j] = std::fma(r, sum - T(4) * mid[j], mid[j]);
  }
}
// arith 2 (r == 1/4): the centre weight 1 - 4r is zero, r * sum (r*x exact)
template <typename T>
void row_jacobi(const T* up, const T* mid, const T* dn, T* out, int64_t n, T r) {
  for (int64_t j = 0; j < n; ++j) out[j] = r * (((dn[j] + mid[j + 1]) + up[j]) + mid[j - 1]);
}
bool host_has_fma() {
  static const bool v = __builtin_cpu_supports("fma");
  return v;
}

template <typename T>
void tb_impl(const T* src, T* dst, const SlabLayout& L, int64_t rb, int64_t re, int k, T r, int arith) {
  const int64_t R = re - rb + 2 * k;  // level-0 rows [rb-k, re+k)
  const int64_t P = L.pitch;
  std::vector<T> A((size_t)(R * P)), B((size_t)(R * P));
  std::memcpy(A.data(), src + L.offset(rb - k, -L.cpad), sizeof(T) * (size_t)(R * P));
  std::memcpy(B.data(), A.data(), sizeof(T) * (size_t)(R * P));
  const int64_t fixed_lo = -L.row0, fixed_hi = L.nrows_global - L.row0;
  const int64_t c = L.cpad;
  T* a = A.data();
  T* b = B.data();
  auto* row_update = arith == 2   ? &row_jacobi<T>
                     : arith == 1 ? (host_has_fma() ? &row_fma_hw<T> : &row_fma_sw<T>)
                                  : &row_exact<T>;
  for (int s = 1; s <= k; ++s) {
    parallel_rows(s, R - s, [&](int64_t lb, int64_t le) {
      for (int64_t li = lb; li < le; ++li) {
        const int64_t row = rb - k + li;  // local slab row
        const T* up = a + (li - 1) * P + c;
        const T* mid = a + li * P + c;
        const T* dn = a + (li + 1) * P + c;
        T* out = b + li * P + c;
        if (row < fixed_lo || row >= fixed_hi) {
          std::memcpy(out, mid, sizeof(T) * (size_t)L.ncols);
          continue;
        }
        row_update(up, mid, dn, out, L.ncols, r);
      }
    }, L.ncols);
    std::swap(a, b);
  }
  for (int64_t i = rb; i < re; ++i)
    std::memcpy(dst + L.offset(i, 0), a + (i - rb + k) * P + c, sizeof(T) * (size_t)L.ncols);
}

template <typename T>
void init_impl(T* f, const SlabLayout& L, const kern::IcParams& ic, const double* xc, const double* yc) {
  parallel_rows(0, L.rows_alloc(), [&](int64_t b, int64_t e) {
    for (int64_t ia = b; ia < e; ++ia) {
      const int64_t i = ia - L.halo;
      const int64_t g = L.row0 + i;
      for (int64_t ja = 0; ja < L.pitch; ++ja) {
        const int64_t j = ja - L.cpad;
        double v;
        const bool in_frame = g >= -1 && g <= L.nrows_global && j >= -1 && j <= L.ncols;
        if (!in_frame) {
          v = ic.pad;
        } else {
          const bool frame = g < 0 || g >= L.nrows_global || j < 0 || j >= L.ncols;
          const double x = xc[g + 1], y = yc[j + 1];
          switch ((kern::IcKind)ic.kind) {
            case kern::IcKind::Uniform:
              v = frame ? ic.b : ic.a;
              break;
            case kern::IcKind::Box:
              v = (x <= ic.x1 && x >= ic.x0 && y <= ic.y1 && y >= ic.y0) ? ic.a : ic.b;
              break;
            case kern::IcKind::IndexBox: {
              const int64_t gi = g + 1, gj = j + 1;
              v = (gi >= ic.i0 && gi < ic.i1 && gj >= ic.j0 && gj < ic.j1) ? ic.a : ic.b;
              break;
            }
            case kern::IcKind::Sine:
              v = frame ? 0.0
                        : ic.a * std::sin(ic.kx * M_PI * (x - ic.x0) / (ic.x1 - ic.x0)) *
                              std::sin(ic.ky * M_PI * (y - ic.y0) / (ic.y1 - ic.y0));
              break;
            default:
              v = ic.a;
          }
        }
        f[ia * L.pitch + ja] = (T)v;
      }
    }
  });
}

template <typename T>
void stats_impl(const T* f, const T* o, const SlabLayout& L, double out[6]) {
  double s = 0, ss = 0, mn = DBL_MAX, mx = -DBL_MAX, dd = 0, md = 0;
  for (int64_t i = 0; i < L.nrows; ++i) {
    const T* row = f + L.offset(i, 0);
    const T* orow = o ? o + L.offset(i, 0) : nullptr;
    for (int64_t j = 0; j < L.ncols; ++j) {
      const double v = (double)row[j];
      s += v;
      ss += v * v;
      mn = std::fmin(mn, v);
      mx = std::fmax(mx, v);
      if (orow) {
        const double d = v - (double)orow[j];
        dd += d * d;
        md = std::fmax(md, std::fabs(d));
      }
    }
  }
  out[0] = s; out[1] = ss; out[2] = mn; out[3] = mx; out[4] = dd; out[5] = md;
}

}  // namespace

int num_threads() {
  static int n = [] {
    const char* e = std::getenv("HEAT2D_CPU_THREADS");
    int v = e ? std::atoi(e) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(v, 64));
  }();
  return n;
}

void tb(DType dt, const void* src, void* dst, const SlabLayout& L, int64_t row_begin, int64_t row_end,
        int k, double r, int arith) {
  HEAT2D_REQUIRE(k >= 1 && k <= L.halo, "k out of range");
  HEAT2D_REQUIRE(arith >= 0 && arith <= 3, "arith must be 0, 1, 2 or 3");
  HEAT2D_REQUIRE(arith != 2 || r == 0.25, "arith 2 (jacobi) needs r == 1/4 exactly");
  // arith 3 (the device kernels' scaled levels, tb_impl.hpp) is not bitwise
  // reproducible across launch plans; the CPU twin runs its unscaled
  // contracted form (arith 1), within the same stated bound of exact
  if (arith == 3) arith = 1;
  if (row_end <= row_begin) return;
  if (dt == DType::F32)
    tb_impl<float>(static_cast<const float*>(src), static_cast<float*>(dst), L, row_begin, row_end, k, (float)r, arith);
  else
    tb_impl<double>(static_cast<const double*>(src), static_cast<double*>(dst), L, row_begin, row_end, k, r, arith);
}

void init(DType dt, void* field, const SlabLayout& L, const kern::IcParams& ic, const double* xc,
          const double* yc) {
  if (dt == DType::F32)
    init_impl<float>(static_cast<float*>(field), L, ic, xc, yc);
  else
    init_impl<double>(static_cast<double*>(field), L, ic, xc, yc);
}

void stats(DType dt, const void* field, const void* other, const SlabLayout& L, double out[6]) {
  if (dt == DType::F32)
    stats_impl<float>(static_cast<const float*>(field), static_cast<const float*>(other), L, out);
  else
    stats_impl<double>(static_cast<const double*>(field), static_cast<const double*>(other), L, out);
}

void pack_rows(DType dt, const void* field, const SlabLayout& L, int64_t row, int64_t nrows, void* buf) {
  const size_t es = dtype_size(dt);
  for (int64_t i = 0; i < nrows; ++i)
    std::memcpy(static_cast<char*>(buf) + (size_t)(i * L.ncols) * es,
                static_cast<const char*>(field) + (size_t)L.offset(row + i, 0) * es, (size_t)L.ncols * es);
}

void unpack_rows(DType dt, void* field, const SlabLayout& L, int64_t row, int64_t nrows, const void* buf) {
  const size_t es = dtype_size(dt);
  for (int64_t i = 0; i < nrows; ++i)
    std::memcpy(static_cast<char*>(field) + (size_t)L.offset(row + i, 0) * es,
                static_cast<const char*>(buf) + (size_t)(i * L.ncols) * es, (size_t)L.ncols * es);
}

}  // namespace cpu
}  // namespace heat2d
