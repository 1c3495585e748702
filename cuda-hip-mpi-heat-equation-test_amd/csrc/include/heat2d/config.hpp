// Run configuration: the reference's `input.dat` (list-directed
// `read(11,*) n, sigma, nu, dom_len, ntime [, soln]`, fortran/serial/heat.f90:11-13,
// fortran/hip/heat.F90:136-140) plus the grid conventions / ICs of every
// reference variant, resolved into solver parameters.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "heat2d/kernels.hpp"

namespace heat2d {

struct InputDat {
  int64_t n = 0;
  double sigma = 0, nu = 0, dom_len = 0;
  int64_t ntime = 0;
  int soln = 0;
  int nfields = 0;  // 5 or 6
};

// Fortran list-directed parse: separators are blanks, commas, newlines; a
// '/' ends the record; `1.0d0` / `1.0D0` exponents accepted; `r*c` repeat
// counts accepted.
InputDat parse_input_text(const std::string& text);
InputDat read_input_file(const std::string& path);

// Grid conventions found in the reference:
//   Ghost     (V7/V8, fortran/hip): n owned points per axis + Dirichlet ghost
//             frame at x = -delta and x = L + delta; x_i = (i-1)*delta.
//   Inclusive (V3-V6): n points per axis INCLUDING the boundary; (n-2)^2
//             unknowns; x(1)=0, x(n)=L, interior by cumulative addition
//             (fortran/serial/heat.f90:28-36).
enum class Convention : int { Ghost = 0, Inclusive = 1 };

struct Problem {
  Convention conv = Convention::Ghost;
  int64_t n_owned = 0;         // owned points per axis
  double delta = 0, dt = 0, r = 0;
  std::vector<double> x;       // n_owned + 2 frame-inclusive coordinates (same for y)
  kern::IcParams ic{};
};

// delta = L/(n-1); dt = sigma*delta^2/nu; r = nu*dt/delta^2 — computed in the
// reference's order (fortran/hip/heat.F90:178-182), so r == sigma up to rounding.
Problem make_problem(const InputDat& in, Convention conv, const std::string& ic_name);

// True if every value this IC puts in the field (interior, frame, pad) lies in
// [m, 2m] for some m > 0. FTCS with r <= 1/4 is a convex combination, so the
// field stays in that range forever (maximum principle), and every sum - 4c of
// the update is then exact (Sterbenz): at r = 1/4 the r * sum form (arith 2,
// "jacobi") rounds bitwise like the reference's c + r*(sum - 4c). The CLI's
// --arith auto uses it (the reference IC: 2 inside, 1 on the frame).
bool ic_sterbenz_safe(const kern::IcParams& ic);

}  // namespace heat2d
