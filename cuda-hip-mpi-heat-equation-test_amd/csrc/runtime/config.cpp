// input.dat parsing and problem set-up (see config.hpp).
#include "heat2d/config.hpp"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <sstream>

#include "heat2d/common.hpp"

namespace heat2d {

namespace {
std::vector<std::string> list_directed_tokens(const std::string& text) {
  std::vector<std::string> out;
  std::string cur;
  auto flush = [&] {
    if (cur.empty()) return;
    // r*c repeat count
    const auto star = cur.find('*');
    if (star != std::string::npos && star > 0 &&
        std::all_of(cur.begin(), cur.begin() + star, [](char c) { return std::isdigit((unsigned char)c); })) {
      const int rep = std::atoi(cur.substr(0, star).c_str());
      const std::string val = cur.substr(star + 1);
      for (int i = 0; i < rep; ++i) out.push_back(val);
    } else {
      out.push_back(cur);
    }
    cur.clear();
  };
  for (char c : text) {
    if (c == '/') break;  // record terminator
    if (std::isspace((unsigned char)c) || c == ',' || c == ';') {
      flush();
    } else {
      cur.push_back(c);
    }
  }
  flush();
  return out;
}

double to_real(std::string s) {
  for (auto& c : s)
    if (c == 'd' || c == 'D' || c == 'q' || c == 'Q') c = 'e';
  char* end = nullptr;
  const double v = std::strtod(s.c_str(), &end);
  HEAT2D_REQUIRE(end && *end == 0, "bad real in input.dat: " + s);
  return v;
}

int64_t to_int(const std::string& s) {
  char* end = nullptr;
  const long long v = std::strtoll(s.c_str(), &end, 10);
  HEAT2D_REQUIRE(end && *end == 0, "bad integer in input.dat: " + s);
  return (int64_t)v;
}
}  // namespace

InputDat parse_input_text(const std::string& text) {
  const auto tok = list_directed_tokens(text);
  HEAT2D_REQUIRE(tok.size() >= 5, "input.dat needs at least 5 fields: n sigma nu dom_len ntime [soln]");
  InputDat in;
  in.n = to_int(tok[0]);
  in.sigma = to_real(tok[1]);
  in.nu = to_real(tok[2]);
  in.dom_len = to_real(tok[3]);
  in.ntime = to_int(tok[4]);
  in.nfields = 5;
  if (tok.size() >= 6) {
    in.soln = (int)to_int(tok[5]);
    in.nfields = 6;
  }
  HEAT2D_REQUIRE(in.n >= 3, "grid size must be >= 3");
  HEAT2D_REQUIRE(in.nu > 0 && in.dom_len > 0, "nu and dom_len must be positive");
  HEAT2D_REQUIRE(in.ntime >= 0, "ntime must be >= 0");
  return in;
}

InputDat read_input_file(const std::string& path) {
  std::ifstream f(path);
  HEAT2D_REQUIRE(f.good(), "cannot open " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return parse_input_text(ss.str());
}

Problem make_problem(const InputDat& in, Convention conv, const std::string& ic_name) {
  Problem p;
  p.conv = conv;
  // reference: delta = dom_len/real(n-1); dt = (sigma*delta**2)/nu; r = (nu*dt)/delta**2
  p.delta = in.dom_len / (double)(in.n - 1);
  p.dt = (in.sigma * (p.delta * p.delta)) / in.nu;
  p.r = (in.nu * p.dt) / (p.delta * p.delta);
  if (conv == Convention::Ghost) {
    p.n_owned = in.n;
    p.x.resize((size_t)in.n + 2);
    for (int64_t g = -1; g <= in.n; ++g) p.x[(size_t)(g + 1)] = (double)g * p.delta;  // xg(i) = (i-1)*delta
  } else {
    p.n_owned = in.n - 2;
    p.x.resize((size_t)in.n);
    p.x[0] = 0.0;
    for (int64_t i = 1; i < in.n - 1; ++i) p.x[(size_t)i] = p.x[(size_t)i - 1] + p.delta;  // cumulative
    p.x[(size_t)in.n - 1] = in.dom_len;
  }
  kern::IcParams& ic = p.ic;
  ic = kern::IcParams{};
  ic.pad = 1.0;
  if (ic_name == "uniform" || ic_name == "mpi") {  // fortran/hip/heat.F90:274-282
    ic.kind = (int)kern::IcKind::Uniform;
    ic.a = 2.0;
    ic.b = 1.0;
  } else if (ic_name == "hat" || ic_name == "serial") {  // fortran/serial/heat.f90:40-48
    ic.kind = (int)kern::IcKind::Box;
    ic.a = 2.0; ic.b = 1.0;
    ic.x0 = 0.5; ic.x1 = 1.5; ic.y0 = 0.5; ic.y1 = 1.5;
  } else if (ic_name == "hat-cuda" || ic_name == "cuda") {  // fortran/cuda_kernel/heat.F90:97-105
    ic.kind = (int)kern::IcKind::Box;
    ic.a = 2.0; ic.b = 1.0;
    ic.x0 = 0.5; ic.x1 = 1.5; ic.y0 = 0.5; ic.y1 = 1.0;
  } else if (ic_name == "hotspot") {  // zero field + unit hot spot (benchmark synthetic data)
    ic.kind = (int)kern::IcKind::Box;
    ic.a = 1.0; ic.b = 0.0; ic.pad = 0.0;
    const double L = in.dom_len;
    ic.x0 = 0.4 * L; ic.x1 = 0.6 * L; ic.y0 = 0.4 * L; ic.y1 = 0.6 * L;
  } else if (ic_name == "sine") {
    ic.kind = (int)kern::IcKind::Sine;
    ic.a = 1.0; ic.pad = 0.0;
    ic.x0 = p.x.front(); ic.x1 = p.x.back(); ic.y0 = ic.x0; ic.y1 = ic.x1;
    ic.kx = 1.0; ic.ky = 1.0;
  } else {
    fail(__FILE__, __LINE__, "unknown IC '" + ic_name + "' (uniform|hat|hat-cuda|hotspot|sine)");
  }
  return p;
}

bool ic_sterbenz_safe(const kern::IcParams& ic) {
  double lo = 0, hi = 0;
  switch ((kern::IcKind)ic.kind) {
    case kern::IcKind::Uniform:
    case kern::IcKind::Box:
    case kern::IcKind::IndexBox:
      lo = std::min({ic.a, ic.b, ic.pad});
      hi = std::max({ic.a, ic.b, ic.pad});
      break;
    case kern::IcKind::Const:
      lo = std::min(ic.a, ic.pad);
      hi = std::max(ic.a, ic.pad);
      break;
    default:  // sine: zero frame
      return false;
  }
  return lo > 0 && hi <= 2 * lo;
}

}  // namespace heat2d
