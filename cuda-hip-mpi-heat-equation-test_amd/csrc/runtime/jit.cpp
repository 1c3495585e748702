// Run-time specialised FTCS kernel (hipRTC): the capability of the reference's
// PyCUDA program (python/cuda/cuda.py:58-89), which renders a CUDA-C kernel
// from a Jinja2 template with the grid sizes and r baked in as literals and
// compiles it with nvcc at run time (SourceModule). Here the source is rendered
// for one slab layout — row count, column count, pitch, origin offset and r
// (as an exact hexadecimal literal) become compile-time constants — and
// compiled for the running device's gfx target with hipRTC, loaded with
// hipModuleLoadData and launched with hipModuleLaunchKernel. Unlike the
// reference it stays device-resident (no per-step host copies), has no
// out-of-bounds reads (python/cuda/cuda.py:70-77) and keeps the
// reference's summation order under -ffp-contract=off, so it is bitwise
// identical to the temporal-blocked engine at any depth.
//
// One FTCS step over the owned rows of a slab (frame / ghost rows are inputs
// only); modules are cached per (device, rendered source).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "heat2d/jit.hpp"

namespace heat2d {

#define H2D_HIP(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) fail(__FILE__, __LINE__, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace {

std::string hex_literal(double v, bool f32) {
  char b[64];
  if (f32) std::snprintf(b, sizeof(b), "%af", (double)(float)v);
  else std::snprintf(b, sizeof(b), "%a", v);
  return b;
}

struct Compiled {
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
};

std::mutex g_mu;
std::map<std::pair<int, std::string>, Compiled> g_cache;  // (device, source) -> module

}  // namespace

std::string jit_render(DType dt, const SlabLayout& L, double r, int arith) {
  const bool f32 = dt == DType::F32;
  const char* T = f32 ? "float" : "double";
  std::string s;
  char line[512];
  s += "// heat2d run-time specialised FTCS step (rendered by csrc/runtime/jit.cpp)\n";
  std::snprintf(line, sizeof(line), "typedef %s real;\n", T);
  s += line;
  std::snprintf(line, sizeof(line),
                "#define NROWS %lldL\n#define NCOLS %lldL\n#define PITCH %lldL\n#define ORIGIN %lldL\n",
                (long long)L.nrows, (long long)L.ncols, (long long)L.pitch, (long long)L.origin());
  s += line;
  s += "#define R (" + hex_literal(r, f32) + ")\n";
  s += "#define FOUR ((real)4)\n";
  // arith 1: the contracted form hipcc's default -ffp-contract=fast gives the
  // reference line; spelled out, since the module is compiled with contraction off
  // arith 2 (r == 1/4): the centre weight 1 - 4r is zero — R * sum
  s += arith == 2   ? "#define UPDATE(c, sum) (R * (sum))\n"
       : arith == 1 ? "#define UPDATE(c, sum) fma(R, (sum) - FOUR * (c), (c))\n"
                    : "#define UPDATE(c, sum) ((c) + R * ((sum) - FOUR * (c)))\n";
  s += R"(
extern "C" __global__ void __launch_bounds__(256) heat2d_jit_ftcs(const real* __restrict__ src,
                                                                  real* __restrict__ dst) {
  const long j = (long)blockIdx.x * 256 + threadIdx.x;  // column (y, fast axis)
  if (j >= NCOLS) return;
  for (long i = blockIdx.y; i < NROWS; i += gridDim.y) {  // row (x, slow axis)
    const long o = ORIGIN + i * PITCH + j;
    const real c = src[o];
    // reference order: T(x+1,y) + T(x,y+1) + T(x-1,y) + T(x,y-1) - 4 T(x,y)
    // (fortran/hip/heat_kernel.cpp:43); frame / ghost rows and columns are
    // inside the allocation, so no bounds test is needed for neighbours
    const real sum = ((src[o + PITCH] + src[o + 1]) + src[o - PITCH]) + src[o - 1];
    dst[o] = UPDATE(c, sum);
  }
}
)";
  return s;
}

JitStencil::JitStencil(DType dt, const SlabLayout& L, double r, int device, int arith) : L_(L) {
  HEAT2D_REQUIRE(L.nrows >= 1 && L.ncols >= 1 && L.halo >= 1 && L.cpad >= 1, "layout needs a ghost frame");
  if (device >= 0) H2D_HIP(hipSetDevice(device));
  H2D_HIP(hipGetDevice(&device_));
  HEAT2D_REQUIRE(arith >= 0 && arith <= 3, "arith must be 0, 1, 2 or 3");
  // arith 3 (scaled levels) has nothing to scale at one step per launch: the
  // contracted form is its one-level case up to the rounding of b and r
  if (arith == 3) arith = 1;
  HEAT2D_REQUIRE(arith != 2 || r == 0.25, "arith 2 (jacobi) needs r == 1/4 exactly");
  src_ = jit_render(dt, L, r, arith);
  std::lock_guard<std::mutex> g(g_mu);
  auto key = std::make_pair(device_, src_);
  auto it = g_cache.find(key);
  if (it != g_cache.end()) {
    fn_ = it->second.fn;
    return;
  }
  hipDeviceProp_t prop;
  H2D_HIP(hipGetDeviceProperties(&prop, device_));
  const std::string code = jit_compile(src_, prop.gcnArchName);
  Compiled c;
  H2D_HIP(hipModuleLoadData(&c.mod, code.data()));
  H2D_HIP(hipModuleGetFunction(&c.fn, c.mod, "heat2d_jit_ftcs"));
  g_cache[key] = c;
  fn_ = c.fn;
}

std::string jit_compile(const std::string& source, const std::string& arch) {
  hiprtcProgram prog;
  auto ck = [](hiprtcResult r, const char* what) {
    if (r != HIPRTC_SUCCESS) fail(__FILE__, __LINE__, std::string(what) + ": " + hiprtcGetErrorString(r));
  };
  ck(hiprtcCreateProgram(&prog, source.c_str(), "heat2d_jit.hip", 0, nullptr, nullptr), "hiprtcCreateProgram");
  const std::string a = "--offload-arch=" + arch;
  const char* opts[] = {a.c_str(), "-O3", "-ffp-contract=off", "-std=c++17"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 4, opts);
  if (rc != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    hiprtcDestroyProgram(&prog);
    fail(__FILE__, __LINE__, std::string("hiprtcCompileProgram: ") + hiprtcGetErrorString(rc) + "\n" + log);
  }
  size_t sz = 0;
  ck(hiprtcGetCodeSize(prog, &sz), "hiprtcGetCodeSize");
  std::string code(sz, '\0');
  ck(hiprtcGetCode(prog, &code[0]), "hiprtcGetCode");
  hiprtcDestroyProgram(&prog);
  return code;
}

void JitStencil::step(const void* src, void* dst, hipStream_t stream) const {
  const unsigned gx = (unsigned)((L_.ncols + 255) / 256);
  const unsigned gy = (unsigned)std::min<int64_t>(L_.nrows, 65535);
  const void* s = src;
  void* d = dst;
  void* args[] = {(void*)&s, (void*)&d};
  H2D_HIP(hipModuleLaunchKernel(fn_, gx, gy, 1, 256, 1, 1, 0, stream, args, nullptr));
}

}  // namespace heat2d
