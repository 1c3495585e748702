// Run-time specialised FTCS kernel via hipRTC (parity with the reference's
// PyCUDA/Jinja2 JIT program, python/cuda/cuda.py). See runtime/jit.cpp.
#pragma once

#include <hip/hip_runtime.h>

#include <string>

#include "heat2d/common.hpp"

namespace heat2d {

// HIP source of one FTCS step specialised for a slab layout and r (sizes,
// pitch, origin and r baked in as literals, r as an exact hex float).
std::string jit_render(DType dt, const SlabLayout& L, double r, int arith = 0);
// Compile HIP source for `arch` (e.g. "gfx950") with hipRTC; returns the code
// object. Needs no GPU (used by the CPU test suite to check the rendering).
std::string jit_compile(const std::string& source, const std::string& arch);

class JitStencil {
 public:
  JitStencil(DType dt, const SlabLayout& L, double r, int device = -1, int arith = 0);
  // dst(owned rows) = one FTCS step of src (allocation bases laid out per L)
  void step(const void* src, void* dst, hipStream_t stream) const;
  const std::string& source() const { return src_; }

 private:
  SlabLayout L_;
  int device_ = 0;
  std::string src_;
  hipFunction_t fn_ = nullptr;
};

}  // namespace heat2d
