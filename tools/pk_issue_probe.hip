// Issue cost of the small-grid march's VALU mix at one and two waves per SIMD
// (would two interleaved marches per wave — more ILP — help
// a 1-wave/SIMD march?). Each wave runs ITERS x 8 independent instructions of
// one kind and times itself with s_memtime (shader clock), so the result is
// cycles per wave-instruction, free of launch and tail effects.
//   kinds: v_add_f32, v_pk_add_f32, v_add_f64, and the fp32 march's own
//   per-level-row mix (4 v_pk_add_f32 + 2 v_add_f32 + 2 v_add_f32 DPP wave_shr)
// build: hipcc --offload-arch=gfx950 -O3 tools/pk_issue_probe.hip -o /tmp/pk_issue_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ __launch_bounds__(256) void probe(unsigned long long* cyc, float* sink, int iters) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  f2 p0 = {a0, a1}, p1 = {a2, a3}, p2 = {a4, a5}, p3 = {a6, a7}, p4 = {a1, a0}, p5 = {a3, a2}, p6 = {a5, a4},
     p7 = {a7, a6};
  double d0 = a0, d1 = a1, d2 = a2, d3 = a3, d4 = a4, d5 = a5, d6 = a6, d7 = a7;
  const float inc = 1.0f / (1 + blockIdx.x);
  const f2 pinc = {inc, inc};
  const double dinc = inc;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 4
  for (int it = 0; it < iters; ++it) {
    if constexpr (KIND == 0) {
#define A(x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(inc))
      A(a0); A(a1); A(a2); A(a3); A(a4); A(a5); A(a6); A(a7);
#undef A
    } else if constexpr (KIND == 1) {
#define P(x) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(pinc))
      P(p0); P(p1); P(p2); P(p3); P(p4); P(p5); P(p6); P(p7);
#undef P
    } else if constexpr (KIND == 2) {
#define D(x) asm volatile("v_add_f64 %0, %0, %1" : "+v"(x) : "v"(dinc))
      D(d0); D(d1); D(d2); D(d3); D(d4); D(d5); D(d6); D(d7);
#undef D
    } else {
      // the march mix: 4 packed adds, 2 plain adds, 2 adds with a DPP wave shift
#define P(x) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(pinc))
#define A(x) asm volatile("v_add_f32 %0, %0, %1" : "+v"(x) : "v"(inc))
#define S(x, y) asm volatile("v_add_f32_dpp %0, %1, %0 wave_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0" : "+v"(x) : "v"(y))
      P(p0); A(a0); P(p1); S(a1, a4); P(p2); A(a2); P(p3); S(a3, a5);
#undef P
#undef A
#undef S
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) / 64;
  if ((threadIdx.x & 63) == 0) cyc[wave] = t1 - t0;
  float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.y + p2.x + p3.y + p4.x + p5.y + p6.x + p7.y +
            (float)(d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7);
  if (s == -1.2345f) sink[0] = s;
}

template <int KIND>
double run(int waves_per_simd, int cus, int iters, int insts_per_iter) {
  // 256-thread blocks = 4 waves = one per SIMD; blocks per CU = waves per SIMD
  const int blocks = cus * waves_per_simd, nw = blocks * 4;
  unsigned long long* d = nullptr;
  float* sink = nullptr;
  (void)hipMalloc(&d, nw * sizeof(unsigned long long));
  (void)hipMalloc(&sink, 4);
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, d, sink, 64);  // warm
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, d, sink, iters);
  (void)hipDeviceSynchronize();
  std::vector<unsigned long long> h(nw);
  (void)hipMemcpy(h.data(), d, nw * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  double mean = 0, mn = 1e300;
  for (auto v : h) {
    mean += (double)v;
    mn = (double)v < mn ? (double)v : mn;
  }
  mean /= nw;
  std::printf("# kind %d, %d waves/SIMD: min %.3f mean %.3f cycles per wave-instruction\n", KIND, waves_per_simd,
              mn / ((double)iters * insts_per_iter), mean / ((double)iters * insts_per_iter));
  (void)hipFree(d);
  (void)hipFree(sink);
  return mean / ((double)iters * insts_per_iter);  // cycles per wave-instruction (each wave's own view)
}

int main() {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int iters = 20000;
  const char* names[4] = {"v_add_f32", "v_pk_add_f32", "v_add_f64", "march mix (4 pk + 2 add + 2 add_dpp)"};
  for (int w = 1; w <= 2; ++w) {
    const double c[4] = {run<0>(w, cus, iters, 8), run<1>(w, cus, iters, 8), run<2>(w, cus, iters, 8),
                         run<3>(w, cus, iters, 8)};
    for (int k = 0; k < 4; ++k)
      std::printf("{\"waves_per_simd\": %d, \"kind\": \"%s\", \"cycles_per_wave_instr\": %.3f, "
                  "\"simd_cycles_per_instr\": %.3f}\n", w, names[k], c[k], c[k] / w);
  }
  return 0;
}
