// Calibrate VALU throughput on this MI355X: fp64 / fp32 add chains with ILP
// independent accumulators per lane, and DPP wave-shift moves.
// build: hipcc --offload-arch=gfx950 -O3 tools/valu_probe.hip -o /tmp/valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>

template <typename T, int ILP>
__global__ __launch_bounds__(256) void add_chain(T* out, int iters, T inc) {
  T acc[ILP];
#pragma unroll
  for (int i = 0; i < ILP; ++i) acc[i] = (T)(threadIdx.x + i);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ILP; ++i) acc[i] = acc[i] + inc;
#pragma unroll
    for (int i = 0; i < ILP; ++i) acc[i] = acc[i] * inc;
  }
  T s = 0;
#pragma unroll
  for (int i = 0; i < ILP; ++i) s += acc[i];
  if (s == (T)-1.2345) out[0] = s;
}

template <int ILP>
__global__ __launch_bounds__(256) void dpp_chain(int* out, int iters) {
  int acc[ILP];
#pragma unroll
  for (int i = 0; i < ILP; ++i) acc[i] = threadIdx.x + i;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ILP; ++i) acc[i] = __builtin_amdgcn_mov_dpp(acc[i], 0x138, 0xF, 0xF, true);
  }
  int s = 0;
#pragma unroll
  for (int i = 0; i < ILP; ++i) s ^= acc[i];
  if (s == 123456789) out[0] = s;
}

template <typename K>
double run(K kernel, int blocks, int iters, double ops_per_lane_iter) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  kernel(blocks, iters);
  hipDeviceSynchronize();
  hipEventRecord(a);
  kernel(blocks, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double lanes = (double)blocks * 256;
  return lanes * iters * ops_per_lane_iter / (ms * 1e-3) / 1e12;  // T lane-ops/s
}

int main() {
  void* buf;
  hipMalloc(&buf, 64);
  const int iters = 20000;
  for (int bpc : {1, 2, 4, 8}) {
    const int blocks = 256 * bpc;
    double d1 = run([&](int bl, int it) { hipLaunchKernelGGL((add_chain<double, 1>), dim3(bl), dim3(256), 0, 0, (double*)buf, it, 1.0000001); }, blocks, iters, 2);
    double d4 = run([&](int bl, int it) { hipLaunchKernelGGL((add_chain<double, 4>), dim3(bl), dim3(256), 0, 0, (double*)buf, it, 1.0000001); }, blocks, iters, 8);
    double d8 = run([&](int bl, int it) { hipLaunchKernelGGL((add_chain<double, 8>), dim3(bl), dim3(256), 0, 0, (double*)buf, it, 1.0000001); }, blocks, iters, 16);
    double f1 = run([&](int bl, int it) { hipLaunchKernelGGL((add_chain<float, 1>), dim3(bl), dim3(256), 0, 0, (float*)buf, it, 1.0000001f); }, blocks, iters, 2);
    double f4 = run([&](int bl, int it) { hipLaunchKernelGGL((add_chain<float, 4>), dim3(bl), dim3(256), 0, 0, (float*)buf, it, 1.0000001f); }, blocks, iters, 8);
    double f8 = run([&](int bl, int it) { hipLaunchKernelGGL((add_chain<float, 8>), dim3(bl), dim3(256), 0, 0, (float*)buf, it, 1.0000001f); }, blocks, iters, 16);
    double p4 = run([&](int bl, int it) { hipLaunchKernelGGL((dpp_chain<4>), dim3(bl), dim3(256), 0, 0, (int*)buf, it); }, blocks, iters, 4);
    double p8 = run([&](int bl, int it) { hipLaunchKernelGGL((dpp_chain<8>), dim3(bl), dim3(256), 0, 0, (int*)buf, it); }, blocks, iters, 8);
    printf("blocks/CU=%d (waves/SIMD=%d): fp64 T-ops/s ilp1 %.1f ilp4 %.1f ilp8 %.1f | fp32 ilp1 %.1f ilp4 %.1f ilp8 %.1f | dpp ilp4 %.1f ilp8 %.1f\n",
           bpc, bpc, d1, d4, d8, f1, f4, f8, p4, p8);
  }
  return 0;
}
