// Cross-process ordering of the IPC halo pulls (runtime/ipc_transport.cpp).
//
// Ranks are processes (one per GPU, or several sharing one); each pulls its
// ghost rows straight out of its neighbours' fields (IPC-mapped). The ordering
// the reference gets from two blocking MPI_Sendrecv per step
// (fortran/hip/heat.F90:212-213) — and the loopback / peer transports get from
// events — comes here from two monotonic counters per rank in host-shared
// memory, advanced ON THE STREAM by two one-thread kernels around the copies:
//   arrive: c = done[me] (exchanges this rank completed); ready[me] = c + 1
//           (its bands of exchange c are written: stream order); then wait
//           until every neighbour p has ready[p] >= c + 1 (its bands written)
//           and done[p] >= c (its pulls of exchange c - 1 — which read this
//           rank's buffer that the next bands overwrite — are finished)
//   (the hipMemcpyAsync pulls)
//   depart: done[me] = c + 1
// No host thread waits per cycle, and nothing in the exchange bakes in a cycle
// number: the counters live in memory, so a captured hipGraph replays it.
// Stores are plain vector stores with system-scope release (the memory is
// host-coherent); the wait spins on system-scope acquire loads with s_sleep,
// and gives up on an abort word or a wall-clock timeout (ctrl[1] records who
// timed out), so a dead peer never leaves a wave spinning.
#include <hip/hip_runtime.h>

#include "heat2d/kernels.hpp"

namespace heat2d {
namespace kern {
namespace {

__device__ __forceinline__ uint64_t ld_acq(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_rel(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(64) void ipc_arrive_kernel(IpcSlot* slots, uint64_t* ctrl, int me, int p0, int p1,
                                                        uint64_t timeout_ticks) {
  if (threadIdx.x != 0) return;
  __threadfence_system();  // this XCD's dirty lines (the band rows) out to memory before the flag
  const uint64_t c = ld_acq(&slots[me].done);
  st_rel(&slots[me].ready, c + 1);
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < 2; ++i) {
    const int p = i ? p1 : p0;
    if (p < 0) continue;
    while (ld_acq(&slots[p].ready) < c + 1 || ld_acq(&slots[p].done) < c) {
      if (ld_acq(&ctrl[0]) != 0) return;  // aborted: drain
      if (wall_clock64() - t0 > timeout_ticks) {
        // the host's check() reports it; the abort word makes every rank's
        // waits return (their hosts then fail at their next synchronisation,
        // before any result of these unsynchronised halos is handed out)
        st_rel(&ctrl[1], (uint64_t)me + 1);
        st_rel(&ctrl[0], (uint64_t)me + 1);
        return;
      }
      __builtin_amdgcn_s_sleep(4);
    }
  }
}

__global__ __launch_bounds__(64) void ipc_depart_kernel(IpcSlot* slots, int me) {
  if (threadIdx.x != 0) return;
  const uint64_t c = ld_acq(&slots[me].done);
  st_rel(&slots[me].done, c + 1);
}

}  // namespace

void launch_ipc_arrive(IpcSlot* slots, uint64_t* ctrl, int me, int p0, int p1, uint64_t timeout_ticks,
                       hipStream_t stream) {
  hipLaunchKernelGGL(ipc_arrive_kernel, dim3(1), dim3(64), 0, stream, slots, ctrl, me, p0, p1, timeout_ticks);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(__FILE__, __LINE__, std::string("ipc_arrive launch: ") + hipGetErrorString(e));
}

void launch_ipc_depart(IpcSlot* slots, int me, hipStream_t stream) {
  hipLaunchKernelGGL(ipc_depart_kernel, dim3(1), dim3(64), 0, stream, slots, me);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) fail(__FILE__, __LINE__, std::string("ipc_depart launch: ") + hipGetErrorString(e));
}

}  // namespace kern
}  // namespace heat2d
