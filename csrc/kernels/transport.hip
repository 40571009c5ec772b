// Put-with-signal kernel of the IPC mailbox transport (SURVEY §5.8 "HIP IPC mailbox").
//
// Reference primitive replaced: comm.Isend([g, DOUBLE], dest=0, tag=i) / Irecv on the
// master (ref src/naive.py:150, :74-79) and the master's p2p "broadcast" of beta
// (ref src/naive.py:97-98).  Here a message is copied by the SENDING GPU straight into
// the receiver's HBM (an IPC-mapped pointer; over xGMI when the peer is another MI355X)
// and then announced by a 64-bit generation flag in shared host memory that the
// receiver's host polls (csrc/runtime/collector.cpp flag probes / ipc.cpp).
//
// Ordering (the classic put + signal pattern): every block copies its chunk with
// 16-byte loads/stores, makes its writes visible at system scope
// (__threadfence_system), and counts itself done on a per-descriptor counter; the
// last block of a descriptor resets the counter and release-stores the flag at system
// scope.  So a receiver that observes flag >= value also observes the payload, without
// relying on kernel-boundary cache semantics across devices.
#include "common.h"
#include "launchers.h"

namespace eh {

__global__ void __launch_bounds__(256) put_signal(PutArgs args) {
  const int k = blockIdx.y;
  if (k >= args.n) return;
  const PutDesc& p = args.d[k];
  const long long nvec = p.bytes / 16;
  const uint4* __restrict__ s = static_cast<const uint4*>(p.src);
  uint4* __restrict__ d = static_cast<uint4*>(p.dst);
  for (long long i = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x; i < nvec;
       i += static_cast<long long>(gridDim.x) * blockDim.x)
    d[i] = s[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int prev = __hip_atomic_fetch_add(p.counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(p.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      // ROCm 7.2 / gfx950: after a returned atomic the compiler may drop the wait that follows
      // the fence's write-back, letting the flag overtake it; keep the wait explicitly.
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(p.flag, p.value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// Signal only (no payload): flag = value once all prior work on the stream is done.
__global__ void signal_only(unsigned long long* flag, unsigned long long value) {
  __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t put_signal_launch(const PutArgs& args, int blocks, hipStream_t st) {
  if (args.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(put_signal, dim3(blocks, args.n), dim3(256), 0, st, args);
  return hipGetLastError();
}

hipError_t signal_launch(unsigned long long* flag, unsigned long long value, hipStream_t st) {
  hipLaunchKernelGGL(signal_only, dim3(1), dim3(1), 0, st, flag, value);
  return hipGetLastError();
}

}  // namespace eh
