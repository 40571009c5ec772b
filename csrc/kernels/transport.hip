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
// 16-byte loads/stores, makes its writes visible at system scope (block_release_system:
// every wave waits for its stores, one lane writes the L2 back), and counts itself done on
// a per-descriptor counter; the last block of a descriptor resets the counter, releases its
// tags the same way and stores the flag.  So a receiver that observes flag >= value also observes the payload, without
// relying on kernel-boundary cache semantics across devices.
//
// Integrity (integrity.h): a tagged descriptor also checksums every row it copies (LDS sums per
// row, one global add per row and block into the sender's scratch) and the last block writes
// one {round + 1, rank, checksum} tag per row into the receiver's tag slots before the flag.
#include <atomic>

#include "common.h"
#include "launchers.h"

namespace eh {

namespace {
__device__ __forceinline__ bool aborted(const int* abort) {
  return abort && __hip_atomic_load(abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

// Terms of one 16-byte vector of a row (es-byte elements starting at element j0).
__device__ __forceinline__ unsigned long long vec_terms(const uint4& v, int es, long long j0) {
  if (es == 8) {
    const unsigned long long a = (static_cast<unsigned long long>(v.y) << 32) | v.x;
    const unsigned long long b = (static_cast<unsigned long long>(v.w) << 32) | v.z;
    return tag_term(a, j0) + tag_term(b, j0 + 1);
  }
  return tag_term(v.x, j0) + tag_term(v.y, j0 + 1) + tag_term(v.z, j0 + 2) + tag_term(v.w, j0 + 3);
}
}  // namespace

__global__ void __launch_bounds__(256) put_signal(PutArgs args) {
  __shared__ unsigned long long row_sum[kMaxTagRows];
  __shared__ int s_last, s_abort;
  const int k = blockIdx.y;
  if (k >= args.n) return;
  const PutDesc& p = args.d[k];
  if (gate_closed(p.gate)) {  // a skipped stale round (launch-uniform): decide the next one's gate
    if (blockIdx.x == 0 && threadIdx.x == 0) put_decide_next_gate(p);
    return;
  }
  if (threadIdx.x == 0) s_abort = aborted(p.abort);  // one read, shared by the block
  __syncthreads();
  if (s_abort) return;  // the pump gave up: nothing is put or announced
  const bool tagged = p.tag != nullptr;
  const long long nvec = p.bytes / 16;
  const long long row_vec = tagged ? nvec / p.rows : 1;  // 16-byte vectors per row
  const int per_vec = 16 / (tagged ? p.es : 16);
  if (tagged) {
    for (int r = threadIdx.x; r < p.rows; r += blockDim.x) row_sum[r] = 0;
    __syncthreads();
  }
  const uint4* __restrict__ s = static_cast<const uint4*>(p.src);
  uint4* __restrict__ d = static_cast<uint4*>(p.dst);
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  // block-uniform trip count, so the wave reductions below run in uniform control flow
  for (long long base = static_cast<long long>(blockIdx.x) * blockDim.x; base < nvec; base += stride) {
    const long long i = base + threadIdx.x;
    const bool act = i < nvec;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (act) {
      v = s[i];
      d[i] = v;
    }
    if (tagged) {
      const long long row = act ? i / row_vec : 0;
      const unsigned long long t = act ? vec_terms(v, p.es, (i - row * row_vec) * per_vec) : 0ull;
      const int r0 = __builtin_amdgcn_readfirstlane(static_cast<int>(row));
      if (__ballot(act && row != r0) == 0) {  // the wave's vectors are all in one row
        const unsigned long long ws = wave_sum_u64(t);
        if ((threadIdx.x & 63) == 0 && ws) atomicAdd(&row_sum[r0], ws);
      } else if (act) {
        atomicAdd(&row_sum[row], t);
      }
    }
  }
  if (tagged) {
    __syncthreads();
    for (int r = threadIdx.x; r < p.rows; r += blockDim.x)
      if (row_sum[r]) atomicAdd(p.csum + r, row_sum[r]);
  }
  block_release_system(p.strict);  // this block's rows (and checksum adds) are out before its count
  if (threadIdx.x == 0) {
    // relaxed: the release above ordered the block's stores; the last block reads only the
    // checksum sums, which are L2 atomics
    const unsigned int prev = count_block_done(p.counter, p.strict);
    s_last = prev == gridDim.x - 1;
    if (s_last) __hip_atomic_store(p.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;  // block-uniform
  if (tagged) {
    for (int r = threadIdx.x; r < p.rows; r += blockDim.x) {
      const unsigned long long sum = atomicExch(p.csum + r, 0ull);  // every block's adds are in
      p.tag[r] = MsgTag{static_cast<unsigned int>(p.value), p.rank, sum};
    }
    if (p.corrupt && threadIdx.x == 0) static_cast<unsigned char*>(p.dst)[1] ^= 0x10;  // test hook
  }
  if (threadIdx.x == 0) put_stamp(p);
  block_release_system(p.strict);  // the tags (and the landing stamp) before the flag
  if (threadIdx.x == 0) {
    publish_u64(p.flag, p.value, p.strict);
    put_decide_next_gate(p);
  }
}

// Signal only (no payload): flag = value once all prior work on the stream is done.
__global__ void signal_only(unsigned long long* flag, unsigned long long value) {
  __threadfence_system();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Stale-round gate of a p2p worker round (engine.cpp WorkerPump::set_skip_stale_comm): the worker's
// beta counter (bumped behind every beta receive on its beta stream) against `at_least`, snapshotted
// into the round's gate word so every kernel of the round reads one launch-uniform value.
__global__ void gate_from_counter(const unsigned long long* counter, unsigned long long at_least, int* gate) {
  const unsigned long long v =
      __hip_atomic_load(const_cast<unsigned long long*>(counter), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(gate, v >= at_least ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Receiver check of the tagged rows of one put: one block, rows in turn (beta: one row).
__global__ void __launch_bounds__(256) verify_rows(const unsigned char* rows, const MsgTag* tags, int nrows, int ld,
                                                   int es, unsigned int round1, unsigned int rank,
                                                   IntegrityErr* err, int where) {
  __shared__ unsigned long long scratch[4];
  for (int r = 0; r < nrows; ++r) {
    const unsigned char* row = rows + static_cast<long long>(r) * ld * es;
    unsigned long long t = 0;
    for (int c = threadIdx.x; c < ld; c += blockDim.x) {
      const unsigned long long bits = es == 8 ? *reinterpret_cast<const unsigned long long*>(row + 8ll * c)
                                              : *reinterpret_cast<const unsigned int*>(row + 4ll * c);
      t += tag_term(bits, c);
    }
    const unsigned long long sum = block_sum_u64(t, scratch);
    if (threadIdx.x == 0) {
      const MsgTag g = tags[r];
      if (g.round1 != round1 || g.rank != rank || g.sum != sum)
        report_integrity(err, static_cast<int>(round1) - 1, where, static_cast<int>(rank), g, sum);
    }
  }
}

__global__ void __launch_bounds__(1024) check_list(const CheckList cl, IntegrityErr* err) {
  __shared__ int claim;
  if (threadIdx.x == 0) claim = 0;
  __syncthreads();
  check_rows_waves(cl, 0, static_cast<int>(blockDim.x >> 6), err, &claim);
}

__global__ void spin_ticks(long long ticks, const int* gate, const unsigned long long* stop, unsigned long long stop_at,
                           long long* rec) {
  if (gate_closed(gate)) return;
  const long long t0 = wall_clock64();
  long long t = t0;
  while (t - t0 < ticks) {
    // the master's run is over (its end-of-run release): nothing this rank still does can matter
    if (stop && __hip_atomic_load(const_cast<unsigned long long*>(stop), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= stop_at)
      break;
    __builtin_amdgcn_s_sleep(127);
    t = wall_clock64();
  }
  if (rec && threadIdx.x == 0) {
    rec[0] = t0;
    rec[1] = t;
  }
}

// Device ping-pong of the transport preflight (parallel/transport.py IpcTransport.preflight), one
// worker rank at a time: the master block writes pattern k into the worker's spare inbox row and
// release-stores the worker's counter; the worker block, spinning on that counter, checks the row,
// echoes it into the master's mailbox row and release-stores its own counter; the master times
// counter store -> echo seen (wall_clock64) and checks the echo.  Every wait has a deadline, so a
// missing peer ends both kernels (status[1] = 1) instead of hanging the GPU.
__device__ __forceinline__ unsigned long long ping_word(int k, int j) {
  return (static_cast<unsigned long long>(k) << 32) | static_cast<unsigned int>(j * 2654435761u);
}
__global__ void __launch_bounds__(256) ping_pong(const PingArgs a, int master) {
  __shared__ int s_ok;
  const int tid = threadIdx.x;
  int errs = 0;
  for (int k = 1; k <= a.iters; ++k) {
    if (master) {
      for (int j = tid; j < a.nwords_out; j += blockDim.x) a.out_row[j] = ping_word(k, j);
      __threadfence_system();
      __syncthreads();
      if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // see put_signal: the counter stays behind the row
        __hip_atomic_store(a.out_flag, static_cast<unsigned long long>(k), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (tid == 0) {
      const long long t0 = wall_clock64();
      int ok = 1;
      while (__hip_atomic_load(const_cast<unsigned long long*>(a.in_flag), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) <
             static_cast<unsigned long long>(k)) {
        if (wall_clock64() - t0 > a.deadline_ticks) {
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (master && a.rtt) a.rtt[k - 1] = wall_clock64() - t0;
      s_ok = ok;
    }
    __syncthreads();
    if (!s_ok) {  // block-uniform
      if (tid == 0) __hip_atomic_store(a.status + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    for (int j = tid; j < a.nwords_in; j += blockDim.x) errs += a.in_row[j] != ping_word(k, j);
    if (!master) {
      for (int j = tid; j < a.nwords_out; j += blockDim.x) a.out_row[j] = a.in_row[j];
      __threadfence_system();
      __syncthreads();
      if (tid == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(a.out_flag, static_cast<unsigned long long>(k), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();  // this round's reads done before the next round's writes
  }
  if (errs) atomicAdd(a.status, errs);
}

hipError_t ping_pong_launch(const PingArgs& a, bool master, hipStream_t st) {
  if (a.iters < 1 || !a.out_flag || !a.in_flag || !a.status || a.nwords_in < 0 || a.nwords_out < 0 ||
      (a.nwords_in && !a.in_row) || (a.nwords_out && !a.out_row))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(ping_pong, dim3(1), dim3(256), 0, st, a, master ? 1 : 0);
  return hipGetLastError();
}

namespace {
std::atomic<int> g_strict_release{1};  // launchers.h: strict until the Trainer chose the job's form
}  // namespace
bool strict_release() { return g_strict_release.load(std::memory_order_relaxed) != 0; }
void set_release_form(bool strict) { g_strict_release.store(strict ? 1 : 0, std::memory_order_relaxed); }

hipError_t put_signal_launch(const PutArgs& args, int blocks, hipStream_t st) {
  if (args.n <= 0) return hipSuccess;
  for (int k = 0; k < args.n; ++k) {
    const PutDesc& p = args.d[k];
    if (p.tag && (p.rows < 1 || p.rows > kMaxTagRows || (p.es != 4 && p.es != 8) || !p.csum ||
                  (p.bytes / 16) % p.rows != 0))
      return hipErrorInvalidValue;
  }
  PutArgs a = args;
  for (int k = 0; k < a.n; ++k) a.d[k].strict = strict_release() ? 1 : 0;  // launchers.h
  hipLaunchKernelGGL(put_signal, dim3(blocks, a.n), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t gate_launch(const unsigned long long* counter, unsigned long long at_least, int* gate, hipStream_t st) {
  if (!counter || !gate) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gate_from_counter, dim3(1), dim3(1), 0, st, counter, at_least, gate);
  return hipGetLastError();
}

hipError_t signal_launch(unsigned long long* flag, unsigned long long value, hipStream_t st) {
  hipLaunchKernelGGL(signal_only, dim3(1), dim3(1), 0, st, flag, value);
  return hipGetLastError();
}

hipError_t verify_rows_launch(const void* rows, const MsgTag* tags, int nrows, int ld, int es,
                              unsigned int round1, unsigned int rank, IntegrityErr* err, int where,
                              hipStream_t st) {
  if (nrows <= 0) return hipSuccess;
  if (!rows || !tags || (es != 4 && es != 8)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(verify_rows, dim3(1), dim3(256), 0, st, static_cast<const unsigned char*>(rows), tags, nrows,
                     ld, es, round1, rank, err, where);
  return hipGetLastError();
}

hipError_t check_list_launch(const CheckList& cl, IntegrityErr* err, hipStream_t st) {
  if (cl.n <= 0) return hipSuccess;
  if (cl.n > kMaxCheckRows || !cl.tags || (cl.es != 4 && cl.es != 8)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(check_list, dim3(1), dim3(1024), 0, st, cl, err);
  return hipGetLastError();
}

hipError_t spin_launch(long long ticks, hipStream_t st, const int* gate, const unsigned long long* stop,
                       unsigned long long stop_at, long long* rec) {
  if (ticks <= 0) return hipSuccess;
  hipLaunchKernelGGL(spin_ticks, dim3(1), dim3(64), 0, st, ticks, gate, stop, stop_at, rec);
  return hipGetLastError();
}

}  // namespace eh
