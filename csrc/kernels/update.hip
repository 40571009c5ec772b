// Master-side decode-combine + GD/AGD model update in ONE launch (K5 + K7 + K8 of SURVEY §2.8).
//
// Reference semantics:
//   combine   g = sum_m a_m * msg_m                      ref src/coded.py:147-149 (lstsq decode),
//                                                        src/approximate_coding.py:150-158 (FRC first-per-group),
//                                                        src/naive.py:109 (plain sum)
//   GD        beta = (1 - 2 alpha eta) beta - (eta/n) g   ref src/naive.py:112-115
//   AGD       theta = 2/(i+2); y = (1-theta) beta + theta u
//             beta' = y - (eta/n) g - 2 alpha eta beta; u = beta + (beta'-beta)/theta   ref src/naive.py:116-122
//             (avoidstragg rescales eta/n by W/(W-s): ref src/avoidstragg.py:116)
//
// The decode coefficients a_m (fp64, solved on the host) and the message pointers are
// passed by value in the kernel arguments, so a round's combine+update is a single
// launch with no host->device copies.  Every column is independent: a thread per
// column streams the m message rows (coalesced), keeps everything in fp64 registers
// and writes beta, u, the betaset history row and the worker-dtype copy of beta that
// the next round's gradient kernels (and the p2p sends) read.
#include "common.h"
#include "launchers.h"

namespace eh {

// Integrity (args.tags != nullptr, integrity.h): while it streams the message rows, every block
// also sums the checksum terms of its columns of each tagged (mailbox) row — one wave reduction
// per tagged row, LDS, one global add per row and block — and the last block compares the sums
// with the senders' tags.  A mismatch is reported to the host-mapped record (the pump raises a
// named error); the update itself cannot be held back without a grid-wide barrier.
template <typename M, typename W>
__global__ void __launch_bounds__(256)
combine_update(const CombineArgs args, double* __restrict__ beta, double* __restrict__ u,
               double* __restrict__ hist, W* __restrict__ beta_w, double* __restrict__ g_out,
               int d, int ld, double decay, double gm, double l2, double theta, int rule,
               long long* __restrict__ stamp) {
  __shared__ unsigned long long vs[kMaxMsgs];
  __shared__ int s_last;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  const bool verify = args.tags != nullptr;  // kernel-uniform
  if (stamp && c == 0) *stamp = wall_clock64();  // device time the round's messages were all ready
  if (verify) {
    for (int m = threadIdx.x; m < args.nmsg; m += blockDim.x) vs[m] = 0;
    __syncthreads();
  } else if (c >= ld) {
    return;
  }
  const bool col = c < d;  // padded columns (d <= c < ld) stay exactly zero
  // The message rows are independent loads (remote ones in fine-grained memory, ~µs each): issue
  // them eight at a time, then accumulate in message order (the same fma chain, bitwise, as a
  // one-at-a-time loop).
  double g = 0.0;
  constexpr int kBatch = 8;
  for (int m0 = 0; m0 < args.nmsg; m0 += kBatch) {
    M raw[kBatch];
#pragma unroll
    for (int k = 0; k < kBatch; ++k)  // padded columns too: the checksum covers the whole row
      raw[k] = (c < ld && m0 + k < args.nmsg) ? static_cast<const M*>(args.msg[m0 + k])[c] : M(0);
#pragma unroll
    for (int k = 0; k < kBatch; ++k)
      if (m0 + k < args.nmsg) g = fma(args.coef[m0 + k], static_cast<double>(raw[k]), g);
    if (verify) {
#pragma unroll
      for (int k = 0; k < kBatch; ++k) {
        if (m0 + k >= args.nmsg || args.tag_row[m0 + k] < 0) continue;  // uniform
        const unsigned long long t = wave_sum_u64(c < ld ? tag_term(elem_bits(raw[k]), c) : 0ull);
        if ((threadIdx.x & 63) == 0 && t) atomicAdd(&vs[m0 + k], t);
      }
    }
  }
  if (verify) {
    __syncthreads();
    for (int m = threadIdx.x; m < args.nmsg; m += blockDim.x)
      if (args.tag_row[m] >= 0 && vs[m]) atomicAdd(args.vsum + m, vs[m]);
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned int prev = __hip_atomic_fetch_add(args.vcount, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      s_last = prev == gridDim.x - 1;
      if (s_last) __hip_atomic_store(args.vcount, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (s_last) {
      for (int m = threadIdx.x; m < args.nmsg; m += blockDim.x) {
        if (args.tag_row[m] < 0) continue;
        const unsigned long long sum = atomicExch(args.vsum + m, 0ull);
        const MsgTag tg = args.tags[args.tag_row[m]];
        if (tg.round1 != args.round1 || tg.rank != args.tag_rank[m] || tg.sum != sum)
          report_integrity(args.err, static_cast<int>(args.round1) - 1, (args.slot << 16) | args.tag_row[m],
                           args.tag_rank[m], tg, sum);
      }
    }
    if (c >= ld) return;
  }
  if (!col) {
    if (beta_w) beta_w[c] = W(0);
    return;
  }
  const double b = beta[c];
  double nb;
  if (rule == 0) {  // GD
    nb = decay * b - gm * g;
  } else {  // AGD (gradient evaluated at beta, exactly as the reference)
    const double yt = (1.0 - theta) * b + theta * u[c];
    nb = yt - gm * g - l2 * b;
    u[c] = b + (nb - b) * (1.0 / theta);
  }
  beta[c] = nb;
  if (hist) hist[c] = nb;
  if (beta_w) beta_w[c] = static_cast<W>(nb);
  if (g_out) g_out[c] = g;
}

// msg dtype: 0 fp64, 1 fp32; worker beta dtype: 0 fp64, 1 fp32
hipError_t combine_update_launch(const CombineArgs& args, int msg_dtype, int w_dtype,
                                 double* beta, double* u, double* hist, void* beta_w,
                                 double* g_out, int d, int ld, double decay, double gm,
                                 double l2, double theta, int rule, hipStream_t st, long long* stamp) {
  const dim3 block(256), grid(ceil_div(ld, 256));
  if (msg_dtype == 0 && w_dtype == 0)
    hipLaunchKernelGGL((combine_update<double, double>), grid, block, 0, st, args, beta, u, hist, (double*)beta_w, g_out, d, ld, decay, gm, l2, theta, rule, stamp);
  else if (msg_dtype == 0 && w_dtype == 1)
    hipLaunchKernelGGL((combine_update<double, float>), grid, block, 0, st, args, beta, u, hist, (float*)beta_w, g_out, d, ld, decay, gm, l2, theta, rule, stamp);
  else if (msg_dtype == 1 && w_dtype == 0)
    hipLaunchKernelGGL((combine_update<float, double>), grid, block, 0, st, args, beta, u, hist, (double*)beta_w, g_out, d, ld, decay, gm, l2, theta, rule, stamp);
  else
    hipLaunchKernelGGL((combine_update<float, float>), grid, block, 0, st, args, beta, u, hist, (float*)beta_w, g_out, d, ld, decay, gm, l2, theta, rule, stamp);
  return hipGetLastError();
}

__global__ void stamp_kernel(long long* out) {
  if (threadIdx.x == 0) *out = wall_clock64();
}

hipError_t stamp_launch(long long* out, hipStream_t st) {
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, st, out);
  return hipGetLastError();
}

}  // namespace eh
