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

template <typename M, typename W>
__global__ void __launch_bounds__(256)
combine_update(const CombineArgs args, double* __restrict__ beta, double* __restrict__ u,
               double* __restrict__ hist, W* __restrict__ beta_w, double* __restrict__ g_out,
               int d, int ld, double decay, double gm, double l2, double theta, int rule,
               long long* __restrict__ stamp) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (stamp && c == 0) *stamp = wall_clock64();  // device time the round's messages were all ready
  if (c >= ld) return;
  if (c >= d) {  // padded columns stay exactly zero
    if (beta_w) beta_w[c] = W(0);
    return;
  }
  // The message rows are independent loads (remote ones in fine-grained memory, ~µs each): issue
  // them eight at a time, then accumulate in message order (the same fma chain, bitwise, as a
  // one-at-a-time loop).
  double g = 0.0;
  constexpr int kBatch = 8;
  for (int m0 = 0; m0 < args.nmsg; m0 += kBatch) {
    double v[kBatch];
#pragma unroll
    for (int k = 0; k < kBatch; ++k)
      v[k] = m0 + k < args.nmsg ? static_cast<double>(static_cast<const M*>(args.msg[m0 + k])[c]) : 0.0;
#pragma unroll
    for (int k = 0; k < kBatch; ++k)
      if (m0 + k < args.nmsg) g = fma(args.coef[m0 + k], v[k], g);
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
