// Post-hoc evaluation over sparse (CSR / one-hot) design matrices with the loss fused in
// (K9 + K10 of SURVEY §2.8 for the real datasets).
//
// Reference (every engine's epilogue, ref src/naive.py:166-169,190-193; ref src/util.py:136-141):
//   predy_i = X.dot(betaset[i])   (scipy CSR x dense, one round at a time)
//   loss_i  = sum(log(1 + exp(-y * predy_i))) / n        or mean((y - predy_i)^2)
// The reference's real datasets are one-hot encoded: every row has the same number of
// non-zeros and every value is 1 (ref src/arrange_real_data.py), so a prediction row is a sum
// of m gathered beta columns.
//
// MI355X design: all R betas at once.  The betas are transposed to Bt [ld, R] (one contiguous
// R-vector per feature; 100 fp64 = 800 B, the whole table 12 MB for covtype, 194 MB for amazon,
// i.e. L2 / Infinity-Cache resident), and each wave walks rows: lanes own prediction columns
// (j = lane + 64 c), a row's column indices are loaded by its first nnz lanes once and broadcast
// with readlane, and every feature costs one coalesced R-vector gather.  The loss is evaluated
// in registers, summed per column across the rows a lane visits, folded across the block's waves
// in LDS and added with one fp64 atomic per column per block; the test set also writes P.
#include <algorithm>

#include "common.h"

namespace eh {

template <typename A, int NC, int LOSS, bool VALS>
__global__ void __launch_bounds__(256)
eval_csr_loss(const long long* __restrict__ row_ptr, const int* __restrict__ col, const A* __restrict__ vals,
              long long n, const A* __restrict__ y, const A* __restrict__ Bt, int R, double* __restrict__ loss,
              A* __restrict__ P) {
  __shared__ double red[4][64 * NC];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const long long nw = static_cast<long long>(gridDim.x) * 4;
  double s[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) s[c] = 0.0;
  for (long long r = static_cast<long long>(blockIdx.x) * 4 + wid; r < n; r += nw) {
    const long long b = row_ptr[r], e = row_ptr[r + 1];
    A p[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) p[c] = A(0);
    for (long long k0 = b; k0 < e; k0 += 64) {
      const int cnt = static_cast<int>(min<long long>(64, e - k0));
      const int my = lane < cnt ? col[k0 + lane] : 0;
      A mv = A(1);
      if constexpr (VALS) mv = lane < cnt ? vals[k0 + lane] : A(0);
      // 8 features per step: their gathers are all issued before the first is consumed (a row
      // is a chain of dependent L2 / Infinity-Cache hits otherwise)
      int k = 0;
      for (; k + 8 <= cnt; k += 8) {
        A g[8][NC];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const A* __restrict__ bt = Bt + static_cast<long long>(__builtin_amdgcn_readlane(my, k + u)) * R;
#pragma unroll
          for (int c = 0; c < NC; ++c) g[u][c] = lane + 64 * c < R ? bt[lane + 64 * c] : A(0);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          A v = A(1);
          if constexpr (VALS) v = readlane_a(mv, k + u);
#pragma unroll
          for (int c = 0; c < NC; ++c) p[c] = fma(v, g[u][c], p[c]);
        }
      }
      for (; k < cnt; ++k) {
        const int f = __builtin_amdgcn_readlane(my, k);  // wave-uniform feature index
        const A* __restrict__ bt = Bt + static_cast<long long>(f) * R;
        A v = A(1);
        if constexpr (VALS) v = readlane_a(mv, k);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          const int j = lane + 64 * c;
          if (j < R) p[c] = fma(v, bt[j], p[c]);
        }
      }
    }
    const double yy = static_cast<double>(y[r]);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int j = lane + 64 * c;
      if (j < R) {
        if (P) P[r * R + j] = p[c];
        const double pp = static_cast<double>(p[c]);
        if constexpr (LOSS == kLogistic) {
          const double m = -yy * pp;  // log(1 + exp(m)), stable
          s[c] += (m > 0.0 ? m : 0.0) + log1p(exp(-fabs(m)));
        } else {
          const double d = yy - pp;
          s[c] += d * d;
        }
      }
    }
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) red[wid][lane + 64 * c] = s[c];
  __syncthreads();
  for (int j = threadIdx.x; j < 64 * NC; j += 256)
    if (j < R) atomicAdd(loss + j, (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]));
}

// dtype 0: fp64 vals/y/Bt/P, 1: fp32.  vals == nullptr: pattern-only (every stored value is 1).
hipError_t eval_csr_loss_launch(int dtype, int loss_kind, const long long* row_ptr, const int* col, const void* vals,
                                long long n, const void* y, const void* Bt, int R, double* loss, void* P,
                                hipStream_t st) {
  if (n == 0 || R == 0) return hipSuccess;
  const int nc = (R + 63) / 64;
  if (nc > 4) return hipErrorInvalidValue;  // R <= 256 betas per pass (the caller chunks)
  const unsigned blocks = static_cast<unsigned>(std::min<long long>((n + 3) / 4, 8192));
#define EH_CSR(A, NC, L, V)                                                                                   \
  hipLaunchKernelGGL((eval_csr_loss<A, NC, L, V>), dim3(blocks), dim3(256), 0, st, row_ptr, col, (const A*)vals, n, \
                     (const A*)y, (const A*)Bt, R, loss, (A*)P)
#define EH_CSR_NC(A, L, V) \
  switch (nc) {            \
    case 1: EH_CSR(A, 1, L, V); break; \
    case 2: EH_CSR(A, 2, L, V); break; \
    default: EH_CSR(A, 4, L, V); break; \
  }
#define EH_CSR_V(A, L) \
  if (vals) { EH_CSR_NC(A, L, true) } else { EH_CSR_NC(A, L, false) }
  if (dtype == 0) {
    if (loss_kind == kLogistic) { EH_CSR_V(double, kLogistic) } else { EH_CSR_V(double, kLeastSquares) }
  } else {
    if (loss_kind == kLogistic) { EH_CSR_V(float, kLogistic) } else { EH_CSR_V(float, kLeastSquares) }
  }
#undef EH_CSR_V
#undef EH_CSR_NC
#undef EH_CSR
  return hipGetLastError();
}

}  // namespace eh
