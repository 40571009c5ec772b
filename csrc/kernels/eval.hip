// Post-hoc evaluation GEMM on MFMA with a fused loss epilogue (K9 + K10 of SURVEY §2.8).
//
// Reference (master epilogue, every engine; ref src/naive.py:186-198):
//   for i in range(rounds):  predy = X.dot(betaset[i]);  loss_i = sum(log(1+exp(-y*predy)))/n
//   (least squares: mean_squared_error(y, predy); ref src/util.py:139-141)
// i.e. P = X . B^T  (n x d times d x R) — a real GEMM, so it runs on the matrix cores:
//   fp64 X : v_mfma_f64_16x16x4_f64   (exact fp64, matches the numpy reference)
//   fp32 / bf16 X : v_mfma_f32_16x16x4_f32 (exact f32 products, bf16 widened on staging)
// Tiling: 256-thread workgroup = 4 waves = 64 rows x (16*NT) columns of P; K staged
// through LDS in 32-deep tiles (row stride padded to 34 elements: conflict-free
// ds_read_b64 for the 16x4 fragment pattern).  The epilogue applies softplus(-y p) or
// (y-p)^2, reduces over the 64 rows (lane shuffles + LDS), and adds one value per
// column per workgroup into the fp64 loss vector; optionally P itself is written (the
// test-set predictions feed the AUC).
#include "common.h"

namespace eh {

using f64x4 = __attribute__((ext_vector_type(4))) double;
using f32x4 = __attribute__((ext_vector_type(4))) float;

template <typename A> struct MfmaT;
template <> struct MfmaT<double> {
  using acc = f64x4;
  __device__ __forceinline__ static acc mma(double a, double b, acc c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // D layout: col = lane & 15, row = (lane >> 4) + 4 * reg
  __device__ __forceinline__ static int row_of(int lane, int reg) { return (lane >> 4) + 4 * reg; }
};
template <> struct MfmaT<float> {
  using acc = f32x4;
  __device__ __forceinline__ static acc mma(float a, float b, acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // D layout: col = lane & 15, row = 4 * (lane >> 4) + reg
  __device__ __forceinline__ static int row_of(int lane, int reg) { return 4 * (lane >> 4) + reg; }
};

template <typename T, typename A>
__device__ __forceinline__ A load_elem(const T* p);
template <> __device__ __forceinline__ double load_elem<double, double>(const double* p) { return *p; }
template <> __device__ __forceinline__ float load_elem<float, float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float load_elem<bf16_t, float>(const bf16_t* p) { return bf16_to_f32(p->bits); }

constexpr int kKT = 32;   // K tile
constexpr int kKS = 34;   // padded LDS row stride (elements)

template <typename T, typename A, int NT, int LOSS>
__global__ void __launch_bounds__(256)
eval_gemm_loss(const T* __restrict__ X, long long ldx, long long n, int d,
               const A* __restrict__ y, const A* __restrict__ B, int ldb, int R,
               double* __restrict__ loss, A* __restrict__ P) {
  using M = MfmaT<A>;
  constexpr int NB = 16 * NT;
  __shared__ A Xs[64 * kKS];
  __shared__ A Bs[NB * kKS];
  __shared__ double red[4][NB];

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const long long row0 = static_cast<long long>(blockIdx.x) * 64;
  const int col0 = blockIdx.y * NB;

  typename M::acc acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = typename M::acc{0, 0, 0, 0};

  for (int k0 = 0; k0 < d; k0 += kKT) {
    // Stage X tile [64][32]: thread -> (row = idx / 32, k = idx % 32), 8 elements each.
    for (int idx = threadIdx.x; idx < 64 * kKT; idx += 256) {
      const int r = idx / kKT, k = idx % kKT;
      const long long gr = row0 + r;
      const int gk = k0 + k;
      Xs[r * kKS + k] = (gr < n && gk < d) ? load_elem<T, A>(X + gr * ldx + gk) : A(0);
    }
    // Stage B tile [NB][32] from betaset rows (k contiguous).
    for (int idx = threadIdx.x; idx < NB * kKT; idx += 256) {
      const int j = idx / kKT, k = idx % kKT;
      const int gj = col0 + j;
      const int gk = k0 + k;
      Bs[j * kKS + k] = (gj < R && gk < d) ? B[static_cast<long long>(gj) * ldb + gk] : A(0);
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < kKT; ks += 4) {
      const A a = Xs[(wid * 16 + (lane & 15)) * kKS + ks + (lane >> 4)];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const A b = Bs[(t * 16 + (lane & 15)) * kKS + ks + (lane >> 4)];
        acc[t] = M::mma(a, b, acc[t]);
      }
    }
    __syncthreads();
  }

  // Epilogue: per-element loss, reduce over this wave's 16 rows, then over 4 waves.
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = col0 + t * 16 + (lane & 15);
    double s = 0.0;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const long long gr = row0 + wid * 16 + M::row_of(lane, reg);
      if (gr < n && j < R) {
        const A p = acc[t][reg];
        if (P) P[gr * R + j] = p;
        const double yy = static_cast<double>(y[gr]);
        const double pp = static_cast<double>(p);
        double l;
        if constexpr (LOSS == kLogistic) {
          const double m = -yy * pp;  // log(1 + exp(m)), stable
          l = (m > 0.0 ? m : 0.0) + log1p(exp(-fabs(m)));
        } else {
          const double e = yy - pp;
          l = e * e;
        }
        s += l;
      }
    }
    s += __shfl_xor(s, 16, kWave);
    s += __shfl_xor(s, 32, kWave);
    if (lane < 16) red[wid][t * 16 + lane] = s;
  }
  __syncthreads();
  for (int j = threadIdx.x; j < NB; j += 256) {
    const int gj = col0 + j;
    if (gj < R) atomicAdd(loss + gj, red[0][j] + red[1][j] + red[2][j] + red[3][j]);
  }
}

// x_dtype: 0 fp64, 1 fp32, 2 bf16.  B/y/P are fp64 for x_dtype 0, fp32 otherwise.
hipError_t eval_gemm_loss_launch(int x_dtype, int loss_kind, const void* X, long long ldx,
                                 long long n, int d, const void* y, const void* B, int ldb,
                                 int R, double* loss, void* P, hipStream_t st) {
  constexpr int NT = 8;
  const dim3 block(256);
  const dim3 grid(static_cast<unsigned>((n + 63) / 64), ceil_div(R, 16 * NT));
  if (n == 0 || R == 0) return hipSuccess;
#define EH_EVAL(T, A, L) \
  hipLaunchKernelGGL((eval_gemm_loss<T, A, NT, L>), grid, block, 0, st, (const T*)X, ldx, n, d, (const A*)y, (const A*)B, ldb, R, loss, (A*)P)
  if (x_dtype == 0) {
    if (loss_kind == kLogistic) EH_EVAL(double, double, kLogistic); else EH_EVAL(double, double, kLeastSquares);
  } else if (x_dtype == 1) {
    if (loss_kind == kLogistic) EH_EVAL(float, float, kLogistic); else EH_EVAL(float, float, kLeastSquares);
  } else {
    if (loss_kind == kLogistic) EH_EVAL(bf16_t, float, kLogistic); else EH_EVAL(bf16_t, float, kLeastSquares);
  }
#undef EH_EVAL
  return hipGetLastError();
}

}  // namespace eh
