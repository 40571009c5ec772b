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
#include <cstdlib>

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

// ---- v2: 128-row tiles, 16-byte staging loads, register prefetch of the next K tile ---------
// Each wave owns 32 rows (2 MFMA m-tiles) x 112 columns (7 n-tiles): 14 independent
// accumulators per wave keep the matrix pipe busy, and every B fragment read from LDS feeds
// two MFMAs.  The next K tile is fetched into registers (16-byte loads) while the current one
// is multiplied out of LDS, so HBM latency hides behind the MFMA chain; 2 blocks per CU.
constexpr int kBM2 = 128;  // rows per block
constexpr int kNT2 = 7;    // 16-column n-tiles per wave (112 columns: R = 100 wastes 12 %)

template <typename T, typename A, int LOSS>
__global__ void __launch_bounds__(256, 2)
eval_gemm_loss_v2(const T* __restrict__ X, long long ldx, long long n, int d,
                  const A* __restrict__ y, const A* __restrict__ B, int ldb, int R,
                  double* __restrict__ loss, A* __restrict__ P) {
  using M = MfmaT<A>;
  constexpr int NT = kNT2;
  constexpr int NB = 16 * NT;
  constexpr int XV = Vec16<T>::N;
  constexpr int BV = Vec16<A>::N;
  __shared__ A Xs[kBM2 * kKS];
  __shared__ A Bs[NB * kKS];
  __shared__ double red[4][NB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const long long row0 = static_cast<long long>(blockIdx.x) * kBM2;
  const int col0 = blockIdx.y * NB;
  // staging: thread -> (row or column tid/2, 16 consecutive k starting at (tid&1)*16)
  const int sr = tid >> 1, sk = (tid & 1) * 16;
  const bool xok = row0 + sr < n;
  const T* __restrict__ xrow = X + (xok ? row0 + sr : 0) * ldx;
  const bool bok = sr < NB && col0 + sr < R;
  const A* __restrict__ brow = B + static_cast<long long>(bok ? col0 + sr : 0) * ldb;

  A xr[16], br[16];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int v = 0; v < 16 / XV; ++v) {
      const int gk = k0 + sk + v * XV;
      A t[XV];
      if (xok && gk < ldx) {
        Vec16<T>::load(xrow + gk, t);
      } else {
#pragma unroll
        for (int e = 0; e < XV; ++e) t[e] = A(0);
      }
#pragma unroll
      for (int e = 0; e < XV; ++e) xr[v * XV + e] = gk + e < d ? t[e] : A(0);
    }
#pragma unroll
    for (int v = 0; v < 16 / BV; ++v) {
      const int gk = k0 + sk + v * BV;
      A t[BV];
      if (bok && gk < ldb) {
        Vec16<A>::load(brow + gk, t);
      } else {
#pragma unroll
        for (int e = 0; e < BV; ++e) t[e] = A(0);
      }
#pragma unroll
      for (int e = 0; e < BV; ++e) br[v * BV + e] = gk + e < d ? t[e] : A(0);
    }
  };

  typename M::acc acc[2][NT];
#pragma unroll
  for (int m = 0; m < 2; ++m)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[m][t] = typename M::acc{0, 0, 0, 0};

  fetch(0);
  for (int k0 = 0; k0 < d; k0 += kKT) {
    __syncthreads();  // the previous tile's MFMA reads are done
#pragma unroll
    for (int e = 0; e < 16; ++e) Xs[sr * kKS + sk + e] = xr[e];
    if (sr < NB) {
#pragma unroll
      for (int e = 0; e < 16; ++e) Bs[sr * kKS + sk + e] = br[e];
    }
    __syncthreads();
    if (k0 + kKT < d) fetch(k0 + kKT);  // in flight while this tile is multiplied
#pragma unroll
    for (int ks = 0; ks < kKT; ks += 4) {
      const int fr = lane & 15, fk = ks + (lane >> 4);
      const A a0 = Xs[(wid * 32 + fr) * kKS + fk];
      const A a1 = Xs[(wid * 32 + 16 + fr) * kKS + fk];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const A b = Bs[(t * 16 + fr) * kKS + fk];
        acc[0][t] = M::mma(a0, b, acc[0][t]);
        acc[1][t] = M::mma(a1, b, acc[1][t]);
      }
    }
  }

  // Epilogue: per-element loss, reduce over the block's rows per column.
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int j = col0 + t * 16 + (lane & 15);
    double s = 0.0;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const long long gr = row0 + wid * 32 + m * 16 + M::row_of(lane, reg);
        if (gr < n && j < R) {
          const A p = acc[m][t][reg];
          if (P) P[gr * R + j] = p;
          const double yy = static_cast<double>(y[gr]);
          const double pp = static_cast<double>(p);
          double l;
          if constexpr (LOSS == kLogistic) {
            const double mm = -yy * pp;
            l = (mm > 0.0 ? mm : 0.0) + log1p(exp(-fabs(mm)));
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
  for (int j = tid; j < NB; j += 256) {
    const int gj = col0 + j;
    if (gj < R) atomicAdd(loss + gj, (red[0][j] + red[1][j]) + (red[2][j] + red[3][j]));
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
  // v2 needs 16-byte aligned rows (every tensor the engine builds: ld is a vector multiple)
  const int xv = x_dtype == 0 ? 2 : (x_dtype == 1 ? 4 : 8), bv = x_dtype == 0 ? 2 : 4;
  const bool aligned = ldx % xv == 0 && ldb % bv == 0 && reinterpret_cast<uintptr_t>(X) % 16 == 0 &&
                       reinterpret_cast<uintptr_t>(B) % 16 == 0;
  if (aligned) {
    const dim3 grid2(static_cast<unsigned>((n + kBM2 - 1) / kBM2), ceil_div(R, 16 * kNT2));
#define EH_EVAL2(T, A, L) \
  hipLaunchKernelGGL((eval_gemm_loss_v2<T, A, L>), grid2, block, 0, st, (const T*)X, ldx, n, d, (const A*)y, (const A*)B, ldb, R, loss, (A*)P)
    if (x_dtype == 0) {
      if (loss_kind == kLogistic) EH_EVAL2(double, double, kLogistic); else EH_EVAL2(double, double, kLeastSquares);
    } else if (x_dtype == 1) {
      if (loss_kind == kLogistic) EH_EVAL2(float, float, kLogistic); else EH_EVAL2(float, float, kLeastSquares);
    } else {
      if (loss_kind == kLogistic) EH_EVAL2(bf16_t, float, kLogistic); else EH_EVAL2(bf16_t, float, kLeastSquares);
    }
#undef EH_EVAL2
    return hipGetLastError();
  }
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
