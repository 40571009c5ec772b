// Worker gradient for sparse (one-hot CSR) design matrices — K4 of SURVEY §2.8.
//
// Reference: the real datasets (amazon / covtype / kc_house / dna) are scipy CSR
// matrices whose values are all 1.0 (ref src/arrange_real_data.py one-hot encoders), and
// workers evaluate X_current.dot(beta) and X_current.T.dot(r) with scipy
// (ref src/replication.py:63-68, src/coded.py:43-46).
//
// MI355X design, two launches per round for every logical worker on this GPU:
//   pass 1 (row pass): a 16-lane group per row sums val * beta[col] over the row's
//     nonzeros (beta stays in L2: <= 242k fp64), reduces with lane shuffles and writes
//     the loss residual r[row] (label encoding coefficient per row).
//   pass 2 (column pass): the transposed product uses a CSC twin stored as COO sorted
//     by key = slot * ld + col.  Each lane takes one entry, the wave does a segmented
//     Hillis-Steele scan keyed on the (sorted) column, and only the last lane of each
//     run issues one float atomic add: one atomic per distinct column per wave
//     instead of one per nonzero.
// Pattern-only storage: vals == nullptr means every stored value is 1.0 (one-hot).
#include "common.h"

namespace eh {

template <typename A, int LOSS, int G>
__global__ void __launch_bounds__(256)
csr_rowpass(const long long* __restrict__ row_ptr, const int* __restrict__ col_idx,
            const A* __restrict__ vals,
            const A* __restrict__ y, const A* __restrict__ coef, const A* __restrict__ beta,
            A* __restrict__ rbuf, long long nrows, int ld) {
  const long long gid = (static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x);
  const long long row = gid / G;
  const int sub = threadIdx.x % G;
  if (row >= nrows) return;  // whole group exits together (G divides 64)
  const long long b = row_ptr[row], e = row_ptr[row + 1];
  A z = A(0);
  for (long long k = b + sub; k < e; k += G) {
    const A v = vals ? vals[k] : A(1);
    z = fma(v, beta[col_idx[k]], z);
  }
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) z += __shfl_xor(z, off, G);
  if (sub == 0) rbuf[row] = residual<LOSS, A>(z, y[row], coef[row]);
}

template <typename A>
__global__ void __launch_bounds__(256)
coo_colpass(const long long* __restrict__ keys, const int* __restrict__ rows,
            const A* __restrict__ vals, const A* __restrict__ rbuf, A* __restrict__ G,
            long long nnz) {
  const long long e = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const bool live = e < nnz;
  long long key = live ? keys[e] : -1;
  A v = live ? (vals ? vals[e] : A(1)) * rbuf[rows[e]] : A(0);
  // Segmented inclusive scan over equal keys (keys are sorted, runs are contiguous).
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const A vu = __shfl_up(v, off, kWave);
    const long long ku = __shfl_up(key, off, kWave);
    if (lane >= off && ku == key) v += vu;
  }
  const long long kn = __shfl_down(key, 1, kWave);
  const bool last = (lane == kWave - 1) || (kn != key);
  if (live && last) atomicAdd(G + key, v);
}

hipError_t grad_sparse_launch(int dtype, int loss, const long long* row_ptr, const int* col_idx,
                              const void* vals, const void* y, const void* coef,
                              const void* beta, void* rbuf, long long nrows,
                              const long long* keys, const int* rows, const void* cvals,
                              long long nnz, void* G, long long gsize, int ld, hipStream_t st) {
  constexpr int Gs = 16;
  const dim3 block(256);
  const dim3 grid1(static_cast<unsigned>((nrows * Gs + 255) / 256));
  const dim3 grid2(static_cast<unsigned>((nnz + 255) / 256));
  const size_t esz = dtype == 0 ? sizeof(double) : sizeof(float);
  hipError_t e = hipMemsetAsync(G, 0, gsize * esz, st);
  if (e != hipSuccess) return e;
  if (nrows == 0) return hipSuccess;
  if (dtype == 0) {
    if (loss == kLogistic)
      hipLaunchKernelGGL((csr_rowpass<double, kLogistic, Gs>), grid1, block, 0, st, row_ptr, col_idx, (const double*)vals, (const double*)y, (const double*)coef, (const double*)beta, (double*)rbuf, nrows, ld);
    else
      hipLaunchKernelGGL((csr_rowpass<double, kLeastSquares, Gs>), grid1, block, 0, st, row_ptr, col_idx, (const double*)vals, (const double*)y, (const double*)coef, (const double*)beta, (double*)rbuf, nrows, ld);
    if (nnz > 0)
      hipLaunchKernelGGL((coo_colpass<double>), grid2, block, 0, st, keys, rows, (const double*)cvals, (const double*)rbuf, (double*)G, nnz);
  } else {
    if (loss == kLogistic)
      hipLaunchKernelGGL((csr_rowpass<float, kLogistic, Gs>), grid1, block, 0, st, row_ptr, col_idx, (const float*)vals, (const float*)y, (const float*)coef, (const float*)beta, (float*)rbuf, nrows, ld);
    else
      hipLaunchKernelGGL((csr_rowpass<float, kLeastSquares, Gs>), grid1, block, 0, st, row_ptr, col_idx, (const float*)vals, (const float*)y, (const float*)coef, (const float*)beta, (float*)rbuf, nrows, ld);
    if (nnz > 0)
      hipLaunchKernelGGL((coo_colpass<float>), grid2, block, 0, st, keys, rows, (const float*)cvals, (const float*)rbuf, (float*)G, nnz);
  }
  return hipGetLastError();
}

}  // namespace eh
