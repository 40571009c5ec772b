// Gradient-code encoding on the device: messages = E . per-partition gradients (K13 of SURVEY §2.8).
//
// Reference: every coded worker evaluates its own message over its (s+1) partitions,
//   cyclic MDS   g_w = sum_p B[w, p] * grad_p      (label encoding y_mod = B[w,p] * y,
//                                                  ref src/coded.py:92-95, 183-185)
//   FRC / AGC    g_w = sum_{p in group(w)} grad_p  (ref src/replication.py:56-68, 191-193)
// which on one machine per worker is the only option.  When several logical workers share
// a GPU they also share partitions (all members of an FRC group hold the same ones, cyclic
// neighbours overlap in s of s+1), so the GPU can stream every distinct partition from HBM
// once, produce grad_p with coefficient 1, and encode all local messages here with the sparse
// encoding matrix E (rows = local messages, CSR over the distinct partitions).  The
// residual is linear in the label coefficient, so the messages are the same sums.
//
// One thread per (message, column): a fixed-order fp64/fp32 dot over the message's few
// nonzeros of E — deterministic, no atomics, coalesced rows of grad_p.
#include "common.h"
#include "launchers.h"

namespace eh {

// sub_begin != nullptr: Gb holds row-block sums (grad_sparse.hip row-blocked column pass) and
// partition p's gradient is the sum of its rows sub_begin[p] .. sub_begin[p + 1] - 1, added first in
// row-block order -- the sub_reduce kernel's arithmetic, one launch less.
template <typename A>
__global__ void __launch_bounds__(256)
encode_messages(const A* __restrict__ Gb, const int* __restrict__ ptr, const int* __restrict__ idx,
                const double* __restrict__ coef, A* __restrict__ G, int ld, const int* __restrict__ gate,
                const int* __restrict__ sub_begin) {
  const int slot = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ld || gate_closed(gate)) return;
  const int b = ptr[slot], e = ptr[slot + 1];
  A s = A(0);
  for (int k = b; k < e; ++k) {
    A g;
    if (sub_begin) {
      // the sub-block rows sixteen loads at a time, added in row order (bitwise the serial loop; a
      // partition of covtype's shape has 13 of them: one dependent load each was ~6 us)
      g = A(0);
      int q = sub_begin[idx[k]];
      const int q1 = sub_begin[idx[k] + 1];
      const A* __restrict__ col = Gb + c;
      for (; q < q1; q += 16) {  // up to 16 loads in flight, predicated past the last one
        A x[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) x[j] = q + j < q1 ? col[static_cast<long long>(q + j) * ld] : A(0);
#pragma unroll
        for (int j = 0; j < 16; ++j)
          if (q + j < q1) g += x[j];
      }
    } else {
      g = Gb[static_cast<long long>(idx[k]) * ld + c];
    }
    s = fma(static_cast<A>(coef[k]), g, s);
  }
  G[static_cast<long long>(slot) * ld + c] = s;
}

hipError_t encode_messages_launch(int dtype, const void* Gb, const int* ptr, const int* idx, const double* coef,
                                  void* G, int nslots, int ld, hipStream_t st, const int* gate, const int* sub_begin) {
  if (nslots == 0) return hipSuccess;
  const dim3 block(256), grid(ceil_div(ld, 256), nslots);
  if (dtype == 0)
    hipLaunchKernelGGL(encode_messages<double>, grid, block, 0, st, (const double*)Gb, ptr, idx, coef, (double*)G, ld, gate,
                       sub_begin);
  else
    hipLaunchKernelGGL(encode_messages<float>, grid, block, 0, st, (const float*)Gb, ptr, idx, coef, (float*)G, ld, gate,
                       sub_begin);
  return hipGetLastError();
}

}  // namespace eh
