// Task tables of the dense worker-gradient kernels (grad_dense.hip, grad_mfma.hip); built on the
// host by erasurehead_amd/ops/grad.py (DenseGradPlan) with the same byte layout.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace eh {

struct Segment {
  const void* X;      // [nrows, ld] row-major, storage type T
  const void* y;      // [nrows] labels, accumulator type A
  double coef;        // label encoding coefficient (cyclic MDS B[w, part]); 1 otherwise
  long long nrows;
};

struct Task {
  int slot;       // output message index
  int seg;        // segment index
  int row_begin;  // rows of the segment handled by this workgroup
  int row_end;
  int slab;       // slab row of this task's partial sum (tasks are dispatched in replica-
                  // interleaved order; slab rows stay contiguous per message slot)
};

// grad_mfma.hip: bf16 replica bundles on the matrix cores (R task slots per workgroup, ld <= 1024)
hipError_t grad_mfma_launch(int loss, const Segment* segs, const Task* tasks, int ntasks, int R, const float* beta,
                            float* slab, int ld, hipStream_t st);
bool mfma_geometry(int ld, int* rows, int* pieces, int* nstage, size_t* lds);

}  // namespace eh
