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

// Which dense-gradient kernel a plan launches: chosen on the host by erasurehead_amd/ops/grad.py
// choose_kernel (a pure function of precision, row width, replication and rows per CU, pinned by
// tests/test_plan_tables.py) and passed typed through the bindings.
enum GradKind : int {
  kGradFused = 0,   // a wave per row (grad_dense_fused / _pair): distinct rows, no co-located replicas
  kGradMulti = 1,   // one-wave replica bundles: rows in registers, every replica from them (grad_dense_multi)
  kGradStaged = 2,  // LDS-staged replica bundles: rows through an LDS ring, a wave per replica
  kGradMfma = 3,    // bf16 replica bundles on MFMA (grad_mfma.hip)
  kGradWide = 4,    // a workgroup per row, 2048 < d <= 8192 fp64 / 16384 fp32 (grad_dense_wide)
};
struct KernelChoice {
  int kind = kGradFused;
  int replicas = 1;  // bundle kinds: task slots (co-located replicas) per bundle
  int fold = 0;      // multi: 4 bundles of one partition per workgroup, folded through LDS
  int lane_epi = 0;  // multi (folded): reduce-scatter + one lane per replica evaluates its residual
  int pair = 0;      // staged: two rows per step share one reduction and one residual evaluation
  int wpr = 0;       // staged: waves per replica (0: 4 / replicas)
  int rows = 2;      // fused: rows in flight per wave (1, 2 = the interleaved pair kernel, 4)
  int beta_lds = 0;  // fused: beta in LDS instead of registers
};

// grad_mfma.hip: bf16 replica bundles on the matrix cores (R task slots per workgroup, ld <= 1024)
hipError_t grad_mfma_launch(int loss, const Segment* segs, const Task* tasks, int ntasks, int R, const float* beta,
                            float* slab, int ld, hipStream_t st, const int* gate = nullptr);
bool mfma_geometry(int ld, int* rows, int* pieces, int* nstage, size_t* lds);

}  // namespace eh
