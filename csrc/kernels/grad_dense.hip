// Fused single-pass worker gradient for dense design matrices (K1+K2+K3+K13 of SURVEY §2.8).
//
// Reference semantics (one logical worker, one message):
//   predy = X_current.dot(beta)                                  ref src/naive.py:137
//   g = -X_current.T.dot( y_mod / (exp(y * predy) + 1) )         ref src/naive.py:138-139,
//                                                                 src/coded.py:183-185 (y_mod = B[w,p]*y)
//   g = -2 X_current.T.dot(y - predy)                             ref src/naive.py:345-346 (least squares)
//
// MI355X design: every row of X is read from HBM exactly once.  A wave owns whole
// rows: its 64 lanes load a row with 16-byte vector loads (1 KiB per wave
// instruction), form the dot product with beta held in registers, butterfly-reduce
// it across the wave, apply the loss epilogue (label encoding fused in as a
// per-segment coefficient) and immediately accumulate r * x_row into a per-lane
// register slice of g.  ROWS rows are loaded per wave iteration as raw 16-byte tiles (every
// load issues before the first conversion waits), so the reduction latency of one row
// overlaps the loads of the others; the rows-in-flight count is tuned per storage type.  At the end each workgroup
// folds its 4 waves through LDS and writes one fp64/fp32 slab row; a second tiny
// kernel sums the slab rows of each output message in a fixed order (bitwise
// reproducible, no float atomics).
//
// The "task" table lets one launch serve every logical worker hosted on this GPU
// (e.g. all 8 FRC/AGC workers at N=1): task -> (output message slot, segment,
// row range); segment -> (partition base pointer, labels, encoding coefficient).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <type_traits>

#include "common.h"
#include "grad_dense.h"
#include "launchers.h"
#include "lds_dma.h"

namespace eh {

template <typename T, typename A, int CPL, int LOSS, int ROWS, bool BL = false>
__global__ void __launch_bounds__(256)
grad_dense_fused(const Segment* __restrict__ segs, const Task* __restrict__ tasks,
                 const A* __restrict__ beta, A* __restrict__ slab, int ld, const int* __restrict__ gate) {
  constexpr int VN = Vec16<T>::N;
  constexpr int NV = CPL / VN;  // vector loads per row per lane
  static_assert(CPL % VN == 0, "CPL must be a multiple of the vector width");
  if (gate_closed(gate)) return;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  A* red = reinterpret_cast<A*>(smem_raw);

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;

  const Task task = tasks[blockIdx.x];
  const Segment seg = segs[task.seg];
  const T* __restrict__ X = static_cast<const T*>(seg.X);
  const A* __restrict__ Y = static_cast<const A*>(seg.y);
  const A coef = static_cast<A>(seg.coef);

  // Column ownership: vector j of lane l covers columns [(j*64+l)*VN, +VN).
  // BL: beta lives in LDS (after the fold area) and is re-read every row instead of pinning
  // NV*VN registers, so more rows fit in flight at the same occupancy.
  A* bl = red + 4 * kWave * CPL;
  bool valid[NV];
  A b[BL ? 1 : NV][VN];
  A g[NV][VN];
  if constexpr (BL) {
    for (int c = threadIdx.x; c < kWave * CPL; c += blockDim.x) bl[c] = c < ld ? beta[c] : A(0);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * kWave + lane) * VN;
    valid[j] = c0 < ld;
#pragma unroll
    for (int v = 0; v < VN; ++v) {
      if constexpr (!BL) b[j][v] = valid[j] ? beta[c0 + v] : A(0);
      g[j][v] = A(0);
    }
  }
  auto bval = [&](int j, int v) -> A {
    if constexpr (BL) return bl[(j * kWave + lane) * VN + v];
    else return b[j][v];
  };

  int r = task.row_begin + wid;
  // Main loop: ROWS rows per wave per iteration, all loads issued before the first reduction
  // (ROWS * NV 16-byte loads in flight per lane).  A software-pipelined variant (the next
  // row in flight while this one is reduced) measured no faster: docs/PERF_NOTES.md.
  for (; r + (ROWS - 1) * nw < task.row_end; r += ROWS * nw) {
    if constexpr (BL) asm volatile("" ::: "memory");  // keep the beta reads inside the loop
    // raw 16-byte tiles: every load of the iteration issues before any conversion waits on one
    // (buffer loads: vmcnt only, zeros past the row end; see common.h make_rsrc)
    typename Vec16<T>::raw xr[ROWS][NV];
    __amdgpu_buffer_rsrc_t rsq[ROWS];
#pragma unroll
    for (int q = 0; q < ROWS; ++q)
      rsq[q] = make_rsrc(X + static_cast<long long>(r + q * nw) * ld, ld * static_cast<int>(sizeof(T)));
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int q = 0; q < ROWS; ++q) {
        const int c0 = (j * kWave + lane) * VN;
        xr[q][j] = buf_load16<typename Vec16<T>::raw>(rsq[q], c0 * static_cast<int>(sizeof(T)));
      }
    A z[ROWS];
#pragma unroll
    for (int q = 0; q < ROWS; ++q) z[q] = A(0);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v)
#pragma unroll
        for (int q = 0; q < ROWS; ++q) z[q] = fma(Vec16<T>::template elem<A>(xr[q][j], v), bval(j, v), z[q]);
#pragma unroll
    for (int q = 0; q < ROWS; ++q) z[q] = wave_allreduce_sum(z[q]);
    A rq[ROWS];
#pragma unroll
    for (int q = 0; q < ROWS; ++q) rq[q] = residual<LOSS, A>(z[q], Y[r + q * nw], coef);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v)
#pragma unroll
        for (int q = 0; q < ROWS; ++q) g[j][v] = fma(rq[q], Vec16<T>::template elem<A>(xr[q][j], v), g[j][v]);
  }
  // Tail: fewer than ROWS rows left for this wave, one at a time.
  for (; r < task.row_end; r += nw) {
    const T* x0 = X + static_cast<long long>(r) * ld;
    A a0[NV][VN];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c0 = (j * kWave + lane) * VN;
      if (valid[j]) {
        Vec16<T>::template load<A, true>(x0 + c0, a0[j]);
      } else {
#pragma unroll
        for (int v = 0; v < VN; ++v) a0[j][v] = A(0);
      }
    }
    A z0 = A(0);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v) z0 = fma(a0[j][v], bval(j, v), z0);
    z0 = wave_allreduce_sum(z0);
    const A r0 = residual<LOSS, A>(z0, Y[r], coef);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v) g[j][v] = fma(r0, a0[j][v], g[j][v]);
  }

  // Fold the waves of this workgroup through LDS, then one slab row per workgroup.
  const int span = kWave * CPL;  // padded columns covered by a wave
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * kWave + lane) * VN;
#pragma unroll
    for (int v = 0; v < VN; ++v) red[wid * span + c0 + v] = g[j][v];
  }
  __syncthreads();
  A* out = slab + static_cast<long long>(task.slab) * ld;
  for (int c = threadIdx.x; c < ld; c += blockDim.x) {
    A s = A(0);
    for (int w = 0; w < nw; ++w) s += red[w * span + c];
    out[c] = s;
  }
}

// ----- Replica bundles in ONE wave: each row is loaded once, into registers, and every replica
// computes its own message from there. -----
// Same bundle table as grad_dense_bundle (R task slots reading the same rows); one wave per bundle.
// The wave double-buffers whole rows in VGPRs (the next row's loads are in flight while the current
// one is computed), so there is no LDS staging and no barrier.  Per row and per replica: its own
// dot product against beta (every replica's chain starts from an opaque zero, so the compiler
// cannot merge the R identical chains: each logical worker does its own arithmetic, as on its own
// machine in the reference), its own residual with its own coefficient and its own gradient
// accumulation; R slab rows are written at the end.
//
// FOLD: the plan lays the bundle table out in workgroups of 4 bundles of one partition (so the same
// replica slot q is the same message in all four; pad bundles fill a workgroup at a partition's
// end).  The four waves fold their accumulators through LDS in a fixed order and wave 0 writes
// one slab row per replica for the workgroup: a quarter of the slab rows for the reduction to read.
// EPI 1: the reduce-scatter + one-lane-per-replica epilogue below; EPI 0: every replica's
// dot product is all-reduced and its residual evaluated wave-uniformly (an inactive replica then
// skips its share).  Measured: the lane form wins on the sharded multi-GPU rank shapes, the wave
// form on the one-GPU headline (ops/grad.py picks per plan; docs/PERF_NOTES.md round 3).
// EPI 2 (pair rows, cpl <= 8): two rows per reduction -- the 2R dot products of a row pair are
// reduce-scattered in one 8-value exchange (wave_reduce_scatter8), lane 8v evaluates value v's
// residual, and both rows' gradients accumulate from four row buffers (the next pair in flight).
// Narrow rows spend most of their time in the per-row cross-lane reductions (d = 256:
// profiles/round3/choices), which this halves.
// stamps (a timeline probe, tools/probes/bundle_stamps.py; nullptr in every production launch): per
// bundle {start, rows done, slab written, XCC id} in wall_clock64 ticks, one vector store of lane 0 each.
// Rows in flight per wave of grad_dense_multi: 2 for fp64 rows (8 KB at d = 1000; 3 measured 1184.5 vs
// 1181 us at the N = 1 rank shape, 278 VGPRs), 3 for fp32 (4 KB rows: 570-573 vs 588-590 us at N = 1, 81-83
// vs 84 at N = 8, profiles/round6/fp32_depth; 4 was slower, round 5), 6 for bf16 (2 KB rows: 12 KB in flight
// per wave; 3 waves per SIMD at R = 3, 169 VGPRs and 2 waves with 8).
template <typename T>
constexpr int kMultiDepth = std::is_same<T, bf16_t>::value ? 6 : std::is_same<T, float>::value ? 3 : 2;

template <typename T, typename A, int CPL, int LOSS, int R, bool FOLD, int EPI = 0>
__global__ void __launch_bounds__(256)
grad_dense_multi(const Segment* __restrict__ segs, const Task* __restrict__ tasks, int nbundles,
                 const A* __restrict__ beta, A* __restrict__ slab, int ld, const int* __restrict__ gate,
                 long long* __restrict__ stamps) {
  constexpr int VN = Vec16<T>::N;
  constexpr int NV = CPL / VN;
  using Rw = typename Vec16<T>::raw;
  if (gate_closed(gate)) return;  // launch-uniform: the FOLD barrier is never half-reached
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bundle = __builtin_amdgcn_readfirstlane(blockIdx.x * (blockDim.x >> 6) + wv);
  if (!FOLD && bundle >= nbundles) return;  // FOLD: every wave reaches the barrier (nbundles % 4 == 0)
  if (stamps && lane == 0) {
    stamps[4 * bundle] = wall_clock64();
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    stamps[4 * bundle + 3] = xcc;
  }
  const Task lead = tasks[bundle * R];
  const bool live = lead.seg >= 0;  // FOLD pad bundles: no rows, zero accumulators
  const Segment ls = segs[live ? lead.seg : 0];
  const T* __restrict__ X = static_cast<const T*>(ls.X);
  const A* __restrict__ Y = static_cast<const A*>(ls.y);
  A coef[R];
  bool act[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const Task tq = tasks[bundle * R + q];
    act[q] = tq.seg >= 0;
    coef[q] = act[q] ? static_cast<A>(segs[tq.seg].coef) : A(0);
  }
  A b[NV][VN], g[R][NV][VN];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * kWave + lane) * VN;
#pragma unroll
    for (int v = 0; v < VN; ++v) {
      b[j][v] = c0 < ld ? beta[c0 + v] : A(0);
#pragma unroll
      for (int q = 0; q < R; ++q) g[q][j][v] = A(0);
    }
  }
  const int rowbytes = ld * static_cast<int>(sizeof(T));
  const int r0 = lead.row_begin, r1 = live ? lead.row_end : r0;
  // A row's label is loaded right behind the row itself, through a buffer descriptor: it is then
  // older than the next row's prefetch, so a step waits for its own row and label only
  // (vmcnt(loads of one row)) and the prefetched row stays in flight.  (Read at use through the
  // segment pointer, it was a flat load issued AFTER the prefetch: every step waited vmcnt(0),
  // which drained the prefetch -- one row in flight per wave, not two.)
  const auto yrs = make_rsrc(Y + r0, (r1 - r0) * static_cast<int>(sizeof(A)));
  // Loads are issued unconditionally (the compiler can then count them: a step waits with
  // vmcnt(one row's loads), not a conservative merge of "prefetched / not prefetched"); a row past
  // the bundle gets a zero-size descriptor, which returns zeros without touching memory.
  auto load = [&](Rw (&x)[NV], A& yv, int r) {
    const bool in = r < r1;
    const auto rs = make_rsrc(X + static_cast<long long>(in ? r : r0) * ld, in ? rowbytes : 0);
#pragma unroll
    for (int j = 0; j < NV; ++j) x[j] = buf_load16<Rw>(rs, (j * kWave + lane) * VN * static_cast<int>(sizeof(T)));
    yv = buf_load_scalar<A>(yrs, (r - r0) * static_cast<int>(sizeof(A)));
  };
  auto step = [&](const Rw (&x)[NV], const A y) {
    A z[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      z[q] = A(0);
      asm volatile("" : "+v"(z[q]));  // opaque start: R separate dot products, not one shared
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v)
#pragma unroll
        for (int q = 0; q < R; ++q) z[q] = fma(Vec16<T>::template elem<A>(x[j], v), b[j][v], z[q]);
    A rr[R];
    if constexpr (R == 1 || EPI == 0) {
#pragma unroll
      for (int q = 0; q < R; ++q) rr[q] = act[q] ? residual<LOSS, A>(wave_allreduce_sum(z[q]), y, coef[q]) : A(0);
    } else {
      // Replicas 0 and 1 share one reduce-scatter (lanes 0-31 end with replica 0's dot product,
      // lanes 32-63 with replica 1's), replica 2 is all-reduced.  Then one lane per replica
      // evaluates that replica's loss epilogue (lane 0, lane 32, lane 1: one exp / divide for all
      // of them instead of one wave-uniform evaluation each) and every lane reads the R residuals.
      static_assert(R <= 3, "one-wave bundles hold at most 3 replicas");
      const bool hi = lane >= 32;
      // opaque copies: a select between two elements of coef[] would otherwise become one
      // lane-indexed load of the array, i.e. coef[] in scratch memory (seen in the fp32 kernel)
      A c0 = coef[0], c1 = coef[1];
      asm volatile("" : "+v"(c0), "+v"(c1));
      A tq = wave_pair_reduce(z[0], z[1], hi), cq = hi ? c1 : c0;
      constexpr int kLane[3] = {0, 32, 1};
      if constexpr (R == 3) {
        const A z2 = wave_allreduce_sum(z[2]);
        if (lane == 1) {
          tq = z2;
          cq = coef[2];
        }
      }
      const A rl = residual_branchfree<LOSS, A>(tq, y, cq);
#pragma unroll
      for (int q = 0; q < R; ++q) rr[q] = act[q] ? readlane_a(rl, kLane[q]) : A(0);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v)
#pragma unroll
        for (int q = 0; q < R; ++q) g[q][j][v] = fma(rr[q], Vec16<T>::template elem<A>(x[j], v), g[q][j][v]);
  };
  // two rows at once (EPI 2): 2R dot products, one reduce-scatter, one residual per lane
  auto step2 = [&](const Rw (&x0)[NV], const Rw (&x1)[NV], const A y0, const A y1, bool two) {
    static_assert(2 * R <= 8, "pair rows hold at most 4 replicas");
    A v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      v[q] = A(0);
      if (q < 2 * R) asm volatile("" : "+v"(v[q]));  // opaque start: separate dot products
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < VN; ++e)
#pragma unroll
        for (int q = 0; q < R; ++q) {
          v[q] = fma(Vec16<T>::template elem<A>(x0[j], e), b[j][e], v[q]);
          v[R + q] = fma(Vec16<T>::template elem<A>(x1[j], e), b[j][e], v[R + q]);
        }
    const A tot = wave_reduce_scatter8(v, lane);  // lanes 8m..8m+7: value m = k R + q
    const int m = lane >> 3, k = m >= R ? 1 : 0, qm = m - k * R;
    A cq = A(0);
#pragma unroll
    for (int q = 0; q < R; ++q)
      if (qm == q) cq = coef[q];
    const A rl = m < 2 * R ? residual_branchfree<LOSS, A>(tot, k ? y1 : y0, cq) : A(0);
    A r0v[R], r1v[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      r0v[q] = act[q] ? readlane_a(rl, 8 * q) : A(0);
      r1v[q] = act[q] && two ? readlane_a(rl, 8 * (R + q)) : A(0);
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int e = 0; e < VN; ++e)
#pragma unroll
        for (int q = 0; q < R; ++q)
          g[q][j][e] = fma(r1v[q], Vec16<T>::template elem<A>(x1[j], e),
                           fma(r0v[q], Vec16<T>::template elem<A>(x0[j], e), g[q][j][e]));
  };
  if constexpr (EPI == 2) {
    Rw xa[NV], xb[NV], xc[NV], xd[NV];
    A ya = A(0), yb = A(0), yc = A(0), yd = A(0);
#pragma unroll
    for (int j = 0; j < NV; ++j) xa[j] = xb[j] = xc[j] = xd[j] = Rw{};  // a missing pair row reads zeros
    load(xa, ya, r0);
    load(xb, yb, r0 + 1);
    for (int r = r0; r < r1; r += 4) {  // four rows per trip: the buffer pairs swap roles
      load(xc, yc, r + 2);
      load(xd, yd, r + 3);
      step2(xa, xb, ya, yb, r + 1 < r1);
      if (r + 2 >= r1) break;
      load(xa, ya, r + 4);
      load(xb, yb, r + 5);
      step2(xc, xd, yc, yd, r + 3 < r1);
    }
  } else if constexpr (kMultiDepth<T> > 2) {
    // Short rows (bf16: 2 KB at d = 1000, two 16-byte vectors per lane): two rows in flight would be 4 KB
    // per wave, too little to cover HBM latency at a CU's share of the stream, so D rows are in flight: a
    // ring of D row buffers, each step issuing the load D - 1 rows ahead before consuming its own row.
    constexpr int D = kMultiDepth<T>;
    Rw xr[D][NV];
    A yr[D];
#pragma unroll
    for (int k = 0; k < D - 1; ++k) load(xr[k], yr[k], r0 + k);
    for (int r = r0; r < r1; r += D) {
#pragma unroll
      for (int k = 0; k < D; ++k) {
        load(xr[(k + D - 1) % D], yr[(k + D - 1) % D], r + k + D - 1);
        step(xr[k], yr[k]);
        if (r + k + 1 >= r1) break;
      }
    }
  } else {
    Rw xa[NV], xb[NV];
    A ya = A(0), yb = A(0);
    load(xa, ya, r0);
    for (int r = r0; r < r1; r += 2) {  // two rows per trip: the buffers swap roles without copies
      load(xb, yb, r + 1);
      step(xa, ya);
      if (r + 1 >= r1) break;
      load(xa, ya, r + 2);
      step(xb, yb);
    }
  }
  if (stamps && lane == 0) stamps[4 * bundle + 1] = wall_clock64();
  if constexpr (FOLD) {
    extern __shared__ __attribute__((aligned(16))) unsigned char fold_raw[];
    A* fb = reinterpret_cast<A*>(fold_raw);  // [3 waves][R][NV * VN][64 lanes]
    if (wv > 0) {
#pragma unroll
      for (int q = 0; q < R; ++q)
#pragma unroll
        for (int j = 0; j < NV; ++j)
#pragma unroll
          for (int v = 0; v < VN; ++v) fb[((((wv - 1) * R + q) * NV + j) * VN + v) * kWave + lane] = g[q][j][v];
    }
    __syncthreads();
    if (wv > 0) return;
#pragma unroll 1
    for (int k = 0; k < 3; ++k)  // one wave's rows at a time: keeps the epilogue's registers low
#pragma unroll
      for (int q = 0; q < R; ++q)
#pragma unroll
        for (int j = 0; j < NV; ++j)
#pragma unroll
          for (int v = 0; v < VN; ++v) g[q][j][v] += fb[(((k * R + q) * NV + j) * VN + v) * kWave + lane];
  }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    if (!act[q]) continue;
    A* out = slab + static_cast<long long>(tasks[bundle * R + q].slab) * ld;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c0 = (j * kWave + lane) * VN;
#pragma unroll
      for (int v = 0; v < VN; ++v)
        if (c0 + v < ld) out[c0 + v] = g[q][j][v];
    }
  }
  if (stamps) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) stamps[4 * bundle + 2] = wall_clock64();
  }
}

// ----- Replica bundles staged through LDS: one HBM read per row, one wave per replica. -----
// Same task table as grad_dense_bundle (R slots per workgroup, all reading the same rows of one
// partition).  The workgroup streams its row range through an NS-stage LDS ring with
// global_load_lds (16-byte LDS-DMA, no staging registers): NS-1 stages are in flight while every
// replica wave computes the oldest one from LDS — its own dot product against beta, residual with
// its own coefficient, and gradient accumulation — and writes its own slab row.  The rows of a
// stage are contiguous in HBM, so a stage is one flat copy split into 1 KiB wave pieces (lane-
// linear LDS image).  Labels ride along as one 4-byte-per-lane LDS-DMA piece.
// (A persistent-grid variant with an atomic bundle ticket and a stage-walk rotation were measured
// slower and removed in round 3: docs/PERF_NOTES.md.)
template <typename T, typename A, int CPL, int LOSS, bool PAIR>
__global__ void __launch_bounds__(512)
grad_dense_staged(const Segment* __restrict__ segs, const Task* __restrict__ tasks,
                  const A* __restrict__ beta, A* __restrict__ slab, int ld, int srows, int pieces, int nstage,
                  int wpr, const int* __restrict__ gate) {
  constexpr int VN = Vec16<T>::N;
  constexpr int NV = CPL / VN;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  if (gate_closed(gate)) return;
  // W waves = R task slots x wpr waves per slot; slot q's waves split each stage's rows
  const int lane = threadIdx.x & 63, W = blockDim.x >> 6, R = W / wpr;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q = w % R, sub = w / R;
  const unsigned lds_base = static_cast<unsigned>(
      reinterpret_cast<size_t>((__attribute__((address_space(3))) unsigned char*)smem_raw));
  const int rowbytes = ld * static_cast<int>(sizeof(T));
  const int data_bytes = W * pieces * 1024;  // one stage buffer: data, then 256 B of labels
  const int buf_bytes = data_bytes + 256;
  using Rw = typename Vec16<T>::raw;
  A b[NV][VN];  // beta
  bool valid[NV];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * kWave + lane) * VN;
    valid[j] = c0 < ld;
#pragma unroll
    for (int v = 0; v < VN; ++v) b[j][v] = valid[j] ? beta[c0 + v] : A(0);
  }
  {  // one bundle per workgroup
    const int bundle = blockIdx.x;
    const Task lead = tasks[bundle * R];  // slot 0 of a bundle is always a real task
    const Task task = tasks[bundle * R + q];
    const bool active = task.seg >= 0;
    const Segment ls = segs[lead.seg];
    const unsigned char* __restrict__ X = static_cast<const unsigned char*>(ls.X);
    const unsigned char* __restrict__ Y = static_cast<const unsigned char*>(ls.y);
    const A coef = active ? static_cast<A>(segs[task.seg].coef) : A(0);
    const int nrows = lead.row_end - lead.row_begin;
    const int nst = (nrows + srows - 1) / srows;
    auto stage_of = [](int t) { return t; };
    const int p_last = nst - 1;  // loop position of the (possibly partial) last stage

    // LDS-DMA loads wave w issues for a stage of nbytes: its 1 KiB pieces (+ labels: wave 0).  Every
    // stage but the last is full, so two counts cover the ring; computing them once keeps integer
    // divisions (and the loop the vectorizer made of a per-stage sum) out of the stage loop.
    auto count_bytes = [&](int nbytes) {
      const int nb = (nbytes + 1023) >> 10;
      return (nb > w ? (nb - w + W - 1) / W : 0) + (w == 0 ? 1 : 0);
    };
    const int cnt_full = count_bytes(srows * rowbytes);
    const int cnt_last = count_bytes((nrows - (nst - 1) * srows) * rowbytes);
    auto issue = [&](int t) {
      const unsigned dst = lds_base + (t % nstage) * buf_bytes;
      const long long r0 = lead.row_begin + static_cast<long long>(stage_of(t)) * srows;
      const int ns = min(srows, static_cast<int>(lead.row_end - r0));
      const int bytes = ns * rowbytes;
      const unsigned char* src = X + r0 * rowbytes;
      for (int blk = w; blk * 1024 < bytes; blk += W)
        glds16(src + min(blk * 1024 + lane * 16, bytes - 16), dst + blk * 1024);
      if (w == 0) {
        const int lb = ns * static_cast<int>(sizeof(A));
        glds4(Y + r0 * sizeof(A) + min(lane * 4, lb - 4), dst + data_bytes);
      }
    };

    A g[NV][VN];
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v) g[j][v] = A(0);
    // beta retired before the counted loads
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int t = 0; t < nstage - 1 && t < nst; ++t) issue(t);
    for (int t = 0; t < nst; ++t) {
      // loads this wave issued after stage t: loop positions t+1 .. hi; only the stage at p_last can be partial
      const int hi = min(t + nstage - 2, nst - 1);
      const int later = hi > t ? (hi - t) * cnt_full + (p_last > t && p_last <= hi ? cnt_last - cnt_full : 0) : 0;
      wait_vmcnt(later);  // this wave's pieces of stage t landed
      __syncthreads();    // every wave's pieces of stage t; stage t-1 consumed by every wave
      if (t + nstage - 1 < nst) issue(t + nstage - 1);  // into the buffer stage t-1 used
      if (!active) continue;
      const unsigned char* buf = smem_raw + (t % nstage) * buf_bytes;
      const A* lab = reinterpret_cast<const A*>(buf + data_bytes);
      const int ns = min(srows, nrows - stage_of(t) * srows);
      if constexpr (PAIR) {
        // Two rows per step with ONE reduction and ONE residual evaluation between them: the two
        // partial dot products are reduce-scattered (lanes 0-31 finish row i, lanes 32-63 row i+1),
        // each lane evaluates the loss epilogue of its half's row (one exp for two rows), and the
        // two residuals are broadcast by readlane.  The rows are re-read from LDS for the update
        // rather than held in registers across the reduction.  A lone last row is paired with
        // itself and weighted 0.
        const bool hi = lane >= 32;
        for (int i = 2 * sub; i < ns; i += 2 * wpr) {
          const bool two = i + 1 < ns;
          const unsigned char* row0 = buf + i * rowbytes;
          const unsigned char* row1 = two ? row0 + rowbytes : row0;
          A z0 = A(0), z1 = A(0);
          if constexpr (std::is_same<T, float>::value) {
            // fp32: both rows' dot products in one packed accumulator {z0, z1} (v_pk_fma_f32)
            typedef float f2 __attribute__((ext_vector_type(2)));
            f2 z01 = f2{0.f, 0.f};
#pragma unroll
            for (int j = 0; j < NV; ++j) {
              const int c0 = min((j * kWave + lane) * VN, ld - VN) * static_cast<int>(sizeof(T));
              const Rw v0 = *reinterpret_cast<const Rw*>(row0 + c0);
              const Rw v1 = *reinterpret_cast<const Rw*>(row1 + c0);
              z01 = __builtin_elementwise_fma(f2{v0.x, v1.x}, f2{b[j][0], b[j][0]}, z01);
              z01 = __builtin_elementwise_fma(f2{v0.y, v1.y}, f2{b[j][1], b[j][1]}, z01);
              z01 = __builtin_elementwise_fma(f2{v0.z, v1.z}, f2{b[j][2], b[j][2]}, z01);
              z01 = __builtin_elementwise_fma(f2{v0.w, v1.w}, f2{b[j][3], b[j][3]}, z01);
            }
            z0 = z01.x;
            z1 = z01.y;
          } else {
#pragma unroll
            for (int j = 0; j < NV; ++j) {
              const int c0 = min((j * kWave + lane) * VN, ld - VN) * static_cast<int>(sizeof(T));
              const Rw v0 = *reinterpret_cast<const Rw*>(row0 + c0);
              const Rw v1 = *reinterpret_cast<const Rw*>(row1 + c0);
#pragma unroll
              for (int v = 0; v < VN; ++v) {
                z0 = fma(Vec16<T>::template elem<A>(v0, v), b[j][v], z0);  // beta is 0 past the row end
                z1 = fma(Vec16<T>::template elem<A>(v1, v), b[j][v], z1);
              }
            }
          }
          const A zs = wave_pair_reduce(z0, z1, hi);
          const A rr = residual_branchfree<LOSS, A>(zs, lab[two && hi ? i + 1 : i], coef);
          const A r0 = readlane_a(rr, 0);
          const A r1 = two ? readlane_a(rr, 32) : A(0);
          asm volatile("" ::: "memory");  // re-read the rows from LDS below
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            const int c0 = min((j * kWave + lane) * VN, ld - VN) * static_cast<int>(sizeof(T));
            const Rw v0 = *reinterpret_cast<const Rw*>(row0 + c0);
            const Rw v1 = *reinterpret_cast<const Rw*>(row1 + c0);
            if constexpr (std::is_same<T, float>::value) {
              typedef float f2 __attribute__((ext_vector_type(2)));
              const f2 rr0 = f2{r0, r0}, rr1 = f2{r1, r1};
              f2 lo = __builtin_elementwise_fma(rr0, f2{v0.x, v0.y}, f2{g[j][0], g[j][1]});
              f2 hi2 = __builtin_elementwise_fma(rr0, f2{v0.z, v0.w}, f2{g[j][2], g[j][3]});
              lo = __builtin_elementwise_fma(rr1, f2{v1.x, v1.y}, lo);
              hi2 = __builtin_elementwise_fma(rr1, f2{v1.z, v1.w}, hi2);
              g[j][0] = lo.x;
              g[j][1] = lo.y;
              g[j][2] = hi2.x;
              g[j][3] = hi2.y;
            } else {
#pragma unroll
              for (int v = 0; v < VN; ++v) {
                const A e0 = Vec16<T>::template elem<A>(v0, v);  // columns past the row end: never written
                const A e1 = Vec16<T>::template elem<A>(v1, v);
                g[j][v] = fma(r1, e1, fma(r0, e0, g[j][v]));
              }
            }
          }
        }
      } else if constexpr (std::is_same<T, float>::value) {
        // fp32: the same row-at-a-time math on packed v_pk_fma_f32 (two columns per instruction).
        // fp32 rows carry twice the elements per byte of fp64, so the VALU issue rate, not HBM, bound
        // the scalar form (0.83 ms vs 0.73 ms of bytes at the headline); z keeps two partial sums.
        typedef float f2 __attribute__((ext_vector_type(2)));
        for (int i = sub; i < ns; i += wpr) {
          const unsigned char* row = buf + i * rowbytes;
          Rw xr[NV];
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            const int c0 = min((j * kWave + lane) * VN, ld - VN) * static_cast<int>(sizeof(T));
            xr[j] = *reinterpret_cast<const Rw*>(row + c0);  // clamped read: see the scalar path below
          }
          f2 z2 = f2{0.f, 0.f};
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            z2 = __builtin_elementwise_fma(f2{xr[j].x, xr[j].y}, f2{b[j][0], b[j][1]}, z2);
            z2 = __builtin_elementwise_fma(f2{xr[j].z, xr[j].w}, f2{b[j][2], b[j][3]}, z2);
          }
          const A rr = residual<LOSS, A>(wave_allreduce_sum(z2.x + z2.y), lab[i], coef);
          const f2 r2 = f2{rr, rr};
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            const f2 lo = __builtin_elementwise_fma(r2, f2{xr[j].x, xr[j].y}, f2{g[j][0], g[j][1]});
            const f2 hi = __builtin_elementwise_fma(r2, f2{xr[j].z, xr[j].w}, f2{g[j][2], g[j][3]});
            g[j][0] = lo.x;
            g[j][1] = lo.y;
            g[j][2] = hi.x;
            g[j][3] = hi.y;
          }
        }
      } else {
        // one row at a time
        for (int i = sub; i < ns; i += wpr) {
          const unsigned char* row = buf + i * rowbytes;
          Rw xr[NV];
#pragma unroll
          for (int j = 0; j < NV; ++j) {
            // Clamped read: past the row end a lane re-reads the row's last vector.  It is not
            // masked: beta is 0 there, so its dot-product terms add exactly 0 (finite data), and the
            // gradient columns it pollutes are never written.  A per-vector select compiled to exec
            // branches and 64-bit moves that cost as much as the row's FMAs.
            const int c0 = min((j * kWave + lane) * VN, ld - VN) * static_cast<int>(sizeof(T));
            xr[j] = *reinterpret_cast<const Rw*>(row + c0);
          }
          A z = A(0);  // one accumulator: four independent chains measured no faster
#pragma unroll
          for (int j = 0; j < NV; ++j)
#pragma unroll
            for (int v = 0; v < VN; ++v) z = fma(Vec16<T>::template elem<A>(xr[j], v), b[j][v], z);
          const A rr = residual<LOSS, A>(wave_allreduce_sum(z), lab[i], coef);
#pragma unroll
          for (int j = 0; j < NV; ++j)
#pragma unroll
            for (int v = 0; v < VN; ++v) g[j][v] = fma(rr, Vec16<T>::template elem<A>(xr[j], v), g[j][v]);
        }
      }
    }
    if (wpr > 1) {  // fold the slot's waves through LDS (the ring is free after this barrier)
      A* fold = reinterpret_cast<A*>(smem_raw);
      __syncthreads();
      if (active && sub > 0) {
#pragma unroll
        for (int j = 0; j < NV; ++j)
#pragma unroll
          for (int v = 0; v < VN; ++v) fold[(((sub - 1) * R + q) * NV * VN + j * VN + v) * kWave + lane] = g[j][v];
      }
      __syncthreads();
      if (active && sub == 0) {
        for (int k = 0; k < wpr - 1; ++k)
#pragma unroll
          for (int j = 0; j < NV; ++j)
#pragma unroll
            for (int v = 0; v < VN; ++v) g[j][v] += fold[((k * R + q) * NV * VN + j * VN + v) * kWave + lane];
      }
    }
    if (active && sub == 0) {
      A* out = slab + static_cast<long long>(task.slab) * ld;
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int c0 = (j * kWave + lane) * VN;
#pragma unroll
        for (int v = 0; v < VN; ++v)
          if (c0 + v < ld) out[c0 + v] = g[j][v];
      }
    }
  }
}

// Stage geometry of grad_dense_staged: rows per stage, 1 KiB pieces per wave and ring depth, measured
// at the headline (docs/PERF_NOTES.md): a 2-stage ring, about 4 waves per workgroup and 2 rows per
// wave per stage (R = 3: 1 wave per replica, 2 rows; R = 2: 2 waves per replica, 4 rows).  Rows
// shrink until the ring fits kStagedLds.
constexpr int kStagedLds = 160 * 1024 - 256;  // 160 KiB per workgroup
struct StagedGeom {
  int srows, pieces, nstage, wpr;
  size_t lds;
};
// R task slots; fold_bytes_per_wave: one wave's gradient slice (64 * CPL accumulators);
// want_wpr > 0: waves per replica chosen by the plan (KernelChoice::wpr), else the default above
static inline bool staged_geometry(int R, int rowbytes, size_t fold_bytes_per_wave, StagedGeom* g, int want_wpr = 0) {
  const int ns = 2;
  const int wpr = want_wpr >= 1 && want_wpr <= 4 && R * want_wpr <= 8 ? want_wpr : std::max(1, 4 / R);
  const int W = R * wpr;
  const size_t fold = static_cast<size_t>(wpr - 1) * R * fold_bytes_per_wave;
  int s = 2 * wpr;
  for (; s >= 1; --s) {
    const int p = (s * rowbytes + W * 1024 - 1) / (W * 1024);
    const size_t bytes = std::max(fold, static_cast<size_t>(ns) * (static_cast<size_t>(W) * p * 1024 + 256));
    if (bytes <= kStagedLds) {
      *g = StagedGeom{s, p, ns, wpr, bytes};
      return true;
    }
  }
  return false;
}

// Two rows per wave per iteration, loads of both rows interleaved per vector (the layout
// that measured fastest for bf16 and fp32).
template <typename T, typename A, int CPL, int LOSS>
__global__ void __launch_bounds__(256)
grad_dense_fused_pair(const Segment* __restrict__ segs, const Task* __restrict__ tasks,
                 const A* __restrict__ beta, A* __restrict__ slab, int ld, const int* __restrict__ gate) {
  constexpr int VN = Vec16<T>::N;
  constexpr int NV = CPL / VN;  // vector loads per row per lane
  static_assert(CPL % VN == 0, "CPL must be a multiple of the vector width");
  if (gate_closed(gate)) return;

  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  A* red = reinterpret_cast<A*>(smem_raw);

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;

  const Task task = tasks[blockIdx.x];
  const Segment seg = segs[task.seg];
  const T* __restrict__ X = static_cast<const T*>(seg.X);
  const A* __restrict__ Y = static_cast<const A*>(seg.y);
  const A coef = static_cast<A>(seg.coef);

  // Column ownership: vector j of lane l covers columns [(j*64+l)*VN, +VN).
  bool valid[NV];
  A b[NV][VN];
  A g[NV][VN];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * kWave + lane) * VN;
    valid[j] = c0 < ld;
#pragma unroll
    for (int v = 0; v < VN; ++v) {
      b[j][v] = valid[j] ? beta[c0 + v] : A(0);
      g[j][v] = A(0);
    }
  }

  int r = task.row_begin + wid;
  // Main loop: two rows per wave per iteration.
  for (; r + nw < task.row_end; r += 2 * nw) {
    const T* x0 = X + static_cast<long long>(r) * ld;
    const T* x1 = X + static_cast<long long>(r + nw) * ld;
    A a0[NV][VN], a1[NV][VN];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c0 = (j * kWave + lane) * VN;
      if (valid[j]) {
        Vec16<T>::template load<A, true>(x0 + c0, a0[j]);
        Vec16<T>::template load<A, true>(x1 + c0, a1[j]);
      } else {
#pragma unroll
        for (int v = 0; v < VN; ++v) { a0[j][v] = A(0); a1[j][v] = A(0); }
      }
    }
    A z0 = A(0), z1 = A(0);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v) {
        z0 = fma(a0[j][v], b[j][v], z0);
        z1 = fma(a1[j][v], b[j][v], z1);
      }
    z0 = wave_allreduce_sum(z0);
    z1 = wave_allreduce_sum(z1);
    const A r0 = residual<LOSS, A>(z0, Y[r], coef);
    const A r1 = residual<LOSS, A>(z1, Y[r + nw], coef);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v) g[j][v] = fma(r1, a1[j][v], fma(r0, a0[j][v], g[j][v]));
  }
  // Tail: at most one row left for this wave.
  if (r < task.row_end) {
    const T* x0 = X + static_cast<long long>(r) * ld;
    A a0[NV][VN];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c0 = (j * kWave + lane) * VN;
      if (valid[j]) {
        Vec16<T>::template load<A, true>(x0 + c0, a0[j]);
      } else {
#pragma unroll
        for (int v = 0; v < VN; ++v) a0[j][v] = A(0);
      }
    }
    A z0 = A(0);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v) z0 = fma(a0[j][v], b[j][v], z0);
    z0 = wave_allreduce_sum(z0);
    const A r0 = residual<LOSS, A>(z0, Y[r], coef);
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v) g[j][v] = fma(r0, a0[j][v], g[j][v]);
  }

  // Fold the waves of this workgroup through LDS, then one slab row per workgroup.
  const int span = kWave * CPL;  // padded columns covered by a wave
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * kWave + lane) * VN;
#pragma unroll
    for (int v = 0; v < VN; ++v) red[wid * span + c0 + v] = g[j][v];
  }
  __syncthreads();
  A* out = slab + static_cast<long long>(task.slab) * ld;
  for (int c = threadIdx.x; c < ld; c += blockDim.x) {
    A s = A(0);
    for (int w = 0; w < nw; ++w) s += red[w * span + c];
    out[c] = s;
  }
}

// ----- Wide rows (2048 < d <= 8192 fp64 / 16384 fp32,bf16): still ONE pass over X. -----
// A whole workgroup owns each row: thread t holds columns (j*BS + t)*VN + [0, VN) for the
// NV 16-byte vectors j, so every load instruction of the block is fully coalesced and each
// thread keeps its slice of beta and of the gradient in registers.  The row dot product is
// finished across the block through LDS once per PAIR of rows (double-buffered LDS slots,
// one barrier per pair); the loss residual is then applied from registers, so X is read
// from HBM exactly once.  Columns are disjoint per thread: the slab row is written
// directly, no LDS fold.
// R > 1: a replica bundle (R task slots per workgroup, all reading the same rows, ops/grad.py): each
// row is loaded once and every replica computes its own dot product, residual (own coefficient) and
// gradient from the registers, so the replicated messages cost one HBM stream (the interleaved
// dispatch re-read them through L2 at ~4 TB/s, profiles/round3/choices).
template <typename T, typename A, int NV, int BS, int LOSS, int R, bool PF = false>
__global__ void __launch_bounds__(BS)
grad_dense_wide(const Segment* __restrict__ segs, const Task* __restrict__ tasks,
                const A* __restrict__ beta, A* __restrict__ slab, int ld, const int* __restrict__ gate) {
  constexpr int VN = Vec16<T>::N;
  constexpr int NW = BS / kWave;
  __shared__ A part[2][2][R][NW];  // [buffer][row of the pair][replica][wave]
  if (gate_closed(gate)) return;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const Task lead = tasks[blockIdx.x * R];  // slot 0 of a bundle is always a real task
  const Segment seg = segs[lead.seg];
  const T* __restrict__ X = static_cast<const T*>(seg.X);
  const A* __restrict__ Y = static_cast<const A*>(seg.y);
  A coef[R];
  bool act[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const Task tq = tasks[blockIdx.x * R + q];
    act[q] = tq.seg >= 0;
    coef[q] = act[q] ? static_cast<A>(segs[tq.seg].coef) : A(0);
  }

  bool valid[NV];
  A b[NV][VN], g[R][NV][VN];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c0 = (j * BS + tid) * VN;
    valid[j] = c0 < ld;
#pragma unroll
    for (int v = 0; v < VN; ++v) {
      b[j][v] = valid[j] ? beta[c0 + v] : A(0);
#pragma unroll
      for (int q = 0; q < R; ++q) g[q][j][v] = A(0);
    }
  }
  int buf = 0;
  // one row pair: R dot products each, cross-wave sums through LDS (one barrier), residuals, gradients
  auto pair = [&](const A (&a0)[NV][VN], const A (&a1)[NV][VN], A y0, A y1, bool two) {
    A z0[R], z1[R];
#pragma unroll
    for (int q = 0; q < R; ++q) {
      z0[q] = A(0);
      z1[q] = A(0);
      asm volatile("" : "+v"(z0[q]), "+v"(z1[q]));  // opaque start: R separate dot products
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v)
#pragma unroll
        for (int q = 0; q < R; ++q) {
          z0[q] = fma(a0[j][v], b[j][v], z0[q]);
          z1[q] = fma(a1[j][v], b[j][v], z1[q]);
        }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      z0[q] = wave_allreduce_sum(z0[q]);
      z1[q] = wave_allreduce_sum(z1[q]);
      if (lane == 0) {
        part[buf][0][q][wid] = z0[q];
        part[buf][1][q][wid] = z1[q];
      }
    }
    __syncthreads();
    A r0[R], r1[R];
    if constexpr (R == 1) {
      A s0 = A(0), s1 = A(0);
#pragma unroll
      for (int w = 0; w < NW; ++w) {  // fixed order: every thread gets the bitwise-same sums
        s0 += part[buf][0][0][w];
        s1 += part[buf][1][0][w];
      }
      r0[0] = residual<LOSS, A>(s0, y0, coef[0]);
      r1[0] = two ? residual<LOSS, A>(s1, y1, coef[0]) : A(0);
    } else {
      // one loss epilogue per lane instead of 2R wave-uniform ones: lane (row k, replica q) = k R + q
      // sums its dot product (same fixed order) and evaluates its residual, then every lane reads
      // the 2R results
      const int k = lane >= R ? 1 : 0, q = lane - k * R;
      A sl = A(0);
      if (lane < 2 * R) {
#pragma unroll
        for (int w = 0; w < NW; ++w) sl += part[buf][k][q][w];
      }
      A cq = A(0);  // this lane's replica coefficient (coef[] stays in registers: no dynamic index)
#pragma unroll
      for (int qq = 0; qq < R; ++qq)
        if (q == qq) cq = coef[qq];
      const A rl = residual_branchfree<LOSS, A>(sl, k ? y1 : y0, cq);
#pragma unroll
      for (int qq = 0; qq < R; ++qq) {
        r0[qq] = act[qq] ? readlane_a(rl, qq) : A(0);
        r1[qq] = act[qq] && two ? readlane_a(rl, R + qq) : A(0);
      }
    }
    buf ^= 1;  // the next pair writes the other buffer: no second barrier needed
#pragma unroll
    for (int j = 0; j < NV; ++j)
#pragma unroll
      for (int v = 0; v < VN; ++v)
#pragma unroll
        for (int q = 0; q < R; ++q) g[q][j][v] = fma(r1[q], a1[j][v], fma(r0[q], a0[j][v], g[q][j][v]));
  };
  if constexpr (PF) {
    // The next pair's loads are issued before this pair's reductions and barrier: with one workgroup
    // per CU (the 512-thread replica rows) nothing else keeps the CU's loads in flight across the
    // barrier.  Buffer loads over the row (range-checked: columns past ld read zeros, no branches)
    // are unconditional -- past the bundle the last pair is read again -- so each step waits for its
    // own pair only.
    using Rw = typename Vec16<T>::raw;
    const int rowbytes = ld * static_cast<int>(sizeof(T));
    auto ldrow = [&](Rw (&x)[NV], int r) {
      const auto rs = make_rsrc(X + static_cast<long long>(r) * ld, rowbytes);
#pragma unroll
      for (int j = 0; j < NV; ++j) x[j] = buf_load16<Rw>(rs, (j * BS + tid) * VN * static_cast<int>(sizeof(T)));
    };
    const int rb = lead.row_begin, re = lead.row_end;
    // labels through a descriptor too, issued ahead of the next pair's rows (a flat load issued after
    // them would make its wait drain the prefetch)
    const auto yrs = make_rsrc(Y + rb, (re - rb) * static_cast<int>(sizeof(A)));
    Rw xa[NV], xb[NV];
    if (rb < re) {
      ldrow(xa, rb);
      ldrow(xb, min(rb + 1, re - 1));
    }
    for (int r = rb; r < re; r += 2) {
      const bool two = r + 1 < re;
      const int rn = r + 2 < re ? r + 2 : r;
      const A y0 = buf_load_scalar<A>(yrs, (r - rb) * static_cast<int>(sizeof(A)));
      const A y1 = buf_load_scalar<A>(yrs, (two ? r + 1 - rb : r - rb) * static_cast<int>(sizeof(A)));
      Rw na[NV], nb[NV];
      ldrow(na, rn);
      ldrow(nb, min(rn + 1, re - 1));
      A a0[NV][VN], a1[NV][VN];
#pragma unroll
      for (int j = 0; j < NV; ++j)
#pragma unroll
        for (int v = 0; v < VN; ++v) {
          a0[j][v] = Vec16<T>::template elem<A>(xa[j], v);
          a1[j][v] = two ? Vec16<T>::template elem<A>(xb[j], v) : A(0);
        }
      pair(a0, a1, y0, two ? y1 : A(0), two);
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        xa[j] = na[j];
        xb[j] = nb[j];
      }
    }
  } else {
    for (int r = lead.row_begin; r < lead.row_end; r += 2) {
      const bool two = r + 1 < lead.row_end;
      const T* x0 = X + static_cast<long long>(r) * ld;
      const T* x1 = X + static_cast<long long>(two ? r + 1 : r) * ld;
      A a0[NV][VN], a1[NV][VN];
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int c0 = (j * BS + tid) * VN;
        if (valid[j]) {
          Vec16<T>::template load<A, true>(x0 + c0, a0[j]);
          Vec16<T>::template load<A, true>(x1 + c0, a1[j]);
        } else {
#pragma unroll
          for (int v = 0; v < VN; ++v) { a0[j][v] = A(0); a1[j][v] = A(0); }
        }
      }
      pair(a0, a1, Y[r], two ? Y[r + 1] : A(0), two);
    }
  }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    if (!act[q]) continue;
    A* out = slab + static_cast<long long>(tasks[blockIdx.x * R + q].slab) * ld;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c0 = (j * BS + tid) * VN;
      if (valid[j]) {
#pragma unroll
        for (int v = 0; v < VN; ++v) out[c0 + v] = g[q][j][v];
      }
    }
  }
}

// Slab reduction, two fixed-order stages (bitwise reproducible, no atomics):
//   stage 1: block (64-column chunk, slot, split) — 4 waves stride over the split's tasks,
//            lane = column, then fold the waves in LDS -> part[slot][split][c]
//   stage 2: G[slot][c] = sum over splits of part[slot][split][c]
// 16 splits x 16 column chunks x slots gives thousands of workgroups for what used to be
// a 32-workgroup serial loop (70 us -> a few us at 2048 tasks x 1000 columns).
constexpr int kSplits = 16;
// Slab reduction form of the non-update paths (set_slab_reduce_mode, for same-box A/B by
// tools/bench_kernels.py --only reduce): 1 = one fused launch for plain reductions and puts
// (slab_reduce_fused[_put]); 2 = fused plain reductions, puts as stage 1 + the put kernel;
// 0 = the two stages everywhere.
static int g_slab_mode = 1;
// Timeline probe of grad_dense_multi (set_grad_stamps; nullptr = off, every production launch).
static long long* g_stamps = nullptr;

template <typename A>
__global__ void __launch_bounds__(256)
slab_reduce_partial(const A* __restrict__ slab, const int* __restrict__ slot_task_begin,
                    A* __restrict__ part, int ld, const int* __restrict__ gate) {
  __shared__ A red[4][kWave];
  if (gate_closed(gate)) return;
  const int slot = blockIdx.y, split = blockIdx.z;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x * kWave + lane;
  const int tb = slot_task_begin[slot], te = slot_task_begin[slot + 1];
  const int per = (te - tb + kSplits - 1) / kSplits;
  const int t0 = tb + split * per;
  const int t1 = min(te, t0 + per);
  A s = A(0);
  if (c < ld)
    for (int t = t0 + wid; t < t1; t += 4) s += slab[static_cast<long long>(t) * ld + c];
  red[wid][lane] = s;
  __syncthreads();
  if (wid == 0 && c < ld)
    part[(static_cast<long long>(slot) * kSplits + split) * ld + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

template <typename A>
__global__ void __launch_bounds__(256)
slab_reduce_final(const A* __restrict__ part, A* __restrict__ G, int ld, const int* __restrict__ gate) {
  const int slot = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= ld || gate_closed(gate)) return;
  A s = A(0);
#pragma unroll
  for (int k = 0; k < kSplits; ++k) s += part[(static_cast<long long>(slot) * kSplits + k) * ld + c];
  G[static_cast<long long>(slot) * ld + c] = s;
}

// Both stages in ONE launch, bitwise the same sums: a 1024-thread block per (64-column chunk, slot),
// wave k = split k.  Lane c of wave k keeps the four interleaved sums stage 1's waves kept (rows
// t0 + w, t0 + w + 4, ... of its split, each in row order; eight rows loaded per step), folds them
// as (s0 + s1) + (s2 + s3), and wave 0 adds the 16 splits in order from A(0) like stage 2.  One launch
// and no partial buffer in HBM instead of two back-to-back launches (5.7 + 4.7 us at the 8-GPU rank
// shape, profiles/round4/prof_shape8).
template <typename A>
__device__ __forceinline__ A fused_split_sum(const A* __restrict__ slab, int t0, int t1, int ld, int c) {
  A acc[4] = {A(0), A(0), A(0), A(0)};
  int t = t0;
  for (; t + 8 <= t1; t += 8) {
    A v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = slab[static_cast<long long>(t + j) * ld + c];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j & 3] += v[j];  // accumulator (t - t0) % 4, rows in order
  }
  for (; t < t1; ++t) acc[(t - t0) & 3] += slab[static_cast<long long>(t) * ld + c];
  return (acc[0] + acc[1]) + (acc[2] + acc[3]);
}

template <typename A>
__device__ __forceinline__ A fused_slab_sum(const A* __restrict__ slab, const int* __restrict__ slot_task_begin,
                                            A (*red)[kWave], int slot, int ld, int c) {
  const int lane = threadIdx.x & 63, k = threadIdx.x >> 6;
  const int tb = slot_task_begin[slot], te = slot_task_begin[slot + 1];
  const int per = (te - tb + kSplits - 1) / kSplits;
  const int t0 = tb + k * per;
  const int t1 = min(te, t0 + per);
  red[k][lane] = c < ld && t0 < t1 ? fused_split_sum(slab, t0, t1, ld, c) : A(0);
  __syncthreads();
  A s = A(0);
  if (k == 0)
#pragma unroll
    for (int q = 0; q < kSplits; ++q) s += red[q][lane];
  return s;  // meaningful in wave 0
}

template <typename A>
__global__ void __launch_bounds__(1024)
slab_reduce_fused(const A* __restrict__ slab, const int* __restrict__ slot_task_begin, A* __restrict__ G, int ld,
                  const int* __restrict__ gate) {
  __shared__ A red[kSplits][kWave];
  if (gate_closed(gate)) return;
  const int slot = blockIdx.y, c = blockIdx.x * kWave + (threadIdx.x & 63);
  const A s = fused_slab_sum(slab, slot_task_begin, red, slot, ld, c);
  if ((threadIdx.x >> 6) == 0 && c < ld) G[static_cast<long long>(slot) * ld + c] = s;
}

// The same with the worker's message put (slab_reduce_final_put's protocol: every block releases its
// columns and counts itself done; the last block writes the tags, releases them and stores the flag).
template <typename A>
__global__ void __launch_bounds__(1024)
slab_reduce_fused_put(const A* __restrict__ slab, const int* __restrict__ slot_task_begin, A* __restrict__ G, int ld,
                      PutDesc put) {
  __shared__ A red[kSplits][kWave];
  __shared__ int s_last, s_live;
  const int slot = blockIdx.y, c = blockIdx.x * kWave + (threadIdx.x & 63);
  const bool w0 = (threadIdx.x >> 6) == 0;
  if (gate_closed(put.gate)) {  // a skipped stale round (launch-uniform): decide the next one's gate
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) put_decide_next_gate(put);
    return;
  }
  if (threadIdx.x == 0) s_live = !(put.abort && __hip_atomic_load(put.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  const A s = fused_slab_sum(slab, slot_task_begin, red, slot, ld, c);  // (its barrier publishes s_live)
  const bool live = s_live;
  if (w0 && c < ld) {
    const long long o = static_cast<long long>(slot) * ld + c;
    G[o] = s;
    if (live) static_cast<A*>(put.dst)[o] = s;
  }
  if (!live) return;  // block-uniform
  if (put.tag && w0) {
    const unsigned long long ws = wave_sum_u64(c < ld ? tag_term(elem_bits(s), c) : 0ull);
    if (threadIdx.x == 0 && ws) atomicAdd(put.csum + slot, ws);
  }
  block_release_system(put.strict);  // this block's mailbox columns (and checksum adds) are out before its count
  if (threadIdx.x == 0) {
    const unsigned int total = gridDim.x * gridDim.y;
    const unsigned int prev = count_block_done(put.counter, put.strict);
    s_last = prev == total - 1;
    if (s_last) __hip_atomic_store(put.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;  // block-uniform
  if (put.tag) {
    for (int r = threadIdx.x; r < static_cast<int>(gridDim.y); r += blockDim.x) {
      const unsigned long long sum = atomicExch(put.csum + r, 0ull);
      put.tag[r] = MsgTag{static_cast<unsigned int>(put.value), put.rank, sum};
    }
    if (put.corrupt && threadIdx.x == 0) static_cast<unsigned char*>(put.dst)[1] ^= 0x10;  // test hook
  }
  if (threadIdx.x == 0) put_stamp(put);
  block_release_system(put.strict);  // the tags (and the landing stamp) before the flag
  if (threadIdx.x == 0) {
    publish_u64(put.flag, put.value, put.strict);
    put_decide_next_gate(put);
  }
}

// Stage 2 fused with the worker's message put (transport.hip's put + signal protocol): every
// block also stores its sums straight into the receiver's mailbox rows (put.dst, the same
// [slot][ld] layout as G), releases them at system scope (block_release_system) and counts
// itself done; the last block resets the counter and stores the flag behind its own release.  Saves the separate put_signal launch on
// every worker round's critical path.  No early return: every thread reaches the barrier.
// Tagged puts (put.tag != nullptr, integrity.h): every block also adds its columns' checksum
// terms of its slot's row into the sender scratch put.csum[slot]; the last block turns the sums
// into the receiver's tags before the flag.  put.abort set: the pump gave up, G is still
// written (the local copy) but nothing is put or announced.
template <typename A>
__global__ void __launch_bounds__(256)
slab_reduce_final_put(const A* __restrict__ part, A* __restrict__ G, int ld, PutDesc put) {
  __shared__ unsigned long long scratch[4];
  __shared__ int s_last, s_live;
  const int slot = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (gate_closed(put.gate)) {  // a skipped stale round (launch-uniform): decide the next one's gate
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) put_decide_next_gate(put);
    return;
  }
  if (threadIdx.x == 0)  // one read, shared: every wave of the block takes the same branch
    s_live = !(put.abort && __hip_atomic_load(put.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  __syncthreads();
  const bool live = s_live;
  unsigned long long term = 0;
  if (c < ld) {
    A s = A(0);
#pragma unroll
    for (int k = 0; k < kSplits; ++k) s += part[(static_cast<long long>(slot) * kSplits + k) * ld + c];
    const long long o = static_cast<long long>(slot) * ld + c;
    G[o] = s;
    if (live) static_cast<A*>(put.dst)[o] = s;
    term = tag_term(elem_bits(s), c);
  }
  if (!live) return;  // block-uniform
  if (put.tag) {
    const unsigned long long bs = block_sum_u64(term, scratch);
    if (threadIdx.x == 0 && bs) atomicAdd(put.csum + slot, bs);
  }
  block_release_system(put.strict);  // this block's mailbox columns (and checksum adds) are out before its count
  if (threadIdx.x == 0) {
    const unsigned int total = gridDim.x * gridDim.y;
    const unsigned int prev = count_block_done(put.counter, put.strict);
    s_last = prev == total - 1;
    if (s_last) __hip_atomic_store(put.counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;  // block-uniform
  if (put.tag) {
    for (int r = threadIdx.x; r < static_cast<int>(gridDim.y); r += blockDim.x) {
      const unsigned long long sum = atomicExch(put.csum + r, 0ull);
      put.tag[r] = MsgTag{static_cast<unsigned int>(put.value), put.rank, sum};
    }
    if (put.corrupt && threadIdx.x == 0) static_cast<unsigned char*>(put.dst)[1] ^= 0x10;  // test hook
  }
  if (threadIdx.x == 0) put_stamp(put);
  block_release_system(put.strict);  // the tags (and the landing stamp) before the flag
  if (threadIdx.x == 0) {
    publish_u64(put.flag, put.value, put.strict);
    put_decide_next_gate(put);
  }
}

// Stage 2 + put of a SMALL message set (nslots * ld <= kPutOneElems: the 8-GPU rank's 3 x 1000) in
// ONE 1024-thread block: no cross-block counter and no second release -- the block sums its
// elements two at a time (32 split loads in flight per thread), keeps the tag checksums in LDS
// (integer adds, order-free), writes the tags, releases once and stores the flag.  The multi-block
// form pays a device-scope atomic round trip and the last block's own release on top.
constexpr int kPutOneElems = 4096, kPutOneSlots = 16;

template <typename A>
__global__ void __launch_bounds__(1024)
slab_reduce_final_put1(const A* __restrict__ part, A* __restrict__ G, int ld, int nslots, PutDesc put) {
  __shared__ unsigned long long tsum[kPutOneSlots];
  __shared__ int s_live;
  const int tid = threadIdx.x;
  if (gate_closed(put.gate)) {  // a skipped stale round (launch-uniform)
    if (tid == 0) put_decide_next_gate(put);
    return;
  }
  if (tid < kPutOneSlots) tsum[tid] = 0;
  if (tid == 0) s_live = !(put.abort && __hip_atomic_load(put.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  __syncthreads();
  const bool live = s_live;
  const int n = nslots * ld;
  for (int e0 = tid; e0 < n; e0 += 2 * static_cast<int>(blockDim.x)) {
    const int e1 = e0 + static_cast<int>(blockDim.x);
    const int q0 = e0 / ld, c0 = e0 - q0 * ld;
    const bool two = e1 < n;
    const int q1 = two ? e1 / ld : q0, c1 = two ? e1 - q1 * ld : c0;
    A v0[kSplits], v1[kSplits];
#pragma unroll
    for (int k = 0; k < kSplits; ++k) {
      v0[k] = part[(static_cast<long long>(q0) * kSplits + k) * ld + c0];
      v1[k] = part[(static_cast<long long>(q1) * kSplits + k) * ld + c1];
    }
    A s0 = A(0), s1 = A(0);
#pragma unroll
    for (int k = 0; k < kSplits; ++k) {  // slab_reduce_final's order
      s0 += v0[k];
      s1 += v1[k];
    }
    G[e0] = s0;
    if (live) static_cast<A*>(put.dst)[e0] = s0;
    if (put.tag) atomicAdd(&tsum[q0], tag_term(elem_bits(s0), c0));
    if (two) {
      G[e1] = s1;
      if (live) static_cast<A*>(put.dst)[e1] = s1;
      if (put.tag) atomicAdd(&tsum[q1], tag_term(elem_bits(s1), c1));
    }
  }
  if (!live) return;  // block-uniform
  if (put.tag) {
    __syncthreads();
    if (tid < nslots) put.tag[tid] = MsgTag{static_cast<unsigned int>(put.value), put.rank, tsum[tid]};
    if (put.corrupt && tid == 0) static_cast<unsigned char*>(put.dst)[1] ^= 0x10;  // test hook
  }
  if (tid == 0) put_stamp(put);
  block_release_system(put.strict);  // the rows, tags (and the landing stamp) before the flag
  if (tid == 0) {
    publish_u64(put.flag, put.value, put.strict);
    put_decide_next_gate(put);
  }
}

// Stage 2 + the master's combine and update of a device-driven local round in one launch
// (MasterPump::run_local; update.hip combine_update's arithmetic).  One block per 64-column chunk:
// its waves sum the chunk's splits for every slot (slab_reduce_final's order; G rows written, sums
// kept in LDS), then wave 0 combines the decoded messages in message order and updates beta / u /
// history / the next worker beta for those columns.  Replaces slab_reduce_final + combine_update
// (one launch less per round), results bitwise unchanged.  (A variant that also folded stage 1 in,
// with the last block of each chunk finishing it, paid a device-scope release fence per block --
// an L2 writeback on every XCD -- and took 427 us: profiles/round3/fused_update.)
// 1024 threads: 16 waves share a chunk's slots (the headline's 22 slots took ~6 dependent rounds of
// split loads per wave at 4 waves, 10.2 us per call: profiles/round3/prof_nt).
template <typename A>
__global__ void __launch_bounds__(1024)
slab_final_update(const A* __restrict__ part, A* __restrict__ G, int ld, int nslots, const LocalUpdate up) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lu_raw[];
  A* gs = reinterpret_cast<A*>(lu_raw);  // [nslots][64] the chunk's message sums
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int c = blockIdx.x * kWave + lane;
  if (up.stamp && blockIdx.x == 0 && threadIdx.x == 0) *up.stamp = wall_clock64();
  for (int q = wid; q < nslots; q += static_cast<int>(blockDim.x >> 6)) {
    A v = A(0);
    if (c < ld) {
#pragma unroll
      for (int k = 0; k < kSplits; ++k) v += part[(static_cast<long long>(q) * kSplits + k) * ld + c];
      G[static_cast<long long>(q) * ld + c] = v;
    }
    gs[q * kWave + lane] = v;
  }
  __syncthreads();
  if (wid != 0 || c >= ld) return;
  A* bw = static_cast<A*>(up.beta_w);
  if (c >= up.d) {  // padded columns stay exactly zero
    if (bw) bw[c] = A(0);
    return;
  }
  double g = 0.0;  // combine_update: the fma chain in message order
  for (int m = 0; m < up.nmsg; ++m) g = fma(up.coef[m], static_cast<double>(gs[up.slot[m] * kWave + lane]), g);
  const double b = up.beta[c];
  double nb;
  if (up.rule == 0) {  // GD
    nb = up.decay * b - up.gm * g;
  } else {  // AGD
    const double yt = (1.0 - up.theta) * b + up.theta * up.u[c];
    nb = yt - up.gm * g - up.l2 * b;
    up.u[c] = b + (nb - b) * (1.0 / up.theta);
  }
  up.beta[c] = nb;
  if (up.hist) up.hist[c] = nb;
  if (bw) bw[c] = static_cast<A>(nb);
}

template <typename A>
static hipError_t slab_reduce_launch(const A* slab, const int* stb, A* part, A* G, int nslots, int ld,
                                     hipStream_t st, const PutDesc* put = nullptr, const int* gate = nullptr) {
  if (put && put->tag && (nslots > kMaxTagRows || !put->csum)) return hipErrorInvalidValue;
  if (put && put->gate != gate) return hipErrorInvalidValue;  // one round, one gate
  PutDesc pd{};
  if (put) {  // the process's release form (launchers.h strict_release)
    pd = *put;
    pd.strict = strict_release() ? 1 : 0;
    put = &pd;
  }
  const dim3 fgrid(ceil_div(ld, kWave), nslots);
  if (g_slab_mode != 0 && !put) {  // both stages in one launch (bitwise the same sums)
    hipLaunchKernelGGL(slab_reduce_fused<A>, fgrid, dim3(1024), 0, st, slab, stb, G, ld, gate);
    return hipGetLastError();
  }
  if (g_slab_mode == 1 && put) {
    hipLaunchKernelGGL(slab_reduce_fused_put<A>, fgrid, dim3(1024), 0, st, slab, stb, G, ld, *put);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(slab_reduce_partial<A>, dim3(ceil_div(ld, kWave), nslots, kSplits), dim3(256), 0, st,
                     slab, stb, part, ld, gate);
  if (put && nslots <= kPutOneSlots && static_cast<long long>(nslots) * ld <= kPutOneElems)
    hipLaunchKernelGGL(slab_reduce_final_put1<A>, dim3(1), dim3(1024), 0, st, part, G, ld, nslots, *put);
  else if (put)
    hipLaunchKernelGGL(slab_reduce_final_put<A>, dim3(ceil_div(ld, 256), nslots), dim3(256), 0, st, part, G, ld, *put);
  else
    hipLaunchKernelGGL(slab_reduce_final<A>, dim3(ceil_div(ld, 256), nslots), dim3(256), 0, st, part, G, ld, gate);
  return hipGetLastError();
}

// ----- Wide-feature fallback (d > 64 * 32): two passes over X, still no atomics. -----
// Pass 1: one wave per row computes z = x_row . beta and stores the loss residual r.
template <typename T, typename A, int LOSS>
__global__ void __launch_bounds__(256)
rowdot_residual(const Segment* __restrict__ segs, const Task* __restrict__ tasks,
                const A* __restrict__ beta, const int* __restrict__ task_row_off,
                A* __restrict__ rbuf, int ld, const int* __restrict__ gate) {
  constexpr int VN = Vec16<T>::N;
  if (gate_closed(gate)) return;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int nw = blockDim.x >> 6;
  const Task task = tasks[blockIdx.x];
  const Segment seg = segs[task.seg];
  const T* __restrict__ X = static_cast<const T*>(seg.X);
  const A* __restrict__ Y = static_cast<const A*>(seg.y);
  const A coef = static_cast<A>(seg.coef);
  const int off = task_row_off[blockIdx.x];
  for (int r = task.row_begin + wid; r < task.row_end; r += nw) {
    const T* x = X + static_cast<long long>(r) * ld;
    A z = A(0);
    for (int c0 = lane * VN; c0 < ld; c0 += kWave * VN) {
      A a[VN];
      Vec16<T>::template load<A, true>(x + c0, a);
#pragma unroll
      for (int v = 0; v < VN; ++v) z = fma(a[v], beta[c0 + v], z);
    }
    z = wave_allreduce_sum(z);
    if (lane == 0) rbuf[off + (r - task.row_begin)] = residual<LOSS, A>(z, Y[r], coef);
  }
}

// Pass 2: slab[task, cols] = sum over the task's rows of r_row * x_row[cols].
template <typename T, typename A>
__global__ void __launch_bounds__(256)
xt_r_tiles(const Segment* __restrict__ segs, const Task* __restrict__ tasks,
           const int* __restrict__ task_row_off, const A* __restrict__ rbuf,
           A* __restrict__ slab, int ld, const int* __restrict__ gate) {
  constexpr int VN = Vec16<T>::N;
  if (gate_closed(gate)) return;
  const Task task = tasks[blockIdx.x];
  const Segment seg = segs[task.seg];
  const T* __restrict__ X = static_cast<const T*>(seg.X);
  const int off = task_row_off[blockIdx.x];
  const int c0 = (blockIdx.y * blockDim.x + threadIdx.x) * VN;
  if (c0 >= ld) return;
  A g[VN];
#pragma unroll
  for (int v = 0; v < VN; ++v) g[v] = A(0);
  for (int r = task.row_begin; r < task.row_end; ++r) {
    A a[VN];
    Vec16<T>::template load<A, true>(X + static_cast<long long>(r) * ld + c0, a);
    const A rr = rbuf[off + (r - task.row_begin)];
#pragma unroll
    for (int v = 0; v < VN; ++v) g[v] = fma(rr, a[v], g[v]);
  }
  A* out = slab + static_cast<long long>(task.slab) * ld + c0;
#pragma unroll
  for (int v = 0; v < VN; ++v) out[v] = g[v];
}

}  // namespace eh

// ---------------------------------------------------------------------------------
// Host launchers (called from bindings.cpp).
namespace eh {

void set_slab_reduce_mode(int mode) { g_slab_mode = mode; }
void set_grad_stamps(void* stamps) { g_stamps = static_cast<long long*>(stamps); }
int slab_reduce_mode() { return g_slab_mode; }

// Wide kernel: 16 elements per thread per row for fp64 (NV = 8), 32 for fp32 (NV = 8) and
// bf16 (NV = 4); the block size BS (256 / 512) covers ld.  (1024-thread blocks would cap a
// wave at 128 VGPRs and spill the two-row register tiles, so wider rows take the two-pass path.)
template <typename T, typename A, int LOSS>
static hipError_t launch_wide(int bs, int R, const Segment* segs, const Task* tasks, int ntasks, const A* beta,
                              A* slab, int ld, hipStream_t st, const int* gate) {
  constexpr int NV = Vec16<T>::N == 8 ? 4 : 8;
  if (R < 1 || R > 3 || ntasks % R) return hipErrorInvalidValue;
  const dim3 grid(ntasks / R);
  // Rows that fill at most half of the NV vectors (fp32 d <= 4096 at 256 threads) take the NV / 2
  // instance: the unused half would still hold R + 3 register tiles (valid[] is a run-time mask),
  // which halves the resident workgroups per CU.
  const bool half = static_cast<long long>(bs) * (NV / 2) * Vec16<T>::N >= ld;
  // fp32 / bf16 rows of <= 2048 columns (32 per lane) fit a quarter of the vectors
  const bool quarter = NV >= 8 && static_cast<long long>(bs) * (NV / 4) * Vec16<T>::N >= ld;
#define EH_WIDE(NV_, BS_, R_)                                                                                     \
  hipLaunchKernelGGL((grad_dense_wide<T, A, NV_, BS_, LOSS, R_>), grid, dim3(BS_), 0, st, segs, tasks, beta, slab, ld, \
                     gate)
#define EH_WIDE_NV(BS_, R_)       \
  do {                            \
    if (quarter)                  \
      EH_WIDE(NV / 4, BS_, R_);   \
    else if (half)                \
      EH_WIDE(NV / 2, BS_, R_);   \
    else                          \
      EH_WIDE(NV, BS_, R_);       \
  } while (0)
  if (bs == 256 && R > 1 && !half) {
    // Replica bundles of full-width rows: 512 threads of NV / 2 vectors cover the same columns.  The
    // 256-thread NV instance holds R + 3 tiles of 2 NV values per thread (fp64 R = 3: 256 VGPRs plus
    // AGPR spills, 1 wave per SIMD); at 512 threads the tiles halve (150 VGPRs) and a CU keeps 8 waves
    // of the bundle in flight instead of 4.  One such workgroup is resident per CU
    // (ops/grad.py wide_slots_per_cu).
    if (R == 2)
      hipLaunchKernelGGL((grad_dense_wide<T, A, NV / 2, 512, LOSS, 2, true>), grid, dim3(512), 0, st, segs, tasks, beta,
                         slab, ld, gate);
    else
      hipLaunchKernelGGL((grad_dense_wide<T, A, NV / 2, 512, LOSS, 3, true>), grid, dim3(512), 0, st, segs, tasks, beta,
                         slab, ld, gate);
  } else if (bs == 256) {
    if (R == 1) EH_WIDE_NV(256, 1); else if (R == 2) EH_WIDE_NV(256, 2); else EH_WIDE_NV(256, 3);
  } else if (bs == 512 && R == 1) {  // (replica bundles of 512-thread rows would spill: R * 16+ accumulators)
    EH_WIDE_NV(512, 1);
  } else {
    return hipErrorInvalidValue;
  }
#undef EH_WIDE_NV
#undef EH_WIDE
  return hipGetLastError();
}

// grad_dense_multi launch; the folded form takes 3 waves' accumulators in dynamic LDS.
template <typename T, typename A, int C, int LOSS, int R>
static hipError_t launch_multi(bool fold, bool lane_epi, bool pair, dim3 grid, dim3 block, hipStream_t st,
                               const Segment* segs, const Task* tasks, int nb, const A* beta, A* slab, int ld,
                               const int* gate) {
  if (!fold) {  // (the lane / pair-row epilogues come with the fold only)
    hipLaunchKernelGGL((grad_dense_multi<T, A, C, LOSS, R, false, 0>), grid, block, 0, st, segs, tasks, nb, beta, slab, ld,
                       gate, g_stamps);
    return hipGetLastError();
  }
  const size_t lds = 3ull * R * C * kWave * sizeof(A);
  auto kern = grad_dense_multi<T, A, C, LOSS, R, true, 0>;
  if (pair) {  // four row buffers: narrow rows only
    if constexpr (C <= 8) kern = grad_dense_multi<T, A, C, LOSS, R, true, 2>;
    else return hipErrorInvalidValue;
  } else if (lane_epi) {
    kern = grad_dense_multi<T, A, C, LOSS, R, true, 1>;
  }
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, grid, block, lds, st, segs, tasks, nb, beta, slab, ld, gate, g_stamps);
  return hipGetLastError();
}

template <typename T, typename A, int LOSS>
static hipError_t launch_fused_cpl(int cpl, const Segment* segs, const Task* tasks, int ntasks,
                                   const A* beta, A* slab, int ld, hipStream_t st, const KernelChoice& k,
                                   const int* gate = nullptr) {
  if (k.kind == kGradMfma) {  // bf16 replica bundles on the matrix cores (grad_mfma.hip)
    if constexpr (std::is_same<T, bf16_t>::value)
      return grad_mfma_launch(LOSS, segs, tasks, ntasks, k.replicas, beta, slab, ld, st, gate);
    return hipErrorInvalidValue;
  }
  if (k.kind == kGradWide || cpl >= 256)  // (rows of 32 columns per lane run 256-thread wide rows too)
    return launch_wide<T, A, LOSS>(cpl >= 256 ? cpl : 256, k.kind == kGradWide ? k.replicas : 1, segs, tasks, ntasks,
                                   beta, slab, ld, st, gate);
  const int R = k.replicas;
  const bool bundled = k.kind == kGradStaged || k.kind == kGradMulti;
  if (bundled && (R < 1 || ntasks % R != 0)) return hipErrorInvalidValue;
  StagedGeom sg{};
  if (k.kind == kGradStaged &&
      (R > 8 || !staged_geometry(R, ld * static_cast<int>(sizeof(T)), 64ull * cpl * sizeof(A), &sg, k.wpr)))
    return hipErrorInvalidValue;
  constexpr int VN = Vec16<T>::N;
  const dim3 block(256);
  const dim3 grid(ntasks);
  // CPL (columns per lane) must be a multiple of the 16-byte vector width VN.
#define EH_IF(C)                                                                                       \
  case C:                                                                                              \
    if constexpr (C % VN == 0) {                                                                       \
      if (k.kind == kGradStaged) { /* rows streamed once through an LDS ring, one wave per replica */  \
        auto kern = k.pair ? grad_dense_staged<T, A, C, LOSS, true> : grad_dense_staged<T, A, C, LOSS, false>; \
        if (sg.lds > 65536) {                                                                          \
          const hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),                \
              hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(sg.lds));                   \
          if (ea != hipSuccess) return ea;                                                             \
        }                                                                                              \
        hipLaunchKernelGGL(kern, dim3(ntasks / R), dim3(64 * R * sg.wpr), sg.lds, st, segs, tasks, beta, \
                           slab, ld, sg.srows, sg.pieces, sg.nstage, sg.wpr, gate);                    \
        return hipGetLastError();                                                                      \
      }                                                                                                \
      if (k.kind == kGradMulti) { /* every replica of a bundle in one wave, rows in registers */       \
        if constexpr (C <= 16) {                                                                       \
          const int nb_ = ntasks / R;                                                                  \
          if (k.fold && nb_ % 4) return hipErrorInvalidValue;                                          \
          const dim3 mg((nb_ + 3) / 4), mb(256);                                                       \
          const bool f = k.fold != 0, le = k.lane_epi != 0, pr = k.pair != 0;                          \
          if (R == 1) return launch_multi<T, A, C, LOSS, 1>(f, le, pr, mg, mb, st, segs, tasks, nb_, beta, slab, ld, gate); \
          if (R == 2) return launch_multi<T, A, C, LOSS, 2>(f, le, pr, mg, mb, st, segs, tasks, nb_, beta, slab, ld, gate); \
          if (R == 3) return launch_multi<T, A, C, LOSS, 3>(f, le, pr, mg, mb, st, segs, tasks, nb_, beta, slab, ld, gate); \
        }                                                                                              \
        return hipErrorInvalidValue;                                                                   \
      }                                                                                                \
      /* fused: a wave per row, k.rows rows in flight (2: the interleaved pair kernel), beta in      \
         registers or LDS */                                                                           \
      const size_t sh = 4ull * kWave * C * sizeof(A);                                                  \
      const size_t shb = sh + kWave * C * sizeof(A);                                                   \
      if (k.beta_lds) {                                                                                \
        if (k.rows == 1)                                                                               \
          hipLaunchKernelGGL((grad_dense_fused<T, A, C, LOSS, 1, true>), grid, block, shb, st, segs, tasks, beta, slab, ld, gate); \
        else if (k.rows == 2)                                                                          \
          hipLaunchKernelGGL((grad_dense_fused<T, A, C, LOSS, 2, true>), grid, block, shb, st, segs, tasks, beta, slab, ld, gate); \
        else                                                                                           \
          hipLaunchKernelGGL((grad_dense_fused<T, A, C, LOSS, 4, true>), grid, block, shb, st, segs, tasks, beta, slab, ld, gate); \
      } else if (k.rows == 1) {                                                                        \
        hipLaunchKernelGGL((grad_dense_fused<T, A, C, LOSS, 1>), grid, block, sh, st, segs, tasks, beta, slab, ld, gate); \
      } else if (k.rows == 4) {                                                                        \
        hipLaunchKernelGGL((grad_dense_fused<T, A, C, LOSS, 4>), grid, block, sh, st, segs, tasks, beta, slab, ld, gate); \
      } else {                                                                                         \
        hipLaunchKernelGGL((grad_dense_fused_pair<T, A, C, LOSS>), grid, block, sh, st, segs, tasks, beta, slab, ld, gate); \
      }                                                                                                \
      return hipGetLastError();                                                                        \
    } else {                                                                                           \
      return hipErrorInvalidValue;                                                                     \
    }
  switch (cpl) {
    EH_IF(2)
    EH_IF(4)
    EH_IF(8)
    EH_IF(16)
    EH_IF(32)
    default:
      return hipErrorInvalidValue;
  }
#undef EH_IF
}

// dtype codes: 0 = fp64 storage/fp64 acc, 1 = fp32/fp32, 2 = bf16 storage/fp32 acc
hipError_t grad_dense_launch(int dtype, int loss, int cpl, const void* segs, const void* tasks,
                             int ntasks, const void* beta, void* slab, const int* slot_task_begin,
                             int nslots, void* part, void* G, int ld, hipStream_t st, const KernelChoice& k,
                             const PutDesc* put, const int* gate) {
  const Segment* S = static_cast<const Segment*>(segs);
  const Task* Tk = static_cast<const Task*>(tasks);
  hipError_t e = hipSuccess;
  if (dtype == 0) {
    e = loss == kLogistic
            ? launch_fused_cpl<double, double, kLogistic>(cpl, S, Tk, ntasks, (const double*)beta, (double*)slab, ld, st, k, gate)
            : launch_fused_cpl<double, double, kLeastSquares>(cpl, S, Tk, ntasks, (const double*)beta, (double*)slab, ld, st, k, gate);
  } else if (dtype == 1) {
    e = loss == kLogistic
            ? launch_fused_cpl<float, float, kLogistic>(cpl, S, Tk, ntasks, (const float*)beta, (float*)slab, ld, st, k, gate)
            : launch_fused_cpl<float, float, kLeastSquares>(cpl, S, Tk, ntasks, (const float*)beta, (float*)slab, ld, st, k, gate);
  } else {
    e = loss == kLogistic
            ? launch_fused_cpl<bf16_t, float, kLogistic>(cpl, S, Tk, ntasks, (const float*)beta, (float*)slab, ld, st, k, gate)
            : launch_fused_cpl<bf16_t, float, kLeastSquares>(cpl, S, Tk, ntasks, (const float*)beta, (float*)slab, ld, st, k, gate);
  }
  if (e != hipSuccess) return e;
  if (dtype == 0) return slab_reduce_launch<double>((const double*)slab, slot_task_begin, (double*)part, (double*)G, nslots, ld, st, put, gate);
  return slab_reduce_launch<float>((const float*)slab, slot_task_begin, (float*)part, (float*)G, nslots, ld, st, put, gate);
}


hipError_t grad_dense_update_launch(int dtype, int loss, int cpl, const void* segs, const void* tasks, int ntasks,
                                    const void* beta, void* slab, const int* stb, int nslots, void* part, void* G,
                                    int ld, hipStream_t st, const KernelChoice& k, const LocalUpdate& up) {
  if (nslots < 1 || nslots > kMaxMsgs || up.nmsg < 0 || up.nmsg > kMaxMsgs || !up.beta) return hipErrorInvalidValue;
  for (int m = 0; m < up.nmsg; ++m)
    if (up.slot[m] < 0 || up.slot[m] >= nslots) return hipErrorInvalidValue;
  const Segment* S = static_cast<const Segment*>(segs);
  const Task* Tk = static_cast<const Task*>(tasks);
  hipError_t e;
  if (dtype == 0)
    e = loss == kLogistic ? launch_fused_cpl<double, double, kLogistic>(cpl, S, Tk, ntasks, (const double*)beta, (double*)slab, ld, st, k)
                          : launch_fused_cpl<double, double, kLeastSquares>(cpl, S, Tk, ntasks, (const double*)beta, (double*)slab, ld, st, k);
  else if (dtype == 1)
    e = loss == kLogistic ? launch_fused_cpl<float, float, kLogistic>(cpl, S, Tk, ntasks, (const float*)beta, (float*)slab, ld, st, k)
                          : launch_fused_cpl<float, float, kLeastSquares>(cpl, S, Tk, ntasks, (const float*)beta, (float*)slab, ld, st, k);
  else
    e = loss == kLogistic ? launch_fused_cpl<bf16_t, float, kLogistic>(cpl, S, Tk, ntasks, (const float*)beta, (float*)slab, ld, st, k)
                          : launch_fused_cpl<bf16_t, float, kLeastSquares>(cpl, S, Tk, ntasks, (const float*)beta, (float*)slab, ld, st, k);
  if (e != hipSuccess) return e;
  const dim3 pgrid(ceil_div(ld, kWave), nslots, kSplits);
  const size_t lds = static_cast<size_t>(nslots) * kWave * (dtype == 0 ? 8 : 4);
  auto go = [&](const void* kern) -> hipError_t {
    if (lds <= 60 * 1024) return hipSuccess;
    return hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  };
  if (dtype == 0) {
    hipLaunchKernelGGL(slab_reduce_partial<double>, pgrid, dim3(256), 0, st, (const double*)slab, stb, (double*)part, ld, nullptr);
    if ((e = go(reinterpret_cast<const void*>(slab_final_update<double>))) != hipSuccess) return e;
    hipLaunchKernelGGL(slab_final_update<double>, dim3(ceil_div(ld, kWave)), dim3(1024), lds, st, (const double*)part,
                       (double*)G, ld, nslots, up);
  } else {
    hipLaunchKernelGGL(slab_reduce_partial<float>, pgrid, dim3(256), 0, st, (const float*)slab, stb, (float*)part, ld, nullptr);
    if ((e = go(reinterpret_cast<const void*>(slab_final_update<float>))) != hipSuccess) return e;
    hipLaunchKernelGGL(slab_final_update<float>, dim3(ceil_div(ld, kWave)), dim3(1024), lds, st, (const float*)part,
                       (float*)G, ld, nslots, up);
  }
  return hipGetLastError();
}

hipError_t grad_dense_twopass_launch(int dtype, int loss, const void* segs, const void* tasks,
                                     int ntasks, const void* beta, const int* task_row_off,
                                     void* rbuf, void* slab, const int* slot_task_begin,
                                     int nslots, void* part, void* G, int ld, hipStream_t st, const int* gate) {
  const Segment* S = static_cast<const Segment*>(segs);
  const Task* Tk = static_cast<const Task*>(tasks);
  const dim3 block(256);
  if (dtype == 0) {
    if (loss == kLogistic)
      hipLaunchKernelGGL((rowdot_residual<double, double, kLogistic>), dim3(ntasks), block, 0, st, S, Tk, (const double*)beta, task_row_off, (double*)rbuf, ld, gate);
    else
      hipLaunchKernelGGL((rowdot_residual<double, double, kLeastSquares>), dim3(ntasks), block, 0, st, S, Tk, (const double*)beta, task_row_off, (double*)rbuf, ld, gate);
    hipLaunchKernelGGL((xt_r_tiles<double, double>), dim3(ntasks, ceil_div(ld, 256 * 2)), block, 0, st, S, Tk, task_row_off, (const double*)rbuf, (double*)slab, ld, gate);
  } else if (dtype == 1) {
    if (loss == kLogistic)
      hipLaunchKernelGGL((rowdot_residual<float, float, kLogistic>), dim3(ntasks), block, 0, st, S, Tk, (const float*)beta, task_row_off, (float*)rbuf, ld, gate);
    else
      hipLaunchKernelGGL((rowdot_residual<float, float, kLeastSquares>), dim3(ntasks), block, 0, st, S, Tk, (const float*)beta, task_row_off, (float*)rbuf, ld, gate);
    hipLaunchKernelGGL((xt_r_tiles<float, float>), dim3(ntasks, ceil_div(ld, 256 * 4)), block, 0, st, S, Tk, task_row_off, (const float*)rbuf, (float*)slab, ld, gate);
  } else {
    if (loss == kLogistic)
      hipLaunchKernelGGL((rowdot_residual<bf16_t, float, kLogistic>), dim3(ntasks), block, 0, st, S, Tk, (const float*)beta, task_row_off, (float*)rbuf, ld, gate);
    else
      hipLaunchKernelGGL((rowdot_residual<bf16_t, float, kLeastSquares>), dim3(ntasks), block, 0, st, S, Tk, (const float*)beta, task_row_off, (float*)rbuf, ld, gate);
    hipLaunchKernelGGL((xt_r_tiles<bf16_t, float>), dim3(ntasks, ceil_div(ld, 256 * 8)), block, 0, st, S, Tk, task_row_off, (const float*)rbuf, (float*)slab, ld, gate);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (dtype == 0) return slab_reduce_launch<double>((const double*)slab, slot_task_begin, (double*)part, (double*)G, nslots, ld, st, nullptr, gate);
  return slab_reduce_launch<float>((const float*)slab, slot_task_begin, (float*)part, (float*)G, nslots, ld, st, nullptr, gate);
}

}  // namespace eh
