// MFMA worker gradient for bf16-stored design matrices: replica bundles on the matrix cores.
//
// Reference math per logical worker (ref src/approximate_coding.py:194-196, src/coded.py:183-185):
//   z = X·beta;  r = -(coef * y) / (exp(y * z) + 1)   (least squares: r = -2 coef (y - z));  g = Xᵀ·r
// A bundle (ops/grad.py) is the R <= 16 co-located messages that read the same rows of one
// partition (FRC/AGC group members, cyclic neighbours): every replica computes its OWN z, residual
// (own coefficient) and gradient.  grad_dense_staged does that on the VALU, one wave per replica;
// for bf16 storage it is compute-bound (0.68 ms for 2 GB at the headline).  Here the R replicas are
// the 16-wide M dimension of two GEMMs per 32-row stage, on v_mfma_f32_16x16x32_bf16:
//
//   GEMM1  Zᵀ[16 replicas x 32 rows] = Bm[16 x d] · X_stageᵀ     Bm row q = beta (q < R), 0 otherwise
//   GEMM2  G[16 replicas x d]       += Rm[16 x 32 rows] · X_stage  Rm[q][row] = residual of replica q
//
// so no replica's work is skipped (each owns a row of Zᵀ, Rm and G).  beta and the residuals are
// fp32: each is split into three bf16 terms (v = v0 + v1 + v2 + O(2^-25 v)) fed as three MFMAs,
// so the products keep fp32 accuracy while X stays exact bf16; accumulation is fp32 in the MFMA.
// (A two-term split measured ~1e-5 absolute error on O(10) gradients: 10x the VALU kernel's.)
//
// Data movement (grad_staged_mfma; grad_vring_mfma below is the same ring fed through registers, an A/B):
// the workgroup (8 waves) streams its row range through a 2-stage LDS ring with
// 16-byte LDS-DMA (global_load_lds, lds_dma.h) exactly like grad_dense_staged; a stage is 32 rows
// (64 KB at d = 1000) + their labels.  GEMM1 reads its B operand (X rows, k = columns) with
// ds_read_b128; GEMM2 needs X with k = rows, read through gfx950's transposing ds_read_b64_tr_b16
// from the same row-major image.  GEMM1's K (columns) is split over the 8 waves and the partial
// Zᵀ tiles are summed through LDS; the residual is evaluated once per (replica, row) by the 512
// threads; GEMM2's N (columns) is split over the waves, each keeping its G tiles in AGPR/VGPRs for
// the whole row range.  Supports ld <= 1024 (K steps per wave KPW = 4, column tiles TPW = 8).
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "grad_dense.h"
#include "lds_dma.h"

namespace eh {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kMfNW = 8;   // waves per workgroup
constexpr int kMfKPW = 4;  // GEMM1 K steps (32 columns) per wave  -> ld <= 8 * 4 * 32 = 1024
constexpr int kMfTPW = 8;  // GEMM2 column tiles (16 columns) per wave

constexpr int kMfSplit = 3;  // bf16 terms per fp32 operand

__device__ __forceinline__ void split_bf16(float v, __bf16 (&t)[kMfSplit]) {
#pragma unroll
  for (int s = 0; s < kMfSplit; ++s) {
    t[s] = static_cast<__bf16>(v);
    v -= static_cast<float>(t[s]);  // exact: the remainder of a round-to-nearest is representable
  }
}

__device__ __forceinline__ f32x4 mma(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// K = 16 form (16-row stages): A[m = l & 15][k = 4 (l >> 4) + j], B[k][n = l & 15], same C map
__device__ __forceinline__ f32x4 mma(bf16x4 a, bf16x4 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, c, 0, 0, 0);
}

// LDS transposing read: lane 4q+p of each 16-lane group passes the address of block row q,
// columns 4p..4p+3; lane i of the group receives column i of the 4 rows (row q in element q).
__device__ __forceinline__ bf16x4 tr_read(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
      (__attribute__((address_space(3))) bf16x4*)(reinterpret_cast<size_t>(p)));
}

// S = rows per stage = K of GEMM2: 32 (v_mfma_f32_16x16x32_bf16, two transposing reads per
// fragment) or 16 (v_mfma_f32_16x16x16_bf16, one read): 16-row stages fit a 4-deep ring, so three
// stages (96 KB at d = 1000) are in flight per CU instead of one 64 KB stage.
//
// PACK (R <= 4): the three bf16 terms of each fp32 operand are rows of the M dimension instead of three
// MFMAs -- A row m = 4 r + s holds term s of replica r (s < 3; row 4 r + 3 and replicas >= R are zero) --
// so each GEMM step is ONE MFMA: the 16-row M tile had 13 of its 16 rows zero at R = 3.  Lane group g of
// the C fragment then holds replica g's three partial sums in registers 0..2, added small terms first.
// (3x fewer MFMAs: the compute of a 32-row stage, measured alone, was 191 us per 2 GB.)
template <int LOSS, int kMfS, bool PACK>
__global__ void __launch_bounds__(512)
grad_staged_mfma(const Segment* __restrict__ segs, const Task* __restrict__ tasks, const float* __restrict__ beta,
                 float* __restrict__ slab, int ld, int R, int pieces, int nstage, const int* __restrict__ gate,
                 int probe) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  if (gate_closed(gate)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned lds_base = static_cast<unsigned>(
      reinterpret_cast<size_t>((__attribute__((address_space(3))) unsigned char*)smem_raw));
  const Task lead = tasks[blockIdx.x * R];  // slot 0 of a bundle is always a real task
  const Segment ls = segs[lead.seg];
  const unsigned char* __restrict__ X = static_cast<const unsigned char*>(ls.X);
  const unsigned char* __restrict__ Y = static_cast<const unsigned char*>(ls.y);
  const int rowbytes = ld * 2;
  const int data_bytes = kMfNW * pieces * 1024;
  const int buf_bytes = data_bytes + 256;
  const int nrows = lead.row_end - lead.row_begin;
  const int nst = (nrows + kMfS - 1) / kMfS;
  float* zred = reinterpret_cast<float*>(smem_raw + nstage * buf_bytes);  // [wave][16][32] partial Zᵀ
  __bf16* rres = reinterpret_cast<__bf16*>(zred + kMfNW * 16 * kMfS);      // [split][16][32] residual terms

  // residual role of this thread: (replica rm, stage row rn); threads past 16 * S (PACK: 4 * S) idle there
  const int rm = tid / kMfS, rn = tid % kMfS;
  const bool rrole = tid < (PACK ? 4 : 16) * kMfS;
  float rcoef = 0.f;
  if (rrole && rm < R) {
    const Task tq = tasks[blockIdx.x * R + rm];
    if (tq.seg >= 0) rcoef = static_cast<float>(segs[tq.seg].coef);
  }
  // GEMM1 A fragments: A[m = lane & 15][k = 8 (lane >> 4) + j] = beta[k] for replica rows m < R
  // (PACK: term m & 3 of beta[k] for replica m >> 2 < R, m & 3 < 3)
  constexpr int NSP = PACK ? 1 : kMfSplit;
  const bool rep_ok = PACK ? ((lane & 15) >> 2) < R && (lane & 3) < kMfSplit : (lane & 15) < R;
  bf16x8 bfr[kMfKPW][NSP];
#pragma unroll
  for (int kk = 0; kk < kMfKPW; ++kk) {
    const int k0 = (w * kMfKPW + kk) * 32 + 8 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 t[kMfSplit];
      split_bf16(rep_ok && k0 + j < ld ? beta[k0 + j] : 0.f, t);
      if constexpr (PACK) {
        const int sm = lane & 3;
        bfr[kk][0][j] = sm == 0 ? t[0] : sm == 1 ? t[1] : t[2];  // (sm == 3: rep_ok false, t all zero)
      } else {
#pragma unroll
        for (int s = 0; s < kMfSplit; ++s) bfr[kk][s][j] = t[s];
      }
    }
  }
  f32x4 g[kMfTPW];
#pragma unroll
  for (int t = 0; t < kMfTPW; ++t) g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  // slab rows of the replicas whose G elements this lane holds (m = 4 (lane >> 4) + reg); looked up
  // before the stage pipeline so no vector load is issued inside it (lds_dma.h, vmcnt counting)
  // (PACK: lane group g holds replica g's three terms: slab_row[0] is replica g's row)
  int slab_row[4];
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) {
    const int m = PACK ? (reg == 0 ? lane >> 4 : R) : 4 * (lane >> 4) + reg;
    slab_row[reg] = -1;
    if (m < R) {
      const Task tq = tasks[blockIdx.x * R + m];
      if (tq.seg >= 0) slab_row[reg] = tq.slab;
    }
  }

  // Every stage, a partial last one included, is DMA'd in full: sources past the task's rows are
  // clamped onto its last 16 valid bytes, so every LDS byte the GEMMs read (rows past the end:
  // residual 0 / beta 0 there; columns past ld: discarded G columns) holds finite data without a
  // per-workgroup zero fill, and every stage costs each wave the same number of loads.
  const int full_bytes = kMfS * rowbytes;
  const int nblk = (full_bytes + 1023) >> 10;
  const int cnt_stage = (nblk > w ? (nblk - w + kMfNW - 1) / kMfNW : 0) + (w == 0 ? 1 : 0);
  auto issue = [&](int t) {
    if (probe == 2) return;  // timing probe: no stage loads (the GEMMs read whatever LDS holds)
    const unsigned dst = lds_base + (t % nstage) * buf_bytes;
    const long long r0 = lead.row_begin + static_cast<long long>(t) * kMfS;
    const int ns = min(kMfS, static_cast<int>(lead.row_end - r0));
    const int bytes = ns * rowbytes;
    const unsigned char* src = X + r0 * rowbytes;
    for (int blk = w; blk < nblk; blk += kMfNW)
      glds16(src + min(blk * 1024 + lane * 16, bytes - 16), dst + blk * 1024);
    if (w == 0) glds4(Y + r0 * 4 + min(lane * 4, ns * 4 - 4), dst + data_bytes);
  };

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // beta / table loads done before the counted loads
  for (int t = 0; t < nstage - 1 && t < nst; ++t) issue(t);
  const int fi = lane & 15, fq = fi >> 2, fp = fi & 3, fg = lane >> 4;
  for (int t = 0; t < nst; ++t) {
    const int later = (min(t + nstage - 2, nst - 1) - t) * cnt_stage;
    if (probe == 2) wait_vmcnt(0);
    else wait_vmcnt(later);  // this wave's pieces of stage t landed
    __syncthreads();    // every wave's pieces; stage t-1, zred and the residuals fully consumed
    if (t + nstage - 1 < nst) issue(t + nstage - 1);
    if (probe == 1) continue;  // timing probe: the stage stream alone
    const unsigned char* buf = smem_raw + (t % nstage) * buf_bytes;
    const float* lab = reinterpret_cast<const float*>(buf + data_bytes);
    const int ns = min(kMfS, nrows - t * kMfS);

    // ---- GEMM1: this wave's K slice of Zᵀ (S / 16 n-tiles of 16 stage rows)
    constexpr int NT = kMfS / 16;
    f32x4 z[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) z[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < kMfKPW; ++kk) {
      const int kstep = w * kMfKPW + kk;
      if (kstep * 32 >= ld) break;  // wave-uniform
      // B[k = column][n = row]: 8 consecutive columns of row (lane & 15); columns past ld are
      // clamped onto the row's last 8 (their beta is 0, the data finite)
      const int col = min(kstep * 32 + 8 * fg, ld - 8);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const bf16x8 x = *reinterpret_cast<const bf16x8*>(buf + (16 * nt + fi) * rowbytes + col * 2);
#pragma unroll
        for (int s = NSP - 1; s >= 0; --s) z[nt] = mma(bfr[kk][s], x, z[nt]);  // small terms first
      }
    }
    // C layout: lane holds C[m = 4 (lane >> 4) + reg][n = lane & 15]  (replica m, stage row n; PACK:
    // replica lane >> 4, its three terms in reg 0..2, added here)
    float* zw = zred + w * 16 * kMfS;
    if constexpr (PACK) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) zw[fg * kMfS + 16 * nt + fi] = (z[nt][2] + z[nt][1]) + z[nt][0];
    } else {
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) zw[(4 * fg + reg) * kMfS + 16 * nt + fi] = z[nt][reg];
    }
    __syncthreads();
    // ---- residual of (replica rm, row rn): fixed-order sum of the waves' K slices
    if (rrole) {
      float zs = 0.f;
#pragma unroll
      for (int v = 0; v < kMfNW; ++v) zs += zred[(v * 16 + rm) * kMfS + rn];
      const float r = rm < R && rn < ns ? residual_hw<LOSS>(zs, lab[rn], rcoef) : 0.f;
      __bf16 t[kMfSplit];
      split_bf16(r, t);
      if constexpr (PACK) {  // A row 4 rm + s; row 4 rm + 3 zero
#pragma unroll
        for (int s = 0; s < 4; ++s) rres[(4 * rm + s) * kMfS + rn] = s < kMfSplit ? t[s < kMfSplit ? s : 0] : __bf16(0.f);
      } else {
#pragma unroll
        for (int s = 0; s < kMfSplit; ++s) rres[(s * 16 + rm) * kMfS + rn] = t[s];
      }
    }
    __syncthreads();
    // ---- GEMM2: G[replica][column] += Rm · X_stage over this wave's column tiles
    if constexpr (kMfS == 32) {
      // A[m = replica lane & 15][k = row 8 (lane >> 4) + j]  (PACK: m = 4 replica + term)
      bf16x8 ar[NSP];
#pragma unroll
      for (int s = 0; s < NSP; ++s) ar[s] = *reinterpret_cast<const bf16x8*>(rres + (s * 16 + fi) * kMfS + 8 * fg);
#pragma unroll
      for (int tt = 0; tt < kMfTPW; ++tt) {
        const int c0 = (w * kMfTPW + tt) * 16;
        if (c0 >= ld) break;  // wave-uniform
        // B[k = row 8 g + j][n = column c0 + i]: rows 8g..8g+3 and 8g+4..8g+7 by two transposing
        // reads (columns past ld land in G columns that are never written)
        const unsigned char* a0 = buf + (8 * fg + fq) * rowbytes + (c0 + 4 * fp) * 2;
        const bf16x4 t0 = tr_read(a0);
        const bf16x4 t1 = tr_read(a0 + 4 * rowbytes);
        const bf16x8 xb = bf16x8{t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
#pragma unroll
        for (int s = NSP - 1; s >= 0; --s) g[tt] = mma(ar[s], xb, g[tt]);
      }
    } else {
      // A[m = replica lane & 15][k = row 4 (lane >> 4) + j]  (PACK: m = 4 replica + term)
      bf16x4 ar[NSP];
#pragma unroll
      for (int s = 0; s < NSP; ++s) ar[s] = *reinterpret_cast<const bf16x4*>(rres + (s * 16 + fi) * kMfS + 4 * fg);
#pragma unroll
      for (int tt = 0; tt < kMfTPW; ++tt) {
        const int c0 = (w * kMfTPW + tt) * 16;
        if (c0 >= ld) break;  // wave-uniform
        // B[k = row 4 g + q][n = column c0 + i]: one transposing read of rows 4g..4g+3
        const bf16x4 xb = tr_read(buf + (4 * fg + fq) * rowbytes + (c0 + 4 * fp) * 2);
#pragma unroll
        for (int s = NSP - 1; s >= 0; --s) g[tt] = mma(ar[s], xb, g[tt]);
      }
    }
  }
  // lane holds G[m = 4 (lane >> 4) + reg][column c0 + (lane & 15)]
#pragma unroll
  for (int tt = 0; tt < kMfTPW; ++tt) {
    const int c0 = (w * kMfTPW + tt) * 16;
    if (c0 >= ld) break;
    const int col = c0 + fi;
    if constexpr (PACK) {
      if (slab_row[0] >= 0 && col < ld)
        slab[static_cast<long long>(slab_row[0]) * ld + col] = (g[tt][2] + g[tt][1]) + g[tt][0];
    } else {
#pragma unroll
      for (int reg = 0; reg < 4; ++reg)
        if (slab_row[reg] >= 0 && col < ld) slab[static_cast<long long>(slab_row[reg]) * ld + col] = g[tt][reg];
    }
  }
}

// (A VGPR-streamed form -- every wave loading its column slice of a stage straight into GEMM1's B-fragment
// registers, a private LDS image for GEMM2 -- measured 0.475 ms with nt loads and 0.345 with the default
// policy against the ring's 0.316: the fragment layout fixes each load instruction at 16 rows x 64 bytes, half
// of every 128-byte line per request.  Removed in round 6; docs/PERF_NOTES.md, profiles/round6/bf16ab.)

// ---- VGPR-staged ring (R <= 4, packed terms, 32-row stages) ---------------------------------------
// grad_staged_mfma's LDS ring and arithmetic, but every stage is loaded into registers two stages ahead
// -- whole 1 KB blocks per wave instruction, full 128-byte lines, the LDS-DMA form's block map -- and
// copied into its LDS buffer with ds_write_b128 once the compute of the stage before has freed it.  Two
// stages (128 KB per CU) are in flight while a third is computed, against the LDS-DMA ring's one (its
// stream alone: 311 us per 2 GB).  Buffer loads past a partial stage's rows return zeros (finite data;
// residual 0 there), so every stage issues the same loads and the compiler waits only for the older one.
constexpr int kVrPieces = 8;  // 1 KB blocks per wave per stage at ld <= 1024 (32 rows x 2 KB / 8 waves)
// The stage loads are inline asm, counted by the kernel (lds_dma.h's reason): through the builtins the
// compiler merged the loop's entry and back-edge states conservatively and waited vmcnt(0) for both
// register sets at every other stage.  base: wave-uniform stage address; off: this lane's byte offset.
__device__ __forceinline__ uint4 vr_load16(const unsigned char* base, int off) {
  uint4 v;
  asm volatile("global_load_dwordx4 %0, %1, %2 nt" : "=v"(v) : "v"(off), "s"(base) : "memory");
  return v;
}
__device__ __forceinline__ float vr_load4(const float* base, int off) {
  float v;
  asm volatile("global_load_dword %0, %1, %2" : "=v"(v) : "v"(off), "s"(base) : "memory");
  return v;
}
// NSET register sets: NSET stages in flight while one is computed (NSET x 32 VGPRs of stage data)
template <int LOSS, int NSET>
__global__ void __launch_bounds__(512)
grad_vring_mfma(const Segment* __restrict__ segs, const Task* __restrict__ tasks, const float* __restrict__ beta,
                float* __restrict__ slab, int ld, int R, const int* __restrict__ gate, int probe) {
  constexpr int S = 32;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  if (gate_closed(gate)) return;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const Task lead = tasks[blockIdx.x * R];  // slot 0 of a bundle is always a real task
  const Segment ls = segs[lead.seg];
  const unsigned char* __restrict__ X = static_cast<const unsigned char*>(ls.X);
  const float* __restrict__ Y = static_cast<const float*>(ls.y);
  const int rowbytes = ld * 2;
  // every stage buffer holds all kVrPieces blocks, so the copies into it are unconditional (a branch per
  // block let the compiler sink the prologue's loads into it, and the loop's waits went conservative)
  constexpr int data_bytes = kMfNW * kVrPieces * 1024;
  constexpr int buf_bytes = data_bytes + 256;
  const int nrows = lead.row_end - lead.row_begin;
  const int nst = (nrows + S - 1) / S;
  float* zred = reinterpret_cast<float*>(smem_raw + 2 * buf_bytes);  // [wave][16][32] partial Zᵀ
  __bf16* rres = reinterpret_cast<__bf16*>(zred + kMfNW * 16 * S);     // [16][32] residual terms
  const int fi = lane & 15, fq = fi >> 2, fp = fi & 3, fg = lane >> 4;

  const int rm = tid / S, rn = tid % S;  // residual role (replica rm, stage row rn) of the first 4 * S threads
  const bool rrole = tid < 4 * S;
  float rcoef = 0.f;
  if (rrole && rm < R) {
    const Task tq = tasks[blockIdx.x * R + rm];
    if (tq.seg >= 0) rcoef = static_cast<float>(segs[tq.seg].coef);
  }
  // GEMM1 A fragments (packed): A[m = lane & 15][k] = term m & 3 of beta[k] for replica m >> 2 < R
  const bool rep_ok = ((lane & 15) >> 2) < R && (lane & 3) < kMfSplit;
  bf16x8 bfr[kMfKPW];
#pragma unroll
  for (int kk = 0; kk < kMfKPW; ++kk) {
    const int k0 = (w * kMfKPW + kk) * 32 + 8 * fg;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      __bf16 t[kMfSplit];
      split_bf16(rep_ok && k0 + j < ld ? beta[k0 + j] : 0.f, t);
      const int sm = lane & 3;
      bfr[kk][j] = sm == 0 ? t[0] : sm == 1 ? t[1] : t[2];
    }
  }
  f32x4 g[kMfTPW];
#pragma unroll
  for (int t = 0; t < kMfTPW; ++t) g[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  int slab_row = -1;  // lane group fg holds replica fg's G
  if (fg < R) {
    const Task tq = tasks[blockIdx.x * R + fg];
    if (tq.seg >= 0) slab_row = tq.slab;
  }

  // stage t into registers, 9 loads per wave: (stages past the last repeat it and are never stored; pieces
  // past a partial stage's rows are clamped onto its last 16 valid bytes, grad_staged_mfma's rule)
  auto load = [&](int t, uint4 (&xr)[kVrPieces], float& yv) {
    const int tc = __builtin_amdgcn_readfirstlane(min(t, nst - 1));
    const long long r0 = lead.row_begin + static_cast<long long>(tc) * S;
    const int ns = min(S, static_cast<int>(lead.row_end - r0));
    const unsigned char* base = X + r0 * rowbytes;
    const int last = ns * rowbytes - 16;
#pragma unroll
    for (int j = 0; j < kVrPieces; ++j) xr[j] = vr_load16(base, min((w + kMfNW * j) * 1024 + lane * 16, last));
    yv = vr_load4(Y + r0, 4 * min(lane & (S - 1), ns - 1));
  };
  auto store = [&](int t, const uint4 (&xr)[kVrPieces], float yv) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NSET - 1) * (kVrPieces + 1)) : "memory");  // this set landed
    if (probe >= 3) {  // timing probes: the loads alone (3: with the stage barriers, 4: without)
      asm volatile("" ::"v"(xr[0].x), "v"(xr[kVrPieces - 1].w), "v"(yv));
      return;
    }
    unsigned char* buf = smem_raw + (t & 1) * buf_bytes;
#pragma unroll
    for (int j = 0; j < kVrPieces; ++j) *reinterpret_cast<uint4*>(buf + (w + kMfNW * j) * 1024 + lane * 16) = xr[j];
    // the labels by every wave (the same values; a store under a branch let the compiler sink the load)
    reinterpret_cast<float*>(buf + data_bytes)[lane & (S - 1)] = yv;
  };
  auto compute = [&](int t) {
    const unsigned char* buf = smem_raw + (t & 1) * buf_bytes;
    const float* lab = reinterpret_cast<const float*>(buf + data_bytes);
    const int ns = min(S, nrows - t * S);
    f32x4 z[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kk = 0; kk < kMfKPW; ++kk) {
      const int kstep = w * kMfKPW + kk;
      if (kstep * 32 >= ld) break;  // wave-uniform
      const int col = min(kstep * 32 + 8 * fg, ld - 8);
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
        z[nt] = mma(bfr[kk], *reinterpret_cast<const bf16x8*>(buf + (16 * nt + fi) * rowbytes + col * 2), z[nt]);
    }
    float* zw = zred + w * 16 * S;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) zw[fg * S + 16 * nt + fi] = (z[nt][2] + z[nt][1]) + z[nt][0];
    __syncthreads();
    if (rrole) {
      float zs = 0.f;
#pragma unroll
      for (int v = 0; v < kMfNW; ++v) zs += zred[(v * 16 + rm) * S + rn];
      const float r = rm < R && rn < ns ? residual_hw<LOSS>(zs, lab[rn], rcoef) : 0.f;
      __bf16 tt[kMfSplit];
      split_bf16(r, tt);
#pragma unroll
      for (int q = 0; q < 4; ++q) rres[(4 * rm + q) * S + rn] = q < kMfSplit ? tt[q < kMfSplit ? q : 0] : __bf16(0.f);
    }
    __syncthreads();
    const bf16x8 ar = *reinterpret_cast<const bf16x8*>(rres + fi * S + 8 * fg);
#pragma unroll
    for (int tt = 0; tt < kMfTPW; ++tt) {
      const int c0 = (w * kMfTPW + tt) * 16;
      if (c0 >= ld) break;  // wave-uniform
      const unsigned char* a0 = buf + (8 * fg + fq) * rowbytes + (c0 + 4 * fp) * 2;
      const bf16x4 t0 = tr_read(a0);
      const bf16x4 t1 = tr_read(a0 + 4 * rowbytes);
      g[tt] = mma(ar, bf16x8{t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]}, g[tt]);
    }
  };
  // NSET register sets, the loop unrolled by NSET so each is named statically.  The copy of stage t
  // follows compute(t - 1) -- the buffer it reuses, t - 2's, was freed by the barrier before compute(t - 1)
  // -- and stages t + 1 .. t + NSET are in flight while stage t is computed.
  uint4 xs[NSET][kVrPieces];
  float ys[NSET];
#pragma unroll
  for (int k = 0; k < NSET; ++k) ys[k] = 0.f;
#pragma unroll
  for (int k = 0; k < kMfKPW; ++k) asm volatile("" ::"v"(bfr[k]));
  asm volatile("" ::"v"(rcoef), "v"(slab_row));
  // the setup's loads done, and its arithmetic kept here, before the counted loads (scheduled past them it
  // brought a compiler wait for beta -- vmcnt(0) -- behind the first stages' loads)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int k = 0; k < NSET; ++k) load(k, xs[k], ys[k]);
  for (int t = 0; t < nst; t += NSET) {
#pragma unroll
    for (int k = 0; k < NSET; ++k) {
      if (t + k >= nst) break;  // block-uniform
      store(t + k, xs[k], ys[k]);
      load(t + k + NSET, xs[k], ys[k]);
      if (probe != 4) __syncthreads();  // stage t + k in LDS; zred and the residuals of the stage before consumed
      if (probe == 0) compute(t + k);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the repeated loads past the last stage
#pragma unroll
  for (int tt = 0; tt < kMfTPW; ++tt) {
    const int c0 = (w * kMfTPW + tt) * 16;
    if (c0 >= ld) break;
    const int col = c0 + fi;
    if (slab_row >= 0 && col < ld) slab[static_cast<long long>(slab_row) * ld + col] = (g[tt][2] + g[tt][1]) + g[tt][0];
  }
}

// ---- layout probes (tests/test_kernels_gpu.py checks them with exact integer data) ---------------
// C[16][16] = A[16][32] · B[32][16] through one v_mfma_f32_16x16x32_bf16 with the fragment maps
// the kernel above assumes.
__global__ void mfma_probe_kernel(const float* A, const float* B, float* C) {
  const int l = threadIdx.x;
  bf16x8 a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = static_cast<__bf16>(A[(l & 15) * 32 + 8 * (l >> 4) + j]);
    b[j] = static_cast<__bf16>(B[(8 * (l >> 4) + j) * 16 + (l & 15)]);
  }
  const f32x4 c = mma(a, b, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) C[(4 * (l >> 4) + reg) * 16 + (l & 15)] = c[reg];
}
// tile: [8 rows][rowlen] bf16 (rowlen % 4 == 0, >= 32).  Group g of 16 lanes reads block rows
// 4 (g & 1) .. +3, columns 16 (g >> 1) .. +15; out[lane][q] = what lane received in element q.
__global__ void tr_probe_kernel(const float* tile, int rowlen, float* out) {
  __shared__ __attribute__((aligned(16))) __bf16 sm[8 * 64];
  const int l = threadIdx.x;
  for (int i = l; i < 8 * rowlen; i += 64) sm[i] = static_cast<__bf16>(tile[i]);
  __syncthreads();
  const int g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const unsigned char* base = reinterpret_cast<const unsigned char*>(sm);
  const bf16x4 v = tr_read(base + (4 * (g & 1) + q) * rowlen * 2 + (16 * (g >> 1) + 4 * p) * 2);
#pragma unroll
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = static_cast<float>(v[e]);
}

hipError_t mfma_probe_launch(const float* A, const float* B, float* C, hipStream_t st) {
  hipLaunchKernelGGL(mfma_probe_kernel, dim3(1), dim3(64), 0, st, A, B, C);
  return hipGetLastError();
}
hipError_t tr_probe_launch(const float* tile, int rowlen, float* out, hipStream_t st) {
  if (rowlen % 4 || rowlen < 32 || rowlen > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(tr_probe_kernel, dim3(1), dim3(64), 0, st, tile, rowlen, out);
  return hipGetLastError();
}

// Geometry of grad_staged_mfma: rows per stage S (32, 2-stage ring: 0.48 vs 0.59 ms for 16-row
// stages in a 4-deep ring at the bf16 headline, profiles/round2/s1_mfma), LDS-DMA pieces per wave per
// stage, ring depth and LDS bytes; false when ld does not fit.
static int g_mfma_rows = 32;
void set_mfma_stage_rows(int rows) { g_mfma_rows = rows == 16 ? 16 : 32; }
// timing probes of grad_staged_mfma (tools/bench_rank_shapes.py --mfma-probe; results are NOT a
// gradient): 1 = the LDS-DMA stage stream and barriers only, 2 = the GEMMs / residuals without loads;
// grad_vring_mfma also 3 = its loads and barriers (no LDS copies), 4 = its loads alone
static int g_mfma_probe = 0;
void set_mfma_probe(int mode) { g_mfma_probe = mode >= 1 && mode <= 4 ? mode : 0; }
// the packed-term form for R <= 4 (default) or the three-MFMA form, for A/B
static bool g_mfma_pack = true;
void set_mfma_pack(bool on) { g_mfma_pack = on; }
// packed bundles (R <= 4) through the VGPR-staged ring (grad_vring_mfma: 3 two register sets, 4 three) or the
// LDS-DMA stage ring (0, the default).
// At the N = 1 rank shape (2 GB; profiles/round6/bf16ab/rows_ab*.jsonl, ring_vs_vring_r8e.jsonl): on two boxes
// 0: 315.3-320.4 us, 3: 312.4-314.7, 4: 318.8-319.0 (stream alone 307.6-310.2 / 301.0-303.3 / 305.1-307.3);
// on a third, four alternating reps, 0: 312.9-316.2, 3: 314.0-319.3.  Within the box-to-box spread: no default.
static int g_mfma_stream = 0;
void set_mfma_stream(int mode) { g_mfma_stream = mode == 3 || mode == 4 ? mode : 0; }

bool mfma_geometry(int ld, int* rows, int* pieces, int* nstage, size_t* lds) {
  if (ld < 8 || ld > kMfNW * kMfKPW * 32 || ld % 8) return false;
  const int S = g_mfma_rows;  // measured: 32-row stages (fewer barriers per byte) win
  const int rowbytes = ld * 2;
  *rows = S;
  *pieces = (S * rowbytes + kMfNW * 1024 - 1) / (kMfNW * 1024);
  const size_t fixed = static_cast<size_t>(kMfNW) * 16 * S * 4 + static_cast<size_t>(kMfSplit) * 16 * S * 2;
  const size_t stage = static_cast<size_t>(kMfNW) * *pieces * 1024 + 256;
  const int maxst = S == 16 ? 4 : 2;
  *nstage = 0;
  for (int ns = maxst; ns >= 2; --ns)
    if (ns * stage + fixed <= 160 * 1024) {
      *nstage = ns;
      break;
    }
  *lds = *nstage * stage + fixed;
  return *nstage >= 2;
}

hipError_t grad_mfma_launch(int loss, const Segment* segs, const Task* tasks, int ntasks, int R, const float* beta,
                            float* slab, int ld, hipStream_t st, const int* gate) {
  if (R < 1 || R > 16 || ntasks % R) return hipErrorInvalidValue;
  int rows = 0, pieces = 0, nstage = 0;
  size_t lds = 0;
  if (!mfma_geometry(ld, &rows, &pieces, &nstage, &lds)) return hipErrorInvalidValue;
  const bool pack = R <= 4 && g_mfma_pack;
  if (pack && (g_mfma_stream == 3 || g_mfma_stream == 4) && rows == 32 && g_mfma_probe != 2) {  // (ld <= 1024)
    auto kern = g_mfma_stream == 3 ? (loss == kLogistic ? grad_vring_mfma<kLogistic, 2> : grad_vring_mfma<kLeastSquares, 2>)
                                   : (loss == kLogistic ? grad_vring_mfma<kLogistic, 3> : grad_vring_mfma<kLeastSquares, 3>);
    constexpr int vlds = 2 * (kMfNW * kVrPieces * 1024 + 256) + kMfNW * 16 * 32 * 4 + 16 * 32 * 2;
    static_assert(vlds <= 160 * 1024, "two stage buffers + partial Z + residuals");
    const hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                              hipFuncAttributeMaxDynamicSharedMemorySize, vlds);
    if (ea != hipSuccess) return ea;
    hipLaunchKernelGGL(kern, dim3(ntasks / R), dim3(64 * kMfNW), vlds, st, segs, tasks, beta, slab, ld, R, gate,
                       g_mfma_probe);
    return hipGetLastError();
  }
  auto pick = [&](auto p32l, auto p32q, auto p16l, auto p16q) {
    return rows == 32 ? (loss == kLogistic ? p32l : p32q) : (loss == kLogistic ? p16l : p16q);
  };
  auto kern = pack ? pick(grad_staged_mfma<kLogistic, 32, true>, grad_staged_mfma<kLeastSquares, 32, true>,
                          grad_staged_mfma<kLogistic, 16, true>, grad_staged_mfma<kLeastSquares, 16, true>)
                   : pick(grad_staged_mfma<kLogistic, 32, false>, grad_staged_mfma<kLeastSquares, 32, false>,
                          grad_staged_mfma<kLogistic, 16, false>, grad_staged_mfma<kLeastSquares, 16, false>);
  const hipError_t ea = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                            hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds));
  if (ea != hipSuccess) return ea;
  hipLaunchKernelGGL(kern, dim3(ntasks / R), dim3(64 * kMfNW), lds, st, segs, tasks, beta, slab, ld, R, pieces,
                     nstage, gate, g_mfma_probe);
  return hipGetLastError();
}

}  // namespace eh
