// Worker gradient for sparse (one-hot CSR) design matrices — K4 of SURVEY §2.8, deterministic.
//
// Reference: the real datasets (amazon / covtype / kc_house / dna) are scipy CSR matrices whose
// values are all 1.0 (ref src/arrange_real_data.py one-hot encoders); every worker evaluates
// X_current.dot(beta) and X_current.T.dot(r) over its (s+1) partitions with scipy
// (ref src/replication.py:63-68, src/coded.py:43-46), so co-located replicas of a partition
// repeat the same work.
//
// MI355X design.  Every DISTINCT local partition p is processed once with coefficient 1:
//   pass 1 (rows): u_r = residual(x_r . beta, y_r, 1) for every distinct row r.  ELL layout
//     (constant nnz per row, every one-hot dataset): idx column-major [m][rows], 16-bit offsets into
//     feature k's category window [lo_k, lo_k + 2^16) when every window fits (half the bytes of
//     int32 columns), a row pair per thread gathering beta from LDS when it fits (else one row per
//     thread, beta from L2); CSR: a 16-lane group per row.
//   pass 2 (columns): g_p = X_p^T u_p from a CSC twin of each partition (row indices sorted by
//     (column, row)), cut into 4096-row sub-blocks and 512-entry tiles.  A 1024-thread workgroup
//     stages one sub-block's residuals in LDS and takes 16 of its tiles, one wave each, 8 entries
//     per lane.  The row indices' top bit flags every run start (first entry of a column or of the
//     tile): the segmented sums restart at the flags -- a sequential sum over the lane's 8 entries,
//     then an affine scan of (continues, sum) over the 64 lanes on DPP -- and each run's sum is
//     compacted in LDS by run index and written to the run's column (the tile's run list).  A column
//     crossing tiles leaves its first part in tail[t1] and its later parts in head[t], added in tile
//     order: by the workgroup itself from LDS when its chunk of tiles ends on a column boundary (the
//     default: chunks sized to one dispatch round of the chip, a wave looping over its tiles with the
//     next one in flight), else by pass 3 (csc_spans); the sub-block sums are added per partition
//     inside the encoding (a naive plan without sub-blocks writes its messages directly).
//   encode (encode.hip): G[message] = sum_p coef(message, p) g_p in a fixed order -- the label
//     encoding is linear in the coefficient (residual(z, y, c) = c residual(z, y, 1)), so one
//     read of a partition feeds every co-located replica with its own coefficient.
// No float atomics anywhere: the gradient is bitwise reproducible from run to run (the old column
// passes added into g with atomics: profiles/round3/suite_nt, round-3 verdict Weak #3).
#include <algorithm>
#include <climits>
#include <type_traits>

#include "common.h"
#include "launchers.h"

namespace eh {

namespace {

constexpr int kTileEntries = 512;  // one wave: 64 lanes x 8 entries
constexpr int kSpanHead = 1, kSpanTail = 2;

// ---- pass 1: rows -------------------------------------------------------------------------------
// A row's fields are processed KB at a time: the KB index loads (HBM) of the next batch are issued
// before the KB beta gathers (L2) of this one, so a thread waits about one HBM and one L2 latency per
// batch instead of per four fields (covtype's 55 fields: 14 dependent HBM + L2 steps per thread were
// 38 us, profiles/round4/r4g).  Past the last field the loads are clamped to it and masked out; the
// sums stay in four chains z[k % 4] in field order (the old order, bitwise).
template <typename A, int LOSS, bool IDX16, bool VALS>
__global__ void __launch_bounds__(256) ell_rows(const SparseArgs a, const A* __restrict__ beta, const int* gate) {
  constexpr int KB = 16;
  if (gate_closed(gate)) return;
  const long long row = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (row >= a.nrows) return;
  const long long n = a.ell_ld;  // row stride of the [m][rows] index / value arrays
  const int m = a.m;
  const A* __restrict__ vals = static_cast<const A*>(a.vals);
  A z[4] = {A(0), A(0), A(0), A(0)};
  auto idx = [&](int kk) -> int {
    if constexpr (IDX16)
      return static_cast<int>(__builtin_nontemporal_load(static_cast<const unsigned short*>(a.ell_idx) +
                                                         static_cast<long long>(kk) * n + row));
    else
      return __builtin_nontemporal_load(static_cast<const int*>(a.ell_idx) + static_cast<long long>(kk) * n + row);
  };
  int cn[KB];
#pragma unroll
  for (int u = 0; u < KB; ++u) cn[u] = idx(min(u, m - 1));
  for (int k0 = 0; k0 < m; k0 += KB) {
    int c[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) c[u] = (IDX16 ? a.lo[min(k0 + u, m - 1)] : 0) + cn[u];
#pragma unroll
    for (int u = 0; u < KB; ++u) cn[u] = idx(min(k0 + KB + u, m - 1));  // next batch in flight
    A bv[KB], v[KB];
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      bv[u] = beta[c[u]];
      v[u] = VALS ? vals[static_cast<long long>(min(k0 + u, m - 1)) * n + row] : A(1);
    }
#pragma unroll
    for (int u = 0; u < KB; ++u)
      if (k0 + u < m) z[u & 3] = fma(v[u], bv[u], z[u & 3]);
  }
  const A zz = (z[0] + z[1]) + (z[2] + z[3]);
  static_cast<A*>(a.u)[row] = residual<LOSS, A>(zz, static_cast<const A*>(a.y)[row], A(1));
}

// beta staged in LDS when it fits (d * sizeof(A) <= kEllLdsBytes: covtype's 15509 columns are 124 KB
// fp64).  Gathered from global memory, each 8-byte beta read pulled a 128-byte L2 line into a 32 KB L1
// that the fields' windows (55 per row) keep thrashing: 21.8M gathers, ~2.8 GB of L2 -> L1 traffic,
// 38-41 us (profiles/round4/r4g, r4i).  From LDS they cost a few cycles.  One 1024-thread workgroup per
// CU (the LDS copy of beta is per workgroup).
//
// A thread takes a PAIR of adjacent rows: the [m][rows] arrays have an even row stride (ops/grad.py
// pads them), so one 4-byte load brings both rows' 16-bit offsets of a field (8 bytes of int32
// columns, 2 values) -- half the load instructions of a row per thread, twice the bytes each.  The
// next batch of fields (or the next pair's first batch) is in flight while this one is gathered, and
// the first batch is issued before beta is staged; the staging itself issues all of a thread's
// loads (16-byte vectors) before its first LDS store.
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kEllLdsBytes = 148 * 1024;
constexpr int kEllMaxFields = 1024;
constexpr int kEllStageVecs = (kEllLdsBytes / 16 + 1023) / 1024;  // 16-byte staging loads per thread

template <typename A, int LOSS, bool IDX16, bool VALS>
__global__ void __launch_bounds__(1024) ell_rows_lds(const SparseArgs a, const A* __restrict__ beta, const int* gate) {
  // fields per batch: two batches (this one and the next) of loads stay within the 64 VGPRs the compiler
  // gives a 1024-thread workgroup, no spills.  (28 fields per batch -- covtype's 55 in two dependent round
  // trips instead of four -- spilled to scratch and took 29.7 vs 17.1 us, also with __launch_bounds__(1024, 1).)
  constexpr int KB = VALS ? 4 : IDX16 ? 16 : 8;
  using IW = std::conditional_t<IDX16, unsigned int, i32x2>;                    // a field of a row pair
  using V2 = std::conditional_t<sizeof(A) == 8, f64x2, f32x2>;                   // its two values
  using V4 = std::conditional_t<sizeof(A) == 8, f64x2, f32x4>;                   // a 16-byte staging vector
  extern __shared__ __attribute__((aligned(16))) unsigned char ell_lds[];
  A* sb = reinterpret_cast<A*>(ell_lds);
  __shared__ int slo[kEllMaxFields];  // the fields' window starts (idx16), read per lane from LDS
  if (gate_closed(gate)) return;
  const long long n = a.nrows, ld = a.ell_ld;
  const int m = a.m;
  const long long npair = (n + 1) >> 1;
  const long long stride = static_cast<long long>(gridDim.x) * blockDim.x;
  const IW* __restrict__ idx = static_cast<const IW*>(a.ell_idx);  // [m][ld / 2] row pairs
  const V2* __restrict__ vals = static_cast<const V2*>(a.vals);
  const long long ldp = ld >> 1;
  auto load = [&](IW (&w)[KB], V2 (&v)[KB], long long q, int k0) {
    const long long qq = min(q, npair - 1);  // (past the last pair: a valid, unused address)
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const long long o = static_cast<long long>(min(k0 + u, m - 1)) * ldp + qq;
      w[u] = __builtin_nontemporal_load(idx + o);
      if constexpr (VALS) v[u] = __builtin_nontemporal_load(vals + o);
    }
  };
  long long q = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  IW w[KB];
  V2 v[KB];
  load(w, v, q, 0);  // in flight while beta is staged
  {  // stage beta (and the window starts): every load of this thread in flight before its stores
    const int nv = a.d * static_cast<int>(sizeof(A)) / 16;
    const V4* __restrict__ bv = reinterpret_cast<const V4*>(beta);
    V4 t[kEllStageVecs];
#pragma unroll
    for (int j = 0; j < kEllStageVecs; ++j) {
      const int i = threadIdx.x + j * 1024;
      if (i < nv) t[j] = bv[i];
    }
    int lo = 0;
    if (IDX16 && static_cast<int>(threadIdx.x) < m) lo = a.lo[threadIdx.x];
    const int tail0 = nv * 16 / static_cast<int>(sizeof(A));
    A tl = A(0);
    if (static_cast<int>(threadIdx.x) < a.d - tail0) tl = beta[tail0 + threadIdx.x];
#pragma unroll
    for (int j = 0; j < kEllStageVecs; ++j) {
      const int i = threadIdx.x + j * 1024;
      if (i < nv) reinterpret_cast<V4*>(sb)[i] = t[j];
    }
    if (static_cast<int>(threadIdx.x) < a.d - tail0) sb[tail0 + threadIdx.x] = tl;
    if (IDX16 && static_cast<int>(threadIdx.x) < m) slo[threadIdx.x] = lo;
  }
  __syncthreads();
  for (; q < npair; q += stride) {
    A z[4] = {A(0), A(0), A(0), A(0)}, y[4] = {A(0), A(0), A(0), A(0)};
    for (int k0 = 0; k0 < m; k0 += KB) {
      IW wn[KB];
      V2 vn[KB];
      if (k0 + KB < m) load(wn, vn, q, k0 + KB);  // the next batch, or the next pair's first
      else load(wn, vn, q + stride, 0);
#pragma unroll
      for (int u = 0; u < KB; ++u)
        if (k0 + u < m) {
          const int lo = IDX16 ? slo[k0 + u] : 0;
          int c0, c1;
          if constexpr (IDX16) {
            c0 = static_cast<int>(w[u] & 0xffffu);
            c1 = static_cast<int>(w[u] >> 16);
          } else {
            c0 = w[u].x;
            c1 = w[u].y;
          }
          z[u & 3] = fma(VALS ? v[u].x : A(1), sb[lo + c0], z[u & 3]);
          y[u & 3] = fma(VALS ? v[u].y : A(1), sb[lo + c1], y[u & 3]);
        }
#pragma unroll
      for (int u = 0; u < KB; ++u) {
        w[u] = wn[u];
        if constexpr (VALS) v[u] = vn[u];
      }
    }
    const long long r = 2 * q;
    const A zz = (z[0] + z[1]) + (z[2] + z[3]);
    static_cast<A*>(a.u)[r] = residual<LOSS, A>(zz, static_cast<const A*>(a.y)[r], A(1));
    if (r + 1 < n) {
      const A yy = (y[0] + y[1]) + (y[2] + y[3]);
      static_cast<A*>(a.u)[r + 1] = residual<LOSS, A>(yy, static_cast<const A*>(a.y)[r + 1], A(1));
    }
  }
}

template <typename A, int LOSS, int G>
__global__ void __launch_bounds__(256) csr_rows(const SparseArgs a, const A* __restrict__ beta, const int* gate) {
  if (gate_closed(gate)) return;
  const long long gid = static_cast<long long>(blockIdx.x) * blockDim.x + threadIdx.x;
  const long long row = gid / G;
  const int sub = threadIdx.x % G;
  if (row >= a.nrows) return;  // whole group exits together (G divides 64)
  // one-hot rows (the same nnz in every row): the row's entries start at row * nnz, one dependent load less
  const long long b = a.csr_fixed ? row * a.csr_fixed : a.row_ptr[row];
  const long long e = a.csr_fixed ? b + a.csr_fixed : a.row_ptr[row + 1];
  const A* __restrict__ vals = static_cast<const A*>(a.vals);
  A z = A(0);
  for (long long q = b + sub; q < e; q += G) z = fma(vals ? vals[q] : A(1), beta[a.col_idx[q]], z);
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) z += __shfl_xor(z, off, G);
  if (sub == 0) static_cast<A*>(a.u)[row] = residual<LOSS, A>(z, static_cast<const A*>(a.y)[row], A(1));
}

// ---- pass 2: CSC tiles, one wave per 512-entry tile ---------------------------------------------
// Row indices carry a run-start flag in their top bit (bit 15 of 16-bit rows, bit 31 of 32-bit ones):
// set on the first entry of every column and of every tile (ops/grad.py csc_tables).  Tile t's
// entries are crow[512 t, 512 t + 512) (every partition is padded to whole tiles).
template <bool ROW16>
__device__ __forceinline__ unsigned tile_rows(const SparseArgs& a, int t, int (&rows)[8]) {
  const int lane = threadIdx.x & 63;
  unsigned fl = 0;  // bit i: entry 8 * lane + i starts a run
  if constexpr (ROW16) {
    const auto rs = make_rsrc(static_cast<const unsigned short*>(a.crow) + static_cast<long long>(t) * kTileEntries,
                              2 * kTileEntries);
    const uint4 r4 = buf_load16<uint4>(rs, 16 * lane);
    const unsigned int rw[4] = {r4.x, r4.y, r4.z, r4.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rows[2 * i] = static_cast<int>(rw[i] & 0x7fffu);
      rows[2 * i + 1] = static_cast<int>((rw[i] >> 16) & 0x7fffu);
      fl |= ((rw[i] >> 15) & 1u) << (2 * i);
      fl |= (rw[i] >> 31) << (2 * i + 1);
    }
  } else {
    const auto rs = make_rsrc(static_cast<const int*>(a.crow) + static_cast<long long>(t) * kTileEntries,
                              4 * kTileEntries);
    const int4 x = buf_load16<int4>(rs, 32 * lane), y = buf_load16<int4>(rs, 32 * lane + 16);
    const int r[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      rows[i] = r[i] & 0x7fffffff;
      fl |= (static_cast<unsigned>(r[i]) >> 31) << i;
    }
  }
  return fl;
}

template <typename A, bool VALS>
__device__ __forceinline__ void tile_vals(const SparseArgs& a, int t, A (&cv)[8]) {
  if constexpr (VALS) {
    const int lane = threadIdx.x & 63;
    const auto vrs = make_rsrc(static_cast<const A*>(a.cvals) + static_cast<long long>(t) * kTileEntries,
                               kTileEntries * static_cast<int>(sizeof(A)));
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = buf_load_scalar<A>(vrs, (8 * lane + i) * static_cast<int>(sizeof(A)));
  }
}

// Wave exclusive prefix of the lane totals `run` (cl: this lane's inclusive counts)
__device__ __forceinline__ int wave_before(int run) {
  const int lane = threadIdx.x & 63;
  int incl = run;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int vv = __shfl_up(incl, off, 64);
    if (lane >= off) incl += vv;
  }
  return incl - run;
}

// The tile's tail end, shared by both column passes: mask the padding, then the segmented sums of
// the 8 entries per lane keyed by column, each run written once (Gs, or head / tail when the column
// crosses tiles).  key[i] is the column of entry 8 * lane + i; v[i] its gathered residual.
template <typename A, bool VALS>
__device__ __forceinline__ void tile_finish(const SparseArgs& a, int t, int p, int n, int c0, int flags,
                                            const int (&key)[8], A (&v)[8], const A (&cv)[8]) {
  const int lane = threadIdx.x & 63;
  // mask the padding
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const bool ok = 8 * lane + i < n;
    A x = ok ? v[i] : A(0);
    if constexpr (VALS) x *= ok ? cv[i] : A(0);
    v[i] = x;
  }
  // segmented sums: sequential inside the lane, then over the lanes
  A s[8];
  s[0] = v[0];
#pragma unroll
  for (int i = 1; i < 8; ++i) s[i] = key[i] == key[i - 1] ? s[i - 1] + v[i] : v[i];
  const int prev_last = __shfl_up(key[7], 1, 64);
  // affine scan x_l = g_l * x_{l-1} + b_l: g_l = 1 iff the whole lane continues the previous lane's key
  int g = (lane > 0 && key[0] == key[7] && prev_last == key[0]) ? 1 : 0;
  A b = s[7];
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const A bp = __shfl_up(b, off, 64);
    const int gp = __shfl_up(g, off, 64);
    if (lane >= off) {
      b = g ? b + bp : b;
      g = g & gp;
    }
  }
  // carry into this lane's first run: the running sum of that key up to the previous lane's end
  const A prev_run = __shfl_up(b, 1, 64);
  const A carry = (lane > 0 && prev_last == key[0]) ? prev_run : A(0);
  const int next_first = __shfl_down(key[0], 1, 64);
  A* __restrict__ gout = static_cast<A*>(a.Gs) + static_cast<long long>(p) * a.ld;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int q = 8 * lane + i;
    if (q >= n) break;
    const int kn = i < 7 ? key[i + 1] : next_first;
    if (q != n - 1 && kn == key[i]) continue;  // not a run end
    const A val = key[i] == key[0] ? s[i] + carry : s[i];
    const bool has_head = key[i] == c0 && (flags & kSpanHead);  // the run reaches back into earlier tiles
    const bool has_tail = q == n - 1 && (flags & kSpanTail);    // the run goes on in later tiles
    if (has_head) static_cast<A*>(a.head)[t] = val;
    if (has_tail) static_cast<A*>(a.tail)[t] = val;
    if (!has_head && !has_tail) gout[key[i]] = val;
  }
}

// Walked boundaries (one partition = one sub-block, residuals gathered from global memory): the wave
// finds every entry's column from the partition's column pointers -- an integer count in LDS, then a
// scan.  `gather(p, rows, v)` fills v[i] = u[rows[i]].
template <typename A, bool ROW16, bool VALS, typename Gather>
__device__ __forceinline__ void tile_pass(const SparseArgs& a, int t, int* __restrict__ cw, Gather gather) {
  const int lane = threadIdx.x & 63;
  const int4 td = a.tiles[t];
  const int p = td.x, base = td.y, c0 = td.z, flags = td.w;
  const int n = min(kTileEntries, a.part_nnz[p] - base);
  const int* __restrict__ cp = a.col_ptr + static_cast<long long>(p) * (a.d + 1);
  // 0. this lane's 8 entries first -- row indices, values, the gathered residuals -- through buffer
  //    descriptors (vmcnt only: the LDS waits of the boundary walk below do not wait for them).
  //    Entries past n are the partition's zero padding (row 0), masked in tile_finish.
  int rows[8];
  tile_rows<ROW16>(a, t, rows);
  A cv[8];
  tile_vals<A, VALS>(a, t, cv);
  A v[8];
  gather(p, rows, v);
  // 1. column boundaries inside the tile: cnt[q] = number of columns c > c0 starting at base + q
  //    (empty columns stack on the next non-empty one's start); integer LDS adds, order-free
#pragma unroll
  for (int i = 0; i < kTileEntries / 64; ++i) cw[i * 64 + lane] = 0;
  __builtin_amdgcn_wave_barrier();
  for (int c = c0 + 1 + lane;; c += 64) {
    const bool in = c <= a.d && cp[min(c, a.d)] < base + n;
    if (in) atomicAdd(&cw[cp[c] - base], 1);
    if (__ballot(in) == 0) break;  // column starts are monotone: none further inside
  }
  __builtin_amdgcn_wave_barrier();
  // 2. the column of each of this lane's 8 entries: c0 + inclusive prefix of cnt
  int cl[8];
  int run = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    run += cw[8 * lane + i];
    cl[i] = run;
  }
  const int before = wave_before(run);
  int key[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) key[i] = c0 + before + cl[i];
  tile_finish<A, VALS>(a, t, p, n, c0, flags, key, v, cv);
}

// One wave per tile, residuals gathered from global memory (one partition = one sub-block).
template <typename A, bool ROW16, bool VALS>
__global__ void __launch_bounds__(256) csc_tiles(const SparseArgs a, const int* gate) {
  __shared__ int cnt[4][kTileEntries];
  if (gate_closed(gate)) return;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= a.ntiles) return;  // wave-uniform; only wave barriers below
  tile_pass<A, ROW16, VALS>(a, t, cnt[threadIdx.x >> 6], [&](int p, const int (&rows)[8], A (&v)[8]) {
    const long long r0 = a.part_row0[p];
    const long long ubytes = (a.nrows - r0) * static_cast<long long>(sizeof(A));
    const auto urs = make_rsrc(static_cast<const A*>(a.u) + r0, static_cast<int>(min(ubytes, static_cast<long long>(INT_MAX))));
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = buf_load_scalar<A>(urs, rows[i] * static_cast<int>(sizeof(A)));
  });
}

// ---- wave scans on DPP: row_shr 1 / 2 / 4 / 8 inside each row of 16 lanes, then row_bcast 15 / 31
// across rows (GFX9 DPP; gfx950 keeps it) -- one VALU op per step, no LDS round trip.  A lane with no
// source in a step takes `old`, the operator's identity.
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i(int old, int x) {
  return __builtin_amdgcn_update_dpp(old, x, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS, typename A>
__device__ __forceinline__ A dpp_a(A old, A x) {
  if constexpr (sizeof(A) == 8) {
    const long long xi = __builtin_bit_cast(long long, x), oi = __builtin_bit_cast(long long, old);
    const unsigned lo = static_cast<unsigned>(dpp_i<CTRL, ROWS>(static_cast<int>(oi), static_cast<int>(xi)));
    const unsigned hi = static_cast<unsigned>(dpp_i<CTRL, ROWS>(static_cast<int>(oi >> 32), static_cast<int>(xi >> 32)));
    return __builtin_bit_cast(A, (static_cast<unsigned long long>(hi) << 32) | lo);
  } else {
    return __builtin_bit_cast(A, dpp_i<CTRL, ROWS>(__builtin_bit_cast(int, old), __builtin_bit_cast(int, x)));
  }
}
__device__ __forceinline__ int wave_incl_sum(int x) {
  x += __builtin_amdgcn_mov_dpp(x, 0x111, 0xf, 0xf, true);  // full rows: bound_ctrl's 0, no identity to set up
  x += __builtin_amdgcn_mov_dpp(x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_mov_dpp(x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_mov_dpp(x, 0x118, 0xf, 0xf, true);
  x += dpp_i<0x142, 0xa>(0, x);  // row_bcast:15 -> rows 1, 3
  x += dpp_i<0x143, 0xc>(0, x);  // row_bcast:31 -> rows 2, 3
  return x;
}
// DPP move over full rows with bound_ctrl: a lane without a source reads 0, so no old value is set up
// (one v_mov_b32_dpp per dword instead of a v_mov of the identity and the DPP move)
template <int CTRL, typename A>
__device__ __forceinline__ A dpp_a0(A x) {
  if constexpr (sizeof(A) == 8) {
    const unsigned long long xi = __builtin_bit_cast(unsigned long long, x);
    const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_mov_dpp(static_cast<int>(xi), CTRL, 0xf, 0xf, true));
    const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_mov_dpp(static_cast<int>(xi >> 32), CTRL, 0xf, 0xf, true));
    return __builtin_bit_cast(A, (static_cast<unsigned long long>(hi) << 32) | lo);
  } else {
    return __builtin_bit_cast(A, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xf, 0xf, true));
  }
}
// h |= h of the DPP source lane, for h in {0.0, 1.0}: the high dword carries the whole value (the low one
// is 0 for both), and an unsigned max with identity 0 folds into one v_max_u32_dpp
template <int CTRL, int ROWS, typename A>
__device__ __forceinline__ A dpp_or01(A h) {
  if constexpr (sizeof(A) == 8) {
    const unsigned hi = static_cast<unsigned>(__builtin_bit_cast(unsigned long long, h) >> 32);
    const unsigned hp = static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(hi), CTRL, ROWS, 0xf, ROWS == 0xf));
    return __builtin_bit_cast(A, static_cast<unsigned long long>(max(hi, hp)) << 32);
  } else {
    const unsigned u = __builtin_bit_cast(unsigned, h);
    const unsigned up = static_cast<unsigned>(__builtin_amdgcn_update_dpp(0, static_cast<int>(u), CTRL, ROWS, 0xf, ROWS == 0xf));
    return __builtin_bit_cast(A, max(u, up));
  }
}
// inclusive scan of x_l = g_l x_{l-1} + b_l over the lanes, carried as h = 1 - g (1: this lane's run, or one
// between it and the source lane, starts a new segment) so every lane without a source holds the
// identity (h = 0, b = 0) that bound_ctrl supplies.  b + g bp is fma(g, bp, b) with g = 1 - h exactly 0 / 1:
// exactly b + bp or b, one op where a select of two doubles took three.
template <int CTRL, int ROWS, typename A>
__device__ __forceinline__ void affine_step(A& h, A& b) {
  A bp;
  if constexpr (ROWS == 0xf) bp = dpp_a0<CTRL>(b);
  else bp = dpp_a<CTRL, ROWS>(A(0), b);
  b = fma(A(1) - h, bp, b);
  h = dpp_or01<CTRL, ROWS>(h);
}
template <typename A>
__device__ __forceinline__ void wave_affine_scan(A h, A& b) {
  affine_step<0x111, 0xf>(h, b);
  affine_step<0x112, 0xf>(h, b);
  affine_step<0x114, 0xf>(h, b);
  affine_step<0x118, 0xf>(h, b);
  affine_step<0x142, 0xa>(h, b);
  affine_step<0x143, 0xc>(h, b);
}

constexpr int kWgWaves = 16;     // waves per column-pass workgroup
constexpr int kMaxWgTiles = 128;  // tiles per workgroup chunk (ops/grad.py SparseGradPlan.WG_TILES <= this):
                                 // wave w takes the chunk's tiles w, w + 16, ...
constexpr int kStageRegs = 4;    // staged residuals per thread: 4096 rows per sub-block (32 KB fp64 / 16 KB fp32);
                                 // 8 (8192 rows) for merged FRC / AGC units (csc_tiles_lds UNITS)
constexpr int kRunCap = 128;     // runs per tile compacted in LDS (covtype: 33 on average, 0.7 % of tiles above)

// A tile's 8 row indices per lane as loaded (16-bit rows: one 16-byte vector, 32-bit rows: two), decoded
// only when the tile is summed -- so the next tile's loads stay in flight meanwhile.
struct TileRaw {
  uint4 x, y;
};
template <bool ROW16>
__device__ __forceinline__ void tile_rows_raw(const SparseArgs& a, int t, TileRaw& r) {
  const int lane = threadIdx.x & 63;
  if constexpr (ROW16) {
    const auto rs = make_rsrc(static_cast<const unsigned short*>(a.crow) + static_cast<long long>(t) * kTileEntries,
                              2 * kTileEntries);
    r.x = buf_load16<uint4>(rs, 16 * lane);
  } else {
    const auto rs = make_rsrc(static_cast<const int*>(a.crow) + static_cast<long long>(t) * kTileEntries,
                              4 * kTileEntries);
    r.x = buf_load16<uint4>(rs, 32 * lane);
    r.y = buf_load16<uint4>(rs, 32 * lane + 16);
  }
}
template <bool ROW16>
__device__ __forceinline__ unsigned tile_rows_decode(const TileRaw& r, int (&rows)[8]) {
  unsigned fl = 0;  // bit i: entry 8 * lane + i starts a run
  if constexpr (ROW16) {
    const unsigned int rw[4] = {r.x.x, r.x.y, r.x.z, r.x.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      rows[2 * i] = static_cast<int>(rw[i] & 0x7fffu);
      rows[2 * i + 1] = static_cast<int>((rw[i] >> 16) & 0x7fffu);
    }
    // the 8 flag bits (bit 15 / 31 of each dword): v_perm_b32 gathers the high byte of every entry (flags at
    // bits 7, 15, 23, 31), the two words' flags interleave to bits 8k and 8k + 4, and one multiply moves
    // entry e's bit to 24 + e (its partial products land on distinct bits: no carries)
    const unsigned p01 = __builtin_amdgcn_perm(rw[1], rw[0], 0x07050301u);
    const unsigned p23 = __builtin_amdgcn_perm(rw[3], rw[2], 0x07050301u);
    const unsigned q = ((p01 >> 7) & 0x01010101u) | ((p23 >> 3) & 0x10101010u);
    fl = (q * 0x01020408u) >> 24;
  } else {
    const unsigned int rw[8] = {r.x.x, r.x.y, r.x.z, r.x.w, r.y.x, r.y.y, r.y.z, r.y.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      rows[i] = static_cast<int>(rw[i] & 0x7fffffffu);
      fl |= (rw[i] >> 31) << i;
    }
  }
  return fl;
}

// Row-blocked column pass: a 1024-thread workgroup takes a chunk of up to kMaxWgTiles tiles of ONE
// sub-block (a.wg) and first copies that sub-block's residuals into LDS (coalesced), so every gather is
// an LDS read.  From global memory each 8-byte gather pulled a 128-byte L2 line into L1 with no reuse
// (rows of a column are spread over the partition): covtype's 21.8M gathers moved ~2.8 GB L2 -> L1,
// 88-92 us (profiles/round4/r4g, r4i).  Each wave sums the chunk's tiles w, w + 16, ... with the next
// tile's rows, values and key in flight while it sums the current one; a chunk of several tiles per
// wave also spreads the 32 KB residual staging over more entries (16 tiles: 16 KB of row indices per
// 32 KB staged).
//
// Keyed runs: the row indices' top bit flags every run start (first entry of a column or of the
// tile), so the segmented sums need no column keys at all -- the flags are the segment boundaries --
// and a run's column is looked up only once, when its sum is written: run r of the tile is column
// a.runs[tk.x + r].  The run sums are compacted into LDS by run index and written by lane r % 64,
// consecutive columns side by side.  (The column-pointer walk before it waited on two more dependent
// loads per workgroup and ran ~420 VALU instructions per tile: the pass was VALU-bound at ~70 % busy,
// profiles/round4/r4y.)
//
// Column-aligned chunks (LOCAL, a.wspan_ptr set): no column leaves the workgroup's chunk, so the tiles'
// head and tail sums stay in LDS and, after one more block barrier, the workgroup adds its crossing
// columns itself (tail of the first tile + the heads of the later ones, in tile order: csc_spans'
// order).  LOCAL is a template parameter so the head / tail stores are LDS or global stores (a pointer
// that may be either is a flat store, which every later wait has to count on both counters).
// UNITS: merged FRC / AGC units (SparseArgs::dst) -- 8192-row sub-blocks and every sum stored into each
// of the unit's message rows; a compile-time variant, so the single-row form keeps its instruction
// stream (a run-time destination loop in the tile loop cost 1.4-5 us per launch on every sparse shape:
// profiles/round6/sparse/tree_ab.txt)
template <typename A, bool ROW16, bool VALS, bool LOCAL, bool UNITS>
__global__ void __launch_bounds__(1024, 2) csc_tiles_lds(const SparseArgs a, const int* gate) {
  __shared__ int run_col[kWgWaves][kRunCap];
  __shared__ A run_val[kWgWaves][kRunCap];
  __shared__ A s_head[LOCAL ? kMaxWgTiles : 1], s_tail[LOCAL ? kMaxWgTiles : 1];
  extern __shared__ __attribute__((aligned(16))) unsigned char usub_raw[];
  A* su = reinterpret_cast<A*>(usub_raw);
  if (gate_closed(gate)) return;
  const int4 wd = a.wg[blockIdx.x];  // (first row of the sub-block, first tile, tiles, rows)
  // LOCAL: this workgroup's crossing columns (at most one per tile boundary: < kMaxWgTiles of them, one
  // per thread), loaded now so their latency hides behind the tiles instead of ending the workgroup
  int4 my_span = make_int4(0, 0, 0, -1);
  if constexpr (LOCAL) {
    const int s0 = a.wspan_ptr[blockIdx.x], s1 = a.wspan_ptr[blockIdx.x + 1];
    if (static_cast<int>(threadIdx.x) < s1 - s0) my_span = a.wspan[s0 + threadIdx.x];
  }
  // wave-uniform in SGPRs: the tile's descriptor is a scalar load and its buffer descriptors need no
  // waterfall loops (a VGPR-held base costs ~60 VALU + 70 SALU instructions of readfirstlane loops)
  const int w = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  const int last = max(wd.z - 1, 0);
  // the wave's first tile in flight while the sub-block's residuals are staged (a wave past the
  // chunk's tiles only stages)
  TileRaw raw;
  A cv[8];
  int4 tk;
  {
    const int t = wd.y + min(w, last);
    tile_rows_raw<ROW16>(a, t, raw);
    tile_vals<A, VALS>(a, t, cv);
    tk = a.tkeys[t];  // (first run, n | runs << 10 | span flags << 20, sub-block, first column)
  }
  const A* __restrict__ ug = static_cast<const A*>(a.u) + wd.x;
  constexpr int STAGE = UNITS ? 2 * kStageRegs : kStageRegs;
  A st[STAGE];
#pragma unroll
  for (int j = 0; j < STAGE; ++j) {
    const int i = threadIdx.x + j * static_cast<int>(blockDim.x);
    st[j] = i < wd.w ? ug[i] : A(0);
  }
#pragma unroll
  for (int j = 0; j < STAGE; ++j) {
    const int i = threadIdx.x + j * static_cast<int>(blockDim.x);
    if (i < wd.w) su[i] = st[j];
  }
  __syncthreads();
  A* __restrict__ hd = LOCAL ? s_head : static_cast<A*>(a.head) + wd.y;  // indexed by the chunk's tile
  A* __restrict__ tl = LOCAL ? s_tail : static_cast<A*>(a.tail) + wd.y;
  for (int j = w; j < wd.z; j += kWgWaves) {  // wave-uniform
    // the next tile's loads first (none past the chunk: a wave with one tile loads nothing more)
    const bool more = j + kWgWaves < wd.z;  // wave-uniform
    TileRaw raw_n = raw;
    A cv_n[8];
    int4 tk_n = tk;
    if (more) {
      const int tn = wd.y + j + kWgWaves;
      tile_rows_raw<ROW16>(a, tn, raw_n);
      tile_vals<A, VALS>(a, tn, cv_n);
      tk_n = a.tkeys[tn];
    }
    const int tky = __builtin_amdgcn_readfirstlane(tk.y);
    const int n = tky & 1023, nruns = (tky >> 10) & 1023, flags = tky >> 20;
    const int p = __builtin_amdgcn_readfirstlane(tk.z), run0 = __builtin_amdgcn_readfirstlane(tk.x);
    const bool compact = nruns <= kRunCap;  // wave-uniform
    const auto rrs = make_rsrc(a.runs + run0, 4 * nruns);
    __builtin_amdgcn_wave_barrier();  // the previous tile's run_col / run_val reads come first
    if (compact) {
      run_col[w][lane] = buf_load_scalar<int>(rrs, 4 * lane);
      run_col[w][lane + 64] = buf_load_scalar<int>(rrs, 4 * (lane + 64));
    }
    int rows[8];
    const unsigned fl = tile_rows_decode<ROW16>(raw, rows);
    // runs before this lane (the tile's first entry is always flagged; padding entries never are)
    const int cnt = __builtin_popcount(fl);
    const int before = wave_incl_sum(cnt) - cnt;
    // this lane's run ends: the entry before a flagged one, and the tile's last entry
    const unsigned long long f0 = __ballot(fl & 1u);
    const unsigned next0 = lane < 63 ? static_cast<unsigned>((f0 >> (lane + 1)) & 1ull) : 1u;
    const int q0 = 8 * lane;
    const unsigned valid = n >= q0 + 8 ? 0xffu : n > q0 ? (1u << (n - q0)) - 1u : 0u;
    unsigned ends = ((fl >> 1) | (next0 << 7)) & valid;
    if (n - 1 >= q0 && n - 1 < q0 + 8) ends |= 1u << (n - 1 - q0);
    A v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = su[rows[i]];
    if (n < kTileEntries) {  // a short tile (a sub-block's last, a chunk's cut one): padding (row 0) counts nothing
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = (valid >> i) & 1u ? v[i] : A(0);
    }
    if constexpr (VALS) {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] *= cv[i];
    }
    // segmented sums: sequential inside the lane, restarting at a flag (fma(keep, s, v) with keep 0 / 1:
    // exactly s + v or v, one op where a select of two doubles took three), then an affine scan over lanes
    A sm[8];
    sm[0] = v[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) sm[i] = fma(static_cast<A>(((fl >> i) & 1u) ^ 1u), sm[i - 1], v[i]);
    A b = sm[7];
    wave_affine_scan(fl ? A(1) : A(0), b);  // h = 0: the whole lane continues the previous lane's run
    const A prev = dpp_a0<0x138>(b);        // wave_shr:1 -- the previous lane's running sum
    const A carry = fl & 1u ? A(0) : prev;       // into this lane's entries before its first flag
    const unsigned cmask = fl ? (fl & (0u - fl)) - 1u : 0xffu;
    // the output rows of sub-block p (wave-uniform): row p, or its shared message rows (SparseArgs::dst)
    // the output row(s) through buffer descriptors (wave-uniform, in SGPRs): a run's store is one instruction
    // on the column's 32-bit byte offset, no 64-bit address per lane (UNITS: one descriptor per message row
    // of the unit; a missing destination gets a zero-size descriptor, its stores dropped)
    const auto grs = make_rsrc(static_cast<A*>(a.Gs) + static_cast<long long>(p) * a.ld, a.ld * static_cast<int>(sizeof(A)));
    __amdgpu_buffer_rsrc_t drs[kSparseMaxDst];
    int nd = 0;  // (a unit's rows come first in its dst entry)
    if constexpr (UNITS) {
#pragma unroll
      for (int q = 0; q < kSparseMaxDst; ++q) {
        const int r = __builtin_amdgcn_readfirstlane(a.dst[p * kSparseMaxDst + q]);
        nd += r >= 0 ? 1 : 0;
        drs[q] = make_rsrc(static_cast<A*>(a.Gs) + static_cast<long long>(r >= 0 ? r : 0) * a.ld,
                           r >= 0 ? a.ld * static_cast<int>(sizeof(A)) : 0);
      }
    }
    auto put = [&](int col, A val) {
      if constexpr (UNITS) {
        const int off = col * static_cast<int>(sizeof(A));
#pragma unroll
        for (int q = 0; q < kSparseMaxDst; ++q)
          if (q < nd) buf_store(drs[q], off, val);
      } else {
        buf_store(grs, col * static_cast<int>(sizeof(A)), val);
      }
    };
    if (compact) {
      // each run end stores its lane-local sum at its run index; the one run that began in an earlier
      // lane (it ends first here, run index before - 1) then gets the carry: sm + carry, as before
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if ((ends >> i) & 1u) run_val[w][before - 1 + __builtin_popcount(fl & ((2u << i) - 1u))] = sm[i];
      if (!(fl & 1u) && ends) run_val[w][before - 1] += carry;
      __builtin_amdgcn_wave_barrier();
      for (int r = lane; r < nruns; r += 64) {
        const A val = run_val[w][r];
        const bool has_head = r == 0 && (flags & kSpanHead);            // the run reaches back into earlier tiles
        const bool has_tail = r == nruns - 1 && (flags & kSpanTail);    // the run goes on in later tiles
        if (has_head) hd[j] = val;
        if (has_tail) tl[j] = val;
        if (!has_head && !has_tail) put(run_col[w][r], val);
      }
    } else {  // many short runs: every run end writes its own sum, the column from global memory
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if ((ends >> i) & 1u) {
          const int r = before + __builtin_popcount(fl & ((2u << i) - 1u)) - 1;
          const A val = (cmask >> i) & 1u ? sm[i] + carry : sm[i];
          const bool has_head = r == 0 && (flags & kSpanHead);
          const bool has_tail = r == nruns - 1 && (flags & kSpanTail);
          if (has_head) hd[j] = val;
          if (has_tail) tl[j] = val;
          if (!has_head && !has_tail) put(buf_load_scalar<int>(rrs, 4 * r), val);
        }
    }
    if (!more) break;
    raw = raw_n;
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = cv_n[i];
    tk = tk_n;
  }
  if constexpr (!LOCAL) return;
  __syncthreads();
  if (my_span.w >= 0) {  // (sub-block, column, first tile, last tile), chunk-relative tiles
    A sum = s_tail[my_span.z];
    for (int k = my_span.z + 1; k <= my_span.w; ++k) sum += s_head[k];
    A* __restrict__ gs = static_cast<A*>(a.Gs);
    if constexpr (UNITS) {
      for (int q = 0; q < kSparseMaxDst; ++q) {
        const int r = a.dst[my_span.x * kSparseMaxDst + q];
        if (r >= 0) gs[static_cast<long long>(r) * a.ld + my_span.y] = sum;
      }
    } else {
      gs[static_cast<long long>(my_span.x) * a.ld + my_span.y] = sum;
    }
  }
}

// Sub-block sums added per partition in sub-block order: Gb[j][c] = sum_s Gs[s][c].
template <typename A>
__global__ void __launch_bounds__(256) sub_reduce(const SparseArgs a, const int* gate) {
  if (gate_closed(gate)) return;
  const int j = blockIdx.y, c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.ld) return;
  const A* __restrict__ gs = static_cast<const A*>(a.Gs);
  A s = A(0);
  for (int q = a.sub_begin[j]; q < a.sub_begin[j + 1]; ++q) s += gs[static_cast<long long>(q) * a.ld + c];
  static_cast<A*>(a.Gb)[static_cast<long long>(j) * a.ld + c] = s;
}

// ---- pass 3: columns crossing tiles (tail of the first tile + the heads of the later ones, in tile
// order) and the columns no entry of the sub-block touches, a thread each.  Within a sub-block of at
// most 4096 rows a column covers at most 9 tiles, so the walk is short (it was one wave per column
// while a partition's column could span ~70 tiles).
template <typename A>
__global__ void __launch_bounds__(256) csc_spans(const SparseArgs a, int, const int* gate) {
  if (gate_closed(gate)) return;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.nspan) {
    const int4 sp = a.span[i];  // (sub-block, column, t1, t2)
    const A* __restrict__ head = static_cast<const A*>(a.head);
    A s = static_cast<const A*>(a.tail)[sp.z];
    for (int t = sp.z + 1; t <= sp.w; t += 8) {  // eight loads in flight, added in tile order
      A h[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) h[j] = t + j <= sp.w ? head[t + j] : A(0);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (t + j <= sp.w) s += h[j];
    }
    static_cast<A*>(a.Gs)[static_cast<long long>(sp.x) * a.ld + sp.y] = s;
  } else if (i < a.nspan + a.nempty) {
    const int2 e = a.empty[i - a.nspan];
    static_cast<A*>(a.Gs)[static_cast<long long>(e.x) * a.ld + e.y] = A(0);
  }
}

}  // namespace

hipError_t grad_sparse_launch(int dtype, int loss, const SparseArgs& a, const void* beta, hipStream_t st,
                              const int* gate) {
  if (a.nrows < 0 || a.ntiles < 0 || a.d <= 0 || a.ld < a.d || !a.Gb || !a.Gs || !a.u) return hipErrorInvalidValue;
  if (a.sub_begin && a.Gs == a.Gb) return hipErrorInvalidValue;
  const dim3 block(256);
  if (a.nrows > 0) {
    const size_t blds = static_cast<size_t>(a.d) * (dtype == 0 ? 8 : 4);
    if (a.ell && blds <= static_cast<size_t>(kEllLdsBytes) && a.m <= kEllMaxFields && a.ell_ld % 2 == 0) {
      static int cus = 0;
      if (!cus) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
          cus = 256;
      }
      // (spreading covtype's 198k row pairs evenly over all 256 CUs instead of 194 full workgroups measured
      // 17.7 vs 17.0 us: the per-workgroup beta staging, not the CU count, sets the pace)
      const dim3 grid(static_cast<unsigned>(std::min<long long>(cus, ((a.nrows + 1) / 2 + 1023) / 1024)));
      auto go = [&](const void* kern) -> hipError_t {
        return blds > 64 * 1024 ? hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                      static_cast<int>(blds))
                                : hipSuccess;
      };
#define EH_ELLL(A_, L_, I_, V_)                                                                                  \
  {                                                                                                              \
    const hipError_t e = go(reinterpret_cast<const void*>(ell_rows_lds<A_, L_, I_, V_>));                        \
    if (e != hipSuccess) return e;                                                                               \
    hipLaunchKernelGGL((ell_rows_lds<A_, L_, I_, V_>), grid, dim3(1024), blds, st, a, (const A_*)beta, gate);   \
  }
#define EH_ELLV(A_, L_)                                              \
  if (a.idx16) {                                                     \
    if (a.vals) EH_ELLL(A_, L_, true, true) else EH_ELLL(A_, L_, true, false)      \
  } else {                                                           \
    if (a.vals) EH_ELLL(A_, L_, false, true) else EH_ELLL(A_, L_, false, false)    \
  }
      if (dtype == 0) {
        if (loss == kLogistic) { EH_ELLV(double, kLogistic) } else { EH_ELLV(double, kLeastSquares) }
      } else {
        if (loss == kLogistic) { EH_ELLV(float, kLogistic) } else { EH_ELLV(float, kLeastSquares) }
      }
#undef EH_ELLV
#undef EH_ELLL
    } else if (a.ell) {
      const dim3 grid(static_cast<unsigned>((a.nrows + 255) / 256));
#define EH_ELL(A_, L_)                                                                                          \
  if (a.idx16) {                                                                                                \
    if (a.vals) hipLaunchKernelGGL((ell_rows<A_, L_, true, true>), grid, block, 0, st, a, (const A_*)beta, gate);  \
    else hipLaunchKernelGGL((ell_rows<A_, L_, true, false>), grid, block, 0, st, a, (const A_*)beta, gate);       \
  } else {                                                                                                      \
    if (a.vals) hipLaunchKernelGGL((ell_rows<A_, L_, false, true>), grid, block, 0, st, a, (const A_*)beta, gate); \
    else hipLaunchKernelGGL((ell_rows<A_, L_, false, false>), grid, block, 0, st, a, (const A_*)beta, gate);      \
  }
      if (dtype == 0) {
        if (loss == kLogistic) { EH_ELL(double, kLogistic) } else { EH_ELL(double, kLeastSquares) }
      } else {
        if (loss == kLogistic) { EH_ELL(float, kLogistic) } else { EH_ELL(float, kLeastSquares) }
      }
#undef EH_ELL
    } else {
      // lanes per CSR row: 8 (16 / 8 / 4 at kc_house 13.45 / 13.2 / 13.05 us, amazon 21.4 / 21.2 / 21.7,
      // covtype 96.7 / 82.7 / 89.0: profiles/round6/sparse/csr_lanes)
      constexpr int Gs = 8;
      const dim3 grid(static_cast<unsigned>((a.nrows * Gs + 255) / 256));
      if (dtype == 0) {
        if (loss == kLogistic)
          hipLaunchKernelGGL((csr_rows<double, kLogistic, Gs>), grid, block, 0, st, a, (const double*)beta, gate);
        else
          hipLaunchKernelGGL((csr_rows<double, kLeastSquares, Gs>), grid, block, 0, st, a, (const double*)beta, gate);
      } else {
        if (loss == kLogistic)
          hipLaunchKernelGGL((csr_rows<float, kLogistic, Gs>), grid, block, 0, st, a, (const float*)beta, gate);
        else
          hipLaunchKernelGGL((csr_rows<float, kLeastSquares, Gs>), grid, block, 0, st, a, (const float*)beta, gate);
      }
    }
  }
  if (a.ntiles > 0 && a.wg) {
    const size_t ulds = static_cast<size_t>(std::max(a.u_lds, 1)) * (dtype == 0 ? 8 : 4);
    // sub-blocks of at most 4096 rows, merged units (shared rows, unblocked only) of at most 8192
    if (a.u_lds > (a.dst ? 2 : 1) * kStageRegs * 1024) return hipErrorInvalidValue;
    if (a.dst && (a.sub_begin || a.nspan || a.nempty)) return hipErrorInvalidValue;
    const dim3 grid(static_cast<unsigned>(a.nwg));
#define EH_TLDS3(A_, R_, V_, L_, S_)                                                                            \
  {                                                                                                              \
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(csc_tiles_lds<A_, R_, V_, L_, S_>),    \
                                             hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(ulds));   \
    if (e != hipSuccess) return e;                                                                               \
    hipLaunchKernelGGL((csc_tiles_lds<A_, R_, V_, L_, S_>), grid, dim3(1024), ulds, st, a, gate);                 \
  }
#define EH_TLDS2(A_, R_, V_, L_)                                   \
  {                                                                \
    if (a.dst) EH_TLDS3(A_, R_, V_, L_, true)                      \
    else EH_TLDS3(A_, R_, V_, L_, false)                           \
  }
#define EH_TLDS(A_, R_, V_)                     \
  {                                               \
    if (a.wspan_ptr) EH_TLDS2(A_, R_, V_, true)   \
    else EH_TLDS2(A_, R_, V_, false)              \
  }
#define EH_TILES(A_)                                                                    \
  if (a.row16) {                                                                        \
    if (a.cvals) EH_TLDS(A_, true, true) else EH_TLDS(A_, true, false)                   \
  } else {                                                                              \
    if (a.cvals) EH_TLDS(A_, false, true) else EH_TLDS(A_, false, false)                 \
  }
    if (dtype == 0) { EH_TILES(double) } else { EH_TILES(float) }
#undef EH_TILES
#undef EH_TLDS
#undef EH_TLDS2
#undef EH_TLDS3
  } else if (a.ntiles > 0) {
    const dim3 grid(static_cast<unsigned>((a.ntiles + 3) / 4));
#define EH_TILES(A_)                                                                                     \
  if (a.row16) {                                                                                         \
    if (a.cvals) hipLaunchKernelGGL((csc_tiles<A_, true, true>), grid, block, 0, st, a, gate);          \
    else hipLaunchKernelGGL((csc_tiles<A_, true, false>), grid, block, 0, st, a, gate);                 \
  } else {                                                                                               \
    if (a.cvals) hipLaunchKernelGGL((csc_tiles<A_, false, true>), grid, block, 0, st, a, gate);         \
    else hipLaunchKernelGGL((csc_tiles<A_, false, false>), grid, block, 0, st, a, gate);                \
  }
    if (dtype == 0) { EH_TILES(double) } else { EH_TILES(float) }
#undef EH_TILES
  }
  const int nout = a.nspan + a.nempty;
  if (nout > 0) {
    const dim3 grid(static_cast<unsigned>((nout + 255) / 256));
    if (dtype == 0) hipLaunchKernelGGL(csc_spans<double>, grid, block, 0, st, a, 0, gate);
    else hipLaunchKernelGGL(csc_spans<float>, grid, block, 0, st, a, 0, gate);
  }
  if (a.sub_begin && a.nparts > 0 && !a.encode_from_subs) {  // sub-block sums -> partitions
    const dim3 grid(static_cast<unsigned>((a.ld + 255) / 256), static_cast<unsigned>(a.nparts));
    if (dtype == 0) hipLaunchKernelGGL(sub_reduce<double>, grid, block, 0, st, a, gate);
    else hipLaunchKernelGGL(sub_reduce<float>, grid, block, 0, st, a, gate);
  }
  return hipGetLastError();
}

}  // namespace eh
