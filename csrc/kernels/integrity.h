// Message integrity tags of the IPC mailbox transport (SURVEY §5.2 "per-slot generation
// counters ... a debug mode that checksums beta per round", here always on).
//
// The reference relies on MPI's per-source ordering for the reuse of msgBuffers[j] and of the
// one beta receive buffer (ref src/naive.py:66-79, :97-110).  Here a message is a put over xGMI
// followed by a release-store of a round counter in host memory; a platform or protocol bug
// that let the counter overtake the payload would silently decode stale or torn rows.  So every
// tagged put also writes, per payload row, a 16-byte tag into the receiver's tag slots:
//     { round + 1 (the counter value), sender rank, checksum of the row }
// before the counter, and the receiver recomputes the checksum over the row it actually reads
// (the master's combine / arbiter for worker messages, a verify kernel on the worker for beta).
//
// Checksum of a row of n elements of es bytes (4 or 8), element bits zero-extended to 64 bits:
//     sum_j bits_j * (2 j + 1)  (mod 2^64)
// Odd multipliers are invertible mod 2^64, so any single corrupted element changes it, an
// element moved to another column changes it, and a stale row from an earlier round changes it
// with overwhelming probability.  It is a plain sum of per-element terms: blocks and waves
// reduce it in any order with integer adds (bitwise deterministic, no float atomics).
#pragma once

#include <hip/hip_runtime.h>

namespace eh {

struct MsgTag {
  unsigned int round1;      // round + 1: the counter value the put announces
  unsigned int rank;        // sender rank
  unsigned long long sum;   // checksum of the row
};
static_assert(sizeof(MsgTag) == 16, "MsgTag is 16 bytes");

// First failed check of a pump, in host-mapped memory (written once, by one thread).
struct IntegrityErr {
  int flag;                 // 1 once filled in
  int round;                // round whose message failed
  int where;                // slot << 16 | mailbox row (worker messages), -1 for beta
  int rank_want;            // sender the receiver expected
  unsigned int round1_got;  // tag fields found
  unsigned int rank_got;
  unsigned long long sum_got;   // checksum in the tag
  unsigned long long sum_calc;  // checksum of the payload as read
};

constexpr int kMaxTagRows = 1024;  // rows of one tagged put descriptor (sender scratch / LDS sums: 8 KB)
constexpr int kMaxCheckRows = 128;  // mailbox rows one deferred check covers (= kMaxMsgs of a decode)

// The mailbox rows a round's decode read, checked AFTER the round (off the critical path: the rows
// stay intact until their ring slot is reused K >= 2 rounds later).  Passed by value to the host
// pump's check kernel; written to device memory by the arbiter for the next round's idle waves.
struct CheckList {
  int n;                          // rows
  int round;                      // the round whose messages they are
  int slot;                       // ring slot
  int es;                         // element bytes
  int ld;
  const void* row[kMaxCheckRows];
  int mrow[kMaxCheckRows];        // mailbox row (tag index within the slot); < 0: skip (a local row)
  int rank[kMaxCheckRows];        // expected sender
  const MsgTag* tags;             // this slot's tags [rows]
};

__host__ __device__ inline unsigned long long tag_term(unsigned long long bits, long long j) {
  return bits * static_cast<unsigned long long>(2 * j + 1);
}

#if defined(__HIPCC__)
// Full-wave u64 sum in VALU cross-lane moves only (DPP quad_perm xor 1 / xor 2, row_half_mirror,
// row_mirror, then gfx950's permlane16 / permlane32 swaps; the same lane pairing as
// common.h wave_allreduce_sum): no LDS crossbar round trips, every lane ends with the total.
template <int CTRL>
__device__ __forceinline__ unsigned long long dpp_u64(unsigned long long v) {
  const unsigned lo = static_cast<unsigned>(__builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<unsigned>(v)), CTRL, 0xf, 0xf, true));
  const unsigned hi = static_cast<unsigned>(__builtin_amdgcn_mov_dpp(static_cast<int>(static_cast<unsigned>(v >> 32)), CTRL, 0xf, 0xf, true));
  return (static_cast<unsigned long long>(hi) << 32) | lo;
}
template <bool ROW16>
__device__ __forceinline__ unsigned long long swap_sum_u64(unsigned long long v) {
  const unsigned l = static_cast<unsigned>(v), h = static_cast<unsigned>(v >> 32);
  const auto lo = ROW16 ? __builtin_amdgcn_permlane16_swap(l, l, false, false) : __builtin_amdgcn_permlane32_swap(l, l, false, false);
  const auto hi = ROW16 ? __builtin_amdgcn_permlane16_swap(h, h, false, false) : __builtin_amdgcn_permlane32_swap(h, h, false, false);
  return ((static_cast<unsigned long long>(hi[0]) << 32) | lo[0]) + ((static_cast<unsigned long long>(hi[1]) << 32) | lo[1]);
}
__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
  v += dpp_u64<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_u64<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_u64<0x141>(v);  // row_half_mirror
  v += dpp_u64<0x140>(v);  // row_mirror
  v = swap_sum_u64<true>(v);
  return swap_sum_u64<false>(v);
}

// Sum over the block of one u64 per thread (every thread must call it; result valid in thread 0).
// scratch: >= blockDim.x / 64 entries of LDS.
__device__ __forceinline__ unsigned long long block_sum_u64(unsigned long long v, unsigned long long* scratch) {
  v = wave_sum_u64(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  unsigned long long s = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < static_cast<int>(blockDim.x >> 6); ++w) s += scratch[w];
  __syncthreads();
  return s;
}

// Checksum of one row of ld es-byte elements, by one wave (lanes stride the columns, four loads in
// flight per lane); every lane returns the total.
__device__ __forceinline__ unsigned long long wave_row_checksum(const void* row, int ld, int es) {
  const int lane = threadIdx.x & 63;
  unsigned long long t = 0;
  if (es == 8) {
    const unsigned long long* p = static_cast<const unsigned long long*>(row);
#pragma unroll 4
    for (int c = lane; c < ld; c += 64) t += tag_term(p[c], c);
  } else {
    const unsigned int* p = static_cast<const unsigned int*>(row);
#pragma unroll 4
    for (int c = lane; c < ld; c += 64) t += tag_term(p[c], c);
  }
  return wave_sum_u64(t);
}

// Waves [w0, w0 + nw) of the block check the rows of `cl`, one wave per row in turn; the first
// mismatch (claimed with atomicCAS on *claim, an LDS int) is reported to err.  Returns (wave-uniform)
// whether this wave found one.
__device__ inline void report_integrity(IntegrityErr* err, int round, int where, int rank_want, const MsgTag& got,
                                        unsigned long long calc);
__device__ inline bool check_rows_waves(const CheckList& cl, int w0, int nw, IntegrityErr* err, int* claim) {
  const int w = static_cast<int>(threadIdx.x >> 6) - w0;
  if (w < 0 || w >= nw) return false;
  bool bad = false;
  for (int m = w; m < cl.n; m += nw) {
    if (cl.mrow[m] < 0) continue;  // a local row (no transport, no tag)
    const unsigned long long sum = wave_row_checksum(cl.row[m], cl.ld, cl.es);
    const MsgTag tg = cl.tags[cl.mrow[m]];
    if (tg.round1 != static_cast<unsigned int>(cl.round + 1) || tg.rank != static_cast<unsigned int>(cl.rank[m]) ||
        tg.sum != sum) {
      bad = true;
      if ((threadIdx.x & 63) == 0 && atomicCAS(claim, 0, 1) == 0)
        report_integrity(err, cl.round, (cl.slot << 16) | cl.mrow[m], cl.rank[m], tg, sum);
    }
  }
  return bad;
}

// Element bits of a row (double / float payloads), zero-extended.
__device__ __forceinline__ unsigned long long elem_bits(double x) {
  return static_cast<unsigned long long>(__double_as_longlong(x));
}
__device__ __forceinline__ unsigned long long elem_bits(float x) { return static_cast<unsigned long long>(__float_as_uint(x)); }

// Record the first failure (caller is a single thread).  Plain vector stores into host-mapped
// memory, then a system-scope release of the flag so the host sees complete fields.
__device__ inline void report_integrity(IntegrityErr* err, int round, int where, int rank_want, const MsgTag& got,
                                        unsigned long long calc) {
  if (!err || __hip_atomic_load(&err->flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return;
  err->round = round;
  err->where = where;
  err->rank_want = rank_want;
  err->round1_got = got.round1;
  err->rank_got = got.rank;
  err->sum_got = got.sum;
  err->sum_calc = calc;
  __threadfence_system();
  __hip_atomic_store(&err->flag, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
#endif

}  // namespace eh
