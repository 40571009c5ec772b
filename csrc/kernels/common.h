// Shared device helpers for the ErasureHead MI355X (gfx950 / CDNA4) kernels.
//
// Everything here is wave64-native: reductions span 64 lanes, loads are 16 bytes
// per lane (one dwordx4 per lane = 1 KiB per wave instruction), and storage types
// are {double, float, bf16} with an fp64 or fp32 accumulator.
#pragma once

#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

namespace eh {

constexpr int kWave = 64;

// bf16 storage is carried as raw uint16 bits; conversion is a shift (exact).
struct bf16_t {
  uint16_t bits;
};

__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}

// Loads of data reached through a pointer table (Segment.X / .y) compile to flat_load, and
// flat loads count in lgkmcnt as well as vmcnt: the LDS / cross-lane waits of a row's wave
// reduction would then also wait for every row tile still in flight.  Buffer loads count in
// vmcnt only, and the descriptor's range check returns zeros past the row end (no per-vector
// bounds branches).  The descriptor base must be wave-uniform (a row, a label array).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
// Cache policy of the design-matrix stream: nt (aux bit 1).  Every X row is read exactly once per
// round from HBM (8 GB per headline round, 32x the Infinity Cache), so default-policy loads only
// churn L2 / MALL.  Measured on a plain 8 KB-row read stream (tools/probes/nt_stream.hip,
// profiles/round3/nt_stream): 5.92 -> 6.62 TB/s at 8 GB, 5.82 -> 6.57 TB/s at 1 GB; sc0 = default.
constexpr int kStreamAux = 2;
template <typename V, int AUX = kStreamAux>
__device__ __forceinline__ V buf_load16(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  static_assert(sizeof(V) == 16, "16-byte vector");
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, byte_off, 0, AUX);
  V out;
  __builtin_memcpy(&out, &v, 16);
  return out;
}
// One 4- / 8-byte element stored through a buffer descriptor (past the descriptor's size: dropped).
template <typename A>
__device__ __forceinline__ void buf_store(__amdgpu_buffer_rsrc_t rs, int byte_off, A v) {
  if constexpr (sizeof(A) == 8) {
    typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
    u32x2 u;
    __builtin_memcpy(&u, &v, 8);
    __builtin_amdgcn_raw_buffer_store_b64(u, rs, byte_off, 0, 0);
  } else {
    unsigned u;
    __builtin_memcpy(&u, &v, 4);
    __builtin_amdgcn_raw_buffer_store_b32(u, rs, byte_off, 0, 0);
  }
}
template <typename A>
__device__ __forceinline__ A buf_load_scalar(__amdgpu_buffer_rsrc_t rs, int byte_off) {
  if constexpr (sizeof(A) == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, byte_off, 0, 0);
    A out;
    __builtin_memcpy(&out, &v, 8);
    return out;
  } else {
    const auto v = __builtin_amdgcn_raw_buffer_load_b32(rs, byte_off, 0, 0);
    A out;
    __builtin_memcpy(&out, &v, 4);
    return out;
  }
}

// 16 bytes through a non-temporal global load (global_load_dwordx4 ... nt): the X stream's policy
// for the kernels that address rows through plain pointers (see kStreamAux).
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
template <typename V>
__device__ __forceinline__ V load16_nt(const void* p) {
  static_assert(sizeof(V) == 16, "16-byte vector");
  const u32x4_nt v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_nt*>(p));
  V out;
  __builtin_memcpy(&out, &v, 16);
  return out;
}

// Storage-type traits: how many elements fit a 16-byte vector load and how to widen.
template <typename T> struct Vec16;
template <> struct Vec16<double> {
  static constexpr int N = 2;
  using raw = double2;
  __device__ __forceinline__ static raw load_raw(const double* p) { return *reinterpret_cast<const raw*>(p); }
  template <typename A>
  __device__ __forceinline__ static A elem(const raw& v, int i) { return static_cast<A>(i == 0 ? v.x : v.y); }
  template <typename A, bool NT = false>
  __device__ __forceinline__ static void load(const double* p, A (&out)[N]) {
    const double2 v = NT ? load16_nt<double2>(p) : *reinterpret_cast<const double2*>(p);
    out[0] = static_cast<A>(v.x);
    out[1] = static_cast<A>(v.y);
  }
};
template <> struct Vec16<float> {
  static constexpr int N = 4;
  using raw = float4;
  __device__ __forceinline__ static raw load_raw(const float* p) { return *reinterpret_cast<const raw*>(p); }
  template <typename A>
  __device__ __forceinline__ static A elem(const raw& v, int i) {
    return static_cast<A>(i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w);
  }
  template <typename A, bool NT = false>
  __device__ __forceinline__ static void load(const float* p, A (&out)[N]) {
    const float4 v = NT ? load16_nt<float4>(p) : *reinterpret_cast<const float4*>(p);
    out[0] = static_cast<A>(v.x);
    out[1] = static_cast<A>(v.y);
    out[2] = static_cast<A>(v.z);
    out[3] = static_cast<A>(v.w);
  }
};
template <> struct Vec16<bf16_t> {
  static constexpr int N = 8;
  using raw = uint4;
  __device__ __forceinline__ static raw load_raw(const bf16_t* p) { return *reinterpret_cast<const raw*>(p); }
  template <typename A>
  __device__ __forceinline__ static A elem(const raw& v, int i) {  // i is a compile-time constant after unrolling
    const uint32_t w = (i >> 1) == 0 ? v.x : (i >> 1) == 1 ? v.y : (i >> 1) == 2 ? v.z : v.w;
    return static_cast<A>(__uint_as_float((i & 1) ? (w & 0xffff0000u) : (w << 16)));
  }
  template <typename A, bool NT = false>
  __device__ __forceinline__ static void load(const bf16_t* p, A (&out)[N]) {
    const uint4 v = NT ? load16_nt<uint4>(p) : *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      out[2 * i] = static_cast<A>(__uint_as_float(w[i] << 16));
      out[2 * i + 1] = static_cast<A>(__uint_as_float(w[i] & 0xffff0000u));
    }
  }
};

// Full-wave sum, every lane ends with the bitwise-same total, in VALU cross-lane moves only
// (no LDS crossbar, no lgkmcnt waits): DPP quad_perm xor 1 and 2, row_half_mirror and
// row_mirror (pairs the quads and half-rows of each 16-lane row), then gfx950's
// v_permlane16_swap / v_permlane32_swap (exchange rows 0<->1, 2<->3, then the two halves).
// Each step adds the partner's value in the same operand order on both partners, so all
// lanes hold identical bits.  fp64 moves its two dwords separately.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(v), CTRL, 0xf, 0xf, true));
}
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float x) { return __uint_as_float(dpp_u32<CTRL>(__float_as_uint(x))); }
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double x) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(x));
  const uint32_t lo = dpp_u32<CTRL>(static_cast<uint32_t>(u)), hi = dpp_u32<CTRL>(static_cast<uint32_t>(u >> 32));
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}
template <bool ROW16>
__device__ __forceinline__ float swap_sum(float x) {
  const uint32_t u = __float_as_uint(x);
  const auto s = ROW16 ? __builtin_amdgcn_permlane16_swap(u, u, false, false)
                       : __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return __uint_as_float(s[0]) + __uint_as_float(s[1]);
}
template <bool ROW16>
__device__ __forceinline__ double swap_sum(double x) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(x));
  const uint32_t l = static_cast<uint32_t>(u), h = static_cast<uint32_t>(u >> 32);
  const auto lo = ROW16 ? __builtin_amdgcn_permlane16_swap(l, l, false, false)
                        : __builtin_amdgcn_permlane32_swap(l, l, false, false);
  const auto hi = ROW16 ? __builtin_amdgcn_permlane16_swap(h, h, false, false)
                        : __builtin_amdgcn_permlane32_swap(h, h, false, false);
  const double a = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi[0]) << 32) | lo[0]));
  const double b = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi[1]) << 32) | lo[1]));
  return a + b;
}
template <typename A>
__device__ __forceinline__ A wave_allreduce_sum(A v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  v = swap_sum<true>(v);   // rows 0<->1, 2<->3
  return swap_sum<false>(v);  // lanes 0-31 <-> 32-63
}

// Two-row reduce-scatter: lanes 0-31 end with the full sum of z0, lanes 32-63 with that of z1
// (one permlane32 exchange, then the within-half steps of wave_allreduce_sum).
__device__ __forceinline__ uint32_t partner32(uint32_t u, bool hi) {
  const auto s = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  return hi ? s[0] : s[1];  // lanes 0-31: s = {self, partner}; lanes 32-63: {partner, self}
}
__device__ __forceinline__ float partner32(float x, bool hi) { return __uint_as_float(partner32(__float_as_uint(x), hi)); }
__device__ __forceinline__ double partner32(double x, bool hi) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(x));
  const uint32_t l = partner32(static_cast<uint32_t>(u), hi), h = partner32(static_cast<uint32_t>(u >> 32), hi);
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(h) << 32) | l));
}
// Exchange with lane ^ 16 (v_permlane16_swap: rows 0<->1, 2<->3), as partner32 does for lane ^ 32.
__device__ __forceinline__ uint32_t partner16(uint32_t u, bool hi) {
  const auto s = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return hi ? s[0] : s[1];
}
__device__ __forceinline__ float partner16(float x, bool hi) { return __uint_as_float(partner16(__float_as_uint(x), hi)); }
__device__ __forceinline__ double partner16(double x, bool hi) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(x));
  const uint32_t l = partner16(static_cast<uint32_t>(u), hi), h = partner16(static_cast<uint32_t>(u >> 32), hi);
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(h) << 32) | l));
}

// Eight-value reduce-scatter: every lane passes v[0..7]; lanes 8j..8j+7 end with the full wave
// sum of v[j] (bitwise the same on all 8).  Halving exchanges with lane ^ 32 (keep 4 values),
// lane ^ 16 (keep 2), the mirrored lane of the 16-lane row (keep 1), then the 8-lane all-reduce:
// 10 cross-lane steps for 8 sums instead of 6 per all-reduced value.
template <typename A>
__device__ __forceinline__ A wave_reduce_scatter8(const A (&v)[8], int lane) {
  const bool h32 = lane >= 32, h16 = (lane & 16) != 0, h8 = (lane & 8) != 0;
  A a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = (h32 ? v[4 + j] : v[j]) + partner32(h32 ? v[j] : v[4 + j], h32);
  A b[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) b[j] = (h16 ? a[2 + j] : a[j]) + partner16(h16 ? a[j] : a[2 + j], h16);
  A c = (h8 ? b[1] : b[0]) + dpp_mov<0x140>(h8 ? b[0] : b[1]);  // row_mirror: lane i <-> 15 - i
  c += dpp_mov<0xB1>(c);
  c += dpp_mov<0x4E>(c);
  c += dpp_mov<0x141>(c);  // row_half_mirror: quad 0 <-> quad 1 of each 8 lanes
  return c;
}

template <typename A>
__device__ __forceinline__ A wave_pair_reduce(A z0, A z1, bool hi) {
  A v = (hi ? z1 : z0) + partner32(hi ? z0 : z1, hi);
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return swap_sum<true>(v);
}
__device__ __forceinline__ float readlane_a(float x, int l) {
  return __uint_as_float(static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(__float_as_uint(x)), l)));
}
__device__ __forceinline__ double readlane_a(double x, int l) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(x));
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(u)), l));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(static_cast<uint32_t>(u >> 32)), l));
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}

// Loss epilogues. r is the per-row coefficient that multiplies x_row in the
// gradient:  g = sum_rows r * x_row.
//   logistic (ref naive.py:137-139):  g = -X^T( ymod / (exp(y*z) + 1) )  ->  r = -ymod * sigmoid(-y z)
//   least squares (ref naive.py:345-346): g = -2 X^T (y - z)                ->  r = -2 * c * (y - z)
enum LossKind : int { kLogistic = 0, kLeastSquares = 1 };

template <typename A>
__device__ __forceinline__ A sigmoid_neg(A t) {
  // 1 / (exp(t) + 1), overflow-free in both directions.
  if (t > A(0)) {
    const A e = exp(-t);
    return e / (A(1) + e);
  }
  return A(1) / (A(1) + exp(t));
}

// Branch-free fp32 sigmoid on the hardware exp2 and reciprocal (each within ~1 ulp): e =
// exp(-|t|) is in (0, 1], so 1 + e is in [1, 2] and neither can overflow.  Used where a wave's
// lanes hold different rows (the MFMA bundles: 0.382 -> 0.371 ms at the bf16 headline).  The
// fp32 staged pair kernel measured SLOWER with it (0.737 -> 0.81 ms, same box,
// profiles/round2/s1_ab_fastsig), so the library form stays the default elsewhere.
__device__ __forceinline__ float sigmoid_neg_hw(float t) {
  const float e = __builtin_amdgcn_exp2f(-__builtin_fabsf(t) * 1.4426950408889634f);
  const float q = __builtin_amdgcn_rcpf(1.0f + e);
  return t > 0.f ? e * q : q;
}
template <int LOSS>
__device__ __forceinline__ float residual_hw(float z, float y, float coef) {
  if constexpr (LOSS == kLogistic) {
    return -(coef * y) * sigmoid_neg_hw(y * z);
  } else {
    return -2.f * coef * (y - z);
  }
}

// Branch-free form for waves whose lanes hold different rows (one exp either way).
template <int LOSS, typename A>
__device__ __forceinline__ A residual_branchfree(A z, A y, A coef) {
  if constexpr (LOSS == kLogistic) {
    const A t = y * z;
    const A e = exp(-fabs(t));
    const A q = A(1) / (A(1) + e);
    return -(coef * y) * (t > A(0) ? e * q : q);
  } else {
    return A(-2) * coef * (y - z);
  }
}

template <int LOSS, typename A>
__device__ __forceinline__ A residual(A z, A y, A coef) {
  if constexpr (LOSS == kLogistic) {
    return -(coef * y) * sigmoid_neg<A>(y * z);
  } else {
    return A(-2) * coef * (y - z);
  }
}

__host__ __device__ constexpr int ceil_div(int a, int b) { return (a + b - 1) / b; }

// Stale-round gate of a lazy-drain worker round (launchers.h PutDesc::gate, engine.cpp WorkerPump):
// nonzero = the master had published the next beta before this round could start, so every kernel
// of the round returns at once.  The value is launch-uniform (written by the previous round's put
// kernel, stream-ordered before this launch), so whole grids return together and no barrier is left
// half-reached.  nullptr = not gated (every other launch).
__device__ __forceinline__ bool gate_closed(const int* gate) {
  if (!gate) return false;
  return __builtin_amdgcn_readfirstlane(__hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0;
}

// Release of a whole workgroup's stores at system scope, the producer form of the MI355X guide
// ("Valid forms"): every wave waits for its own stores, the workgroup joins, and ONE lane writes
// back the XCD's L2 and waits for the write-back.  After it thread 0 issues RELAXED flag / counter
// stores.  Replaces __threadfence_system() by every thread (one L2 write-back + invalidate per
// wave: 16 per 1024-thread arbiter) and release-ordered flag stores (one more write-back per store:
// the arbiter's per-target counters made its release grow with the rank count, 4.3 us at 2 ranks,
// 12.2 at 8, profiles/round3/arbiter_books).  Call from every thread (block-uniform control flow).
//
// strict (launchers.h strict_release()): the forms before round 4 on top -- every thread also fences
// at system scope, and publish_u64 / the block counters are release / acq_rel ordered.  The default of
// any job whose ranks sit on different GPUs (engine/loops.py select_release_form): the relaxed forms
// are measured only with every rank on one GPU so far.
__device__ __forceinline__ void block_release_system(bool strict = false) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (strict) __threadfence_system();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    // the compiler may drop the wait behind the write-back (ROCm 7.2 / gfx950): keep it explicit
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}
// A flag / counter store that announces what block_release_system released (one thread calls it).
__device__ __forceinline__ void publish_u64(unsigned long long* p, unsigned long long v, bool strict) {
  if (strict)
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  else
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// The per-launch block counter of a multi-block put: the previous count.
__device__ __forceinline__ unsigned int count_block_done(unsigned int* counter, bool strict) {
  return strict ? __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT)
                : __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace eh
