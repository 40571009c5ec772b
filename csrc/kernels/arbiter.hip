// Device-side master round (see arbiter.h): poll -> stop rule -> decode -> combine + update ->
// beta(i+1) into the worker inboxes -> drain -> release the workers' beta counters.
//
// Reference loop replaced (per round, ref src/approximate_coding.py:131-183, src/naive.py:97-123):
// Isend beta to every worker; Waitany until the stop rule; decode; GD/AGD update; Waitall.
//
// One workgroup of 1024 threads (one column each at d <= 1024, so the combine is a couple of
// batches of independent message loads).  Wave 0 polls the workers' shared 64-bit round counters (one
// lane per worker rank, system-scope acquire loads of host memory) and keeps the collector's books
// wave-parallel (one lane per probe of a poll: rank sort, prefix-summed stop-rule counts).  Probes
// that complete in the same poll are ordered by the round's tie permutation, then by probe id,
// exactly like Collector::process_ready for delay-free rounds (csrc/runtime/collector.cpp), so a
// replay of the logged arrivals reproduces the update.
// Every spin has a deadline (a.deadline_ticks): a round that times out sets a.abort, skips its
// update and its broadcast, and every later arbiter returns at once, so the grid always drains.
#include "arbiter.h"
#include "common.h"
#include "launchers.h"

namespace eh {

namespace {

__device__ __forceinline__ bool rule_holds(int rule, int k, int W, int G, int cnt0, int cnt1, int cntg) {
  switch (rule) {
    case 0: return cnt0 >= W;                    // kRuleAll
    case 1: return cnt0 >= k;                    // kRuleCount
    case 2: return cnt0 >= k || cntg >= G;       // kRuleFrc
    case 3: return cnt1 >= W && cntg >= G;       // kRulePartialFrc
    case 4: return cnt1 >= W && cnt0 >= k;       // kRulePartialCount
    default: return true;
  }
}

// Polls are relaxed system-scope loads (they bypass the caches); the poll that ends step 1 is followed
// by ONE acquire fence of wave 0 before the barrier that releases the other waves' message loads (the
// MI355X guide's consumer form: an acquire per poll is an L1 invalidate each, 2-3x slower per hop).
// strict (launchers.h strict_release): every poll is an acquire load, the form before round 4.
__device__ __forceinline__ unsigned long long load_counter(const unsigned long long* p, bool strict) {
  if (strict) return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Inclusive prefix sum over the wave (every lane active).
__device__ __forceinline__ int wave_scan(int v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const int u = __shfl_up(v, dd, 64);
    if (lane >= dd) v += u;
  }
  return v;
}
// Bitwise OR over the wave (every lane active); every lane ends with the result.
__device__ __forceinline__ unsigned long long wave_or(unsigned long long v) {
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const unsigned lo = __shfl_xor(static_cast<unsigned>(v), dd, 64);
    const unsigned hi = __shfl_xor(static_cast<unsigned>(v >> 32), dd, 64);
    v |= static_cast<unsigned long long>(hi) << 32 | lo;
  }
  return v;
}

}  // namespace

template <typename M>
__global__ void __launch_bounds__(1024) arbiter_round(const ArbArgs a, int i, int check_prev) {
  __shared__ int s_pw[kArbMaxProbes], s_pp[kArbMaxProbes], s_ps[kArbMaxProbes];
  __shared__ int batch[kArbMaxProbes];
  __shared__ int s_bkey[kArbMaxProbes], s_sorted[kArbMaxProbes];  // a poll's batch: tie ranks, sorted messages
  __shared__ int s_gfirst[kArbMaxW];
  __shared__ int got_sh[2 * kArbMaxW];
  // the round's tables in LDS: thread 0's books and decode walk them serially (a dependent global load
  // per step cost ~15 us per round)
  __shared__ int s_key[kArbMaxProbes];  // tie rank of each probe's worker
  __shared__ int s_group[kArbMaxW], s_nsh[2 * kArbMaxW], s_nrows[2 * kArbMaxW];
  __shared__ int s_rows[2 * kArbMaxW * kArbMaxRows];
  __shared__ double s_trow[kArbMaxW];   // decode-table row of the round's completion pattern
  // the whole decode table when it is small (2^W * W <= 4096 doubles: W <= 9, the headline's 2 KB):
  // copied by waves 1-15 while wave 0 polls, so the completion pattern's row is an LDS read after the
  // stop instead of a dependent global load on the stop -> release path
  __shared__ double s_table[kArbLdsTable];
  __shared__ int arr_w[2 * kArbMaxW], arr_p[2 * kArbMaxW];
  __shared__ long long arr_t[2 * kArbMaxW];
  __shared__ const void* mptr[kMaxMsgs];
  __shared__ double mcoef[kMaxMsgs];
  __shared__ int mrow[kMaxMsgs];  // kind << 24 | row of every used buffer row
  __shared__ unsigned long long scratch[16];
  __shared__ int s_narr, s_nmsg, s_status, s_bad;
  __shared__ unsigned long long s_mask;
  __shared__ unsigned long long s_bsum;
  const int tid = threadIdx.x;
  int* lg = a.log + static_cast<long long>(i) * kArbLogInts;
  long long* tl = a.tlog + static_cast<long long>(i) * kArbLogTicks;
  if (__hip_atomic_load(a.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {  // an earlier round failed
    if (tid == 0) lg[0] = 3;
    return;
  }
  const int* tie = a.tie + static_cast<long long>(i) * a.W;
  for (int q = tid; q < a.nprobe; q += blockDim.x) {
    const int w = a.probe_w[q];
    s_pw[q] = w;
    s_pp[q] = a.probe_p[q];
    s_ps[q] = a.probe_src[q];
    s_key[q] = tie[w];
  }
  for (int m = tid; m < 2 * a.W; m += blockDim.x) {
    got_sh[m] = 0;
    s_nsh[m] = a.nsh[m];
    s_nrows[m] = a.msg_nrows[m];
  }
  for (int e = tid; e < 2 * a.W * kArbMaxRows; e += blockDim.x) s_rows[e] = a.msg_rows[e];
  for (int w = tid; w < a.W; w += blockDim.x) s_group[w] = a.group_of[w];
  if (tid == 0) {
    s_narr = 0;
    s_nmsg = 0;
    s_status = 0;
    s_bad = 0;
  }
  __syncthreads();

  const bool table_dec = (a.decode == 3 || a.decode == 4) && a.table;
  const bool lds_table = table_dec && a.W <= 12 && (1ll << a.W) * a.W <= kArbLdsTable;
  if (lds_table && tid >= 64) {
    const int n = (1 << a.W) * a.W;
    for (int e = tid - 64; e < n; e += blockDim.x - 64) s_table[e] = a.table[e];
  }
  // this round's update constants and the first 1024 columns of beta / u, loaded while the workers
  // compute (off the stop-rule -> release path)
  const double decay = a.decay[i], gm = a.gm[i], l2 = a.l2[i], theta = a.theta[i];
  const double b_pre = tid < a.d ? a.beta[tid] : 0.0;
  const double u_pre = tid < a.d && a.update_rule != 0 ? a.u[tid] : 0.0;

  // ---- 1. poll until the stop rule holds (wave 0) -------------------------------------------
  unsigned long long seen = 0;  // sources seen so far (wave-uniform)
  if (tid < 64) {
    const long long t0 = wall_clock64();
    const unsigned long long all_src = a.nsrc >= 64 ? ~0ull : ((1ull << a.nsrc) - 1);
    const unsigned long long below = tid == 0 ? 0ull : (~0ull >> (64 - tid));  // lanes under this one
    // the collector's books, wave-uniform (every lane holds the same values)
    unsigned long long got0 = 0, gdone = 0;
    int cnt0 = 0, cnt1 = 0, cntg = 0, stopped = 0, narr = 0;
    for (int it = 0;; ++it) {
      const long long t = wall_clock64();
      const bool mine = tid < a.nsrc && !(seen >> tid & 1) && load_counter(reinterpret_cast<const unsigned long long*>(a.src_flag[tid]), a.strict) >= static_cast<unsigned long long>(i + 1);
      const unsigned long long nm = __ballot(mine);
      if (it == 0 || nm) {
        // (a) this poll's batch: its probes in probe-id order (the local ones on the first poll)
        int nb = 0;
        for (int q0 = 0; q0 < a.nprobe; q0 += 64) {
          const int q = q0 + tid;
          bool in = false;
          if (q < a.nprobe) {
            const int s = s_ps[q];
            in = (s < 0 && it == 0) || (s >= 0 && (nm >> s & 1));
          }
          const unsigned long long m = __ballot(in);
          if (in) {
            const int x = nb + __popcll(m & below);
            batch[x] = q;
            s_bkey[x] = s_key[q];
          }
          nb += __popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
        // (b) (tie rank, probe id) order: the batch is in probe-id order, so an element's place is the
        // number of elements with a smaller tie rank plus the earlier ones with its own
        for (int x0 = 0; x0 < nb; x0 += 64) {
          const int x = x0 + tid;
          if (x < nb) {
            const int kx = s_bkey[x];
            int pos = 0;
            for (int y = 0; y < nb; ++y) {
              const int ky = s_bkey[y];
              pos += (ky < kx || (ky == kx && y < x)) ? 1 : 0;
            }
            const int q = batch[x];
            s_sorted[pos] = 2 * s_pw[q] + s_pp[q];
          }
        }
        __builtin_amdgcn_wave_barrier();
        // (c) the books in that order, 64 elements at a time.  An element completes its message when
        // the shards counted before plus the earlier elements of the same message reach nsh; the
        // completions are the arrivals, the stop rule's counts are prefix sums over them, and the
        // first arrival at which the rule holds is the last one recorded (later ones are late).
        for (int j0 = 0; j0 < nb && !stopped; j0 += 64) {
          const int j = j0 + tid;
          const bool valid = j < nb;
          const int mi = valid ? s_sorted[j] : 0;
          int before = 0;
          const int jend = min(j0 + 64, nb);
          for (int y = j0; y < jend; ++y) before += (y < j && s_sorted[y] == mi) ? 1 : 0;
          const int prev = valid ? got_sh[mi] : 0;
          for (int gg = tid; gg < kArbMaxW; gg += 64) s_gfirst[gg] = 64;
          __builtin_amdgcn_wave_barrier();
          if (valid) atomicAdd(&got_sh[mi], 1);
          const bool comp = valid && prev + before + 1 == s_nsh[mi];
          const int w = mi >> 1, p = mi & 1;
          const int g = s_group[w];
          const bool a0 = comp && p == 0, a1 = comp && p == 1;
          if (a0) atomicMin(&s_gfirst[g], tid);
          __builtin_amdgcn_wave_barrier();
          const bool gf = a0 && !(gdone >> g & 1) && s_gfirst[g] == tid;  // its group's first p = 0 arrival
          const int c0 = cnt0 + wave_scan(a0 ? 1 : 0), c1 = cnt1 + wave_scan(a1 ? 1 : 0), cg = cntg + wave_scan(gf ? 1 : 0);
          const unsigned long long hm = __ballot(comp && rule_holds(a.rule, a.k, a.W, a.n_groups, c0, c1, cg));
          const int last = hm ? __ffsll(hm) - 1 : 63;
          const bool rec = comp && tid <= last;
          const unsigned long long rm = __ballot(rec);
          if (rec) {
            const int x = narr + __popcll(rm & below);
            arr_w[x] = w;
            arr_p[x] = p;
            arr_t[x] = t;
          }
          narr += __popcll(rm);
          cnt0 += __popcll(__ballot(rec && p == 0));
          cnt1 += __popcll(__ballot(rec && p == 1));
          cntg += __popcll(__ballot(rec && gf));
          got0 |= wave_or((rec && p == 0) ? 1ull << w : 0ull);
          gdone |= wave_or((rec && gf) ? 1ull << g : 0ull);
          if (hm) stopped = 1;
        }
        seen |= nm;
      }
      stopped = __builtin_amdgcn_readfirstlane(stopped);
      if (stopped) break;
      if ((seen & all_src) == all_src && a.nsrc > 0 && it > 0) {  // everything is in and the rule never held
        if (tid == 0) s_status = 2;
        break;
      }
      if (t - t0 > a.deadline_ticks) {
        if (tid == 0) s_status = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    // acquire for everything the flags announced (the mailbox rows every wave reads after the barrier)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // the completion pattern (every p = 0 arrival) and its decode-table row, one lane per worker
    const unsigned long long mask = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(got0)) |
                                    static_cast<unsigned long long>(__builtin_amdgcn_readfirstlane(
                                        static_cast<unsigned>(got0 >> 32))) << 32;
    if (tid == 0) {
      s_mask = mask;
      s_narr = narr;
    }
    if (table_dec && !lds_table)
      for (int w = tid; w < a.W; w += 64)
        s_trow[w] = (mask >> w & 1) ? a.table[static_cast<long long>(mask) * a.W + w] : 0.0;
  } else if (a.tags && check_prev && tid == 64) {
    // the previous round's mailbox rows were checked against their senders' tags by a side-stream
    // kernel during this round's local gradient (arbiter_check, queued ahead of this kernel): a
    // failure there fails this round
    if (__hip_atomic_load(&a.err->flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)) s_bad = 1;
  }
  __syncthreads();
  if (s_status == 0 && s_bad) s_status = kArbIntegrity;  // a torn / stale message of round i-1
  if (s_status != 0) {
    if (tid == 0) {
      __hip_atomic_store(a.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lg[0] = s_status;
      lg[1] = s_narr;
    }
    return;
  }
  // (no further fence: wave 0's acquire after the poll invalidated this CU's caches, and the barrier
  // orders every wave's loads after it)
  if (tid == 0) tl[3] = wall_clock64();

  // ---- 2. decode (wave 0, one lane per arrival; MasterPump::decode's message order) ------------
  // Arrival x contributes its message rows iff: p = 1 and a partial decode (2, 4); p = 0 and decode 0;
  // p = 0, decode 1 / 2 and the first p = 0 arrival of its FRC group.  Then, for the table decodes
  // (3, 4), every worker of the completion pattern in worker order with its table coefficient.  Each
  // lane's rows land at its exclusive prefix sum (wave scan), so the combine order is the serial one.
  const int slot = i % a.K;
  if (tid < 64) {
    auto scan = [&](int v) {  // inclusive prefix sum over the wave
#pragma unroll
      for (int dd = 1; dd < 64; dd <<= 1) {
        const int u = __shfl_up(v, dd, 64);
        if (tid >= dd) v += u;
      }
      return v;
    };
    auto put_rows = [&](int w, int p, double c, int pos) {
      const int mi = 2 * w + p;
      for (int r = 0; r < s_nrows[mi] && pos + r < kMaxMsgs; ++r) {
        const int e = s_rows[mi * kArbMaxRows + r];
        const int row = e & 0xffffff;
        mptr[pos + r] = (e >> 24) == 0
                            ? static_cast<const void*>(static_cast<const M*>(a.G) + (static_cast<long long>(slot) * a.g_rows + row) * a.ld)
                            : static_cast<const void*>(static_cast<const M*>(a.rbuf) + (static_cast<long long>(slot) * a.r_rows + row) * a.ld);
        mcoef[pos + r] = c;
        mrow[pos + r] = e;
      }
    };
    const bool frc = a.decode == 1 || a.decode == 2;
    if (frc) {  // first p = 0 arrival of every group
      for (int g = tid; g < kArbMaxW; g += 64) batch[g] = 1 << 30;  // (batch is free after the poll)
      __builtin_amdgcn_wave_barrier();
      for (int x = tid; x < s_narr; x += 64)
        if (arr_p[x] == 0) atomicMin(&batch[s_group[arr_w[x]]], x);
      __builtin_amdgcn_wave_barrier();
    }
    int base = 0;
    for (int x0 = 0; x0 < s_narr; x0 += 64) {  // arrival order
      const int x = x0 + tid;
      int nr = 0;
      if (x < s_narr) {
        const int w = arr_w[x], p = arr_p[x];
        const bool use = p == 1 ? (a.decode == 2 || a.decode == 4)
                                : (a.decode == 0 || (frc && batch[s_group[w]] == x));
        if (use) nr = s_nrows[2 * w + p];
      }
      const int incl = scan(nr);
      if (nr) put_rows(arr_w[x], arr_p[x], 1.0, base + incl - nr);
      base += __shfl(incl, 63, 64);
    }
    if (a.decode == 3 || a.decode == 4) {  // the table's coefficients, worker order
      if (!a.table) {
        if (tid == 0) s_status = 2;
      } else {
        const unsigned long long mask = s_mask;
        for (int w0 = 0; w0 < a.W; w0 += 64) {
          const int w = w0 + tid;
          const bool on = w < a.W && (mask >> w & 1);
          // (the LDS copy is complete: waves 1-15 wrote it before the barrier that ended the poll)
          const double c = on ? (lds_table ? s_table[static_cast<int>(mask) * a.W + w] : s_trow[w]) : 0.0;
          if (__ballot(on && c != c) && tid == 0) s_status = 2;  // NaN: completion pattern without a table row
          const int nr = on ? s_nrows[2 * w] : 0;
          const int incl = scan(nr);
          if (nr) put_rows(w, 0, c, base + incl - nr);
          base += __shfl(incl, 63, 64);
        }
      }
    }
    if (tid == 0) {
      s_nmsg = min(base, kMaxMsgs + 1);
      if (base > kMaxMsgs) s_status = 2;
    }
  }
  __syncthreads();
  if (s_status != 0) {
    if (tid == 0) {
      __hip_atomic_store(a.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lg[0] = s_status;
      lg[1] = s_narr;
    }
    return;
  }

  if (tid == 0) tl[4] = wall_clock64();

  // ---- 3. combine + update, beta(i+1) into beta_in and every worker inbox -------------------
  // With tags on, the loop also sums the checksum terms of beta(i+1) for its inbox tags (the
  // column loop has a block-uniform trip count for the block reduction after it).
  const bool vfy = a.tags != nullptr;
  M* bin_next = static_cast<M*>(a.beta_in) + static_cast<long long>(i + 1) * a.ld;
  unsigned long long bterm = 0;
  for (int c0 = 0; c0 < a.ld; c0 += blockDim.x) {
    const int c = c0 + tid;
    const bool in = c < a.ld;
    M out = M(0);
    double g = 0.0;
    constexpr int kB = 16;  // independent loads first, then the fma chain in message order
    for (int m0 = 0; m0 < s_nmsg; m0 += kB) {
      M v[kB];
#pragma unroll
      for (int q = 0; q < kB; ++q) v[q] = (in && m0 + q < s_nmsg) ? static_cast<const M*>(mptr[m0 + q])[c] : M(0);
#pragma unroll
      for (int q = 0; q < kB; ++q)
        if (m0 + q < s_nmsg) g = fma(mcoef[m0 + q], static_cast<double>(v[q]), g);
    }
    if (in && c < a.d) {
      const double b = c0 == 0 ? b_pre : a.beta[c];
      double nb;
      if (a.update_rule == 0) {
        nb = decay * b - gm * g;
      } else {
        const double yt = (1.0 - theta) * b + theta * (c0 == 0 ? u_pre : a.u[c]);
        nb = yt - gm * g - l2 * b;
        a.u[c] = b + (nb - b) * (1.0 / theta);
      }
      a.beta[c] = nb;
      a.hist[static_cast<long long>(i) * a.ld + c] = nb;
      out = static_cast<M>(nb);
    }
    if (in) {
      if (i + 1 <= a.R) bin_next[c] = out;
      for (int t = 0; t < a.ntarget && i + 1 < a.R; ++t)
        reinterpret_cast<M*>(a.targets[2 * t])[static_cast<long long>(i + 1) * a.ld + c] = out;
      bterm += tag_term(elem_bits(out), c);
    }
  }
  if (vfy) {
    const unsigned long long bs = block_sum_u64(bterm, scratch);
    if (tid == 0) s_bsum = bs;
  }
  __syncthreads();
  if (tid == 0) tl[1] = wall_clock64();

  // ---- 4. drain: every worker rank's round-i message has landed ------------------------------
  if (a.drain && tid < 64) {
    const long long t0 = wall_clock64();
    const unsigned long long all_src = a.nsrc >= 64 ? ~0ull : ((1ull << a.nsrc) - 1);
    for (;;) {
      const bool mine = tid < a.nsrc && !(seen >> tid & 1) && load_counter(reinterpret_cast<const unsigned long long*>(a.src_flag[tid]), a.strict) >= static_cast<unsigned long long>(i + 1);
      seen |= __ballot(mine);
      if ((seen & all_src) == all_src) break;
      if (wall_clock64() - t0 > a.deadline_ticks) {
        if (tid == 0) s_status = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (s_status != 0) {  // a worker rank is gone: do not release the next round
    if (tid == 0) {
      __hip_atomic_store(a.abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lg[0] = s_status;
      lg[1] = s_narr;
    }
    return;
  }

  // ---- 5. release beta(i+1): the inbox rows are visible before every worker's counter -------
  if (vfy && i + 1 < a.R)
    for (int t = tid; t < a.ntarget; t += blockDim.x)
      reinterpret_cast<MsgTag*>(reinterpret_cast<char*>(a.targets[2 * t]) + a.inbox_tag_off)[i + 1] =
          MsgTag{static_cast<unsigned int>(i + 2), 0u, s_bsum};
  block_release_system(a.strict);  // one write-back for every inbox row and tag (common.h)
  if (tid == 0) {
    if (i + 1 < a.R) {
      for (int t = 0; t < a.ntarget; ++t)  // relaxed unless strict: ordered by the release above
        publish_u64(reinterpret_cast<unsigned long long*>(a.targets[2 * t + 1]), static_cast<unsigned long long>(i + 2),
                    a.strict);
    }
    const long long te = wall_clock64();
    tl[2] = te;
    if (i + 1 < a.R) a.tlog[static_cast<long long>(i + 1) * kArbLogTicks] = te;  // next round's start
    lg[0] = 0;
    lg[1] = s_narr;
    lg[2] = s_nmsg;
    for (int x = 0; x < s_narr; ++x) {
      lg[4 + 2 * x] = arr_w[x];
      lg[5 + 2 * x] = arr_p[x];
      tl[kArbTickArr + x] = arr_t[x];
    }
  }
  if (vfy) {  // this round's decoded rows for the next arbiter's idle waves (or the segment's tail check):
              // one thread per row, local rows marked -1 (not checked)
    CheckList& cl = a.checks[i & 1];
    for (int m = tid; m < s_nmsg && m < kMaxMsgs; m += blockDim.x) {
      const bool mb = (mrow[m] >> 24) == 1;
      const int row = mrow[m] & 0xffffff;
      cl.row[m] = mptr[m];
      cl.mrow[m] = mb ? row : -1;
      cl.rank[m] = mb ? a.row_rank[row] : 0;
    }
    if (tid == 0) {
      cl.n = min(s_nmsg, kMaxMsgs);
      cl.round = i;
      cl.slot = slot;
      cl.es = static_cast<int>(sizeof(M));
      cl.ld = a.ld;
      cl.tags = a.tags + static_cast<long long>(slot) * a.r_rows;
    }
  }
}

// Round i's decoded mailbox rows against their senders' tags: one workgroup on a side stream, queued
// behind arbiter i and ahead of arbiter i+1 (MasterPump::run_device), so it runs during round i+1's
// local gradient; the rows stay intact until their slot comes back (K >= 2 rounds later).
__global__ void __launch_bounds__(1024) arbiter_check(const ArbArgs a, int i) {
  __shared__ int claim;
  if (threadIdx.x == 0) claim = 0;
  __syncthreads();
  if (__hip_atomic_load(a.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
  check_rows_waves(a.checks[i & 1], 0, static_cast<int>(blockDim.x >> 6), a.err, &claim);
}

hipError_t arbiter_round_launch(const ArbArgs& a, int round, int msg_dtype, hipStream_t st, bool check_prev) {
  if (a.W > kArbMaxW || a.nprobe > kArbMaxProbes || a.nsrc > kArbMaxSrc || a.nsrc > 64) return hipErrorInvalidValue;
  ArbArgs b = a;
  b.strict = strict_release() ? 1 : 0;
  if (msg_dtype == 0)
    hipLaunchKernelGGL(arbiter_round<double>, dim3(1), dim3(1024), 0, st, b, round, check_prev ? 1 : 0);
  else
    hipLaunchKernelGGL(arbiter_round<float>, dim3(1), dim3(1024), 0, st, b, round, check_prev ? 1 : 0);
  return hipGetLastError();
}

hipError_t arbiter_check_launch(const ArbArgs& a, int round, hipStream_t st) {
  if (!a.tags) return hipSuccess;
  hipLaunchKernelGGL(arbiter_check, dim3(1), dim3(1024), 0, st, a, round);
  return hipGetLastError();
}

}  // namespace eh
