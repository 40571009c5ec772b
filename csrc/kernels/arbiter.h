// Device-side master round ("arbiter"): the master's stop rule, decode, combine + update and
// beta broadcast of one round in ONE single-workgroup kernel (csrc/kernels/arbiter.hip).
//
// Host-driven multi-GPU rounds pay a host hop between the last worker message and the next
// beta: the host sees the flag, decodes, launches the combine, then the put.  The arbiter
// kernel is queued ahead on the master's stream behind the master's own gradient; it polls
// the workers' shared round counters itself, applies the collector's rules (same arrival
// order, tie permutation and stop rules as csrc/runtime/collector.cpp for delay-free rounds),
// decodes, updates beta and writes beta(i+1) straight into every worker inbox, then (after
// the drain) release-stores the workers' beta counters.  Used by MasterPump::run_device.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "integrity.h"

namespace eh {

constexpr int kArbMaxW = 64;          // workers (bitmasks)
constexpr int kArbMaxProbes = 512;    // expected shards per round
constexpr int kArbMaxSrc = 64;        // worker ranks (one shared counter each)
constexpr int kArbMaxRows = 16;       // buffer rows (shards) of one message
constexpr int kArbLdsTable = 4096;    // decode-table doubles kept in LDS (2^W * W, W <= 9)
constexpr int kArbLogInts = 4 + 4 * kArbMaxW;   // per round: status, n_arrivals, n_used, -, then (w, p) pairs
// per round: t_begin, t_dec (combine done), t_end (released), t_join (poll joined), t_decoded (decode
// done), -, -, -, then one tick per arrival
constexpr int kArbTickArr = 8;
constexpr int kArbLogTicks = kArbTickArr + 2 * kArbMaxW;

struct ArbArgs {
  int W, n_groups, rule, k, decode, drain;
  int nprobe, nsrc, ntarget, K, ld, d, g_rows, r_rows, R, update_rule;
  long long deadline_ticks;              // poll budget per round, wall_clock64 ticks
  const int* group_of;                   // [W]
  const int* probe_w;                    // [nprobe]
  const int* probe_p;                    // [nprobe]
  const int* probe_src;                  // [nprobe]: -1 local (done when the kernel starts), j >= 0 source j
  const int* nsh;                        // [2W] shards per message (2w + part)
  const int* msg_nrows;                  // [2W]
  const int* msg_rows;                   // [2W][kArbMaxRows]: kind << 24 | row (kind 0 local G, 1 mailbox)
  const unsigned long long* src_flag;    // [nsrc] device addresses of the workers' message counters
  const double* table;                   // [2^W][W] decode table (kTable) or nullptr; NaN = unknown pattern
  const int* tie;                        // [R][W] tie rank of each worker (smaller first)
  const double* decay;                   // [R] update schedule (csrc/kernels/update.hip)
  const double* gm;
  const double* l2;
  const double* theta;
  double* beta;                          // [ld]
  double* u;                             // [ld]
  double* hist;                          // [R][ld]
  void* beta_in;                         // [R + 1][ld], message dtype
  const void* G;                         // [K][g_rows][ld] local messages
  const void* rbuf;                      // [K][r_rows][ld] mailbox
  const unsigned long long* targets;     // [ntarget][2]: worker inbox base, its beta counter address
  int* log;                              // [R][kArbLogInts]
  long long* tlog;                       // [R][kArbLogTicks]
  int* abort;                            // set by a failed round: every later arbiter returns at once
  // Integrity (integrity.h; tags == nullptr: off): the mailbox rows round i decodes are checked
  // against their senders' tags by arbiter_check on a side stream during round i+1's local
  // gradient (arbiter i+1 fails if it found one), and beta(i+1) carries a tag into every worker
  // inbox (inbox base + inbox_tag_off, one per round).
  const MsgTag* tags;                    // [K][r_rows] mailbox tags
  const int* row_rank;                   // [r_rows] sender rank of each mailbox row
  long long inbox_tag_off;               // bytes from a worker inbox base to its tag slots
  CheckList* checks;                     // [2] device memory: the mailbox rows rounds i-1 / i decoded
  IntegrityErr* err;                     // host-mapped: the first failed check
  int strict;                            // set by arbiter_round_launch (launchers.h strict_release)
};
// Round statuses in the log: 0 ok, 1 timeout, 2 not decodable, 3 skipped, 4 integrity failure of the
// PREVIOUS round's messages (found by its arbiter_check; details in ArbArgs::err).
constexpr int kArbIntegrity = 4;

// msg_dtype 0 fp64 / 1 fp32 (messages, beta_in, inboxes)
// check_prev: round-1's rows were checked (arbiter_check) before this launch: fail on a reported error
hipError_t arbiter_round_launch(const ArbArgs& a, int round, int msg_dtype, hipStream_t st, bool check_prev);
// round's decoded mailbox rows against their tags (a no-op with tags off)
hipError_t arbiter_check_launch(const ArbArgs& a, int round, hipStream_t st);

}  // namespace eh
