// Host-side launch interface of every gfx950 kernel in csrc/kernels/*.hip.
//
// Shared by the Python bindings (csrc/bindings.cpp), the IPC runtime (csrc/runtime/ipc.cpp)
// and the native round executors (csrc/runtime/engine.cpp).  Every launcher enqueues on
// the given HIP stream and returns the launch error; shapes are validated by the callers.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdlib>

#include "integrity.h"

namespace eh {

// Release form of every put / signal / arbiter release in this process (transport.hip).  strict: the
// release-ordered forms (common.h block_release_system(strict), publish_u64) and acquire polls in the
// arbiter; relaxed: one lane's system fence + relaxed flag stores (measured with ranks on one GPU).
// The launchers stamp it into PutDesc::strict / ArbArgs::strict at every launch.  STRICT until the
// job says otherwise: the Trainer picks the form from the ranks' device map before any transport
// exists (engine/loops.py select_release_form: relaxed only when every rank shares one GPU).
bool strict_release();
void set_release_form(bool strict);

// ---- worker gradient (grad_dense.hip, grad_sparse.hip) -------------------------------
// dtype: 0 fp64 storage/acc, 1 fp32/fp32, 2 bf16 storage/fp32 acc; loss: 0 logistic, 1 least squares
// k: the kernel the plan chose (grad_dense.h KernelChoice)
// Slab-reduction scratch of the dense launchers ("part"): [nslots][kSlabSplits][ld] partial sums in
// the accumulator type.
constexpr long long kSlabSplits = 16;  // grad_dense.hip kSplits
inline long long slab_part_bytes(long long nslots, long long ld, long long acc_bytes) {
  return nslots * kSlabSplits * ld * acc_bytes;
}

struct PutDesc;
struct KernelChoice;
// Slab reduction form (grad_dense.hip g_slab_mode): 1 fused launches (default), 2 fused plain /
// two-stage puts, 0 two stages.
void set_slab_reduce_mode(int mode);
// rows per LDS stage of the bf16 MFMA bundles (grad_mfma.hip): 32 (default) or 16 (a 4-deep ring), for A/B
void set_mfma_stage_rows(int rows);
void set_mfma_probe(int mode);  // timing probes only (grad_mfma.hip): 1 stage stream alone, 2 compute alone
void set_mfma_pack(bool on);    // bf16 MFMA bundles with R <= 4: bf16 terms packed into M (default) or 3 MFMAs
void set_mfma_stream(int mode);  // packed bf16 bundles: 0 LDS-DMA ring (default),
                                 // VGPR-staged ring 3 (two register sets) / 4 (three)
// Timeline probe: grad_dense_multi launches write {start, rows done, slab written, XCC} ticks per bundle
// into `stamps` (int64 [4 * bundles]); nullptr turns it off (tools/probes/bundle_stamps.py).
void set_grad_stamps(void* stamps);
int slab_reduce_mode();
// put (optional): fuse the message put + signal into the final slab reduction; put->dst
// receives the nslots x ld result rows, put->bytes is ignored.
hipError_t grad_dense_launch(int dtype, int loss, int cpl, const void* segs, const void* tasks,
                             int ntasks, const void* beta, void* slab, const int* slot_task_begin,
                             int nslots, void* part, void* G, int ld, hipStream_t st, const KernelChoice& k,
                             const PutDesc* put = nullptr, const int* gate = nullptr);
hipError_t grad_dense_twopass_launch(int dtype, int loss, const void* segs, const void* tasks,
                                     int ntasks, const void* beta, const int* task_row_off,
                                     void* rbuf, void* slab, const int* slot_task_begin,
                                     int nslots, void* part, void* G, int ld, hipStream_t st,
                                     const int* gate = nullptr);
// Sparse (CSR / one-hot ELL) gradient of every DISTINCT local partition with coefficient 1
// (grad_sparse.hip): row pass -> u, deterministic CSC tile pass -> Gb [nparts][ld]; the launcher's
// device encoding then forms the messages (encode.hip).  Host tables: ops/grad.py SparseGradPlan.
struct SparseArgs {
  // pass 1: rows (all distinct rows, partitions concatenated)
  int ell;                      // 1: ELL (constant nnz m per row), 0: CSR
  int idx16;                    // ELL: uint16 offsets into window lo[k] (else int32 columns)
  int m;                        // ELL nnz per row
  long long nrows;
  const void* ell_idx;          // [m][ell_ld] uint16 | int32 (rows past nrows: padding)
  long long ell_ld;             // ELL row stride (>= nrows; even: the LDS row pass loads row pairs)
  const int* lo;                // [m] category window starts (idx16)
  const long long* row_ptr;     // CSR [nrows + 1]
  int csr_fixed;                // CSR with the same nnz in every row (one-hot data): that nnz, row_ptr unread; else 0
  const int* col_idx;           // CSR [nnz]
  const void* vals;             // ELL [m][ell_ld] or CSR [nnz] values; nullptr: pattern-only (1.0)
  const void* y;                // [nrows] labels (acc dtype)
  void* u;                      // [nrows] residual with coefficient 1 (acc dtype)
  // pass 2: CSC tiles of 512 entries
  int row16;                    // CSC row indices uint16 (partition-relative) | int32
  const void* crow;             // [entries] per partition sorted by (column, row), each partition padded to 512;
                                //   top bit: the entry starts a run (first of its column or of its tile)
  const void* cvals;            // [entries] values in CSC order; nullptr: pattern-only
  const int* col_ptr;           // [nparts][d + 1] partition-relative entry offsets
  const int4* tiles;            // [ntiles] (partition, base entry, column of the base entry, span flags 1 head / 2 tail)
  int ntiles;
  const long long* part_entry0; // [nparts] first (padded) entry of each partition
  const long long* part_row0;   // [nparts] first row of each partition
  const int* part_nnz;          // [nparts]
  void* head;                   // [ntiles] partial sums of columns reaching back into earlier tiles
  void* tail;                   // [ntiles] partial sums of columns going on in later tiles
  // pass 3: columns crossing tiles and empty columns
  const int4* span;             // [nspan] (partition, column, first tile, last tile)
  int nspan;
  const int2* empty;            // [nempty] (partition, column)
  int nempty;
  void* Gb;                     // [nparts][ld] output (acc dtype)
  int d, ld;
  // row-blocked column pass (ops/grad.py csc_tables row_block): the "partitions" of pass 2 / 3 above
  // are sub-blocks of rows; wg == nullptr: one wave per tile gathering the residuals from memory
  const int4* wg;               // [nwg] (first row of the sub-block, first tile, tiles <= 16, rows): one workgroup each
  int nwg;
  int u_lds;                    // rows of the largest sub-block (its residuals staged in LDS)
  void* Gs;                     // [nsub][ld] pass 2 / 3 output (== Gb without sub-blocks)
  const int* sub_begin;         // [nparts + 1] sub-blocks of each partition; nullptr: Gs is Gb
  int nparts;
  int encode_from_subs;         // 1: the encoding that follows adds the sub-block sums itself (no sub_reduce)
  const int* runs;              // row-blocked pass: the column of every run (CSC rows flag run starts), per tile
  const int4* tkeys;            // [ntiles] (first run, n | runs << 10 | span flags << 20, sub-block, first column)
  // column-aligned chunks (csc_tables wg_spans): workgroup k adds its own crossing columns
  // wspan[wspan_ptr[k] .. wspan_ptr[k + 1]) = (sub-block, column, first, last tile of the chunk) from
  // LDS after its tiles; nullptr: heads / tails go through memory to csc_spans
  const int4* wspan;
  const int* wspan_ptr;         // [nwg + 1]
  // shared message rows (ops/grad.py SparseGradPlan units): the column pass writes sub-block p's sums to
  // rows dst[p][0..] of Gs (at most kSparseMaxDst, -1 padded) instead of row p: every replica of an
  // identical message (an FRC / AGC group's members) gets its row from the one pass over its rows
  const int* dst;
};
constexpr int kSparseMaxDst = 4;
hipError_t grad_sparse_launch(int dtype, int loss, const SparseArgs& a, const void* beta, hipStream_t st,
                              const int* gate = nullptr);

// layout probes of the bf16 MFMA gradient (grad_mfma.hip): one 16x16x32 product; one transposing read
hipError_t mfma_probe_launch(const float* A, const float* B, float* C, hipStream_t st);
hipError_t tr_probe_launch(const float* tile, int rowlen, float* out, hipStream_t st);

// ---- device encoding of shared-partition gradients (encode.hip) ---------------------------
// G[slot] = sum_{k in [ptr[slot], ptr[slot+1])} coef[k] * Gb[idx[k]]; dtype 0 fp64, 1 fp32
hipError_t encode_messages_launch(int dtype, const void* Gb, const int* ptr, const int* idx, const double* coef,
                                  void* G, int nslots, int ld, hipStream_t st, const int* gate = nullptr,
                                  const int* sub_begin = nullptr);

// ---- post-hoc evaluation GEMM (eval.hip) -----------------------------------------------
hipError_t eval_gemm_loss_launch(int x_dtype, int loss_kind, const void* X, long long ldx,
                                 long long n, int d, const void* y, const void* B, int ldb,
                                 int R, double* loss, void* P, hipStream_t st);

// ---- post-hoc evaluation over CSR / one-hot rows (eval_sparse.hip) ---------------------------
// Bt: betas transposed [ld, R] (R <= 256); vals == nullptr: pattern-only; dtype 0 fp64, 1 fp32
hipError_t eval_csr_loss_launch(int dtype, int loss_kind, const long long* row_ptr, const int* col, const void* vals,
                                long long n, const void* y, const void* Bt, int R, double* loss, void* P,
                                hipStream_t st);

// ---- master combine + update (update.hip) -----------------------------------------------
constexpr int kMaxMsgs = 128;
struct CombineArgs {
  const void* msg[kMaxMsgs];
  double coef[kMaxMsgs];
  int nmsg;
};
// One device-driven local round's decode-combine + update fused into the gradient's slab reduction
// (grad_dense_update_launch): the decoded messages are rows of this launch's G.
struct LocalUpdate {
  int nmsg;
  int slot[kMaxMsgs];        // G row of every decoded message, in combine order
  double coef[kMaxMsgs];
  double* beta;              // [ld] fp64 master state
  double* u;                 // [ld] AGD state
  double* hist;              // [ld] this round's history row
  void* beta_w;              // [ld] next round's worker beta (message dtype)
  long long* stamp;          // device time the round's messages were all reduced (or nullptr)
  int d, rule;
  double decay, gm, l2, theta;
};
// Gradient + slab reduction + combine + GD/AGD update in three launches (grad_dense.hip
// slab_final_update); bitwise equal to grad_dense_launch followed by combine_update_launch.
hipError_t grad_dense_update_launch(int dtype, int loss, int cpl, const void* segs, const void* tasks, int ntasks,
                                    const void* beta, void* slab, const int* slot_task_begin, int nslots, void* part,
                                    void* G, int ld, hipStream_t st, const KernelChoice& k, const LocalUpdate& up);

// msg dtype / worker-beta dtype: 0 fp64, 1 fp32; rule 0 GD, 1 AGD
hipError_t combine_update_launch(const CombineArgs& args, int msg_dtype, int w_dtype,
                                 double* beta, double* u, double* hist, void* beta_w,
                                 double* g_out, int d, int ld, double decay, double gm,
                                 double l2, double theta, int rule, hipStream_t st,
                                 long long* stamp = nullptr);
// one device timestamp (wall_clock64, hipDeviceAttributeWallClockRate kHz) into *out
hipError_t stamp_launch(long long* out, hipStream_t st);

// ---- IPC mailbox put + signal (transport.hip) -------------------------------------------
constexpr int kMaxPuts = 16;
struct PutDesc {
  const void* src;
  void* dst;
  long long bytes;            // multiple of 16
  unsigned long long* flag;   // device-accessible address of the flag (host-registered shm)
  unsigned long long value;   // flag value announced once the payload is visible
  unsigned int* counter;      // per-descriptor block counter (device memory, zero between launches)
  // Integrity tag (integrity.h), off when tag == nullptr: one MsgTag per payload row is written
  // into the receiver's tag slots before the flag.  csum: per-row sender scratch [rows] (zero
  // between launches); rows <= kMaxTagRows; es: element bytes (4 / 8); corrupt: test hook that
  // flips one payload byte after the checksum (a torn put the receiver must catch).
  MsgTag* tag;
  unsigned long long* csum;
  int rows;
  int es;
  unsigned int rank;
  int corrupt;
  // Abort word (host-mapped, nullptr = none): once non-zero, the put and its signal are skipped
  // (a pump that gave up releases its queued stream waits without announcing stale rounds).
  const int* abort;
  // Stale-round gate of a lazy-drain worker round (engine.cpp WorkerPump::set_skip_stale; nullptr =
  // off).  gate: this round's word (common.h gate_closed): nonzero = the round was skipped, nothing
  // is put or announced.  next_gate: the next round's word, decided by this launch once (after the
  // signal, or at once when skipped): 1 iff the worker's beta counter (beta_flag, its device address)
  // has reached stale_next, i.e. the master published the beta AFTER the next round's, so the next
  // round is stale before it starts (the replacement of the reference's send Cancel, ref
  // src/coded.py:178-180: a late worker jumps to the newest beta instead of computing stale rounds).
  const int* gate;
  int* next_gate;
  const unsigned long long* beta_flag;
  unsigned long long stale_next;
  int strict;  // set by the launchers from strict_release() (common.h block_release_system)
  // Landing stamp (nullptr = off): the last block writes {value, wall_clock64} here just before the
  // flag's release, so a receiver that sees the flag at `value` reads when that put landed on the
  // sender's clock (the collector orders physically late ranks' messages by it: csrc/runtime/
  // collector.h "Device times"); the value tells a slot of this round from one an older round (or a
  // skipped round) left.  stamp: the receiver-visible 16-byte slot (host-mapped ring); stamp_log: the
  // sender's own per-round record (ticks only).
  long long* stamp;
  long long* stamp_log;
};
#if defined(__HIPCC__)
// The landing stamp of a put (one thread of the last block, before the release that precedes the flag).
__device__ __forceinline__ void put_stamp(const PutDesc& p) {
  if (!p.stamp && !p.stamp_log) return;
  const long long t = static_cast<long long>(wall_clock64());
  if (p.stamp) {
    p.stamp[0] = static_cast<long long>(p.value);
    p.stamp[1] = t;
  }
  if (p.stamp_log) *p.stamp_log = t;
}
// The next round's gate word (one thread of the launch calls it).
__device__ __forceinline__ void put_decide_next_gate(const PutDesc& p) {
  if (!p.next_gate) return;
  const unsigned long long b =
      __hip_atomic_load(const_cast<unsigned long long*>(p.beta_flag), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(p.next_gate, b >= p.stale_next ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
#endif
struct PutArgs {
  PutDesc d[kMaxPuts];
  int n;
};
hipError_t put_signal_launch(const PutArgs& args, int blocks, hipStream_t st);
hipError_t signal_launch(unsigned long long* flag, unsigned long long value, hipStream_t st);
// *gate = (*counter >= at_least), one thread, stream-ordered (a p2p worker round's stale-round gate).
hipError_t gate_launch(const unsigned long long* counter, unsigned long long at_least, int* gate, hipStream_t st);

// Receiver-side check of the tagged rows of one put (integrity.h): rows [nrows][ld] of es-byte
// elements against tags[nrows] for counter value round1 and sender `rank`; first failure -> err.
hipError_t verify_rows_launch(const void* rows, const MsgTag* tags, int nrows, int ld, int es,
                              unsigned int round1, unsigned int rank, IntegrityErr* err, int where,
                              hipStream_t st);
// Deferred check of the mailbox rows one round decoded (integrity.h CheckList): one workgroup,
// one wave per row; the first mismatch goes to err (host-mapped).
hipError_t check_list_launch(const CheckList& cl, IntegrityErr* err, hipStream_t st);
// Transport preflight ping-pong (transport.hip ping_pong), one block per side.
struct PingArgs {
  unsigned long long* out_row;       // the row this side writes (the peer's memory)
  const unsigned long long* in_row;  // the row this side reads (its own memory)
  int nwords_out, nwords_in;         // 64-bit words per row (0: counters only)
  unsigned long long* out_flag;      // counter this side release-stores
  const unsigned long long* in_flag; // counter this side polls
  int iters;
  long long deadline_ticks;          // per wait (wall_clock64 ticks)
  long long* rtt;                    // [iters] master: ticks from its store to the echo (nullptr: worker)
  int* status;                       // [2]: payload words that differed, 1 on a timeout
};
hipError_t ping_pong_launch(const PingArgs& a, bool master, hipStream_t st);
// Spin on the device for `ticks` wall_clock64 ticks (a physically late worker, --delay-on worker), after
// the round's gradient and before its put; a skipped round (gate_closed) does not spin, and a spin
// ends early once *stop >= stop_at (the master's end-of-run release of a lazy-drain run).
// rec (nullptr = off): [start, end] of the spin in wall_clock64 ticks (not written when the gate is closed).
hipError_t spin_launch(long long ticks, hipStream_t st, const int* gate = nullptr,
                       const unsigned long long* stop = nullptr, unsigned long long stop_at = 0,
                       long long* rec = nullptr);

}  // namespace eh
