// Native round executors: the master's and the IPC workers' per-round hot loops in C++.
//
// Reference loop (every engine, ref src/naive.py:88-150, src/approximate_coding.py:136-207):
//   master: Isend beta to all -> Waitany until the stop rule -> decode -> GD/AGD update
//   worker: Wait(beta) -> gradient -> [delay] -> Isend(g)
// On the MI355X the Python engine (erasurehead_amd/engine/trainer.py) owns setup and
// bookkeeping, while these executors run the latency-critical part of a round with the
// GIL released and no per-call Python overhead:
//
//  MasterPump::finish(i)  wait for the stop rule (Collector) -> decode on the host
//                         (plain sum / first arrival per FRC group / cyclic-MDS
//                         coefficients from a bitmask table) -> combine+update launch
//                         -> [drain] -> begin(i+1): push beta(i+1) to every worker
//                         inbox (put+signal), launch the master's own workers'
//                         gradient, register the round's arrival probes.
//  WorkerPump::run(a, b)  for each round: spin on the beta round counter, launch the
//                         gradient of every local logical worker, put+signal the
//                         messages into the master's mailbox ring.
//
// Everything is stream-ordered on the rank's compute stream; the only host waits are the
// collector's poll and the worker's beta counter.
#include <c10/hip/HIPStream.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdlib>

#include "kernels/arbiter.h"
#include "kernels/grad_dense.h"
#include "kernels/launchers.h"
#include "runtime/collector.h"
#include "runtime/comm.h"

namespace {

// roctx ranges for rocprofv3 --marker-trace, enabled by ERASUREHEAD_TRACE=1.
bool trace_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("ERASUREHEAD_TRACE");
    return e && e[0] && e[0] != '0';
  }();
  return on;
}

struct Range {
  explicit Range(const char* name) : on(trace_enabled()) {
    if (on) roctxRangePushA(name);
  }
  ~Range() {
    if (on) roctxRangePop();
  }
  bool on;
};

namespace py = pybind11;
using at::Tensor;

void hcheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

void need(bool ok, const std::string& msg) {
  if (!ok) throw std::invalid_argument(msg);
}

int acc_code(const Tensor& t) {
  if (t.scalar_type() == at::kDouble) return 0;
  if (t.scalar_type() == at::kFloat) return 1;
  throw std::invalid_argument("accumulator tensors must be float64 or float32");
}

void need_gpu(const Tensor& t, const char* name) {
  need(t.is_cuda() && t.is_contiguous(), std::string(name) + " must be a contiguous GPU tensor");
}

// ------------------------------------------------------------------------ GradLauncher
// The per-round gradient launch of one rank's local messages, captured once from the
// Python plan (ops/grad.py).  The plan object keeps every referenced tensor alive; the
// launcher also holds references.
struct GradLauncher {
  int kind = 0;  // 0 dense fused, 1 dense two-pass, 2 sparse
  int dtype = 0, loss = 0, cpl = 0, ntasks = 0, nslots = 0, ld = 0;
  eh::KernelChoice choice{};
  const void* segs = nullptr;
  const void* tasks = nullptr;
  void* slab = nullptr;
  const int* stb = nullptr;
  void* part = nullptr;
  const int* task_row_off = nullptr;
  void* rbuf = nullptr;
  int acc = 0;
  eh::SparseArgs sa{};  // kind 2 (grad_sparse.hip); Gb is the launch's output
  // optional device encoding (csrc/kernels/encode.hip): the kernels above write the distinct
  // partitions' gradients into Gb, then G[slot] = sum_k coef * Gb[idx] for the enc_slots messages
  void* Gb = nullptr;
  const int* enc_ptr = nullptr;
  const int* enc_idx = nullptr;
  const double* enc_coef = nullptr;
  int enc_slots = 0;
  std::vector<Tensor> keep;

  // gate: a lazy-drain worker round's stale-round gate (common.h gate_closed); nullptr = always run
  hipError_t launch(const void* beta, void* G, hipStream_t st, const int* gate = nullptr) const {
    if (!Gb) return launch_raw(beta, G, st, gate);
    if (kind == 2 && sa.sub_begin) {  // row-blocked sparse pass: the encoding adds the sub-block sums
      eh::SparseArgs a = sa;
      a.Gb = Gb;
      a.encode_from_subs = 1;
      const hipError_t e = eh::grad_sparse_launch(acc, loss, a, beta, st, gate);
      if (e != hipSuccess) return e;
      return eh::encode_messages_launch(acc, sa.Gs, enc_ptr, enc_idx, enc_coef, G, enc_slots, ld, st, gate,
                                        sa.sub_begin);
    }
    const hipError_t e = launch_raw(beta, Gb, st, gate);
    if (e != hipSuccess) return e;
    return eh::encode_messages_launch(acc, Gb, enc_ptr, enc_idx, enc_coef, G, enc_slots, ld, st, gate);
  }

  // Dense fused plans without device encoding can hand their result rows straight to the
  // receiver's mailbox from the final reduction kernel (grad_dense.hip slab_reduce_final_put).
  bool can_fuse_put(int rows) const { return kind == 0 && !Gb && ntasks > 0 && nslots == rows; }
  // Device-driven local rounds: the combine + update ride the slab reduction (grad_dense_update_launch).
  bool can_fuse_update() const { return kind == 0 && !Gb && ntasks > 0; }
  hipError_t launch_update(const void* beta, void* G, const eh::LocalUpdate& up, hipStream_t st) const {
    return eh::grad_dense_update_launch(dtype, loss, cpl, segs, tasks, ntasks, beta, slab, stb, nslots, part, G, ld,
                                        st, choice, up);
  }
  hipError_t launch_put(const void* beta, void* G, const eh::PutDesc& put, hipStream_t st) const {
    return eh::grad_dense_launch(dtype, loss, cpl, segs, tasks, ntasks, beta, slab, stb, nslots, part, G, ld, st,
                                 choice, &put, put.gate);
  }

  hipError_t launch_raw(const void* beta, void* G, hipStream_t st, const int* gate = nullptr) const {
    switch (kind) {
      case 0:
        return ntasks ? eh::grad_dense_launch(dtype, loss, cpl, segs, tasks, ntasks, beta, slab, stb, nslots, part, G,
                                              ld, st, choice, nullptr, gate)
                      : hipSuccess;
      case 1:
        return ntasks ? eh::grad_dense_twopass_launch(dtype, loss, segs, tasks, ntasks, beta, task_row_off, rbuf, slab,
                                                      stb, nslots, part, G, ld, st, gate)
                      : hipSuccess;
      case 2: {
        eh::SparseArgs a = sa;
        a.Gb = G;
        if (!a.sub_begin) a.Gs = G;  // no sub-blocks: pass 2 / 3 write the partitions directly
        return eh::grad_sparse_launch(acc, loss, a, beta, st, gate);
      }
      default:
        return hipErrorInvalidValue;
    }
  }
};

std::shared_ptr<GradLauncher> make_dense(int64_t dtype, int64_t loss, int64_t cpl, const Tensor& segs,
                                         const Tensor& tasks, const Tensor& slab, const Tensor& stb,
                                         const Tensor& part, int64_t ld, std::optional<Tensor> task_row_off,
                                         std::optional<Tensor> rbuf, const eh::KernelChoice& choice) {
  for (auto* t : {&segs, &tasks, &slab, &stb, &part}) need_gpu(*t, "dense plan operand");
  need(tasks.dim() == 2 && tasks.size(1) == 5 && tasks.scalar_type() == at::kInt, "tasks must be int32 [n,5]");
  need(stb.scalar_type() == at::kInt, "slot_task_begin must be int32");
  auto g = std::make_shared<GradLauncher>();
  g->dtype = (int)dtype;
  g->loss = (int)loss;
  g->cpl = (int)cpl;
  g->choice = choice;
  g->ld = (int)ld;
  g->ntasks = (int)tasks.size(0);
  g->nslots = (int)stb.numel() - 1;
  need(part.numel() * part.element_size() >= eh::slab_part_bytes(g->nslots, ld, dtype == 0 ? 8 : 4),
       "part must hold the slab partial sums (grad.py DenseGradPlan)");
  g->segs = segs.data_ptr();
  g->tasks = tasks.data_ptr();
  g->slab = slab.data_ptr();
  g->stb = stb.data_ptr<int>();
  g->part = part.data_ptr();
  g->keep = {segs, tasks, slab, stb, part};
  g->acc = dtype == 0 ? 0 : 1;
  if (task_row_off) {
    need(rbuf.has_value(), "two-pass plan needs rbuf");
    need_gpu(*task_row_off, "task_row_off");
    need_gpu(*rbuf, "rbuf");
    g->kind = 1;
    g->task_row_off = task_row_off->data_ptr<int>();
    g->rbuf = rbuf->data_ptr();
    g->keep.push_back(*task_row_off);
    g->keep.push_back(*rbuf);
  } else {
    need(cpl <= 32 ? cpl * 64 >= ld
                   : ((cpl == 256 || cpl == 512) && cpl * (dtype == 0 ? 16 : 32) >= ld),
         "cpl (narrow: columns per lane, wide: block size) must cover ld");
    g->kind = 0;
  }
  return g;
}

// Sparse plan (ops/grad.py SparseGradPlan): every distinct local partition once; the plan's device
// encoding (set_encode) forms the messages.  Tensors are kept alive by the launcher.
std::shared_ptr<GradLauncher> make_sparse(int64_t loss, const Tensor& y, const Tensor& u, std::optional<Tensor> ell_idx,
                                          std::optional<Tensor> lo, std::optional<Tensor> row_ptr,
                                          std::optional<Tensor> col_idx, std::optional<Tensor> vals, const Tensor& crow,
                                          std::optional<Tensor> cvals, const Tensor& col_ptr, const Tensor& tiles,
                                          const Tensor& part_entry0, const Tensor& part_row0, const Tensor& part_nnz,
                                          const Tensor& head, const Tensor& tail, const Tensor& span,
                                          const Tensor& empty, int64_t nparts, int64_t d, int64_t ld,
                                          std::optional<Tensor> wg, int64_t u_lds, std::optional<Tensor> Gs,
                                          std::optional<Tensor> sub_begin, std::optional<Tensor> runs,
                                          std::optional<Tensor> tkeys, std::optional<Tensor> wspan,
                                          std::optional<Tensor> wspan_ptr, std::optional<Tensor> dst, int64_t csr_fixed) {
  for (auto* t : {&y, &u, &crow, &col_ptr, &tiles, &part_entry0, &part_row0, &part_nnz, &head, &tail, &span, &empty})
    need_gpu(*t, "sparse plan operand");
  need(tiles.scalar_type() == at::kInt && tiles.dim() == 2 && tiles.size(1) == 4, "tiles: int32 [n, 4]");
  need(span.scalar_type() == at::kInt && span.dim() == 2 && span.size(1) == 4, "span: int32 [n, 4]");
  need(empty.scalar_type() == at::kInt && empty.dim() == 2 && empty.size(1) == 2, "empty: int32 [n, 2]");
  need(col_ptr.scalar_type() == at::kInt && col_ptr.numel() == nparts * (d + 1), "col_ptr: int32 [nparts, d + 1]");
  need(part_entry0.scalar_type() == at::kLong && part_row0.scalar_type() == at::kLong &&
           part_nnz.scalar_type() == at::kInt && part_nnz.numel() == nparts,
       "partition offsets");
  need(crow.scalar_type() == at::kShort || crow.scalar_type() == at::kInt, "crow: int16 | int32");
  auto g = std::make_shared<GradLauncher>();
  g->kind = 2;
  g->loss = (int)loss;
  g->acc = acc_code(y);
  need(acc_code(u) == g->acc && acc_code(head) == g->acc && acc_code(tail) == g->acc, "acc dtype mismatch");
  g->ld = (int)ld;
  g->nslots = (int)nparts;
  eh::SparseArgs& a = g->sa;
  a.nrows = y.numel();
  a.y = y.data_ptr();
  a.u = u.data_ptr();
  g->keep = {y, u, crow, col_ptr, tiles, part_entry0, part_row0, part_nnz, head, tail, span, empty};
  if (ell_idx) {
    need_gpu(*ell_idx, "ell_idx");
    need(ell_idx->dim() == 2 && ell_idx->size(1) >= a.nrows, "ell_idx: [m, >= rows]");
    a.ell_ld = ell_idx->size(1);
    a.ell = 1;
    a.idx16 = ell_idx->scalar_type() == at::kShort ? 1 : 0;
    need(a.idx16 || ell_idx->scalar_type() == at::kInt, "ell_idx: int16 | int32");
    a.m = (int)ell_idx->size(0);
    a.ell_idx = ell_idx->data_ptr();
    if (a.idx16) {
      need(lo.has_value() && lo->numel() == a.m && lo->scalar_type() == at::kInt, "lo: int32 [m]");
      need_gpu(*lo, "lo");
      a.lo = lo->data_ptr<int>();
      g->keep.push_back(*lo);
    }
    g->keep.push_back(*ell_idx);
  } else {
    need(row_ptr.has_value() && col_idx.has_value(), "CSR row pass needs row_ptr / col_idx");
    need_gpu(*row_ptr, "row_ptr");
    need_gpu(*col_idx, "col_idx");
    need(row_ptr->scalar_type() == at::kLong && row_ptr->numel() == a.nrows + 1, "row_ptr: int64 [rows + 1]");
    a.row_ptr = reinterpret_cast<const long long*>(row_ptr->data_ptr<int64_t>());
    a.col_idx = col_idx->data_ptr<int>();
    need(csr_fixed >= 0 && (csr_fixed == 0 || col_idx->numel() == csr_fixed * a.nrows), "csr_fixed: nnz of every row");
    a.csr_fixed = (int)csr_fixed;
    g->keep.push_back(*row_ptr);
    g->keep.push_back(*col_idx);
  }
  if (vals) {
    need_gpu(*vals, "vals");
    need(acc_code(*vals) == g->acc, "vals dtype");
    need(!ell_idx || vals->sizes() == ell_idx->sizes(), "ELL vals: the shape of ell_idx");
    a.vals = vals->data_ptr();
    g->keep.push_back(*vals);
  }
  a.row16 = crow.scalar_type() == at::kShort ? 1 : 0;
  a.crow = crow.data_ptr();
  if (cvals) {
    need_gpu(*cvals, "cvals");
    need(acc_code(*cvals) == g->acc && cvals->numel() == crow.numel(), "cvals: acc dtype, one per CSC entry");
    a.cvals = cvals->data_ptr();
    g->keep.push_back(*cvals);
  }
  a.col_ptr = col_ptr.data_ptr<int>();
  a.tiles = reinterpret_cast<const int4*>(tiles.data_ptr<int>());
  a.ntiles = (int)tiles.size(0);
  need(crow.numel() >= static_cast<int64_t>(a.ntiles) * 512, "crow: every partition padded to whole 512-entry tiles");
  need(head.numel() >= a.ntiles && tail.numel() >= a.ntiles, "head / tail: one per tile");
  a.part_entry0 = reinterpret_cast<const long long*>(part_entry0.data_ptr<int64_t>());
  a.part_row0 = reinterpret_cast<const long long*>(part_row0.data_ptr<int64_t>());
  a.part_nnz = part_nnz.data_ptr<int>();
  a.head = head.data_ptr();
  a.tail = tail.data_ptr();
  a.span = reinterpret_cast<const int4*>(span.data_ptr<int>());
  a.nspan = (int)span.size(0);
  a.empty = reinterpret_cast<const int2*>(empty.data_ptr<int>());
  a.nempty = (int)empty.size(0);
  a.d = (int)d;
  a.ld = (int)ld;
  if (wg) {  // row-blocked column pass: `nparts` above counts sub-blocks
    need_gpu(*wg, "wg");
    need(wg->scalar_type() == at::kInt && wg->dim() == 2 && wg->size(1) == 4, "wg: int32 [n, 4]");
    need(u_lds > 0 && u_lds * (g->acc == 0 ? 8 : 4) <= 96 * 1024, "u_lds: sub-block rows staged in LDS (<= 96 KB)");
    {  // the column pass's chunks: 1..128 tiles each (grad_sparse.hip kMaxWgTiles), rows staged in LDS
      const Tensor wc = wg->cpu();
      const int* W = wc.data_ptr<int>();
      for (int64_t k = 0; k < wg->size(0); ++k)
        need(W[4 * k + 2] >= 1 && W[4 * k + 2] <= 128 && W[4 * k + 1] >= 0 && W[4 * k + 1] + W[4 * k + 2] <= tiles.size(0) &&
                 W[4 * k + 3] <= u_lds,
             "wg: (row0, first tile, 1..128 tiles, rows <= u_lds)");
    }
    a.wg = reinterpret_cast<const int4*>(wg->data_ptr<int>());
    a.nwg = (int)wg->size(0);
    a.u_lds = (int)u_lds;
    g->keep.push_back(*wg);
    need(runs.has_value() && tkeys.has_value(), "the row-blocked column pass needs the run lists (runs, tkeys)");
    need_gpu(*runs, "runs");
    need_gpu(*tkeys, "tkeys");
    need(runs->scalar_type() == at::kInt && runs->numel() >= 1, "runs: int32 [runs]");
    need(tkeys->scalar_type() == at::kInt && tkeys->dim() == 2 && tkeys->size(0) == a.ntiles && tkeys->size(1) == 4,
         "tkeys: int32 [tiles, 4]");
    a.runs = runs->data_ptr<int>();
    a.tkeys = reinterpret_cast<const int4*>(tkeys->data_ptr<int>());
    g->keep.push_back(*runs);
    g->keep.push_back(*tkeys);
    if (wspan_ptr) {  // column-aligned chunks: every crossing column summed inside its workgroup
      need(wspan.has_value(), "wspan_ptr needs wspan");
      need_gpu(*wspan, "wspan");
      need_gpu(*wspan_ptr, "wspan_ptr");
      need(a.nspan == 0, "column-aligned chunks leave no global spans");
      need(wspan->scalar_type() == at::kInt && wspan->dim() == 2 && wspan->size(1) == 4, "wspan: int32 [n, 4]");
      need(wspan_ptr->scalar_type() == at::kInt && wspan_ptr->numel() == a.nwg + 1, "wspan_ptr: int32 [workgroups + 1]");
      // the kernel indexes its LDS head / tail arrays with these: checked once, on the host
      const Tensor sp = wspan->cpu(), pp = wspan_ptr->cpu(), wc = wg->cpu();
      const int* P = pp.data_ptr<int>();
      const int* S = sp.data_ptr<int>();
      const int* W = wc.data_ptr<int>();
      need(P[0] == 0 && P[a.nwg] == sp.size(0), "wspan_ptr: [0, .., spans]");
      for (int k = 0; k < a.nwg; ++k) {
        need(P[k] <= P[k + 1] && P[k + 1] - P[k] < 128, "wspan_ptr: non-decreasing, < 128 spans per workgroup");
        for (int i = P[k]; i < P[k + 1]; ++i) {
          const int* e = S + 4 * i;
          need(e[0] >= 0 && e[0] < nparts && e[1] >= 0 && e[1] < d && e[2] >= 0 && e[2] < e[3] && e[3] < W[4 * k + 2],
               "wspan: (sub-block, column, first tile < last tile < the workgroup's tiles)");
        }
      }
      a.wspan = reinterpret_cast<const int4*>(wspan->data_ptr<int>());
      a.wspan_ptr = wspan_ptr->data_ptr<int>();
      g->keep.push_back(*wspan);
      g->keep.push_back(*wspan_ptr);
    }
  }
  if (dst) {  // shared message rows of merged FRC / AGC units (ops/grad.py SparseGradPlan.units)
    need_gpu(*dst, "dst");
    need(!sub_begin && wg && a.nspan == 0, "shared message rows need unblocked units and the row-blocked column pass");
    need(dst->scalar_type() == at::kInt && dst->dim() == 2 && dst->size(0) == nparts &&
             dst->size(1) == eh::kSparseMaxDst,
         "dst: int32 [units, 4]");
    const Tensor dc = dst->cpu();
    const int* D = dc.data_ptr<int>();
    for (int64_t k = 0; k < dst->numel(); ++k) need(D[k] >= -1 && D[k] < 4096, "dst: message rows or -1");
    a.dst = dst->data_ptr<int>();
    g->keep.push_back(*dst);
  }
  if (sub_begin) {
    need(Gs.has_value(), "sub-blocks need their Gs buffer");
    need_gpu(*sub_begin, "sub_begin");
    need_gpu(*Gs, "Gs");
    need(sub_begin->scalar_type() == at::kInt && sub_begin->numel() >= 2, "sub_begin: int32 [partitions + 1]");
    need(Gs->dim() == 2 && Gs->size(0) == nparts && Gs->size(1) == ld && acc_code(*Gs) == g->acc,
         "Gs: [sub-blocks, ld] in the accumulator dtype");
    a.sub_begin = sub_begin->data_ptr<int>();
    a.nparts = (int)sub_begin->numel() - 1;
    a.Gs = Gs->data_ptr();
    g->nslots = a.nparts;  // Gb rows: the partitions
    g->keep.push_back(*sub_begin);
    g->keep.push_back(*Gs);
  }
  return g;
}

// One buffer row a decode uses: its address, coefficient and, for a mailbox row, its row index
// (its integrity tag; -1 for a local row).
struct Used {
  const void* p;
  double c;
  int row;
};
using UsedRows = std::vector<Used>;

// Host-mapped integrity record (integrity.h) and abort word of a pump.
struct HostMapped {
  void* host = nullptr;
  void* dev = nullptr;
  explicit HostMapped(size_t bytes) {
    hcheck(hipHostMalloc(&host, bytes, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
    std::memset(host, 0, bytes);
    hcheck(hipHostGetDevicePointer(&dev, host, 0), "hipHostGetDevicePointer");
  }
  ~HostMapped() {
    if (host) hipHostFree(host);
  }
  HostMapped(const HostMapped&) = delete;
  HostMapped& operator=(const HostMapped&) = delete;
};

// Test hook ERASUREHEAD_SABOTAGE=<what>:<rank>:<round> (what: msg | beta): the named put flips one
// payload byte after its checksum, so the receiver must report a torn message.  ("handshake:<rank>":
// that rank never answers the IPC handshake, parallel/transport.py.)  Read at every put, so a test can
// arm it for one Trainer of a process and disarm it before the next (bench.py first-contact ladder).
bool sabotage(const char* what, int rank, int round) {
  const char* e = std::getenv("ERASUREHEAD_SABOTAGE");
  if (e == nullptr || e[0] == '\0') return false;
  const std::string spec(e);
  return spec == std::string(what) + ":" + std::to_string(rank) + ":" + std::to_string(round);
}

std::string integrity_message(const eh::IntegrityErr& e, bool beta) {
  char buf[512];
  if (beta)
    std::snprintf(buf, sizeof(buf),
                  "message integrity check failed: beta of round %d from rank %d: tag says round %d rank %u "
                  "checksum %016llx, payload checksum %016llx",
                  e.round, e.rank_want, static_cast<int>(e.round1_got) - 1, e.rank_got, e.sum_got, e.sum_calc);
  else
    std::snprintf(buf, sizeof(buf),
                  "message integrity check failed: round %d, rank %d's message in mailbox slot %d row %d: tag says "
                  "round %d rank %u checksum %016llx, payload checksum %016llx",
                  e.round, e.rank_want, e.where >> 16, e.where & 0xffff, static_cast<int>(e.round1_got) - 1, e.rank_got,
                  e.sum_got, e.sum_calc);
  return buf;
}

// Decode kinds (codes/schemes.py)
enum DecodeKind : int {
  kSumPart0 = 0,       // naive, avoidstragg: every arrived main message, coefficient 1
  kFirstPerGroup = 1,  // FRC / AGC: first arrival of each group
  kPartialFrc = 2,     // partial replication: all first parts + first second part per group
  kTable = 3,          // cyclic MDS: coefficients from the completion-bitmask table
  kPartialTable = 4,   // partial coded: all first parts + table-decoded coded parts
};

// ------------------------------------------------------------------------- MasterPump
class MasterPump {
 public:
  MasterPump(eh::Collector* col, int W, int R, int K, int d, int ld, int device, double timeout)
      : col_(col), W_(W), R_(R), K_(K), d_(d), ld_(ld), device_(device), timeout_(timeout) {
    need(col != nullptr, "collector required");
    need(W > 0 && R > 0 && K > 0 && ld >= d && d > 0, "bad pump dimensions");
    stream_ = c10::hip::getCurrentHIPStream(device).stream();
    t_start_.assign(R, 0.0);
    upd_ev_.assign(R, {nullptr, nullptr});
    loc_ev_.assign(K, nullptr);
    for (auto& e : loc_ev_) hcheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    index_.assign(2 * W, {});
    err_ = std::make_unique<HostMapped>(sizeof(eh::IntegrityErr));
    const auto i64 = at::TensorOptions().dtype(at::kLong).device(at::Device(at::kCUDA, device));
    csum_ = at::zeros({eh::kMaxPuts * eh::kMaxTagRows}, i64);  // beta put checksums
  }
  ~MasterPump() {
    if (chk_stream_) {
      hipStreamSynchronize(chk_stream_);
      hipStreamDestroy(chk_stream_);
      hipEventDestroy(arb_ev_);
      hipEventDestroy(chk_ev_);
    }
    if (dev_stream_) {
      hipStreamSynchronize(dev_stream_);
      for (auto g : graphs_) hipGraphExecDestroy(g);
      hipStreamDestroy(dev_stream_);
      hipEventDestroy(join_ev_);
    }
    for (auto e : loc_ev_)
      if (e) hipEventDestroy(e);
    for (auto& p : upd_ev_) {
      if (p.first) hipEventDestroy(p.first);
      if (p.second) hipEventDestroy(p.second);
    }
    for (auto& t : tev_)
      for (auto e : t)
        if (e) hipEventDestroy(e);
    // per-peer comm streams: destroyed without a sync (a receive from a dead peer may never end;
    // the transport aborts its communicator at close)
    for (auto e : rev_)
      if (e) hipEventDestroy(e);
    if (bev_) hipEventDestroy(bev_);
    if (ref_ev_) hipEventDestroy(ref_ev_);
    for (auto& [r, st] : send_st_) hipStreamDestroy(st);
    for (auto& [r, st] : recv_st_)
      if (!send_st_.count(r) || send_st_.at(r) != st) hipStreamDestroy(st);  // a shared link stream once
  }

  // Per-round HIP-event timing of the beta puts and the local gradient launch (bench.py's
  // per-rank breakdown); off by default: each record costs the host about a microsecond.
  void set_timing(bool on) {
    timing_ = on;
    if (on && tev_.empty()) tev_.assign(R_, {nullptr, nullptr, nullptr, nullptr});
  }
  // (put_ms [R], kernel_ms [R]); -1 where a round was not timed.  Syncs the stream.
  std::pair<std::vector<double>, std::vector<double>> timing_ms() {
    hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    std::vector<double> put(R_, -1.0), ker(R_, -1.0);
    for (int i = 0; i < (int)tev_.size(); ++i) {
      const auto& t = tev_[i];
      float ms = 0.f;
      if (t[0] && t[1] && hipEventElapsedTime(&ms, t[0], t[1]) == hipSuccess) put[i] = ms;
      if (t[2] && t[3] && hipEventElapsedTime(&ms, t[2], t[3]) == hipSuccess) ker[i] = ms;
    }
    return {put, ker};
  }

  void set_state(const Tensor& beta, const Tensor& u, const Tensor& hist, const Tensor& beta_in) {
    arb_ready_ = false;  // the device arbiter copies this state
    need_gpu(beta, "beta");
    need_gpu(u, "u");
    need_gpu(hist, "hist");
    need_gpu(beta_in, "beta_in");
    need(beta.scalar_type() == at::kDouble && u.scalar_type() == at::kDouble && hist.scalar_type() == at::kDouble,
         "beta/u/hist must be float64");
    need(beta.numel() == ld_ && u.numel() == ld_, "beta/u must have ld elements");
    need(hist.dim() == 2 && hist.size(0) >= R_ && hist.size(1) == ld_, "hist must be [R, ld]");
    need(beta_in.dim() == 2 && beta_in.size(0) >= R_ + 1 && beta_in.size(1) == ld_, "beta_in must be [R+1, ld]");
    beta_ = beta;
    u_ = u;
    hist_ = hist;
    beta_in_ = beta_in;
    acc_ = acc_code(beta_in);
    es_ = acc_ == 0 ? 8 : 4;
  }

  // local messages: row order of G ([K, n_loc, ld]); each (worker, part).  A (worker, part) may
  // appear several times (partition shards of one message): decode sums all its rows.
  void set_local(std::shared_ptr<GradLauncher> g, const Tensor& G, const std::vector<std::pair<int, int>>& msgs) {
    arb_ready_ = false;  // the device arbiter copies this state
    need_gpu(G, "G");
    need(G.dim() == 3 && G.size(0) == K_ && G.size(2) == ld_, "G must be [K, n_loc, ld]");
    need(acc_code(G) == acc_, "G dtype must match beta_in");
    need((int64_t)msgs.size() <= G.size(1), "more local messages than G rows");
    launcher_ = std::move(g);
    G_ = G;
    n_loc_ = (int)msgs.size();
    g_rows_ = (int)G.size(1);
    local_.clear();
    for (auto& ix : index_)
      ix.erase(std::remove_if(ix.begin(), ix.end(), [](const std::pair<int, int>& e) { return e.first == 0; }),
               ix.end());
    for (int j = 0; j < n_loc_; ++j) {
      check_wp(msgs[j].first, msgs[j].second);
      local_.push_back({msgs[j].first, msgs[j].second, j, 0});
      index_[2 * msgs[j].first + msgs[j].second].push_back({0, j});
    }
  }

  // remote messages: (worker, part, mailbox row, host address of the sender's round counter, sender rank)
  void set_remote(const Tensor& rbuf, const std::vector<std::tuple<int, int, int, uintptr_t, int>>& msgs) {
    arb_ready_ = false;  // the device arbiter copies this state
    need_gpu(rbuf, "rbuf");
    need(rbuf.dim() == 3 && rbuf.size(0) == K_ && rbuf.size(2) == ld_, "rbuf must be [K, rows, ld]");
    need(acc_code(rbuf) == acc_, "rbuf dtype must match beta_in");
    rbuf_ = rbuf;
    r_rows_ = (int)rbuf.size(1);
    remote_.clear();
    row_rank_.assign(r_rows_, 0);
    for (auto& ix : index_)
      ix.erase(std::remove_if(ix.begin(), ix.end(), [](const std::pair<int, int>& e) { return e.first == 1; }),
               ix.end());
    for (const auto& [w, p, row, addr, rank] : msgs) {
      check_wp(w, p);
      need(row >= 0 && row < r_rows_, "mailbox row out of range");
      need(addr != 0 || comm_, "null flag address");
      need(rank > 0 && rank < 256, "sender rank out of range");
      remote_.push_back({w, p, row, addr});
      row_rank_[row] = rank;
      index_[2 * w + p].push_back({1, row});
    }
  }

  // Stream-ordered p2p instead of the IPC mailbox (runtime/comm.h: RCCL, or its single-GPU loopback):
  // ranks = (worker rank, first mailbox row, rows) of every rank that sends messages; `peers` = every
  // worker rank (each receives beta).  Call after set_skip_stale, before set_remote.  beta(i) goes out
  // with one send per peer on that peer's own stream; round i's messages of rank r arrive with one
  // receive into its mailbox rows, and the HIP event behind it is the collector's probe.
  //
  // Streams (each parks its own waits: a stream that shares a hardware queue would hold back the
  // other streams of that queue, so the count must stay within GPU_MAX_HW_QUEUES):
  //   drain all / carry  ONE link stream per peer, beta(i) send then round i's receive.  Per pair this
  //                      is the order both sides need anyway (a worker cannot use beta(i+1) before it
  //                      has sent round i), and a late peer still blocks only its own link: W - 1 + the
  //                      compute stream, 8 at 8 ranks.
  //   lazy               a send and a receive stream per peer: beta(i+1) must reach a late rank while its
  //                      round-i receive is still pending, so it can find round i stale (WorkerPump::
  //                      set_skip_stale_comm): 2 (W - 1) + 1, 15 at 8 ranks.
  void set_comm(std::shared_ptr<eh::P2PComm> comm, const std::vector<std::tuple<int, int, int>>& ranks,
                const std::vector<int>& peers) {
    need(comm != nullptr, "null communicator");
    arb_ready_ = false;
    comm_ = std::move(comm);
    comm_ranks_ = ranks;
    comm_peers_ = peers;
    auto mk = [](hipStream_t* st) { hcheck(hipStreamCreateWithFlags(st, hipStreamNonBlocking), "hipStreamCreate"); };
    for (int r : peers) mk(&send_st_[r]);
    for (const auto& [r, row0, n] : ranks) {
      need(n > 0 && row0 >= 0, "bad mailbox rows of a rank");
      if (!skip_ && send_st_.count(r))
        recv_st_[r] = send_st_.at(r);  // the pair's link stream
      else
        mk(&recv_st_[r]);
    }
    rev_.assign(static_cast<size_t>(K_) * ranks.size(), nullptr);
    for (auto& e : rev_) hcheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    if (!bev_) hcheck(hipEventCreateWithFlags(&bev_, hipEventDisableTiming), "hipEventCreate");
  }
  std::string comm_kind() const { return comm_ ? comm_->kind() : "ipc"; }

  // Integrity tags (csrc/kernels/integrity.h): mbox_tags = device address of the mailbox's tag
  // slots [K][rows]; inbox_tag_off = bytes from a worker inbox base to its tag slots [R + 1].
  // on = false keeps the transport untagged (A/B runs).
  void set_integrity(uintptr_t mbox_tags, int64_t inbox_tag_off, bool on) {
    arb_ready_ = false;
    need(!on || (mbox_tags != 0 && inbox_tag_off > 0), "integrity tags need the tag slots");
    tags_ = on;
    mbox_tags_ = mbox_tags;
    inbox_tag_off_ = inbox_tag_off;
  }
  bool integrity() const { return tags_; }

  // Raise the first integrity failure any deferred check of this pump reported (host-mapped record).
  int64_t check_rows_cut() const { return check_rows_cut_; }
  void check_integrity() const {
    const auto* e = static_cast<const eh::IntegrityErr*>(err_->host);
    if (__atomic_load_n(&e->flag, __ATOMIC_ACQUIRE)) throw std::runtime_error(integrity_message(*e, false));
  }
  // End of a run: check the last round's rows too, then raise any failure.  Syncs the stream.
  void final_check() {
    flush_check();
    hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    check_integrity();
  }

  // Device-side drain (after_combine): (host address, device address) of every worker rank's
  // message flag.  Empty = the host drains before pushing the next beta.
  // Returns whether the device-side drain is on (off when the device cannot wait on a value).
  bool set_drain_flags(const std::vector<std::pair<uintptr_t, uintptr_t>>& flags) {
    for (const auto& f : flags) need(f.first != 0 && f.second != 0, "null drain flag");
    int can = 0;
    const bool ok = hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, device_) == hipSuccess && can;
    drain_flags_ = ok ? flags : std::vector<std::pair<uintptr_t, uintptr_t>>{};
    return ok && !flags.empty();
  }

  // beta pushes: (inbox base device pointer [R+1, ld], flag device address) per worker rank
  void set_puts(const std::vector<std::pair<uintptr_t, uintptr_t>>& targets, const Tensor& counters) {
    arb_ready_ = false;  // the device arbiter copies this state
    need(counters.is_cuda() && counters.scalar_type() == at::kInt && counters.numel() >= (int64_t)targets.size(),
         "counters must be int32 GPU [>= n targets]");
    for (const auto& t : targets) need(t.first != 0 && t.second != 0, "null put target");
    targets_ = targets;
    counters_ = counters;
  }

  void set_schedule(const std::vector<double>& decay, const std::vector<double>& gm, const std::vector<double>& l2,
                    const std::vector<double>& theta, int update_rule, const std::vector<double>& delays, int stop_rule,
                    int k, bool drain) {
    arb_ready_ = false;  // the device arbiter copies this state
    need((int)decay.size() >= R_ && (int)gm.size() >= R_ && (int)l2.size() >= R_ && (int)theta.size() >= R_,
         "schedule arrays must cover R rounds");
    need((int64_t)delays.size() >= (int64_t)R_ * W_, "delays must be [R*W]");
    decay_ = decay;
    gm_ = gm;
    l2_ = l2;
    theta_ = theta;
    update_rule_ = update_rule;
    delays_ = delays;
    stop_rule_ = stop_rule;
    k_ = k;
    drain_ = drain;
  }

  // --delay-on worker: virtual delays the collector applies to REMOTE messages (the worker ranks
  // are physically late themselves); default: the same table as the local messages.
  void set_remote_delays(const std::vector<double>& delays) {
    arb_ready_ = false;
    need((int64_t)delays.size() >= (int64_t)R_ * W_, "remote delays must be [R*W]");
    remote_delays_ = delays;
  }
  // Device times of physically late ranks' messages (collector.h "Device times").  IPC: worker rank r's
  // puts write {round + 1, landing ticks} into 16-byte ring slots [r][i % ring] of shared host memory (ring_host) on
  // that rank's GPU clock clocks[r] = (tick0, t0, hz).  p2p: the receive events become timing events,
  // read against a reference event of this GPU calibrated against the host clock here.
  void set_device_times(const std::vector<std::tuple<int, double, double, double>>& clocks, uintptr_t ring_host,
                        int ring) {
    need(ring >= 1 || comm_, "stamp ring must have >= 1 slot");
    dev_times_ = true;
    for (const auto& [r, tick0, t0, hz] : clocks) {
      need(hz > 0.0, "device clock rate must be > 0");
      clocks_[r] = eh::DeviceClock{tick0, t0, hz};
    }
    ring_host_ = ring_host;
    ring_ = ring;
    if (comm_) {
      for (auto& e : rev_) {  // timing events: the collector reads their device times
        hcheck(hipEventDestroy(e), "hipEventDestroy");
        hcheck(hipEventCreate(&e), "hipEventCreate");
      }
      calibrate_ref_event();
    }
  }
  // Per-round device records (tests/lazy_check.py): [R + 1][2] wall_clock64 stamps just before and just
  // after round j's beta put kernels (-1: not put by put_beta, e.g. released by the arbiter).
  void set_records(bool on) {
    rec_ = on ? at::full({R_ + 1, 2}, -1, at::TensorOptions().dtype(at::kLong).device(at::Device(at::kCUDA, device_)))
              : Tensor();
  }
  Tensor records() {
    hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    return rec_.defined() ? rec_.cpu() : Tensor();
  }
  py::list probe_log() const {
    py::list out;
    for (const auto& r : col_->probe_log()) out.append(py::make_tuple(r.worker, r.part, r.round, r.t_seen, r.outcome));
    return out;
  }
  // Drain "lazy" (engine/trainer.py): the collector skips stale virtual rounds (collector.h) and, with
  // IPC targets, finish_run() tells every worker rank the run is over so its queued rounds are stale.
  void set_skip_stale(bool on) {
    need(!(on && comm_ && !comm_streams_split()), "set_skip_stale(true) after set_comm: the link streams are shared");
    skip_ = on;
    col_->set_skip_stale(on);
  }
  // Whether every peer's receive has a stream of its own (lazy drain) rather than the pair's link stream.
  bool comm_streams_split() const {
    for (const auto& [r, st] : recv_st_)
      if (send_st_.count(r) && send_st_.at(r) == st) return false;
    return true;
  }
  // The compute stream and every distinct comm stream, in creation order (tests: stream_wait_probe).
  std::vector<uintptr_t> stream_handles() const {
    std::vector<uintptr_t> out{reinterpret_cast<uintptr_t>(stream_)};
    std::set<hipStream_t> seen;
    for (const auto* m : {&send_st_, &recv_st_})
      for (const auto& [r, st] : *m)
        if (seen.insert(st).second) out.push_back(reinterpret_cast<uintptr_t>(st));
    return out;
  }
  // Distinct comm streams this pump created (rank_report: hardware-queue budget).
  int comm_streams() const {
    std::set<hipStream_t> all;
    for (const auto& [r, st] : send_st_) all.insert(st);
    for (const auto& [r, st] : recv_st_) all.insert(st);
    return static_cast<int>(all.size());
  }
  // End of the master's rounds (stream-ordered after its last beta put): with skip_stale on, every
  // worker's beta counter goes to R + 1 (as if beta(R) were out), so whatever a late worker rank still
  // has queued is stale and skipped (its gate), and its final signal lets the collector drain.
  void finish_run() {
    if (!skip_) return;
    col_->end_run(eh::Collector::now());
    if (comm_) {  // p2p: the end-of-run beta(R) to every message-sending rank (WorkerPump::run_comm_skip's last wait)
      put_beta_comm(R_, true);
      return;
    }
    for (const auto& t : targets_)
      hcheck(eh::signal_launch(reinterpret_cast<unsigned long long*>(t.second), static_cast<unsigned long long>(R_) + 1,
                               stream_),
             "signal(end of run)");
  }
  int skipped() const { return col_->skipped(); }
  int stale_arrivals() const { return col_->stale_arrivals(); }
  // --slow-ranks: this rank launches its local gradient `n` times per round (a slower GPU).
  void set_repeat(int n) {
    need(n >= 1, "repeat must be >= 1");
    repeat_ = n;
  }

  void set_decode(int kind, const std::vector<int>& group_of, int n_groups) {
    arb_ready_ = false;  // the device arbiter copies this state
    need((int)group_of.size() == W_, "group_of must have W entries");
    need(!((kind == kTable || kind == kPartialTable) && W_ > 64), "table decode supports at most 64 workers");
    decode_kind_ = kind;
    group_of_ = group_of;
    n_groups_ = n_groups;
  }
  void add_table(uint64_t mask, const std::vector<double>& coefs) {
    arb_ready_ = false;  // the device arbiter copies this state
    need((int)coefs.size() == W_, "table row must have W coefficients");
    table_[mask] = coefs;
  }

  // ---- round execution ---------------------------------------------------------------
  void begin(int i) {
    Range tr("eh.master.begin");
    need(i >= 0 && i < R_, "round out of range");
    need(beta_in_.defined(), "set_state first");
    const int slot = i % K_;
    if (i >= K_ && !col_->wait_seen(i - K_, timeout_))  // the ring slot's previous round must have landed
      throw std::runtime_error("MasterPump round " + std::to_string(i) + ": messages of round " +
                               std::to_string(i - K_) + " still in flight after the round timeout; mailbox slot " +
                               std::to_string(slot) + " cannot be reused");
    const double t = eh::Collector::now();
    col_->begin_round(i, t, stop_rule_, k_);
    t_start_[i] = t;
    char* bin = static_cast<char*>(beta_in_.data_ptr());
    const void* src = bin + static_cast<int64_t>(i) * ld_ * es_;
    if (i != prepub_) put_beta(i);  // else already queued behind the device-side drain of round i-1
    const double* dl = delays_.data() + static_cast<int64_t>(i) * W_;
    const double* dr = remote_delays_.empty() ? dl : remote_delays_.data() + static_cast<int64_t>(i) * W_;
    if (n_loc_ > 0 && launcher_) {
      char* g = static_cast<char*>(G_.data_ptr()) + static_cast<int64_t>(slot) * g_rows_ * ld_ * es_;
      if (timing_) record_t(i, 2);
      for (int k = 0; k < repeat_; ++k) hcheck(launcher_->launch(src, g, stream_), "local gradient");
      if (timing_) record_t(i, 3);
      hcheck(hipEventRecord(loc_ev_[slot], stream_), "hipEventRecord");
      for (const auto& m : local_)
        col_->add_event_probe(m.w, m.p, i, reinterpret_cast<uintptr_t>(loc_ev_[slot]), dl[m.w]);
    }
    flush_check();  // round i-1's mailbox rows, behind this round's beta and local gradient
    if (comm_) {  // one receive per sending rank into its mailbox rows; the event behind it is the probe
      char* rb = static_cast<char*>(rbuf_.data_ptr()) + static_cast<int64_t>(slot) * r_rows_ * ld_ * es_;
      for (size_t k = 0; k < comm_ranks_.size(); ++k) {
        const auto& [r, row0, n] = comm_ranks_[k];
        hipStream_t rs = recv_st_.at(r);
        comm_->recv(r, rb + static_cast<int64_t>(row0) * ld_ * es_, static_cast<int64_t>(n) * ld_ * es_, rs);
        hipEvent_t ev = rev_[static_cast<size_t>(slot) * comm_ranks_.size() + k];
        hcheck(hipEventRecord(ev, rs), "hipEventRecord(recv)");
        for (const auto& m : remote_)
          if (m.row >= row0 && m.row < row0 + n)
            col_->add_event_probe(m.w, m.p, i, reinterpret_cast<uintptr_t>(ev), dr[m.w], !remote_delays_.empty(),
                                  dev_times_ && !remote_delays_.empty() ? reinterpret_cast<uintptr_t>(ref_ev_) : 0,
                                  ref_t_);
      }
      return;
    }
    for (const auto& m : remote_) {  // physically late ranks (remote delays set): seen = arrived
      const bool physical = !remote_delays_.empty();
      uintptr_t stamp = 0;
      eh::DeviceClock clk{};
      const int r = row_rank_[m.row];
      if (physical && dev_times_ && ring_host_ && clocks_.count(r)) {  // its landing time on its own GPU clock
        stamp = ring_host_ + 2 * sizeof(int64_t) * (static_cast<uintptr_t>(r) * ring_ + i % ring_);
        clk = clocks_.at(r);
      }
      col_->add_flag_probe(m.w, m.p, i, m.flag, static_cast<uint64_t>(i + 1), dr[m.w], physical, stamp, clk);
    }
  }

  // Returns (status, arrivals [(worker, part, t_rel)], t_start, t_decoded, t_end, t_waited):
  // status 0 ok, 1 timeout (decoded with what arrived), 2 host decode needed (no table
  // row: call resolve()).
  py::tuple finish(int i, bool publish_next) {
    int status;
    std::vector<eh::Arrival> arr;
    double t_dec = 0, t_end = 0;
    {
      py::gil_scoped_release nogil;
      bool ok;
      {
        Range tr("eh.master.wait");
        ok = col_->wait(timeout_);
      }
      t_waited_ = eh::Collector::now();
      check_integrity();  // an earlier round's combine found a torn / stale message
      arr = col_->arrivals();
      UsedRows used;
      Range tr("eh.master.decode_update");
      const bool decoded = decode(i, arr, used);
      if (!decoded) {
        status = 2;
      } else {
        status = ok ? 0 : 1;
        combine(i, used);
        t_dec = eh::Collector::now();
        t_end = after_combine(i, publish_next);
      }
    }
    return pack(status, arr, i, t_dec, t_end);
  }

  // Host-decoded fallback: coefs[(w, part)] for the given arrivals.
  py::tuple resolve(int i, const std::vector<std::tuple<int, int, double>>& coefs, bool publish_next) {
    std::vector<eh::Arrival> arr = col_->arrivals();
    double t_dec, t_end;
    {
      py::gil_scoped_release nogil;
      UsedRows used;
      for (const auto& [w, p, c] : coefs) push_msg(used, i % K_, w, p, c);
      combine(i, used);
      t_dec = eh::Collector::now();
      t_end = after_combine(i, publish_next);
    }
    return pack(0, arr, i, t_dec, t_end);
  }

  // ---- device-driven rounds (single process, no injected delay) -------------------------
  // Every message is local and finishes with the one gradient launch, so the arrival order
  // (and with it the decode) is fixed before the GPU runs: the collector still decides it,
  // from host probes seen at the round start (ties break by the collector's seeded per-round
  // permutation, exactly like the simultaneous HIP-event probes of begin()).  The host decodes round i and
  // enqueues  grad(i) -> combine_update(i)  while the GPU still runs earlier rounds, so the
  // device never waits for the host between rounds.  With `graph` the whole segment is captured into hipGraphs (at most
  // kGraphRounds rounds each) and replayed with one launch per graph.
  // stamps: int64 GPU [R + 1]; stamps[a] = device time before round a, stamps[i + 1] = start
  // of round i's update (its messages are done).  Returns the arrivals of every round.
  static constexpr int kGraphRounds = 256;

  py::list run_local(int a, int b, bool graph, const Tensor& stamps) {
    need(a >= 0 && a <= b && b <= R_, "round range out of bounds");
    need(remote_.empty() && targets_.empty(), "device-driven rounds need every message local");
    need(n_loc_ > 0 && launcher_ != nullptr, "no local messages");
    need(stamps.is_cuda() && stamps.scalar_type() == at::kLong && stamps.numel() >= R_ + 1, "stamps: int64 [R+1]");
    for (int i = a; i < b; ++i)
      for (int w = 0; w < W_; ++w) need(delays_[static_cast<int64_t>(i) * W_ + w] == 0.0, "injected delay present");
    std::vector<std::vector<eh::Arrival>> arrs;
    std::vector<UsedRows> useds;
    arrs.reserve(b - a);
    useds.reserve(b - a);
    auto decode_round = [&](int i) {
      const double t = eh::Collector::now();
      col_->begin_round(i, t, stop_rule_, k_);
      t_start_[i] = t;
      for (const auto& m : local_) col_->mark_seen(col_->add_host_probe(m.w, m.p, i, 0.0), t);
      need(col_->wait(timeout_), "local arrivals did not satisfy the stop rule");
      UsedRows used;
      need(decode(i, col_->arrivals(), used), "completion pattern missing from the decode table");
      arrs.push_back(col_->arrivals());
      useds.push_back(std::move(used));
      if (drain_) col_->drain(i, timeout_);
    };
    if (graph) {  // a captured segment needs every round decoded before the capture
      Range tr("eh.master.decode_ahead");
      for (int i = a; i < b; ++i) decode_round(i);
    }
    long long* st = reinterpret_cast<long long*>(stamps.data_ptr<int64_t>());
    char* bin = static_cast<char*>(beta_in_.data_ptr());
    // The rounds run on the pump's own stream (the legacy default stream cannot be captured),
    // ordered after everything already on the caller's stream and before anything after.
    if (!dev_stream_) {
      hcheck(hipStreamCreateWithFlags(&dev_stream_, hipStreamNonBlocking), "hipStreamCreate");
      hcheck(hipEventCreateWithFlags(&join_ev_, hipEventDisableTiming), "hipEventCreate");
    }
    hcheck(hipEventRecord(join_ev_, stream_), "hipEventRecord");
    hcheck(hipStreamWaitEvent(dev_stream_, join_ev_, 0), "hipStreamWaitEvent");
    const hipStream_t caller = stream_;
    stream_ = dev_stream_;  // launcher_/combine() enqueue on stream_
    struct Restore {
      hipStream_t& s;
      hipStream_t v;
      ~Restore() { s = v; }
    } restore{stream_, caller};
    auto enqueue = [&](int i0, int i1) {
      for (int i = i0; i < i1; ++i) {
        // stream mode: decode round i just before enqueueing it, so the host decodes round i + 1
        // while the GPU runs round i (no host-only stretch at the start of a timed segment)
        if (!graph) decode_round(i);
        const int slot = i % K_;
        char* g = static_cast<char*>(G_.data_ptr()) + static_cast<int64_t>(slot) * g_rows_ * ld_ * es_;
        eh::LocalUpdate up;
        if (fused_update_ && launcher_->can_fuse_update() && local_update(i, useds[i - a], g, st + i + 1, &up)) {
          hcheck(launcher_->launch_update(bin + static_cast<int64_t>(i) * ld_ * es_, g, up, stream_),
                 "local gradient + update");
          continue;
        }
        hcheck(launcher_->launch(bin + static_cast<int64_t>(i) * ld_ * es_, g, stream_), "local gradient");
        combine(i, useds[i - a], false, st + i + 1);
      }
    };
    Range tr("eh.master.device_rounds");
    hcheck(eh::stamp_launch(st + a, stream_), "stamp");
    if (!graph) {
      enqueue(a, b);
    } else {
      for (int c0 = a; c0 < b; c0 += kGraphRounds) {
        const int c1 = std::min(b, c0 + kGraphRounds);
        hipGraph_t gr = nullptr;
        hipGraphExec_t ex = nullptr;
        hcheck(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal), "hipStreamBeginCapture");
        try {
          enqueue(c0, c1);
        } catch (...) {
          hipStreamEndCapture(stream_, &gr);
          if (gr) hipGraphDestroy(gr);
          throw;
        }
        hcheck(hipStreamEndCapture(stream_, &gr), "hipStreamEndCapture");
        hcheck(hipGraphInstantiate(&ex, gr, nullptr, nullptr, 0), "hipGraphInstantiate");
        hipGraphDestroy(gr);
        hcheck(hipGraphLaunch(ex, stream_), "hipGraphLaunch");
        graphs_.push_back(ex);
      }
      ++graph_segments_;
    }
    hcheck(hipEventRecord(join_ev_, dev_stream_), "hipEventRecord");
    hcheck(hipStreamWaitEvent(caller, join_ev_, 0), "hipStreamWaitEvent");
    py::list out;
    for (const auto& arr : arrs) {
      py::list lst;
      for (const auto& x : arr) lst.append(py::make_tuple(x.worker, x.part, x.t_rel));
      out.append(lst);
    }
    return out;
  }

  // ---- device-driven rounds with remote workers (csrc/kernels/arbiter.hip) -----------------
  // sources: (host address, device address) of every worker rank's message counter; a remote
  // message belongs to the source with its flag's host address.
  void set_sources(const std::vector<std::pair<uintptr_t, uintptr_t>>& srcs) {
    for (const auto& f : srcs) need(f.first != 0 && f.second != 0, "null source counter");
    arb_src_ = srcs;
    arb_ready_ = false;
  }

  // Why rounds [a, b) cannot run on the device arbiter ("" = they can).
  std::string device_blocker(int a, int b) const {
    if (comm_) return "messages travel over " + comm_->kind() + " (the arbiter polls IPC counters)";
    if (remote_.empty() || arb_src_.empty()) return "no remote workers";
    if ((int)arb_src_.size() > eh::kArbMaxSrc) return "more than 64 worker ranks";
    if (W_ > eh::kArbMaxW) return "more than 64 workers";
    if ((int)(local_.size() + remote_.size()) > eh::kArbMaxProbes) return "too many message shards";
    if ((decode_kind_ == kTable || decode_kind_ == kPartialTable) && W_ > 16) return "decode table too large";
    size_t rows = 0;  // worst case of one decode: every buffer row of every message
    for (const auto& ix : index_) {
      if ((int)ix.size() > eh::kArbMaxRows) return "message with more than 16 shards";
      rows += ix.size();
    }
    if (rows > static_cast<size_t>(eh::kMaxMsgs)) return "more than 128 message rows in a decode";
    for (const auto& m : remote_) {
      bool found = false;
      for (const auto& f : arb_src_) found |= f.first == m.flag;
      if (!found) return "remote message without a source counter";
    }
    for (int i = a; i < b; ++i)
      if (!no_delay(i)) return "injected delays (virtual arrival times live on the host)";
    return "";
  }

  // Enqueue rounds [a, b): the master's own gradient, then one arbiter kernel per round that
  // polls the workers' counters, decides, updates and releases the next beta.  Nothing waits on
  // the host; device_log() reads the rounds back.
  void run_device(int a, int b, double deadline_s) {
    need(a >= 0 && a <= b && b <= R_, "round range out of bounds");
    const std::string why = device_blocker(a, b);
    need(why.empty(), "device-driven rounds: " + why);
    if (!arb_ready_) arb_prepare();
    // a new segment starts clean: no abort from an earlier failed segment (whose failure device_log
    // reports; the engine does not continue a run past it)
    hcheck(hipMemsetAsync(arb_abort_.data_ptr(), 0, sizeof(int), stream_), "hipMemsetAsync(abort)");
    eh::ArbArgs args = arb_args_;
    args.deadline_ticks = static_cast<long long>(std::max(0.001, deadline_s) * stamp_hz());
    long long* tlog = reinterpret_cast<long long*>(arb_tlog_.data_ptr<int64_t>());
    char* bin = static_cast<char*>(beta_in_.data_ptr());
    if (a < b && a != prepub_) {  // beta(a) was not released by an earlier arbiter
      put_beta(a);
      hcheck(eh::stamp_launch(tlog + static_cast<int64_t>(a) * eh::kArbLogTicks, stream_), "stamp");
    }
    // Integrity checks ride a side stream: check(i) waits for arbiter i, runs during round i+1's local
    // gradient, and arbiter i+1 waits for it (it fails the round if check(i) found a torn row).
    const bool chk = args.tags != nullptr;
    if (chk && !chk_stream_) {
      hcheck(hipStreamCreateWithFlags(&chk_stream_, hipStreamNonBlocking), "hipStreamCreate");
      hcheck(hipEventCreateWithFlags(&arb_ev_, hipEventDisableTiming), "hipEventCreate");
      hcheck(hipEventCreateWithFlags(&chk_ev_, hipEventDisableTiming), "hipEventCreate");
    }
    for (int i = a; i < b; ++i) {
      if (n_loc_ > 0 && launcher_) {
        char* g = static_cast<char*>(G_.data_ptr()) + static_cast<int64_t>(i % K_) * g_rows_ * ld_ * es_;
        for (int k = 0; k < repeat_; ++k)
          hcheck(launcher_->launch(bin + static_cast<int64_t>(i) * ld_ * es_, g, stream_), "local gradient");
      }
      if (chk && i > a) hcheck(hipStreamWaitEvent(stream_, chk_ev_, 0), "hipStreamWaitEvent");
      hcheck(eh::arbiter_round_launch(args, i, acc_, stream_, chk && i > a), "arbiter_round");
      if (chk) {
        hcheck(hipEventRecord(arb_ev_, stream_), "hipEventRecord");
        hcheck(hipStreamWaitEvent(chk_stream_, arb_ev_, 0), "hipStreamWaitEvent");
        hcheck(eh::arbiter_check_launch(args, i, chk_stream_), "arbiter_check");
        hcheck(hipEventRecord(chk_ev_, chk_stream_), "hipEventRecord");
      }
    }
    if (b > a) {
      if (chk) hcheck(hipStreamWaitEvent(stream_, chk_ev_, 0), "hipStreamWaitEvent");  // device_log sees it
      prepub_ = b;
    }
  }

  // Rounds [a, b) of run_device: (status, arrivals [(worker, part, t_rel)], t_decoded, t_end), times
  // in seconds from the round's beta release.  status 0 ok, 1 timeout, 2 not decodable on the
  // device, 3 skipped after an earlier failure.  Syncs the pump stream.
  py::list device_log(int a, int b) {
    need(arb_ready_, "run_device first");
    hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    const Tensor lg = arb_log_.cpu(), tl = arb_tlog_.cpu();
    const int* L = lg.data_ptr<int>();
    const int64_t* T = tl.data_ptr<int64_t>();
    const double hz = stamp_hz();
    py::list out;
    for (int i = a; i < b; ++i) {
      const int* l = L + static_cast<int64_t>(i) * eh::kArbLogInts;
      const int64_t* t = T + static_cast<int64_t>(i) * eh::kArbLogTicks;
      py::list arr;
      const int n = std::min(l[1], 2 * eh::kArbMaxW);
      for (int x = 0; x < n && l[0] == 0; ++x)
        arr.append(py::make_tuple(l[4 + 2 * x], l[5 + 2 * x], (t[eh::kArbTickArr + x] - t[0]) / hz));
      std::string why;
      const auto* e = static_cast<const eh::IntegrityErr*>(err_->host);
      if (l[0] == eh::kArbIntegrity || (l[0] == 3 && __atomic_load_n(&e->flag, __ATOMIC_ACQUIRE)))
        why = integrity_message(*e, false);
      // per-round ticks: poll (release of beta(i) -> stop rule), update (stop rule -> combine and
      // checks done), release (-> beta(i+1) released, drain included); seconds
      const double t_stop = l[0] == 0 && n > 0 ? (t[eh::kArbTickArr + n - 1] - t[0]) / hz : -1.0;
      // inside the update: poll joined (all waves past the barrier + acquire), decode done
      const py::tuple sub = py::make_tuple((t[3] - t[0]) / hz, (t[4] - t[0]) / hz);
      out.append(py::make_tuple(l[0], arr, (t[1] - t[0]) / hz, (t[2] - t[0]) / hz, why, t_stop, sub));
    }
    return out;
  }

  // Wall-clock rate of the device timestamps (Hz).
  double stamp_hz() const {
    int khz = 0;
    hcheck(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_), "hipDeviceGetAttribute");
    return 1e3 * khz;
  }
  int graphs_launched() const { return (int)graphs_.size(); }
  // run_local: combine + update inside the slab reduction (default) or as their own launches (A/B, tests)
  void set_fused_update(bool on) { fused_update_ = on; }

  // Update-kernel durations (ms) of every round run so far (host sync).
  std::vector<double> update_ms() {
    hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    std::vector<double> out(R_, 0.0);
    for (int i = 0; i < R_; ++i) {
      auto& p = upd_ev_[i];
      if (p.first && p.second) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.first, p.second) == hipSuccess) out[i] = ms;
      }
    }
    return out;
  }

 private:
  struct Msg {
    int w, p, row;
    uintptr_t flag;
  };

  void check_wp(int w, int p) const { need(w >= 0 && w < W_ && (p == 0 || p == 1), "bad (worker, part)"); }

  void record_t(int i, int which) {
    hipEvent_t& e = tev_[i][which];
    if (!e) hcheck(hipEventCreate(&e), "hipEventCreate");
    hcheck(hipEventRecord(e, stream_), "hipEventRecord");
  }

  static int blocks_for(long long bytes) {
    const long long v = bytes / 16;
    return (int)std::max<long long>(1, std::min<long long>(64, (v + 4095) / 4096));
  }

  // every buffer row (one per shard) of message (w, p) in ring slot `slot`, each with coefficient c
  void push_msg(UsedRows& used, int slot, int w, int p, double c) const {
    const auto& ix = index_[2 * w + p];
    if (ix.empty()) throw std::logic_error("message without a buffer");
    for (const auto& [kind, row] : ix) {
      const char* base = kind == 0 ? static_cast<const char*>(G_.data_ptr()) + static_cast<int64_t>(slot) * g_rows_ * ld_ * es_
                                   : static_cast<const char*>(rbuf_.data_ptr()) + static_cast<int64_t>(slot) * r_rows_ * ld_ * es_;
      used.push_back({base + static_cast<int64_t>(row) * ld_ * es_, c, kind == 0 ? -1 : row});
    }
  }

  bool decode(int i, const std::vector<eh::Arrival>& arr, UsedRows& used) const {
    const int slot = i % K_;
    std::vector<char> gdone(std::max(n_groups_, 1), 0);
    uint64_t mask = 0;
    for (const auto& a : arr) {
      if (a.part == 1) {
        if (decode_kind_ == kPartialFrc || decode_kind_ == kPartialTable) push_msg(used, slot, a.worker, 1, 1.0);
        continue;
      }
      switch (decode_kind_) {
        case kSumPart0:
          push_msg(used, slot, a.worker, 0, 1.0);
          break;
        case kFirstPerGroup:
        case kPartialFrc: {
          const int g = group_of_[a.worker];
          if (!gdone[g]) {
            gdone[g] = 1;
            push_msg(used, slot, a.worker, 0, 1.0);
          }
          break;
        }
        default:
          mask |= (uint64_t)1 << a.worker;
      }
    }
    if (decode_kind_ == kTable || decode_kind_ == kPartialTable) {
      auto it = table_.find(mask);
      if (it == table_.end()) return false;
      for (int w = 0; w < W_; ++w)
        if (mask >> w & 1) push_msg(used, slot, w, 0, it->second[w]);
    }
    return true;
  }

  // events: time the update with HIP events (host-driven rounds); stamp: device timestamp
  // written by the update kernel at its start (device-driven rounds, graph capture).
  // Round i's combine + update as a LocalUpdate over the G rows of this launch (run_local); false
  // when a decoded row is not one of them.
  bool local_update(int i, const UsedRows& used, const char* g, long long* stamp, eh::LocalUpdate* up) const {
    if ((int)used.size() > eh::kMaxMsgs) return false;
    const int64_t rb = static_cast<int64_t>(ld_) * es_;
    up->nmsg = (int)used.size();
    for (int m = 0; m < up->nmsg; ++m) {
      const int64_t off = static_cast<const char*>(used[m].p) - g;
      if (used[m].row >= 0 || off < 0 || off % rb || off / rb >= launcher_->nslots) return false;
      up->slot[m] = static_cast<int>(off / rb);
      up->coef[m] = used[m].c;
    }
    up->beta = beta_.data_ptr<double>();
    up->u = u_.data_ptr<double>();
    up->hist = hist_.data_ptr<double>() + static_cast<int64_t>(i) * ld_;
    up->beta_w = static_cast<char*>(beta_in_.data_ptr()) + static_cast<int64_t>(i + 1) * ld_ * es_;
    up->stamp = stamp;
    up->d = d_;
    up->rule = update_rule_;
    up->decay = decay_[i];
    up->gm = gm_[i];
    up->l2 = l2_[i];
    up->theta = theta_[i];
    return true;
  }
  void combine(int i, const UsedRows& used, bool events = true,
               long long* stamp = nullptr) {
    need((int)used.size() <= eh::kMaxMsgs, "too many messages for one combine");
    eh::CombineArgs a{};
    a.nmsg = (int)used.size();
    bool remote = false;
    for (int m = 0; m < a.nmsg; ++m) {
      a.msg[m] = used[m].p;
      a.coef[m] = used[m].c;
      remote |= used[m].row >= 0;
    }
    if (comm_ && remote) {  // order the combine after the receives it reads (their events are complete)
      const int slot = i % K_;
      for (size_t k = 0; k < comm_ranks_.size(); ++k) {
        const auto& [r, row0, n] = comm_ranks_[k];
        bool hit = false;
        for (const auto& u : used) hit |= u.row >= row0 && u.row < row0 + n;
        if (hit) hcheck(hipStreamWaitEvent(stream_, rev_[static_cast<size_t>(slot) * comm_ranks_.size() + k], 0),
                        "hipStreamWaitEvent(recv)");
      }
    }
    if (tags_ && remote) {  // the mailbox rows it reads are checked after the next round starts
      eh::CheckList& cl = check_;
      const int slot = i % K_;
      cl = eh::CheckList{};
      cl.round = i;
      cl.slot = slot;
      cl.es = es_;
      cl.ld = ld_;
      cl.tags = reinterpret_cast<const eh::MsgTag*>(mbox_tags_) + static_cast<int64_t>(slot) * r_rows_;
      for (const auto& u : used)
        if (u.row >= 0) {
          if (cl.n >= eh::kMaxCheckRows) {  // the check list is full: counted, reported by the trainer
            ++check_rows_cut_;
            continue;
          }
          cl.row[cl.n] = u.p;
          cl.mrow[cl.n] = u.row;
          cl.rank[cl.n] = row_rank_[u.row];
          ++cl.n;
        }
      check_pending_ = cl.n > 0;
    }
    auto& ev = upd_ev_[i];
    if (events) {
      if (!ev.first) hcheck(hipEventCreate(&ev.first), "hipEventCreate");
      if (!ev.second) hcheck(hipEventCreate(&ev.second), "hipEventCreate");
      hcheck(hipEventRecord(ev.first, stream_), "hipEventRecord");
    }
    char* bin = static_cast<char*>(beta_in_.data_ptr());
    hcheck(eh::combine_update_launch(a, acc_, acc_, beta_.data_ptr<double>(), u_.data_ptr<double>(),
                                     hist_.data_ptr<double>() + static_cast<int64_t>(i) * ld_,
                                     bin + static_cast<int64_t>(i + 1) * ld_ * es_, nullptr, d_, ld_, decay_[i], gm_[i],
                                     l2_[i], theta_[i], update_rule_, stream_, stamp),
           "combine_update");
    if (events) hcheck(hipEventRecord(ev.second, stream_), "hipEventRecord");
  }

  // Device copies of everything the arbiter reads (arbiter.h ArbArgs); built once.
  void arb_prepare() {
    const auto dev = beta_.device();
    auto ints = [&](const std::vector<int>& v) {
      return at::from_blob(const_cast<int*>(v.data()), {(int64_t)v.size()}, at::kInt).clone().to(dev);
    };
    auto dbl = [&](const std::vector<double>& v) {
      return at::from_blob(const_cast<double*>(v.data()), {(int64_t)v.size()}, at::kDouble).clone().to(dev);
    };
    auto u64 = [&](const std::vector<int64_t>& v) {
      return at::from_blob(const_cast<int64_t*>(v.data()), {(int64_t)v.size()}, at::kLong).clone().to(dev);
    };
    std::vector<int> pw, pp, ps;
    for (const auto& m : local_) {  // probe order = begin(): local event probes, then the flag probes
      pw.push_back(m.w);
      pp.push_back(m.p);
      ps.push_back(-1);
    }
    for (const auto& m : remote_) {
      int src = -1;
      for (int j = 0; j < (int)arb_src_.size(); ++j)
        if (arb_src_[j].first == m.flag) src = j;
      pw.push_back(m.w);
      pp.push_back(m.p);
      ps.push_back(src);
    }
    std::vector<int> nsh(2 * W_, 0), nrows(2 * W_, 0), rows(2 * W_ * eh::kArbMaxRows, 0);
    for (int q = 0; q < (int)pw.size(); ++q) ++nsh[2 * pw[q] + pp[q]];
    for (int mi = 0; mi < 2 * W_; ++mi) {
      nrows[mi] = (int)index_[mi].size();
      for (int r = 0; r < nrows[mi]; ++r) rows[mi * eh::kArbMaxRows + r] = (index_[mi][r].first << 24) | index_[mi][r].second;
    }
    std::vector<int> tie(static_cast<size_t>(R_) * W_, 0);
    const int64_t seed = col_->tie_seed();
    if (seed >= 0) {
      std::vector<int> ord(W_);
      for (int i = 0; i < R_; ++i) {
        for (int w = 0; w < W_; ++w) ord[w] = w;
        std::sort(ord.begin(), ord.end(), [&](int x, int y) {
          const uint64_t kx = eh::Collector::tie_key(seed, i, x), ky = eh::Collector::tie_key(seed, i, y);
          return kx != ky ? kx < ky : x < y;
        });
        for (int r = 0; r < W_; ++r) tie[static_cast<size_t>(i) * W_ + ord[r]] = r;
      }
    }
    std::vector<double> table;
    if (decode_kind_ == kTable || decode_kind_ == kPartialTable) {
      table.assign((size_t{1} << W_) * W_, std::nan(""));
      for (const auto& [mask, coefs] : table_)
        if (mask < (uint64_t{1} << W_))
          for (int w = 0; w < W_; ++w) table[mask * W_ + w] = coefs[w];
    }
    std::vector<int64_t> src, tgt;
    for (const auto& f : arb_src_) src.push_back(static_cast<int64_t>(f.second));
    for (const auto& t : targets_) {
      tgt.push_back(static_cast<int64_t>(t.first));
      tgt.push_back(static_cast<int64_t>(t.second));
    }
    arb_keep_ = {ints(group_of_), ints(pw), ints(pp), ints(ps), ints(nsh), ints(nrows), ints(rows), ints(tie),
                 dbl(decay_), dbl(gm_), dbl(l2_), dbl(theta_), u64(src.empty() ? std::vector<int64_t>{0} : src),
                 u64(tgt.empty() ? std::vector<int64_t>{0, 0} : tgt),
                 table.empty() ? at::Tensor() : dbl(table),
                 ints(row_rank_.empty() ? std::vector<int>{0} : row_rank_)};
    arb_log_ = at::zeros({static_cast<int64_t>(R_) * eh::kArbLogInts}, at::TensorOptions().dtype(at::kInt).device(dev));
    arb_tlog_ = at::zeros({static_cast<int64_t>(R_) * eh::kArbLogTicks}, at::TensorOptions().dtype(at::kLong).device(dev));
    arb_abort_ = at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(dev));
    eh::ArbArgs g{};
    g.W = W_;
    g.n_groups = n_groups_;
    g.rule = stop_rule_;
    g.k = k_;
    g.decode = decode_kind_;
    g.drain = drain_ ? 1 : 0;
    g.nprobe = (int)pw.size();
    g.nsrc = (int)arb_src_.size();
    g.ntarget = (int)targets_.size();
    g.K = K_;
    g.ld = ld_;
    g.d = d_;
    g.g_rows = g_rows_;
    g.r_rows = r_rows_;
    g.R = R_;
    g.update_rule = update_rule_;
    g.group_of = arb_keep_[0].data_ptr<int>();
    g.probe_w = arb_keep_[1].data_ptr<int>();
    g.probe_p = arb_keep_[2].data_ptr<int>();
    g.probe_src = arb_keep_[3].data_ptr<int>();
    g.nsh = arb_keep_[4].data_ptr<int>();
    g.msg_nrows = arb_keep_[5].data_ptr<int>();
    g.msg_rows = arb_keep_[6].data_ptr<int>();
    g.tie = arb_keep_[7].data_ptr<int>();
    g.decay = arb_keep_[8].data_ptr<double>();
    g.gm = arb_keep_[9].data_ptr<double>();
    g.l2 = arb_keep_[10].data_ptr<double>();
    g.theta = arb_keep_[11].data_ptr<double>();
    g.src_flag = reinterpret_cast<const unsigned long long*>(arb_keep_[12].data_ptr<int64_t>());
    g.targets = reinterpret_cast<const unsigned long long*>(arb_keep_[13].data_ptr<int64_t>());
    g.table = arb_keep_[14].defined() ? arb_keep_[14].data_ptr<double>() : nullptr;
    g.beta = beta_.data_ptr<double>();
    g.u = u_.data_ptr<double>();
    g.hist = hist_.data_ptr<double>();
    g.beta_in = beta_in_.data_ptr();
    g.G = G_.defined() ? G_.data_ptr() : nullptr;
    g.rbuf = rbuf_.defined() ? rbuf_.data_ptr() : nullptr;
    g.log = arb_log_.data_ptr<int>();
    g.tlog = reinterpret_cast<long long*>(arb_tlog_.data_ptr<int64_t>());
    g.abort = arb_abort_.data_ptr<int>();
    g.tags = tags_ ? reinterpret_cast<const eh::MsgTag*>(mbox_tags_) : nullptr;
    g.row_rank = arb_keep_[15].data_ptr<int>();
    g.inbox_tag_off = inbox_tag_off_;
    arb_checks_ = at::zeros({static_cast<int64_t>(2 * sizeof(eh::CheckList))}, at::TensorOptions().dtype(at::kByte).device(dev));
    g.checks = reinterpret_cast<eh::CheckList*>(arb_checks_.data_ptr());
    g.err = static_cast<eh::IntegrityErr*>(err_->dev);
    arb_args_ = g;
    arb_ready_ = true;
  }

  // push beta(j) into every worker inbox (put + signal kernels on the pump stream)
  // one send of beta(j) per worker rank, each on its own stream behind the update that wrote it
  // senders_only: only the ranks that send messages -- the end-of-run beta(R) goes to the WorkerPumps
  // with stale-round skipping (set_skip_stale_comm) and nowhere else: a rank hosting no message runs
  // the Python worker loop, which receives beta(0..R-1) only, and an unmatched send could hold the
  // pump's stream (comm.h: a send blocks until the peer's matching call).
  void put_beta_comm(int j, bool senders_only = false) {
    const void* src = static_cast<const char*>(beta_in_.data_ptr()) + static_cast<int64_t>(j) * ld_ * es_;
    hcheck(hipEventRecord(bev_, stream_), "hipEventRecord(beta)");
    for (int r : comm_peers_) {
      if (senders_only && std::none_of(comm_ranks_.begin(), comm_ranks_.end(),
                                       [r](const auto& c) { return std::get<0>(c) == r && std::get<2>(c) > 0; }))
        continue;
      hcheck(hipStreamWaitEvent(send_st_.at(r), bev_, 0), "hipStreamWaitEvent(beta)");
      comm_->send(r, src, static_cast<int64_t>(ld_) * es_, send_st_.at(r));
    }
  }
  void put_beta(int j) {
    int64_t* rec = rec_.defined() && j <= R_ ? rec_.data_ptr<int64_t>() + 2 * static_cast<int64_t>(j) : nullptr;
    if (rec) hcheck(eh::stamp_launch(reinterpret_cast<long long*>(rec), stream_), "stamp(beta put)");
    put_beta_kernels(j);
    if (rec) hcheck(eh::stamp_launch(reinterpret_cast<long long*>(rec + 1), stream_), "stamp(beta put)");
  }
  // The reference event of device-timed receive events: the sample with the shortest host round trip.
  void calibrate_ref_event() {
    std::vector<hipEvent_t> evs(8, nullptr);
    double best = 1e30;
    int pick = 0;
    for (size_t k = 0; k < evs.size(); ++k) {
      hcheck(hipEventCreate(&evs[k]), "hipEventCreate");
      const double ta = eh::Collector::now();
      hcheck(hipEventRecord(evs[k], stream_), "hipEventRecord(ref)");
      hcheck(hipEventSynchronize(evs[k]), "hipEventSynchronize(ref)");
      const double tb = eh::Collector::now();
      if (tb - ta < best) {
        best = tb - ta;
        pick = static_cast<int>(k);
        ref_t_ = 0.5 * (ta + tb);
      }
    }
    if (ref_ev_) hipEventDestroy(ref_ev_);
    ref_ev_ = evs[pick];
    for (size_t k = 0; k < evs.size(); ++k)
      if (static_cast<int>(k) != pick) hipEventDestroy(evs[k]);
  }
  void put_beta_kernels(int j) {
    if (comm_) {
      if (timing_) record_t(j, 0);
      put_beta_comm(j);
      if (timing_) record_t(j, 1);
      return;
    }
    if (targets_.empty()) return;
    const void* src = static_cast<const char*>(beta_in_.data_ptr()) + static_cast<int64_t>(j) * ld_ * es_;
    if (timing_) record_t(j, 0);
    for (size_t k0 = 0; k0 < targets_.size(); k0 += eh::kMaxPuts) {
      eh::PutArgs a{};
      a.n = 0;
      for (size_t k = k0; k < targets_.size() && a.n < eh::kMaxPuts; ++k) {
        auto& d = a.d[a.n];
        d = eh::PutDesc{src, reinterpret_cast<char*>(targets_[k].first) + static_cast<int64_t>(j) * ld_ * es_,
                        static_cast<long long>(ld_) * es_,
                        reinterpret_cast<unsigned long long*>(targets_[k].second),
                        static_cast<unsigned long long>(j + 1),
                        reinterpret_cast<unsigned int*>(counters_.data_ptr<int>()) + k};
        if (tags_) {
          d.tag = reinterpret_cast<eh::MsgTag*>(reinterpret_cast<char*>(targets_[k].first) + inbox_tag_off_) + j;
          d.csum = reinterpret_cast<unsigned long long*>(csum_.data_ptr<int64_t>()) + a.n * eh::kMaxTagRows;
          d.rows = 1;
          d.es = es_;
          d.rank = 0;
          d.corrupt = sabotage("beta", static_cast<int>(k) + 1, j) ? 1 : 0;
        }
        ++a.n;
      }
      hcheck(eh::put_signal_launch(a, blocks_for(static_cast<long long>(ld_) * es_), stream_), "put_signal(beta)");
    }
    if (timing_) record_t(j, 1);
  }

  // Enqueue the pending check of the last combined round (integrity.h CheckList): off the round's
  // critical path, the rows stay intact until slot reuse K >= 2 rounds later.
  void flush_check() {
    if (!check_pending_) return;
    check_pending_ = false;
    hcheck(eh::check_list_launch(check_, static_cast<eh::IntegrityErr*>(err_->dev), stream_), "check_list");
  }

  // No virtual delay applies in round i: the local messages' entries of the delay table and the remote
  // ones of the remote table (a physically late rank's own lateness is no virtual delay).
  bool no_delay(int i) const {
    const double* dl = delays_.data() + static_cast<int64_t>(i) * W_;
    const double* dr = remote_delays_.empty() ? dl : remote_delays_.data() + static_cast<int64_t>(i) * W_;
    for (const auto& m : local_)
      if (dl[m.w] != 0.0) return false;
    for (const auto& m : remote_)
      if (dr[m.w] != 0.0) return false;
    return true;
  }

  double after_combine(int i, bool publish_next) {
    const bool next = publish_next && i + 1 < R_;
    if (drain_ && next && !drain_flags_.empty() && no_delay(i) && no_delay(i + 1)) {
      // Device-side drain: the pump stream waits until every worker rank's round-i flag is set
      // (hipStreamWaitValue64 on the shared flags), then pushes beta(i+1) — queued now, so the
      // put leaves as soon as the last message lands instead of after a host wake-up + launch.
      // The host drain below still gates the round's bookkeeping (t_start of round i+1).
      for (const auto& f : drain_flags_)
        hcheck(hipStreamWaitValue64(stream_, reinterpret_cast<void*>(f.second), static_cast<uint64_t>(i + 1),
                                    hipStreamWaitValueGte),
               "hipStreamWaitValue64(message flag)");
      put_beta(i + 1);
      prepub_ = i + 1;
      Range tr("eh.master.drain");
      if (!col_->drain(i, timeout_)) {
        // a worker rank is gone: release the queued waits (store the value they wait for) so no
        // wait is left on the GPU; its late message, if any, lands in a slot nobody reads
        for (const auto& f : drain_flags_) {
          auto* h = reinterpret_cast<uint64_t*>(f.first);
          if (__atomic_load_n(h, __ATOMIC_ACQUIRE) < static_cast<uint64_t>(i + 1))
            __atomic_store_n(h, static_cast<uint64_t>(i + 1), __ATOMIC_RELEASE);
        }
      }
    } else if (drain_) {
      Range tr("eh.master.drain");
      col_->drain(i, timeout_);
    }
    const double t_end = eh::Collector::now();
    if (next) begin(i + 1);
    return t_end;
  }

  py::tuple pack(int status, const std::vector<eh::Arrival>& arr, int i, double t_dec, double t_end) const {
    py::list lst;
    for (const auto& a : arr) lst.append(py::make_tuple(a.worker, a.part, a.t_rel));
    return py::make_tuple(status, lst, t_start_[i], t_dec, t_end, t_waited_);
  }

  eh::Collector* col_;
  int W_, R_, K_, d_, ld_, device_;
  double timeout_;
  hipStream_t stream_ = nullptr;
  int acc_ = 0, es_ = 8;
  Tensor beta_, u_, hist_, beta_in_, G_, rbuf_, counters_;
  std::shared_ptr<GradLauncher> launcher_;
  int n_loc_ = 0, g_rows_ = 1, r_rows_ = 1;
  std::vector<Msg> local_, remote_;
  std::vector<std::vector<std::pair<int, int>>> index_;  // [2*w+p] -> (0 local | 1 remote, row) per shard
  std::vector<std::pair<uintptr_t, uintptr_t>> targets_;
  std::vector<std::pair<uintptr_t, uintptr_t>> drain_flags_;
  int prepub_ = -1;  // round whose beta is already queued (device-side drain / the arbiter)
  std::shared_ptr<eh::P2PComm> comm_;                 // stream-ordered p2p (set_comm); null: IPC mailbox
  // device times of physically late ranks (set_device_times) and per-round records (set_records)
  bool dev_times_ = false;
  std::map<int, eh::DeviceClock> clocks_;
  uintptr_t ring_host_ = 0;
  int ring_ = 1;
  hipEvent_t ref_ev_ = nullptr;
  double ref_t_ = 0.0;
  Tensor rec_;
  std::vector<std::tuple<int, int, int>> comm_ranks_;  // (rank, first mailbox row, rows) of every sender
  std::vector<int> comm_peers_;                        // every worker rank (beta receivers)
  std::map<int, hipStream_t> send_st_, recv_st_;       // per-peer streams
  std::vector<hipEvent_t> rev_;                        // [K][sender] receive-done events (collector probes)
  hipEvent_t bev_ = nullptr;                           // beta(j) written (the sends wait on it)
  bool tags_ = false;               // integrity tags on (set_integrity)
  int64_t check_rows_cut_ = 0;      // decoded mailbox rows past a round's check list (kMaxCheckRows): unchecked
  uintptr_t mbox_tags_ = 0;         // device address of the mailbox tag slots [K][r_rows]
  int64_t inbox_tag_off_ = 0;       // worker inbox base -> its tag slots
  std::vector<int> row_rank_;       // [r_rows] sender rank of each mailbox row
  std::unique_ptr<HostMapped> err_;  // first integrity failure (eh::IntegrityErr)
  Tensor csum_;                     // beta put checksum scratch
  eh::CheckList check_{};           // mailbox rows of the last combined round, checked after the next begins
  bool check_pending_ = false;
  std::vector<std::pair<uintptr_t, uintptr_t>> arb_src_;
  bool arb_ready_ = false;
  eh::ArbArgs arb_args_{};
  std::vector<Tensor> arb_keep_;
  Tensor arb_log_, arb_tlog_, arb_abort_, arb_checks_;
  std::vector<double> decay_, gm_, l2_, theta_, delays_, remote_delays_;
  int repeat_ = 1;
  int update_rule_ = 0, stop_rule_ = 0, k_ = 0;
  bool drain_ = false;
  bool skip_ = false;  // drain "lazy": stale-round skipping (set_skip_stale)
  int decode_kind_ = kSumPart0, n_groups_ = 1;
  std::vector<int> group_of_;
  std::map<uint64_t, std::vector<double>> table_;
  std::vector<double> t_start_;
  double t_waited_ = 0.0;  // host time the last wait() returned (phase timing)
  std::vector<std::pair<hipEvent_t, hipEvent_t>> upd_ev_;
  std::vector<hipEvent_t> loc_ev_;
  std::vector<hipGraphExec_t> graphs_;  // device-driven segments (destroyed after a sync)
  hipStream_t dev_stream_ = nullptr;     // stream of the device-driven rounds (capturable)
  bool fused_update_ = true;              // run_local: combine + update inside the slab reduction
  hipStream_t chk_stream_ = nullptr;     // run_device: arbiter_check kernels beside the local gradient
  hipEvent_t arb_ev_ = nullptr, chk_ev_ = nullptr;
  hipEvent_t join_ev_ = nullptr;
  int graph_segments_ = 0;
  bool timing_ = false;
  std::vector<std::array<hipEvent_t, 4>> tev_;  // [round] put start/end, gradient start/end
};

// ------------------------------------------------------------------------- WorkerPump
class WorkerPump {
 public:
  WorkerPump(std::shared_ptr<GradLauncher> g, const Tensor& inbox, const Tensor& G, int n_loc, uintptr_t mbox_base,
             int mbox_rows, int row0, uintptr_t beta_flag_host, uintptr_t msg_flag_dev, const Tensor& counters,
             int K, int device, double timeout, uintptr_t beta_flag_dev)
      : g_(std::move(g)), inbox_(inbox), G_(G), n_(n_loc), mbox_(mbox_base), mbox_rows_(mbox_rows), row0_(row0),
        bflag_(reinterpret_cast<uint64_t*>(beta_flag_host)), bflag_dev_(reinterpret_cast<void*>(beta_flag_dev)),
        mflag_(reinterpret_cast<unsigned long long*>(msg_flag_dev)), counters_(counters), K_(K), timeout_(timeout) {
    need_gpu(inbox, "inbox");
    need_gpu(G, "G");
    need(G.dim() == 3 && G.size(0) == K && G.size(2) == inbox.size(1), "G must be [K, n, ld]");
    need(acc_code(G) == acc_code(inbox), "G/inbox dtype mismatch");
    need(n_loc >= 0 && n_loc <= G.size(1), "n_loc out of range");
    need(row0 >= 0 && row0 + n_loc <= mbox_rows, "mailbox rows out of range");
    need(beta_flag_host != 0 && msg_flag_dev != 0 && mbox_base != 0, "null address");
    need(counters.is_cuda() && counters.scalar_type() == at::kInt && counters.numel() >= 1, "counters");
    ld_ = (int)inbox.size(1);
    R_ = (int)inbox.size(0) - 1;
    device_ = device;
    es_ = acc_code(G) == 0 ? 8 : 4;
    g_rows_ = (int)G.size(1);
    stream_ = c10::hip::getCurrentHIPStream(device).stream();
    wait_s_.assign(R_, -1.0);
    fuse_put_ = g_->can_fuse_put(n_loc);
    // Device-side beta wait: the stream itself waits for the flag (hipStreamWaitValue64 on the
    // host-registered shared flag), so round i's kernels are already queued when beta(i) lands
    // instead of after a host wake-up + launch.  The host stays one round ahead and keeps the
    // timeout.  beta_flag_dev = 0 selects the host-side wait (the caller's policy).
    int can = 0;
    if (bflag_dev_ && hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, device) == hipSuccess)
      dwait_ = can != 0;
    err_ = std::make_unique<HostMapped>(sizeof(eh::IntegrityErr));
    abort_ = std::make_unique<HostMapped>(sizeof(int));
    csum_ = at::zeros({eh::kMaxTagRows}, at::TensorOptions().dtype(at::kLong).device(at::Device(at::kCUDA, device)));
  }
  // Stream-ordered p2p worker (runtime/comm.h: RCCL, or its single-GPU loopback): every round is
  // recv(beta) -> gradient -> [late spin] -> send(messages) on this rank's stream, enqueued one round
  // ahead of the beta that has landed (the host waits on the event behind the previous receive).
  WorkerPump(std::shared_ptr<GradLauncher> g, const Tensor& inbox, const Tensor& G, int n_loc,
             std::shared_ptr<eh::P2PComm> comm, int K, int device, double timeout)
      : g_(std::move(g)), inbox_(inbox), G_(G), n_(n_loc), mbox_(0), mbox_rows_(0), row0_(0), bflag_(nullptr),
        mflag_(nullptr), K_(K), timeout_(timeout), comm_(std::move(comm)) {
    need(comm_ != nullptr, "null communicator");
    need_gpu(inbox, "inbox");
    need_gpu(G, "G");
    need(G.dim() == 3 && G.size(0) == K && G.size(2) == inbox.size(1), "G must be [K, n, ld]");
    need(acc_code(G) == acc_code(inbox), "G/inbox dtype mismatch");
    need(n_loc >= 0 && n_loc <= G.size(1), "n_loc out of range");
    ld_ = (int)inbox.size(1);
    R_ = (int)inbox.size(0) - 1;
    device_ = device;
    es_ = acc_code(G) == 0 ? 8 : 4;
    g_rows_ = (int)G.size(1);
    stream_ = c10::hip::getCurrentHIPStream(device).stream();
    wait_s_.assign(R_, -1.0);
    for (auto& e : rev_) hcheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    err_ = std::make_unique<HostMapped>(sizeof(eh::IntegrityErr));
    abort_ = std::make_unique<HostMapped>(sizeof(int));
  }
  bool fused_put() const { return fuse_put_; }
  bool device_wait() const { return dwait_; }
  std::string comm_kind() const { return comm_ ? comm_->kind() : "ipc"; }

  // --delay-on worker: seconds this rank is physically late in every round.  A device spin
  // (wall_clock64 + s_sleep) between the gradient and the put, so the put really leaves late
  // while the rounds stay queued; the put is then its own kernel (not fused into the reduction).
  void set_delays(const std::vector<double>& seconds) {
    need((int)seconds.size() >= R_, "delays must cover R rounds");
    int khz = 0;
    hcheck(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_), "hipDeviceGetAttribute");
    late_ticks_.assign(R_, 0);
    for (int i = 0; i < R_; ++i)
      late_ticks_[i] = static_cast<long long>(std::min(seconds[i], 3600.0) * 1e3 * khz);
    if (std::any_of(late_ticks_.begin(), late_ticks_.end(), [](long long t) { return t > 0; })) fuse_put_ = false;
  }
  // --slow-ranks: the gradient runs `n` times per round.
  void set_repeat(int n) {
    need(n >= 1, "repeat must be >= 1");
    repeat_ = n;
  }

  // Drain "lazy": stale-round skipping (the replacement of the reference's send Cancel, ref
  // src/coded.py:178-180).  Every round's kernels carry a gate word (common.h gate_closed); round i's
  // put decides round i+1's: skip it iff this rank's beta counter (beta_flag_dev, its device address)
  // already says beta(i+2) is out, i.e. the master finished round i+1 before this rank could start it.
  // Decided on the device when the previous round ends, so a rank that fell behind (a late spin, a
  // slow GPU) jumps to the newest beta instead of computing stale rounds.  IPC mailbox only (RCCL has
  // no cancel: a skipped send would desynchronise the FIFO pairing).
  void set_skip_stale(uintptr_t beta_flag_dev) {
    need(!comm_, "stale-round skipping needs the IPC mailbox (p2p sends cannot be skipped)");
    need(beta_flag_dev != 0, "null beta flag");
    skip_flag_ = reinterpret_cast<const unsigned long long*>(beta_flag_dev);
    gate_ = at::zeros({R_ + 1}, at::TensorOptions().dtype(at::kInt).device(at::Device(at::kCUDA, device_)));
  }
  // The same over stream-ordered p2p (RCCL / loopback / rccl-self), where a send cannot be skipped: the
  // rank receives beta on a stream of its own, one round AHEAD of its compute (the reference pre-posts
  // every Irecv, ref src/naive.py:66-70), and bumps a device counter behind every receive (value j + 1
  // <=> beta(j) landed).  Round i's gate is snapshotted from it just before the round's gradient: closed
  // iff beta(i+1) already landed, i.e. the master decided round i before this rank could start it.  A
  // skipped round still SENDS (its stale rows keep the FIFO pairing of the master's receives) and lands
  // after its round ended, so the master drains it and never decodes it (collector.h stale arrivals).
  // The master's end-of-run beta(R) (MasterPump::finish_run) closes every round still queued.
  void set_skip_stale_comm() {
    need(comm_ != nullptr, "p2p stale-round skipping needs a communicator");
    if (skip_comm_) return;
    skip_comm_ = true;
    gate_ = at::zeros({R_ + 1}, at::TensorOptions().dtype(at::kInt).device(at::Device(at::kCUDA, device_)));
    bcount_ = at::zeros({1}, at::TensorOptions().dtype(at::kLong).device(at::Device(at::kCUDA, device_)));
    hcheck(hipStreamCreateWithFlags(&bst_, hipStreamNonBlocking), "hipStreamCreate(beta)");
    bev_.assign(R_ + 1, nullptr);
    for (auto& e : bev_) hcheck(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
  }
  bool skip_stale() const { return skip_flag_ != nullptr || skip_comm_; }

  // IPC: every message put writes {round + 1, landing ticks} into this rank's ring of shared host memory,
  // 16-byte slot i % ring (ring_dev: device address of the ring), read by the master's collector
  // (collector.h "Device times").
  void set_stamp_ring(uintptr_t ring_dev, int ring) {
    need(ring_dev == 0 || ring >= 1, "stamp ring must have >= 1 slot");
    ring_dev_ = ring_dev;
    ring_ = ring;
  }
  // Per-round device records (wall_clock64 ticks, -1 = not recorded), tests/lazy_check.py:
  //   [0] landing stamp of the round's put (IPC, written by the put kernel before its flag)
  //   [1] [2] just before / after the round's put or send      [3] [4] spin start / end (--delay-on worker)
  //   [5] [6] just before / after the stale-round gate (p2p)    [7] [8] just before / after the counter bump
  //   that announces beta(i) landed on this rank (p2p with stale-round skipping)
  //   [9] the round's start on this rank's stream: right behind its beta wait (device wait / receive), or
  //   where the host enqueued the round after its own wait -- the worker half of the master's chain
  static constexpr int kRec = 10;
  void set_records(bool on) {
    rec_ = on ? at::full({R_ + 1, kRec}, -1, at::TensorOptions().dtype(at::kLong).device(at::Device(at::kCUDA, device_)))
              : Tensor();
  }
  Tensor records() {
    hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    if (bst_) hcheck(hipStreamSynchronize(bst_), "hipStreamSynchronize");
    return rec_.defined() ? rec_.cpu() : Tensor();
  }
  // Rounds this rank skipped as stale (syncs the stream).
  std::vector<int> skipped_rounds() {
    std::vector<int> out;
    if (!gate_.defined()) return out;
    hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    const Tensor g = gate_.cpu();
    const int* v = g.data_ptr<int>();
    for (int i = 0; i < R_; ++i)
      if (v[i]) out.push_back(i);
    return out;
  }

  // Integrity tags (csrc/kernels/integrity.h): mbox_tags = this rank's view of the master
  // mailbox's tag slots [K][mbox_rows]; inbox_tags = its own inbox's tag slots [R + 1].  Every
  // message put carries a tag per row; every beta is checked after the round that read it.
  // Returns whether tags are on: a rank hosting more than kMaxTagRows message rows puts them untagged
  // (the caller records why) rather than failing its setup.
  bool set_integrity(uintptr_t mbox_tags, uintptr_t inbox_tags, int rank, bool on) {
    need(!on || (mbox_tags != 0 && inbox_tags != 0), "integrity tags need the tag slots");
    if (n_ > eh::kMaxTagRows) on = false;
    tags_ = on;
    mtags_ = reinterpret_cast<eh::MsgTag*>(mbox_tags);
    itags_ = reinterpret_cast<const eh::MsgTag*>(inbox_tags);
    rank_ = rank;
    return tags_;
  }
  // Raise the first failed beta check (host-mapped record), after releasing this rank's queued work.
  void check_integrity() {
    const auto* e = static_cast<const eh::IntegrityErr*>(err_->host);
    if (!__atomic_load_n(&e->flag, __ATOMIC_ACQUIRE)) return;
    stop_queued();
    throw std::runtime_error("rank " + std::to_string(rank_) + ": " + integrity_message(*e, true));
  }
  ~WorkerPump() {
    for (auto e : rev_)
      if (e) hipEventDestroy(e);
    // the beta stream is destroyed without a sync (a receive from a master that is gone may never end; the
    // transport aborts its communicator at close), like the master's per-peer streams
    for (auto e : bev_)
      if (e) hipEventDestroy(e);
    if (bst_) hipStreamDestroy(bst_);
    for (auto& t : tev_)
      for (auto e : t)
        if (e) hipEventDestroy(e);
  }

  void set_timing(bool on) {
    timing_ = on;
    if (on && tev_.empty()) tev_.assign(R_, {nullptr, nullptr, nullptr});
  }
  // (beta_wait_s [R], kernel_ms [R], put_ms [R]); -1 where a round was not timed.  Syncs the stream.
  std::tuple<std::vector<double>, std::vector<double>, std::vector<double>> timing() {
    hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    std::vector<double> ker(R_, -1.0), put(R_, -1.0);
    for (int i = 0; i < (int)tev_.size(); ++i) {
      const auto& t = tev_[i];
      float ms = 0.f;
      if (t[0] && t[1] && hipEventElapsedTime(&ms, t[0], t[1]) == hipSuccess) ker[i] = ms;
      if (t[1] && t[2] && hipEventElapsedTime(&ms, t[1], t[2]) == hipSuccess) put[i] = ms;
    }
    return {wait_s_, ker, put};
  }

  // Rounds [a, b).  Returns -1 when every round was issued, else the round whose beta
  // did not arrive within the timeout.
  int run(int a, int b) {
    if (comm_) return run_comm(a, b);
    py::gil_scoped_release nogil;
    for (int i = a; i < b; ++i) {
      need(i >= 0 && i < R_, "round out of range");
      Range tr("eh.worker.round");
      if (dwait_) {
        // enqueue round i once beta(i-1) is in: one round of lookahead, host timeout kept
        if (i > a && !host_wait(i, i - 1)) return release(i - 1);
        check_integrity();
        if (n_ == 0) continue;
        hcheck(hipStreamWaitValue64(stream_, bflag_dev_, static_cast<uint64_t>(i + 1), hipStreamWaitValueGte),
               "hipStreamWaitValue64(beta flag)");
      } else {
        if (!host_wait(i + 1, i)) return i;
        check_integrity();
        if (n_ == 0) continue;
      }
      stamp(i, 9, stream_);
      const int slot = i % K_;
      const char* beta = static_cast<const char*>(inbox_.data_ptr()) + static_cast<int64_t>(i) * ld_ * es_;
      char* g = static_cast<char*>(G_.data_ptr()) + static_cast<int64_t>(slot) * g_rows_ * ld_ * es_;
      const long long bytes = static_cast<long long>(n_) * ld_ * es_;
      eh::PutDesc pd{g, reinterpret_cast<char*>(mbox_) + (static_cast<int64_t>(slot) * mbox_rows_ + row0_) * ld_ * es_,
                     bytes, mflag_, static_cast<unsigned long long>(i + 1),
                     reinterpret_cast<unsigned int*>(counters_.data_ptr<int>())};
      pd.abort = static_cast<const int*>(abort_->dev);
      const int* gate = nullptr;  // stale-round gate of this round (set_skip_stale)
      if (skip_flag_) {
        int* gw = gate_.data_ptr<int>();
        gate = gw + i;
        pd.gate = gate;
        pd.next_gate = gw + i + 1;
        pd.beta_flag = skip_flag_;
        pd.stale_next = static_cast<unsigned long long>(i) + 3;  // round i+1 is stale once beta(i+2) is out
      }
      if (tags_) {
        pd.tag = mtags_ + static_cast<int64_t>(slot) * mbox_rows_ + row0_;
        pd.csum = reinterpret_cast<unsigned long long*>(csum_.data_ptr<int64_t>());
        pd.rows = n_;
        pd.es = es_;
        pd.rank = static_cast<unsigned int>(rank_);
        pd.corrupt = sabotage("msg", rank_, i) ? 1 : 0;
      }
      if (ring_dev_) pd.stamp = reinterpret_cast<long long*>(ring_dev_) + 2 * (i % ring_);
      pd.stamp_log = rec_at(i, 0);
      if (timing_) record_t(i, 0);
      for (int k = 1; k < repeat_; ++k) hcheck(g_->launch(beta, g, stream_, gate), "worker gradient (slow rank)");
      if (fuse_put_) {  // gradient + put + signal in one stream order, no separate put kernel
        hcheck(g_->launch_put(beta, g, pd, stream_), "worker gradient + put");
        if (timing_) record_t(i, 1);
      } else {
        hcheck(g_->launch(beta, g, stream_, gate), "worker gradient");
        if (timing_) record_t(i, 1);
        if (!late_ticks_.empty() && late_ticks_[i] > 0)  // after compute, before the send (ref src/naive.py:141-148)
          hcheck(eh::spin_launch(late_ticks_[i], stream_, gate, skip_flag_, static_cast<unsigned long long>(R_) + 1,
                                 rec_at(i, 3)),
                 "late worker spin");
        eh::PutArgs pa{};
        pa.n = 1;
        pa.d[0] = pd;
        const int blocks = (int)std::max<long long>(1, std::min<long long>(64, (bytes / 16 + 4095) / 4096));
        stamp(i, 1, stream_);
        hcheck(eh::put_signal_launch(pa, blocks, stream_), "put_signal(messages)");
        stamp(i, 2, stream_);
      }
      if (timing_) record_t(i, 2);
      if (tags_)  // beta(i) against its tag, behind the round that read it (off the critical path)
        hcheck(eh::verify_rows_launch(beta, itags_ + i, 1, ld_, es_, static_cast<unsigned int>(i + 1), 0u,
                                      static_cast<eh::IntegrityErr*>(err_->dev), -1, stream_),
               "verify_rows(beta)");
    }
    if (dwait_ && b > a && !host_wait(b, b - 1)) return release(b - 1);
    if (skip_flag_ && b == R_ && n_ > 0)  // every round is put or skipped: the master's collector can drain
      hcheck(eh::signal_launch(mflag_, static_cast<unsigned long long>(R_), stream_), "signal(rounds done)");
    if (tags_) {  // the last rounds' checks
      hcheck(hipStreamSynchronize(stream_), "hipStreamSynchronize");
      check_integrity();
    }
    return -1;
  }

 private:
  // Beta receives of rounds <= j on the beta stream (set_skip_stale_comm), each followed by the counter
  // bump and its event.
  void post_beta_upto(int j) {
    const int64_t bbytes = static_cast<int64_t>(ld_) * es_;
    auto* cnt = reinterpret_cast<unsigned long long*>(bcount_.data_ptr<int64_t>());
    for (; posted_ <= std::min(j, R_); ++posted_) {
      char* beta = static_cast<char*>(inbox_.data_ptr()) + static_cast<int64_t>(posted_) * bbytes;
      comm_->recv(0, beta, bbytes, bst_);
      stamp(posted_, 7, bst_);
      hcheck(eh::signal_launch(cnt, static_cast<unsigned long long>(posted_) + 1, bst_), "signal(beta landed)");
      stamp(posted_, 8, bst_);
      hcheck(hipEventRecord(bev_[posted_], bst_), "hipEventRecord(beta)");
    }
  }
  // run_comm with stale-round skipping (set_skip_stale_comm).
  int run_comm_skip(int a, int b) {
    py::gil_scoped_release nogil;
    if (posted_ == 0) posted_ = a;  // a resumed run: the master's first beta is beta(a)
    need(posted_ >= a, "rounds must run in order");
    auto* cnt = reinterpret_cast<const unsigned long long*>(bcount_.data_ptr<int64_t>());
    int* gw = gate_.data_ptr<int>();
    for (int i = a; i < b; ++i) {
      need(i >= 0 && i < R_, "round out of range");
      Range tr("eh.worker.round");
      if (i > a && !event_wait(bev_[i - 1], i - 1)) {  // beta(i-1) never came: the master is gone
        comm_->abort();
        return i - 1;
      }
      // beta(i+1) (or the end-of-run beta(R)) may land while round i waits.  Never past the segment: the
      // master publishes beta(b) only after the fence between segments (Trainer.run timed_start), and a
      // receive still posted would hold this rank's device synchronisation at that fence.
      post_beta_upto(b == R_ ? i + 1 : std::min(i + 1, b - 1));
      hcheck(hipStreamWaitEvent(stream_, bev_[i], 0), "hipStreamWaitEvent(beta)");
      if (n_ == 0) continue;
      stamp(i, 9, stream_);
      const char* beta = static_cast<const char*>(inbox_.data_ptr()) + static_cast<int64_t>(i) * ld_ * es_;
      char* g = static_cast<char*>(G_.data_ptr()) + static_cast<int64_t>(i % K_) * g_rows_ * ld_ * es_;
      // closed iff beta(i+1) landed before this round starts (value i + 2)
      stamp(i, 5, stream_);
      hcheck(eh::gate_launch(cnt, static_cast<unsigned long long>(i) + 2, gw + i, stream_), "gate(stale round)");
      stamp(i, 6, stream_);
      if (timing_) record_t(i, 0);
      for (int k = 0; k < repeat_; ++k) hcheck(g_->launch(beta, g, stream_, gw + i), "worker gradient");
      if (timing_) record_t(i, 1);
      if (!late_ticks_.empty() && late_ticks_[i] > 0)  // a skipped round does not spin; the end of the run stops one
        hcheck(eh::spin_launch(late_ticks_[i], stream_, gw + i, cnt, static_cast<unsigned long long>(R_) + 1,
                               rec_at(i, 3)),
               "late worker spin");
      stamp(i, 1, stream_);
      comm_->send(0, g, static_cast<int64_t>(n_) * ld_ * es_, stream_);  // always: the FIFO pairing
      stamp(i, 2, stream_);
      if (timing_) record_t(i, 2);
    }
    if (b > a && !event_wait(bev_[b - 1], b - 1)) {
      comm_->abort();
      return b - 1;
    }
    if (b == R_) {  // the master's end-of-run beta(R): nothing may stay posted on the communicator
      post_beta_upto(R_);
      if (!event_wait(bev_[R_], R_ - 1)) {
        comm_->abort();
        return R_ - 1;
      }
    }
    return -1;
  }
  int run_comm(int a, int b) {
    if (skip_comm_) return run_comm_skip(a, b);
    py::gil_scoped_release nogil;
    const int64_t bbytes = static_cast<int64_t>(ld_) * es_;
    for (int i = a; i < b; ++i) {
      need(i >= 0 && i < R_, "round out of range");
      Range tr("eh.worker.round");
      if (i > a && !event_wait(rev_[(i - 1) % 2], i - 1)) {  // beta(i-1) never came: the master is gone
        comm_->abort();
        return i - 1;
      }
      char* beta = static_cast<char*>(inbox_.data_ptr()) + static_cast<int64_t>(i) * bbytes;
      comm_->recv(0, beta, bbytes, stream_);
      hcheck(hipEventRecord(rev_[i % 2], stream_), "hipEventRecord(beta)");
      if (n_ == 0) continue;
      stamp(i, 9, stream_);
      char* g = static_cast<char*>(G_.data_ptr()) + static_cast<int64_t>(i % K_) * g_rows_ * ld_ * es_;
      if (timing_) record_t(i, 0);
      for (int k = 0; k < repeat_; ++k) hcheck(g_->launch(beta, g, stream_), "worker gradient");
      if (timing_) record_t(i, 1);
      if (!late_ticks_.empty() && late_ticks_[i] > 0)  // after compute, before the send (ref src/naive.py:141-148)
        hcheck(eh::spin_launch(late_ticks_[i], stream_, nullptr, nullptr, 0, rec_at(i, 3)), "late worker spin");
      stamp(i, 1, stream_);
      comm_->send(0, g, static_cast<int64_t>(n_) * ld_ * es_, stream_);
      stamp(i, 2, stream_);
      if (timing_) record_t(i, 2);
    }
    if (b > a && !event_wait(rev_[(b - 1) % 2], b - 1)) {
      comm_->abort();
      return b - 1;
    }
    return -1;
  }
  // Host poll of a receive event (comm mode); records the wait under round `rec`.
  bool event_wait(hipEvent_t ev, int rec) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (int spin = 0;; ++spin) {
      const hipError_t q = hipEventQuery(ev);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) hcheck(q, "hipEventQuery(beta)");
      if (spin < 4096) {
#if defined(__x86_64__)
        _mm_pause();
#endif
        continue;
      }
      if (std::chrono::duration<double>(clk::now() - t0).count() > timeout_) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
    wait_s_[rec] = std::chrono::duration<double>(clk::now() - t0).count();
    return true;
  }

  // Host poll until the beta flag reaches `target`; records the wait under round `rec`.
  bool host_wait(uint64_t target, int rec) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (int spin = 0; __atomic_load_n(bflag_, __ATOMIC_ACQUIRE) < target; ++spin) {
      if (spin < 4096) {
#if defined(__x86_64__)
        _mm_pause();
#endif
        continue;
      }
      if (std::chrono::duration<double>(clk::now() - t0).count() > timeout_) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
    wait_s_[rec] = std::chrono::duration<double>(clk::now() - t0).count();
    return true;
  }
  // Timeout with device-side waits queued: the master is gone (or late beyond the timeout).  The
  // queued rounds must not announce messages computed on a beta that never arrived, so the abort
  // word goes up FIRST (every queued put / put+signal kernel checks it and skips its put and its
  // signal), then this rank's own stream waits are released (the flag value they wait for) so no
  // wait is left on the GPU.  Returns the round that timed out.
  int release(int bad) {
    stop_queued();
    return bad;
  }
  void stop_queued() {
    if (comm_) {
      comm_->abort();
      return;
    }
    __atomic_store_n(static_cast<int*>(abort_->host), 1, __ATOMIC_RELEASE);
    if (dwait_) {
      const uint64_t top = static_cast<uint64_t>(R_) + 1;
      if (__atomic_load_n(bflag_, __ATOMIC_ACQUIRE) < top) __atomic_store_n(bflag_, top, __ATOMIC_RELEASE);
    }
    hipStreamSynchronize(stream_);
  }

  void record_t(int i, int which) {
    hipEvent_t& e = tev_[i][which];
    if (!e) hcheck(hipEventCreate(&e), "hipEventCreate");
    hcheck(hipEventRecord(e, stream_), "hipEventRecord");
  }
  // Address of record field `f` of round i (nullptr when records are off).
  long long* rec_at(int i, int f) {
    if (!rec_.defined() || i < 0 || i > R_) return nullptr;
    return reinterpret_cast<long long*>(rec_.data_ptr<int64_t>()) + static_cast<int64_t>(i) * kRec + f;
  }
  void stamp(int i, int f, hipStream_t st) {
    if (long long* p = rec_at(i, f)) hcheck(eh::stamp_launch(p, st), "stamp(record)");
  }

  std::shared_ptr<GradLauncher> g_;
  Tensor inbox_, G_;
  int n_;
  uintptr_t mbox_;
  int mbox_rows_, row0_;
  uint64_t* bflag_;
  void* bflag_dev_ = nullptr;
  uintptr_t ring_dev_ = 0;  // set_stamp_ring
  int ring_ = 1;
  Tensor rec_;              // set_records
  unsigned long long* mflag_;
  Tensor counters_;
  int K_;
  double timeout_;
  int ld_ = 0, R_ = 0, es_ = 8, g_rows_ = 1;
  hipStream_t stream_ = nullptr;
  bool timing_ = false;
  bool fuse_put_ = false;
  bool dwait_ = false;
  bool tags_ = false;
  eh::MsgTag* mtags_ = nullptr;          // master mailbox tag slots (this rank's mapping)
  const eh::MsgTag* itags_ = nullptr;    // own inbox tag slots
  int rank_ = 0;
  std::unique_ptr<HostMapped> err_;      // first failed beta check (eh::IntegrityErr)
  std::unique_ptr<HostMapped> abort_;    // int: queued puts skip themselves once set
  Tensor csum_;                          // tagged put checksum scratch [kMaxTagRows]
  std::vector<long long> late_ticks_;    // [R] device spin before the put (--delay-on worker)
  const unsigned long long* skip_flag_ = nullptr;  // beta counter read by the stale-round gates (lazy drain)
  Tensor gate_;                          // int32 [R + 1] stale-round gates (1 = round skipped)
  bool skip_comm_ = false;               // p2p stale-round skipping (set_skip_stale_comm)
  Tensor bcount_;                        // int64 [1]: j + 1 once beta(j) landed (p2p skipping)
  hipStream_t bst_ = nullptr;            // beta receive stream (p2p skipping)
  std::vector<hipEvent_t> bev_;          // [R + 1] beta(j) landed (p2p skipping)
  int posted_ = 0;                       // beta receives posted on bst_ so far
  int repeat_ = 1;                       // gradient launches per round (--slow-ranks)
  int device_ = 0;
  std::shared_ptr<eh::P2PComm> comm_;    // stream-ordered p2p (null: IPC mailbox)
  std::array<hipEvent_t, 2> rev_{};      // beta receive-done events of the last two rounds (comm mode)
  std::vector<std::array<hipEvent_t, 3>> tev_;  // [round] gradient start, gradient end = put start, put end
  std::vector<double> wait_s_;                  // [round] host seconds spent waiting for beta
};

}  // namespace

namespace eh {
// Test probe of hardware-queue independence: a wait on its own host flag, then an event, on every given
// stream; the flags are released in REVERSE order and each stream's event must complete before the next
// release.  A stream sharing an in-order hardware queue with an earlier one stays parked behind that
// stream's unreleased wait (its event times out).  Every flag is released before returning, so nothing
// stays queued.  Returns, per stream, whether its event completed within `timeout` seconds of its release.
std::vector<bool> stream_wait_probe(const std::vector<uintptr_t>& streams, double timeout) {
  const size_t n = streams.size();
  uint64_t* h = nullptr;
  hcheck(hipHostMalloc(reinterpret_cast<void**>(&h), sizeof(uint64_t) * std::max<size_t>(1, n),
                       hipHostMallocMapped | hipHostMallocCoherent),
         "hipHostMalloc(probe flags)");
  for (size_t k = 0; k < n; ++k) h[k] = 0;
  uint64_t* d = nullptr;
  hcheck(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0), "hipHostGetDevicePointer");
  std::vector<hipEvent_t> ev(n, nullptr);
  std::vector<bool> ok(n, false);
  for (size_t k = 0; k < n; ++k) {
    hipStream_t st = reinterpret_cast<hipStream_t>(streams[k]);
    hcheck(hipEventCreateWithFlags(&ev[k], hipEventDisableTiming), "hipEventCreate");
    hcheck(hipStreamWaitValue64(st, d + k, 1, hipStreamWaitValueGte), "hipStreamWaitValue64(probe)");
    hcheck(hipEventRecord(ev[k], st), "hipEventRecord(probe)");
  }
  {
    py::gil_scoped_release nogil;
    for (size_t j = 0; j < n; ++j) {
      const size_t k = n - 1 - j;
      __atomic_store_n(h + k, uint64_t{1}, __ATOMIC_RELEASE);
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        const hipError_t q = hipEventQuery(ev[k]);
        if (q == hipSuccess) { ok[k] = true; break; }
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout) break;
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    }
    for (size_t k = 0; k < n; ++k) __atomic_store_n(h + k, uint64_t{1}, __ATOMIC_RELEASE);
    for (size_t k = 0; k < n; ++k) hipEventSynchronize(ev[k]);
  }
  for (auto e : ev) hipEventDestroy(e);
  hipHostFree(h);
  return ok;
}

// This GPU's wall_clock64 against the host clock (Collector::now): (tick0, t0, hz) such that
// t = t0 + (ticks - tick0) / hz.  A one-thread kernel stores its clock into host-mapped memory and the
// host spins until it lands; of `tries` samples the one with the shortest launch -> seen time wins (its
// t0 lags the device store by the store's visibility latency, about a microsecond).
std::tuple<double, double, double> device_clock(int device, int tries) {
  int khz = 0;
  hcheck(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device), "hipDeviceGetAttribute");
  need(khz > 0, "device reports no wall clock rate");
  HostMapped slot(sizeof(long long));
  auto* h = static_cast<volatile long long*>(slot.host);
  hipStream_t st = c10::hip::getCurrentHIPStream(device).stream();
  hcheck(hipStreamSynchronize(st), "hipStreamSynchronize");
  double best = 1e30, tick0 = 0.0, t0 = 0.0;
  py::gil_scoped_release nogil;
  for (int k = 0; k < std::max(1, tries); ++k) {
    *h = -1;
    const double ta = eh::Collector::now();
    hcheck(eh::stamp_launch(static_cast<long long*>(slot.dev), st), "stamp(clock)");
    double tb = ta;
    for (;;) {
      tb = eh::Collector::now();
      if (*h != -1) break;
      if (tb - ta > 5.0) throw std::runtime_error("device_clock: the stamp never landed");
    }
    if (tb - ta < best) {
      best = tb - ta;
      tick0 = static_cast<double>(*h);
      t0 = tb;
    }
  }
  hcheck(hipStreamSynchronize(st), "hipStreamSynchronize");
  return {tick0, t0, 1e3 * khz};
}

void bind_engine(py::module& m) {
  m.def("stream_wait_probe", &stream_wait_probe, py::arg("streams"), py::arg("timeout"));
  m.def("device_clock", &device_clock, py::arg("device"), py::arg("tries") = 16,
        "(tick0, t0, hz): this GPU's wall_clock64 against the host clock, t = t0 + (ticks - tick0) / hz");
  py::class_<GradLauncher, std::shared_ptr<GradLauncher>>(m, "GradLauncher")
      .def_static("dense", &make_dense, py::arg("dtype"), py::arg("loss"), py::arg("cpl"), py::arg("segs"),
                  py::arg("tasks"), py::arg("slab"), py::arg("slot_task_begin"), py::arg("part"), py::arg("ld"),
                  py::arg("task_row_off") = py::none(), py::arg("rbuf") = py::none(),
                  py::arg("choice") = eh::KernelChoice{})
      .def_static("sparse", &make_sparse, py::arg("loss"), py::arg("y"), py::arg("u"), py::arg("ell_idx"), py::arg("lo"),
                  py::arg("row_ptr"), py::arg("col_idx"), py::arg("vals"), py::arg("crow"), py::arg("cvals"),
                  py::arg("col_ptr"), py::arg("tiles"), py::arg("part_entry0"), py::arg("part_row0"),
                  py::arg("part_nnz"), py::arg("head"), py::arg("tail"), py::arg("span"), py::arg("empty"),
                  py::arg("nparts"), py::arg("d"), py::arg("ld"), py::arg("wg") = py::none(), py::arg("u_lds") = 0,
                  py::arg("Gs") = py::none(), py::arg("sub_begin") = py::none(),
                  py::arg("runs") = py::none(), py::arg("tkeys") = py::none(), py::arg("wspan") = py::none(),
                  py::arg("wspan_ptr") = py::none(), py::arg("dst") = py::none(), py::arg("csr_fixed") = 0)
      .def("set_encode",
           [](GradLauncher& g, const Tensor& ptr, const Tensor& idx, const Tensor& coef, const Tensor& Gb) {
             for (auto* t : {&ptr, &idx, &coef, &Gb}) need_gpu(*t, "encode operand");
             need(ptr.scalar_type() == at::kInt && idx.scalar_type() == at::kInt, "encode ptr/idx must be int32");
             need(coef.scalar_type() == at::kDouble, "encode coefficients must be fp64");
             need(Gb.dim() == 2 && Gb.size(0) == g.nslots && Gb.size(1) == g.ld && acc_code(Gb) == g.acc,
                  "Gb must be [distinct partitions, ld] in the accumulator dtype");
             need(idx.numel() == coef.numel(), "encode idx/coef size mismatch");
             g.enc_slots = (int)ptr.numel() - 1;
             g.Gb = Gb.data_ptr();
             g.enc_ptr = ptr.data_ptr<int>();
             g.enc_idx = idx.data_ptr<int>();
             g.enc_coef = coef.data_ptr<double>();
             for (auto* t : {&ptr, &idx, &coef, &Gb}) g.keep.push_back(*t);
           })
      .def(
          "launch",
          [](const GradLauncher& g, const Tensor& beta, const Tensor& G, std::optional<Tensor> gate) {
            need_gpu(beta, "beta");
            need_gpu(G, "G");
            if (gate) need(gate->is_cuda() && gate->scalar_type() == at::kInt && gate->numel() >= 1, "gate: int32 GPU");
            hcheck(g.launch(beta.data_ptr(), G.data_ptr(), c10::hip::getCurrentHIPStream(G.device().index()).stream(),
                            gate ? gate->data_ptr<int>() : nullptr),
                   "GradLauncher.launch");
          },
          py::arg("beta"), py::arg("G"), py::arg("gate") = py::none());
  py::class_<MasterPump>(m, "MasterPump")
      .def(py::init<eh::Collector*, int, int, int, int, int, int, double>(), py::arg("collector"), py::arg("W"),
           py::arg("R"), py::arg("K"), py::arg("d"), py::arg("ld"), py::arg("device"), py::arg("timeout"),
           py::keep_alive<1, 2>())
      .def("set_state", &MasterPump::set_state)
      .def("set_local", &MasterPump::set_local)
      .def("set_remote", &MasterPump::set_remote)
      .def("set_puts", &MasterPump::set_puts)
      .def("set_drain_flags", &MasterPump::set_drain_flags)
      .def("set_remote_delays", &MasterPump::set_remote_delays)
      .def("set_comm", &MasterPump::set_comm, py::arg("comm"), py::arg("ranks"), py::arg("peers"))
      .def_property_readonly("comm_kind", &MasterPump::comm_kind)
      .def("set_repeat", &MasterPump::set_repeat)
      .def("set_skip_stale", &MasterPump::set_skip_stale, py::arg("on"))
      .def_property_readonly("comm_streams", &MasterPump::comm_streams)
      .def("stream_handles", &MasterPump::stream_handles)
      .def("finish_run", &MasterPump::finish_run)
      .def_property_readonly("skipped", &MasterPump::skipped)
      .def_property_readonly("stale_arrivals", &MasterPump::stale_arrivals)
      .def("set_integrity", &MasterPump::set_integrity, py::arg("mbox_tags"), py::arg("inbox_tag_off"), py::arg("on"))
      .def_property_readonly("integrity", &MasterPump::integrity)
      .def("check_integrity", &MasterPump::check_integrity)
      .def("check_rows_cut", &MasterPump::check_rows_cut)
      .def("final_check", &MasterPump::final_check)
      .def("set_sources", &MasterPump::set_sources)
      .def("device_blocker", &MasterPump::device_blocker)
      .def("run_device", &MasterPump::run_device, py::arg("a"), py::arg("b"), py::arg("deadline_s"))
      .def("device_log", &MasterPump::device_log)
      .def("set_schedule", &MasterPump::set_schedule)
      .def("set_decode", &MasterPump::set_decode)
      .def("add_table", &MasterPump::add_table)
      .def("begin", &MasterPump::begin, py::call_guard<py::gil_scoped_release>())
      .def("finish", &MasterPump::finish)
      .def("resolve", &MasterPump::resolve)
      .def("update_ms", &MasterPump::update_ms)
      .def("run_local", &MasterPump::run_local, py::arg("a"), py::arg("b"), py::arg("graph"), py::arg("stamps"))
      .def("stamp_hz", &MasterPump::stamp_hz)
      .def("set_timing", &MasterPump::set_timing)
      .def("timing_ms", &MasterPump::timing_ms)
      .def("graphs_launched", &MasterPump::graphs_launched)
      .def("set_fused_update", &MasterPump::set_fused_update, py::arg("on"))
      .def("set_device_times", &MasterPump::set_device_times, py::arg("clocks"), py::arg("ring_host"), py::arg("ring"))
      .def("set_records", &MasterPump::set_records, py::arg("on"))
      .def("records", &MasterPump::records)
      .def("probe_log", [](MasterPump& p) { return p.probe_log(); });
  py::class_<WorkerPump>(m, "WorkerPump")
      .def(py::init<std::shared_ptr<GradLauncher>, const Tensor&, const Tensor&, int, uintptr_t, int, int, uintptr_t,
                    uintptr_t, const Tensor&, int, int, double, uintptr_t>(),
           py::arg("g"), py::arg("inbox"), py::arg("G"), py::arg("n_loc"), py::arg("mbox_base"), py::arg("mbox_rows"),
           py::arg("row0"), py::arg("beta_flag_host"), py::arg("msg_flag_dev"), py::arg("counters"), py::arg("K"),
           py::arg("device"), py::arg("timeout"), py::arg("beta_flag_dev") = 0)
      .def(py::init<std::shared_ptr<GradLauncher>, const Tensor&, const Tensor&, int, std::shared_ptr<eh::P2PComm>, int,
                    int, double>(),
           py::arg("g"), py::arg("inbox"), py::arg("G"), py::arg("n_loc"), py::arg("comm"), py::arg("K"),
           py::arg("device"), py::arg("timeout"))
      .def_property_readonly("comm_kind", &WorkerPump::comm_kind)
      .def("run", &WorkerPump::run)
      .def_property_readonly("fused_put", &WorkerPump::fused_put)
      .def_property_readonly("device_wait", &WorkerPump::device_wait)
      .def("set_timing", &WorkerPump::set_timing)
      .def("set_delays", &WorkerPump::set_delays)
      .def("set_repeat", &WorkerPump::set_repeat)
      .def("set_skip_stale", &WorkerPump::set_skip_stale, py::arg("beta_flag_dev"))
      .def("set_skip_stale_comm", &WorkerPump::set_skip_stale_comm)
      .def_property_readonly("skip_stale", &WorkerPump::skip_stale)
      .def("skipped_rounds", &WorkerPump::skipped_rounds)
      .def("set_integrity", &WorkerPump::set_integrity, py::arg("mbox_tags"), py::arg("inbox_tags"), py::arg("rank"),
           py::arg("on"))
      .def("check_integrity", &WorkerPump::check_integrity)
      .def("timing", &WorkerPump::timing)
      .def("set_stamp_ring", &WorkerPump::set_stamp_ring, py::arg("ring_dev"), py::arg("ring"))
      .def("set_records", &WorkerPump::set_records, py::arg("on"))
      .def("records", &WorkerPump::records);
}
}  // namespace eh
