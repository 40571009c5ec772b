// Python bindings of the native ErasureHead MI355X runtime (_C extension).
//
// Every kernel entry point launches on the caller's current HIP stream (the engine
// pins compute, per-peer receive and update work to separate streams) and validates
// shapes on the host before launch, so a malformed table can never reach the GPU.
#include <c10/hip/HIPStream.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <optional>
#include <stdexcept>
#include <string>
#include <vector>

#include "runtime/collector.h"

#include "kernels/launchers.h"

namespace eh {
void bind_ipc(pybind11::module& m);     // csrc/runtime/ipc.cpp
void bind_engine(pybind11::module& m);  // csrc/runtime/engine.cpp
}  // namespace eh

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

void check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

hipStream_t stream_of(const Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

void need(bool ok, const std::string& msg) {
  if (!ok) throw std::invalid_argument(msg);
}

void need_cuda(const Tensor& t, const char* name) {
  need(t.is_cuda(), std::string(name) + " must be a GPU tensor");
  need(t.is_contiguous(), std::string(name) + " must be contiguous");
}

// dtype code of the worker compute path: 0 fp64, 1 fp32, 2 bf16 storage (fp32 acc)
int acc_code(const Tensor& t) {
  if (t.scalar_type() == at::kDouble) return 0;
  if (t.scalar_type() == at::kFloat) return 1;
  throw std::invalid_argument("accumulator tensors must be float64 or float32");
}

constexpr int64_t kSplits = 16;  // must match csrc/kernels/grad_dense.hip

void need_part(const Tensor& part, int64_t nslots, int64_t ld, int ac) {
  need_cuda(part, "part");
  need(part.numel() >= nslots * kSplits * ld && acc_code(part) == ac, "part must be [nslots*16*ld] acc dtype");
}

void grad_dense(int64_t dtype, int64_t loss, int64_t cpl, const Tensor& segs, const Tensor& tasks,
                const Tensor& beta, const Tensor& slab, const Tensor& slot_task_begin, const Tensor& part,
                const Tensor& G, int64_t ld, int64_t variant) {
  need_cuda(segs, "segs");
  need_cuda(tasks, "tasks");
  need_cuda(beta, "beta");
  need_cuda(slab, "slab");
  need_cuda(slot_task_begin, "slot_task_begin");
  need_cuda(G, "G");
  const int64_t ntasks = tasks.size(0);
  const int64_t nslots = slot_task_begin.numel() - 1;
  need(tasks.dim() == 2 && tasks.size(1) == 5 && tasks.scalar_type() == at::kInt, "tasks must be int32 [ntasks, 5]");
  need(segs.scalar_type() == at::kByte && segs.numel() % 32 == 0, "segs must be packed uint8 [nseg*32]");
  need(slab.dim() == 2 && slab.size(0) >= ntasks && slab.size(1) == ld, "slab must be [>=ntasks, ld]");
  need(G.dim() == 2 && G.size(0) == nslots && G.size(1) == ld, "G must be [nslots, ld]");
  need(beta.numel() >= ld, "beta must have >= ld elements");
  need(ld % (dtype == 0 ? 2 : dtype == 1 ? 4 : 8) == 0, "ld must be a multiple of the 16-byte vector width");
  need(cpl <= 32 ? cpl * 64 >= ld
                   : ((cpl == 256 || cpl == 512) && cpl * (dtype == 0 ? 16 : 32) >= ld),
         "cpl (narrow: columns per lane, wide: block size) must cover ld");
  const int ac = dtype == 0 ? 0 : 1;
  need(acc_code(beta) == ac && acc_code(slab) == ac && acc_code(G) == ac, "beta/slab/G dtype mismatch");
  need_part(part, nslots, ld, ac);
  if (ntasks == 0) return;
  check(eh::grad_dense_launch((int)dtype, (int)loss, (int)cpl, segs.data_ptr(), tasks.data_ptr(), (int)ntasks,
                              beta.data_ptr(), slab.data_ptr(), slot_task_begin.data_ptr<int>(), (int)nslots,
                              part.data_ptr(), G.data_ptr(), (int)ld, stream_of(G), (int)variant),
        "grad_dense");
}

void grad_dense_twopass(int64_t dtype, int64_t loss, const Tensor& segs, const Tensor& tasks,
                        const Tensor& beta, const Tensor& task_row_off, const Tensor& rbuf,
                        const Tensor& slab, const Tensor& slot_task_begin, const Tensor& part, const Tensor& G,
                        int64_t ld) {
  need_cuda(segs, "segs");
  need_cuda(tasks, "tasks");
  need_cuda(beta, "beta");
  need_cuda(task_row_off, "task_row_off");
  need_cuda(rbuf, "rbuf");
  need_cuda(slab, "slab");
  need_cuda(G, "G");
  const int64_t ntasks = tasks.size(0);
  const int64_t nslots = slot_task_begin.numel() - 1;
  need(slab.dim() == 2 && slab.size(0) >= ntasks && slab.size(1) == ld, "slab must be [>=ntasks, ld]");
  need(G.dim() == 2 && G.size(0) == nslots && G.size(1) == ld, "G must be [nslots, ld]");
  need(task_row_off.numel() >= ntasks, "task_row_off too small");
  need_part(part, nslots, ld, acc_code(G));
  need(rbuf.numel() >= 1 && acc_code(rbuf) == acc_code(G) && acc_code(beta) == acc_code(G), "rbuf/beta dtype");
  if (ntasks == 0) return;
  check(eh::grad_dense_twopass_launch((int)dtype, (int)loss, segs.data_ptr(), tasks.data_ptr(), (int)ntasks,
                                      beta.data_ptr(), task_row_off.data_ptr<int>(), rbuf.data_ptr(),
                                      slab.data_ptr(), slot_task_begin.data_ptr<int>(), (int)nslots,
                                      part.data_ptr(), G.data_ptr(), (int)ld, stream_of(G)),
        "grad_dense_twopass");
}

void grad_sparse(int64_t loss, const Tensor& row_ptr, const Tensor& col_idx, const OptT& vals,
                 const Tensor& y, const Tensor& coef, const Tensor& beta, const Tensor& rbuf,
                 const Tensor& keys, const Tensor& rows, const OptT& cvals, const Tensor& G, int64_t ld) {
  for (auto* p : {&row_ptr, &col_idx, &y, &coef, &beta, &rbuf, &keys, &rows, &G}) need_cuda(*p, "sparse operand");
  need(row_ptr.scalar_type() == at::kLong && keys.scalar_type() == at::kLong, "row_ptr/keys must be int64");
  need(col_idx.scalar_type() == at::kInt && rows.scalar_type() == at::kInt, "col_idx/rows must be int32");
  const int ac = acc_code(G);
  need(acc_code(y) == ac && acc_code(coef) == ac && acc_code(beta) == ac && acc_code(rbuf) == ac, "dtype mismatch");
  const int64_t nrows = row_ptr.numel() - 1;
  need(y.numel() == nrows && coef.numel() == nrows && rbuf.numel() >= nrows, "row arrays must match row_ptr");
  need(keys.numel() == rows.numel(), "keys/rows size mismatch");
  if (vals) need(vals->is_cuda() && acc_code(*vals) == ac && vals->numel() == col_idx.numel(), "vals mismatch");
  if (cvals) need(cvals->is_cuda() && acc_code(*cvals) == ac && cvals->numel() == keys.numel(), "cvals mismatch");
  check(eh::grad_sparse_launch(ac, (int)loss, (const long long*)row_ptr.data_ptr<int64_t>(),
                               col_idx.data_ptr<int>(), vals ? vals->data_ptr() : nullptr, y.data_ptr(),
                               coef.data_ptr(), beta.data_ptr(), rbuf.data_ptr(), (long long)nrows,
                               (const long long*)keys.data_ptr<int64_t>(), rows.data_ptr<int>(),
                               cvals ? cvals->data_ptr() : nullptr, (long long)keys.numel(), G.data_ptr(),
                               (long long)G.numel(), (int)ld, stream_of(G)),
        "grad_sparse");
}

void encode_messages(const Tensor& Gb, const Tensor& ptr, const Tensor& idx, const Tensor& coef, const Tensor& G) {
  for (auto* p : {&Gb, &ptr, &idx, &coef, &G}) need_cuda(*p, "encode operand");
  need(ptr.scalar_type() == at::kInt && idx.scalar_type() == at::kInt, "ptr/idx must be int32");
  need(coef.scalar_type() == at::kDouble && coef.numel() == idx.numel(), "coef must be fp64, one per idx");
  const int ac = acc_code(G);
  need(acc_code(Gb) == ac && Gb.dim() == 2 && G.dim() == 2 && Gb.size(1) == G.size(1), "Gb/G mismatch");
  need(ptr.numel() == G.size(0) + 1, "ptr must have nslots + 1 entries");
  check(eh::encode_messages_launch(ac, Gb.data_ptr(), ptr.data_ptr<int>(), idx.data_ptr<int>(),
                                   coef.data_ptr<double>(), G.data_ptr(), (int)G.size(0), (int)G.size(1),
                                   stream_of(G)),
        "encode_messages");
}

void grad_ell(int64_t loss, const Tensor& idx, const OptT& vals, const Tensor& y, const Tensor& coef,
              const Tensor& beta, const Tensor& rbuf, const Tensor& chunks, const Tensor& lo, const Tensor& width,
              int64_t max_width, const Tensor& G, int64_t ld) {
  for (auto* p : {&idx, &y, &coef, &beta, &rbuf, &chunks, &lo, &width, &G}) need_cuda(*p, "ell operand");
  need(idx.dim() == 2 && idx.scalar_type() == at::kInt, "idx must be int32 [m, nrows]");
  need(chunks.dim() == 2 && chunks.size(1) == 4 && chunks.scalar_type() == at::kInt, "chunks must be int32 [n, 4]");
  need(lo.scalar_type() == at::kInt && width.scalar_type() == at::kInt, "lo/width must be int32");
  const int64_t m = idx.size(0), nrows = idx.size(1);
  need(lo.numel() == m && width.numel() == m, "lo/width must have m entries");
  const int ac = acc_code(G);
  need(acc_code(y) == ac && acc_code(coef) == ac && acc_code(beta) == ac && acc_code(rbuf) == ac, "dtype mismatch");
  need(y.numel() == nrows && coef.numel() == nrows && rbuf.numel() >= nrows, "row arrays must match idx");
  need(G.dim() == 2 && G.size(1) == ld && beta.numel() >= ld, "G must be [nslots, ld]");
  if (vals) need(vals->is_cuda() && acc_code(*vals) == ac && vals->sizes() == idx.sizes(), "vals must match idx");
  need(nrows < (int64_t(1) << 31), "ELL rows must fit int32");
  check(eh::grad_ell_launch(ac, (int)loss, idx.data_ptr<int>(), vals ? vals->data_ptr() : nullptr, y.data_ptr(),
                            coef.data_ptr(), beta.data_ptr(), rbuf.data_ptr(), (long long)nrows, (int)m,
                            chunks.data_ptr(), (int)chunks.size(0), lo.data_ptr<int>(), width.data_ptr<int>(),
                            (int)max_width, G.data_ptr(), (long long)G.numel(), (int)ld, stream_of(G)),
        "grad_ell");
}

void combine_update(const std::vector<Tensor>& msgs, const std::vector<double>& coefs, const Tensor& beta,
                    const Tensor& u, const OptT& hist, const OptT& beta_w, const OptT& g_out, int64_t d,
                    double decay, double gm, double l2, double theta, int64_t rule) {
  need(msgs.size() == coefs.size(), "msgs/coefs length mismatch");
  need(static_cast<int>(msgs.size()) <= eh::kMaxMsgs, "too many messages for one combine");
  need_cuda(beta, "beta");
  need_cuda(u, "u");
  need(beta.scalar_type() == at::kDouble && u.scalar_type() == at::kDouble, "beta/u must be float64");
  const int64_t ld = beta.numel();
  need(d <= ld, "d must be <= ld");
  eh::CombineArgs args{};
  args.nmsg = static_cast<int>(msgs.size());
  int mcode = 0;
  for (size_t i = 0; i < msgs.size(); ++i) {
    need_cuda(msgs[i], "message");
    need(msgs[i].numel() >= ld, "message shorter than ld");
    const int c = acc_code(msgs[i]);
    if (i == 0) mcode = c;
    need(c == mcode, "all messages must share a dtype");
    args.msg[i] = msgs[i].data_ptr();
    args.coef[i] = coefs[i];
  }
  int wcode = 0;
  if (beta_w) {
    need_cuda(*beta_w, "beta_w");
    need(beta_w->numel() == ld, "beta_w size mismatch");
    wcode = acc_code(*beta_w);
  }
  if (hist) need(hist->is_cuda() && hist->scalar_type() == at::kDouble && hist->numel() >= d, "hist mismatch");
  if (g_out) need(g_out->is_cuda() && g_out->scalar_type() == at::kDouble && g_out->numel() >= d, "g_out mismatch");
  check(eh::combine_update_launch(args, mcode, wcode, beta.data_ptr<double>(), u.data_ptr<double>(),
                                  hist ? hist->data_ptr<double>() : nullptr, beta_w ? beta_w->data_ptr() : nullptr,
                                  g_out ? g_out->data_ptr<double>() : nullptr, (int)d, (int)ld, decay, gm, l2,
                                  theta, (int)rule, stream_of(beta)),
        "combine_update");
}

void eval_gemm_loss(int64_t loss_kind, const Tensor& X, int64_t n, int64_t d, const Tensor& y, const Tensor& B,
                    const Tensor& loss_out, const OptT& P) {
  need_cuda(X, "X");
  need_cuda(y, "y");
  need_cuda(B, "B");
  need_cuda(loss_out, "loss_out");
  need(X.dim() == 2 && X.size(0) >= n && X.size(1) >= d, "X must be [>=n, >=d]");
  int xcode;
  if (X.scalar_type() == at::kDouble) xcode = 0;
  else if (X.scalar_type() == at::kFloat) xcode = 1;
  else if (X.scalar_type() == at::kBFloat16) xcode = 2;
  else throw std::invalid_argument("X must be float64, float32 or bfloat16");
  const int ac = xcode == 0 ? 0 : 1;
  need(acc_code(y) == ac && acc_code(B) == ac, "y/B dtype must match the accumulator of X");
  need(B.dim() == 2 && B.size(1) >= d, "B must be [R, >=d]");
  need(y.numel() >= n, "y too short");
  const int64_t R = B.size(0);
  need(loss_out.scalar_type() == at::kDouble && loss_out.numel() >= R, "loss_out must be float64 [R]");
  if (P) need(P->is_cuda() && acc_code(*P) == ac && P->numel() >= n * R, "P must be [n, R]");
  check(eh::eval_gemm_loss_launch(xcode, (int)loss_kind, X.data_ptr(), X.size(1), n, (int)d, y.data_ptr(),
                                  B.data_ptr(), (int)B.size(1), (int)R, loss_out.data_ptr<double>(),
                                  P ? P->data_ptr() : nullptr, stream_of(X)),
        "eval_gemm_loss");
}

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "ErasureHead MI355X native runtime: gfx950 HIP kernels + arrival collector + IPC mailbox";
  eh::bind_ipc(m);
  eh::bind_engine(m);
  m.def("grad_dense", &grad_dense);
  m.def("grad_dense_twopass", &grad_dense_twopass);
  m.def("grad_sparse", &grad_sparse);
  m.def("grad_ell", &grad_ell);
  m.def("encode_messages", &encode_messages);
  m.def("combine_update", &combine_update);
  m.def("eval_gemm_loss", &eval_gemm_loss);
  m.attr("MAX_MSGS") = eh::kMaxMsgs;

  namespace py = pybind11;
  py::class_<eh::Arrival>(m, "Arrival")
      .def_readonly("worker", &eh::Arrival::worker)
      .def_readonly("part", &eh::Arrival::part)
      .def_readonly("round", &eh::Arrival::round)
      .def_readonly("t_rel", &eh::Arrival::t_rel)
      .def_readonly("probe", &eh::Arrival::probe)
      .def("__repr__", [](const eh::Arrival& a) {
        return "Arrival(worker=" + std::to_string(a.worker) + ", part=" + std::to_string(a.part) +
               ", round=" + std::to_string(a.round) + ", t_rel=" + std::to_string(a.t_rel) + ")";
      });
  py::class_<eh::Collector>(m, "Collector")
      .def(py::init<int, std::vector<int>, int>(), py::arg("n_workers"), py::arg("group_of"), py::arg("n_groups"))
      .def_static("now", &eh::Collector::now)
      .def("begin_round", &eh::Collector::begin_round)
      .def("add_event_probe", &eh::Collector::add_event_probe)
      .def("add_host_probe", &eh::Collector::add_host_probe)
      .def("add_flag_probe", &eh::Collector::add_flag_probe)
      .def("mark_seen", &eh::Collector::mark_seen)
      .def("step", &eh::Collector::step, py::call_guard<py::gil_scoped_release>())
      .def("wait", &eh::Collector::wait, py::call_guard<py::gil_scoped_release>())
      .def("drain", &eh::Collector::drain, py::call_guard<py::gil_scoped_release>())
      .def("wait_seen", &eh::Collector::wait_seen, py::call_guard<py::gil_scoped_release>())
      .def("arrivals", &eh::Collector::arrivals)
      .def("late_arrivals", &eh::Collector::late_arrivals)
      .def("pending", &eh::Collector::pending)
      .def("pending_upto", &eh::Collector::pending_upto)
      .def("stopped", &eh::Collector::stopped);
}
