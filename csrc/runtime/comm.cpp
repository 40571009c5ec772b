// RcclComm / LoopbackComm: the two implementations of eh::P2PComm (comm.h).
//
//  * RcclComm: one 2-rank RCCL communicator per direction per (master, worker) pair, created with
//    ncclCommInitRank from ids the ranks exchange over gloo (parallel/transport.py CommTransport).
//    send / recv are ncclSend / ncclRecv of bytes on the caller's stream.  The library is the one
//    torch ships (the extension links torch's librccl, so a process holds ONE RCCL).
//  * LoopbackComm: FIFO send/recv with the same stream semantics through a receiver-owned IPC
//    staging ring of `depth` slots per channel.  send #s waits (hipStreamWaitValue64) until the
//    receiver consumed #s-depth, copies into slot s % depth and release-stores ready = s
//    (put + signal kernel); recv #s waits for ready >= s, copies out and stores consumed = s.
#include "runtime/comm.h"

#include <c10/hip/HIPStream.h>
#include <pybind11/stl.h>
#include <rccl/rccl.h>
#include <torch/extension.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "kernels/launchers.h"

namespace {
namespace py = pybind11;
using at::Tensor;

void hcheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void ncheck(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}
void need(bool ok, const std::string& msg) {
  if (!ok) throw std::invalid_argument(msg);
}

py::bytes nccl_unique_id() {
  ncclUniqueId id;
  ncheck(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
}

class RcclComm : public eh::P2PComm {
 public:
  // links: (peer global rank, "out" | "in", unique id bytes, my rank in that 2-rank communicator),
  // initialised in the given order (both sides list their shared links in the same order).
  RcclComm(int device, const std::vector<std::tuple<int, std::string, std::string, int>>& links) : device_(device) {
    hcheck(hipSetDevice(device), "hipSetDevice");
    for (const auto& [peer, dir, idb, me] : links) {
      need(idb.size() == sizeof(ncclUniqueId), "RcclComm: bad unique id");
      need(dir == "out" || dir == "in", "RcclComm: direction is out or in");
      need(me == 0 || me == 1, "RcclComm: 2-rank communicators");
      ncclUniqueId id;
      std::memcpy(&id, idb.data(), sizeof(id));
      ncclComm_t c = nullptr;
      {
        py::gil_scoped_release nogil;  // blocks until the peer joins
        ncheck(ncclCommInitRank(&c, 2, id, me), "ncclCommInitRank");
      }
      (dir == "out" ? out_ : in_)[peer] = Link{c, 1 - me};
    }
  }
  ~RcclComm() override {
    for (auto* m : {&out_, &in_})
      for (auto& [p, l] : *m)
        if (l.comm && !aborted_) ncclCommDestroy(l.comm);
  }
  void send(int peer, const void* buf, int64_t bytes, hipStream_t st) override {
    const Link& l = link(out_, peer, "send");
    ncheck(ncclSend(buf, static_cast<size_t>(bytes), ncclUint8, l.peer, l.comm, st), "ncclSend");
  }
  void recv(int peer, void* buf, int64_t bytes, hipStream_t st) override {
    const Link& l = link(in_, peer, "recv");
    ncheck(ncclRecv(buf, static_cast<size_t>(bytes), ncclUint8, l.peer, l.comm, st), "ncclRecv");
  }
  void abort() override {
    if (aborted_) return;
    aborted_ = true;
    for (auto* m : {&out_, &in_})
      for (auto& [p, l] : *m)
        if (l.comm) ncclCommAbort(l.comm);
  }
  std::string kind() const override { return "rccl"; }

 private:
  struct Link {
    ncclComm_t comm = nullptr;
    int peer = 0;  // the peer's rank inside the 2-rank communicator
  };
  const Link& link(const std::map<int, Link>& m, int peer, const char* what) const {
    need(!aborted_, "RcclComm: aborted");
    auto it = m.find(peer);
    if (it == m.end()) throw std::invalid_argument(std::string("RcclComm: no ") + what + " link to rank " + std::to_string(peer));
    return it->second;
  }
  int device_;
  bool aborted_ = false;
  std::map<int, Link> out_, in_;
};

class LoopbackComm : public eh::P2PComm {
 public:
  // channels: (peer, "out" | "in", staging ring device address (this process's mapping), slot bytes,
  // depth, ready flag device address, consumed flag device address, ready host address, consumed
  // host address).  The flags are 64-bit counters in host-registered shared memory.
  LoopbackComm(int device,
               const std::vector<std::tuple<int, std::string, uintptr_t, int64_t, int, uintptr_t, uintptr_t, uintptr_t,
                                            uintptr_t>>& chans)
      : device_(device) {
    counters_ = at::zeros({static_cast<int64_t>(2 * chans.size() + 2)},
                          at::TensorOptions().dtype(at::kInt).device(at::Device(at::kCUDA, device)));
    int k = 0;
    for (const auto& [peer, dir, ring, cap, depth, rdy_d, con_d, rdy_h, con_h] : chans) {
      need(dir == "out" || dir == "in", "LoopbackComm: direction is out or in");
      need(ring && rdy_d && con_d && rdy_h && con_h && cap > 0 && cap % 16 == 0 && depth >= 1, "LoopbackComm: bad channel");
      int can = 0;
      hcheck(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, device), "hipDeviceGetAttribute");
      need(can != 0, "LoopbackComm needs hipStreamWaitValue64");
      Chan c{reinterpret_cast<char*>(ring), cap, depth, reinterpret_cast<unsigned long long*>(rdy_d),
             reinterpret_cast<unsigned long long*>(con_d), reinterpret_cast<uint64_t*>(rdy_h),
             reinterpret_cast<uint64_t*>(con_h), 0,
             reinterpret_cast<unsigned int*>(counters_.data_ptr<int>()) + k++};
      (dir == "out" ? out_ : in_)[peer] = c;
    }
  }
  void send(int peer, const void* buf, int64_t bytes, hipStream_t st) override {
    Chan& c = chan(out_, peer, bytes);
    const uint64_t s = ++c.seq;
    if (s > static_cast<uint64_t>(c.depth))  // slot s % depth is free once #s-depth was consumed
      hcheck(hipStreamWaitValue64(st, c.consumed, s - c.depth, hipStreamWaitValueGte), "hipStreamWaitValue64(consumed)");
    copy_signal(buf, c.ring + static_cast<int64_t>(s % c.depth) * c.cap, bytes, c.ready, s, c.counter, st);
  }
  void recv(int peer, void* buf, int64_t bytes, hipStream_t st) override {
    Chan& c = chan(in_, peer, bytes);
    const uint64_t s = ++c.seq;
    hcheck(hipStreamWaitValue64(st, c.ready, s, hipStreamWaitValueGte), "hipStreamWaitValue64(ready)");
    copy_signal(c.ring + static_cast<int64_t>(s % c.depth) * c.cap, buf, bytes, c.consumed, s, c.counter, st);
  }
  void abort() override {  // release every queued wait of this rank's channels (data is garbage after)
    const uint64_t top = uint64_t{1} << 62;
    for (auto* m : {&out_, &in_})
      for (auto& [p, c] : *m) {
        __atomic_store_n(c.ready_h, top, __ATOMIC_RELEASE);
        __atomic_store_n(c.consumed_h, top, __ATOMIC_RELEASE);
      }
  }
  std::string kind() const override { return "loopback"; }

 private:
  struct Chan {
    char* ring;
    int64_t cap;
    int depth;
    unsigned long long* ready;
    unsigned long long* consumed;
    uint64_t* ready_h;
    uint64_t* consumed_h;
    uint64_t seq;
    unsigned int* counter;
  };
  Chan& chan(std::map<int, Chan>& m, int peer, int64_t bytes) {
    auto it = m.find(peer);
    if (it == m.end()) throw std::invalid_argument("LoopbackComm: no channel to rank " + std::to_string(peer));
    need(bytes > 0 && bytes <= it->second.cap && bytes % 16 == 0, "LoopbackComm: message larger than its slot");
    return it->second;
  }
  static void copy_signal(const void* src, void* dst, int64_t bytes, unsigned long long* flag, uint64_t v,
                          unsigned int* counter, hipStream_t st) {
    eh::PutArgs a{};
    a.n = 1;
    a.d[0] = eh::PutDesc{src, dst, bytes, flag, v, counter};
    const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(64, (bytes / 16 + 4095) / 4096)));
    hcheck(eh::put_signal_launch(a, blocks, st), "put_signal(loopback)");
  }
  int device_;
  Tensor counters_;
  std::map<int, Chan> out_, in_;
};

// RcclSelfLoop: RCCL on ONE GPU, for the one-GPU test box (RCCL refuses two ranks on one device).
// The master and its worker ranks are threads of one process (parallel/dist.py ThreadEnv), each
// with its own stream; every (sender, receiver) channel owns a 1-rank RCCL communicator and a
// staging ring of `depth` slots.  send #s waits until the receiver consumed #s-depth, moves the
// payload into slot s % depth with a GROUPED ncclSend + ncclRecv to self (RCCL's own p2p kernel does
// the copy) and release-stores ready = s; recv #s waits for ready >= s, copies the slot out and
// stores consumed = s.  So the pumps' comm mode runs RCCL calls (ncclCommInitRank, ncclSend,
// ncclRecv, ncclGroupStart/End) on the test box with the exact FIFO semantics of RcclComm.
class RcclSelfLoop {
 public:
  RcclSelfLoop(int device, int world, int depth, int64_t cap) : device_(device), world_(world), depth_(depth), cap_(cap) {
    need(world >= 2 && depth >= 1 && cap > 0 && cap % 16 == 0, "RcclSelfLoop: bad shape");
    hcheck(hipSetDevice(device), "hipSetDevice");
    int can = 0;
    hcheck(hipDeviceGetAttribute(&can, hipDeviceAttributeCanUseStreamWaitValue, device), "hipDeviceGetAttribute");
    need(can != 0, "RcclSelfLoop needs hipStreamWaitValue64");
    const int nch = 2 * (world - 1);
    hcheck(hipHostMalloc(reinterpret_cast<void**>(&flags_h_), sizeof(uint64_t) * 2 * nch,
                         hipHostMallocMapped | hipHostMallocCoherent),
           "hipHostMalloc(flags)");
    std::memset(flags_h_, 0, sizeof(uint64_t) * 2 * nch);
    hcheck(hipHostGetDevicePointer(reinterpret_cast<void**>(&flags_d_), flags_h_, 0), "hipHostGetDevicePointer");
    counters_ = at::zeros({nch}, at::TensorOptions().dtype(at::kInt).device(at::Device(at::kCUDA, device)));
    rings_ = at::zeros({static_cast<int64_t>(nch) * depth * cap}, at::TensorOptions().dtype(at::kByte).device(
                                                                     at::Device(at::kCUDA, device)));
    chans_.resize(nch);
    for (int k = 0; k < nch; ++k) {
      ncclUniqueId id;
      ncheck(ncclGetUniqueId(&id), "ncclGetUniqueId");
      Chan& c = chans_[k];
      ncheck(ncclCommInitRank(&c.comm, 1, id, 0), "ncclCommInitRank(1 rank)");
      c.ring = static_cast<char*>(rings_.data_ptr()) + static_cast<int64_t>(k) * depth * cap;
      c.ready_h = flags_h_ + 2 * k;
      c.consumed_h = flags_h_ + 2 * k + 1;
      c.ready_d = reinterpret_cast<unsigned long long*>(flags_d_ + 2 * k);
      c.consumed_d = reinterpret_cast<unsigned long long*>(flags_d_ + 2 * k + 1);
      c.counter = reinterpret_cast<unsigned int*>(counters_.data_ptr<int>()) + k;
    }
  }
  ~RcclSelfLoop() {
    hipDeviceSynchronize();
    for (auto& c : chans_)
      if (c.comm) aborted_ ? ncclCommAbort(c.comm) : ncclCommDestroy(c.comm);
    if (flags_h_) hipHostFree(flags_h_);
  }
  // from -> to, called by the sending thread on its stream
  void send(int from, int to, const void* buf, int64_t bytes, hipStream_t st) {
    Chan& c = chan(from, to, bytes);
    const uint64_t s = ++c.send_seq;
    if (s > static_cast<uint64_t>(depth_))
      hcheck(hipStreamWaitValue64(st, c.consumed_d, s - depth_, hipStreamWaitValueGte), "hipStreamWaitValue64(consumed)");
    void* slot = c.ring + static_cast<int64_t>(s % depth_) * cap_;
    ncheck(ncclGroupStart(), "ncclGroupStart");
    ncheck(ncclSend(buf, static_cast<size_t>(bytes), ncclUint8, 0, c.comm, st), "ncclSend(self)");
    ncheck(ncclRecv(slot, static_cast<size_t>(bytes), ncclUint8, 0, c.comm, st), "ncclRecv(self)");
    ncheck(ncclGroupEnd(), "ncclGroupEnd");
    hcheck(eh::signal_launch(c.ready_d, s, st), "signal(ready)");
    ++sends_;
  }
  // from -> to, called by the receiving thread on its stream
  void recv(int from, int to, void* buf, int64_t bytes, hipStream_t st) {
    Chan& c = chan(from, to, bytes);
    const uint64_t s = ++c.recv_seq;
    hcheck(hipStreamWaitValue64(st, c.ready_d, s, hipStreamWaitValueGte), "hipStreamWaitValue64(ready)");
    eh::PutArgs a{};
    a.n = 1;
    a.d[0] = eh::PutDesc{c.ring + static_cast<int64_t>(s % depth_) * cap_, buf, bytes, c.consumed_d, s, c.counter};
    const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(64, (bytes / 16 + 4095) / 4096)));
    hcheck(eh::put_signal_launch(a, blocks, st), "put_signal(self-loop recv)");
  }
  void abort() {  // release every queued wait (data after it is garbage)
    aborted_ = true;
    const uint64_t top = uint64_t{1} << 62;
    for (auto& c : chans_) {
      __atomic_store_n(c.ready_h, top, __ATOMIC_RELEASE);
      __atomic_store_n(c.consumed_h, top, __ATOMIC_RELEASE);
    }
  }
  int64_t rccl_sends() const { return sends_; }
  int world() const { return world_; }

 private:
  struct Chan {
    ncclComm_t comm = nullptr;
    char* ring = nullptr;
    uint64_t* ready_h = nullptr;
    uint64_t* consumed_h = nullptr;
    unsigned long long* ready_d = nullptr;
    unsigned long long* consumed_d = nullptr;
    unsigned int* counter = nullptr;
    uint64_t send_seq = 0, recv_seq = 0;
  };
  // channels: k = r - 1 for master -> worker rank r, world - 1 + r - 1 for r -> master
  Chan& chan(int from, int to, int64_t bytes) {
    need(bytes > 0 && bytes <= cap_ && bytes % 16 == 0, "RcclSelfLoop: message larger than its slot");
    need((from == 0) != (to == 0) && from >= 0 && to >= 0 && from < world_ && to < world_,
         "RcclSelfLoop: channels run between the master (0) and a worker rank");
    return from == 0 ? chans_[to - 1] : chans_[world_ - 1 + from - 1];
  }
  int device_, world_, depth_;
  int64_t cap_;
  uint64_t* flags_h_ = nullptr;
  uint64_t* flags_d_ = nullptr;
  Tensor counters_, rings_;
  std::vector<Chan> chans_;
  bool aborted_ = false;
  std::atomic<int64_t> sends_{0};
};

// One thread-rank's view of an RcclSelfLoop: send(peer) = channel (me -> peer), recv(peer) = (peer -> me).
class RcclSelfView : public eh::P2PComm {
 public:
  RcclSelfView(std::shared_ptr<RcclSelfLoop> loop, int me) : loop_(std::move(loop)), me_(me) {
    need(me >= 0 && me < loop_->world(), "RcclSelfView: rank out of range");
  }
  void send(int peer, const void* buf, int64_t bytes, hipStream_t st) override { loop_->send(me_, peer, buf, bytes, st); }
  void recv(int peer, void* buf, int64_t bytes, hipStream_t st) override { loop_->recv(peer, me_, buf, bytes, st); }
  void abort() override { loop_->abort(); }
  std::string kind() const override { return "rccl-self"; }

 private:
  std::shared_ptr<RcclSelfLoop> loop_;
  int me_;
};

hipStream_t cur_stream(const Tensor& t) { return c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

}  // namespace

namespace eh {
void bind_comm(py::module& m) {
  m.def("nccl_unique_id", &nccl_unique_id);
  py::class_<P2PComm, std::shared_ptr<P2PComm>>(m, "P2PComm")
      .def("send", [](P2PComm& c, int peer, const Tensor& t) {
        need(t.is_cuda() && t.is_contiguous(), "send: contiguous GPU tensor");
        c.send(peer, t.data_ptr(), t.numel() * t.element_size(), cur_stream(t));
      })
      .def("recv", [](P2PComm& c, int peer, const Tensor& t) {
        need(t.is_cuda() && t.is_contiguous(), "recv: contiguous GPU tensor");
        c.recv(peer, t.data_ptr(), t.numel() * t.element_size(), cur_stream(t));
      })
      .def("abort", &P2PComm::abort)
      .def_property_readonly("kind", &P2PComm::kind);
  py::class_<RcclComm, P2PComm, std::shared_ptr<RcclComm>>(m, "RcclComm")
      .def(py::init<int, const std::vector<std::tuple<int, std::string, std::string, int>>&>(), py::arg("device"),
           py::arg("links"));
  py::class_<RcclSelfLoop, std::shared_ptr<RcclSelfLoop>>(m, "RcclSelfLoop")
      .def(py::init<int, int, int, int64_t>(), py::arg("device"), py::arg("world"), py::arg("depth"), py::arg("cap"),
           py::call_guard<py::gil_scoped_release>())
      .def("view", [](std::shared_ptr<RcclSelfLoop> l, int me) { return std::make_shared<RcclSelfView>(l, me); })
      .def("abort", &RcclSelfLoop::abort)
      .def_property_readonly("rccl_sends", &RcclSelfLoop::rccl_sends);
  py::class_<RcclSelfView, P2PComm, std::shared_ptr<RcclSelfView>>(m, "RcclSelfView");
  py::class_<LoopbackComm, P2PComm, std::shared_ptr<LoopbackComm>>(m, "LoopbackComm")
      .def(py::init<int, const std::vector<std::tuple<int, std::string, uintptr_t, int64_t, int, uintptr_t, uintptr_t,
                                                      uintptr_t, uintptr_t>>&>(),
           py::arg("device"), py::arg("channels"));
}
}  // namespace eh
