// IPC mailbox runtime: exported device regions, shared-host generation flags and the
// put+signal launcher (csrc/kernels/transport.hip).  SURVEY §5.8 "Alternative fast
// path: HIP IPC mailbox" — the low-latency replacement for the reference's mpi4py
// Isend/Irecv (ref src/naive.py:66-79, :97-98, :150).
//
//  * IpcRegion  — a raw hipMalloc'd buffer (never the caching allocator, so the IPC
//                 handle covers exactly this buffer) that other processes open with
//                 hipIpcOpenMemHandle (same GPU or a peer MI355X over xGMI) and view as
//                 torch tensors;
//  * ShmFlags   — an array of 64-bit flags in POSIX shared memory, registered with
//                 hipHostRegister so every GPU can release-store into it while hosts
//                 poll it with acquire loads (a flag is a monotone round counter);
//  * put_signal — one launch that copies up to 16 (src, dst) payloads and announces
//                 each with its flag (put + signal).
#include <c10/hip/HIPStream.h>
#include <fcntl.h>
#include <pybind11/stl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <torch/extension.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "kernels/launchers.h"

namespace {
namespace py = pybind11;
using at::Tensor;

void hcheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

at::ScalarType dtype_of(const std::string& s) {
  if (s == "float64") return at::kDouble;
  if (s == "float32") return at::kFloat;
  if (s == "int32") return at::kInt;
  if (s == "uint8") return at::kByte;
  throw std::invalid_argument("unsupported dtype " + s);
}

class IpcRegion : public std::enable_shared_from_this<IpcRegion> {
 public:
  // Owner: allocate on `device`.  fine_grained: coherent memory (hipDeviceMallocFinegrained)
  // for mailboxes that a peer GPU writes while this GPU may hold cached lines of them.
  IpcRegion(int64_t nbytes, int device, bool fine_grained) : bytes_(nbytes), device_(device), owner_(true) {
    if (nbytes <= 0) throw std::invalid_argument("IpcRegion: nbytes must be > 0");
    hcheck(hipSetDevice(device), "hipSetDevice");
    if (fine_grained)
      hcheck(hipExtMallocWithFlags(&ptr_, static_cast<size_t>(nbytes), hipDeviceMallocFinegrained),
             "hipExtMallocWithFlags(IpcRegion)");
    else
      hcheck(hipMalloc(&ptr_, static_cast<size_t>(nbytes)), "hipMalloc(IpcRegion)");
    hcheck(hipMemset(ptr_, 0, static_cast<size_t>(nbytes)), "hipMemset(IpcRegion)");
    hcheck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  }
  // Importer: open a handle exported by another process, mapped for `device`.
  IpcRegion(const std::string& handle, int64_t nbytes, int device) : bytes_(nbytes), device_(device), owner_(false) {
    if (handle.size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("IpcRegion: bad handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle.data(), sizeof(h));
    hcheck(hipSetDevice(device), "hipSetDevice");
    hcheck(hipIpcOpenMemHandle(&ptr_, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  }
  ~IpcRegion() { close(); }
  void close() {
    if (!ptr_) return;
    hipSetDevice(device_);
    if (owner_)
      hipFree(ptr_);
    else
      hipIpcCloseMemHandle(ptr_);
    ptr_ = nullptr;
  }
  py::bytes handle() const {
    if (!owner_) throw std::logic_error("IpcRegion: only the owner exports a handle");
    hipIpcMemHandle_t h;
    hcheck(hipIpcGetMemHandle(&h, ptr_), "hipIpcGetMemHandle");
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }
  // A tensor view [shape] of `dtype` starting `offset` bytes into the region; the view
  // keeps the region alive.
  Tensor view(const std::string& dtype, std::vector<int64_t> shape, int64_t offset) {
    if (!ptr_) throw std::logic_error("IpcRegion: closed");
    const auto st = dtype_of(dtype);
    int64_t n = 1;
    for (auto s : shape) n *= s;
    const int64_t need = offset + n * static_cast<int64_t>(c10::elementSize(st));
    if (offset < 0 || need > bytes_) throw std::out_of_range("IpcRegion::view out of range");
    auto self = shared_from_this();
    auto opts = at::TensorOptions().dtype(st).device(at::Device(at::kCUDA, device_));
    return torch::from_blob(static_cast<char*>(ptr_) + offset, shape, [self](void*) {}, opts);
  }
  uintptr_t ptr() const { return reinterpret_cast<uintptr_t>(ptr_); }
  int64_t nbytes() const { return bytes_; }

 private:
  void* ptr_ = nullptr;
  int64_t bytes_;
  int device_;
  bool owner_;
};

class ShmFlags {
 public:
  // register_gpu=false keeps the flags host-only (CPU tests of the polling logic).
  ShmFlags(const std::string& name, int64_t n, bool create, bool register_gpu = true)
      : name_(name), n_(n), owner_(create) {
    if (n <= 0) throw std::invalid_argument("ShmFlags: n must be > 0");
    bytes_ = ((static_cast<size_t>(n) * 8 + 4095) / 4096) * 4096;
    fd_ = shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd_ < 0) throw std::runtime_error("shm_open(" + name + ") failed: " + std::strerror(errno));
    if (create && ftruncate(fd_, static_cast<off_t>(bytes_)) != 0) {
      ::close(fd_);
      shm_unlink(name.c_str());
      throw std::runtime_error("ftruncate failed");
    }
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (p == MAP_FAILED) {
      ::close(fd_);
      throw std::runtime_error("mmap failed");
    }
    host_ = static_cast<unsigned long long*>(p);
    if (create) std::memset(p, 0, bytes_);
    if (register_gpu) {
      const hipError_t e = hipHostRegister(p, bytes_, hipHostRegisterMapped | hipHostRegisterPortable);
      if (e != hipSuccess) {
        munmap(p, bytes_);
        ::close(fd_);
        if (create) shm_unlink(name.c_str());
        host_ = nullptr;
        hcheck(e, "hipHostRegister(flags)");
      }
      registered_ = true;
      void* d = nullptr;
      hcheck(hipHostGetDevicePointer(&d, p, 0), "hipHostGetDevicePointer(flags)");
      dev_ = static_cast<unsigned long long*>(d);
    }
  }
  ~ShmFlags() { close(); }
  void close() {
    if (!host_) return;
    if (registered_) hipHostUnregister(host_);
    munmap(host_, bytes_);
    ::close(fd_);
    unlink();
    host_ = nullptr;
  }
  // Remove the name once every process has mapped it (the mappings stay valid), so a
  // crashed run never leaves a file behind in /dev/shm.
  void unlink() {
    if (owner_ && !unlinked_) shm_unlink(name_.c_str());
    unlinked_ = true;
  }
  void check(int64_t i) const {
    if (!host_) throw std::logic_error("ShmFlags: closed");
    if (i < 0 || i >= n_) throw std::out_of_range("ShmFlags index");
  }
  uint64_t load(int64_t i) const {
    check(i);
    return __atomic_load_n(host_ + i, __ATOMIC_ACQUIRE);
  }
  void store(int64_t i, uint64_t v) {
    check(i);
    __atomic_store_n(host_ + i, v, __ATOMIC_RELEASE);
  }
  uintptr_t host_addr(int64_t i) const {
    check(i);
    return reinterpret_cast<uintptr_t>(host_ + i);
  }
  uintptr_t dev_addr(int64_t i) const {
    check(i);
    if (!dev_) throw std::logic_error("ShmFlags: not registered with the GPU");
    return reinterpret_cast<uintptr_t>(dev_ + i);
  }
  // Spin (then back off) until flag[i] >= v; false on timeout.  GIL released by the binding.
  bool wait_ge(int64_t i, uint64_t v, double timeout) const {
    check(i);
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    for (int spin = 0;; ++spin) {
      if (__atomic_load_n(host_ + i, __ATOMIC_ACQUIRE) >= v) return true;
      if (spin < 20000) {
#if defined(__x86_64__)
        _mm_pause();
#endif
        continue;
      }
      if (std::chrono::duration<double>(clk::now() - t0).count() > timeout) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  int64_t size() const { return n_; }

 private:
  std::string name_;
  int64_t n_;
  bool owner_;
  size_t bytes_ = 0;
  int fd_ = -1;
  unsigned long long* host_ = nullptr;
  unsigned long long* dev_ = nullptr;
  bool registered_ = false;
  bool unlinked_ = false;
};

// puts: list of (src tensor, dst tensor, flag device address, flag value); one launch on
// the current stream of src's device.  counters: int32 device tensor with >= len(puts)
// zero-initialised entries, private to the calling stream.
void put_signal(const std::vector<std::tuple<Tensor, Tensor, uintptr_t, uint64_t>>& puts, const Tensor& counters,
                int64_t blocks) {
  if (puts.empty()) return;
  if (static_cast<int>(puts.size()) > eh::kMaxPuts) throw std::invalid_argument("put_signal: at most 16 puts");
  if (!counters.is_cuda() || counters.scalar_type() != at::kInt || counters.numel() < (int64_t)puts.size())
    throw std::invalid_argument("put_signal: counters must be int32 GPU [>= n]");
  eh::PutArgs a{};
  a.n = static_cast<int>(puts.size());
  int64_t maxb = 0;
  for (int k = 0; k < a.n; ++k) {
    const auto& [src, dst, flag, value] = puts[k];
    if (!src.is_cuda() || !dst.is_cuda() || !src.is_contiguous() || !dst.is_contiguous())
      throw std::invalid_argument("put_signal: src/dst must be contiguous GPU tensors");
    const int64_t nb = src.numel() * src.element_size();
    if (nb != dst.numel() * dst.element_size()) throw std::invalid_argument("put_signal: size mismatch");
    if (nb % 16 || reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 || reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16)
      throw std::invalid_argument("put_signal: payloads must be 16-byte aligned multiples of 16 bytes");
    if (flag == 0) throw std::invalid_argument("put_signal: null flag");
    a.d[k] = eh::PutDesc{src.data_ptr(), dst.data_ptr(), nb, reinterpret_cast<unsigned long long*>(flag), value,
                         reinterpret_cast<unsigned int*>(counters.data_ptr<int>()) + k};
    maxb = std::max(maxb, nb);
  }
  if (blocks <= 0) blocks = std::max<int64_t>(1, std::min<int64_t>(64, (maxb / 16 + 4095) / 4096));
  const auto& src0 = std::get<0>(puts[0]);
  hcheck(eh::put_signal_launch(a, static_cast<int>(blocks),
                               c10::hip::getCurrentHIPStream(src0.device().index()).stream()),
         "put_signal");
}

// One gated put (launchers.h PutDesc::gate, the lazy-drain stale-round gate) of src into dst with its
// signal, and the next round's gate decided from the beta counter at beta_flag (device address):
// the engine's WorkerPump builds the same descriptor; this entry point serves the kernel tests.
void put_signal_gated(const Tensor& src, const Tensor& dst, uintptr_t flag, uint64_t value, const Tensor& counters,
                      const Tensor& gate, uintptr_t beta_flag, uint64_t stale_next) {
  for (auto* t : {&src, &dst, &counters, &gate})
    if (!t->is_cuda() || !t->is_contiguous()) throw std::invalid_argument("put_signal_gated: GPU contiguous tensors");
  if (gate.scalar_type() != at::kInt || gate.numel() < 2) throw std::invalid_argument("put_signal_gated: gate int32 [2]");
  const int64_t nb = src.numel() * src.element_size();
  if (nb != dst.numel() * dst.element_size() || nb % 16 || flag == 0 || beta_flag == 0)
    throw std::invalid_argument("put_signal_gated: sizes / addresses");
  eh::PutArgs a{};
  a.n = 1;
  auto& d = a.d[0];
  d = eh::PutDesc{src.data_ptr(), dst.data_ptr(), nb, reinterpret_cast<unsigned long long*>(flag), value,
                  reinterpret_cast<unsigned int*>(counters.data_ptr<int>())};
  d.gate = gate.data_ptr<int>();
  d.next_gate = gate.data_ptr<int>() + 1;
  d.beta_flag = reinterpret_cast<const unsigned long long*>(beta_flag);
  d.stale_next = stale_next;
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(64, (nb / 16 + 4095) / 4096)));
  hcheck(eh::put_signal_launch(a, blocks, c10::hip::getCurrentHIPStream(src.device().index()).stream()),
         "put_signal_gated");
}

// One tagged put (csrc/kernels/integrity.h) of src [rows, ld] into dst, with one MsgTag per row into
// `tags` (uint8 [rows * 16], on any device the GPU can write); csum: int64 zeroed scratch [>= rows].
// The engine's pumps build the same descriptors natively; this entry point serves the kernel tests.
void put_signal_tagged(const Tensor& src, const Tensor& dst, const Tensor& tags, uintptr_t flag, uint64_t value,
                       int64_t rank, const Tensor& counters, const Tensor& csum, bool corrupt) {
  for (auto* t : {&src, &dst, &tags, &counters, &csum})
    if (!t->is_cuda() || !t->is_contiguous()) throw std::invalid_argument("put_signal_tagged: GPU contiguous tensors");
  if (src.dim() != 2 || dst.sizes() != src.sizes() || src.scalar_type() != dst.scalar_type())
    throw std::invalid_argument("put_signal_tagged: src/dst must be [rows, ld] of one dtype");
  const int64_t rows = src.size(0), es = src.element_size();
  if ((es != 4 && es != 8) || (src.size(1) * es) % 16 || rows < 1 || rows > eh::kMaxTagRows)
    throw std::invalid_argument("put_signal_tagged: rows of fp32/fp64, 16-byte multiples, 1..64 rows");
  if (tags.numel() * tags.element_size() < rows * 16 || csum.scalar_type() != at::kLong || csum.numel() < rows)
    throw std::invalid_argument("put_signal_tagged: tags [rows*16 bytes], csum int64 [rows]");
  if (flag == 0) throw std::invalid_argument("put_signal_tagged: null flag");
  eh::PutArgs a{};
  a.n = 1;
  auto& d = a.d[0];
  d = eh::PutDesc{src.data_ptr(), dst.data_ptr(), src.numel() * es, reinterpret_cast<unsigned long long*>(flag), value,
                  reinterpret_cast<unsigned int*>(counters.data_ptr<int>())};
  d.tag = static_cast<eh::MsgTag*>(tags.data_ptr());
  d.csum = reinterpret_cast<unsigned long long*>(csum.data_ptr<int64_t>());
  d.rows = static_cast<int>(rows);
  d.es = static_cast<int>(es);
  d.rank = static_cast<unsigned int>(rank);
  d.corrupt = corrupt ? 1 : 0;
  const int64_t nb = src.numel() * es;
  const int blocks = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(64, (nb / 16 + 4095) / 4096)));
  hcheck(eh::put_signal_launch(a, blocks, c10::hip::getCurrentHIPStream(src.device().index()).stream()),
         "put_signal_tagged");
}

// Check the rows [n, ld] of one put against tags (uint8 [n * 16]) for counter value round1 and sender
// `rank`; returns the first failure as a dict (empty when every row matches).  Synchronises.
py::dict verify_rows(const Tensor& rows, const Tensor& tags, int64_t round1, int64_t rank) {
  if (!rows.is_cuda() || !tags.is_cuda() || rows.dim() != 2) throw std::invalid_argument("verify_rows: GPU [n, ld]");
  void* h = nullptr;
  void* dptr = nullptr;
  hcheck(hipHostMalloc(&h, sizeof(eh::IntegrityErr), hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc");
  std::memset(h, 0, sizeof(eh::IntegrityErr));
  hcheck(hipHostGetDevicePointer(&dptr, h, 0), "hipHostGetDevicePointer");
  const hipStream_t st = c10::hip::getCurrentHIPStream(rows.device().index()).stream();
  hipError_t e = eh::verify_rows_launch(rows.data_ptr(), static_cast<const eh::MsgTag*>(tags.data_ptr()),
                                        static_cast<int>(rows.size(0)), static_cast<int>(rows.size(1)),
                                        static_cast<int>(rows.element_size()), static_cast<unsigned int>(round1),
                                        static_cast<unsigned int>(rank), static_cast<eh::IntegrityErr*>(dptr), 0, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  const eh::IntegrityErr r = *static_cast<eh::IntegrityErr*>(h);
  hipHostFree(h);
  hcheck(e, "verify_rows");
  py::dict out;
  if (r.flag) {
    out["round"] = r.round;
    out["round1_got"] = r.round1_got;
    out["rank_got"] = r.rank_got;
    out["sum_got"] = r.sum_got;
    out["sum_calc"] = r.sum_calc;
  }
  return out;
}

void signal(uintptr_t flag, uint64_t value, int64_t device) {
  if (flag == 0) throw std::invalid_argument("signal: null flag");
  hcheck(eh::signal_launch(reinterpret_cast<unsigned long long*>(flag), value,
                           c10::hip::getCurrentHIPStream(device).stream()),
         "signal");
}

// Topology probes for the IPC handshake: which local device index a PCI bus id maps to (ranks
// may see different HIP_VISIBLE_DEVICES sets) and whether one device can map the other's memory.
std::string pci_bus_id(int device) {
  char buf[64] = {0};
  hcheck(hipDeviceGetPCIBusId(buf, sizeof(buf), device), "hipDeviceGetPCIBusId");
  return std::string(buf);
}
int device_by_pci(const std::string& bus) {
  int dev = -1;
  if (hipDeviceGetByPCIBusId(&dev, bus.c_str()) != hipSuccess) return -1;
  return dev;
}
bool can_access_peer(int device, int peer) {
  if (device == peer) return true;
  int ok = 0;
  hcheck(hipDeviceCanAccessPeer(&ok, device, peer), "hipDeviceCanAccessPeer");
  return ok != 0;
}

}  // namespace

namespace eh {
void bind_ipc(py::module& m) {
  py::class_<IpcRegion, std::shared_ptr<IpcRegion>>(m, "IpcRegion")
      .def(py::init<int64_t, int, bool>(), py::arg("nbytes"), py::arg("device"), py::arg("fine_grained") = false)
      .def(py::init<const std::string&, int64_t, int>(), py::arg("handle"), py::arg("nbytes"), py::arg("device"))
      .def("handle", &IpcRegion::handle)
      .def("view", &IpcRegion::view, py::arg("dtype"), py::arg("shape"), py::arg("offset") = 0)
      .def("close", &IpcRegion::close)
      .def_property_readonly("ptr", &IpcRegion::ptr)
      .def_property_readonly("nbytes", &IpcRegion::nbytes);
  py::class_<ShmFlags, std::shared_ptr<ShmFlags>>(m, "ShmFlags")
      .def(py::init<const std::string&, int64_t, bool, bool>(), py::arg("name"), py::arg("n"), py::arg("create"),
           py::arg("register_gpu") = true)
      .def("load", &ShmFlags::load)
      .def("store", &ShmFlags::store)
      .def("host_addr", &ShmFlags::host_addr)
      .def("dev_addr", &ShmFlags::dev_addr)
      .def("wait_ge", &ShmFlags::wait_ge, py::call_guard<py::gil_scoped_release>())
      .def("close", &ShmFlags::close)
      .def("unlink", &ShmFlags::unlink)
      .def_property_readonly("size", &ShmFlags::size);
  m.def("put_signal", &put_signal, py::arg("puts"), py::arg("counters"), py::arg("blocks") = 0);
  // Preflight ping-pong (transport.hip ping_pong): blocks until this side's kernel ends.
  m.def(
      "ping_pong",
      [](uintptr_t out_row, uintptr_t in_row, int64_t nwords_out, int64_t nwords_in, uintptr_t out_flag,
         uintptr_t in_flag, int64_t iters, double deadline_s, bool master, int64_t device) {
        hcheck(hipSetDevice(static_cast<int>(device)), "hipSetDevice");
        const auto dev = at::Device(at::kCUDA, static_cast<c10::DeviceIndex>(device));
        Tensor rtt = at::zeros({std::max<int64_t>(1, iters)}, at::TensorOptions().dtype(at::kLong).device(dev));
        Tensor status = at::zeros({2}, at::TensorOptions().dtype(at::kInt).device(dev));
        int khz = 0;
        hcheck(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, static_cast<int>(device)), "wall clock rate");
        eh::PingArgs a{};
        a.out_row = reinterpret_cast<unsigned long long*>(out_row);
        a.in_row = reinterpret_cast<const unsigned long long*>(in_row);
        a.nwords_out = static_cast<int>(nwords_out);
        a.nwords_in = static_cast<int>(nwords_in);
        a.out_flag = reinterpret_cast<unsigned long long*>(out_flag);
        a.in_flag = reinterpret_cast<const unsigned long long*>(in_flag);
        a.iters = static_cast<int>(iters);
        a.deadline_ticks = static_cast<long long>(deadline_s * 1e3 * khz);
        a.rtt = master ? reinterpret_cast<long long*>(rtt.data_ptr<int64_t>()) : nullptr;
        a.status = status.data_ptr<int>();
        const hipStream_t st = c10::hip::getCurrentHIPStream(static_cast<c10::DeviceIndex>(device)).stream();
        {
          py::gil_scoped_release nogil;
          hcheck(eh::ping_pong_launch(a, master, st), "ping_pong");
          hcheck(hipStreamSynchronize(st), "ping_pong sync");
        }
        const Tensor st_h = status.cpu();
        py::dict out;
        out["payload_errors"] = st_h[0].item<int>();
        out["timeout"] = st_h[1].item<int>() != 0;
        if (master) out["rtt_us"] = (rtt.to(at::kDouble) * (1e3 / khz)).cpu();
        return out;
      },
      py::arg("out_row"), py::arg("in_row"), py::arg("nwords_out"), py::arg("nwords_in"), py::arg("out_flag"),
      py::arg("in_flag"), py::arg("iters"), py::arg("deadline_s"), py::arg("master"), py::arg("device"));
  m.def("signal", &signal, py::arg("flag"), py::arg("value"), py::arg("device"));
  m.def("put_signal_gated", &put_signal_gated, py::arg("src"), py::arg("dst"), py::arg("flag"), py::arg("value"),
        py::arg("counters"), py::arg("gate"), py::arg("beta_flag"), py::arg("stale_next"));
  m.def("put_signal_tagged", &put_signal_tagged, py::arg("src"), py::arg("dst"), py::arg("tags"), py::arg("flag"),
        py::arg("value"), py::arg("rank"), py::arg("counters"), py::arg("csum"), py::arg("corrupt") = false);
  m.def("verify_rows", &verify_rows, py::arg("rows"), py::arg("tags"), py::arg("round1"), py::arg("rank"));
  m.def("pci_bus_id", &pci_bus_id, py::arg("device"));
  m.def("device_by_pci", &device_by_pci, py::arg("bus_id"));
  m.def("can_access_peer", &can_access_peer, py::arg("device"), py::arg("peer"));
}
}  // namespace eh
