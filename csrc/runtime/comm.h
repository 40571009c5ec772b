// Stream-ordered point-to-point messaging between the master and the worker ranks, for the
// native round executors (engine.cpp) when the IPC mailbox cannot be used (several nodes, or
// GPUs without peer access) — SURVEY §5.8 "RCCL p2p over a dedicated 2-rank communicator per
// (master, worker) pair".
//
// Reference primitives replaced: comm.Isend / Irecv / Waitany between the master and every
// worker (ref src/naive.py:66-110, src/approximate_coding.py:102-183).  Semantics here are those
// of ncclSend / ncclRecv: both calls only ENQUEUE on the given HIP stream; the stream blocks until
// the peer's matching call, messages of one direction of one pair are matched in FIFO order, and
// completion is observed with a HIP event recorded behind the receive (the master's collector
// polls those events: the native "Waitany").  One communicator per direction per pair, so a
// straggling worker never blocks another pair, and beta sends never queue behind message
// receives.
//
// Two implementations behind one interface:
//   RcclComm      ncclSend / ncclRecv on 2-rank communicators created from ncclGetUniqueId ids that
//                 the ranks exchange over the gloo control plane (RCCL from the torch build).
//   LoopbackComm  the same FIFO send/recv semantics with device-to-device copies through an IPC
//                 staging ring (put + signal kernels, hipStreamWaitValue64 on shared counters).  RCCL
//                 refuses two ranks on one GPU; this lets the single-GPU test box run the exact
//                 pump code the RCCL path runs, at 2-8 ranks.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace eh {

class P2PComm {
 public:
  virtual ~P2PComm() = default;
  // Enqueue a send of `bytes` from `buf` to `peer` (a global rank) on `st`.
  virtual void send(int peer, const void* buf, int64_t bytes, hipStream_t st) = 0;
  // Enqueue a receive of `bytes` into `buf` from `peer` on `st`.
  virtual void recv(int peer, void* buf, int64_t bytes, hipStream_t st) = 0;
  // Unblock every operation still queued (a timed-out peer); the communicator is unusable after.
  virtual void abort() = 0;
  virtual std::string kind() const = 0;
};

}  // namespace eh
