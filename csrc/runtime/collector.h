// Straggler-aware arrival collector: the native "Waitany" of the engine.
//
// Reference: the master's wait-for-the-fastest loop is an MPI Waitany over
// pre-posted Irecvs plus a per-scheme stop condition
//   naive         while cnt < W                                   ref src/naive.py:103
//   cyclic/avoid  while cnt < W - s                               ref src/coded.py:137, src/avoidstragg.py:106
//   FRC / AGC     while cnt_workers < k and cnt_groups < n_groups  ref src/approximate_coding.py:144
//   partial_*     first parts from all W AND (groups | W - s)     ref src/partial_replication.py:166,
//                                                                 src/partial_coded.py:174
// and an optional Waitall drain (ref src/approximate_coding.py:182-183).
//
// Here a "probe" is one expected message (worker, part, round).  GPU probes are HIP
// events recorded behind the RCCL receive (or behind the local gradient kernel for
// workers hosted in the master's own process); host probes are completed by the
// caller (gloo / CPU path).  The poll loop runs in C++ with the GIL released.
//
// Straggler model: the reference injects  sleep(Exp(0.5)[w])  on the worker after
// compute and before the send (ref src/naive.py:141-148).  GPUs never sleep here;
// the same deterministic delay is applied by the collector as a virtual arrival time
//     ready = max(t_start(round), finish(w, round-1)) + (t_seen - t_start(round)) + delay
// which reproduces the reference's arrival order and wall-clock (including the lag a
// straggler carries into the next round when the scheme does not drain), while the
// hardware stays busy.  delay = +inf models a dead worker (an erasure that never
// arrives; bounded by the round timeout instead of hanging like the reference).
//
// Shards: with partition sharding (engine/trainer.py) one logical message (worker, part) is
// computed as n shards on possibly different ranks (one per partition it reads) and the master
// sums them.  The message arrives when its LAST shard is ready; its arrival time is that
// shard's (the max over shards, since ready probes are processed in time order).
//
// Tie model: messages that become ready at the same instant (every local message of one
// process shares the gradient kernel's HIP event; with add_delay = 0 nothing separates
// them) are ordered by a per-round permutation of the workers seeded by (tie_seed, round)
// — the stand-in for the reference's Waitany order, which varies with real timing from
// round to round.  Ordering such ties by worker id instead would let AGC stop on the same
// k workers every round and never cover the last FRC groups' partitions.  tie_seed < 0
// restores the plain probe (worker) order.
//
// Physical probes: with physically late worker ranks (--delay-on worker) a remote message's seen
// time IS its arrival (ready = t_seen, or +inf for a dead worker): no virtual carry-over, the rank
// really was late.  Compute time of a virtual probe is the physical busy time of THIS round:
// t_seen - max(t_start, the seen time of that message in the latest earlier round it was seen), so work
// queued behind an earlier round on one stream is not counted twice when lag carries over.  The seen
// times are kept per round: shards of ONE round seen at t1 < t2 both count from the round start (not
// the second from the first).
//
// Stale-round skipping (drain "lazy", engine/trainer.py): a worker that is still busy with an
// earlier round when the round AFTER a probe's round begins skips that round, exactly like a
// physical worker whose gate finds the next beta already published (csrc/kernels/common.h
// gate_closed): the probe never arrives, the worker's finish time carries over to its next round.
// The decision for a probe of round j is taken when round j+1 begins (or when the probe is seen, if
// later): skipped iff its virtual start max(t_start(j), finish(w, j-1)) >= t_start(j+1).  An IPC flag
// probe first seen with its counter already past round j (a later round's put landed) is skipped too:
// the worker rank may have skipped round j on the device, and round j is over at the master either way.
// Both parts of a partial scheme's worker share one virtual start, so they skip together.  Over
// stream-ordered p2p (RCCL / loopback) a round the worker skipped on the device still sends its stale
// rows (FIFO pairing): they land after their round ended and are drained as stale, never decoded.  The
// event probe cannot tell them from a computed round, so with virtual delays on top of physical skipping
// the carried virtual finish of that worker can come out late; the decode is unaffected.
//
// Device times (physical probes): the seen time of a physically late rank's message is by default
// the host's poll time, so when the host thread is descheduled two messages that landed far apart
// can be seen in one sweep and ordered by the tie permutation.  With a device time source the seen
// time is WHEN THE MESSAGE LANDED on a GPU clock mapped to the host clock: an IPC flag probe reads
// the landing stamp its put kernel wrote just before the flag (launchers.h PutDesc::stamp), an event
// probe reads its timing event against a reference event.  Arrival order is then the landing order
// up to the flag's visibility latency (microseconds), whatever the host scheduler did.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace eh {

enum RuleKind : int {
  kRuleAll = 0,           // every worker's part 0
  kRuleCount = 1,         // k part-0 arrivals
  kRuleFrc = 2,           // k workers OR every group covered
  kRulePartialFrc = 3,    // all part-1 AND every group covered by part 0
  kRulePartialCount = 4,  // all part-1 AND k part-0 arrivals
};

// Device clock -> host clock (Collector::now): t = t0 + (ticks - tick0) / hz.
struct DeviceClock {
  double tick0 = 0.0, t0 = 0.0, hz = 0.0;
  double to_host(double ticks) const { return t0 + (ticks - tick0) / hz; }
};

// What became of a probe (Collector::probe_log).
enum ProbeOutcome : int { kPending = -1, kDecoded = 0, kLate = 1, kStale = 2, kSkipped = 3, kShard = 4 };

struct ProbeRecord {
  int worker, part, round;
  double t_seen;  // relative to the round's start; NaN if never seen
  int outcome;    // ProbeOutcome
};

struct Arrival {
  int worker;
  int part;
  int round;
  double t_rel;  // virtual arrival time relative to the round start
  int probe;
};

class Collector {
 public:
  Collector(int n_workers, std::vector<int> group_of, int n_groups);

  static double now();

  void begin_round(int round, double t_start, int rule, int k);
  // Seed of the per-round tie permutation (< 0: ties keep probe order); see the tie model above.
  void set_tie_seed(int64_t seed) { tie_seed_ = seed; }
  int64_t tie_seed() const { return tie_seed_; }
  // Tie rank of `worker` in `round` (smaller first); the permutation any host code can replay.
  static uint64_t tie_key(int64_t seed, int round, int worker);
  // Message (worker, part) is delivered as n >= 1 shards (probes); default 1.
  void set_shards(int worker, int part, int n);
  // physical: the probe's seen time is its arrival (see "Physical probes" above).
  // ref_event (timing-enabled, like `event`; 0 = host poll time): the event's device time relative to
  // ref_event, plus ref_t, is its seen time (see "Device times").
  int add_event_probe(int worker, int part, int round, uintptr_t event, double delay, bool physical = false,
                      uintptr_t ref_event = 0, double ref_t = 0.0);
  int add_host_probe(int worker, int part, int round, double delay, bool physical = false);
  // IPC mailbox probe: arrived once the 64-bit flag at `flag_addr` (shared host memory,
  // release-stored by the sending GPU) reaches `value` (csrc/runtime/ipc.cpp).  stamp_addr (0 = host
  // poll time): the put's {value, landing ticks} slot on the sender's clock `clk` (see "Device times");
  // used only when the flag reads exactly `value` and the slot names it (a skipped round leaves an
  // older round's slot, an end-of-run signal no slot at all: those fall back to the poll time).
  int add_flag_probe(int worker, int part, int round, uintptr_t flag_addr, uint64_t value, double delay,
                     bool physical = false, uintptr_t stamp_addr = 0, DeviceClock clk = {});
  // Every probe so far: (worker, part, round, seen time from its round's start, outcome).
  std::vector<ProbeRecord> probe_log() const;
  void mark_seen(int probe, double t);
  // Stale-round skipping of virtual probes (drain "lazy"; see above).  Off: lag carries over and
  // every round's message is delivered in order (the reference's no-Waitall schemes).
  void set_skip_stale(bool on) { skip_stale_ = on; }
  // End of the master's rounds at time t (skip_stale only): like the start of one more round, every
  // virtual probe whose worker could not start its round before t is skipped (the physical workers
  // get the same release: MasterPump::finish_run).  No round may begin after it.
  void end_run(double t);
  bool skip_stale() const { return skip_stale_; }
  // Virtual probes skipped as stale so far, and stale arrivals (a round's message after the round
  // ended: drained, never decoded).
  int skipped() const { return n_skipped_; }
  int stale_arrivals() const { return n_stale_; }

  // Process everything that is ready; returns true once the current round's stop rule holds.
  bool step();
  // Blocking poll until the stop rule holds or `timeout` seconds after the round start.
  // Returns true when the rule was satisfied, false on timeout.
  bool wait(double timeout);
  // Blocking: until every probe of rounds <= `round` has arrived (dead ones: been seen).
  bool drain(int round, double timeout);
  // Blocking: until every probe of rounds <= `round` has been SEEN (its data landed), whatever
  // its virtual arrival time — the condition for reusing that round's mailbox slot.
  bool wait_seen(int round, double timeout);

  const std::vector<Arrival>& arrivals() const { return cur_; }
  std::vector<Arrival> late_arrivals(int round) const;  // arrivals after the stop, this round
  int pending() const;
  // Live probes of rounds <= `round` that a drain would still wait for.
  int pending_upto(int round) const;
  bool stopped() const { return stopped_; }

 private:
  struct Probe {
    int worker, part, round;
    hipEvent_t ev;
    const uint64_t* flag;  // IPC flag probe (nullptr otherwise)
    uint64_t fval;
    bool host;
    bool seen;
    bool arrived;
    double t_seen;
    double delay;
    double ready;
    bool physical;
    bool skipped;
    double start;  // virtual start (seen virtual probes)
    const int64_t* stamp = nullptr;  // {flag value, device landing ticks} slot (flag probes; see "Device times")
    DeviceClock clk{};
    hipEvent_t ref_ev = nullptr;     // reference event of a device-timed event probe
    double ref_t = 0.0;
    int outcome = kPending;
  };
  int add_probe(const Probe& p);
  // Skip a seen virtual probe whose next round began before its start (skip_stale_).
  bool maybe_skip(Probe& p);
  void poll_events(double t);
  bool process_ready(double t, bool stop_at_rule);
  bool rule_holds() const;
  double finish_of(int worker, int round) const;

  int W_;
  std::vector<int> group_of_;
  int n_groups_;
  int round_ = -1;
  double t_start_ = 0.0;
  int rule_ = kRuleAll;
  int k_ = 0;
  bool stopped_ = false;
  int64_t tie_seed_ = -1;
  std::vector<uint64_t> tie_;  // [worker] tie key of the current round
  std::vector<int> nsh_;       // [2 * worker + part] shards per message
  std::vector<int> got_sh_;    // [2 * worker + part] shards of the current round ready so far
  std::vector<double> round_start_;
  std::vector<std::vector<double>> finish_;  // [worker][round] virtual finish
  // [2 * worker + part][round] latest seen time over that round's shards of the message (-inf: none yet)
  std::vector<std::vector<double>> seen_at_;
  double busy_from(int mi, int round, double t_start) const;
  bool skip_stale_ = false;
  int n_skipped_ = 0, n_stale_ = 0;
  std::vector<Probe> probes_;
  std::vector<int> live_;  // probe ids not yet arrived
  std::vector<Arrival> cur_;
  std::vector<Arrival> late_;
  // per current round counters
  std::vector<char> got0_, got1_, group_done_;
  int cnt0_ = 0, cnt1_ = 0, cnt_groups_ = 0;
};

}  // namespace eh
