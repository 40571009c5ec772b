// Native arrival collector (see collector.h for the reference semantics it reproduces).
#include "collector.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <limits>
#include <stdexcept>
#include <string>
#include <thread>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace eh {

static constexpr double kInf = std::numeric_limits<double>::infinity();

Collector::Collector(int n_workers, std::vector<int> group_of, int n_groups)
    : W_(n_workers), group_of_(std::move(group_of)), n_groups_(n_groups) {
  if (W_ <= 0) throw std::invalid_argument("Collector: n_workers must be > 0");
  if (static_cast<int>(group_of_.size()) != W_) group_of_.assign(W_, 0);
  for (int g : group_of_)
    if (g < 0 || g >= std::max(n_groups_, 1)) throw std::invalid_argument("Collector: bad group id");
  finish_.assign(W_, {});
  got0_.assign(W_, 0);
  got1_.assign(W_, 0);
  group_done_.assign(std::max(n_groups_, 1), 0);
  nsh_.assign(2 * W_, 1);
  got_sh_.assign(2 * W_, 0);
  seen_at_.assign(2 * W_, {});
}

void Collector::set_shards(int worker, int part, int n) {
  if (worker < 0 || worker >= W_ || part < 0 || part > 1 || n < 1)
    throw std::invalid_argument("Collector::set_shards: bad (worker, part, n)");
  nsh_[2 * worker + part] = n;
}

uint64_t Collector::tie_key(int64_t seed, int round, int worker) {
  // splitmix64 of (seed, round, worker): distinct workers get independent uniform keys, so the
  // sort below orders tied workers by a uniformly random permutation that changes every round
  uint64_t z = static_cast<uint64_t>(seed) * 0x9E3779B97F4A7C15ull ^ (static_cast<uint64_t>(round) << 32) ^
               static_cast<uint64_t>(worker);
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

double Collector::now() {
  using namespace std::chrono;
  return duration<double>(steady_clock::now().time_since_epoch()).count();
}

void Collector::begin_round(int round, double t_start, int rule, int k) {
  if (round <= round_) throw std::invalid_argument("Collector: rounds must increase");
  round_ = round;
  t_start_ = t_start;
  rule_ = rule;
  k_ = k;
  stopped_ = false;
  if (static_cast<int>(round_start_.size()) <= round) round_start_.resize(round + 1, 0.0);
  round_start_[round] = t_start;
  cur_.clear();
  late_.clear();
  std::fill(got0_.begin(), got0_.end(), 0);
  std::fill(got1_.begin(), got1_.end(), 0);
  std::fill(group_done_.begin(), group_done_.end(), 0);
  cnt0_ = cnt1_ = cnt_groups_ = 0;
  std::fill(got_sh_.begin(), got_sh_.end(), 0);
  tie_.assign(W_, 0);
  if (tie_seed_ >= 0)
    for (int w = 0; w < W_; ++w) tie_[w] = tie_key(tie_seed_, round, w);
  // the start of this round decides whether a worker still busy with the previous one skips it
  if (skip_stale_)
    for (int id : live_) maybe_skip(probes_[id]);
}

void Collector::end_run(double t) {
  if (!skip_stale_ || round_ < 0) return;
  const int r = round_ + 1;
  if (static_cast<int>(round_start_.size()) <= r) round_start_.resize(r + 1, 0.0);
  round_start_[r] = t;
  round_ = r;  // later arrivals of the last round count as stale
  stopped_ = true;
  for (int id : live_) maybe_skip(probes_[id]);
}

int Collector::add_probe(const Probe& p) {
  if (p.worker < 0 || p.worker >= W_) throw std::invalid_argument("Collector: bad worker");
  if (p.part < 0 || p.part > 1) throw std::invalid_argument("Collector: bad part");
  probes_.push_back(p);
  live_.push_back(static_cast<int>(probes_.size()) - 1);
  return static_cast<int>(probes_.size()) - 1;
}

int Collector::add_event_probe(int worker, int part, int round, uintptr_t event, double delay, bool physical,
                               uintptr_t ref_event, double ref_t) {
  Probe p{worker, part, round, reinterpret_cast<hipEvent_t>(event), nullptr, 0, false, false, false, 0.0,
          delay, kInf, physical, false, 0.0};
  p.ref_ev = reinterpret_cast<hipEvent_t>(ref_event);
  p.ref_t = ref_t;
  return add_probe(p);
}

int Collector::add_host_probe(int worker, int part, int round, double delay, bool physical) {
  return add_probe(Probe{worker, part, round, nullptr, nullptr, 0, true, false, false, 0.0, delay, kInf, physical,
                         false, 0.0});
}

int Collector::add_flag_probe(int worker, int part, int round, uintptr_t flag_addr, uint64_t value, double delay,
                              bool physical, uintptr_t stamp_addr, DeviceClock clk) {
  if (flag_addr == 0) throw std::invalid_argument("Collector: null flag");
  if (stamp_addr != 0 && !(clk.hz > 0.0)) throw std::invalid_argument("Collector: a stamp needs a device clock");
  Probe p{worker, part, round, nullptr, reinterpret_cast<const uint64_t*>(flag_addr), value, false,
          false, false, 0.0, delay, kInf, physical, false, 0.0};
  p.stamp = reinterpret_cast<const int64_t*>(stamp_addr);
  p.clk = clk;
  return add_probe(p);
}

std::vector<ProbeRecord> Collector::probe_log() const {
  std::vector<ProbeRecord> out;
  out.reserve(probes_.size());
  for (const Probe& p : probes_) {
    const double ts = p.round < static_cast<int>(round_start_.size()) ? round_start_[p.round] : 0.0;
    out.push_back({p.worker, p.part, p.round, p.seen ? p.t_seen - ts : std::numeric_limits<double>::quiet_NaN(),
                   p.outcome});
  }
  return out;
}

bool Collector::maybe_skip(Probe& p) {
  if (!skip_stale_ || p.physical || !p.seen || p.arrived || p.round >= round_) return false;
  if (p.start < round_start_[p.round + 1]) return false;  // the worker began it before the next beta
  p.skipped = p.arrived = true;
  p.outcome = kSkipped;
  ++n_skipped_;
  finish_[p.worker][p.round] = finish_of(p.worker, p.round - 1);  // never ran: the finish carries over
  return true;
}

double Collector::busy_from(int mi, int round, double t_start) const {
  // the latest earlier round in which this message was seen (rounds a worker skipped have no entry)
  const auto& sa = seen_at_[mi];
  for (int r = std::min(round, static_cast<int>(sa.size())) - 1; r >= 0; --r)
    if (sa[r] > -kInf) return std::max(t_start, sa[r]);
  return t_start;
}

double Collector::finish_of(int worker, int round) const {
  if (round < 0) return -kInf;
  const auto& f = finish_[worker];
  if (round >= static_cast<int>(f.size())) return -kInf;
  return f[round];
}

void Collector::mark_seen(int id, double t) {
  Probe& p = probes_.at(id);
  if (p.seen || p.arrived) return;
  p.seen = true;
  p.t_seen = t;
  const double ts = p.round < static_cast<int>(round_start_.size()) ? round_start_[p.round] : t;
  const int mi = 2 * p.worker + (p.part ? 1 : 0);
  const double from = busy_from(mi, p.round, ts);  // this round's work began after the previous round's
  auto& sa = seen_at_[mi];
  if (static_cast<int>(sa.size()) <= p.round) sa.resize(p.round + 1, -kInf);
  sa[p.round] = std::max(sa[p.round], t);
  auto& f = finish_[p.worker];
  if (static_cast<int>(f.size()) <= p.round) f.resize(p.round + 1, -kInf);
  if (p.physical) {  // a really late rank: seen = arrived
    p.start = ts;
    p.ready = t + p.delay;
  } else {
    p.start = std::max(ts, finish_of(p.worker, p.round - 1));
    p.ready = p.start + std::max(0.0, t - from) + p.delay;
    if (maybe_skip(p)) return;
  }
  f[p.round] = std::max(f[p.round], p.ready);
}

void Collector::poll_events(double t) {
  // Query every distinct event ONCE per sweep: probes that share an event (all local
  // messages behind one gradient launch) must become visible together, otherwise an
  // event completing mid-sweep would order simultaneous messages by sweep position.
  std::vector<std::pair<hipEvent_t, bool>> done;
  for (int id : live_) {
    Probe& p = probes_[id];
    if (p.seen || p.host || p.arrived) continue;
    if (p.flag) {
      const uint64_t v = __atomic_load_n(p.flag, __ATOMIC_ACQUIRE);
      if (v < p.fval) continue;
      // Lazy drain, virtual probe, counter already PAST this round when first seen: a later round's put
      // landed, so this round is over at the master either way -- and the worker rank may have skipped it
      // on the device (its gate found beta(i+1) out), i.e. it never ran.  Charging it compute time would
      // push the worker's virtual finish out for rounds that follow, so it leaves as skipped.
      if (skip_stale_ && !p.physical && v > p.fval && p.round < round_) {
        p.skipped = p.arrived = true;
        p.outcome = kSkipped;
        ++n_skipped_;
        auto& f = finish_[p.worker];
        if (static_cast<int>(f.size()) <= p.round) f.resize(p.round + 1, -kInf);
        f[p.round] = finish_of(p.worker, p.round - 1);
        continue;
      }
      // the landing stamp was written before the flag's release: after the acquire above the slot holds this
      // round's put iff the flag reads exactly its value and the slot names that value
      double ts = t;
      if (p.stamp && v == p.fval && static_cast<uint64_t>(__atomic_load_n(p.stamp, __ATOMIC_RELAXED)) == p.fval)
        ts = p.clk.to_host(static_cast<double>(__atomic_load_n(p.stamp + 1, __ATOMIC_RELAXED)));
      mark_seen(id, ts);
      continue;
    }
    int hit = -1;
    for (int k = 0; k < static_cast<int>(done.size()); ++k)
      if (done[k].first == p.ev) { hit = k; break; }
    if (hit < 0) {
      const hipError_t e = hipEventQuery(p.ev);
      if (e != hipSuccess && e != hipErrorNotReady)
        throw std::runtime_error(std::string("Collector: hipEventQuery failed: ") + hipGetErrorString(e));
      done.emplace_back(p.ev, e == hipSuccess);
      hit = static_cast<int>(done.size()) - 1;
    }
    if (!done[hit].second) continue;
    double ts = t;
    float ms = 0.f;
    if (p.ref_ev && hipEventElapsedTime(&ms, p.ref_ev, p.ev) == hipSuccess) ts = p.ref_t + 1e-3 * ms;
    mark_seen(id, ts);
  }
}

bool Collector::rule_holds() const {
  switch (rule_) {
    case kRuleAll: return cnt0_ >= W_;
    case kRuleCount: return cnt0_ >= k_;
    case kRuleFrc: return cnt0_ >= k_ || cnt_groups_ >= n_groups_;
    case kRulePartialFrc: return cnt1_ >= W_ && cnt_groups_ >= n_groups_;
    case kRulePartialCount: return cnt1_ >= W_ && cnt0_ >= k_;
    default: return true;
  }
}

bool Collector::process_ready(double t, bool /*stop_at_rule*/) {
  // Ready probes, in virtual arrival order (skipped ones leave the live list here too).
  std::vector<int> ready;
  bool gone = false;
  for (int id : live_) {
    const Probe& p = probes_[id];
    gone |= p.arrived;
    if (!p.arrived && p.seen && p.ready <= t) ready.push_back(id);
  }
  if (ready.empty()) {
    if (gone)
      live_.erase(std::remove_if(live_.begin(), live_.end(), [&](int id) { return probes_[id].arrived; }), live_.end());
    return stopped_;
  }
  std::sort(ready.begin(), ready.end(), [&](int a, int b) {
    const Probe& pa = probes_[a];
    const Probe& pb = probes_[b];
    if (pa.ready != pb.ready) return pa.ready < pb.ready;
    if (pa.round == round_ && pb.round == round_ && tie_[pa.worker] != tie_[pb.worker])
      return tie_[pa.worker] < tie_[pb.worker];  // seeded per-round tie permutation
    return a < b;
  });
  for (int id : ready) {
    Probe& p = probes_[id];
    p.arrived = true;
    const Arrival a{p.worker, p.part, p.round, p.ready - round_start_[p.round], id};
    if (p.round != round_) {  // stale message of an earlier round: drained, ignored
      ++n_stale_;
      p.outcome = kStale;
      continue;
    }
    const int mi = 2 * p.worker + (p.part ? 1 : 0);
    if (++got_sh_[mi] < nsh_[mi]) {  // more shards of this message still to come
      p.outcome = kShard;
      continue;
    }
    if (stopped_) {
      late_.push_back(a);
      p.outcome = kLate;
      continue;
    }
    p.outcome = kDecoded;
    cur_.push_back(a);
    if (p.part == 0) {
      if (!got0_[p.worker]) {
        got0_[p.worker] = 1;
        ++cnt0_;
        const int g = group_of_[p.worker];
        if (!group_done_[g]) {
          group_done_[g] = 1;
          ++cnt_groups_;
        }
      }
    } else if (!got1_[p.worker]) {
      got1_[p.worker] = 1;
      ++cnt1_;
    }
    if (rule_holds()) stopped_ = true;
  }
  live_.erase(std::remove_if(live_.begin(), live_.end(), [&](int id) { return probes_[id].arrived; }),
              live_.end());
  return stopped_;
}

bool Collector::step() {
  const double t = now();
  poll_events(t);
  return process_ready(t, true);
}

static void pause_for(double dt) {
  if (dt > 2e-4) {
    std::this_thread::sleep_for(std::chrono::duration<double>(std::min(dt - 1e-4, 1e-3)));
  } else {
#if defined(__x86_64__)
    for (int i = 0; i < 32; ++i) _mm_pause();
#endif
  }
}

bool Collector::wait(double timeout) {
  if (round_ < 0) throw std::logic_error("Collector::wait before begin_round");
  if (rule_holds()) stopped_ = true;  // e.g. k = 0
  for (;;) {
    const double t = now();
    poll_events(t);
    if (process_ready(t, true)) return true;
    if (t - t_start_ > timeout) return false;
    double next = kInf;
    for (int id : live_) {
      const Probe& p = probes_[id];
      if (p.seen && !p.arrived) next = std::min(next, p.ready);
    }
    bool unseen_event = false;
    for (int id : live_)
      if (!probes_[id].seen && !probes_[id].host && !probes_[id].arrived) { unseen_event = true; break; }
    double dt = next - t;
    if (unseen_event) dt = std::min(dt, 2e-5);  // keep polling hardware events tightly
    dt = std::min(dt, t_start_ + timeout - t);
    pause_for(std::max(dt, 0.0));
  }
}

bool Collector::drain(int round, double timeout) {
  const double t0 = now();
  for (;;) {
    const double t = now();
    poll_events(t);
    process_ready(t, true);
    bool left = false;
    double next = kInf;
    bool unseen_event = false;
    for (int id : live_) {
      const Probe& p = probes_[id];
      if (p.round > round || p.arrived) continue;
      if (p.seen && std::isinf(p.delay)) continue;  // dead worker: its message was received
      left = true;
      if (p.seen) next = std::min(next, p.ready);
      else if (!p.host) unseen_event = true;
    }
    if (!left) return true;
    if (t - t0 > timeout) return false;
    double dt = next - t;
    if (unseen_event) dt = std::min(dt, 2e-5);
    pause_for(std::max(std::min(dt, t0 + timeout - t), 0.0));
  }
}

bool Collector::wait_seen(int round, double timeout) {
  const double t0 = now();
  for (;;) {
    const double t = now();
    poll_events(t);
    process_ready(t, true);
    bool left = false;
    for (int id : live_) {
      const Probe& p = probes_[id];
      if (p.round <= round && !p.seen && !p.arrived) {
        left = true;
        break;
      }
    }
    if (!left) return true;
    if (t - t0 > timeout) return false;
    pause_for(2e-5);
  }
}

std::vector<Arrival> Collector::late_arrivals(int round) const {
  if (round != round_) return {};
  return late_;
}

int Collector::pending() const {
  int n = 0;
  for (int id : live_) n += probes_[id].arrived ? 0 : 1;
  return n;
}

int Collector::pending_upto(int round) const {
  int n = 0;
  for (int id : live_) {
    const Probe& p = probes_[id];
    if (p.round > round || p.arrived) continue;
    if (p.seen && std::isinf(p.delay)) continue;
    ++n;
  }
  return n;
}

}  // namespace eh
