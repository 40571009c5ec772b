// Host-only self test of the arrival collector, built under AddressSanitizer +
// UndefinedBehaviorSanitizer by tools/sanitize_host.sh (GPU sanitizers are not available
// on the MI355X pool; the collector's state machine is pure host code and is checked here).
// Only host probes are used, so no HIP call is ever made.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <set>
#include <stdexcept>
#include <vector>

#include "collector.h"

#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                     \
    }                                                                   \
  } while (0)

using eh::Collector;

static std::set<int> workers_of(const std::vector<eh::Arrival>& a, int part = 0) {
  std::set<int> s;
  for (const auto& x : a)
    if (x.part == part) s.insert(x.worker);
  return s;
}

int main() {
  const double inf = std::numeric_limits<double>::infinity();
  // 1. AGC / FRC stop rule: W = 6 in 3 groups of 2, k = 3, virtual delays order the arrivals.
  {
    Collector c(6, {0, 0, 1, 1, 2, 2}, 3);
    const double delays[6] = {0.004, 0.001, 0.006, 0.002, 0.008, 0.003};
    for (int round = 0; round < 20; ++round) {
      const double t0 = Collector::now();
      c.begin_round(round, t0, eh::kRuleFrc, 3);
      for (int w = 0; w < 6; ++w) c.mark_seen(c.add_host_probe(w, 0, round, delays[w]), t0);
      CHECK(c.wait(5.0));
      // fastest three are workers 1, 3, 5 -> one per group -> stop after 3 arrivals
      CHECK(workers_of(c.arrivals()) == std::set<int>({1, 3, 5}));
      for (size_t i = 1; i < c.arrivals().size(); ++i) CHECK(c.arrivals()[i - 1].t_rel <= c.arrivals()[i].t_rel);
      CHECK(c.drain(round, 5.0));
      CHECK(c.pending_upto(round) == 0);
    }
  }
  // 2. Cyclic count rule with a dead worker (+inf delay): the round completes with W - s,
  //    the dead probe never arrives but does not block the drain.
  {
    Collector c(4, {0, 1, 2, 3}, 4);
    for (int round = 0; round < 5; ++round) {
      const double t0 = Collector::now();
      c.begin_round(round, t0, eh::kRuleCount, 3);
      for (int w = 0; w < 4; ++w) c.mark_seen(c.add_host_probe(w, 0, round, w == 2 ? inf : 0.0005 * w), t0);
      CHECK(c.wait(5.0));
      CHECK(workers_of(c.arrivals()) == std::set<int>({0, 1, 3}));
      CHECK(c.drain(round, 1.0));
    }
  }
  // 3. Partial rule: all first parts AND every group of second parts.
  {
    Collector c(4, {0, 0, 1, 1}, 2);
    const double t0 = Collector::now();
    c.begin_round(0, t0, eh::kRulePartialFrc, 4);
    for (int w = 0; w < 4; ++w) {
      c.mark_seen(c.add_host_probe(w, 1, 0, 0.0001), t0);
      c.mark_seen(c.add_host_probe(w, 0, 0, 0.001 * (w + 1)), t0);
    }
    CHECK(c.wait(5.0));
    CHECK(workers_of(c.arrivals(), 1).size() == 4);
    CHECK(workers_of(c.arrivals(), 0) == std::set<int>({0, 1, 2}));
    CHECK(c.drain(0, 5.0));
  }
  // 4. No drain: a straggler's lag carries into the next round (finish of round i-1 bounds
  //    the start of round i), so it is still late in round 1 without a delay of its own.
  {
    Collector c(3, {0, 1, 2}, 3);
    double t0 = Collector::now();
    c.begin_round(0, t0, eh::kRuleCount, 2);
    c.mark_seen(c.add_host_probe(0, 0, 0, 0.0), t0);
    c.mark_seen(c.add_host_probe(1, 0, 0, 0.0), t0);
    c.mark_seen(c.add_host_probe(2, 0, 0, 0.05), t0);
    CHECK(c.wait(5.0));
    CHECK(workers_of(c.arrivals()) == std::set<int>({0, 1}));
    t0 = Collector::now();
    c.begin_round(1, t0, eh::kRuleCount, 2);
    for (int w = 0; w < 3; ++w) c.mark_seen(c.add_host_probe(w, 0, 1, 0.0), t0);
    CHECK(c.wait(5.0));
    CHECK(workers_of(c.arrivals()) == std::set<int>({0, 1}));
    CHECK(c.drain(1, 5.0));
    CHECK(c.pending() == 0);
  }
  // 5. Invalid input is rejected, not undefined.
  {
    bool threw = false;
    try {
      Collector c(2, {0, 5}, 2);
    } catch (const std::invalid_argument&) {
      threw = true;
    }
    CHECK(threw);
  }
  std::printf("collector selftest ok\n");
  return 0;
}
