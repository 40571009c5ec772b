"""Check a lazy-drain run (drain "lazy": no wait for stragglers, stale rounds skipped) against the
ranks' own device records -- no model of host or GPU scheduling.

Every physically late worker rank records, on its GPU clock (Trainer device_records, csrc/runtime/
engine.cpp WorkerPump::set_records), when each round's put landed (the stamp its put kernel writes just
before the flag), its spin, and the brackets around its stale-round decisions; the master records the
brackets around every beta put and its collector's probe log (each message's seen time, which for a
physically late rank IS its landing time: collector.h "Device times", and what became of it).  The
checks are implications between those stamps, exact up to the flag's visibility latency:

  * decode: the decoded set of round i is the stop rule replayed over round i's messages in landing
    order, every message that landed counted (the collector's inputs, from the probe log);
  * landing order: the collector's order of a round's messages is the order of the workers' own landing
    stamps (IPC: the same stamps, so equal order is exact);
  * skips: a rank skipped round i+1 only if beta(i+2) was out before its round-i decision ended, and ran
    it only if beta(i+2) was not out when the decision began (IPC: the put kernel decides; p2p: the
    gate kernel against the worker's own beta-landed counter);
  * spins: every round a rank ran spun its full scheduled delay (or was released by the end of the run).
"""
import numpy as np

VIS = 50e-6  # seconds: a flag becomes visible to the host poller this long after its put's stamp, at most

DECODED, LATE, STALE, SKIPPED, SHARD = 0, 1, 2, 3, 4


def stop_prefix(order, rule, k, groups):
    """Workers of ``order`` (landing order) up to and including the one that makes the stop rule hold."""
    got, cov = [], set()
    n_groups = len(set(groups))
    for w in order:
        got.append(w)
        cov.add(groups[w])
        if (rule == "all" and len(got) == len(groups)) or (rule == "count" and len(got) >= k) or \
                (rule == "frc" and (len(got) >= k or len(cov) == n_groups)):
            break
    return got


def _by_rank(records):
    return {int(x["rank"]): x for x in records if x is not None}


def check_lazy_device(arrivals, records, owner, skipped, delays, rule, k, groups, transport):
    """arrivals[i]: decoded workers of round i in arrival order; records: every rank's device_records
    (rank 0 the master); owner: worker -> rank (one worker per worker rank, none on rank 0); skipped:
    rounds each rank skipped; delays [R, W] seconds.  Returns counts of what was compared."""
    recs = _by_rank(records)
    master = recs[0]
    R, W = np.asarray(delays).shape
    rank_of = {int(w): int(o) for w, o in owner.items()}
    assert 0 not in rank_of.values(), "the device checks need a dedicated master (no worker on rank 0)"
    worker_of = {r: w for w, r in rank_of.items()}
    bp = np.asarray(master["beta_put"], dtype=np.float64)  # [R + 1][pre, post] master GPU ticks
    probes = [p for p in master["probes"] if p[3] is not None]
    out = {"rounds": 0, "order": 0, "skips": 0, "spins": 0, "inversions": 0, "tail_after_next_beta": 0}
    for i in range(R):
        mine = sorted((p for p in probes if p[2] == i and p[4] in (DECODED, LATE, STALE)), key=lambda p: p[3])
        order = [int(p[0]) for p in mine]
        dec = [int(w) for w in arrivals[i]]
        assert sorted(dec) == sorted(int(p[0]) for p in mine if p[4] == DECODED), (i, dec, mine)
        pred = stop_prefix(order, rule, k, groups)
        if sorted(pred) != sorted(dec):
            # only a flag that became visible after a later-stamped one (within VIS) may reorder the stop
            last = max(p[3] for p in mine if p[4] == DECODED)
            early_late = [p for p in mine if p[4] != DECODED and p[3] < last]
            assert early_late and all(last - p[3] <= VIS for p in early_late), (i, order, dec, mine)
            out["inversions"] += 1
        out["rounds"] += 1
        # the collector's order of the round's decoded and late messages is the workers' own landing order
        # (IPC: the stamps it read; a stale message may have been seen after its sender's next put, at the
        # host's poll time, and a rank that skipped the round has no landing stamp)
        if transport == "ipc":
            cur = [int(p[0]) for p in mine if p[4] in (DECODED, LATE)]
            land = {w: recs[rank_of[w]]["rounds"][i][0] for w in cur}
            assert all(v >= 0 for v in land.values()), (i, land)
            assert cur == sorted(cur, key=lambda w: (land[w], w)), (i, cur, land)
            out["order"] += 1
            # the lazy drain: some message of this round landed after the next beta had left
            if i + 1 < R and bp[i + 1][1] >= 0:
                for p in mine:
                    w = int(p[0])
                    lw = recs[rank_of[w]]["rounds"][i][0]
                    out["tail_after_next_beta"] += int(p[4] != DECODED and lw >= 0 and lw > bp[i + 1][1])
    for r, rec in recs.items():
        if r == 0:
            continue
        rows = np.asarray(rec["rounds"], dtype=np.float64)
        hz = float(rec["clock"][3])
        sk = set(skipped[r])
        w = worker_of[r]
        for i in range(R):
            ran = i not in sk
            if ran and delays[i][w] > 0 and np.isfinite(delays[i][w]):
                s0, s1 = rows[i][3], rows[i][4]
                assert s0 >= 0 and s1 >= s0, (r, i, rows[i])
                full = s1 - s0 >= delays[i][w] * hz - 2
                released = bp[R - 1][0] >= 0 and s1 >= bp[R - 1][0]  # the end of the run stops a spin early
                assert full or released, (r, i, s1 - s0, delays[i][w] * hz)
                if transport == "ipc":
                    assert rows[i][0] >= s1, (r, i, rows[i])  # the put landed after the spin
                out["spins"] += 1
            if transport == "ipc" and i + 2 < R and bp[i + 2][0] >= 0:
                # round i's put kernel decided round i + 1 (skipped rounds decide at once, after put_pre)
                lo = rows[i][0] if rows[i][0] >= 0 else rows[i][1]
                if (i + 1) in sk:
                    assert bp[i + 2][0] <= rows[i][2], (r, i, "skip without beta(i+2) out", bp[i + 2], rows[i])
                else:
                    assert bp[i + 2][1] > lo, (r, i, "ran although beta(i+2) was out", bp[i + 2], rows[i])
                out["skips"] += 1
            if transport != "ipc" and i + 1 <= R and rows[i][5] >= 0 and rows[i + 1][7] >= 0:
                # p2p: round i's gate against this rank's own beta(i+1)-landed counter bump
                if i in sk:
                    assert rows[i + 1][7] <= rows[i][6], (r, i, "skip before beta(i+1) landed", rows[i], rows[i + 1])
                else:
                    assert rows[i + 1][8] > rows[i][5], (r, i, "ran although beta(i+1) had landed", rows[i], rows[i + 1])
                out["skips"] += 1
    return out
