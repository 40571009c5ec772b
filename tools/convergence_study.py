"""The paper's claim, measured: convergence vs wall-clock under the reference straggler model.

    python tools/convergence_study.py [--out DIR] [--rounds 100] [--serial] [--quick]

Every scheme runs the headline problem (synthetic GMM 1e6 x 1e3, fp64, W = 8 workers,
AGD, eta = 10, alpha = 1/n) for 100 rounds with add_delay = 1: the reference's
Exp(mean 0.5 s) delay per worker per round, seeded by the round index
(ref src/approximate_coding.py:198-205, src/naive.py:141-148), applied as a virtual arrival
time by the native collector (csrc/runtime/collector.h), so the master's waits are real
wall-clock waits while the GPU never sleeps.

Schemes (ref main.py:62-92): naive; cyclic-MDS s=2; FRC s=1 and s=3; AGC s=1 k=6, s=3 k=6 and
the uneven s=2 k=6 extension (groups {0,1,2},{3,4,5},{6,7}); and, with --drain lazy (no wait for
the straggler tail, stale rounds skipped), cyclic s=2, FRC s=1, AGC s=1 k=6 and the uneven AGC.

Per scheme:
  sum_timeset_s        reference `timeset` semantics: round start -> decoded + updated
                       (excludes the Waitall tail, ref src/approximate_coding.py:175 vs :182-183)
  delay_floor_s        the exact injected-delay floor of that stop rule (utils/delay.delay_floor;
                       with carried lag for the schemes without a drain)
  overhead_ms_per_round (sum_timeset - floor) / rounds: compute + communication + decode
  loop_wallclock_s     true loop time including the drained straggler tail
  iters / seconds to the COMMON target = naive's 100-round training loss + 1 %
Each scheme runs in its own process (they overlap their idle delay time on one GPU; the
~1.5 ms of compute per 0.2-1.3 s round rarely collides).  Training loss is evaluated on
every partition (fix_quirks: no off-by-one partition).  Writes convergence.jsonl and
convergence.md (with a loss-vs-seconds table).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# name -> (is_coded, coded_ver, s, k, drain): drain None = the scheme's reference behaviour (FRC / AGC
# wait for the tail, the others carry lag); "lazy" = no wait, stale rounds skipped (engine/trainer.py)
SCHEMES = {
    "naive": (0, 0, 0, 0, None),
    "cyclic_s2": (1, 0, 2, 0, None),
    "frc_s1": (1, 1, 1, 0, None),
    "frc_s3": (1, 1, 3, 0, None),
    "agc_s1_k6": (1, 3, 1, 6, None),
    "agc_s3_k6": (1, 3, 3, 6, None),
    "agc_s2_k6_uneven": (1, 3, 2, 6, None),
    "cyclic_s2_lazy": (1, 0, 2, 0, "lazy"),
    "frc_s1_lazy": (1, 1, 1, 0, "lazy"),
    "agc_s1_k6_lazy": (1, 3, 1, 6, "lazy"),
    "agc_s2_k6_uneven_lazy": (1, 3, 2, 6, "lazy"),
}


def run_one(name: str, rounds: int, n_rows: int, n_cols: int, out: str) -> None:
    import torch

    from erasurehead_amd.config import RunConfig
    from erasurehead_amd.engine import Trainer, evaluate
    from erasurehead_amd.parallel.dist import DistEnv
    from erasurehead_amd.utils.delay import delay_floor, schedule

    is_coded, ver, s, k, drain = SCHEMES[name]
    W = 8
    cfg = RunConfig(W + 1, n_rows, n_cols, "/tmp/eh_conv/", 0, "synthetic", is_coded, s, 0, ver, k, 1, "AGD",
                    num_itrs=rounds, data="synthetic", data_seed=1234, seed=0, allow_uneven_groups=True,
                    verbose=True, round_timeout=120.0, drain=drain)
    env = DistEnv(device=torch.device("cuda" if torch.cuda.is_available() else "cpu"))
    tr = Trainer(cfg, env)
    t0 = time.perf_counter()
    # progress every 10 rounds (a 100-round naive run waits ~130 s of virtual delays)
    res = tr.run(log=lambda line: print(f"[{name}] {line.strip()}", flush=True))
    wall = time.perf_counter() - t0
    sch = tr.scheme
    tr.cfg.fix_quirks = True
    ev = evaluate(tr, res, write=False)
    if drain == "lazy":  # the event model with stale-round skipping, zero compute (utils/delay.schedule)
        d = np.stack([np.random.RandomState(i).exponential(0.5, W) for i in range(rounds)])
        rule = "count" if ver == 0 else "frc"
        kk = W - s if ver == 0 else (k if ver == 3 else W)
        floor = _schedule_floor(d, rule, kk, list(sch.group_of))
    elif name == "naive":
        floor = delay_floor(W, rounds, stop_count=W)
    elif ver == 0:
        floor = delay_floor(W, rounds, stop_count=W - s, carry=True)
    else:
        kk = k if ver == 3 else W
        floor = delay_floor(W, rounds, groups=list(sch.group_of), k=kk)
    rec = {
        "scheme": name, "s": s, "k": k, "drain": tr.drain_mode, "rounds": rounds, "n_rows": n_rows, "n_cols": n_cols,
        "stale_skipped": int(tr.rank_stats.get("stale_skipped_virtual", 0) or 0),
        "sum_timeset_s": float(np.sum(res.timeset)), "delay_floor_s": float(floor),
        "overhead_ms_per_round": 1e3 * (float(np.sum(res.timeset)) - floor) / rounds,
        "loop_wallclock_s": float(np.sum(res.loop_time)), "run_wallclock_s": wall,
        "timeouts": int(res.timeouts),
        "train_loss": [float(x) for x in ev.training_loss], "test_auc": [float(x) for x in ev.auc],
        "timeset": [float(x) for x in res.timeset], "loop_time": [float(x) for x in res.loop_time],
        "used_workers_per_round": float(np.mean([(np.asarray(r) >= 0).sum() for r in res.worker_timeset])),
    }
    with open(out, "w") as f:
        f.write(json.dumps(rec) + "\n")
    print(f"[{name}] done: sum timeset {rec['sum_timeset_s']:.2f} s, floor {floor:.2f} s, "
          f"loop {rec['loop_wallclock_s']:.2f} s, final loss {rec['train_loss'][-1]:.5f}", flush=True)


def _schedule_floor(d, rule, k, groups) -> float:
    """Sum of the master's round lengths in the zero-compute lazy-drain event model (t_R)."""
    from erasurehead_amd.utils.delay import schedule_floors

    return schedule_floors(d, rule, k, groups, drain="lazy")[1]


def summarize(recs, out_dir: str) -> str:
    naive = recs["naive"]
    target = naive["train_loss"][-1] * 1.01
    rows = []
    for name, r in recs.items():
        tl = np.asarray(r["train_loss"])
        hit = np.nonzero(tl <= target)[0]
        cum_ts = np.cumsum(r["timeset"])
        cum_lp = np.cumsum(r["loop_time"])
        r["loss_target"] = target
        r["iters_to_target"] = int(hit[0]) + 1 if hit.size else None
        r["timeset_s_to_target"] = float(cum_ts[hit[0]]) if hit.size else None
        r["wallclock_s_to_target"] = float(cum_lp[hit[0]]) if hit.size else None
        rows.append(r)
    lines = ["# Convergence vs wall-clock under the reference straggler model (MI355X, one GPU)", "",
             "Rows named *_lazy run with `--drain lazy`: the master never waits for the straggler tail and a "
             "worker still busy when the next beta is out skips that round; the others keep the reference's "
             "behaviour (FRC / AGC drain every round, cyclic carries lag).  `loop wall-clock` is the real "
             "time of the rounds, drain included.", "",
             f"Headline problem {naive['n_rows']} x {naive['n_cols']} fp64, W = 8, AGD, eta = 10, add_delay = 1 "
             f"(Exp(0.5) per worker per round, seed = round), {naive['rounds']} rounds.  Common target = naive's "
             f"final training loss + 1 % = {target:.5f}.  Generated by `tools/convergence_study.py`.", "",
             "| scheme | Σtimeset s | delay floor s | overhead ms/round | loop wall-clock s | iters to target | "
             "Σtimeset s to target | wall-clock s to target | final train loss | final AUC | workers used/round |",
             "|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        f = lambda x, p=3: "—" if x is None else f"{x:.{p}f}"  # noqa: E731
        lines.append(f"| {r['scheme']} | {r['sum_timeset_s']:.2f} | {r['delay_floor_s']:.2f} | "
                     f"{r['overhead_ms_per_round']:.2f} | {r['loop_wallclock_s']:.2f} | "
                     f"{r['iters_to_target'] if r['iters_to_target'] is not None else '—'} | "
                     f"{f(r['timeset_s_to_target'], 2)} | {f(r['wallclock_s_to_target'], 2)} | "
                     f"{r['train_loss'][-1]:.5f} | {r['test_auc'][-1]:.4f} | {r['used_workers_per_round']:.2f} |")
    lines += ["", "## Training loss vs cumulative Σtimeset (seconds)", "",
              "| round | " + " | ".join(r["scheme"] for r in rows) + " |", "|---|" + "---|" * len(rows)]
    R = naive["rounds"]
    for i in sorted(set([0, 1, 2, 4, 9, 19, 29, 49, 74, R - 1])):
        if i >= R:
            continue
        cells = []
        for r in rows:
            cells.append(f"{r['train_loss'][i]:.4f} @ {np.cumsum(r['timeset'])[i]:.1f}s")
        lines.append(f"| {i + 1} | " + " | ".join(cells) + " |")
    text = "\n".join(lines) + "\n"
    with open(os.path.join(out_dir, "convergence.md"), "w") as f:
        f.write(text)
    with open(os.path.join(out_dir, "convergence.jsonl"), "w") as f:
        for r in rows:
            f.write(json.dumps(r) + "\n")
    return text


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "convergence"))
    ap.add_argument("--rounds", type=int, default=100)
    ap.add_argument("--n-rows", type=int, default=1_000_000)
    ap.add_argument("--n-cols", type=int, default=1000)
    ap.add_argument("--only", default=None, help="comma-separated scheme names")
    ap.add_argument("--serial", action="store_true")
    ap.add_argument("--naive-from", default=None, help="reuse a naive.json of an earlier run (split runs)")
    ap.add_argument("--one", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--one-out", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.one:
        run_one(a.one, a.rounds, a.n_rows, a.n_cols, a.one_out)
        return 0
    os.makedirs(a.out, exist_ok=True)
    names = a.only.split(",") if a.only else list(SCHEMES)
    if a.naive_from:
        import shutil

        shutil.copy(a.naive_from, os.path.join(a.out, "naive.json"))
        names = [n for n in names if n != "naive"]
    elif "naive" not in names:
        names = ["naive"] + names
    procs = []
    for n in names:
        cmd = [sys.executable, os.path.abspath(__file__), "--one", n, "--one-out", os.path.join(a.out, f"{n}.json"),
               "--rounds", str(a.rounds), "--n-rows", str(a.n_rows), "--n-cols", str(a.n_cols)]
        p = subprocess.Popen(cmd)
        if a.serial:
            if p.wait() != 0:
                return 1
        else:
            procs.append(p)
    bad = [p.wait() for p in procs]
    if any(bad):
        print("some scheme runs failed:", bad, file=sys.stderr)
    recs = {}
    for n in (["naive"] if a.naive_from else []) + names:
        path = os.path.join(a.out, f"{n}.json")
        if os.path.exists(path):
            with open(path) as f:
                recs[n] = json.loads(f.readline())
    if "naive" in recs:
        print(summarize(recs, a.out))
    return 1 if any(bad) else 0


if __name__ == "__main__":
    sys.exit(main())
