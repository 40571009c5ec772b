"""One parametrised A/B runner: an environment matrix x bench.py arguments -> one JSON line per run.

Replaces the one-off gpu_*_ab.sh / sweep_*.sh scripts of earlier rounds.  Every run is a child
`python bench.py ...` under its own time limit (a run that fails or times out is recorded, and the
runner stops: nothing more is started on the GPU after a failure).  Progress goes to stderr as
each run ends, so a long matrix keeps the remote runner's liveness check fed.

    python tools/ab.py --out gpurun_out/x/ab.jsonl [--reps 2] [--timeout 600] \\
        --run 'label | ENV=a ENV2=b | --gpus 8 --steps 20 --no-floor' \\
        --run 'other | | --gpus 8 --steps 20 --no-floor --shard message'

A run spec is 'label | environment assignments | bench.py arguments'.  Each output line holds the
label, the environment, the arguments, the repetition, the wall time and the bench JSON (or the
error tail).  `--summary` prints label -> ms_per_step (median over repetitions) at the end;
`python tools/ab.py --table FILE` prints the per-label medians of a finished jsonl.
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse_run(spec: str):
    parts = [p.strip() for p in spec.split("|")]
    if len(parts) != 3:
        raise ValueError(f"run spec needs 'label | env | args': {spec!r}")
    label, env_s, args_s = parts
    env = {}
    for tok in shlex.split(env_s):
        k, _, v = tok.partition("=")
        env[k] = v
    return label, env, shlex.split(args_s)


def run_one(label, env, args, rep, timeout):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *args]
    full_env = dict(os.environ, **env)
    full_env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    t0 = time.time()
    try:
        r = subprocess.run(cmd, env=full_env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
        rc, out, err = r.returncode, r.stdout, r.stderr
    except subprocess.TimeoutExpired as e:
        rc, out, err = 124, (e.stdout or b"").decode() if isinstance(e.stdout, bytes) else (e.stdout or ""), "timeout"
    rec = {"label": label, "env": env, "args": args, "rep": rep, "rc": rc, "wall_s": round(time.time() - t0, 1)}
    line = next((ln for ln in reversed(out.strip().splitlines()) if ln.startswith("{")), None)
    if rc == 0 and line:
        rec["bench"] = json.loads(line)
    else:
        rec["error_tail"] = (out[-1500:] + "\n" + err[-3000:]).strip()
    return rec


def table(path: str) -> None:
    """Per label of an ab.py jsonl: medians of ms/step, of the per-round phase ticks and of rank 0's
    arbiter / pump microseconds (was tools/ab_table.py)."""
    from collections import defaultdict

    rows = defaultdict(lambda: defaultdict(list))
    for line in open(path):
        r = json.loads(line)
        b = r.get("bench")
        if not b:
            continue
        d = rows[r["label"]]
        d["ms"].append(b["ms_per_step"])
        for k, v in (b.get("phases_us") or {}).items():
            d[k].append(v)
        r0 = (b.get("ranks") or [{}])[0]
        for k in ("arbiter_poll_us", "arbiter_update_us", "release_us", "decode_update_us", "put_beta_us"):
            if k in r0:
                d["r0." + k].append(r0[k])
    for label, d in rows.items():
        print(label.ljust(22), "  ".join(f"{k}={statistics.median(v):.4g}" for k, v in d.items()))


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else list(argv)
    if argv[:1] == ["--table"]:  # python tools/ab.py --table FILE
        table(argv[1])
        return 0
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--out", required=True)
    ap.add_argument("--run", action="append", default=[], help="'label | ENV=v ... | bench args'")
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--timeout", type=float, default=600)
    ap.add_argument("--interleave", action="store_true", help="rep-major order (A B A B) instead of A A B B")
    ap.add_argument("--summary", action="store_true")
    a = ap.parse_args(argv)
    runs = [parse_run(s) for s in a.run]
    order = ([(r, k) for k in range(a.reps) for r in runs] if a.interleave
             else [(r, k) for r in runs for k in range(a.reps)])
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    results = {}
    ok = True
    with open(a.out, "a") as f:
        for (label, env, args), k in order:
            rec = run_one(label, env, args, k, a.timeout)
            f.write(json.dumps(rec) + "\n")
            f.flush()
            ms = rec.get("bench", {}).get("ms_per_step")
            print(f"[ab] {label} rep {k}: rc {rec['rc']} ms/step {ms} ({rec['wall_s']} s)", file=sys.stderr, flush=True)
            if rec["rc"] != 0:
                print(rec.get("error_tail", "")[-2000:], file=sys.stderr, flush=True)
                ok = False
                break  # after a failure nothing more is started
            results.setdefault(label, []).append(ms)
    if a.summary:
        for label, v in results.items():
            print(json.dumps({"label": label, "ms_per_step_median": statistics.median(v), "n": len(v)}))
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
