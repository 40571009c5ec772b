"""Build provenance: the native library carries the hash of the csrc/ tree it was built from,
and the loader refuses (or rebuilds) a library that does not match the sources next to it."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_built_library_matches_tree(native):
    from erasurehead_amd._ext import provenance

    p = provenance()
    assert p["fresh"], p
    assert native.SOURCE_HASH == p["tree"]


def test_kernel_comment_edit_makes_build_stale(tmp_path):
    csrc = tmp_path / "csrc"
    shutil.copytree(os.path.join(ROOT, "csrc"), csrc)
    env = dict(os.environ, ERASUREHEAD_CSRC_DIR=str(csrc))
    probe = ("from erasurehead_amd._ext import native, StaleBuildError\n"
             "try:\n    native(build_if_missing=False)\nexcept StaleBuildError as e:\n    print('STALE', e)\n"
             "else:\n    print('FRESH')\n")
    out = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.stdout.startswith("FRESH"), out.stdout + out.stderr  # an identical copy hashes the same
    k = csrc / "kernels" / "update.hip"
    k.write_text(k.read_text() + "\n// a comment edit changes the tree hash\n")
    out = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert out.stdout.startswith("STALE"), out.stdout + out.stderr
    assert "stale native build" in out.stdout


def _hold_build_lock(q, hold_s):
    import time
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import build_ext  # type: ignore

    with build_ext._build_lock():
        t0 = time.monotonic()
        time.sleep(hold_s)
        q.put((t0, time.monotonic()))


def test_build_lock_serializes_processes():
    """torchrun starts every rank at once: ranks that find a stale library must build one at a time
    (the later ones then find the objects and the library current) instead of racing on build/."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_hold_build_lock, args=(q, 0.4)) for _ in range(3)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    spans = sorted(q.get(timeout=5) for _ in ps)
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert b0 >= a1, f"overlapping build-lock holders: {spans}"


def test_baseline_md_mi355x_section_is_generated():
    """Round-5 verdict item 7: every MI355X number in BASELINE.md comes from a measurement file --
    the section is tools/baseline_md.py's rendering of the driver's newest BENCH_r*.json and the
    newest profiles/round*/ records, verbatim (regenerate with `python tools/baseline_md.py --write`)."""
    import importlib.util
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("baseline_md", os.path.join(root, "tools", "baseline_md.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with open(os.path.join(root, "BASELINE.md")) as f:
        text = f.read()
    assert mod.render() in text
    assert text.count("## MI355X measurements") == 1
