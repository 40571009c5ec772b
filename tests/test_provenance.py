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
