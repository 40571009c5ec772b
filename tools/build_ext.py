"""In-tree build of the native extension ``erasurehead_amd/_C*.so`` for gfx950.

No hipify, no torch JIT cache: HIP kernels are compiled with ``hipcc --offload-arch=gfx950``
(device + host code in one fat object), the host-only runtime and the pybind/torch bindings
with ``g++`` against the HIP runtime headers, then everything is linked with ``hipcc -shared``.
Objects are cached under ``build/`` and rebuilt only when a source or header changed.

Provenance: a SHA-256 over every ``csrc/`` source and header plus this build script
(:func:`source_hash`) is compiled into the library as the string ``EH_SOURCE_HASH:<hex>``
and exposed as ``_C.SOURCE_HASH``.  ``erasurehead_amd._ext.native()`` reads it from the
``.so`` file BEFORE loading it and rebuilds (or, with ``build_if_missing=False``, refuses
with :class:`StaleBuildError`) when it differs from the tree, so a shipped ``.so`` can
never silently run code other than the sources next to it.  A hash mismatch forces a
full rebuild regardless of file mtimes.

Usage:  python tools/build_ext.py [--force] [-j N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import contextlib
import fcntl
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "objs")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


HASH_MARKER = b"EH_SOURCE_HASH:"


def _hash_inputs(csrc: str = CSRC):
    files = []
    for ext in ("*.hip", "*.cpp", "*.h"):
        files += glob.glob(os.path.join(csrc, "**", ext), recursive=True)
    files = sorted(files, key=lambda p: os.path.relpath(p, csrc))
    return files


def _defines():
    """Build-time defines (part of the provenance hash); none by default."""
    return []


def source_hash(csrc: str = CSRC) -> str:
    """SHA-256 over the native sources (relative path + bytes), the build script and its defines."""
    h = hashlib.sha256()
    h.update(" ".join(_defines()).encode() + b"\0")
    for p in _hash_inputs(csrc):
        if p.endswith("_selftest.cpp"):
            continue
        h.update(os.path.relpath(p, csrc).replace(os.sep, "/").encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    with open(os.path.abspath(__file__), "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def embedded_hash(so_path: str):
    """The source hash compiled into a built library (read from the file; nothing is loaded)."""
    try:
        with open(so_path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    k = data.find(HASH_MARKER)
    if k < 0:
        return None
    v = data[k + len(HASH_MARKER): k + len(HASH_MARKER) + 64]
    try:
        return v.decode("ascii")
    except UnicodeDecodeError:
        return None


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce

    inc = ce.include_paths(device_type="cuda")
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def target_path() -> str:
    return os.path.join(ROOT, "erasurehead_amd", "_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _headers():
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _stale(obj: str, src: str, headers) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src, *headers])


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


@contextlib.contextmanager
def _build_lock():
    """One build at a time per tree: ranks that all find a stale library (torchrun starts N at once)
    queue here, and the ones after the first find the objects and library already current."""
    os.makedirs(os.path.join(ROOT, "build"), exist_ok=True)
    with open(os.path.join(ROOT, "build", ".build.lock"), "w") as f:
        fcntl.flock(f, fcntl.LOCK_EX)
        try:
            yield
        finally:
            fcntl.flock(f, fcntl.LOCK_UN)


def build(force: bool = False, jobs: int = 0, verbose: bool = False) -> str:
    with _build_lock():
        return _build(force, jobs, verbose)


def _build(force: bool, jobs: int, verbose: bool) -> str:
    inc, torchlib, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    os.makedirs(BUILD, exist_ok=True)
    headers = _headers()
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{CSRC}"]
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    cpp_srcs = sorted(p for p in glob.glob(os.path.join(CSRC, "runtime", "*.cpp")) if not p.endswith("_selftest.cpp"))
    cpp_srcs.append(os.path.join(CSRC, "bindings.cpp"))
    jobs_list = []
    for s in hip_srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        cmd = [os.path.join(ROCM, "bin", "hipcc"), "-c", s, "-o", o, f"--offload-arch={ARCH}",
               "-munsafe-fp-atomics", *common, *_defines()]
        jobs_list.append((s, o, cmd))
    for s in cpp_srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        cmd = ["g++", "-c", s, "-o", o, *common, "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
               f"-I{ROCM}/include", *[f"-I{p}" for p in inc], f"-I{pyinc}",
               "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", "-w"]
        jobs_list.append((s, o, cmd))
    out = target_path()
    want = source_hash()
    if embedded_hash(out) not in (None, want) and os.path.exists(out):
        force = True  # the library was built from other sources: never trust mtimes then
    hsrc = os.path.join(BUILD, "source_hash.cpp")
    text = ('// generated by tools/build_ext.py: hash of the csrc/ tree this library was built from\n'
            f'extern "C" __attribute__((used)) const char eh_source_hash[] = "{HASH_MARKER.decode()}{want}";\n')
    if not os.path.exists(hsrc) or open(hsrc).read() != text:
        with open(hsrc, "w") as f:
            f.write(text)
    jobs_list.append((hsrc, hsrc + ".o", ["g++", "-c", hsrc, "-o", hsrc + ".o", "-O2", "-fPIC"]))
    todo = [(s, o, c) for (s, o, c) in jobs_list if force or _stale(o, s, headers)]
    n = jobs or min(len(todo), max(1, (os.cpu_count() or 4)), 8) or 1
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        futs = {ex.submit(_run, c): s for (s, o, c) in todo}
        for f in cf.as_completed(futs):
            log = f.result()
            if verbose:
                print("compiled", os.path.relpath(futs[f], ROOT), log, flush=True)
    objs = [o for (_, o, _) in jobs_list]
    if force or todo or not os.path.exists(out) or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        tmp = f"{out}.{os.getpid()}.tmp"
        link = [os.path.join(ROCM, "bin", "hipcc"), "-shared", "-fPIC", "-o", tmp, *objs,
                f"--offload-arch={ARCH}", f"-L{torchlib}", f"-Wl,-rpath,{torchlib}",
                "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip", "-lamdhip64",
                "-lrccl",  # torch's librccl (first -L): one RCCL per process (csrc/runtime/comm.cpp)
                f"-L{ROCM}/lib", f"-Wl,-rpath,{ROCM}/lib", "-lrocprofiler-sdk-roctx"]
        _run(link)
        if embedded_hash(tmp) != want:
            raise RuntimeError("build: linked library does not carry the tree's source hash")
        os.replace(tmp, out)
        if verbose:
            print("linked", os.path.relpath(out, ROOT), flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=0)
    a = ap.parse_args()
    print(build(force=a.force, jobs=a.j, verbose=True))
