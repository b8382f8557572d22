"""Build the HIP library ``libpipnet_amd.so`` in-tree for gfx950 (hipcc, no JIT cache).

The .so is git-ignored but travels to the GPU box with the repo snapshot.  ``build()``
is idempotent: it recompiles only when a source or header is newer than the library.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "libpipnet_amd.so")
ARCH = os.environ.get("PIPNET_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def _deps():
    return sources() + glob.glob(os.path.join(CSRC, "*.hpp")) + glob.glob(os.path.join(REPO, "include", "*.h"))


def is_stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    return any(os.path.getmtime(p) > t for p in _deps())


def _wait(pr) -> None:
    proc, src = pr
    if proc.wait() != 0:
        raise subprocess.CalledProcessError(proc.returncode, f"hipcc {src}")


def build(force: bool = False, verbose: bool = False) -> str:
    """Compile if stale.  Concurrent callers (one process per GPU under torchrun) serialise on
    a file lock and re-check staleness, so only the first one compiles."""
    if not force and not is_stale():
        return LIB
    import fcntl
    with open(os.path.join(PKG, ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            if not force and not is_stale():
                return LIB
            return _build_locked(verbose)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)


def _build_locked(verbose: bool) -> str:
    objs, procs = [], []
    jobs = max(1, min(int(os.environ.get("MAX_JOBS", "8")), 16))
    for src in sources():          # one hipcc per translation unit, at most `jobs` at once
        obj = os.path.join(CSRC, os.path.basename(src)[:-4] + ".o")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
               "-I", os.path.join(REPO, "include")]
        if verbose:
            print(" ".join(cmd), flush=True)
        if len(procs) >= jobs:
            _wait(procs.pop(0))
        procs.append((subprocess.Popen(cmd), src))
        objs.append(obj)
    for pr in procs:
        _wait(pr)
    tmp = LIB + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
