"""Build the HIP library ``libpipnet_amd.so`` in-tree for gfx950 (hipcc, no JIT cache).

The .so is git-ignored but travels to the GPU box with the repo snapshot.  ``build()``
is idempotent: it recompiles only when the sha256 of the sources (csrc/*.hip, csrc/*.hpp,
include/*.h) differs from the digest the library was built from.  The digest is compiled
into the library (``pipnet_amd_source_digest``) and ``_lib.load()`` checks it against the
tree, so a shipped binary that does not match its sources fails loudly -- file mtimes play
no part.  A sidecar ``libpipnet_amd.so.digest`` lets ``is_stale`` decide without loading.
"""
from __future__ import annotations

import glob
import hashlib
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


def source_digest() -> str:
    """sha256 over (relative path, contents) of every source the library is built from."""
    h = hashlib.sha256()
    for p in sorted(_deps()):
        h.update(os.path.relpath(p, REPO).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


DIGEST_FILE = LIB + ".digest"

# the sources that define each kernel family (namespace prefix of the rocprof kernel name):
# a PMC measurement of one family (profiles/traffic_latest.json) is stamped with their digest
KERNEL_SOURCES = {
    "pipnet_gemm::": ["gemm_f32.hip", "gemm_f32_impl.hpp", "common.hpp"],
    "pipnet_bf16::": ["conv_bf16.hip", "gemm_bf16_impl.hpp", "common.hpp"],
    "cnblock_mlp_kernel": ["mlp_f32.hip", "common.hpp"],
}


def kernel_source_digest(kernel_name: str) -> str:
    """sha256 of the sources of ``kernel_name``'s family; '' when the family is unknown."""
    files = next((v for k, v in KERNEL_SOURCES.items() if kernel_name.startswith(k)), None)
    if files is None:
        return ""
    h = hashlib.sha256()
    for f in files:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read() + b"\0")
    return h.hexdigest()


def is_stale() -> bool:
    if not os.path.exists(LIB) or not os.path.exists(DIGEST_FILE):
        return True
    with open(DIGEST_FILE) as f:
        return f.read().strip() != source_digest()


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
    digest = source_digest()
    jobs = max(1, min(int(os.environ.get("MAX_JOBS", "8")), 16))
    for src in sources():          # one hipcc per translation unit, at most `jobs` at once
        obj = os.path.join(CSRC, os.path.basename(src)[:-4] + ".o")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
               "-I", os.path.join(REPO, "include"), f'-DPIPNET_SRC_DIGEST="{digest}"']
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
    with open(DIGEST_FILE + ".tmp", "w") as f:
        f.write(digest + "\n")
    os.replace(DIGEST_FILE + ".tmp", DIGEST_FILE)
    for o in objs:
        os.remove(o)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
