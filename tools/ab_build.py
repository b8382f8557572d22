"""Build an A/B variant of libpipnet_amd.so with extra compile definitions, for build-time
experiments (the product library has no runtime switches):

    python tools/ab_build.py NAME -DMACRO=VALUE [...]      -> tools/ab/libpipnet_NAME.so

Same sources and source digest as the product build (so ``_lib.load`` accepts it); load it
with ``PIPNET_AMD_LIB=tools/ab/libpipnet_NAME.so``.  Object files go to a temporary directory."""
import os
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from count_pipnet_amd import build  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    if len(sys.argv) < 2:
        raise SystemExit(__doc__)
    name, defs = sys.argv[1], sys.argv[2:]
    out = os.path.join(HERE, "ab", f"libpipnet_{name}.so")
    digest = build.source_digest()
    with tempfile.TemporaryDirectory() as tmp:
        procs, objs = [], []
        for src in build.sources():
            obj = os.path.join(tmp, os.path.basename(src)[:-4] + ".o")
            cmd = [build.HIPCC, f"--offload-arch={build.ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
                   "-I", os.path.join(build.REPO, "include"), f'-DPIPNET_SRC_DIGEST="{digest}"'] + defs
            procs.append(subprocess.Popen(cmd))
            objs.append(obj)
        for p in procs:
            if p.wait() != 0:
                raise SystemExit(f"hipcc failed ({p.args[6]})")
        subprocess.run([build.HIPCC, f"--offload-arch={build.ARCH}", "-shared", "-fPIC", "-o", out] + objs, check=True)
    print(out)


if __name__ == "__main__":
    main()
