"""Build libplakar_cdc.so (HIP, gfx950) in-tree and the CPU oracle (test infrastructure).

    python -m plakar_amd.build            # both
    python -m plakar_amd.build --lib-only

hipcc cross-compiles for gfx950 without a GPU, so this runs in the build
container; the built .so travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_DIR = os.path.join(HERE, "_lib")
LIB = os.path.join(LIB_DIR, "libplakar_cdc.so")
SOURCES = [os.path.join(HERE, "csrc", f) for f in ("cdc_kernels.hip", "cdc_digest.hip", "cdc_api.cpp",
                                                    "cdc_packer.cpp", "cdc_collector.cpp",
                                                    "cdc_encode.hip", "cdc_sha256.cpp", "cdc_backup.cpp")]
HEADERS = [os.path.join(HERE, "csrc", "cdc_internal.h"), os.path.join(ROOT, "include", "plakar_cdc.h")]
ARCH = os.environ.get("PLAKAR_CDC_ARCH", "gfx950")


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force=False, verbose=True, out=None, defines=()):
    """Build the library (out: another path for an experiment variant,
    defines: extra -D flags for it)."""
    target = out or LIB
    if not force and not defines and not _stale(target, SOURCES + HEADERS):
        return target
    os.makedirs(os.path.dirname(target), exist_ok=True)
    tmp = target + ".tmp"
    cmd = ["hipcc", f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(ROOT, "include"), "-Wall", "-Wno-unused-function",
           "-o", tmp] + [f"-D{d}" for d in defines] + SOURCES
    if verbose:
        print("[plakar_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, target)
    return target


def build_oracle(verbose=True):
    """Compile oracle/ (CPU checker; never linked into the product)."""
    cmd = ["make", "-s", "-C", os.path.join(ROOT, "oracle")]
    if verbose:
        print("[plakar_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return os.path.join(ROOT, "oracle", "_build", "liboracle.so")


def build_ctests(verbose=True):
    """Compile the C-level boundary test (tests/c/abi_threads.c) against the
    library and the CPU oracle (its checker) into tests/_build/."""
    out_dir = os.path.join(ROOT, "tests", "_build")
    os.makedirs(out_dir, exist_ok=True)
    exe = os.path.join(out_dir, "abi_threads")
    src = [os.path.join(ROOT, "tests", "c", "abi_threads.c"), os.path.join(ROOT, "oracle", "fastcdc_oracle.c")]
    if not _stale(exe, src + [LIB] + HEADERS):
        return exe
    cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-I", os.path.join(ROOT, "include"), "-o", exe] + src + \
          ["-L", LIB_DIR, "-lplakar_cdc", "-Wl,-rpath,$ORIGIN/../../plakar_amd/_lib", "-lpthread"]
    if verbose:
        print("[plakar_amd.build]", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return exe


if __name__ == "__main__":
    build_lib(force="--force" in sys.argv)
    if "--lib-only" not in sys.argv:
        build_oracle()
        build_ctests()
