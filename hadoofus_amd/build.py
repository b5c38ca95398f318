"""Build libhadoofus_crc32c.so in-tree for gfx950 (MI355X) with hipcc.

The shared library is the product: the C ABI of include/hadoofus_crc32c.h and
the drop-in symbols of include/crc32c.h.  It is built in-tree so the .so
travels with the repository snapshot to the GPU box.

A second library, libhadoofus_crc32c_diag.so, is the same sources compiled
with -DHDFS_CRC32C_DIAG: tuning shapes, read probes, the load-only twin and
result-dropping store policies (include/hadoofus_crc32c_diag.h).  Only
tools/ experiments and bench.py's ceiling measurement load it; the product
library contains none of that code and reads no tuning knob from the
environment.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
LIBDIR = os.path.join(HERE, "lib")
LIB = os.path.join(LIBDIR, "libhadoofus_crc32c.so")
DIAG_LIB = os.path.join(LIBDIR, "libhadoofus_crc32c_diag.so")
SOURCES = ["crc32c_kernels.hip", "crc32c_engine.cpp", "crc32c_packets.cpp"]
DIAG_SOURCES = SOURCES + ["crc32c_probes.hip"]
HEADERS = ["crc32c_internal.h", "crc32c_tables.h", "crc32c_packets.h", "crc32c_engine.h", "crc32c_frame.h",
           "exports.map"]
PUBLIC = ["hadoofus_crc32c.h", "crc32c.h", "hadoofus_crc32c_diag.h"]
ARCH = os.environ.get("HADOOFUS_OFFLOAD_ARCH", "gfx950")


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.isabs(c) and os.path.exists(c) or not os.path.isabs(c)):
            return c
    raise RuntimeError("hipcc not found")


def _stale(lib, sources):
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    deps = [os.path.join(CSRC, f) for f in sources + HEADERS] + [os.path.join(INCLUDE, f) for f in PUBLIC]
    return any(os.path.getmtime(d) > t for d in deps)


def _cmd(out, sources, extra):
    # -amdgpu-atomic-optimizer-strategy=None: the kernels' atomics are
    # already single-lane (ticket counters, pool claims) or pre-reduced per
    # wave; the optimizer's ballot/mbcnt scaffolding around each one cost
    # VALU in the hot loop (verify +0.6-0.9 % in a binary A/B,
    # tools/exp_ab_libs.py, profiles/r01/exp_ab_libs_atomic_optimizer.json).
    return [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
            "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
            "-Wall", "-Wno-unused-function", f"-Wl,--version-script={os.path.join(CSRC, 'exports.map')}",
            f"-I{INCLUDE}", f"-I{CSRC}"] + extra + ["-o", out] + [os.path.join(CSRC, f) for f in sources]


def build(force=False, verbose=False, diag=True):
    """Build the release library (and, with diag=True, the diagnostic one,
    in parallel).  Returns the release library's path."""
    os.makedirs(LIBDIR, exist_ok=True)
    jobs = []
    if force or _stale(LIB, SOURCES):
        jobs.append((LIB, _cmd(LIB + ".tmp", SOURCES, [])))
    if diag and (force or _stale(DIAG_LIB, DIAG_SOURCES)):
        jobs.append((DIAG_LIB, _cmd(DIAG_LIB + ".tmp", DIAG_SOURCES, ["-DHDFS_CRC32C_DIAG"])))
    procs = []
    for out, cmd in jobs:
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((out, cmd, subprocess.Popen(cmd)))
    for out, cmd, p in procs:
        if p.wait() != 0:
            raise subprocess.CalledProcessError(p.returncode, cmd)
        os.replace(out + ".tmp", out)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
