"""Build libpntf.so for gfx950 with hipcc (one kernel per translation unit, in parallel).

    python -m pntf.build [--jobs N] [--force]

Objects go to p-ntfields_amd/build/ (git-ignored); the shared library lands next to this
file (p-ntfields_amd/pntf/libpntf.so) so it travels with the repo snapshot to the GPU box.
A stamp of the sources and flags skips the rebuild when nothing changed.
"""
import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)                      # p-ntfields_amd/
REPO = os.path.dirname(ROOT)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(PKG, "libpntf.so")

ARCH = "gfx950"
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-I" + INCLUDE,
            "-I" + CSRC, "-Wno-unused-result"]

UNITS = (
    [("field_d%d_k%d" % (d, k), "pntf_kernels.hip", ["-DPNTF_DIM=%d" % d, "-DPNTF_KIND=%d" % k])
     for d in (3, 6) for k in range(5)]
    + [("plan_d%d" % d, "pntf_kernels.hip", ["-DPNTF_DIM=%d" % d, "-DPNTF_PLAN"]) for d in (3, 6)]
    + [("residual_d%d" % d, "pntf_kernels.hip", ["-DPNTF_DIM=%d" % d, "-DPNTF_RESIDUAL"])
       for d in (3, 6)]
    + [("util", "pntf_kernels.hip", ["-DPNTF_UTIL"]), ("capi", "pntf_capi.hip", [])]
)


def hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.sep not in c or os.path.exists(c)):
            return c
    return "hipcc"


def _stamp():
    h = hashlib.sha256()
    for d in (CSRC, INCLUDE):
        for name in sorted(os.listdir(d)):
            with open(os.path.join(d, name), "rb") as fh:
                h.update(name.encode() + fh.read())
    h.update(repr((CXXFLAGS, UNITS)).encode())
    return h.hexdigest()


def _compile(unit):
    name, src, defs = unit
    obj = os.path.join(BUILD, name + ".o")
    cmd = [hipcc()] + CXXFLAGS + defs + ["-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (name, " ".join(cmd), r.stderr))
    return obj


def build(jobs=None, force=False, verbose=True):
    os.makedirs(BUILD, exist_ok=True)
    stamp_path = os.path.join(BUILD, "stamp")
    stamp = _stamp()
    if not force and os.path.exists(LIB) and os.path.exists(stamp_path):
        with open(stamp_path) as fh:
            if fh.read() == stamp:
                if verbose:
                    print("libpntf.so up to date")
                return LIB
    jobs = jobs or min(len(UNITS), max(1, min(16, os.cpu_count() or 1)))
    if verbose:
        print("building libpntf.so (%d units, %d jobs, %s)" % (len(UNITS), jobs, ARCH))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, UNITS))
    tmp = LIB + ".tmp"
    cmd = [hipcc(), "-shared", "-fPIC", "--offload-arch=" + ARCH] + objs + ["-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed:\n%s\n%s" % (" ".join(cmd), r.stderr))
    os.replace(tmp, LIB)
    with open(stamp_path, "w") as fh:
        fh.write(stamp)
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    build(a.jobs, a.force)
    sys.exit(0)
