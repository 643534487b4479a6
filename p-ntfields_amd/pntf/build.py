"""Build libpntf.so for gfx950 with hipcc (one kernel per translation unit, in parallel).

    python -m pntf.build [--jobs N] [--force]

Objects go to p-ntfields_amd/build/<unit>/ (git-ignored) with the device assembly kept
beside them; the shared library lands next to this file (p-ntfields_amd/pntf/libpntf.so) so
it travels with the repo snapshot to the GPU box.  A stamp of the sources and flags skips the
rebuild when nothing changed.

Codegen guards fail the build instead of shipping a wrong kernel:
  * no scratch use and no VGPR spills (a spilling build of the field kernel corrupted results,
    DESIGN.md §7), except a recorded number of in-register (AGPR) spills for the units of
    VGPR_SPILL_ALLOWED;
  * no SGPR spills in the headline wide units (SGPR_SPILL_FREE);
  * every saved-σ scratch load carries the nt policy (scratch_policy_violations);
  * no packed-fp32 VALU ops (v_pk_{mul,add,fma}_f32) in device code: round 1 blamed them for
    the lanes 12-15 corruption that the store-data guard below explains; the
    device is still compiled with -packed-fp32-ops, which costs nothing here;
  * no vector store of more than 8 bytes whose data VGPRs the very next instruction overwrites
    (store_data_hazards).  On gfx950 that overwrite corrupts the stored data in lanes 12-15 of
    every 16-lane row; LLVM's hazard recognizer pads the pair except for MUBUF stores with an
    SGPR soffset, so every 16-byte buffer store is followed by an s_nop that reads its data
    (pntf_field.h bstore; measured: tests/diag).
A summary of every kernel's registers and spills is written to build/report.json.
"""
import argparse
import concurrent.futures as cf
import glob
import hashlib
import json
import os
import re
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
            "-I" + CSRC, "-Wno-unused-result",
            "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops",
            "-save-temps=obj", "-Rpass-analysis=kernel-resource-usage"]
PACKED_FP32 = re.compile(r"\bv_pk_(mul|add|fma)_f32\b")
# saved-σ scratch: the stores and loads of a wave's slot go through one buffer descriptor
SCRATCH_STORE = re.compile(r"buffer_store_dwordx4 v\[\d+:\d+\], v\d+, (s\[\d+:\d+\])[^\n]*\bnt\b")
BUFFER_LOAD = re.compile(r"buffer_load_dwordx4 v\[\d+:\d+\], v\d+, (s\[\d+:\d+\])([^\n]*)")
# units whose kernels keep a saved-σ scratch slot (τ-only / travel-time kernels have none)
SCRATCH_UNITS = re.compile(r"^(field_d\d_k[123]|fsplit_d\d_k[123]|wide_d\d_k[123]|plan_d\d|plan_split_d\d|"
                           r"residual_d\d)$")


WIDE_STORE = re.compile(r"^(buffer|global|scratch|flat)_store_dwordx[34]\b")


def _vregs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def store_data_hazards(asm):
    """Store-data guard: (line, instruction) of every VALU instruction that
    writes a data VGPR of a vector store of more than 8 bytes with no wait state between them (an
    s_nop k gives k + 1).  Straight-line over the listing, so a store at the end of a block and
    the first instruction of the next are also paired (conservative)."""
    out, pend, meta = [], set(), False
    for ln, line in enumerate(asm.splitlines(), 1):
        s = line.strip()
        meta = (meta or s.startswith(".amdgpu_metadata")) and \
            not s.startswith(".end_amdgpu_metadata")
        if meta or not s or s[0] in ";." or s.endswith(":") or line[:1] not in " \t":
            continue
        parts = s.split(";")[0].replace(",", " ").split()
        op, ops = parts[0], parts[1:]
        # VALU / MFMA writers only: a load's data returns hundreds of cycles after it issues
        dst = _vregs(ops[0]) if op.startswith("v_") and ops else set()
        if dst & pend:
            out.append((ln, s))
        pend = set()
        if WIDE_STORE.match(op):      # MUBUF: vdata first; FLAT/global/scratch: vaddr, vdata
            pend = _vregs(ops[0] if op.startswith("buffer") else ops[1])
    return out


def scratch_policy_violations(asm):
    """Stale-L1 guard.  A persistent wave rewrites its scratch slot for every
    tile and its stores do not refresh the CU's vector L1, so every load through the scratch
    descriptor (the one the nt stores use) must carry the nt policy (bypass L1).  Returns
    (scratch descriptors, nt loads through them, loads through them without nt)."""
    # per kernel: a unit may hold several instantiations (wide_field_kernel<DIM, KIND, BL>),
    # whose register allocations can give the scratch and weight descriptors each other's SGPRs
    bodies = [b for b in re.split(r"(?m)^(?=_Z\w+:)", asm) if b.startswith("_Z")] or [asm]
    descs_all, good, bad = set(), 0, 0
    for body in bodies:
        descs = set(SCRATCH_STORE.findall(body))
        descs_all |= descs
        for m in BUFFER_LOAD.finditer(body):
            if m.group(1) in descs:
                if re.search(r"\bnt\b", m.group(2)):
                    good += 1
                else:
                    bad += 1
    return descs_all, good, bad

# units whose kernels must not spill SGPRs either: the headline τ+∇τ kernel and its τ-only /
# travel-time siblings, in their LDS-table instantiation (the narrow 16-pair kernels still spill
# ~24-335 SGPRs to VGPR lanes)
SGPR_SPILL_FREE = re.compile(r"^wide_d\d_k[014]$")
# VGPR spills that stay in the register file (to AGPRs, ScratchSize 0) accepted per unit, as
# measured when the unit was last changed; more than this fails the build.  None since the
# quad kernels run 8 waves with a 16-fragment ring (the 4-wave SOLO planner kept 2 beside its
# 32-fragment ring; with -DPNTF_QWAVES=4 raise these back to 2).
QRING_MFMA, QRING_SOLO = 16, 22   # quad weight-ring depths (fragments per wave)
VGPR_SPILL_ALLOWED = {"plan_quad_solo_d3": 0, "plan_quad_solo_d6": 0}

UNITS = (
    [("field_d%d_k%d" % (d, k), "pntf_kernels.hip", ["-DPNTF_DIM=%d" % d, "-DPNTF_KIND=%d" % k])
     for d in (3, 6) for k in range(5)]
    + [("fsplit_d%d_k%d" % (d, k), "pntf_kernels.hip",
        ["-DPNTF_DIM=%d" % d, "-DPNTF_KIND=%d" % k, "-DPNTF_SPLIT_FIELD"])
       for d in (3, 6) for k in range(5)]
    # wide kernels (pntf_wide.h): a 2-step ring (32-64 fp32 MFMAs of 64 cycles ahead; 24-48
    # bf16 MFMAs of 32 cycles in the split-bf16 layers, 6 fragments per step)
    # (block-major encoder layers, PNTF_X6_BM, where they stay spill-free: τ, travel time, and
    # τ+∇τ at dim 3 — the headline)
    # (round 6: the accumulate-in-bank engine, pntf_wide.h xlayer; the dim-6 units, whose
    # 12-float pair state sits beside the ring, run a 1-step ring to stay spill-free)
    + [("wide_d%d_k%d" % (d, k), "pntf_kernels.hip",
        ["-DPNTF_DIM=%d" % d, "-DPNTF_KIND=%d" % k, "-DPNTF_WIDE_FIELD",
         "-DPNTF_PF_STEPS=%d" % (2 if d == 3 else 1),
         "-DPNTF_WIDE_X6=1", "-DPNTF_RING_NL=6", "-DPNTF_X6_BM=%d" % (k in (0, 4) or (d, k) == (3, 1))])
       for d in (3, 6) for k in range(5)]
    # plan_kernel<6> holds the 6-dof path state beside the ring: a 2-step ring keeps it
    # spill-free (the 4-step ring spills 2 VGPRs there).
    + [("plan_d3", "pntf_kernels.hip", ["-DPNTF_DIM=3", "-DPNTF_PLAN"]),
       ("plan_d6", "pntf_kernels.hip", ["-DPNTF_DIM=6", "-DPNTF_PLAN", "-DPNTF_PF_STEPS=2"])]
    + [("plan_split_d%d" % d, "pntf_kernels.hip", ["-DPNTF_DIM=%d" % d, "-DPNTF_PLAN_SPLIT"])
       for d in (3, 6)]
    # quad kernels (pntf_quad.h): 4-pair tiles, σ10 in LDS (no scratch slot)
    # the ∇τ kernels run a QRING_MFMA-fragment weight ring per wave (PNTF_QRING; QRING_SOLO in
    # the SOLO units), its loads pinned in program order (PNTF_QPIN, pntf_quad.h qfetch); the
    # τ-only kernels stream the forward half with 8 (quad tiles)
    + [("quad_d%d_k%d" % (d, k), "pntf_kernels.hip",
        ["-DPNTF_DIM=%d" % d, "-DPNTF_KIND=%d" % k, "-DPNTF_QUAD_FIELD"]
        + (["-DPNTF_QRING=%d" % QRING_MFMA] if k in (1, 2, 3) else []))
       for d in (3, 6) for k in range(5)]
    + [("plan_quad_d%d" % d, "pntf_kernels.hip",
        ["-DPNTF_DIM=%d" % d, "-DPNTF_PLAN_QUAD", "-DPNTF_QSOLO=0", "-DPNTF_QRING=%d" % QRING_MFMA])
       for d in (3, 6)]
    # single-query planner (the reference's Q = 1 loop): quad layout, layers on the VALU
    + [("plan_quad_solo_d%d" % d, "pntf_kernels.hip",
        ["-DPNTF_DIM=%d" % d, "-DPNTF_PLAN_QUAD", "-DPNTF_QSOLO=1", "-DPNTF_QRING=%d" % QRING_SOLO])
       for d in (3, 6)]
    + [("residual_d%d" % d, "pntf_kernels.hip", ["-DPNTF_DIM=%d" % d, "-DPNTF_RESIDUAL"])
       for d in (3, 6)]
    + [("util", "pntf_kernels.hip", ["-DPNTF_UTIL"]), ("capi", "pntf_capi.hip", []),
       ("train", "pntf_train.hip", []), ("gemm", "pntf_gemm.hip", []),
       ("mesh", "pntf_mesh.hip", [])]
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


def unit_ids():
    """Per-unit code identity: sha256 of the shared headers, the unit's source file, its
    defines and the flags.  Baked into libpntf.so (pntf_build_info) so a PMC summary collected
    from one build can be matched to the kernel that a later run actually loads."""
    hdr = hashlib.sha256()
    for name in sorted(os.listdir(CSRC)) + ["pntf.h"]:
        if name.endswith(".h"):
            path = os.path.join(INCLUDE if name == "pntf.h" else CSRC, name)
            with open(path, "rb") as fh:
                hdr.update(name.encode() + fh.read())
    ids = {}
    for name, src, defs in UNITS:
        h = hdr.copy()
        with open(os.path.join(CSRC, src), "rb") as fh:
            h.update(fh.read())
        h.update(repr((CXXFLAGS, defs)).encode())
        ids[name] = h.hexdigest()[:16]
    return ids


def _resources(stderr):
    """Per-kernel register / spill figures from -Rpass-analysis=kernel-resource-usage."""
    out, cur = {}, None
    for line in stderr.splitlines():
        m = re.search(r"remark:.*Function Name: (\S+)", line)
        if m:
            cur = out.setdefault(m.group(1), {})
            continue
        m = re.search(r"remark:.*?\s(VGPRs|AGPRs|TotalSGPRs|VGPRs Spill|SGPRs Spill|"
                      r"ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+) ", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return out


def _compile(unit, uid=None):
    name, src, defs = unit
    d = os.path.join(BUILD, name)
    os.makedirs(d, exist_ok=True)
    obj = os.path.join(d, name + ".o")
    # per-unit cache: a unit whose code identity (and, for capi, the whole build-info string)
    # is unchanged since its last successful compile is not rebuilt
    key = None if uid is None else uid + (
        "" if name != "capi" else repr(sorted(unit_ids().items())))
    idp = os.path.join(d, "unit.id")
    if uid is not None and os.path.exists(obj) and os.path.exists(idp):
        with open(idp) as fh:
            prev = json.load(fh)
        if prev.get("id") == key:
            return obj, prev.get("res", {})
    if name == "capi":
        defs = defs + ['-DPNTF_BUILD_INFO="%s"' % ";".join(
            "%s=%s" % kv for kv in sorted(unit_ids().items()))]
    cmd = [hipcc()] + CXXFLAGS + defs + ["-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=d)
    if r.returncode != 0:
        raise RuntimeError("hipcc failed for %s:\n%s\n%s" % (name, " ".join(cmd), r.stderr))
    res = _resources(r.stderr)
    # Spills to scratch memory are what broke the 2-waves/SIMD build: any scratch use fails.
    # A VGPR "spill" with no scratch is a copy into an AGPR (a register move); only the units
    # of VGPR_SPILL_ALLOWED may have them, at most the recorded count.
    bad = {k: v for k, v in res.items() if v.get("ScratchSize [bytes/lane]", 0) or
           v.get("VGPRs Spill", 0) > VGPR_SPILL_ALLOWED.get(name, 0)}
    if bad:
        raise RuntimeError("VGPR spills / scratch in %s: %s" % (name, bad))
    if SGPR_SPILL_FREE.match(name):
        # the env-table-in-LDS instantiation (BL = true, "Lb1E": the headline's, <= 13 envs at
        # dim 3); the global-table one of the accumulate-in-bank engine keeps a few SGPR
        # spills to VGPR lanes beside its B pointers (round 6)
        sbad = {k: v["SGPRs Spill"] for k, v in res.items()
                if v.get("SGPRs Spill", 0) and "Lb1E" in k}
        if sbad:
            raise RuntimeError("SGPR spills in %s (must stay spill-free): %s" % (name, sbad))
    for asm in glob.glob(os.path.join(d, "*amdgcn*gfx950*.s")):
        with open(asm) as fh:
            text = fh.read()
        m = PACKED_FP32.search(text)
        if m:
            raise RuntimeError("packed-fp32 op %s in %s (hazard guard)" % (m.group(0), asm))
        hz = store_data_hazards(text)
        if hz:
            raise RuntimeError("store-data hazard in %s (%d, first %s)" % (asm, len(hz), hz[0]))
        if SCRATCH_UNITS.match(name):
            with open(asm) as fh:
                descs, good, bad = scratch_policy_violations(fh.read())
            if not descs or not good or bad:
                raise RuntimeError("scratch-slot policy guard in %s: descriptors %s, %d nt "
                                   "loads, %d loads without nt" % (asm, descs, good, bad))
    for f in glob.glob(os.path.join(d, "*")):
        if not f.endswith((".o", ".s")):
            os.remove(f)
    out = {name + ":" + k: v for k, v in res.items()}
    if uid is not None:
        with open(idp, "w") as fh:
            json.dump({"id": key, "res": out}, fh)
    return obj, out


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
    ids = unit_ids()
    with cf.ThreadPoolExecutor(jobs) as ex:
        results = list(ex.map(lambda u: _compile(u, None if force else ids[u[0]]), UNITS))
    objs = [o for o, _ in results]
    report = {}
    for _, res in results:
        report.update(res)
    with open(os.path.join(BUILD, "report.json"), "w") as fh:
        json.dump(report, fh, indent=1, sort_keys=True)
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
