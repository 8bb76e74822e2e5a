"""Build libafs.so (HIP, gfx950) in-tree with hipcc.

Usage: python -m areafunctionsynthesis_amd.build [--force]
The shared library lands next to this file so it travels with the repository snapshot.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libafs.so")
ARCH = os.environ.get("AFS_OFFLOAD_ARCH", "gfx950")

SOURCES = ["afs_capi.cpp", "afs_comm.cpp", "afs_tables.cpp", "tds_lane.hip", "tds_tree.hip", "tds_plan.hip",
           "af_kernels.hip", "audio_kernels.hip"]
HEADERS = ["afs_model.h", "afs_ctx.h", "afs_gather.h", "afs_af.h", "afs_lane.h", "afs_tree.h", "afs_audio.h", "tree_core.h", "tree_plan.h", "tree_kernel.h",
           os.path.join("..", "..", "include", "afs.h")]
# Per-source extra flags.
# The tree kernel contracts a*b+c into fma (-ffp-contract=fast-honor-pragmas after COMMON's
# =off; plain "fast" ignores the `#pragma clang fp contract(off)` that keeps the tube
# interpolation uncontracted like K5's and the reference's, tests/test_plan_gpu.py): 8 % fewer
# VALU instructions in its time loop, +3.5 % end to end (A/B, profiles/r02ac_contract_ab.txt);
# its results stay within the parity tolerances (the reference's own build with FMA
# contraction differs from its -O2 build by up to 5.7e-9 over a second).  The
# plan kernel (K5, the reference's discrete constriction decisions) and the lane kernel (the
# reference's operation order) keep COMMON's -ffp-contract=off.
# The tree kernel is built without machine-level loop-invariant code motion: hoisting the
# lanes' loop-invariant comparisons out of the time loop kept ~50 lane masks alive in SGPR
# pairs, more than the wave has, and their spills cost ~100 v_readlane/v_writelane and ~130
# AGPR moves per sample (A/B: 89.0 vs 89.25 ms per launch).
# The machine scheduler's iterative-ilp strategy (re-schedules each region for latency once
# the register budget is known): 25.9 k -> 25.2 k cycles per wave-sample, +1.5-2 % end to
# end (A/B alternated, profiles/r03k_sched_ab.txt; iterative-minreg -16 %, post-RA machine
# scheduler / no machine sinking / no memop clustering neutral or slower).  Instruction order
# only: the results are bit-identical.
# -fno-signed-zeros: the reference's accumulations from 0.0 (`double u = 0.0; u += x;`, ~35 per
# sample) are kept as written in the source and compile to x; they differ from x only for x = -0,
# and no comparison, product or sum in this kernel tells -0 from +0 except in a zero result (no
# division by a possibly-zero value, no copysign).  A/B: profiles/r04n_nsz_ab.txt.
TREE_FLAGS = ["-mllvm", "-disable-machine-licm", "-ffp-contract=fast-honor-pragmas", "-fno-signed-zeros", "-mllvm", "-amdgpu-sched-strategy=iterative-ilp"]
PER_SOURCE: dict = {"tds_tree.hip": list(TREE_FLAGS)}
# (AFS_TREE_FLAGS: extra compiler flags for the tree kernel, for A/B builds of scheduler options)
if os.environ.get("AFS_TREE_FLAGS"):
    PER_SOURCE["tds_tree.hip"] = TREE_FLAGS + os.environ["AFS_TREE_FLAGS"].split()

COMMON = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function",
          # keep the reference's rounding: no contraction of a*b+c into fma (except the tree
          # kernel, TREE_FLAGS)
          "-ffp-contract=off", "-fno-strict-aliasing", "-Wno-unknown-pragmas"]


def _hipcc() -> str:
    for p in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.sep not in p or os.path.exists(p):
            return p
    return "hipcc"


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    if os.path.getmtime(os.path.abspath(__file__)) > t:  # (flags changed)
        return True
    for f in SOURCES + HEADERS:
        if os.path.getmtime(os.path.join(CSRC, f)) > t:
            return True
    return False


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not _stale():
        return LIB
    objdir = os.path.join(HERE, "_obj")
    os.makedirs(objdir, exist_ok=True)
    objs = []
    for src in SOURCES:
        obj = os.path.join(objdir, os.path.splitext(src)[0] + ".o")
        lang = ["-x", "hip"] if src.endswith(".cpp") else []
        cmd = ([_hipcc(), "-c"] + lang + [os.path.join(CSRC, src), "-o", obj, f"--offload-arch={ARCH}"] + COMMON
               + PER_SOURCE.get(src, []))
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
        objs.append(obj)
    cmd = [_hipcc(), "-shared", "-o", LIB + ".tmp", f"--offload-arch={ARCH}", "-fPIC"] + objs + ["-ldl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(LIB + ".tmp", LIB)
    return LIB


# the headers the synthesis kernels' objects are compiled from (host-only headers excluded)
KERNEL_HEADERS = {"tds_tree.hip": ["afs_model.h", "afs_tree.h", "tree_core.h", "tree_plan.h", "tree_kernel.h",
                                   os.path.join("..", "..", "include", "afs.h")],
                  "tds_plan.hip": ["afs_model.h", "afs_tree.h", "tree_plan.h", os.path.join("..", "..", "include", "afs.h")]}


def kernel_digest(source: str = "tds_tree.hip") -> str:
    """Digest of what one kernel's object is built from (the source file, the headers it
    includes, its compiler flags): the committed PMC summaries (profiles/pmc_*.json) are keyed
    by it, so bench.py quotes a counter figure only for the kernel it is timing."""
    import hashlib
    import re
    h = hashlib.sha1()
    for f in [source] + KERNEL_HEADERS.get(source, HEADERS):
        h.update(f.encode())
        with open(os.path.join(CSRC, f), encoding="utf-8") as fh:
            text = fh.read()
        # (comments and blank space do not change the object: documentation edits keep the key)
        text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
        text = re.sub(r"//[^\n]*", " ", text)
        h.update(" ".join(text.split()).encode())
    h.update(repr((COMMON, PER_SOURCE.get(source, []))).encode())
    return h.hexdigest()[:12]


if __name__ == "__main__":
    build(force="--force" in sys.argv)
