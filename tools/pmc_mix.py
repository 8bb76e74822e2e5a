"""Dynamic instruction mix and cycle split of the synthesis kernel from the three SQ passes of
tools/session.sh (step `mix`, one bench step each): instructions and cycles per
wave-sample (--upw utterances per wave: 4 for the one-wave kernel, 2 for the wave pairs).  Writes
profiles/pmc_mix.json under bench.py's key and the kernel sources' digest, and prints a table.

usage: python tools/pmc_mix.py --tag r03h [--dir gpurun_out/r03h] [--batch 8192 --samples 44100 --hop 441]
"""
import argparse
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
from pmc_sq_fp64 import store  # noqa: E402

# SQ_WAVE_CYCLES, SQ_ACTIVE_INST_* and SQ_WAIT_* count quad-cycles on gfx950 (x 4)
QUAD = ("SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
        "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY")


def totals(path, kernel):
    tot = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--kernel", default="tree_synth_kernel")
    ap.add_argument("--workload", default="static")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=44100)
    ap.add_argument("--hop", type=int, default=441)
    ap.add_argument("--digest", default=None)
    ap.add_argument("--upw", type=float, default=4,
                    help="utterances per wave (4: the one-wave 16-lane kernel; 2: the wave pairs, two waves per "
                         "four utterances; 1: the voice kernel)")
    a = ap.parse_args()
    d = a.dir or os.path.join(ROOT, "gpurun_out", a.tag)
    t = {}
    for p in ("pmc_mix1", "pmc_mix2", "pmc_mix3"):
        t.update(totals(os.path.join(d, p, "run_counter_collection.csv"), a.kernel))
    ws = float(a.batch) * a.samples / a.upw  # wave-samples of one step
    per = {k: (4.0 if k in QUAD else 1.0) * v / ws for k, v in t.items() if k != "SQ_WAVES"}
    f64 = sum(per.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS"))
    valu = per["SQ_INSTS_VALU"]
    mix = {
        "valu": valu,
        "valu_fp64_arith": f64,
        "valu_fp64_add": per.get("SQ_INSTS_VALU_ADD_F64"),
        "valu_fp64_mul": per.get("SQ_INSTS_VALU_MUL_F64"),
        "valu_fp64_fma": per.get("SQ_INSTS_VALU_FMA_F64"),
        "valu_fp64_trans": per.get("SQ_INSTS_VALU_TRANS_F64"),
        "valu_int32": per.get("SQ_INSTS_VALU_INT32"),
        "valu_int64": per.get("SQ_INSTS_VALU_INT64"),
        "valu_cvt": per.get("SQ_INSTS_VALU_CVT"),
        "valu_other": valu - f64 - sum(per.get(k, 0.0) for k in ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64",
                                                                 "SQ_INSTS_VALU_CVT")),
        "salu": per.get("SQ_INSTS_SALU"),
        "lds": per.get("SQ_INSTS_LDS"),
        "smem": per.get("SQ_INSTS_SMEM"),
        "branch": per.get("SQ_INSTS_BRANCH"),
        "vmem_rd": per.get("SQ_INSTS_VMEM_RD"),
        "vmem_wr": per.get("SQ_INSTS_VMEM_WR"),
        "wave_cycles": per.get("SQ_WAVE_CYCLES"),
        "active_any_cycles": per.get("SQ_ACTIVE_INST_ANY"),
        "active_valu_cycles": per.get("SQ_ACTIVE_INST_VALU"),
        "active_lds_cycles": per.get("SQ_ACTIVE_INST_LDS"),
        "active_salu_cycles": per.get("SQ_ACTIVE_INST_SCA"),
        "wait_inst_any_cycles": per.get("SQ_WAIT_INST_ANY"),
        "wait_any_cycles": per.get("SQ_WAIT_ANY"),
    }
    entry = {"tag": a.tag, "per_wave_sample": mix, "utterances_per_wave": a.upw,
             "note": f"per wave and audio sample ({a.upw} utterances per wave); VALU other = moves, selects, AGPR copies, DPP "
                     "moves, lane reads/writes, compares (everything that is not fp64 arithmetic, int or cvt); "
                     "cycle counters x 4 (quad-cycles)"}
    from areafunctionsynthesis_amd.build import kernel_digest
    store(os.path.join(ROOT, "profiles", "pmc_mix.json"), f"{a.kernel}|{a.workload}|B={a.batch}|T={a.samples}|hop={a.hop}",
          entry, a.digest or kernel_digest())
    for k, v in mix.items():
        print(f"{k:24s} {v:10.1f}" if v is not None else f"{k:24s}        n/a")


if __name__ == "__main__":
    main()
