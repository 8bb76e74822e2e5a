"""Executed fp64 work of the synthesis kernel from the SQ pass of tools/r02_session.sh (step
`sq`, one bench step): SQ_INSTS_VALU_FLOPS_FP64 counts flops per wave-instruction, so
lane-flops per utterance-sample = counter / wave-samples x 64 lanes / 4 utterances per wave --
written to profiles/pmc_sq_fp64.json under bench.py's key.

usage: python tools/pmc_sq_fp64.py --tag r02c [--dir gpurun_out/r02c] [--batch 8192 --samples 44100 --hop 441]
"""
import argparse
import csv
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def store(path: str, key: str, entry: dict, digest: str) -> None:
    """Merge entry into the JSON summary at path under key and the kernel sources' digest
    (areafunctionsynthesis_amd.build.kernel_digest of the tree the counters were taken on), with
    the commit it was measured at."""
    import subprocess
    try:
        entry["commit"] = subprocess.check_output(["git", "-C", ROOT, "rev-parse", "--short=10", "HEAD"],
                                                  text=True).strip()
    except Exception:
        entry["commit"] = None
    entry["digest"] = digest
    db = json.load(open(path)) if os.path.exists(path) else {}
    cur = db.get(key)
    if not isinstance(cur, dict) or "tag" in cur:  # (old layout: one entry per key)
        cur = {}
    cur[digest] = entry
    db[key] = cur
    with open(path, "w") as f:
        json.dump(db, f, indent=1, sort_keys=True)
        f.write("\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--digest", default=None, help="kernel_digest() of the measured tree (default: this tree)")
    ap.add_argument("--kernel", default="tree_synth_kernel")
    ap.add_argument("--workload", default="static")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=44100)
    ap.add_argument("--hop", type=int, default=441)
    ap.add_argument("--upw", type=float, default=4, help="utterances per wave (4: the 16-lane kernel, 1: the voice kernel)")
    a = ap.parse_args()
    d = a.dir or os.path.join(ROOT, "gpurun_out", a.tag)
    tot = {}
    for r in csv.DictReader(open(os.path.join(d, "pmc_sq", "run_counter_collection.csv"))):
        if a.kernel in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    utt_samples = float(a.batch) * a.samples  # one step: every launch of the step summed
    waves = tot["SQ_WAVES"]
    wave_samples = utt_samples / a.upw        # a.upw utterances per wave
    entry = {
        "tag": a.tag,
        "lane_flops_per_sample": tot["SQ_INSTS_VALU_FLOPS_FP64"] / wave_samples * 64.0 / a.upw,
        "utterances_per_wave": a.upw,
        "waves_per_launch_sum": waves,
        "valu_insts_per_wave_sample": tot["SQ_INSTS_VALU"] / wave_samples,
        "wave_cycles_per_wave_sample": 4.0 * tot["SQ_WAVE_CYCLES"] / wave_samples,
        "wait_any_cycles_per_wave_sample": 4.0 * tot["SQ_WAIT_ANY"] / wave_samples,
        "active_valu_cycles_per_wave_sample": 4.0 * tot["SQ_ACTIVE_INST_VALU"] / wave_samples,
        "note": "SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_ACTIVE_INST_VALU count quad-cycles (x 4); per wave-sample = "
                "per wave and audio sample (a wave holds utterances_per_wave utterances)",
    }
    import sys
    sys.path.insert(0, ROOT)
    from areafunctionsynthesis_amd.build import kernel_digest
    store(os.path.join(ROOT, "profiles", "pmc_sq_fp64.json"), f"{a.kernel}|{a.workload}|B={a.batch}|T={a.samples}|hop={a.hop}",
          entry, a.digest or kernel_digest())
    print(json.dumps(entry))


if __name__ == "__main__":
    main()
