"""Summarise the FETCH_SIZE / WRITE_SIZE passes of tools/gpu_session.sh (step `pmc`) into the
per-launch HBM traffic that bench.py reports as roofline.traffic.

usage: python tools/pmc_traffic.py --tag r01_v2j [--batch 8192 --seconds 1 --fs 44100 --hop 441]

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts half the bytes of a coalesced streaming read,
so it is doubled; WRITE_SIZE is taken as is.  The result is merged into profiles/pmc_traffic.json
under a key that names the workload, so bench.py only uses it for the same configuration.
"""
from __future__ import annotations

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


def key(kernel: str, workload: str, batch: int, samples: int, hop: int) -> str:
    return f"{kernel}|{workload}|B={batch}|T={samples}|hop={hop}"


def per_launch(path: str, kernel: str) -> list[float]:
    rows = [r for r in csv.DictReader(open(path)) if kernel in r["Kernel_Name"]]
    return [float(r["Counter_Value"]) for r in rows]


PLAN_KERNELS = ("plan_kernel", "plan_hop_iv_kernel", "plan_hop_wave_kernel")  # K5: dense / hop mode


def plan_total(path: str) -> float:
    return sum(float(r["Counter_Value"]) for r in csv.DictReader(open(path))
               if any(k in r["Kernel_Name"] for k in PLAN_KERNELS))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--dir", default=None)
    ap.add_argument("--digest", default=None, help="kernel_digest() of the measured tree (default: this tree)")
    ap.add_argument("--kernel", default="tree_synth_kernel")
    ap.add_argument("--workload", default="static")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--samples", type=int, default=44100)
    ap.add_argument("--hop", type=int, default=441)
    ap.add_argument("--plan-fetch-factor", type=float, default=2.0,
                    help="read bytes per FETCH_SIZE byte of K5's kernels: 2 since K5 copies its block's frames "
                         "to LDS with coalesced loads (fetch_calib b128 / b64_row16)")
    ap.add_argument("--plan-calibration", default="profiles/r05m_fetch_calib.txt",
                    help="where --plan-fetch-factor was measured")
    a = ap.parse_args()
    a.dir = a.dir or os.path.join(ROOT, "gpurun_out", a.tag)
    fetch = per_launch(os.path.join(a.dir, "pmc_fetch", "run_counter_collection.csv"), a.kernel)
    write = per_launch(os.path.join(a.dir, "pmc_write", "run_counter_collection.csv"), a.kernel)
    if not fetch or not write:
        raise SystemExit("no launches of the kernel in the PMC passes")
    kib = 1024.0
    fetch_b = 2.0 * kib * sum(fetch) / len(fetch)   # gfx950: FETCH_SIZE = half the read bytes
    write_b = kib * sum(write) / len(write)
    plan_f = plan_total(os.path.join(a.dir, "pmc_fetch", "run_counter_collection.csv"))
    plan_w = plan_total(os.path.join(a.dir, "pmc_write", "run_counter_collection.csv"))
    entry = {
        "tag": a.tag,
        "launches": len(fetch),
        "fetch_size_kib": fetch, "write_size_kib": write,
        "read_bytes_per_launch": fetch_b, "write_bytes_per_launch": write_b,
        "traffic_bytes_per_launch": fetch_b + write_b,
        "correction": "read = 2 x FETCH_SIZE (gfx950; calibrated for this kernel's read patterns -- 8-B loads of "
                      "16-lane rows, 16-B loads, lane-0 8-B loads -- by tools/microbench/fetch_calib: each reports "
                      "half the bytes of the 128-B lines it reads, profiles/r02_fetch_calib.txt), write = WRITE_SIZE; "
                      "KiB -> bytes",
    }
    if plan_f or plan_w:  # K5 (all its kernels), the noise-source plan producer of the same launches
        launches = len(fetch)
        frames = a.batch * (a.samples // a.hop + 1) * 1072.0 / launches  # each frame once
        records = a.batch * (-(-a.samples // a.hop)) * 544.0 / launches    # each hop record once
        entry["plan_kernel_fetch_size_kib_per_launch"] = plan_f / launches
        entry["plan_kernel_read_bytes_per_launch"] = a.plan_fetch_factor * kib * plan_f / launches
        entry["plan_kernel_write_bytes_per_launch"] = kib * plan_w / launches
        entry["plan_kernel_traffic_bytes_per_launch"] = (a.plan_fetch_factor * kib * plan_f + kib * plan_w) / launches
        entry["plan_kernel_algorithmic_bytes_per_launch"] = frames + records
        entry["plan_kernel_traffic_ratio"] = entry["plan_kernel_traffic_bytes_per_launch"] / (frames + records)
        entry["plan_kernel_traffic_ratio"] = entry["plan_kernel_traffic_bytes_per_launch"] / (frames + records)
        entry["plan_kernel_correction"] = (f"read = {a.plan_fetch_factor:g} x FETCH_SIZE: K5 copies each block's "
                                           "frames to LDS with coalesced loads, the pattern fetch_calib calibrates "
                                           "at 2 (b128, b64_row16); the per-lane walk over 1072-B frames that K5 "
                                           "used before (rec1072) reports 7.5x a coalesced read's FETCH_SIZE for "
                                           f"the same bytes, i.e. it re-fetched lines ({a.plan_calibration}); "
                                           "write = WRITE_SIZE; algorithmic = every frame read once + every hop "
                                           "record written once")
    import sys
    sys.path.insert(0, ROOT)
    from areafunctionsynthesis_amd.build import kernel_digest
    store(os.path.join(ROOT, "profiles", "pmc_traffic.json"), key(a.kernel, a.workload, a.batch, a.samples, a.hop),
          entry, a.digest or kernel_digest())
    print(json.dumps(entry))


if __name__ == "__main__":
    main()
