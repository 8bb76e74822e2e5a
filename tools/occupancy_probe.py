"""Register / LDS budget of the synthesis kernel per lane width and waves-per-SIMD target
(development tool, CPU only): hipcc's kernel-resource-usage remarks for tds_tree.hip built with
the product's flags plus -DAFS_TREE_W / -DAFS_TREE_MIN_WAVES.  usage: python tools/occupancy_probe.py
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from areafunctionsynthesis_amd.build import COMMON, TREE_FLAGS  # noqa: E402

FIELDS = ("VGPRs", "AGPRs", "VGPRs Spill", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]")


def probe(w: int, waves: int):
    cmd = (["/opt/rocm/bin/hipcc", "-c", "-x", "hip", os.path.join(ROOT, "areafunctionsynthesis_amd", "csrc", "tds_tree.hip"),
            "-o", "/tmp/occ_probe.o", "--offload-arch=gfx950"] + COMMON + TREE_FLAGS +
           [f"-DAFS_TREE_W={w}", f"-DAFS_TREE_MIN_WAVES={waves}", "-Rpass-analysis=kernel-resource-usage"])
    txt = subprocess.run(cmd, capture_output=True, text=True).stderr
    out, cur = {}, None
    for line in txt.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        for f in FIELDS:
            m = re.search(r"remark:\s+" + re.escape(f) + r": (\d+)", line)
            if m and cur:
                out[cur][f] = int(m.group(1))
    return out


def main():
    for w, waves in ((16, 1), (16, 2), (32, 1), (32, 2)):
        print(f"== -DAFS_TREE_W={w} -DAFS_TREE_MIN_WAVES={waves} (the 64-lane voice kernel is instantiated in every build)")
        for f, d in probe(w, waves).items():
            m = re.search(r"tree_synth_kernelILi(\d)ELb(\d)ELi(\d+)E", f)
            if not m:
                continue
            model = "two-mass" if m.group(1) == "1" else "triangular"
            plan = "hop records" if m.group(2) == "1" else "dense plans"
            print(f"  tree_synth_kernel<{model}, {plan}, W={m.group(3)}>: " +
                  ", ".join(f"{k} {d.get(k, 0)}" for k in FIELDS))


if __name__ == "__main__":
    main()
