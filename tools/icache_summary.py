"""Per-kernel instruction-cache counters of tools/icache_probe.sh passes (development tool)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    out, tags = sys.argv[1], sys.argv[2:]
    for t in tags:
        files = glob.glob(os.path.join(out, f"ic_{t}", "**", "*counter_collection.csv"), recursive=True)
        if not files:
            print(t, "no counter file")
            continue
        acc = defaultdict(lambda: defaultdict(float))
        for f in files:
            for r in csv.DictReader(open(f)):
                k = r.get("Kernel_Name", "?")
                if "tree_synth" not in k:
                    continue
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        for k, c in acc.items():
            hits, miss = c.get("SQC_ICACHE_HITS", 0.0), c.get("SQC_ICACHE_MISSES", 0.0)
            waves, cyc = c.get("SQ_WAVES", 0.0), c.get("SQ_WAVE_CYCLES", 0.0)
            rate = miss / max(1.0, hits + miss)
            print(f"{t:8s} {k[:60]:60s} icache hits {hits:.3e} misses {miss:.3e} miss rate {rate:.4f} "
                  f"waves {waves:.0f} wave-cycles {cyc:.3e}")


if __name__ == "__main__":
    main()
