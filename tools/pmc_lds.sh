#!/bin/bash
# LDS counter pass over the phase profiler's kernel (development tool; run on the GPU box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-lds}
OUT=$PWD/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${PP_ARGS:-"--batch 8192 --seconds 0.02"}
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL --output-format csv -d $OUT -o run -- python3 $GRAFT_REPO_ROOT/tools/phase_prof/run.py $ARGS) > $OUT/log.txt 2>&1 || { echo "pmc pass failed"; tail -5 $OUT/log.txt; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
tot = collections.defaultdict(float)
for r in csv.DictReader(open(f)):
    if "tree_prof" in r["Kernel_Name"]:
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
w = tot["SQ_WAVES"]
for k, v in sorted(tot.items()):
    print(f"{k:26s} {v:14.6g}  per wave {v / w:12.1f}")
PY
