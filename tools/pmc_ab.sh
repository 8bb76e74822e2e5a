#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
for t in AD AF; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && AFS_LIB=$GRAFT_REPO_ROOT/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pab_${t}_$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 0 --seconds 0.25) > gpurun_out/pab_${t}_$c.log 2>&1 || { echo "STOP $t $c"; exit 3; }
    python3 - "$t" "$c" <<'PY'
import csv, glob, sys
t, c = sys.argv[1], sys.argv[2]
f = glob.glob(f"gpurun_out/pab_{t}_{c}/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "tree_synth" in r["Kernel_Name"]]
print(t, c, "KiB per launch", v, "bytes/sample", [x * 1024 / (8192 * 11025) for x in v])
PY
  done
done
