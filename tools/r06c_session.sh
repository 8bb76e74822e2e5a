set -u
cd $GRAFT_REPO_ROOT
bash tools/session.sh r06c test smoke || exit 1
mkdir -p gpurun_out/r06c
for t in base tone2; do AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_$t.so timeout -k 10 300 python tools/lib_equal.py write /tmp/eq_$t.npz > gpurun_out/r06c/eq_$t.log 2>&1 || { echo "eq $t failed"; exit 1; }; done
python tools/lib_equal.py compare /tmp/eq_base.npz /tmp/eq_tone2.npz > gpurun_out/r06c/eq_compare.txt; cat gpurun_out/r06c/eq_compare.txt
AB="base tone2" AB_BATCH=8192 AB_SECONDS=0.64 timeout -k 10 900 bash tools/ab.sh > gpurun_out/r06c/ab_tone2_8192.txt 2>&1; cat gpurun_out/r06c/ab_tone2_8192.txt
