mkdir -p gpurun_out/r03f
timeout -k 10 400 python -u -m pytest tests/test_plan_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r03f/plan_default.log 2>&1
st=$?; echo "default status $st"; tail -5 gpurun_out/r03f/plan_default.log
if [ $st -ne 0 ] && [ $st -ne 1 ]; then exit $st; fi
AFS_LIB=$PWD/areafunctionsynthesis_amd/libafs_planoff.so timeout -k 10 400 python -u -m pytest tests/test_plan_gpu.py -v --timeout 300 --timeout-method thread > gpurun_out/r03f/plan_cseoff.log 2>&1
st=$?; echo "cse-off status $st"; grep -E "PASS|FAIL|differ" gpurun_out/r03f/plan_cseoff.log | head -30
