# one-off GPU call (round 3): GPU suite, scaling sweep of the adaptive split, profile refresh
set -o pipefail
mkdir -p gpurun_out/r03b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_configs.py > gpurun_out/r03b/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03b/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/prof_scaling.py 20 > gpurun_out/r03b/scaling_main.jsonl 2>&1 || exit 3
for v in rounds2 rounds8 tail8; do
  PT_HIP_LIB=$PWD/pathtracerpython_amd/_lib/variants/$v.so timeout -k 10 200 python scripts/prof_scaling.py 20 > gpurun_out/r03b/scaling_$v.jsonl 2>&1 || exit 4
done
cat gpurun_out/r03b/scaling_*.jsonl
if [ $rc -ne 0 ]; then exit 1; fi
bash scripts/refresh_profiles.sh r03 > gpurun_out/r03b/refresh.log 2>&1; rc=$?
tail -5 gpurun_out/r03b/refresh.log; exit $rc
