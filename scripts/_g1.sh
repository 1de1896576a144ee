# one-off GPU call (round 3): GPU suite, then per-band scaling sweeps
set -o pipefail
mkdir -p gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --deselect tests/test_gpu_configs.py > gpurun_out/r03a/gputest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03a/gputest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python scripts/prof_scaling.py 20 > gpurun_out/r03a/scaling_main.jsonl 2>&1 || exit 3
for v in 16 32 64; do
  PT_HIP_LIB=$PWD/pathtracerpython_amd/_lib/variants/split$v.so timeout -k 10 200 python scripts/prof_scaling.py 20 > gpurun_out/r03a/scaling_split$v.jsonl 2>&1 || exit 4
done
cat gpurun_out/r03a/scaling_*.jsonl
