#!/bin/bash
# Quick loop: handover + parity tests, wave traces, bench pairs (handover 1 / 0).
set -o pipefail
mkdir -p gpurun_out/r03q
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py -m gpu -x -q -s --timeout 240 --timeout-method thread -k "handover or bench_mode or graph or draws_ahead or config1 or golden" > gpurun_out/r03q/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/r03q/pytest.log; exit 1; }
grep -E "passed|failed|handover steps" gpurun_out/r03q/pytest.log | tail -8
bash tools/gpu_r03_wt.sh || exit 1
for i in 1 2; do
  for ho in 1 0; do
    f=gpurun_out/r03q/bench_ho${ho}_$i.log
    MPPI_HANDOVER=$ho timeout -k 10 200 python -u bench.py --no-cpu-baseline > $f 2>&1 || { echo "bench rc=$?"; tail -5 $f; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], d['ms_per_step'], d['kernel_ms']['rollout_launch'], d['engine']['handover'], d['engine']['wait_timeouts'])" $f "ho=$ho"
  done
done
