#!/bin/bash
# Round 3: the whole GPU suite, then interleaved bench pairs with the fifth wave's rows handed over
# (MPPI_HANDOVER=1, the default) and kept on the doubled SIMD (0).  Logs under gpurun_out/r03ho/.
set -o pipefail
mkdir -p gpurun_out/r03ho
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/r03ho/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|handover steps" gpurun_out/r03ho/pytest.log | tail -30
if [ $rc -gt 1 ]; then exit $rc; fi
for i in 1 2 3; do
  for ho in 1 0; do
    MPPI_HANDOVER=$ho timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/r03ho/bench_ho${ho}_$i.log 2>&1 || { echo "bench ho=$ho rc=$?"; tail -20 gpurun_out/r03ho/bench_ho${ho}_$i.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().split('\n')[-1]); print(sys.argv[2], d['ms_per_step'], d['kernel_ms']['rollout_launch'])" gpurun_out/r03ho/bench_ho${ho}_$i.log ho=$ho
  done
done
exit $rc
