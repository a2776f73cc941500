#!/bin/bash
# Round 3: the launch-path equality tests, then the whole GPU suite.  Logs under gpurun_out/r03paths/.
set -o pipefail
O=gpurun_out/r03paths
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_launch_paths.py -v -s --timeout 200 --timeout-method thread > $O/pytest_paths.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest_paths.log | tail -20
if [ $rc -ne 0 ]; then tail -60 $O/pytest_paths.log; exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -20
exit $rc
