#!/bin/bash
# Round 3: the one-rank RCCL path, then the whole GPU suite.  Logs under gpurun_out/r03rccl/.
set -o pipefail
O=gpurun_out/r03rccl
mkdir -p $O
NCCL_DEBUG=INFO timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py -v -s --timeout 200 --timeout-method thread > $O/pytest_rccl.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|NCCL INFO (Init|Channel 00|comm 0x)" $O/pytest_rccl.log | head -20
if [ $rc -ne 0 ]; then tail -60 $O/pytest_rccl.log; exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" $O/pytest.log | tail -20
exit $rc
