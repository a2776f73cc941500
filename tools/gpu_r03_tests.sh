#!/bin/bash
# Round 3: smoke + the whole GPU suite (one pytest process), logs under gpurun_out/r03t/.
set -o pipefail
mkdir -p gpurun_out/r03t
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03t/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/r03t/smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/r03t/pytest.log 2>&1
rc=$?
tail -40 gpurun_out/r03t/pytest.log
exit $rc
