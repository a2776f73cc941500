#!/bin/bash
# Round 3: smoke, the whole GPU suite, then the profile set (tools/gpu_r03_profile.sh).
set -o pipefail
mkdir -p gpurun_out/r03full
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03full/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/r03full/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 700 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/r03full/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r03full/pytest.log | tail -20
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_r03_profile.sh || exit 1
exit $rc
