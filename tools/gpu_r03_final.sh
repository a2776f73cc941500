#!/bin/bash
# Round 3 closing set (run via gpurun): smoke, the whole GPU suite in one pytest process, then the
# profile set (tools/gpu_r03_profile.sh: bench line, rocprofv3 kernel stats + trace, PMC passes,
# the BASELINE sizes).  Logs under gpurun_out/r03g/ and gpurun_out/r03prof/.
set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03g/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/r03g/smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/r03g/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r03g/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_r03_profile.sh
