#!/bin/bash
# smoke + the whole GPU suite, then the one-wave objective A/B (bench part of gpu_r03_owcost.sh),
# then the closing profile set (gpu_r03_profile.sh).
set -o pipefail
mkdir -p gpurun_out/r03g
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03g/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 gpurun_out/r03g/smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > gpurun_out/r03g/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/r03g/pytest.log | grep -v "^tests.*PASSED$" | tail -20
tail -3 gpurun_out/r03g/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
SKIP_TESTS=1 bash tools/gpu_r03_owcost.sh || exit 1
bash tools/gpu_r03_profile.sh || exit 1
bash tools/gpu_r03_cs_ab.sh
mkdir -p gpurun_out/r03gsg
for i in 1 2; do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --graph $g --horizon-steps 128 --smoothing 10 --steps 100 > gpurun_out/r03gsg/g${g}_$i.json 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/r03gsg/g${g}_$i.json').read().strip().split('\n')[-1]); print('4096x128 SG graph=$g ms/update %.4f launch %.4f graph_updates %d' % (d['ms_per_step'], d['kernel_ms']['rollout_launch'], d['engine']['graph_updates_timed']))"
  done
done
