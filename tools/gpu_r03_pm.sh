#!/bin/bash
# Point-mass path (configs[1]): its parity tests, then the 1024 x 32 bench (three runs).
set -o pipefail
O=gpurun_out/r03pm
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "point_mass|FAILED|ERROR|passed|failed" $O/pytest.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload point_mass > $O/pm_$i.json 2> $O/pm_$i.err || { echo "bench rc=$?"; tail -5 $O/pm_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/pm_$i.json').read().strip().split('\n')[-1]); k=d['kernel_ms']; print('pm ms/update %.4f launch %.4f breakdown %s' % (d['ms_per_step'], k['rollout_launch'], k['breakdown_untimed']))"
done
