#!/bin/bash
# The whole GPU suite, then configs[4]'s share per GPU (8192 x 128, SG w = 10: the two-launch split)
# eager against the five-node hipGraph, interleaved.  Output: gpurun_out/r03gs/.
set -o pipefail
O=gpurun_out/r03gs
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FAILED|ERROR" $O/pytest.log | tail -10
tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
for i in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --graph $g --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10 --steps 100 > $O/g${g}_$i.json 2> $O/g${g}_$i.err || { echo "bench rc=$?"; tail -5 $O/g${g}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/g${g}_$i.json').read().strip().split('\n')[-1]); print('8192x128 SG graph=$g ms/update %.4f launch %.4f graph_updates %d' % (d['ms_per_step'], d['kernel_ms']['rollout_launch'], d['engine']['graph_updates_timed']))"
  done
done
