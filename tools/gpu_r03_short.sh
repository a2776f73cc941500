#!/bin/bash
# The driver's short bench (--steps 20 --warmup 5) against longer timed regions and warm-ups.
set -o pipefail
O=gpurun_out/r03short
mkdir -p $O
i=0
for kw in "20 5" "20 5" "20 50" "200 5" "200 10" "2000 10" "20 5"; do
  set -- $kw
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps $1 --warmup $2 > $O/b$i.json 2> $O/b$i.err || { echo "bench rc=$?"; tail -5 $O/b$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$i.json').read().strip().split('\n')[-1]); print('steps $1 warmup $2 ms/update %.4f launch %.4f samples %d' % (d['ms_per_step'], d['kernel_ms']['rollout_launch'], d['kernel_ms']['rollout_launch_samples']))"
done
