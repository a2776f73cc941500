#!/bin/bash
# Soak: long default-bench runs (20000 and 50000 updates) - bounded in-launch waits must never time
# out (engine.wait_timeouts == 0) and the rate must hold; then 2000 updates at 8192 x 128 SG (split).
set -o pipefail
O=gpurun_out/r03soak
mkdir -p $O
for n in 20000 50000; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps $n --warmup 10 > $O/s$n.json 2> $O/s$n.err || { echo "soak $n rc=$?"; tail -5 $O/s$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/s$n.json').read().strip().split('\n')[-1]); print('steps $n ms/update %.4f wait_timeouts %d launch %.4f' % (d['ms_per_step'], d['engine']['wait_timeouts'], d['kernel_ms']['rollout_launch']))"
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2000 --warmup 10 --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10 > $O/split.json 2> $O/split.err || { echo "split soak rc=$?"; tail -5 $O/split.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/split.json').read().strip().split('\n')[-1]); print('8192x128 SG 2000 ms/update %.4f wait_timeouts %d' % (d['ms_per_step'], d['engine']['wait_timeouts']))"
