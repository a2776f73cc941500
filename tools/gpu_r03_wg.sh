#!/bin/bash
# The weight-reduce HBM roofline in the bench line (kernel_times slot [6]): a few parity tests, the
# default bench and the point-mass bench.
set -o pipefail
mkdir -p gpurun_out/r03wg
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "event_ring or config3 or point_mass" --timeout 120 --timeout-method thread || exit 1
timeout -k 10 120 python -u bench.py > gpurun_out/r03wg/bench.json 2> gpurun_out/r03wg/bench.err || exit 1
timeout -k 10 120 python -u bench.py --workload point_mass --no-cpu-baseline > gpurun_out/r03wg/pm.json 2> gpurun_out/r03wg/pm.err || exit 1
python3 - <<'PY'
import json
for f in ("gpurun_out/r03wg/bench.json", "gpurun_out/r03wg/pm.json"):
    d = json.loads(open(f).read().strip().split("\n")[-1])
    print(d["ms_per_step"], d["kernel_ms"]["breakdown_untimed"], d["hbm"].get("weight_reduce"))
PY
