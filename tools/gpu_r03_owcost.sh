#!/bin/bash
# Round 3: the objective inside one-wave launches (past one round of workgroups) - the equality
# tests and the scale parity, then 32768 x 64 and 65536 x 128 SG with the objective in the launch
# and in fr_step_cost_kernel (MPPI_COSTS_IN_LAUNCH=0), interleaved.  Output: gpurun_out/r03w/.
set -o pipefail
O=gpurun_out/r03w
mkdir -p $O
[ -z "$SKIP_TESTS" ] && timeout -k 10 600 python -u -m pytest tests/test_gpu_launch_paths.py tests/test_gpu_scale.py -v -s \
    --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
[ -z "$SKIP_TESTS" ] && tail -25 $O/pytest.log
if [ -z "$SKIP_TESTS" ] && [ $rc -ne 0 ]; then exit $rc; fi
b() {   # name env args...
    local n=$1 e=$2; shift 2
    timeout -k 10 300 env $e python -u bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -5 $O/$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().split('\n')[-1]); print('%-18s ms/update %.4f value %.3e launch %.4f' % ('$n', d['ms_per_step'], d['value'], d['kernel_ms']['rollout_launch']))"
}
for i in 1 2; do
  b s32k_cil1_$i MPPI_COSTS_IN_LAUNCH=1 --steps 20 --warmup 3 --samples-per-gpu 32768 || exit 1
  b s32k_cil0_$i MPPI_COSTS_IN_LAUNCH=0 --steps 20 --warmup 3 --samples-per-gpu 32768 || exit 1
  b s64k_cil1_$i MPPI_COSTS_IN_LAUNCH=1 --steps 8 --warmup 2 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10 || exit 1
  b s64k_cil0_$i MPPI_COSTS_IN_LAUNCH=0 --steps 8 --warmup 2 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10 || exit 1
done
b default MPPI_COSTS_IN_LAUNCH=1 || exit 1
