#!/bin/bash
# Round 3: the two-launch split (fr_coop_update_split) and the one-wave lead rounds ahead of it
# (fr_coop_update_lead_rows) - their equality tests and the scale parity, then the configs[4] per-GPU
# workload (8192 x 128, SG w = 10), 8192 x 64 and 32768 x 64 with the split and without it
# (MPPI_SPLIT=0), interleaved.  Output: gpurun_out/r03s/.
set -o pipefail
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_launch_paths.py tests/test_gpu_scale.py -k "split or config or bench_mode" -v -s \
    --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -15 $O/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
b() {   # name env args...
    local n=$1 e=$2; shift 2
    timeout -k 10 300 env $e python -u bench.py --no-cpu-baseline "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n rc=$?"; tail -5 $O/$n.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().split('\n')[-1]); print('%-18s ms/update %.4f value %.3e launch %.4f' % ('$n', d['ms_per_step'], d['value'], d['kernel_ms']['rollout_launch']))"
}
for i in 1 2; do
  b sg_split_$i MPPI_SPLIT=1 --steps 40 --warmup 5 --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10 || exit 1
  b sg_onewave_$i MPPI_SPLIT=0 --steps 40 --warmup 5 --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10 || exit 1
  b h64_split_$i MPPI_SPLIT=1 --steps 60 --warmup 5 --samples-per-gpu 8192 || exit 1
  b h64_onewave_$i MPPI_SPLIT=0 --steps 60 --warmup 5 --samples-per-gpu 8192 || exit 1
  b s32k_split_$i MPPI_SPLIT=1 --steps 20 --warmup 3 --samples-per-gpu 32768 || exit 1
  b s32k_onewave_$i MPPI_SPLIT=0 --steps 20 --warmup 3 --samples-per-gpu 32768 || exit 1
done
b s64k_sg_split MPPI_SPLIT=1 --steps 8 --warmup 2 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10 || exit 1
b s64k_sg_onewave MPPI_SPLIT=0 --steps 8 --warmup 2 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10 || exit 1
b default MPPI_SPLIT=1 || exit 1
