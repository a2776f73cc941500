# GPU parity tests, then the bench at the default and the larger BASELINE workloads (run via gpurun).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/sizes
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
run() {   # name args...
    local n=$1; shift
    timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/sizes/$n.json 2> gpurun_out/sizes/$n.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/sizes/$n.json')); k=d['kernel_ms']; b=k['breakdown_untimed']; print('%-10s %s ms/update %.4f dyn %.4f cost %.4f sample %.4f reduce %.4f' % ('$n', d['metric'][-40:], d['ms_per_step'], k['rollout_dynamics'], k['rollout_cost'], b['sample'], b['reduce']))"
}
run c3 --steps 30 --warmup 3
run s32k --steps 10 --warmup 2 --samples-per-gpu 32768
run s8k_h128_sg --steps 10 --warmup 2 --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10
run s64k_h128_sg --steps 5 --warmup 2 --samples-per-gpu 65536 --horizon-steps 128 --smoothing 10
run s4094 --steps 30 --warmup 3 --samples-per-gpu 4094
run s4080 --steps 30 --warmup 3 --samples-per-gpu 4080
