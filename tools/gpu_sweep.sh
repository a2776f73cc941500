# rollout-kernel time vs samples per GPU (run via gpurun from the repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
for s in ${SWEEP:-2048 4090 4094 4096 6142 8192}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --samples-per-gpu $s > gpurun_out/sweep/s$s.json 2>gpurun_out/sweep/s$s.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sweep/s$s.json')); k=d['kernel_ms']; print($s, 'ms/update %.3f rollout %.3f optimal %.3f sample %.3f reduce %.3f' % (d['ms_per_step'], k['rollout'], k['optimal_rollout'], k['sample'], k['reduce']))"
done
