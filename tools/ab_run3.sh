# A/B timing (run via gpurun): the HBM-records path against the objective inside the rollout launch
# (MPPI_COST_KERNEL=fused), same library, two rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
one() {   # name [VAR=value]
    local n=$1
    env $2 timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || return 1
    python -c "import json; d=json.load(open('gpurun_out/ab/$n.json')); k=d['kernel_ms']; b=k['breakdown_untimed']; print('%-6s ms/update %.4f rollout %.4f cost %.4f sample %.4f reduce %.4f' % ('$n', d['ms_per_step'], k['rollout_dynamics'], k['rollout_cost'], b['sample'], b['reduce']))"
}
for r in 1 2; do
    one rec$r && one fused$r MPPI_COST_KERNEL=fused || exit 1
done
