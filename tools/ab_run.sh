# Time each built variant (run via gpurun): bench line per variant, rollout kernel ms.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for d in gpurun_variants/*/; do
    n=$(basename $d)
    MPPI_AMD_LIB=$PWD/$d/libmppi_amd.so timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/$n.json')); k=d['kernel_ms']; print('%-12s ms/update %.4f dyn %.4f cost %.4f' % ('$n', d['ms_per_step'], k['rollout_dynamics'], k['rollout_cost']))"
done
