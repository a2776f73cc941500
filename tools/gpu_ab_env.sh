# A/B timing of gpurun_variants/* under each MPPI_FUSE_SAMPLE setting in $FUSE_SET (run via gpurun).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for rep in 1 2; do
for f in ${FUSE_SET:-0 1}; do
for d in gpurun_variants/*/; do
    n=$(basename $d)
    MPPI_FUSE_SAMPLE=$f MPPI_AMD_LIB=$PWD/$d/libmppi_amd.so timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab/$n.f$f.json 2> gpurun_out/ab/$n.f$f.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab/$n.f$f.json')); k=d['kernel_ms']; print('%-10s fuse=$f ms/update %.4f dyn %.4f cost %.4f' % ('$n', d['ms_per_step'], k['rollout_dynamics'], k['rollout_cost']))"
done; done; done
