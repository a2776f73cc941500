# A/B (run via gpurun): gradient-split variants under gpurun_variants/ with bench.py, and the
# round's previous bench loop (tools/bench_prev.py: timing events read inside the loop) on base,
# alternating, three rounds; then parity tests on the gs16 variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gs
for rep in 1 2 3; do
for n in base gs16 gs32 prev; do
    lib=gpurun_variants/$n/libmppi_amd.so; b=bench.py
    [ $n = prev ] && lib=gpurun_variants/base/libmppi_amd.so && b=tools/bench_prev.py
    PYTHONPATH=$PWD MPPI_AMD_LIB=$PWD/$lib timeout -k 10 120 python $b --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/gs/$n.$rep.json 2> gpurun_out/gs/$n.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/gs/$n.$rep.json')); k=d['kernel_ms']; print('%-6s ms/update %.4f dyn %.4f reduce %.4f' % ('$n', d['ms_per_step'], k['rollout_dynamics'], k['breakdown_untimed']['reduce']))"
done
done
MPPI_AMD_LIB=$PWD/gpurun_variants/gs16/libmppi_amd.so timeout -k 10 300 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gs/pytest_gs16.log 2>&1; rc=$?; tail -2 gpurun_out/gs/pytest_gs16.log; exit $rc
