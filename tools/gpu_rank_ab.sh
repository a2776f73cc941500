# Rank-tile split A/B (run via gpurun): the stable-order / draws-ahead parity tests on each
# gpurun_variants/js* build, then bench rounds and a kernel trace per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rk
for n in js2 js4; do
    MPPI_AMD_LIB=$PWD/gpurun_variants/$n/libmppi_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "draws_ahead or stable_order or config3 or shards" --timeout 120 --timeout-method thread > gpurun_out/rk/pytest_$n.log 2>&1; rc=$?; echo "$n: $(tail -1 gpurun_out/rk/pytest_$n.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2 3; do
for n in js1 js2 js4; do
    MPPI_AMD_LIB=$PWD/gpurun_variants/$n/libmppi_amd.so timeout -k 10 120 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/rk/$n.$rep.json 2> gpurun_out/rk/$n.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/rk/$n.$rep.json')); k=d['kernel_ms']; print('$n ms/update %.4f dyn %.4f' % (d['ms_per_step'], k['rollout_dynamics']))"
done
done
for n in js1 js2 js4; do
    MPPI_AMD_LIB=$PWD/gpurun_variants/$n/libmppi_amd.so timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/rk/tr_$n -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/rk/tr_$n.err || exit 1
    python3 tools/trace_seq.py gpurun_out/rk/tr_$n/run_kernel_trace.csv $n | grep "rank_draw_kernel  \|dur rank\|period"
done
