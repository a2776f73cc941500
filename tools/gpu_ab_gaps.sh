# A/B of the variants under gpurun_variants/ (run via gpurun): a bench line and a kernel trace
# per variant, then the per-update kernel durations and the gaps between them (trace_seq.py).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/abg
for rep in 1 2; do
for d in gpurun_variants/*/; do
    n=$(basename $d)
    MPPI_AMD_LIB=$PWD/$d/libmppi_amd.so timeout -k 10 120 python bench.py --steps 40 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/abg/$n.$rep.json 2> gpurun_out/abg/$n.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/abg/$n.$rep.json')); k=d['kernel_ms']; print('%-8s ms/update %.4f dyn %.4f' % ('$n', d['ms_per_step'], k['rollout_dynamics']))"
done
done
for d in gpurun_variants/*/; do
    n=$(basename $d)
    MPPI_AMD_LIB=$PWD/$d/libmppi_amd.so timeout -k 10 180 rocprofv3 --kernel-trace -d gpurun_out/abg/tr_$n -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/abg/tr_$n.err || exit 1
    python3 tools/trace_seq.py $(ls gpurun_out/abg/tr_$n/*/run_kernel_trace.csv gpurun_out/abg/tr_$n/run_kernel_trace.csv 2>/dev/null | head -1) $n
done
