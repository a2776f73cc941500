# Kernel-trace each built variant (run via gpurun): per-kernel average durations per variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/abp
for d in gpurun_variants/*/; do
    n=$(basename $d)
    MPPI_AMD_LIB=$PWD/$d/libmppi_amd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abp/$n -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/abp/$n.json 2> gpurun_out/abp/$n.err || exit 1
    python3 tools/trace_gaps.py gpurun_out/abp/$n/run_kernel_trace.csv "$n" || exit 1
done
