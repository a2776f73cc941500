# Phase traces (PHASE_TRACE builds under gpurun_variants/phase*) and A/B timing of the others.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/phase
for d in gpurun_variants/phase*/; do
    n=$(basename $d)
    rm -f gpurun_out/phase/$n.bin
    MPPI_WAVE_TRACE=$PWD/gpurun_out/phase/$n.bin MPPI_AMD_LIB=$PWD/$d/libmppi_amd.so timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/phase/$n.json 2> gpurun_out/phase/$n.err || exit 1
    echo "== $n"; case $n in *fk*) m=fk;; *) m=;; esac; python3 tools/phase_trace.py gpurun_out/phase/$n.bin 1026 $m || exit 1
done
mkdir -p gpurun_out/ab
for d in gpurun_variants/*/; do
    n=$(basename $d)
    case $n in phase*) continue;; esac
    MPPI_AMD_LIB=$PWD/$d/libmppi_amd.so timeout -k 10 120 python bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/ab/$n.json 2> gpurun_out/ab/$n.err || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab/$n.json')); k=d['kernel_ms']; print('%-12s ms/update %.4f dyn %.4f cost %.4f' % ('$n', d['ms_per_step'], k['rollout_dynamics'], k['rollout_cost']))"
done
