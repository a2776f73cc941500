# Host turnaround stamps (MPPI_HOST_TRACE=1, printed at destroy) around a bench run (run via gpurun).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ht
for rep in 1 2; do
MPPI_HOST_TRACE=1 timeout -k 10 120 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/ht/bench.$rep.json 2> gpurun_out/ht/bench.$rep.err || exit 1
python -c "import json; d=json.load(open('gpurun_out/ht/bench.$rep.json')); print('ms/update %.4f dyn %.4f' % (d['ms_per_step'], d['kernel_ms']['rollout_dynamics']))"
cat gpurun_out/ht/bench.$rep.err
done
