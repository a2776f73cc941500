# Tail draws (run via gpurun): the draws-ahead / shard parity tests, then the whole GPU suite, then
# bench A/B of MPPI_TAIL_DRAWS=0 / 1 (three interleaved rounds) and a kernel trace of the default.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/tail
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "draws_ahead or shards or event_ring" --timeout 120 --timeout-method thread > gpurun_out/tail/pytest_draws.log 2>&1; rc=$?; tail -4 gpurun_out/tail/pytest_draws.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/tail/pytest_all.log 2>&1; rc=$?; tail -2 gpurun_out/tail/pytest_all.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
for f in 0 1; do
    MPPI_TAIL_DRAWS=$f timeout -k 10 120 python bench.py --steps 40 --warmup 3 --no-cpu-baseline > gpurun_out/tail/t$f.$rep.json 2> gpurun_out/tail/t$f.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/tail/t$f.$rep.json')); k=d['kernel_ms']; print('tail=$f ms/update %.4f dyn %.4f' % (d['ms_per_step'], k['rollout_dynamics']))"
done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/tail/tr -o run --output-format csv -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > /dev/null 2> gpurun_out/tail/tr.err || exit 1
python3 tools/trace_seq.py gpurun_out/tail/tr/run_kernel_trace.csv tail
