# One GPU call (via gpurun): parity tests, A/B (tools/ab_run3.sh), PMC passes and the rollout
# launch's HBM traffic, smoke, the bench line and its kernel-trace profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/t gpurun_out/o
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/t/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/t/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_run3.sh || exit 1
bash tools/gpu_pmc.sh > gpurun_out/o/pmc.log 2>&1 || { tail -5 gpurun_out/o/pmc.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc gpurun_out/o/r01o_pmc_rollout.json > /dev/null && cp gpurun_out/o/r01o_pmc_rollout.json profiles/ || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/o/smoke.log 2>&1 && tail -1 gpurun_out/o/smoke.log || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/o/bench.json 2> gpurun_out/o/bench.err && cat gpurun_out/o/bench.json || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/o/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/o/bench_prof.json 2> gpurun_out/o/prof.err && echo prof ok
