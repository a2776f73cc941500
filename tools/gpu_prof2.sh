# kernel-trace stats at 4096 and 32768 samples per GPU (run via gpurun from the repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof4k -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench4k.json 2> gpurun_out/bench4k.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof32k -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --samples-per-gpu 32768 > gpurun_out/bench32k.json 2> gpurun_out/bench32k.err && echo ok
