set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof32k -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --samples-per-gpu 32768 > gpurun_out/bench32k.json 2> gpurun_out/bench32k.err && echo ok
