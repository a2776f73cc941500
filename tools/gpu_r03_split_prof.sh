#!/bin/bash
# rocprofv3 kernel stats of configs[4]'s share per GPU (8192 x 128, SG w = 10: the two-launch split)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r03sp
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --samples-per-gpu 8192 --horizon-steps 128 --smoothing 10 --steps 100 > $O/bench.json 2> $O/trace.err || { echo "trace rc=$?"; tail -5 $O/trace.err; exit 1; }
head -12 $O/trace/run_kernel_stats.csv
