# rocprofv3 kernel-trace stats of one bench case (run via gpurun): tools/gpu_prof_case.sh name bench-args...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
n=$1; shift
mkdir -p gpurun_out/prof_$n
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > gpurun_out/prof_$n/bench.json 2> gpurun_out/prof_$n/err.log || exit 1
f=$(find gpurun_out/prof_$n -name 'run_kernel_stats.csv' | head -1)
python3 -c "
import csv,sys
for x in csv.DictReader(open('$f')): print('%-60s %6s %10.1f us %6.2f%%' % (x['Name'][:60], x['Calls'], float(x['AverageNs'])/1e3, float(x['Percentage'])))
"
