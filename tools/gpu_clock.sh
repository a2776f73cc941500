# effective clock of the rollout kernel at several wave counts (run via gpurun)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/clock
mkdir -p $D
for s in ${SWEEP:-1022 4094}; do
  timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $D -o s$s --output-format csv -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline --samples-per-gpu $s > $D/s$s.log 2>&1 || exit 1
  python3 tools/clock_probe.py $D s$s
done
