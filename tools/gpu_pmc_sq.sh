# SQ issue/stall counters for the update's kernels (run via gpurun from the repo root)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/pmcsq
mkdir -p $D
B="python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline"
run() {   # name counters...
    local n=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d $D -o $n --output-format csv -- $B > $D/$n.log 2>&1
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY && \
run st SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
for n in sq st; do python3 tools/pmc_summary.py $D/${n}_counter_collection.csv > $D/${n}_summary.txt; done && \
cat $D/*_summary.txt | grep -E 'coop'
