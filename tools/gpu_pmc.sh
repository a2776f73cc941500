# PMC passes for the update's kernels (run via gpurun from the repo root).  One counter group per
# pass (TCC FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
D=gpurun_out/pmc
mkdir -p $D
B="python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline"
run() {   # name counters...
    local n=$1; shift
    timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-trace -d $D -o $n --output-format csv -- $B > $D/$n.log 2>&1
}
run sq SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_ANY && \
run lat SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
run flops SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL && \
run fetch FETCH_SIZE GRBM_GUI_ACTIVE && \
run write WRITE_SIZE && \
for n in sq lat flops fetch write; do python3 tools/pmc_summary.py $D/${n}_counter_collection.csv > $D/${n}_summary.txt; done && \
cat $D/*_summary.txt | grep -E 'coop|step_cost|sample_kernel|rank_|gradient|finish'
