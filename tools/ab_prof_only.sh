# kernel-trace A/B of gpurun_variants/* (no tests); run via gpurun
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_prof.sh
