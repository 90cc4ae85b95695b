# Parity of the classic cases, species A/B direct vs partitioned, trace, PMC.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu/gpu_cp_ab_short.sh && bash tools/gpu/gpu_cp_trace.sh && bash tools/gpu/gpu_cp_pmc.sh
