# MLST after moving compact loci to the wide kernel: bench line with CPU
# baseline, kernel trace, and the PMC traffic passes for the mlst workload.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu/gpu_mlst.sh || exit $?
WORKLOADS=mlst bash tools/gpu/gpu_pmc_traffic.sh > gpurun_out/pmct_mlst.log 2>&1 || { tail -20 gpurun_out/pmct_mlst.log; exit 20; }
tail -20 gpurun_out/pmct_mlst.log
