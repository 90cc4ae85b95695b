# Lookup mix with the HBM read and write streams separated in time (tools/phasemix.hip)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/phase
timeout -k 10 120 ./tools/phasemix > gpurun_out/phase/phasemix.txt 2>&1 || { cat gpurun_out/phase/phasemix.txt; exit 5; }
cat gpurun_out/phase/phasemix.txt
