# Which part of the lookup mix costs its rate: gathers+stores, entry loads+gathers, prefetched entries (tools/l2gather.hip m)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/l2p
timeout -k 10 120 ./tools/l2gather m > gpurun_out/l2p/parts.txt 2>&1 || { cat gpurun_out/l2p/parts.txt; exit 5; }
cat gpurun_out/l2p/parts.txt
