# Lookup mix with narrower row stores (rows packed to 14 / 12 B), tools/l2gather.hip
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/l2p
timeout -k 10 120 ./tools/l2gather p > gpurun_out/l2p/packed.txt 2>&1 || { cat gpurun_out/l2p/packed.txt; exit 5; }
cat gpurun_out/l2p/packed.txt
