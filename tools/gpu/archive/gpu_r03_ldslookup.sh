# LDS-resident fine partitions vs today's L2-resident partitions for the COBS
# lookup, on synthetic config-2-shaped entries (tools/ldslookup.hip).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ldsl
timeout -k 10 240 ./tools/ldslookup ${LDSL_ARGS:-} > gpurun_out/ldsl/out.txt 2>&1 || { cat gpurun_out/ldsl/out.txt; exit 5; }
cat gpurun_out/ldsl/out.txt
