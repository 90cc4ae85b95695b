# L2 request rate of the rbloom lookup (TCC_REQ / TCC_HIT / TCC_MISS, one pass), genus bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmcbreq; rm -rf $P; mkdir -p $P
B="bench.py --workload genus --steps 3 --warmup 1 --no-cpu-baseline --no-host-path"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE --kernel-include-regex "bloom_lookup|bloom_bucket|bloom_resolve" --output-format csv -d $P/p1 -o run -- python3 $B > $P/p1.json 2> $P/p1.err || { tail -20 $P/p1.err; exit 30; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --kernel-include-regex "bloom_lookup" --output-format csv -d $P/t -o run -- python3 $B > $P/t.json 2> $P/t.err || { tail -20 $P/t.err; exit 31; }
python3 tools/pmc_kernels.py $P "genus lookup requests" $P/pmc.json > /dev/null
python3 - <<'PY'
import json, csv
d = json.load(open("gpurun_out/pmcbreq/pmc.json"))
st = {r["Name"]: float(r["AverageNs"]) for r in csv.DictReader(open("gpurun_out/pmcbreq/t/run_kernel_stats.csv"))}
for k, v in d["kernels"].items():
    print(k[:40], "req %.4g hit %.3f gui %.4g" % (v.get("TCC_REQ_sum", 0), v.get("l2_hit_rate", 0), v.get("GRBM_GUI_ACTIVE", 0)))
for n, ns in st.items():
    print(n[:60], "%.3f ms" % (ns / 1e6))
PY
