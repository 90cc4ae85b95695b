set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmc2
mkdir -p $P
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $P/p1 -o run -- python $B > $P/p1.json 2> $P/p1.err || { tail -20 $P/p1.err; exit 30; }
timeout -k 10 400 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $P/p2 -o run -- python $B > $P/p2.json 2> $P/p2.err || { tail -20 $P/p2.err; exit 31; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $P/p3 -o run -- ./tools/randgather 16 614 > $P/p3.json 2> $P/p3.err || { tail -20 $P/p3.err; exit 32; }
python3 tools/pmc_summary.py $P probe_cobs_fast
echo "-- randgather"
python3 - <<'PY'
import csv, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/pmc2/p3/run_counter_collection.csv")):
    agg[(r["Kernel_Name"][:30], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k, len(v), [f"{x:.4g}" for x in v[:8]])
PY
