set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/gather
mkdir -p $P
timeout -k 10 240 ./tools/randgather 64 614 4096 > $P/rates.json 2> $P/rates.err || { cat $P/rates.err; exit 3; }
grep table_MB $P/rates.json
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $P/pmc -o run -- ./tools/randgather 614 > $P/pmc.json 2> $P/pmc.err || { tail -20 $P/pmc.err; exit 32; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/gather/pmc/run_counter_collection.csv")))
agg = collections.OrderedDict()
for r in rows:
    if "gather" not in r["Kernel_Name"]:
        continue
    key = (int(r["Dispatch_Id"]), r["Kernel_Name"][:22])
    agg.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {c.replace("TCC_EA0_RDREQ", ""): f"{x:.3g}" for c, x in sorted(v.items())})
PY
