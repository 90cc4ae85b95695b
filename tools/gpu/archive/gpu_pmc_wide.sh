# PMC comparison of the narrow (D=100) and wide (D=1000) probes on equal-size (1.23 GB) banks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmcw
mkdir -p $P
timeout -k 10 120 rocprofv3 -L > $P/counters.txt 2>&1 || true
grep -o "TCP_UTCL1[A-Z_]*\|TCP_TCC_READ_REQ[A-Z_]*\|TCC_EA0_RDREQ[A-Z0-9_]*\|TA_BUSY[a-z_]*\|TCP_PENDING[A-Z_]*\|TCC_TAG_STALL[A-Z_]*" $P/counters.txt | sort -u | tr '\n' ' '; echo
i=0
for cfg in "--docs 100 --genome-len 8000000" "--docs 1000 --genome-len 1000000"; do
  i=$((i+1))
  B="bench.py --steps 2 --warmup 1 --no-cpu-baseline --totals-only $cfg"
  j=0
  for ctr in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_HIT_sum TCC_MISS_sum" \
             "TCP_TCC_READ_REQ_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_PENDING_STALL_CYCLES_sum" \
             "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU" \
             "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum"; do
    j=$((j+1))
    echo "== cfg$i pass$j: $ctr"
    timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $P/c${i}_p$j -o run -- python $B > $P/c${i}_p$j.json 2> $P/c${i}_p$j.err || { tail -5 $P/c${i}_p$j.err; echo "pass failed"; }
  done
done
python3 - <<'PY'
import collections, csv, glob
for i in (1, 2):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/pmcw/c{i}_p*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "probe_cobs" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"-- cfg{i}")
    for k, v in sorted(agg.items()):
        print(f"{k:40s} n={len(v):2d} avg={sum(v) / len(v):.4g}")
PY
