# Round-4 PMC passes over the partitioned rbloom (genus) pipeline: traffic
# (FETCH_SIZE, WRITE_SIZE), L2 requests / hit rate, and the shader-side
# counters, one group per pass -> gpurun_out/pmc04g/pmc.json (bench.py reads
# profiles/r04_pmc_bloompart.json for the genus line's lookup_l2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmc04g
rm -rf $P; mkdir -p $P
B="bench.py --workload genus --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-e2e"
RX="bloom_|part_"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "$RX" --output-format csv -d $P/p$i -o run -- python3 $B > $P/p$i.json 2> $P/p$i.err || { tail -20 $P/p$i.err; exit 30; }
done
python3 tools/pmc_kernels.py $P "genus, partitioned rbloom at round-4 HEAD" $P/pmc.json > /dev/null
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/pmc04g/pmc.json"))
for k, v in d["kernels"].items():
    hb = v.get("hbm_bytes", 0) / 1e9
    print(f"{k[:48]:48s} hbm {hb:6.2f} GB  req {v.get('TCC_REQ_sum', 0):.4g}  l2hit {v.get('l2_hit_rate', 0):.3f}  TCP_pend {v.get('TCP_PENDING_STALL_CYCLES_sum', 0):.3g}")
print("hbm_bytes_per_step", d["hbm_bytes_per_step"] / 1e9)
PY
