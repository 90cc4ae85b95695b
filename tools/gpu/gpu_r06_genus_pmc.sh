# Round 6: the new GPU tests (per-handle probe options, doc-slice staging,
# atomic saves) after the prefetch removal; then the partitioned rbloom
# (genus) pipeline's PMC at HEAD, one counter group per
# pass -> gpurun_out/pmc06g/pmc.json (-> profiles/r06_pmc_bloompart.json),
# and the genus bench line with per-pass times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r06b; mkdir -p $F
timeout -k 10 300 python -u -m pytest tests/test_gpu_probe_options.py tests/test_gpu_bank_files.py tests/test_gpu_doc_slices.py -x -q --timeout 200 --timeout-method thread > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 11; }
tail -1 $F/tests.log
P=gpurun_out/pmc06g
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
python3 tools/pmc_kernels.py $P "genus, partitioned rbloom at round-6 HEAD" $P/pmc.json > /dev/null
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/pmc06g/pmc.json"))
for k, v in d["kernels"].items():
    hb = v.get("hbm_bytes", 0) / 1e9
    print(f"{k[:48]:48s} hbm {hb:6.2f} GB  req {v.get('TCC_REQ_sum', 0):.4g}  l2hit {v.get('l2_hit_rate', 0):.3f}  TCP_pend {v.get('TCP_PENDING_STALL_CYCLES_sum', 0):.3g}")
print("hbm_bytes_per_step", d["hbm_bytes_per_step"] / 1e9)
PY
timeout -k 10 300 python -u bench.py --workload genus --no-host-path > $F/genus.json 2> $F/genus.err || { tail -30 $F/genus.err; exit 13; }
python3 -c "import json; d=json.loads(open('$F/genus.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], d['checks']['ok'], r['probe_ms_avg'], r.get('pass_ms_avg'), r.get('frac'), r.get('traffic_frac'))"
