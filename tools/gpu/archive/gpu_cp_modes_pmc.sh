# Lookup operating points: PMC of the default lookup (~6.4 ms) vs all 6 gathers in flight
# (LOOKUP 2, ~8.7 ms) and 4 workgroups per CU: L2 hit rate, HBM bytes, L2 requests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmcmodes; rm -rf $P; mkdir -p $P
B="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-path"
for cfg in "d:XSPECT2_AMD_CP_LOOKUP=0" "l2:XSPECT2_AMD_CP_LOOKUP=2" "c4:XSPECT2_AMD_CP_PERCU=4"; do
  lab=${cfg%%:*}; ev=${cfg#*:}; mkdir -p $P/$lab
  i=0
  for grp in "TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_TAG_STALL_sum"; do
    i=$((i+1))
    env $ev timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "cobs_lookup" --output-format csv -d $P/$lab/p$i -o run -- python3 $B > $P/$lab/p$i.json 2> $P/$lab/p$i.err || { tail -20 $P/$lab/p$i.err; exit 30; }
  done
  python3 tools/pmc_kernels.py $P/$lab "$lab" $P/$lab.json > /dev/null
  python3 - "$P/$lab.json" "$lab" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    print(sys.argv[2], k[:40], "hit %.3f" % v.get("l2_hit_rate", 0), "hbm %.2f GB" % (v.get("hbm_bytes", 0) / 1e9),
          "req %.3g" % v.get("TCC_REQ_sum", 0), "ea_rd %.3g" % v.get("TCC_EA0_RDREQ_sum", 0),
          "ea_wr %.3g" % v.get("TCC_EA0_WRREQ_sum", 0), "tagstall %.3g" % v.get("TCC_TAG_STALL_sum", 0),
          "gui %.3g" % v.get("GRBM_GUI_ACTIVE", 0))
PY
done
