# Owner-map lookups as defaults: parity of both partitioned probes (and the old
# binary-search lookups), then species and genus bench lines interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03own2; mkdir -p $F
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -1 $F/parity.log
run() {  # label, workload, env...
  local lab=$1 wl=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --no-host-path --no-e2e > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));r=d['roofline'];print('$lab', round(d['ms_per_step'],3), round(r['probe_ms_avg'],3), {k: round(v,3) for k,v in r.get('pass_ms_avg',{}).items()})"
}
run g_base1 genus XSPECT2_AMD_BL_LOOKUP=0
run g_own1 genus XSPECT2_AMD_BL_LOOKUP=1
run g_base2 genus XSPECT2_AMD_BL_LOOKUP=0
run g_own2 genus XSPECT2_AMD_BL_LOOKUP=1
run s_base species XSPECT2_AMD_CP_LOOKUP=0
run s_own species
