# Resolve: rows in flight per lane (XSPECT2_AMD_CP_RU 4 / 8 default / 12 / 16), interleaved, with a trace of each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02ru; mkdir -p $F
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2; do
  run ru8_$i XSPECT2_AMD_CP_RU=8
  run ru12_$i XSPECT2_AMD_CP_RU=12
  run ru16_$i XSPECT2_AMD_CP_RU=16
  run ru4_$i XSPECT2_AMD_CP_RU=4
done
