# Partitioned COBS probe: bank partition size (XSPECT2_AMD_CP_SHIFT = log2 rows: 16 = 1 MiB,
# 17 = 2 MiB default, 18 = 4 MiB) x bucket block (CK), interleaved, one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02shift; mkdir -p $F
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2; do
  run s17_$i XSPECT2_AMD_CP_SHIFT=17
  run s16_$i XSPECT2_AMD_CP_SHIFT=16
  run s18_$i XSPECT2_AMD_CP_SHIFT=18
  run s16ck4096_$i XSPECT2_AMD_CP_SHIFT=16 XSPECT2_AMD_CP_CK=4096
  run s17ck4096_$i XSPECT2_AMD_CP_SHIFT=17 XSPECT2_AMD_CP_CK=4096
done
