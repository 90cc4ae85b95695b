# Resolve: first-round blocks staggered (s_sleep loops of ~3.4 us x k x S for the k-th block on a
# CU) so that co-resident blocks run their load and count phases out of step; interleaved A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02stagger; rm -rf $F; mkdir -p $F
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2; do
  run s0_$i XSPECT2_AMD_CP_STAGGER=0
  run s1_$i XSPECT2_AMD_CP_STAGGER=1
  run s3_$i XSPECT2_AMD_CP_STAGGER=3
  run s5_$i XSPECT2_AMD_CP_STAGGER=5
done
