# rbloom bucket pass changes (k-mer -> read map and one LDS atomic per index; then the closed-form LCG) against the previous
# commit's library (head), genus bench, interleaved, one box; rbloom parity subset first.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02bb2; mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "bloom or genus or single_filter or rbloom" > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 12; }
tail -2 $F/tests.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload genus --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2 3; do
  run head_$i XSPECT2_AMD_LIB_VARIANT=head
  run new_$i XSPECT2_AMD_CP_PAD=4
done
