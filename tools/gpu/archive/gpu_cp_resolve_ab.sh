# Resolve: the read search of the count phase moved into the first load pass (overlaps the rows in flight).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
F=gpurun_out/r02rsearch; rm -rf $F; mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "partitioned or mixed_streams or over_mall or degenerate or species_model_same" > $F/tests.log 2>&1 || { tail -40 $F/tests.log; exit 12; }
tail -2 $F/tests.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-host-path --no-cpu-baseline > $F/$lab.json 2> $F/$lab.err || { tail -20 $F/$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/$lab.json'));print('$lab', round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
}
for i in 1 2 3; do
  run head_$i XSPECT2_AMD_LIB_VARIANT=head
  run new_$i XSPECT2_AMD_CP_PAD=4
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$F/trace" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-host-path --no-cpu-baseline > "$R/$F/trace.log" 2>&1 || { tail -20 "$R/$F/trace.log"; exit 14; }
cd "$R" && python3 tools/kstats.py $F/trace/run_kernel_stats.csv | sed -n '2,4p'
