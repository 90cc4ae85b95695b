# Direct vs partitioned COBS probe at small batches (species bank, 614 MB): where is the crossover?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02small; mkdir -p $F
for r in 2000 10000 30000 100000 300000; do
  for m in 0 2; do
    XSPECT2_AMD_COBS_PART=$m timeout -k 10 300 python bench.py --reads $r --steps 20 --warmup 5 --no-cpu-baseline --no-host-path > $F/r${r}_m$m.json 2> $F/r${r}_m$m.err || { tail -20 $F/r${r}_m$m.err; exit 13; }
    python3 -c "import json;d=json.load(open('$F/r${r}_m$m.json'));print('reads $r mode $m', round(d['ms_per_step'],4), round(d['roofline']['probe_ms_avg'],4))"
  done
done
