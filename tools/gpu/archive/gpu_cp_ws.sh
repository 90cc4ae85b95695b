# Partitioned COBS probe in workspace-bounded block ranges: parity, then the
# species step at workspace caps of 24 GiB (1 range), 8 GiB (3), 4 GiB (6),
# 1 GiB (21), and 4M reads per step (84 GB of entries -> 4 ranges of 24 GiB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02ws; mkdir -p $F
echo "== parity"; timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py -k "classic or mixed_streams or over_mall" > $F/parity.log 2>&1 || { tail -40 $F/parity.log; exit 12; }
tail -1 $F/parity.log
run() {  # label, args, env...
  local lab=$1; local a=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-host-path $a > $F/ab_$lab.json 2> $F/ab_$lab.err || { tail -20 $F/ab_$lab.err; exit 13; }
  python3 -c "import json;d=json.load(open('$F/ab_$lab.json'));c=d['cpu_baseline'] or {};print('$lab', '%.4g'%d['value'], round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3), 'mism', c.get('parity_sample_mismatches'))"
}
run ws24g "--no-cpu-baseline" XSPECT2_AMD_CP_WS_MB=24576
run ws8g "--no-cpu-baseline" XSPECT2_AMD_CP_WS_MB=8192
run ws4g "--no-cpu-baseline" XSPECT2_AMD_CP_WS_MB=4096
run ws1g "--no-cpu-baseline" XSPECT2_AMD_CP_WS_MB=1024
run reads4m "--reads 4000000 --steps 5 --warmup 2 --no-cpu-baseline" XSPECT2_AMD_CP_WS_MB=24576
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > $F/host.json 2> $F/host.err || { tail -20 $F/host.err; exit 14; }
python3 -c "import json;d=json.load(open('$F/host.json'));print('host_path', json.dumps(d['host_path']))"
