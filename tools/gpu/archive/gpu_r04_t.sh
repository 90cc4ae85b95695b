# Round 4: config 3's per-GPU shard (12.5 M reads) end to end from a 3.9 GB
# FASTQ (bench.py's end_to_end legs at that size): windows reach the batch
# budget, so the per-call cost is spread over ~15 calls of 256 MiB.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04t; mkdir -p $F
timeout -k 10 900 python -u bench.py --reads 12500000 --steps 5 --warmup 2 --no-host-path --no-cpu-baseline > $F/config3_e2e.json 2> $F/config3_e2e.err || { tail -30 $F/config3_e2e.err; exit 12; }
python3 -c "
import json; d=json.loads([l for l in open('$F/config3_e2e.json') if l.startswith('{')][-1])
print(d['value'], d['roofline']['probe_ms_avg'], d['end_to_end']['file_bytes'], {k:(round(v['ms'],1), round(v['first_ms'],1)) for k,v in d['end_to_end'].items() if isinstance(v, dict)})"
