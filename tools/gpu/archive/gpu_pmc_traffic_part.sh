# HBM-side traffic of the partitioned rbloom pipeline (all its kernels, per query), as
# MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE and WRITE_SIZE in separate passes,
# FETCH_SIZE doubled on gfx950.  Full-size launches only (--no-host-path).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmcp
rm -rf $P; mkdir -p $P
B="bench.py --workload genus --steps 3 --warmup 1 --no-cpu-baseline --no-host-path"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "bloom_|part_" --output-format csv -d $P/f -o run -- python3 $B > $P/f.json 2> $P/f.err || { tail -20 $P/f.err; exit 30; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "bloom_|part_" --output-format csv -d $P/w -o run -- python3 $B > $P/w.json 2> $P/w.err || { tail -20 $P/w.err; exit 31; }
python3 - <<'PY'
import collections, csv, glob, json
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmcp/*/run_counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')
        if 'build_' in name:
            continue
        agg[name][r['Counter_Name']].append(float(r['Counter_Value']))
per = {}
for k, c in agg.items():
    if 'FETCH_SIZE' in c and 'WRITE_SIZE' in c:
        f = sum(c['FETCH_SIZE']) / len(c['FETCH_SIZE']); w = sum(c['WRITE_SIZE']) / len(c['WRITE_SIZE'])
        per[k] = {'dispatches': len(c['FETCH_SIZE']), 'FETCH_SIZE': f, 'WRITE_SIZE': w, 'hbm_bytes': (2 * f + w) * 1024}
bench = json.loads(open('gpurun_out/pmcp/f.json').read().strip().splitlines()[-1])
out = {'workload': 'genus (partitioned rbloom pipeline)', 'reads': bench['config']['reads_per_gpu'],
       'kernels': per, 'hbm_bytes_per_step': sum(v['hbm_bytes'] for v in per.values()),
       'source': 'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, --kernel-include-regex "bloom_|part_", per-dispatch averages summed over the pipeline; (2*FETCH_SIZE + WRITE_SIZE) KB'}
print(json.dumps(out, indent=1))
json.dump(out, open('gpurun_out/pmcp/traffic_part.json', 'w'), indent=1)
PY
