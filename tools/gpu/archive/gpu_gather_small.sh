# random 16-B row gather rate vs table size, incl. L2-resident tables (4 MB L2 per XCD)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 ./tools/randgather 0.5 1 2 3 4 8 16 32 64 128 256 614 > gpurun_out/randgather_small.json
python3 -c "
import json
d=json.load(open('gpurun_out/randgather_small.json'))
for r in d['results']:
    if r['alloc']=='hipMalloc': print('%7.1f MB %-6s %6.1f G rows/s' % (r['table_MB'], r['policy'], r['Grows_per_s']))
"
