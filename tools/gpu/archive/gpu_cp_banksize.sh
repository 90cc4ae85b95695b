# Direct vs partitioned COBS probe by bank size (species, D=100, 1M x 150 bp reads):
# genomes of 4e6 (614 MB bank), 2e6, 1e6, 4e5, 1e5 bp.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r02bank; mkdir -p $F
for g in 2000000 1000000 400000 100000; do
  for m in 0 2; do
    XSPECT2_AMD_COBS_PART=$m timeout -k 10 300 python bench.py --genome-len $g --steps 10 --warmup 3 --no-host-path --no-cpu-baseline > $F/g${g}_m$m.json 2> $F/g${g}_m$m.err || { tail -20 $F/g${g}_m$m.err; exit 13; }
    python3 -c "import json;d=json.load(open('$F/g${g}_m$m.json'));print('genome $g mode $m bank %.0f MB'%(d['config']['bank_device_bytes']/1e6), round(d['ms_per_step'],3), round(d['roofline']['probe_ms_avg'],3))"
  done
done
