# Round 4: the device reader's timeline with entry / return / prefetch marks
# (end-to-end legs of the config-2 reads), and the genus bench line with its
# lookup_l2 from profiles/r04_pmc_bloompart.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04b; mkdir -p $F
timeout -k 10 300 python -u tools/fx_dev_trace.py --bank --reads 1000000 --batch-mb 256 > $F/fxtrace.json 2> $F/fxtrace.err || { tail -30 $F/fxtrace.err; exit 20; }
cat $F/fxtrace.json
timeout -k 10 600 python -u bench.py --workload genus --no-e2e > $F/genus.json 2> $F/genus.err || { tail -30 $F/genus.err; exit 13; }
cut -c1-400 $F/genus.json
