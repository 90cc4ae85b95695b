# HBM-side traffic of the direct probe kernels per workload, as
# MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE and WRITE_SIZE in
# separate passes, FETCH_SIZE doubled on gfx950; plus the 128/64/32-B
# read-request split.  Since round 6 the banks are put on the direct / gather
# kernels with bench.py --probe-path direct (the species and genus defaults
# are the partitioned pipelines; MLST's compact banks have only this path),
# and only the full-size launches are profiled (--no-host-path --no-e2e).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/pmct
mkdir -p $P
for w in ${WORKLOADS:-species genus mlst}; do
  B="bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-host-path --no-e2e --probe-path direct"
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $P/$w/f -o run -- python $B > $P/$w.f.json 2> $P/$w.f.err || { tail -20 $P/$w.f.err; exit 30; }
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $P/$w/w -o run -- python $B > $P/$w.w.json 2> $P/$w.w.err || { tail -20 $P/$w.w.err; exit 31; }
  timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $P/$w/r -o run -- python $B > $P/$w.r.json 2> $P/$w.r.err || { tail -20 $P/$w.r.err; exit 32; }
  echo "done $w"
done
python3 tools/traffic_summary.py $P > gpurun_out/pmct/traffic.json
cat gpurun_out/pmct/traffic.json
rm -rf $P/*/
