# wide classic banks (slot kernel) + MLST
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for kh in "21 7 300" "21 7 1000"; do
  set -- $kh
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --k $1 --hashes $2 --docs $3 --genome-len 1000000 > gpurun_out/kh_$1_$2_$3.json 2> gpurun_out/kh.err || { tail -20 gpurun_out/kh.err; exit 8; }
  python3 -c "import json;d=json.load(open('gpurun_out/kh_$1_$2_$3.json'));r=d['roofline'];print('k=$1 h=$2 D=$3: probe %.2f ms  %.0f GB/s frac %.3f  %.3e probes/s' % (r['probe_ms_avg'], r['achieved'], r['frac'], d['value']))"
done
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --workload mlst > gpurun_out/mlst.json 2> gpurun_out/kh.err || { tail -20 gpurun_out/kh.err; exit 9; }
python3 -c "import json;d=json.load(open('gpurun_out/mlst.json'));r=d['roofline'];print('mlst: probe %.2f ms step %.2f ms %.3e' % (r['probe_ms_avg'], d['ms_per_step'], d['value']))"
