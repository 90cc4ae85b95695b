# Packed ids in the file predictions: the whole GPU suite, then the end-to-end
# benchmark (classify leg: predict_columnar + save of 1 M reads).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r03ids; mkdir -p $F
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/all.log 2>&1 || { tail -40 $F/all.log; exit 12; }
tail -2 $F/all.log
timeout -k 10 800 python -u tools/bench_e2e.py --reads 1000000 --dir /tmp/e2e > $F/e2e.json 2> $F/e2e.err || { tail -20 $F/e2e.err; exit 13; }
python -c "import json; d=json.load(open('$F/e2e.json')); print({k: v for k, v in d.items() if k.startswith(('classify', 'e2e_dev', 'dparse', 'json', 'pipeline'))})"
