# Round 5: bank payloads streamed from their files (pread by 8 threads into a
# pinned ring, DMA per piece) instead of vector + ifstream + pageable copy:
# the model-load probe, then the whole GPU suite (open / open_docs / saved
# files are covered there).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r05q; mkdir -p $F
timeout -k 10 300 python3 tools/open_probe.py > $F/open2.json 2> $F/open2.err || { tail -20 $F/open2.err; exit 10; }
cat $F/open2.json
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $F/gpu_tests.log 2>&1 || { tail -40 $F/gpu_tests.log; exit 11; }
tail -2 $F/gpu_tests.log
