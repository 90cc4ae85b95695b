# Round 4: fixed cost of a probe call vs its size (tools/probe_sizes.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
F=gpurun_out/r04g; mkdir -p $F
timeout -k 10 300 python -u tools/probe_sizes.py > $F/sizes.json 2> $F/sizes.err || { tail -30 $F/sizes.err; exit 20; }
grep -v amdgpu $F/sizes.err | tail -8
