#!/bin/bash
# build_variant.sh NAME "EXTRA FLAGS" — in-tree variant library for A/B runs
set -e
name=$1; extra=$2
cd /root/repo/xspect2_amd
mkdir -p _build/$name
for f in csrc/xs_probe_wide.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -Wno-pass-failed -Wno-unused-result -I ../include $extra -c $f -o _build/$name/$(basename $f).o
done
objs=""
for o in _build/*.o; do b=$(basename $o); if [ -f _build/$name/$b ]; then objs="$objs _build/$name/$b"; else objs="$objs $o"; fi; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o libxspect_hip.$name.so $objs
echo built libxspect_hip.$name.so
