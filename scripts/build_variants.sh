#!/bin/bash
# build libreth_hip.so variants for kernel A/B runs: build_ab/<name>.so from -D flags (build_ab/
# travels to the GPU box, unlike build/; delete it when the A/B is done)
# usage: scripts/build_variants.sh name1 "-DFLAG=1 ..." name2 "..."
set -e
cd "$(dirname "$0")/.."
out=${VARIANT_DIR:-build_ab}; mkdir -p $out
srcs=$(python -c "import __graft_entry__ as g; print(' '.join('reth_amd/csrc/' + s for s in g.HIP_SOURCES))")
pids=()
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Xclang -target-feature -Xclang -packed-fp32-ops $2 -o $out/$1.so $srcs &
  pids+=($!)
  shift 2
done
for p in "${pids[@]}"; do wait $p; done
ls -la $out
