#!/bin/bash
# A/B variant of the library: the product sources with extra -D flags, into
# reth_amd/libreth_hip_<name>.so (git-ignored; loaded through RTH_LIB_PATH, never by default)
#   scripts/build_variant_lib.sh wg128 -DCONV_WG_BLOCKS=128
set -eu
cd "$(dirname "$0")/.."
name=$1; shift
ID=$(python -c "from reth_amd import _lib; print(_lib.source_build_id())")
SRCS=$(python -c "import __graft_entry__ as g, os; print(' '.join(os.path.join('reth_amd/csrc', s) for s in g.HIP_SOURCES))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Wall -Xclang -target-feature -Xclang -packed-fp32-ops "$@" \
    -DRTH_BUILD_ID="\"$ID\"" -o "reth_amd/libreth_hip_$name.so" $SRCS
echo "built reth_amd/libreth_hip_$name.so ($*)"
