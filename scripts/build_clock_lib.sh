#!/bin/bash
# the diagnostic library for scripts/conv_clock.py: the product sources built with
# -DRTH_CLOCK_STAMPS (k_conv_bias_relu stamps its in-kernel clock) into
# reth_amd/libreth_hip_clk.so (git-ignored; loaded through RTH_LIB_PATH, never by default)
set -eu
cd "$(dirname "$0")/.."
ID=$(python -c "from reth_amd import _lib; print(_lib.source_build_id())")
SRCS=$(python -c "import __graft_entry__ as g, os; print(' '.join(os.path.join('reth_amd/csrc', s) for s in g.HIP_SOURCES))")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -Wall -Xclang -target-feature -Xclang -packed-fp32-ops -DRTH_CLOCK_STAMPS \
    -DRTH_BUILD_ID="\"$ID\"" -o reth_amd/libreth_hip_clk.so $SRCS
echo built reth_amd/libreth_hip_clk.so
