#!/bin/bash
# conv2 / conv3 forward: fp32-MFMA vs the default hybrid (x9 where it is faster) per batch size
# (bench_conv.py per process; the switch points are process-wide env knobs)
mkdir -p gpurun_out
export CONV_NS=${CONV_NS:-128,256,384,512,640,768,1024}
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 240 python -u scripts/bench_conv.py > gpurun_out/x9sweep_$tag.log 2>&1 || return 1
  echo "== $tag"; grep -v "conv1\|amdgpu.ids" gpurun_out/x9sweep_$tag.log
}
run f32 RTH_CONV_F32MFMA=1 &&
run hybrid RTH_X9_WG_PER_CU=1 &&
run x9all RTH_CONV2_X9_MAX=100000
