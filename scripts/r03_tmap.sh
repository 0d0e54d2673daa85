#!/bin/bash
# conv3 x9 tile-map LDS layout vs the rotation swizzle (build_ab/tmap0.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_learner_full_gpu.py tests/test_fused_learner_gpu.py > gpurun_out/tm.log 2>&1; tail -n 2 gpurun_out/tm.log
export CONV_NS=256,512,768,1024
for v in tmap tmap0 tmap; do
  lib=""; [ $v = tmap0 ] && lib=build_ab/tmap0.so
  RTH_LIB_PATH=$lib timeout -k 10 200 python -u scripts/bench_conv.py 2>&1 | grep conv3 | sed "s/^/$v /"
done
BENCH_ARGS=--no-sweep bash scripts/ab_env.sh 3 300 "tmap" "tmap0 RTH_LIB_PATH=build_ab/tmap0.so"
