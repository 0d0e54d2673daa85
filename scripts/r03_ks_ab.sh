#!/bin/bash
# x9 K-part variants (build_ab/*.so from scripts/build_variants.sh): conv tests, microbench, loop A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in c3ks3 c2ks4; do
  RTH_LIB_PATH=build_ab/$v.so timeout -k 10 300 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k "not impl" > gpurun_out/t_$v.log 2>&1
  echo "$v tests: $(tail -n 1 gpurun_out/t_$v.log)"
done
export CONV_NS=256,512,768,1024
for v in default c3ks3 c2ks2 c2ks4; do
  lib=""; [ $v != default ] && lib=build_ab/$v.so
  RTH_LIB_PATH=$lib timeout -k 10 200 python -u scripts/bench_conv.py 2>&1 | grep -v "conv1\|amdgpu" | sed "s/^/$v /"
done
BENCH_ARGS=--no-sweep bash scripts/ab_env.sh 2 200 "default" "c3ks3 RTH_LIB_PATH=build_ab/c3ks3.so"
