#!/bin/bash
# k_conv_dgrad prefetch depth / waves per workgroup variants: alone, then in the loop
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base dgD8 dgD2 dgW4; do
  echo "== $v"; RTH_LIB_PATH=$PWD/build_ab/$v.so timeout -k 10 200 python scripts/bench_dgrad.py 2>&1 | grep "32x20x20" || exit 1
done
scripts/ab_bench.sh ${ROUNDS:-3} ${STEPS:-500} build_ab/base.so build_ab/dgD8.so build_ab/dgW4.so build_ab/dgD2.so
