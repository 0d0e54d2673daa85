#!/bin/bash
# conv3 channel-split A/B (build/variants/c3ns{1,2,4}.so from scripts/build_variants.sh):
# parity of each variant (conv + fused learner tests), conv alone, then interleaved loop runs
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in c3ns2 c3ns4; do
  echo "== tests $v"
  RTH_LIB_PATH=$PWD/build/variants/$v.so timeout -k 10 300 python -m pytest tests/test_conv_gpu.py tests/test_fused_learner_gpu.py \
    -q -x --timeout 120 --timeout-method thread > gpurun_out/c3ns_tests_$v.log 2>&1; rc=$?
  tail -1 gpurun_out/c3ns_tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
for v in c3ns1 c3ns2 c3ns4; do
  echo "== conv alone $v"
  RTH_LIB_PATH=$PWD/build/variants/$v.so timeout -k 10 300 python scripts/bench_conv.py > gpurun_out/c3ns_conv_$v.log 2>&1 || exit $?
  grep "conv3" gpurun_out/c3ns_conv_$v.log | head -3
done
for r in 1 2; do for v in c3ns1 c3ns2 c3ns4; do
  echo "== loop $v $r"
  RTH_LIB_PATH=$PWD/build/variants/$v.so timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline > gpurun_out/c3ns_loop_${v}_$r.log 2>&1 || exit $?
  grep '^{' gpurun_out/c3ns_loop_${v}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['ms_per_step_window_median'], d['roofline']['mean_launch_us'], d['roofline']['frac'])"
done; done
