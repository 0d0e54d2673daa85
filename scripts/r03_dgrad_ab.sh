timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_fused_learner_gpu.py > gpurun_out/ct.log 2>&1; tail -n 2 gpurun_out/ct.log
for v in 1 0 1; do RTH_DGRAD_XCD=$v timeout -k 10 120 python scripts/bench_dgrad.py 2>&1 | grep -v amdgpu.ids | sed "s/^/xcd=$v /"; done
BENCH_ARGS=--no-sweep bash scripts/ab_env.sh 2 200 "xcd1 RTH_DGRAD_XCD=1" "xcd0 RTH_DGRAD_XCD=0"
timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-sweep > gpurun_out/bq.log 2>&1; tail -n 1 gpurun_out/bq.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step']); [print(k, json.dumps(d[k])[:700]) for k in ('roofline','roofline_conv2','conv_iteration_alone')]"
