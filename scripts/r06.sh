#!/bin/bash
# round-6 GPU steps (each under its own limit; stop on a crash / timeout)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 limit=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 4 "gpurun_out/$name.log" | cut -c1-600
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
summ() {  # ms/step of bench logs
  for f in "$@"; do
    python -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
h={e['kernel'].split(' ')[0]: e.get('mean_launch_us') for e in d.get('roofline_hbm', [])}
print(sys.argv[1], d['ms_per_step'], d.get('ms_per_step_window_median'), 'clip_adam', h.get('rth_clip_adam'), 'tree', h.get('k_tree_update_sub'), h.get('k_tree_sample'))" "$f" 2>/dev/null
  done
}
for what in "$@"; do
  case $what in
    prof)  # steady-state kernel profile + the HBM counter passes of the same command shape
      step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" \
          -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep
      step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep
      step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep ;;
    tests) step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    dp8)  # 8 ranks on one GPU over gloo: bench.py's multi-rank path and its teardown (shutdown())
      RTH_SHARE_GPU=1 RTH_DIST_BACKEND=gloo step dp8_gloo_rehearsal 900 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --faithful --steps 20 \
          --warmup 5 --no-cpu-baseline --no-sweep ;;
    dp2)  # the driver's N = 2 command shape (weak scaling: 256 actors, 1 M rows, B = 512 per rank), both ranks on one GPU
      RTH_SHARE_GPU=1 RTH_DIST_BACKEND=gloo step dp2_gloo_rehearsal 900 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 20 --warmup 5 ;;
    driver) step bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    breakout) step breakout 600 python bench.py --workload breakout ;;
    span) RTH_BENCH_SPAN=1 step span 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-sweep ;;
    ab)  # interleaved A/B of library variants: AB_LIBS="name=path ..." (RTH_LIB_PATH), 2 rounds
      for r in 1 2; do
        for nv in ${AB_LIBS:-}; do
          n=${nv%%=*}; p=${nv#*=}
          RTH_LIB_PATH=$p step ab_${n}_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        done
      done
      summ gpurun_out/ab_*.log ;;
    *) echo "unknown step $what"; exit 2 ;;
  esac
done
