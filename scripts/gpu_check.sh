#!/bin/bash
# GPU-box check: each step has its own time limit; stop at the first crash/timeout
# (pytest rc 0/1 = ran to completion, anything else ends the call).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case "$step" in
    tests) run pytest_gpu 1200 python -m pytest tests -m gpu -q -rf ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py ;;
    benchq) run bench_quick 600 python bench.py --steps 50 --warmup 10 --cpu-iters 5 ;;
    variants)
      run bench_nchw 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --nchw
      run bench_cl 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline
      run bench_cl_find 900 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --conv-benchmark ;;
    bg) run bench_graph 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline ;;
    mtune) for m in 1 2 4 8; do RTH_COPY_HWC_M=$m run bench_m$m 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline; done ;;
    probetree) export TMPDIR=/tmp; run probe_tree 600 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$PWD/gpurun_out/ptree" -o run -- python scripts/probe_tree.py ;;
    ktune) export TMPDIR=/tmp; for k in 1 2 3 4; do for b in 64 256; do RTH_FIND_K=$k RTH_SAMPLE_BS=$b run probe_tree_k${k}_b$b 300 \
            rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/ktune_k${k}_b$b" -o run -- python scripts/probe_tree.py; done; done ;;
    kbench) export TMPDIR=/tmp; for kb in ${KB:-2_64}; do k=${kb%_*}; b=${kb#*_}; RTH_FIND_K=$k RTH_SAMPLE_BS=$b run kbench_k${k}_b$b 600 \
            rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/kbench_k${k}_b$b" -o run -- python bench.py --steps 60 --warmup 10 --no-cpu-baseline; done ;;
    dp2) RTH_SHARE_GPU=1 RTH_DIST_BACKEND=gloo run bench_dp2 900 python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 30 --warmup 10 \
            --capacity 100000 --no-cpu-baseline ${DP2_ARGS:-} ;;
    dpt) run pytest_dp 900 python -u -m pytest tests/test_dp_gpu.py tests/test_apex_gpu.py tests/test_fused_learner_gpu.py \
            -v -rf -x --timeout 300 --timeout-method thread ;;
    phases) run tree_phases 300 python scripts/probe_tree_phases.py ;;
    prio) for pr in 0 -1; do RTH_LEARNER_PRIORITY=$pr run bench_prio$pr 600 python bench.py --steps 200 --warmup 20 --no-cpu-baseline; done ;;
    convt) run pytest_conv 600 python -m pytest tests/test_conv_gpu.py -q -rf -x ;;
    dgrad) run bench_dgrad 300 python scripts/bench_dgrad.py &&
           for v in hip miopen hip2 miopen2; do
             if [ "${v:0:3}" = hip ]; then export RTH_HIP_DGRAD=1; else unset RTH_HIP_DGRAD; fi
             run bench_dgrad_$v 600 python bench.py --steps 400 --warmup 20 --no-cpu-baseline; done; unset RTH_HIP_DGRAD ;;
    dgv) for v in build/variants/*.so; do b=$(basename $v .so); RTH_LIB_PATH=$PWD/$v run bench_dgrad_$b 300 python scripts/bench_dgrad.py; done ;;
    span) for v in miopen; do
             if [ $v = hip ]; then export RTH_HIP_DGRAD=1; else unset RTH_HIP_DGRAD; fi
             RTH_BENCH_SPAN=1 run bench_span_$v 600 python bench.py --steps 400 --warmup 20 --no-cpu-baseline; done
          unset RTH_HIP_DGRAD ;;
    knobs) for w in 1 3 2; do RTH_CONV_WG_PER_CU=$w run bench_wpc$w 600 python bench.py --steps 400 --warmup 20 --no-cpu-baseline; done
           for pr in 0 -1; do RTH_LEARNER_PRIORITY=$pr run bench_prio$pr 600 python bench.py --steps 400 --warmup 20 --no-cpu-baseline; done ;;
    convb) run bench_conv 300 python scripts/bench_conv.py ;;
    wgv) for v in build/variants/*.so; do b=$(basename $v .so); RTH_LIB_PATH=$PWD/$v run bench_wgrad_$b 300 python scripts/bench_wgrad.py; done ;;
    convwpc) for w in 1 2 3 4; do RTH_CONV_WG_PER_CU=$w run bench_conv_wpc$w 300 python scripts/bench_conv.py; done ;;
    convv) for v in build/variants/*.so; do b=$(basename $v .so); RTH_LIB_PATH=$PWD/$v run bench_conv_$b 300 python scripts/bench_conv.py; done ;;
    convprof) export TMPDIR=/tmp; run prof_conv 300 rocprofv3 --kernel-trace --output-format csv \
            -d "$PWD/gpurun_out/prof_conv" -o run -- python scripts/bench_conv.py ;;
    convpmc) export TMPDIR=/tmp
         run pmc_conv_a 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
            SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv \
            -d "$PWD/gpurun_out/pmc_conv_a" -o run -- python scripts/conv_pmc.py &&
         run pmc_conv_b 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM \
            --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc_conv_b" -o run -- python scripts/conv_pmc.py ;;
    probe) run probe 300 python scripts/probe_qnet.py ;;
    host) run host_probe 300 python scripts/host_probe.py ;;
    breakout) run bench_breakout 900 python bench.py --workload breakout --steps 50 --warmup 10 --no-cpu-baseline ;;
    hostprof) export TMPDIR=/tmp; run host_prof 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/hp" -o run -- python scripts/host_probe.py ;;
    variants2)
      run bench_eager 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --eager
      run bench_graph 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline
      run bench_graph_nchw 600 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --nchw
      run bench_graph_nofind 900 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-conv-benchmark ;;
    pmc) export TMPDIR=/tmp
         run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
            -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline
         run pmc_write 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
            -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
    prof1) export TMPDIR=/tmp; run rocprof_1s 900 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$PWD/gpurun_out/prof" -o run -- python bench.py --steps 100 --warmup 20 --no-cpu-baseline ;;
    prof) export TMPDIR=/tmp; run rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$PWD/gpurun_out/prof" -o run -- python bench.py --steps 100 --warmup 10 --no-cpu-baseline ;;
    # the evidence set for a round: the bench line, its rocprof kernel trace + stats, and the two
    # PMC passes of the same command (scripts/summarize_profile.py TAG --steps 200 reads them)
    evidence) export TMPDIR=/tmp
         run bench_evidence 900 python bench.py &&
         run rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv \
            -d "$PWD/gpurun_out/prof" -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline &&
         run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
            -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline &&
         run pmc_write 900 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
            -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline ;;
  esac
done
