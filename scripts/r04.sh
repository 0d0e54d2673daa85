#!/bin/bash
# round-4 GPU steps (each under its own limit; stop on a crash / timeout):
#   transient = per-step GPU times of the driver's command shape (--steps 20 --warmup 5)
#               with / without the in-window timers and the conv probe, and after a long warmup
#   tests     = the GPU test suite;  smoke = __graft_entry__.smoke()
#   bench     = the driver's command
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
for s in "$@"; do
  case "$s" in
    transient)
      RTH_BENCH_STEPTIMES=1 step tr_default 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_NOTIMER=1 step tr_notimer 300 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline --no-sweep --no-probe
      RTH_BENCH_STEPTIMES=1 step tr_longwarm 300 python bench.py --steps 20 --warmup 300 --no-cpu-baseline --no-sweep
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_NOTIMER=1 step tr_longwarm_notimer 300 python bench.py --steps 20 --warmup 300 \
          --no-cpu-baseline --no-sweep --no-probe ;;
    transient2)
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_NOTIMER=1 step tr2_short 300 python bench.py --steps 40 --warmup 5 \
          --no-cpu-baseline --no-sweep --no-probe
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_NOTIMER=1 step tr2_long 300 python bench.py --steps 40 --warmup 300 \
          --no-cpu-baseline --no-sweep --no-probe ;;
    learnerfull) step learner_full 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
          tests/test_learner_full_gpu.py ;;
    newtests) step new_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
          tests/test_apex_gpu.py tests/test_learner_full_gpu.py tests/test_zmtp_gpu.py tests/test_dropin_gpu.py ;;
    benchdiag) RTH_BENCH_STEPTIMES=1 step bench_diag 600 python bench.py --steps 40 --warmup 5 --no-cpu-baseline ;;
    first)
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_PROFILE0=1 step first_prof 300 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline --no-sweep --probe-steps 0
      RTH_BENCH_STEPTIMES=1 RTH_BENCH_SETTLE_SYNC=16 step first_sync16 300 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline --no-sweep --probe-steps 0
      RTH_BENCH_STEPTIMES=1 step first_nosettle 300 python bench.py --steps 20 --warmup 5 --settle 0 \
          --no-cpu-baseline --no-sweep --probe-steps 0
      RTH_BENCH_STEPTIMES=1 step first_plain 300 python bench.py --steps 20 --warmup 5 \
          --no-cpu-baseline --no-sweep --probe-steps 0 ;;
    dp8) RTH_SHARE_GPU=1 RTH_DIST_BACKEND=gloo step dp8_gloo_rehearsal 900 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --faithful --steps 20 \
          --warmup 5 --no-cpu-baseline --no-sweep ;;
    fstore) step fstore_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
          tests/test_frame_store_gpu.py tests/test_replay_gpu.py tests/test_atari_loop_gpu.py tests/test_gemm_tuning_gpu.py ;;
    breakout) step bench_breakout 900 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
      step bench_breakout_fs 900 python bench.py --workload breakout --frame-store --steps 100 --warmup 10 \
          --no-cpu-baseline --no-sweep ;;
    dgradt) step dgrad_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
          tests/test_conv_gpu.py tests/test_fused_learner_gpu.py tests/test_learner_full_gpu.py ;;
    dgradab) for r in 1 2; do
        RTH_MIOPEN_DGRAD3=1 RTH_DGRAD2_F32=1 step ab_miopen_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep --probe-steps 0
        RTH_DGRAD2_F32=1 step ab_x9dgrad3_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep \
            --probe-steps 0
        step ab_x9dgrad_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep --probe-steps 0
      done
      grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ab_*.log ;;
    treet) step tree_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
          tests/test_sumtree_gpu.py tests/test_scale_gpu.py tests/test_samplers_gpu.py tests/test_replay_gpu.py ;;
    treeab) for r in 1 2; do
        for v in "notop:RTH_TREE_LDS_TOP=0" "top:RTH_TREE_LDS_TOP=1" "lane1:RTH_FIND_GROUP=0 RTH_FIND_K=1" \
                 "lane2:RTH_FIND_GROUP=0 RTH_FIND_K=2"; do
          ( export ${v#*:}; step ab_tree_${v%%:*}_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline \
              --no-sweep ) || exit $?
        done
      done
      for f in gpurun_out/ab_tree_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
h = {r["kernel"]: r["mean_launch_us"] for r in d["roofline_hbm"]}
print(sys.argv[1], d["ms_per_step"], "sample_us", h["k_tree_sample"], "update_us", h["k_tree_update_sub"])
PY
      done ;;
    treepmc) for v in "notop:RTH_TREE_LDS_TOP=0" "top:RTH_TREE_LDS_TOP=1" "lane1:RTH_FIND_GROUP=0 RTH_FIND_K=1" \
                      "lane2:RTH_FIND_GROUP=0 RTH_FIND_K=2"; do
        ( export ${v#*:}; step pmc_tree_${v%%:*} 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
            --kernel-include-regex "k_tree_sample" -d "$PWD/gpurun_out/pmc_tree_${v%%:*}" -o run -- \
            python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep --settle 16 --probe-steps 0 ) || exit $?
      done
      python scripts/summarize_profile.py --tree-pmc gpurun_out/pmc_tree_* | tee gpurun_out/tree_pmc.txt ;;
    breakprof) step prof_breakout 600 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$PWD/gpurun_out/prof_bo" -o run -- python bench.py --workload breakout --steps 60 --warmup 5 \
          --no-cpu-baseline --no-sweep --probe-steps 0
      python scripts/stream_busy.py gpurun_out/prof_bo/run_kernel_trace.csv 60 | tee gpurun_out/breakout_streams.txt ;;
    kbench) step conv_kernel_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
          tests/test_conv_gpu.py -k "dgrad or wgrad"
      RTH_DGRAD2_X9=1 step conv_kernel_tests_x9d2 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
          tests/test_conv_gpu.py -k "dgrad"
      step bench_dgrad_dflt 300 python scripts/bench_dgrad.py
      RTH_DGRAD3_F32=1 step bench_dgrad_f32 300 python scripts/bench_dgrad.py
      RTH_DGRAD2_X9=1 step bench_dgrad2_x9 300 python scripts/bench_dgrad.py
      step bench_wgrad 300 python scripts/bench_wgrad_f32.py ;;
    wgxab) for r in 1 2; do
        step ab_wgmiopen_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep \
            --probe-steps 0
        RTH_HIP_WGRAD=x9 step ab_wgx9_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep --probe-steps 0
      done
      grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ab_wg*.log ;;
    diagfs) RTH_HIP_WGRAD=x9 step diag_fstore_eager 300 python -u scripts/diag_fstore.py
      RTH_HIP_WGRAD=x9 step diag_fstore_graph 300 python -u scripts/diag_fstore.py graph ;;
    d2ab) for r in 1 2; do
        step ab_d2f32_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep --probe-steps 0
        RTH_DGRAD2_X9=1 step ab_d2x9_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep \
            --probe-steps 0
      done
      grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ab_d2*.log ;;
    boab) for r in 1 2; do
        step ab_bo_dflt_$r 300 python bench.py --workload breakout --steps 100 --warmup 5 --no-cpu-baseline --no-sweep \
            --probe-steps 0
        RTH_ACTOR_COUNTED_FC=1 step ab_bo_cfc_$r 300 python bench.py --workload breakout --steps 100 --warmup 5 \
            --no-cpu-baseline --no-sweep --probe-steps 0
      done
      grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bo_*.log ;;
    bwdpmc) for ps in "sq:SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
                 "inst:GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_IDX_ACTIVE" \
                 "fetch:FETCH_SIZE" "write:WRITE_SIZE"; do
        CONV_LAYERS=d2,d3,w2,w3 step pmc_bwd_${ps%%:*} 120 rocprofv3 --pmc ${ps#*:} --kernel-trace --output-format csv \
            -d "$PWD/gpurun_out/pmc_bwd_${ps%%:*}" -o run -- python scripts/conv_pmc.py
      done
      python scripts/summarize_conv_pmc.py r04 | tail -40 ;;
    final1) step bench_final 600 python bench.py
      RTH_BENCH_SPAN=1 step span 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-sweep
      step bench_breakout_final 600 python bench.py --workload breakout --frame-store --steps 100 --warmup 10 \
          --no-cpu-baseline --no-sweep
      step bench_breakout_full 600 python bench.py --workload breakout --full-rows --steps 100 --warmup 10 \
          --no-cpu-baseline --no-sweep ;;
    final2) step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" \
          -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep
      step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep
      step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep ;;
    final3) step bench_atari 600 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-sweep --env atari
      step bench_atari_h2d 600 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-sweep --env atari-h2d ;;
    wgxab2) for r in 1 2; do
        step ab_w2base_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep --probe-steps 0
        for sp in 16 32 128; do
          RTH_HIP_WGRAD=x9 RTH_WGX_SPLITS=$sp step ab_w2s${sp}_$r 300 python bench.py --steps 300 --warmup 5 \
              --no-cpu-baseline --no-sweep --probe-steps 0
        done
      done
      grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/ab_w2*.log ;;
    fsab) for r in 1 2; do
        step ab_pong_full_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep --probe-steps 0
        step ab_pong_fs_$r 300 python bench.py --frame-store --steps 300 --warmup 5 --no-cpu-baseline --no-sweep \
            --probe-steps 0
      done
      grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/ab_pong_*.log ;;
    fc) step fc_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_fc_gpu.py
      step bench_fc 300 python scripts/bench_fc.py
      RTH_FC_SPLITS=16 step bench_fc_s16 300 python scripts/bench_fc.py
      RTH_FC_SPLITS=32 step bench_fc_s32 300 python scripts/bench_fc.py ;;
    fcab) RTH_FC_X9=1 step fc_learner_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
          tests/test_learner_full_gpu.py tests/test_fused_learner_gpu.py tests/test_learner_gpu.py tests/test_actor_gpu.py tests/test_apex_gpu.py
      for r in 1 2; do
        step ab_fc0_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep --probe-steps 0
        RTH_FC_X9=1 step ab_fc1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep \
            --probe-steps 0
      done
      grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/ab_fc*.log ;;
    benchfs) step bench_fs_default 600 python bench.py --frame-store ;;
    c2ab)  # conv2 fp32-MFMA tile shapes: waves per workgroup x channel parts per pixel tile
      for v in 8,1 8,2 8,4 16,1 16,2 16,4; do
        RTH_CONV2_WAVES=${v%,*} RTH_CONV2_NS=${v#*,} CONV_NS=1024,512,256 step c2_micro_${v/,/_} 120 python scripts/bench_conv.py
        grep conv2 gpurun_out/c2_micro_${v/,/_}.log
      done
      for v in 8,2 16,1 16,2; do
        RTH_CONV2_WAVES=${v%,*} RTH_CONV2_NS=${v#*,} step c2_tests_${v/,/_} 300 python -u -m pytest -x -q --timeout 120 \
            --timeout-method thread tests/test_conv_gpu.py
      done
      for r in 1 2; do
        for v in 8,1 8,2 16,1 16,2; do
          RTH_CONV2_WAVES=${v%,*} RTH_CONV2_NS=${v#*,} step c2_ab_${v/,/_}_$r 300 python bench.py --steps 300 --warmup 5 \
              --no-cpu-baseline --no-sweep
        done
      done
      for f in gpurun_out/c2_ab_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[1], d["ms_per_step"], d["roofline"]["mean_launch_us"], d["roofline"]["frac"])
PY
      done ;;
    ppab)  # the data gradients' kernels packed in the forward's pack launch vs one pack launch each
      step pp_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py \
          tests/test_fused_learner_gpu.py tests/test_learner_gpu.py tests/test_frame_store_gpu.py
      for r in 1 2; do
        for v in 0 1; do
          RTH_DGRAD_PREPACK=$v step pp_ab_${v}_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        done
      done
      for f in gpurun_out/pp_ab_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[1], d["ms_per_step"], d["roofline"]["mean_launch_us"], d["roofline"]["frac"])
PY
      done ;;
    clk)  # conv2's in-kernel clock (diagnostic build), the ballot compaction, two bench runs
      step clk_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_actor_gpu.py \
          tests/test_conv_gpu.py tests/test_apex_gpu.py
      RTH_LIB_PATH=reth_amd/libreth_hip_clk.so step conv_clock 120 python scripts/conv_clock.py
      RTH_LIB_PATH=reth_amd/libreth_hip_clk.so CLK_N=512 step conv_clock512 120 python scripts/conv_clock.py
      for r in 1 2; do
        step clk_bench_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      cat gpurun_out/conv_clock.log gpurun_out/conv_clock512.log | grep kernel
      for f in gpurun_out/clk_bench_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[1], d["ms_per_step"], d["roofline"]["mean_launch_us"], d["roofline"]["frac"])
PY
      done ;;
    sideab)  # FC1's weight gradient on a side stream vs in line (+ the wider conv1 reduce in both)
      step side_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_learner_gpu.py \
          tests/test_learner_gpu.py tests/test_apex_gpu.py tests/test_dp_gpu.py tests/test_rccl_gpu.py \
          tests/test_learner_full_gpu.py tests/test_conv_gpu.py
      for r in 1 2; do
        for v in 0 1; do
          RTH_FC1_WGRAD_SIDE=$v step side_ab_${v}_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        done
      done
      for f in gpurun_out/side_ab_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[1], d["ms_per_step"], d["roofline"]["mean_launch_us"], d["roofline"]["frac"])
PY
      done ;;
    dp8fs) RTH_SHARE_GPU=1 RTH_DIST_BACKEND=gloo step dp8_gloo_rehearsal_fs 900 python -m torch.distributed.run \
          --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --faithful \
          --steps 20 --warmup 5 --no-cpu-baseline --no-sweep ;;
    hbab) step hb_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_learner_gpu.py \
          tests/test_fused_learner_gpu.py tests/test_learner_full_gpu.py
      for r in 1 2; do
        RTH_HB_BATCHED=0 step ab_hb0_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        step ab_hb1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      for f in gpurun_out/ab_hb*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
h = {r["kernel"]: r["mean_launch_us"] for r in d["roofline_hbm"]}
print(sys.argv[1], d["ms_per_step"], "td_heads_backward_us", h.get("k_td_heads_backward"))
PY
      done ;;
    wredab) step wred_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py \
          tests/test_learner_full_gpu.py tests/test_fused_learner_gpu.py
      for r in 1 2; do
        RTH_WGRED_WIDE=0 step ab_wred0_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep \
            --probe-steps 0
        step ab_wred1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep --probe-steps 0
      done
      grep -H -o '"ms_per_step": [0-9.]*' gpurun_out/ab_wred*.log ;;
    rccl) step rccl_test 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_rccl_gpu.py ;;
    evid)  # the round's closing evidence on the final tree: suite, smoke, default bench, span, profiles
      step gpu_tests 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests
      step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
      step bench_final 600 python bench.py
      RTH_BENCH_SPAN=1 step span 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-sweep ;;
    evid2)
      step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" \
          -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep
      step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep
      step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep
      step bench_breakout_final 600 python bench.py --workload breakout --steps 100 --warmup 10 \
          --no-cpu-baseline --no-sweep
      step bench_driver 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    wgbab)  # conv1 weight-gradient partial blocks (CONV_WG_BLOCKS, variant libraries) 256 / 128 / 512
      for v in wg128 wg512; do
        RTH_LIB_PATH=reth_amd/libreth_hip_$v.so step wgb_tests_$v 300 python -u -m pytest -x -q --timeout 120 \
            --timeout-method thread tests/test_conv_gpu.py tests/test_fused_learner_gpu.py
      done
      for r in 1 2; do
        step wgb_ab_base_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        for v in wg128 wg512; do
          RTH_LIB_PATH=reth_amd/libreth_hip_$v.so step wgb_ab_${v}_$r 300 python bench.py --steps 300 --warmup 5 \
              --no-cpu-baseline --no-sweep
        done
      done
      for f in gpurun_out/wgb_ab_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[1], d["ms_per_step"], d["ms_per_step_windows"])
PY
      done ;;
    c2mb2)  # conv2 fp32 MFMA with 32-pixel wave tiles (CONV2_MB=2, variant library)
      RTH_LIB_PATH=reth_amd/libreth_hip_c2mb2.so CONV_NS=1024,512,256 step c2mb2_micro 120 python scripts/bench_conv.py
      CONV_NS=1024,512,256 step c2mb1_micro 120 python scripts/bench_conv.py
      grep conv2 gpurun_out/c2mb2_micro.log gpurun_out/c2mb1_micro.log
      RTH_LIB_PATH=reth_amd/libreth_hip_c2mb2.so step c2mb2_tests 300 python -u -m pytest -x -q --timeout 120 \
          --timeout-method thread tests/test_conv_gpu.py
      for r in 1 2; do
        step c2mb_ab_base_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_c2mb2.so step c2mb_ab_mb2_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep
      done
      for f in gpurun_out/c2mb_ab_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[1], d["ms_per_step"], d["roofline"]["mean_launch_us"], d["roofline"]["frac"])
PY
      done ;;
    c1nb)  # conv1 forward: tiles whose windows are in flight (C1_NBUF, variant libraries) 3 / 2 / 4
      for v in c1nb2 c1nb4; do
        RTH_LIB_PATH=reth_amd/libreth_hip_$v.so CONV_NS=1024,512,256 step ${v}_micro 120 python scripts/bench_conv.py
        RTH_LIB_PATH=reth_amd/libreth_hip_$v.so step ${v}_tests 300 python -u -m pytest -x -q --timeout 120 \
            --timeout-method thread tests/test_conv_gpu.py
      done
      CONV_NS=1024,512,256 step c1nb3_micro 120 python scripts/bench_conv.py
      grep -h "conv1" gpurun_out/c1nb*_micro.log
      for r in 1 2; do
        step c1nb_ab_base_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        for v in c1nb2 c1nb4; do
          RTH_LIB_PATH=reth_amd/libreth_hip_$v.so step c1nb_ab_${v}_$r 300 python bench.py --steps 300 --warmup 5 \
              --no-cpu-baseline --no-sweep
        done
      done
      for f in gpurun_out/c1nb_ab_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[1], d["ms_per_step"], d["ms_per_step_windows"])
PY
      done ;;
    x9wg)  # x9 conv workgroups per CU (runtime RTH_X9_WG_PER_CU): 1 (default) vs 2
      RTH_X9_WG_PER_CU=2 step x9wg_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
          tests/test_conv_gpu.py
      for r in 1 2; do
        step x9wg_ab_1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_X9_WG_PER_CU=2 step x9wg_ab_2_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      for f in gpurun_out/x9wg_ab_*.log; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
print(sys.argv[1], d["ms_per_step"], d["ms_per_step_windows"], d["roofline_conv3"]["mean_launch_us"])
PY
      done ;;
    convtests)
      step conv_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py
      RTH_X9_WG_PER_CU=2 step conv_tests_wg2 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
          tests/test_conv_gpu.py ;;
    rccldbg) step rccl_dbg 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_gpu.py ;;
    tests) step gpu_tests 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
  esac
done
