#!/bin/bash
# round-5 GPU steps (each under its own limit; stop on a crash / timeout)
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
pmc() {  # one rocprofv3 counter pass over a script: pmc NAME SCRIPT COUNTERS...
  local name=$1 script=$2; shift 2
  echo "== pmc $name ($(date +%T))"
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc_$name" \
      -o run -- python "$script" > "gpurun_out/pmc_$name.log" 2>&1
  local rc=$?
  echo "pmc $name rc=$rc"; tail -n 3 "gpurun_out/pmc_$name.log"
  [ $rc -eq 0 ] || exit $rc
}
summ() {  # print ms/step and the roofline fields of bench logs
  for f in "$@"; do python - "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{"metric"')][-1])
h = {r["kernel"]: r["mean_launch_us"] for r in d.get("roofline_hbm", [])}
print(sys.argv[1], d["ms_per_step"], d.get("ms_per_step_windows"), "conv2", d["roofline"].get("mean_launch_us"),
      d["roofline"]["frac"], {k: h[k] for k in sorted(h)})
PY
  done
}
for s in "$@"; do
  case "$s" in
    bench) step bench 600 python bench.py --gpus 1 --steps 20 --warmup 5 ;;
    benchlong) step bench_long 600 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      summ gpurun_out/bench_long.log ;;
    fwdpmc)  # SQ counters for the torso forward kernels at the learner's 1,024 samples
      export CONV_LAYERS=1,2,3
      pmc fwd_sq scripts/conv_pmc.py SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
          SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
      pmc fwd_inst scripts/conv_pmc.py GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES \
          SQ_LDS_IDX_ACTIVE
      unset CONV_LAYERS ;;
    adambench) step adam_alone1 120 python scripts/bench_adam.py
      RTH_ADAM_ONE_PASS=1 step adam_alone2 120 python scripts/bench_adam.py
      step adam_prof 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/adam_prof" -o run \
          -- python scripts/bench_adam.py  # (the two-launch default)
      python - <<'PY'
import csv, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open("gpurun_out/adam_prof/run_kernel_trace.csv")):
    if "adam" in r["Kernel_Name"] or "sqsum" in r["Kernel_Name"]:
        d[r["Kernel_Name"][:60]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in d.items():
    v.sort(); print(k, len(v), "median us", v[len(v) // 2], "min", v[0])
PY
      ;;
    adamab)  # one-launch clip+Adam vs the two-launch form, interleaved
      for r in 1 2; do
        RTH_ADAM_ONE_PASS=1 step ab_adam1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        step ab_adam2_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/ab_adam*.log ;;
    c1ab)  # conv1: each byte converted once per window pair (k_conv1_u8_share) vs r04's kernel
      step c1_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py
      CONV_NS=1024,512,256 step c1_micro_share 120 python scripts/bench_conv.py
      RTH_CONV1_NOSHARE=1 CONV_NS=1024,512,256 step c1_micro_noshare 120 python scripts/bench_conv.py
      RTH_LIB_PATH=reth_amd/libreth_hip_c1nb2.so CONV_NS=1024,512,256 step c1_micro_nb2 120 python scripts/bench_conv.py
      RTH_LIB_PATH=reth_amd/libreth_hip_c1nb1.so CONV_NS=1024,512,256 step c1_micro_nb1 120 python scripts/bench_conv.py
      grep -h "conv1" gpurun_out/c1_micro_*.log
      for r in 1 2; do
        step c1ab_share_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_CONV1_NOSHARE=1 step c1ab_noshare_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_c1nb2.so step c1ab_nb2_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/c1ab_*.log ;;
    c2diag)  # conv2 fp32-MFMA forward with parts removed (diagnostic variant libraries, wrong results)
      CONV_NS=1024,512 step c2d_dflt 120 python scripts/bench_conv.py
      for v in noloada noldsb noepi mfmaonly; do
        RTH_LIB_PATH=reth_amd/libreth_hip_$v.so CONV_NS=1024,512 step c2d_$v 120 python scripts/bench_conv.py
      done
      grep -H "conv2" gpurun_out/c2d_*.log ;;
    tdstages) step td_stages 300 python scripts/diag_td_stages.py gpurun_out/td_stages.json ;;
    treeab)  # tree sample: deep kernel (10 staged levels) with K = 3 (default) / 2 / 4 vs r04's kernel
      step tree_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sumtree_gpu.py \
          tests/test_scale_gpu.py tests/test_samplers_gpu.py tests/test_replay_gpu.py
      RTH_DEEP_K=2 step tree_tests_k2 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
          tests/test_sumtree_gpu.py tests/test_scale_gpu.py -k "sample or find or scale"
      RTH_DEEP_K=4 step tree_tests_k4 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
          tests/test_sumtree_gpu.py tests/test_scale_gpu.py -k "sample or find or scale"
      for r in 1 2; do
        step treeab_k3_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_DEEP_K=2 step treeab_k2_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_DEEP_K=4 step treeab_k4_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_TREE_SAMPLE_DEEP=0 step treeab_r04_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline \
            --no-sweep
        RTH_DEEP_K=2 RTH_LIB_PATH=reth_amd/libreth_hip_deep256.so step treeab_w256k2_$r 300 python bench.py --steps 300 \
            --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/treeab_*.log ;;
    treephase) RTH_TREE_TIMING=1 step tree_phases 300 python scripts/probe_tree_phases.py ;;
    prof)  # steady-state kernel profile + the HBM counter passes of the same command shape
      step rocprof_stats 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" \
          -o run -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-sweep
      step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep
      step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv --kernel-include-regex "rth::" \
          -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sweep ;;
    span) RTH_BENCH_SPAN=1 step span 300 python bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-sweep ;;
    tdfc) RTH_FC_X9=1 step td_stages_fcx9 300 python scripts/diag_td_stages.py gpurun_out/td_stages_fcx9.json ;;
    c2sched)  # conv2 tile schedules: tests, alone, in the loop
      step c2s_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py \
          -k "schedules or conv_f32_nhwc or partial or upto"
      for v in static ns2 pw2; do
        RTH_CONV2_SCHED=$v CONV_NS=1024,512,256 step c2s_micro_$v 120 python scripts/bench_conv.py
      done
      grep -H "conv2" gpurun_out/c2s_micro_*.log
      for r in 1 2; do
        for v in static ns2 pw2; do
          RTH_CONV2_SCHED=$v step c2sab_${v}_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        done
      done
      summ gpurun_out/c2sab_*.log ;;
    topab)  # tree update: the top pass as a concurrent extra workgroup (2) vs r04's last-workgroup form (1)
      RTH_TREE_FUSE_TOP=2 step top_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sumtree_gpu.py \
          tests/test_scale_gpu.py tests/test_samplers_gpu.py tests/test_replay_gpu.py tests/test_frame_store_gpu.py
      RTH_TREE_FUSE_TOP=2 RTH_TREE_TIMING=1 step tree_phases_top2 300 python scripts/probe_tree_phases.py
      for r in 1 2; do
        RTH_TREE_FUSE_TOP=2 step topab_2_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        step topab_1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/topab_*.log ;;
    fcf)  # FC1 on the fp32 MFMA without LDS (rth_fc_f32): tests, alone (ring depth, splits), in the loop
      step fcf_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fc_gpu.py
      step fcf_micro 120 python scripts/bench_fc.py
      RTH_FCF_NST=2 FC_MS=256,512,1024 step fcf_micro_nst2 120 python scripts/bench_fc.py
      RTH_FCF_NST=4 FC_MS=256,512,1024 step fcf_micro_nst4 120 python scripts/bench_fc.py
      RTH_FCF_SPLITS=16 FC_MS=256,512,1024 step fcf_micro_s16 120 python scripts/bench_fc.py
      RTH_FCF_SPLITS=4 FC_MS=256,512,1024 step fcf_micro_s4 120 python scripts/bench_fc.py
      grep -h "M=" gpurun_out/fcf_micro*.log
      for r in 1 2; do
        step fcab_blas_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC=f32 step fcab_f32_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC=f32 RTH_FC_MAX_ROWS=512 step fcab_f32s_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline \
            --no-sweep
      done
      summ gpurun_out/fcab_*.log ;;
    c2ts)  # conv2: the ragged last round split into channel parts (ts2 / ts4) vs static
      step c2ts_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py \
          -k "schedules or conv_f32_nhwc or partial or upto"
      for v in static ts4big; do
        RTH_CONV2_SCHED=$v CONV_NS=1024,512,256 step c2ts_micro_$v 120 python scripts/bench_conv.py
      done
      grep -H "conv2" gpurun_out/c2ts_micro_*.log
      for r in 1 2 3; do
        for v in static ts4big; do
          RTH_CONV2_SCHED=$v step c2tsab_${v}_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        done
      done
      summ gpurun_out/c2tsab_*.log ;;
    boab)  # Breakout: the tree update in two passes (RTH_TREE_PASSES=2: the append's run of leaves
      # spread over level-15 subtrees first) vs one pass
      step boab_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_scale_gpu.py
      for r in 1 2 3 4; do
        RTH_TREE_PASSES=1 step boab_1pass_$r 600 python bench.py --workload breakout --steps 100 --warmup 10 \
            --no-cpu-baseline --no-sweep
        step boab_2pass_$r 600 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/boab_*.log ;;
    bots)  # Breakout (actor stream critical, 2,048-sample actor forwards): conv2 split tail (ts4big) vs static
      for r in 1 2 3; do
        RTH_CONV2_SCHED=static step bots_static_$r 600 python bench.py --workload breakout --steps 100 --warmup 10 \
            --no-cpu-baseline --no-sweep
        step bots_ts8big_$r 600 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/bots_*.log ;;
    maskab)  # conv3's data gradient with conv2's ReLU mask + bias slabs in its epilogue vs the separate launch
      step mask_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py \
          tests/test_fused_learner_gpu.py tests/test_learner_full_gpu.py tests/test_frame_store_gpu.py
      for r in 1 2 3; do
        step maskab_on_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_DGRAD_MASK=0 step maskab_off_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/maskab_*.log ;;
    cfcab)  # Pong: the actors' FC1 over the N acting rows + the device-counted terminal rows (counted FC) vs 2N rows
      for r in 1 2 3; do
        step cfcab_dflt_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_ACTOR_COUNTED_FC=1 step cfcab_cfc_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/cfcab_*.log ;;
    fcx9s)  # Pong: the 512-row FC1 forwards (actors, target pass) on rth_fc_x9 (48 KB of LDS) vs hipBLASLt (80 KB)
      for r in 1 2 3; do
        RTH_FC=blas step fcx9s_blas_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC=x9 RTH_FC_MAX_ROWS=512 step fcx9s_x9_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline \
            --no-sweep
      done
      summ gpurun_out/fcx9s_*.log ;;
    fadvab)  # the frame head advanced by k_frames_push's last workgroup vs a second launch
      for r in 1 2 3; do
        step fadvab_ticket_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FRAMES_ADVANCE_LAUNCH=1 step fadvab_launch_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline \
            --no-sweep
      done
      summ gpurun_out/fadvab_*.log ;;
    fidab)  # frames in place (batches as frame ids, conv1 reads the store) vs the gather's stacks
      for r in 1 2 3; do
        RTH_FRAME_IDS=0 step fidab_stacks_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FRAME_IDS=1 step fidab_ids_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/fidab_*.log ;;
    prioab)  # stream priorities: the actor stream high (RTH_ACTOR_PRIORITY=-1) vs both normal
      for r in 1 2 3; do
        step prioab_dflt_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_ACTOR_PRIORITY=-1 step prioab_actor_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline \
            --no-sweep
      done
      summ gpurun_out/prioab_*.log ;;
    wgab)  # conv2 / conv3 weight gradients: MIOpen (default) vs its deterministic solvers vs rth_conv_wgrad_x9 / _f32
      for r in 1 2; do
        step wgab_dflt_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_CUDNN_DET=1 step wgab_det_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_HIP_WGRAD=x9 step wgab_x9_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_HIP_WGRAD=f32 step wgab_f32_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/wgab_*.log ;;
    c2x9ab)  # conv2 on k_conv_x9 for the small launches (actors ~256+; + the 512-sample target pass) vs fp32 MFMA
      for r in 1 2; do
        step c2x9ab_dflt_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_CONV2_X9_MAX=300 step c2x9ab_300_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_CONV2_X9_MAX=600 step c2x9ab_600_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/c2x9ab_*.log ;;
    # cumab (the learner stream on a CU-masked queue, a knob since removed): profiles/r05/ab_log.txt
    fcrowsab)  # the actors' counted FC1: reduce + counted rows in one launch (default) vs two launches
      for r in 1 2 3; do
        step fcrowsab_fused_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_ROWS_FUSED=0 step fcrowsab_two_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline \
            --no-sweep
      done
      summ gpurun_out/fcrowsab_*.log ;;
    # nostk (the gather without its stack assembly, RTH_DIAG_NO_STACKS=1, a timing-only build of
    # commit 'Diagnostic: RTH_DIAG_NO_STACKS=1'): profiles/r05/ab_log.txt
    fct)  # FC1 x9 on the 128 x 128 tile (both operands split once per workgroup): tests, alone per form
      step fct_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fc_gpu.py
      RTH_FC_TILE=64 step fct_micro_t64 120 python scripts/bench_fc.py
      RTH_FC_TILE=128 step fct_micro_t128 120 python scripts/bench_fc.py
      grep -h "M=" gpurun_out/fct_micro_*.log ;;
    fctab2)  # in the loop: the <= 512-row FC1 forwards on the 128 tile at 16 (default) / 8 / 4 k splits vs the 64 x 128 tile
      for r in 1 2 3; do
        RTH_FC_TILE=128 step fct2_t128_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_TILE=128 RTH_FCT_SPLITS=8 step fct2_s8_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_TILE=128 RTH_FCT_SPLITS=4 step fct2_s4_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_TILE=64 step fct2_t64_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/fct2_*.log ;;
    fctab3)  # in the loop: 128 tile at 16 (default) / 24 / 32 k splits; every FC1 on x9 at 16 splits (the learner's 1,024 rows too)
      for r in 1 2 3; do
        RTH_FC_TILE=128 step fct3_s16_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_TILE=128 RTH_FCT_SPLITS=24 step fct3_s24_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_TILE=128 RTH_FCT_SPLITS=32 step fct3_s32_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_TILE=128 RTH_FCT_SPLITS=16 RTH_FC_MAX_ROWS=0 step fct3_all16_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/fct3_*.log ;;
    fctab4)  # in the loop: the 128 tile by default (16 k splits at most) vs at most 32 (the actors' 256 rows: 256 workgroups) vs 64 x 128
      for r in 1 2 3; do
        step fct4_dflt_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FCT_MAXSPLITS=32 step fct4_m32_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_TILE=64 step fct4_t64_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/fct4_*.log ;;
    fctbo)  # Breakout: the 512-row FC1 (target pass) on the 128 tile (default) vs 64 x 128; + the actors' 2,048 rows on x9
      for r in 1 2; do
        step fctbo_dflt_$r 300 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
        RTH_FC_TILE=64 step fctbo_t64_$r 300 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
        RTH_FC_MAX_ROWS=2048 step fctbo_a2k_$r 300 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline \
            --no-sweep
      done
      summ gpurun_out/fctbo_*.log ;;
    fctab5)  # the late-r05 FC1 rule (every forward but the learner's on x9) vs at most 512 rows on x9 (the earlier rule), Pong + Breakout
      for r in 1 2; do
        step fct5_po_dflt_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_MAX_ROWS=512 step fct5_po_m512_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        step fct5_bo_dflt_$r 300 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
        RTH_FC_MAX_ROWS=512 step fct5_bo_m512_$r 300 python bench.py --workload breakout --steps 100 --warmup 10 \
            --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/fct5_*.log ;;
    ldsab)  # CU-exclusive launches by padded LDS (RTH_LDS_MIN_<CLASS> bytes per workgroup; a knob of a build since removed)
      for r in 1 2; do
        step lds_dflt_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LDS_MIN_C1=98304 step lds_c1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LDS_MIN_X9=98304 step lds_x9_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LDS_MIN_DG=98304 step lds_dg_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LDS_MIN_W1=98304 step lds_w1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/lds_*.log ;;
    adam2)  # clip+Adam: partials + bias corrections read ahead of the chunk (the norm reduced while it is in flight) vs r05's
      # earlier k_adam (reth_amd/libreth_hip_adamprev.so: the chunk first, every workgroup evaluating the fp64 pow)
      step adam2_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_optim_gpu.py
      step adam2_alone_new 120 python scripts/bench_adam.py
      RTH_LIB_PATH=reth_amd/libreth_hip_adamprev.so step adam2_alone_prev 120 python scripts/bench_adam.py
      for r in 1 2 3; do
        step adam2_new_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_adamprev.so step adam2_prev_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep
      done
      grep -h clip_adam gpurun_out/adam2_alone_*.log
      summ gpurun_out/adam2_new_*.log gpurun_out/adam2_prev_*.log ;;
    fcrd)  # 128-tile x9 FC1: fragments read term-major (the MFMAs' consumption order) vs mb-major (libreth_hip_fcprev.so)
      FC_MS=256,512,2048 step fcrd_alone_new 120 python scripts/bench_fc.py
      RTH_LIB_PATH=reth_amd/libreth_hip_fcprev.so FC_MS=256,512,2048 step fcrd_alone_prev 120 python scripts/bench_fc.py
      for r in 1 2 3; do
        step fcrd_new_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_fcprev.so step fcrd_prev_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep
      done
      grep -h "M=" gpurun_out/fcrd_alone_*.log | sed "s/rth_fc_f32.*//"
      summ gpurun_out/fcrd_new_*.log gpurun_out/fcrd_prev_*.log ;;
    knobab)  # on the late-r05 tree: conv workgroups per CU 1 (RTH_CONV_WG_PER_CU=1) and conv2's split tail for the learner's launch (ts4big) vs default
      for r in 1 2 3; do
        step knob_dflt_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_CONV_WG_PER_CU=1 step knob_wg1_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_CONV2_SCHED=ts4big step knob_ts4_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/knob_*.log ;;
    redab)  # FC1 split-K reduce with every partial loaded ahead (unrolled) vs the runtime-count loop (libreth_hip_redprev.so)
      step red_tests 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fc_gpu.py
      RTH_FC_TILE=128 FC_M=256,512 step red_kt_new 120 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$PWD/gpurun_out/red_new" -o run -- python scripts/fc_pmc.py
      RTH_LIB_PATH=reth_amd/libreth_hip_redprev.so FC_M=256,512 step red_kt_prev 120 rocprofv3 --kernel-trace --stats \
          --output-format csv -d "$PWD/gpurun_out/red_prev" -o run -- python scripts/fc_pmc.py
      grep -h "reduce" gpurun_out/red_new/run_kernel_stats.csv gpurun_out/red_prev/run_kernel_stats.csv | cut -c1-160
      for r in 1 2 3; do
        step red_new_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_redprev.so step red_prev_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/red_new_*.log gpurun_out/red_prev_*.log ;;
    boprio)  # Breakout (actor stream critical): the actor stream at high priority; conv2 whole tiles (static) vs the ts4big default
      for r in 1 2; do
        step boprio_dflt_$r 300 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
        RTH_ACTOR_PRIORITY=-1 step boprio_hi_$r 300 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
        RTH_CONV2_SCHED=static step boprio_static_$r 300 python bench.py --workload breakout --steps 100 --warmup 10 \
            --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/boprio_*.log ;;
    ldab)  # serialized-load loops made batched: conv3 dgrad's masked epilogue (mask loads ahead), the frame push copy (2 loads
      # ahead) vs HEAD before them (libreth_hip_ldprev.so)
      step ld_tests 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py \
          tests/test_frame_store_gpu.py
      for r in 1 2 3; do
        step ld_new_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_ldprev.so step ld_prev_$r 300 python bench.py --steps 300 --warmup 5 \
            --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/ld_new_*.log gpurun_out/ld_prev_*.log ;;
    deepab)  # tree sample: 512 / 1,024-lane workgroups (one or half a workgroup for B = 512: one staged top) vs 256
      RTH_LIB_PATH=reth_amd/libreth_hip_deep512.so step deep_tests 300 python -u -m pytest -x -q --timeout 200 \
          --timeout-method thread tests/test_sumtree_gpu.py tests/test_replay_gpu.py
      for r in 1 2 3; do
        step deep_256_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_deep512.so step deep_512_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_deep1024.so step deep_1024_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/deep_*_[0-9].log ;;
    deepab2)  # tree sample: 128-lane workgroups (4 for B = 512) vs 256
      RTH_LIB_PATH=reth_amd/libreth_hip_deep128.so step deep2_tests 300 python -u -m pytest -x -q --timeout 200 \
          --timeout-method thread tests/test_sumtree_gpu.py tests/test_replay_gpu.py
      for r in 1 2 3; do
        step deep2_256_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_LIB_PATH=reth_amd/libreth_hip_deep128.so step deep2_128_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/deep2_*_[0-9].log ;;
    fcpmc)  # per-kernel durations (x9 GEMM vs reduce) and SQ counters of the FC1 x9 forms at FC_M rows
      fcsum() {  # fcsum DIR: median duration and counters per kernel
        python - "$1" <<'PY'
import collections, csv, os, statistics as st, sys
d = sys.argv[1]
for f in ("run_kernel_trace.csv", "run_counter_collection.csv"):
    p = os.path.join(d, f)
    if not os.path.exists(p):
        continue
    v = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        if "fc" not in k:
            continue
        v[k]["us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if "Counter_Name" in r:
            v[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in v.items():
        print(d.split("/")[-1], k, {n: round(st.median(x), 2) for n, x in c.items()})
PY
      }
      for form in t64 t128; do  # (r05: also 4 waves, 2 chunks in flight, coalesced staging loads -- removed)
        case $form in t64) e="RTH_FC_TILE=64";; t128) e="RTH_FC_TILE=128";; esac
        env $e timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/fct_$form" -o run \
            -- python scripts/fc_pmc.py > gpurun_out/fct_$form.log 2>&1 || exit 1
        fcsum gpurun_out/fct_$form
      done
      for form in t64 t128; do
        case $form in t64) e="RTH_FC_TILE=64";; t128) e="RTH_FC_TILE=128";; esac
        env $e timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
            SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --kernel-trace \
            --output-format csv -d "$PWD/gpurun_out/fcp_$form" -o run -- python scripts/fc_pmc.py \
            > gpurun_out/fcp_$form.log 2>&1 || exit 1
        fcsum gpurun_out/fcp_$form
      done ;;
    fctab)  # in the loop: FC1 <= 512 rows on the x9 128 tile (RTH_FC_TILE=128) / every FC1 on x9 (RTH_FC_MAX_ROWS=0,
      # the learner's 1,024 rows on the 128 tile) vs the default (<= 512 rows on the 64 x 128 tile, 1,024 on hipBLASLt)
      for r in 1 2; do
        RTH_FC_TILE=128 step fctab_t128_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        RTH_FC_MAX_ROWS=0 step fctab_all_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
        step fctab_t64_$r 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep
      done
      summ gpurun_out/fctab_*.log ;;
    dp8)  # 8 ranks on one GPU over gloo: bench.py's multi-rank path and its teardown (shutdown())
      RTH_SHARE_GPU=1 RTH_DIST_BACKEND=gloo step dp8_gloo_rehearsal 900 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --faithful --steps 20 \
          --warmup 5 --no-cpu-baseline --no-sweep
      grep -c '"metric"' gpurun_out/dp8_gloo_rehearsal.log ;;
    breakout)  # BASELINE configs[2]: the driver's command shape and a longer run
      step bench_breakout_driver 600 python bench.py --workload breakout --steps 20 --warmup 5 --no-cpu-baseline \
          --no-sweep
      step bench_breakout 600 python bench.py --workload breakout --steps 100 --warmup 10 --no-cpu-baseline --no-sweep
      summ gpurun_out/bench_breakout_driver.log gpurun_out/bench_breakout.log ;;
    tests) step gpu_tests 1100 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    t:*) f=${s#t:}; step "t_$(basename ${f//,/_} .py)" 900 python -u -m pytest -x -v --timeout 300 \
          --timeout-method thread ${f//,/ } ;;
  esac
done
