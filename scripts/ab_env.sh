#!/bin/bash
# A/B of environment settings in one box: interleaved bench runs, one line per run.
# usage: scripts/ab_env.sh ROUNDS STEPS "NAME:VAR=val VAR2=val" "NAME2:" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1 steps=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for spec in "$@"; do
    name=${spec%%:*} envs=${spec#*:}
    env $envs timeout -k 10 300 python bench.py --steps "$steps" --warmup 30 --no-cpu-baseline --no-sweep \
      > "gpurun_out/abe_${name}_$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name round $r failed rc=$rc"; tail -5 "gpurun_out/abe_${name}_$r.log"; exit $rc; fi
    python - "$name" "$r" "gpurun_out/abe_${name}_$r.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
d = json.loads(line)
hbm = {e["kernel"].split(" ")[0]: e["mean_launch_us"] for e in d["roofline_hbm"]}
print(f"{sys.argv[1]:>16} round {sys.argv[2]}: {d['ms_per_step']:.4f} ms/step windows {d['ms_per_step_windows']} "
      f"conv2 {d['roofline']['mean_launch_us']} {hbm}", flush=True)
PY
  done
done
