#!/bin/bash
# A/B of library variants in one box: interleaved bench runs, one line per run.
# usage: scripts/ab_bench.sh ROUNDS STEPS variant1.so variant2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
rounds=$1 steps=$2; shift 2
for r in $(seq 1 "$rounds"); do
  for v in "$@"; do
    b=$(basename "$v" .so)
    RTH_LIB_PATH=$PWD/$v timeout -k 10 300 python bench.py --steps "$steps" --warmup 30 --no-cpu-baseline \
      > "gpurun_out/ab_${b}_$r.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$b round $r failed rc=$rc"; tail -5 "gpurun_out/ab_${b}_$r.log"; exit $rc; fi
    python - "$b" "$r" "gpurun_out/ab_${b}_$r.log" <<'PY'
import json, sys
line = [l for l in open(sys.argv[3]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"{sys.argv[1]:>24} round {sys.argv[2]}: {d['ms_per_step']:.4f} ms/step  {d['value']:.0f} env-steps/s", flush=True)
PY
  done
done
