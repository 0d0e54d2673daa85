#!/bin/bash
# A/B of the working tree against a snapshot of the previous commit in ab_old/ (Python-side
# changes): interleaved bench runs, one line per run.  usage: scripts/ab_tree.sh ROUNDS STEPS
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq 1 "$1"); do
  for side in new old; do
    dir=.; [ $side = old ] && dir=ab_old
    (cd $dir && timeout -k 10 300 python bench.py --steps "$2" --warmup 30 --no-cpu-baseline --no-sweep) \
      > "gpurun_out/abt_${side}_$r.log" 2>&1 || { echo "$side round $r failed"; tail -5 "gpurun_out/abt_${side}_$r.log"; exit 1; }
    python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/abt_${side}_$r.log') if l.startswith('{')][-1])
print(f'$side round $r: {d[\"ms_per_step\"]:.4f} ms/step  {d[\"value\"]:.0f} env-steps/s', flush=True)"
  done
done
