#!/bin/bash
# r06 interleaved in-loop A/B: each ARMS entry "name|env assignments|bench flags", 2 rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  while IFS='|' read -r name envs flags; do
    [ -z "$name" ] && continue
    env $envs timeout -k 10 300 python bench.py --steps 300 --warmup 5 --no-cpu-baseline --no-sweep $flags \
      > gpurun_out/ab_${name}_$r.log 2>&1 || { echo "arm $name failed"; tail -5 gpurun_out/ab_${name}_$r.log; exit 1; }
    python - gpurun_out/ab_${name}_$r.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], d['ms_per_step'], d.get('ms_per_step_window_median'), d.get('ms_per_step_windows'))
PY
  done <<< "$ARMS"
done
