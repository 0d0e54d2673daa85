set -u
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for v in "" noload noepi both; do
  lib=""; [ -n "$v" ] && lib=$PWD/reth_amd/libreth_hip_$v.so
  echo "== $v"
  RTH_LIB_PATH=$lib WGF_ONLY=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/diag_$v" -o run -- python scripts/bench_wgrad_f32.py 2>&1 | grep rth_conv || exit 1
  python - "$PWD/gpurun_out/diag_$v/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rth::' in r['Name']: print('   ', r['Name'][:60], round(float(r['AverageNs'])/1e3, 2))
PY
done
