timeout -k 10 300 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k wgrad > gpurun_out/wg.log 2>&1; tail -n 2 gpurun_out/wg.log
for sp in 64 32; do RTH_WGX_SPLITS=$sp timeout -k 10 120 python scripts/bench_wgrad_f32.py 2>&1 | grep -v amdgpu | sed "s/^/splits=$sp /"; done
