set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bcr_gpu.py tests/test_band16_gpu.py tests/test_deferred_gpu.py tests/test_route_invariance_gpu.py tests/test_c2_parity_gpu.py > gpurun_out/r06_tests7.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/r06_bench7.log 2>&1
