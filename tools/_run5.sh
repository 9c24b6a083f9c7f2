set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/debug_wide.py 512,4096 > gpurun_out/r06_debug_wide.log 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_bcr_gpu.py tests/test_band16_gpu.py tests/test_route_invariance_gpu.py > gpurun_out/r06_tests5a.log 2>&1 && \
timeout -k 10 200 python -u tools/c1_latency.py > gpurun_out/r06_c1_latency.jsonl 2>&1 && \
GPX_SMALL64=0 timeout -k 10 200 python -u tools/c1_latency.py --oracle 0 > gpurun_out/r06_c1_latency_chain.jsonl 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_callers_gpu.py tests/test_api.py tests/test_c_abi_gpu.py tests/test_deferred_gpu.py tests/test_distributed_gpu.py > gpurun_out/r06_tests5b.log 2>&1
