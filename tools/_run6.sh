set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/c1_latency.py > gpurun_out/r06_c1_latency.jsonl 2>&1 && \
GPX_SMALL_DIRECT=0 timeout -k 10 200 python -u tools/c1_latency.py --oracle 0 > gpurun_out/r06_c1_latency_dma.jsonl 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_deferred_gpu.py tests/test_gpu_parity.py tests/test_callers_gpu.py tests/test_api.py tests/test_c_abi_gpu.py tests/test_distributed_gpu.py > gpurun_out/r06_tests6.log 2>&1
