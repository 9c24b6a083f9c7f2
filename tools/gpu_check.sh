#!/bin/bash
# One GPU-box pass over the round gates (run from the repo root via gpurun):
#   pytest -m gpu, smoke(), then the default bench line. Each step has its own time limit and
#   the chain stops at the first failure. Outputs: gpurun_out/<tag>_{gpu_tests,smoke,bench}.log
# usage: tools/gpu_check.sh TAG [extra bench args]
TAG=${1:-r03}
shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${TAG}_gpu_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 500 python bench.py "$@" > gpurun_out/${TAG}_bench.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
tail -1 gpurun_out/${TAG}_bench.log
python tools/bench_summary.py default gpurun_out/${TAG}_bench.log
