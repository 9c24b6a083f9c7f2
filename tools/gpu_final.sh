#!/bin/bash
# The round's closing GPU pass in one call: the gates (tools/gpu_check.sh: pytest -m gpu, smoke,
# the default bench line), the profiles (tools/profile_round4.sh without its own bench) and the
# device ceilings of the width classes (tools/band_throughput.py: 2048 problems of one class in
# 4 concurrent batches, no host loop).
# usage: tools/gpu_final.sh TAG
TAG=${1:-r04z}
bash tools/gpu_check.sh "$TAG" && SKIP_BENCH=1 bash tools/profile_round4.sh "$TAG" || exit 1
for e in 1.18 1.6 1.9 2.3; do
  timeout -k 10 180 python tools/band_throughput.py --b 512 --g 4 --reps 10 --ell $e > gpurun_out/${TAG}_tp.tmp 2>&1 \
    || { tail -5 gpurun_out/${TAG}_tp.tmp; exit 1; }
  echo "$e $(tail -1 gpurun_out/${TAG}_tp.tmp)" | tee -a gpurun_out/${TAG}_throughput.txt | cut -c1-200
done
