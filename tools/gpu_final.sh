#!/bin/bash
# The round's closing GPU pass in one call: the gates (tools/gpu_check.sh: pytest -m gpu, smoke,
# the default bench line) and then the profiles (tools/profile_round4.sh without its own bench).
# usage: tools/gpu_final.sh TAG
TAG=${1:-r04z}
bash tools/gpu_check.sh "$TAG" && SKIP_BENCH=1 bash tools/profile_round4.sh "$TAG"
