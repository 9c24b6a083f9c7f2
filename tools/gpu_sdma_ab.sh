#!/bin/bash
# Copies through the SDMA engines (default) or as blit kernels on the streams' own queues.
TAG=${1:-sdab}
bash tools/ab_env.sh $TAG "HSA_ENABLE_SDMA=1" "HSA_ENABLE_SDMA=0" "HSA_ENABLE_SDMA=1" "HSA_ENABLE_SDMA=0"
