#!/usr/bin/env bash
# GPU parity suite on the current build, then the headline / bunny / khaslana A/B over AB_LIBS3
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/par.log 2>&1
rc=$?; tail -3 gpurun_out/par.log; [ $rc -eq 0 ] || exit 1
bash tools/ab_three.sh
