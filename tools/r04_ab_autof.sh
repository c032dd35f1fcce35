#!/usr/bin/env bash
# Pass size against the 256 MB Infinity Cache: cornell with the auto pass size's path target at
# 2.56 M (F = 4: both path buffers fit the cache) .. 82 M (F = 128, the default)
set -u
cd "$(dirname "$0")/.."
AB_TAG=autof AB_ROUNDS=3 AB_ENVS="PT_AUTO_PATHS=2560000;PT_AUTO_PATHS=5120000;PT_AUTO_PATHS=20480000;PT_AUTO_PATHS=83886080" \
  AB_ARGS="--steps 40 --warmup 8" bash tools/ab_env.sh
