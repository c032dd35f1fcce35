#!/usr/bin/env bash
# k_bounce occupancy on khaslana 1600^2 d12 (LDS pad: 6 -> 5 / 4 / 3 blocks per CU), bunny baseline
set -u
cd "$(dirname "$0")/.."
AB_TAG=occ_khaslana AB_ROUNDS=3 AB_ENVS="PT_BOUNCE_LDS_PAD=0;PT_BOUNCE_LDS_PAD=1024;PT_BOUNCE_LDS_PAD=6000;PT_BOUNCE_LDS_PAD=14000" \
  AB_ARGS="--scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12 --steps 20 --warmup 5" bash tools/ab_env.sh && \
AB_TAG=occ_bunny AB_ROUNDS=3 AB_ENVS="PT_BOUNCE_LDS_PAD=0;PT_BOUNCE_LDS_PAD=3000" \
  AB_ARGS="--scene scenes/cornell_obj_bnnuy.json --steps 20 --warmup 5" bash tools/ab_env.sh
