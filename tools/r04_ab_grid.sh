set -u
cd /root/repo
AB_TAG=cornell AB_ROUNDS=3 AB_ENVS="PT_GRID=-1;PT_GRID=1" bash tools/ab_env.sh && \
AB_TAG=bunny AB_ROUNDS=3 AB_ENVS="PT_GRID=-1;PT_GRID=1" AB_ARGS="--scene scenes/cornell_obj_bnnuy.json" bash tools/ab_env.sh
