set -u
export PT_BVH_TREE_INFO=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "bnnuy or khaslana or phatphuck or skewed or mesh or bvh or intersections_match" > gpurun_out/r03_sah_tests.log 2>&1; rc=$?; tail -5 gpurun_out/r03_sah_tests.log; [ $rc -eq 0 ] || exit $rc
AB_TAG=sah_bunny AB_ROUNDS=3 AB_ENVS="PT_BVH_TREE=ref;PT_BVH_TREE=sah" AB_ARGS="--steps 48 --warmup 4 --scene scenes/cornell_obj_bnnuy.json" timeout -k 10 400 bash tools/ab_env.sh || exit 5
AB_TAG=sah_khaslana AB_ROUNDS=3 AB_ENVS="PT_BVH_TREE=ref;PT_BVH_TREE=sah" AB_ARGS="--steps 32 --warmup 2 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12" timeout -k 10 400 bash tools/ab_env.sh || exit 6
