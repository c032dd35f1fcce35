#!/usr/bin/env bash
# GPU box: full parity suite, the headline bench line, then the mesh configs (tools/bvh_check.sh).
# Every GPU step has its own time limit; a failing step ends the script.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 2; }
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline', d['ms_per_step'], d['value'], d['roofline']['frac'], d['kernels']['per_launch_bounce_ms'])"
bash tools/bvh_check.sh
