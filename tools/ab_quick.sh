set -u
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -20 gpurun_out/b.log; exit 2; }
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('headline', d['ms_per_step'], d['kernels']['per_launch_bounce_ms'])"
bash tools/bvh_check.sh
