set -u
cd $GRAFT_REPO_ROOT 2>/dev/null || cd /root/repo
B="python bench.py --steps 400 --warmup 20 --no-cpu-baseline --no-configs --no-api --no-spread"
timeout -k 10 200 $B > gpurun_out/single.json 2>/dev/null || exit 2
( timeout -k 10 200 $B > gpurun_out/c1.json 2>/dev/null ) &
p1=$!
( timeout -k 10 200 $B > gpurun_out/c2.json 2>/dev/null ) &
p2=$!
wait $p1; wait $p2
python3 - <<'PY'
import json
for f in ("single","c1","c2"):
    d=json.loads(open("gpurun_out/%s.json"%f).read().strip().splitlines()[-1]); print(f, d["ms_per_step"], d["value"])
PY
