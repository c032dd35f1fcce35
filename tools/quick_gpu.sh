set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
[ -n "${NO_SEC:-}" ] || timeout -k 10 300 python tools/section_times.py > gpurun_out/sec.log 2>&1 || exit 3
timeout -k 10 300 python tools/ab_variants.py --variants ${AB_VARIANTS:-2} --fpp ${AB_FPP:-8} --rounds 3 --pipeline ${AB_PIPELINE:-0} > gpurun_out/ab0.log 2>&1 || exit 4
python3 - <<'PY'
import json
import os
if not os.environ.get("NO_SEC"): d=json.load(open("gpurun_out/sec.log")); print(d["cycle_share"], d["exact_tests_per_live_lane"], d["loop_iters_per_wave"])
d=json.load(open("gpurun_out/ab0.log"))
for k,v in d["results"].items(): print(k, round(v["ms_per_frame_median"],4), v["per_launch_bounce_ms_then_frame_ms_combine_ms"])
PY
