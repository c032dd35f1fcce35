#!/usr/bin/env bash
# fused material grouping: parity frames, then A/B sort on / off (fused) and staged + sort
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
    -k "material_sort or frames_bitexact or multi_frame" > gpurun_out/r03_mg_tests.log 2>&1; rc=$?; tail -4 gpurun_out/r03_mg_tests.log; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import json, os, subprocess, sys, statistics as st
res = {}
for scene, res_, depth, steps in [("cornell_glass_test", None, None, 48), ("cornell_multiple_glass", None, None, 48),
                                  ("cornell_obj_khaslana", "1600x1600", 12, 32)]:
    for rnd in range(3):
        for name, extra in [("fused", []), ("fused_sort", ["--sort"]), ("staged_sort", ["--sort", "--pipeline", "staged"])]:
            cmd = [sys.executable, "bench.py", "--no-cpu-baseline", "--no-configs", "--no-api", "--no-spread",
                   "--scene", f"scenes/{scene}.json", "--steps", str(steps), "--warmup", "4"] + extra
            if res_: cmd += ["--res", res_, "--depth", str(depth)]
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(out.stderr[-2000:]); sys.exit(3)
            line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
            res.setdefault(scene, {}).setdefault(name, []).append(line["ms_per_step"])
for s, d in res.items():
    print(s, {k: (round(st.median(v), 4), v) for k, v in d.items()})
json.dump(res, open("gpurun_out/r03_mg_ab.json", "w"), indent=1)
PY
