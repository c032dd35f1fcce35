#!/usr/bin/env bash
# BASELINE configs 2-5 on one GPU (fused and staged), one bench line each -> gpurun_out/configs.jsonl
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p "$OUT"
: > "$OUT/configs.jsonl"
run() {   # run TAG ARGS...
    local tag=$1; shift
    timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/cfg_$tag.log" 2>&1
    local rc=$?
    if [ $rc -ne 0 ]; then echo "$tag rc=$rc"; tail -5 "$OUT/cfg_$tag.log"; exit $rc; fi
    tail -1 "$OUT/cfg_$tag.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); d['tag']='$tag'; print(json.dumps(d))" >> "$OUT/configs.jsonl"
    echo "$tag ok"
}
run c2_fused   --steps 100 --warmup 10
run c2_staged  --steps 100 --warmup 10 --pipeline staged
run c3_fused   --steps 100 --warmup 10 --scene scenes/cornell_glass_test.json
run c3_staged  --steps 100 --warmup 10 --scene scenes/cornell_glass_test.json --sort --pipeline staged
run c4_fused   --steps 50 --warmup 8 --scene scenes/cornell_obj_bnnuy.json
run c4_staged  --steps 50 --warmup 8 --scene scenes/cornell_obj_bnnuy.json --pipeline staged
run c5_fused   --steps 16 --warmup 4 --scene scenes/cornell_obj_khaslana.json --res 1600x1600 --depth 12
echo "configs done"
