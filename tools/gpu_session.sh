#!/usr/bin/env bash
# One GPU-box session: GPU parity tests, the bench line, a rocprofv3 kernel-trace summary.
# Each GPU step has its own time limit; a fault / abort / timeout stops the session.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {   # step NAME TIMEOUT CMD...
    local name=$1 to=$2; shift 2
    echo "== $name (timeout ${to}s) =="
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    tail -n 25 "$OUT/$name.log"
    echo "== $name rc=$rc =="
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
    step pytest_gpu 900 python -m pytest tests -m gpu -q -rf --timeout 300 -p no:cacheprovider
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py --steps 100 --warmup 10
    step bench_staged 600 python bench.py --steps 100 --warmup 10 --pipeline staged --no-cpu-baseline
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python bench.py --steps 100 --warmup 10 --no-cpu-baseline
    step rocprof_staged 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_staged" -o run --output-format csv -- \
        python bench.py --steps 100 --warmup 10 --no-cpu-baseline --pipeline staged
fi
if [ "$MODE" = all ] || [ "$MODE" = pmc ]; then
    step pmc_fused 900 env PMC_TAG=fused_ bash tools/pmc.sh
    step pmc_staged 900 env PMC_TAG=staged_ PMC_SETS="FETCH_SIZE;WRITE_SIZE" bash tools/pmc.sh --pipeline staged
fi
echo "session done"
