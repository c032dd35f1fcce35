#!/usr/bin/env bash
# Round-3 GPU session: full GPU parity suite, the default bench line (headline + api + configs
# sub-records + cpu baseline) and a rocprofv3 kernel-trace summary of the bench.  Each GPU step
# has its own time limit; a failure other than test failures stops the session.
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
    tail -n 15 "$OUT/$name.log"
    echo "== $name rc=$rc =="
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = tests ]; then
    step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"}
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench_k20 300 python bench.py --steps 20 --warmup 5
    cp "$OUT/bench_k20.log" "$OUT/bench_k20.json" 2>/dev/null
    step bench 300 python bench.py --steps 100 --warmup 10
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 240 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-configs --no-api
fi
echo "session done"
