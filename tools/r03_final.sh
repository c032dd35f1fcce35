#!/usr/bin/env bash
# Round-3 end-of-round session on the final build: GPU parity suite, the driver-shaped and the
# default bench lines, rocprofv3 kernel stats + PMC digests + section counters
# (tools/r03_profiles.sh), the VALU attribution (tools/valu_attrib.sh).  Each step has its own
# time limit; a failure other than test failures stops the session.
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
    tail -n 3 "$OUT/$name.log"
    echo "== $name rc=$rc =="
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
    return 0
}
step pytest_gpu 500 python -u -m pytest tests -m gpu -x -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider
step bench_k20 300 python bench.py --steps 20 --warmup 5
step bench 300 python bench.py --steps 100 --warmup 10
step profiles 600 bash tools/r03_profiles.sh all
step valu 300 bash tools/valu_attrib.sh
echo "final session done"
