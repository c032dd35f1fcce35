#!/usr/bin/env bash
# Round-4 GPU session: tools/r04_session.sh STEP...  (steps: new, gpu, bench, bench100, profiles)
# Each step has its own time limit; a failure other than test failures stops the session.
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
    tail -n 5 "$OUT/$name.log"
    echo "== $name rc=$rc =="
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name rc=$rc"; exit $rc; fi
    return 0
}
PYT="python -u -m pytest -x -q -rf --timeout 200 --timeout-method thread -p no:cacheprovider"
for s in "$@"; do
    case $s in
        new) step pytest_new 400 $PYT tests/test_multi_device.py tests/test_dropin.py -m gpu ;;
        gpu) step pytest_gpu 700 $PYT tests -m gpu ;;
        bench) step bench_k20 300 python bench.py --steps 20 --warmup 5 ;;
        bench100) step bench 300 python bench.py --steps 100 --warmup 10 ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
echo "session done"
