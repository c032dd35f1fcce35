#!/usr/bin/env bash
# Builds the reference-pin harnesses into oracle/_ref/ (git-ignored) and regenerates the
# committed fixtures under tests/golden/.  Needs /root/reference (this container only).
#   rng_pin     : hipcc host build against rocThrust (the reference's RNG dependency)
#   ingest_pin  : g++ build of the reference's own src/utilities.cpp + vendored glm / json
set -euo pipefail
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
REPO="$(cd "$HERE/../.." && pwd)"
REF="${REF:-/root/reference}"
OUT="$REPO/oracle/_ref"
GOLD="$REPO/tests/golden"
mkdir -p "$OUT" "$GOLD"
hipcc -O1 -x hip --offload-arch=gfx950 "$HERE/rng_pin.cpp" -o "$OUT/rng_pin"
g++ -std=c++17 -O2 -I "$REF/src" -I "$REF/external/include" "$HERE/ingest_pin.cpp" "$REF/src/utilities.cpp" \
    -o "$OUT/ingest_pin"
"$OUT/rng_pin" > "$GOLD/rng_pin.json"
SCENES=$(ls "$REF"/scenes/*.json)
"$OUT/ingest_pin" $SCENES | python3 -c '
import json, os, sys
d = json.load(sys.stdin)
d["scenes"] = {os.path.basename(k): v for k, v in d["scenes"].items()}
json.dump(d, sys.stdout, separators=(",", ":"))
' > "$GOLD/ingest_pin.json"
echo "fixtures written: $GOLD/rng_pin.json $GOLD/ingest_pin.json"
# ref_harness: the reference's own intersections.cu / scene.cpp / utilities.cpp / stb.cpp / image.cpp,
# compiled in place with g++ against the CUDA runtime headers shipped in this image (real headers,
# no stand-ins; the .cu file is plain host C++ under -x c++).  Unbuildable without those headers.
CUDAINC="${CUDAINC:-/usr/local/lib/python3.10/dist-packages/triton/backends/nvidia/include}"
if [ -f "$CUDAINC/cuda_runtime.h" ]; then
    if [ ! -x "$OUT/ref_harness" ] || [ "$HERE/ref_harness.cpp" -nt "$OUT/ref_harness" ]; then
        g++ -std=c++17 -O2 -ffp-contract=off -w -I "$CUDAINC" -I "$REF/src" -I "$REF/external/include" \
            -x c++ "$REF/src/intersections.cu" -x none "$REF/src/scene.cpp" "$REF/src/utilities.cpp" \
            "$REF/src/stb.cpp" "$REF/src/image.cpp" "$HERE/ref_harness.cpp" -o "$OUT/ref_harness"
    fi
    python3 "$HERE/make_ref_fixtures.py" "$OUT/ref_harness" "$GOLD/ref_pin.json"
else
    echo "ref_harness skipped: no CUDA runtime headers at $CUDAINC"
fi
# dropin_main: a main.cpp-shaped caller compiled against the reference's own headers and host
# sources (Scene from scene.cpp) + the drop-in (project3-cuda-path-tracer-2025_amd/dropin/pathtrace.cpp),
# linked against libptamd.so -- proves the drop-in links behind main.cpp's calls
PKGDIR="$REPO/project3-cuda-path-tracer-2025_amd"
if [ -f "$CUDAINC/cuda_runtime.h" ] && [ -f "$PKGDIR/build/libptamd.so" ]; then
    g++ -std=c++17 -O2 -ffp-contract=off -w -I "$CUDAINC" -I "$REF/src" -I "$REF/external/include" -I "$REPO/include" \
        "$HERE/dropin_main.cpp" "$PKGDIR/dropin/pathtrace.cpp" "$REF/src/scene.cpp" "$REF/src/utilities.cpp" \
        "$REF/src/stb.cpp" -L "$PKGDIR/build" -lptamd -Wl,-rpath,'$ORIGIN/../../project3-cuda-path-tracer-2025_amd/build' \
        -o "$OUT/dropin_main"
    echo "drop-in caller built: $OUT/dropin_main"
fi
# viewer_pin: main.cpp's camera controls restated on the reference's own Scene (scene.cpp) and glm,
# replaying tests/golden/viewer_events.txt -> tests/golden/viewer_pin.json (headless viewer, pt_viewer.h)
if [ -f "$CUDAINC/cuda_runtime.h" ]; then
    g++ -std=c++17 -O2 -ffp-contract=off -w -I "$CUDAINC" -I "$REF/src" -I "$REF/external/include" \
        "$HERE/viewer_pin.cpp" "$REF/src/scene.cpp" "$REF/src/utilities.cpp" "$REF/src/stb.cpp" -o "$OUT/viewer_pin"
    {
        echo '{"events": "viewer_events.txt", "scenes": {'
        echo '"cornell.json": '; "$OUT/viewer_pin" "$REF/scenes/cornell.json" "$GOLD/viewer_events.txt" | sed -n '/^{"frames"/,$p'
        echo ', "viewer_scene.json": '; "$OUT/viewer_pin" "$GOLD/viewer_scene.json" "$GOLD/viewer_events.txt" | sed -n '/^{"frames"/,$p'
        echo '}}'
    } | python3 -c 'import json, sys; json.dump(json.load(sys.stdin), sys.stdout, separators=(",", ":"))' \
        > "$GOLD/viewer_pin.json"
    echo "viewer fixtures: $GOLD/viewer_pin.json"
fi
