"""Re-serialises the reference's scene files (data, /root/reference/scenes/*.json) into
scenes/ so the GPU box (which has no /root/reference) has the same inputs.

The values are untouched (json round-trips every number exactly); objects are written
compactly, one top-level section per line, with material keys sorted (their order never
mattered: nlohmann::json objects are std::maps, scene.cpp:53).  Run once in this container:
    python tools/import_scenes.py
"""
import glob
import json
import os
import sys

REF = os.environ.get("REF", "/root/reference")
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scenes")


def main():
    os.makedirs(DST, exist_ok=True)
    for path in sorted(glob.glob(os.path.join(REF, "scenes", "*.json"))):
        with open(path) as f:
            data = json.load(f)
        out = os.path.join(DST, os.path.basename(path))
        with open(out, "w") as f:
            f.write("{\n")
            keys = ["Camera", "Materials", "Objects"] + [k for k in data if k not in ("Camera", "Materials", "Objects")]
            keys = [k for k in keys if k in data]
            for i, k in enumerate(keys):
                v = data[k]
                if k == "Materials":
                    body = "{" + ",\n  ".join(json.dumps(n) + ":" + json.dumps(v[n], sort_keys=True, separators=(",", ":"))
                                             for n in sorted(v)) + "}"
                elif k == "Objects":
                    body = "[" + ",\n  ".join(json.dumps(o, sort_keys=True, separators=(",", ":")) for o in v) + "]"
                else:
                    body = json.dumps(v, sort_keys=True, separators=(",", ":"))
                f.write(f" {json.dumps(k)}:{body}{',' if i + 1 < len(keys) else ''}\n")
            f.write("}\n")
        with open(out) as f:
            assert json.load(f) == data, out
    print(f"imported {len(glob.glob(os.path.join(DST, '*.json')))} scenes into {os.path.abspath(DST)}", file=sys.stderr)


if __name__ == "__main__":
    main()
