"""Generates tests/golden/corrupt/: truncated or corrupt scene JSON, OBJ and PNG files for the
sanitizer build of the host ingest (tests/test_sanitized_ingest.py).  Deterministic; the files are
committed.  Naming: bad_* must be refused (PT_E_INVALID, or texture id -1 for a scene whose texture
is bad), ok_* must load; nothing may produce a sanitizer report.

    python tests/golden/make_corrupt_corpus.py
"""
import json
import os
import struct
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "corrupt")
REPO = os.path.dirname(os.path.dirname(HERE))


def w(name, data):
    with open(os.path.join(OUT, name), "wb") as f:
        f.write(data if isinstance(data, bytes) else data.encode())


def png(width, height, ctype, depth, rows, interlace=0, plte=None, extra=b"", zdata=None, ihdr=None):
    def chunk(t, b):
        return struct.pack(">I", len(b)) + t + b + struct.pack(">I", zlib.crc32(t + b) & 0xffffffff)
    hd = ihdr if ihdr is not None else struct.pack(">IIBBBBB", width, height, depth, ctype, 0, 0, interlace)
    body = chunk(b"IHDR", hd)
    if plte is not None:
        body += chunk(b"PLTE", plte)
    body += extra
    body += chunk(b"IDAT", zdata if zdata is not None else zlib.compress(rows, 9))
    return b"\x89PNG\r\n\x1a\n" + body + chunk(b"IEND", b"")


def main():
    os.makedirs(OUT, exist_ok=True)
    for f in os.listdir(OUT):
        os.remove(os.path.join(OUT, f))
    # ---- PNG ----
    rows = b"".join(b"\x00" + bytes((x * 16 + y) & 255 for x in range(16 * 4)) for y in range(16))
    good = png(16, 16, 6, 8, rows)
    w("ok_rgba16.png", good)
    for k in (8, 20, 33, 40, len(good) // 2, len(good) - 13):
        w(f"bad_trunc_{k}.png", good[:k])
    w("ok_trunc_iend_crc.png", good[:-1])   # stb_image stops at IEND's type, before its CRC
    w("bad_signature.png", b"\x89PNX" + good[4:])
    w("bad_ihdr_len.png", png(16, 16, 6, 8, rows, ihdr=struct.pack(">IIBBBB", 16, 16, 8, 6, 0, 0)))
    w("bad_width0.png", png(0, 16, 6, 8, rows))
    w("bad_width_huge.png", png(1 << 31, 16, 6, 8, rows))
    w("bad_dims_bomb.png", png(16384, 16384, 6, 8, rows))      # 1 GiB promised, 1 KiB given
    w("bad_depth3.png", png(16, 16, 6, 3, rows))
    w("bad_ctype5.png", png(16, 16, 5, 8, rows))
    w("bad_palette_missing.png", png(16, 16, 3, 8, b"".join(b"\x00" + bytes(16) for _ in range(16))))
    prow = b"".join(b"\x00" + bytes((x * 7) & 255 for x in range(16)) for _ in range(16))
    w("bad_palette_index.png", png(16, 16, 3, 8, prow, plte=bytes(3 * 4)))
    w("ok_palette.png", png(16, 16, 3, 8, prow, plte=bytes(range(256)) * 3))
    w("bad_filter7.png", png(16, 16, 6, 8, b"\x07" + rows[1:]))
    w("bad_zlib_header.png", png(16, 16, 6, 8, rows, zdata=b"\x78\x00" + zlib.compress(rows)[2:]))
    w("bad_zlib_garbage.png", png(16, 16, 6, 8, rows, zdata=b"\x78\x9c" + bytes(range(200))))
    w("bad_inflate_bomb.png", png(16, 16, 6, 8, rows, zdata=zlib.compress(bytes(64 << 20), 9)))
    w("bad_short_data.png", png(16, 16, 6, 8, rows[: len(rows) // 3]))
    irow = bytes(16 * 16 * 4 + 16 * 2)
    w("bad_interlaced_short.png", png(16, 16, 6, 8, irow[:100], interlace=1))
    w("bad_interlace2.png", png(16, 16, 6, 8, rows, interlace=2))
    w("ok_bad_crc.png", good[:29] + b"\x00\x00\x00\x00" + good[33:])   # CRCs are not checked (stb_image)
    w("bad_empty.png", b"")
    w("bad_chunk_len.png", good[:8] + b"\xff\xff\xff\xf0" + good[12:])
    # ---- OBJ ----
    tri = "v 0 0 0\nv 1 0 0\nv 0 1 0\nv 1 1 0\nvt 0 0\nvn 0 0 1\n"
    w("ok_tri.obj", tri + "f 1 2 3\n")
    w("ok_quad.obj", tri + "f 1/1/1 2/1/1 4/1/1 3/1/1\n")
    w("ok_ngon.obj", tri + "f " + " ".join(str(1 + i % 4) for i in range(100)) + "\n")
    w("ok_missing_refs.obj", tri + "f 1/9/9 2//7 3/5\n")           # bad vt / vn: zero uv, face normal
    w("ok_nan.obj", "v nan inf -inf\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    w("ok_two_coords.obj", "v 1 2\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    w("ok_garbage_coords.obj", "v a b c\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    w("ok_short_face.obj", tri + "f 1 2\nf 1 2 3\n")
    w("bad_index0.obj", tri + "f 0 1 2\n")
    w("bad_index_big.obj", tri + "f 1 2 99\n")
    w("bad_index_neg.obj", tri + "f -1 -2 -9\n")
    w("bad_quad_index.obj", tri + "f 1 2 3 77\n")                   # the quad split reads positions first
    w("bad_index_huge.obj", tri + "f 1 2 99999999999999999999\n")
    w("ok_long_line.obj", tri + "# " + "x" * (1 << 20) + "\nf 1 2 3\n")
    w("ok_empty.obj", "")
    w("ok_binary.obj", bytes(range(256)) * 16)
    # ---- scene JSON ----
    with open(os.path.join(REPO, "scenes", "cornell.json")) as f:
        base = f.read()
    d = json.loads(base)
    w("ok_cornell.json", base)
    for frac in (0.0, 0.1, 0.5, 0.9):
        w(f"bad_trunc_{int(frac * 100)}.json", base[: int(len(base) * frac)])
    w("bad_trunc_last.json", base.rstrip()[:-1])
    w("bad_deep_nest.json", '{"Materials": ' + "[" * 100000 + "]" * 100000 + "}")
    w("bad_whitespace.json", "   \n\t ")
    w("bad_bom.json", "﻿" + base)
    w("bad_nul.json", base[:50] + "\x00" + base[50:])
    w("bad_trailing.json", base + "}")
    w("bad_unterminated_string.json", '{"Materials": {"a')
    w("bad_escape_end.json", '{"Materials": {"a\\')
    w("bad_u_escape.json", '{"Materials": {"\\u12')
    w("bad_nan_token.json", base.replace('"DEPTH":8', '"DEPTH":NaN'))

    def variant(name, f):
        v = json.loads(base)
        f(v)
        w(name, json.dumps(v).replace("Infinity", "1e999"))
    variant("bad_depth_string.json", lambda v: v["Camera"].__setitem__("DEPTH", "eight"))
    variant("bad_depth_inf.json", lambda v: v["Camera"].__setitem__("DEPTH", float("inf")))
    variant("bad_depth_huge_float.json", lambda v: v["Camera"].__setitem__("DEPTH", 1e300))
    variant("bad_res_short.json", lambda v: v["Camera"].__setitem__("RES", [800]))
    variant("bad_res_string.json", lambda v: v["Camera"].__setitem__("RES", "800x800"))
    variant("bad_res_negative.json", lambda v: v["Camera"].__setitem__("RES", [-5, 800]))
    variant("bad_res_huge.json", lambda v: v["Camera"].__setitem__("RES", [100000, 100000]))
    variant("bad_res_float_huge.json", lambda v: v["Camera"].__setitem__("RES", [1e20, 800]))
    variant("bad_fovy_null.json", lambda v: v["Camera"].__setitem__("FOVY", None))
    variant("bad_eye_short.json", lambda v: v["Camera"].__setitem__("EYE", [1, 2]))
    variant("bad_no_camera.json", lambda v: v.pop("Camera"))
    variant("bad_no_materials.json", lambda v: v.pop("Materials"))
    variant("bad_objects_object.json", lambda v: v.__setitem__("Objects", {"a": 1}))
    variant("bad_object_number.json", lambda v: v["Objects"].append(5))
    variant("bad_object_no_type.json", lambda v: v["Objects"][0].pop("TYPE"))
    variant("bad_material_number.json", lambda v: v["Objects"][0].__setitem__("MATERIAL", 5))
    variant("ok_material_unknown.json", lambda v: v["Objects"][0].__setitem__("MATERIAL", "nope"))
    variant("ok_huge_int.json", lambda v: v["Camera"].__setitem__("ITERATIONS", 99999999999999999999))
    variant("ok_eye_overflow.json", lambda v: v["Camera"].__setitem__("EYE", [1e39, 0, 0]))
    variant("ok_scale_zero.json", lambda v: v["Objects"][0].__setitem__("SCALE", [0, 0, 0]))
    variant("ok_res_tiny.json", lambda v: v["Camera"].__setitem__("RES", [1, 1]))
    for obj in sorted(f for f in os.listdir(OUT) if f.endswith(".obj")):
        def add(v, obj=obj):
            v["Objects"].append({"TYPE": "obj", "PATH": "/" + obj, "MATERIAL": "diffuse_red",
                                 "TRANS": [0, 0, 0], "ROTAT": [0, 0, 0], "SCALE": [1, 1, 1]})
        tag = obj[:-4]
        variant(("bad_" if tag.startswith("bad_") else "ok_") + "scene_" + tag.split("_", 1)[1] + ".json", add)
    variant("bad_scene_obj_missing.json", lambda v: v["Objects"].append(
        {"TYPE": "obj", "PATH": "/not_there.obj", "MATERIAL": "diffuse_red", "TRANS": [0, 0, 0],
         "ROTAT": [0, 0, 0], "SCALE": [1, 1, 1]}))
    for p in sorted(f for f in os.listdir(OUT) if f.endswith(".png")):
        def tex(v, p=p):
            v["Materials"]["diffuse_red"]["TEXTURE"] = p
        tag = p[:-4]
        variant(("badtex_" if tag.startswith("bad_") else "ok_") + "scene_tex_" + tag.split("_", 1)[1] + ".json", tex)
    variant("bad_bump_no_scale.json", lambda v: v["Materials"]["diffuse_red"].__setitem__("BUMP_MAP", "ok_rgba16.png"))
    print(len(os.listdir(OUT)), "files in", OUT)


if __name__ == "__main__":
    main()
