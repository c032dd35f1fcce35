"""The scene loader's PNG decoder (host/png_decode.cpp; the reference uses stbi_load with
STBI_rgb_alpha, scene.cpp:366-392) against an independent decoder (Pillow) on PNGs of every
colour type / bit depth, compression level and filter choice; expected RGBA follows
stb_image's conversion rules (grey -> g,g,g,255; 16-bit keeps the high byte; palette + tRNS)."""
import os
import sys

import numpy as np
import pytest

from conftest import PKG

PIL = pytest.importorskip("PIL.Image")


def _ptamd():
    sys.path.insert(0, PKG)
    import ptamd
    return ptamd


def _img(h=37, w=53, c=3, seed=0):
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:h, 0:w]
    base = np.stack([(x * 5 + y * 3 + k * 40) % 256 for k in range(c)], -1)
    noise = rng.integers(0, 256, (h, w, c))
    return np.where(rng.random((h, w, 1)) < 0.3, noise, base).astype(np.uint8)


@pytest.mark.parametrize("mode", ["RGB", "RGBA", "L", "LA", "P", "PT", "1"])
@pytest.mark.parametrize("level", [0, 1, 9])
def test_png_modes_match_pillow(mode, level, tmp_path):
    ptamd = _ptamd()
    if mode in ("RGB", "RGBA"):
        im = PIL.fromarray(_img(c=len(mode)), mode)
    elif mode == "L":
        im = PIL.fromarray(_img(c=1)[..., 0], "L")
    elif mode == "LA":
        im = PIL.fromarray(_img(c=2), "LA")
    elif mode == "1":
        im = PIL.fromarray(_img(c=1)[..., 0] > 127)
    else:
        im = PIL.fromarray(_img(c=3), "RGB").quantize(colors=50)
    path = str(tmp_path / f"t_{mode}_{level}.png")
    kw = {"compress_level": level}
    if mode == "PT":
        kw["transparency"] = bytes(range(0, 250, 5))     # per-palette-entry alpha (tRNS)
    im.save(path, **kw)
    got = ptamd.load_texture(path)
    want = np.asarray(PIL.open(path).convert("RGBA"))
    assert got.shape == want.shape
    assert np.array_equal(got, want)


def test_png_16bit_keeps_high_byte(tmp_path):
    ptamd = _ptamd()
    rng = np.random.default_rng(3)
    a = rng.integers(0, 65536, (21, 17), dtype=np.uint16)
    path = str(tmp_path / "g16.png")
    PIL.fromarray(a.astype(np.int32), "I").convert("I;16").save(path)
    raw = np.asarray(PIL.open(path)).astype(np.uint16)      # the stored 16-bit samples
    got = ptamd.load_texture(path)
    g = (raw >> 8).astype(np.uint8)
    assert np.array_equal(got[..., 0], g) and np.array_equal(got[..., 1], g) and np.array_equal(got[..., 2], g)
    assert (got[..., 3] == 255).all()


def test_png_errors(tmp_path):
    ptamd = _ptamd()
    with pytest.raises(ptamd.PtError):
        ptamd.load_texture(str(tmp_path / "missing.png"))
    bad = tmp_path / "bad.png"
    bad.write_bytes(b"\x89PNG\r\n\x1a\n" + b"\x00" * 20)
    with pytest.raises(ptamd.PtError):
        ptamd.load_texture(str(bad))
    im = PIL.fromarray(_img(), "RGB")
    good = tmp_path / "trunc.png"
    im.save(good)
    data = good.read_bytes()
    good.write_bytes(data[: len(data) // 2])
    with pytest.raises(ptamd.PtError):
        ptamd.load_texture(str(good))


def _png_chunk(tag, body):
    import struct
    import zlib
    return struct.pack(">I", len(body)) + tag + body + struct.pack(">I", zlib.crc32(tag + body) & 0xffffffff)


@pytest.mark.parametrize("w,h", [(13, 11), (1, 1), (9, 3), (33, 17)])
def test_png_adam7_interlaced(w, h, tmp_path):
    """Adam7 interlacing (Pillow cannot write it): hand-built RGB PNG, filters cycling 0..4."""
    import struct
    import zlib
    ptamd = _ptamd()
    img = _img(h, w, 3, seed=w * h)
    xo, yo, xs, ys = [0, 4, 0, 2, 0, 1, 0], [0, 0, 4, 0, 2, 0, 1], [8, 8, 4, 4, 2, 2, 1], [8, 8, 8, 4, 4, 2, 2]
    raw = bytearray()
    ftype = 0
    for p in range(7):
        sub = img[yo[p]::ys[p], xo[p]::xs[p]]
        if sub.size == 0:
            continue
        prev = np.zeros(sub.shape[1] * 3, np.int32)
        for row in sub:
            cur = row.reshape(-1).astype(np.int32)
            left = np.concatenate([np.zeros(3, np.int32), cur[:-3]])
            upleft = np.concatenate([np.zeros(3, np.int32), prev[:-3]])
            if ftype == 0:
                f = cur
            elif ftype == 1:
                f = cur - left
            elif ftype == 2:
                f = cur - prev
            elif ftype == 3:
                f = cur - (left + prev) // 2
            else:
                pa, pb, pc = abs(prev - upleft), abs(left - upleft), abs(left + prev - 2 * upleft)
                pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, upleft))
                f = cur - pred
            raw += bytes([ftype]) + bytes((f % 256).astype(np.uint8))
            prev = cur
            ftype = (ftype + 1) % 5
    png = b"\x89PNG\r\n\x1a\n" + _png_chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 1))
    png += _png_chunk(b"IDAT", zlib.compress(bytes(raw), 6)) + _png_chunk(b"IEND", b"")
    path = tmp_path / "i.png"
    path.write_bytes(png)
    got = ptamd.load_texture(str(path))
    assert np.array_equal(got[..., :3], img) and (got[..., 3] == 255).all()


REF_TEX = "/root/reference/scenes/textures"


@pytest.mark.skipif(not os.path.isdir(REF_TEX), reason="reference checkout not present (GPU box)")
def test_reference_textures_match_pillow():
    """The PNG textures the reference's scenes name, decoded by both decoders."""
    ptamd = _ptamd()
    pngs = [f for f in sorted(os.listdir(REF_TEX)) if f.endswith(".png")]
    assert pngs
    for f in pngs:
        got = ptamd.load_texture(os.path.join(REF_TEX, f))
        want = np.asarray(PIL.open(os.path.join(REF_TEX, f)).convert("RGBA"))
        assert np.array_equal(got, want), f
