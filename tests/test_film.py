"""The output side (viewer.cpp:109-132, image.cpp:24-58): the display tonemap
against the oracle's restatement (bit-exact), the PNG / BMP writers decoded
back, progressive accumulation, and progressive passes of the device path code
(sample_offset) against one call with all samples."""
import struct
import zlib

import numpy as np
import pytest

import first_raytracer_amd as frt
import oracle


def test_tonemap_matches_oracle():
    rng = np.random.default_rng(3)
    film = np.concatenate([rng.random(3000) * 0.05, rng.random(3000) * 4.0, [0.0, 1e-9, 30.0, 1e3]]).astype(np.float32)
    film = np.pad(film, (0, (-len(film)) % 3)).reshape(1, -1, 3)
    got = frt.tonemap_u8(film)
    want = np.zeros(film.size, np.uint8)
    oracle.lib().ora_tonemap_u8(oracle.darr(film.reshape(-1).astype(np.float64))[1], film.size, want.ctypes.data)
    assert np.array_equal(got.reshape(-1), want)


def read_png(path):
    b = open(path, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w, h = 8, b"", None, None
    while pos < len(b):
        n, = struct.unpack(">I", b[pos:pos + 4]); t = b[pos + 4:pos + 8]; d = b[pos + 8:pos + 8 + n]
        assert struct.unpack(">I", b[pos + 8 + n:pos + 12 + n])[0] == zlib.crc32(t + d)
        if t == b"IHDR":
            w, h, depth, ctype = struct.unpack(">IIBB", d[:10])
            assert (depth, ctype) == (8, 2)
        elif t == b"IDAT":
            idat += d
        pos += 12 + n
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    assert (raw[:, 0] == 0).all()
    return raw[:, 1:].reshape(h, w, 3)


def test_png_and_bmp_roundtrip(tmp_path):
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (37, 53, 3), dtype=np.uint8)          # y = 0 bottom row
    frt.write_image(str(tmp_path / "a"), img, "png")                  # extension appended (image.cpp:42)
    png = read_png(str(tmp_path / "a.png"))
    assert np.array_equal(png, img[::-1])                              # top-down rows (flip on write)
    frt.write_image(str(tmp_path / "b.bmp"), img, "bmp")
    b = open(str(tmp_path / "b.bmp"), "rb").read()
    assert b[:2] == b"BM" and struct.unpack("<ii", b[18:26]) == (53, 37)
    row = (3 * 53 + 3) & ~3
    pix = np.frombuffer(b[54:], np.uint8).reshape(37, row)[:, :3 * 53].reshape(37, 53, 3)[:, :, ::-1]
    assert np.array_equal(pix, img)                                    # bottom-up rows = film order
    frt.write_image(str(tmp_path / "c"), img, "jpg")                   # the reference's switch: BMP bytes
    assert open(str(tmp_path / "c.jpg"), "rb").read() == b


def test_film_accumulate():
    rng = np.random.default_rng(1)
    a, b = rng.random(30).astype(np.float32), rng.random(30).astype(np.float32)
    acc = frt.film_accumulate(a.copy(), 16, b, 48)
    assert np.allclose(acc, (a * 16 + b * 48) / 64, rtol=1e-6)
    assert np.array_equal(frt.film_accumulate(np.zeros(30, np.float32), 0, b, 7), b)


def test_progressive_passes_equal_one_call(cornell_obj):
    """Samples [0, 8) in one call == passes [0, 3) + [3, 8) accumulated
    (the RNG is keyed by the global sample index)."""
    hs = frt.HostScene("cornell_box_obj", cornell_obj, 1.0)
    nx = ny = 32
    pix = np.arange(nx * ny, dtype=np.int32)
    full, st = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 8, seed=2), pix)
    p1, _ = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 3, seed=2), pix)
    p2, _ = frt.selftest_path_host(hs, frt.RenderParams.make(nx, ny, 5, seed=2, sample_offset=3), pix)
    acc = frt.film_accumulate(p1, 3, p2, 5)
    assert np.allclose(acc, full, rtol=1e-5, atol=1e-7)
    assert not np.allclose(p2, full[:len(p2)], rtol=1e-3)
