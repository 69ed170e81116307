"""The native C++ side on the GPU: frt_render (the reference's main() with
flags) through frt::renderer<path_gpu / pssmlt_gpu> and frt_render_multi,
against the Python binding's film.  The CLI runs as a child process."""
import os
import subprocess

import numpy as np
import pytest

import first_raytracer_amd as frt

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "first_raytracer_amd", "frt_render")


def read_pfm(path):
    with open(path, "rb") as f:
        assert f.readline().strip() == b"PF"
        w, h = (int(x) for x in f.readline().split())
        assert float(f.readline()) < 0          # little endian
        return np.frombuffer(f.read(), "<f4").reshape(h, w, 3)


def test_cli_path_matches_binding(cornell_obj, tmp_path):
    out = str(tmp_path / "c.pfm")
    png = str(tmp_path / "c.png")
    r = subprocess.run([CLI, "--scene", "cornell", "--obj", cornell_obj, "--res", "64x48", "--ns", "8",
                        "--seed", "3", "--out", out, "--png", png], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Rays/second" in r.stdout or "rays" in r.stdout.lower()
    img = read_pfm(out)
    from test_film import read_png
    assert np.array_equal(read_png(png), frt.tonemap_u8(img)[::-1])   # display bytes, top-down rows
    ctx = frt.Context(0)
    try:
        ctx.upload(frt.HostScene("cornell_box_obj", cornell_obj, 64 / 48))
        film, _ = ctx.render(frt.RenderParams.make(64, 48, 8, seed=3))
    finally:
        ctx.close()
    assert np.array_equal(img, film)            # same streams, same film order (y = 0 bottom)


def test_cli_pssmlt(cornell_obj, tmp_path):
    out = str(tmp_path / "m.pfm")
    r = subprocess.run([CLI, "--scene", "cornell", "--obj", cornell_obj, "--res", "64x48", "--ns", "16",
                        "--integrator", "pssmlt", "--chains", "3072", "--out", out],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    img = read_pfm(out)
    assert np.isfinite(img).all() and img.mean() > 0.01


@pytest.mark.parametrize("integ,code", [("ao", frt.FRT_INTEGRATOR_AO), ("normals", frt.FRT_INTEGRATOR_NORMALS)])
def test_cli_ao_normals_match_binding(cornell_obj, tmp_path, integ, code):
    """renderer<ao_gpu> / renderer<normals_gpu> (ao.h, debug_renderer.h) with --env."""
    out = str(tmp_path / f"{integ}.pfm")
    r = subprocess.run([CLI, "--scene", "cornell", "--obj", cornell_obj, "--res", "64x48", "--ns", "4",
                        "--seed", "5", "--integrator", integ, "--env", "1,0.5,0.25", "--out", out],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    img = read_pfm(out)
    ctx = frt.Context(0)
    try:
        hs = frt.HostScene("cornell_box_obj", cornell_obj, 64 / 48)
        hs.set_env((1.0, 0.5, 0.25))
        ctx.upload(hs)
        film, _ = ctx.render(frt.RenderParams.make(64, 48, 4, seed=5, integrator=code))
    finally:
        ctx.close()
    assert np.array_equal(img, film)
