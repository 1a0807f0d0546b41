"""The C++ drop-in (include/simplepath_amd.hpp): tests/cpp/drop_in_main.cpp is the reference's
main.cpp flow (parse_scene_file -> integrator fallback -> create_integrator -> render, main.cpp:
368-397) compiled and linked as a host program would (g++ -I include -l simplepath_hip), i.e. the
change INTEGRATION.md describes.  CPU: it builds and reports errors as the reference does; GPU: its
PFM equals the CPU oracle bit for bit."""
import os
import subprocess

import numpy as np
import pytest

import simplepath_amd as sp
from tests import _oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "_build", "drop_in_main")


@pytest.fixture(scope="module")
def exe():
    if os.path.isdir("/root/reference") or not os.path.exists(EXE):  # build container: (re)build it
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True, timeout=600)
    return EXE


def read_pfm(path):
    with open(path, "rb") as fh:
        assert fh.readline().strip() == b"PF"
        w, h = (int(x) for x in fh.readline().split())
        scale = float(fh.readline())
        data = np.frombuffer(fh.read(), dtype="<f4" if scale < 0 else ">f4")
    return data.reshape(h, w, 3)[::-1]  # rows bottom-up in the file (Image/Image.cpp:40)


def run(exe, *args):
    return subprocess.run([exe, *args], capture_output=True, text=True, timeout=300)


def test_drop_in_reports_reference_errors(exe, scene_dir, tmp_path):
    (tmp_path / "ex.sp").write_text("version: 1\n\nmaterial_layered {\n}\n")
    r = run(exe, str(tmp_path / "ex.sp"))
    assert r.returncode == 2 and "ParsingException: Unknown type 'material_layered' on line 3" in r.stderr
    r = run(exe, os.path.join(scene_dir, "bunny.sp"), "--integrator", "path_guiding")
    assert r.returncode == 1 and "Unknown integrator type" in r.stderr
    r = run(exe, str(tmp_path / "missing.sp"))
    assert r.returncode == 2


@pytest.mark.gpu
@pytest.mark.parametrize("integrator,extra", [("direct_lighting", []), ("iterative_rrnee", []),
                                              ("direct_lighting", ["--from-desc"])])
def test_drop_in_render_matches_oracle(exe, scene_dir, tmp_path, integrator, extra):
    out = str(tmp_path / "img.pfm")
    path = os.path.join(scene_dir, "bunny.sp")
    r = run(exe, path, "--samples", "3", "--integrator", integrator, "--bvh", "1", "--size", "48", "32",
            "--output", out, *extra)
    assert r.returncode == 0, r.stderr
    img = read_pfm(out)
    s = sp.Scene.from_file(path)
    s.set_resolution(48, 32)
    tiles, _ = _oracle.render(s, sp.string_to_integrator_type(integrator), 3, variant="spm")
    ref = sp.tiles_to_image(48, 32, tiles)
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))
