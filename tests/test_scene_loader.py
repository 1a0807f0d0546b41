"""Host scene loading mirrors base/FileParser.cpp and base/PlyReader.cpp."""
import os

import numpy as np
import pytest

import simplepath_amd as sp
from simplepath_amd import scenes


def test_bunny_scene_structure(scene_dir):
    s = sp.Scene.from_file(os.path.join(scene_dir, "bunny.sp"))
    i = s.info()
    assert (i.image_width, i.image_height) == (1000, 600)
    assert i.integrator_type == 0  # not specified -> DirectLighting at render time (main.cpp:390)
    assert i.num_lights == 1 and i.num_materials == 7 and i.num_shapes == 1
    v, f = scenes.bunny_mesh()
    assert i.num_triangles == 4 * f.shape[0]
    d = s.desc()
    kinds = np.ctypeslib.as_array(d.prim_kind, shape=(d.num_prims,))
    # meshes first (file order), then the plane: FileParser pass 3 order
    assert (kinds[:-1] == 0).all() and kinds[-1] == 2
    verts = np.ctypeslib.as_array(d.vertices, shape=(i.num_vertices, 3))
    # mesh 0: translate 2.25, scale 10 -> world x range around 2.25
    n0 = v.shape[0]
    assert 2.25 - 1.0 < verts[:n0, 0].mean() < 2.25 + 1.0
    assert abs(verts[:, 1].min() - 0.329874) < 1e-3  # bunnies sit on the plane


def test_parse_errors():
    with pytest.raises(sp.SimplePathError) as e:
        sp.Scene.from_string("version: 2\n")
    assert "Unable to parse version 2" in str(e.value)
    with pytest.raises(sp.SimplePathError) as e:
        sp.Scene.from_string("version: 1\nbogus_type {\n}\n")
    assert "Unknown type 'bogus_type'" in str(e.value)
    with pytest.raises(sp.SimplePathError) as e:
        sp.Scene.from_string('version: 1\nmaterial_lambertian {\n name: "a"\n diffuse: 1 1 1\n}\n'
                             'material_lambertian {\n name: "a"\n diffuse: 1 1 1\n}\n'
                             "perspective_camera {\n origin: 0 0 1\n look_at: 0 0 0\n}\n")
    assert "already exists" in str(e.value)


def test_set_resolution_rebuilds_camera(scene_dir):
    s = sp.Scene.from_file(os.path.join(scene_dir, "bunny.sp"))
    a = s.desc().camera.transform
    vz0 = list(a.vz)
    s.set_resolution(1920, 1080)
    b = s.desc().camera.transform
    assert s.width == 1920 and s.height == 1080
    assert list(b.vz) != vz0
