import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the C-ABI on the device)")


@pytest.fixture(scope="session")
def scene_dir(tmp_path_factory):
    from simplepath_amd import scenes
    d = str(tmp_path_factory.mktemp("scenes"))
    scenes.write_bunny_scene(d)
    # the scan-like bunny (cupped ears, surface relief): a harder robustness workload
    scenes.write_bunny_scan_scene(d)
    scenes.write_spheres_scene(d)
    # image-lit material_spheres.sp with a small synthetic HDR map (the 4k map is the bench's)
    scenes.write_material_spheres_scene(d, 96, 48, image="night_96x48.pfm")
    # lucy.sp / elf.sp (PLY rotated by the scene, binary STL with vertex welding) at small sizes
    scenes.write_lucy_scene(d, n=40, name="lucy_small.sp")
    scenes.write_elf_scene(d, n=24, max_depth=16, name="elf_small.sp")
    # recursion deeper than the device's in-register levels (32)
    scenes.write_closed_room_scene(d, max_depth=40)
    # a reference BVH 172 levels deep (geometric wedge strip): the stackless walk
    scenes.write_wedge_strip_scene(d)
    return d
