"""Numerics contract: samplers and RSQRTSS emulation against their golden sources."""
import ctypes as C
import os

import numpy as np

import simplepath_amd as sp
from tests import _oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "sampler_golden.npy")


def test_oracle_sampler_matches_libstdcxx_golden():
    g = np.load(GOLD)
    L = _oracle.load("glibc")
    for (x, y) in {(int(a), int(b)) for a, b, _ in g}:
        rows = g[(g[:, 0] == x) & (g[:, 1] == y)][:, 2]
        out = np.zeros(rows.size, dtype=np.float32)
        L.orc_mt_stream(((x << 16) | y) ^ 0xB0AE9D99, rows.size, out.ctypes.data_as(C.POINTER(C.c_float)))
        assert np.array_equal(out.view(np.uint32), rows), (x, y)


def test_rsqrt_table_verified_against_host_instruction():
    bits, ok = C.c_int32(), C.c_int32()
    sp.lib().sp_rsqrt_table_info(C.byref(bits), C.byref(ok))
    assert ok.value == 1 and 8 <= bits.value <= 23
    L = _oracle.load("glibc")
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.uniform(1e-6, 1e6, 20000).astype(np.float32),
                         np.array([1.0, 2.0, 4.0, 0.25, 3.0e-38, 1.0e38], dtype=np.float32)])
    for x in xs:
        # the emulated RSQRTSS then the reference's Newton step == oracle's intrinsic path
        r = sp.lib().sp_host_rsqrt_emulated(float(x))
        r32 = np.float32(r)
        a = np.float32(x)
        newton = np.float32(np.float32(1.5) * r32) + np.float32(np.float32(np.float32(a * np.float32(-0.5)) * r32) * np.float32(r32 * r32))
        assert np.float32(L.orc_rsqrt(float(x))) == newton


def test_rsqrt_table_override_round_trip(scene_dir):
    """sp_rsqrt_table_set: building a scene with this host's own table installed as an override
    (table emulation) gives the same bits as the RSQRTSS instruction; a different table changes the
    host-built normals (it is really used); NULL restores the host's table."""
    import os

    import simplepath_amd as sp

    path = os.path.join(scene_dir, "bunny.sp")

    def normals():
        s = sp.Scene.from_file(path)
        d = s.desc()
        n = np.ctypeslib.as_array(d.normals, shape=(d.info.num_vertices, 3)).copy()
        cam = np.array(list(d.camera.transform.vx) + list(d.camera.transform.vz))
        return n, cam

    base_n, base_cam = normals()
    t = sp.rsqrt_table()
    assert t["entries"].size == 2 << t["bits"]
    try:
        sp.set_rsqrt_table(t)
        n, cam = normals()
        assert np.array_equal(n.view(np.uint32), base_n.view(np.uint32))
        assert np.array_equal(cam, base_cam)
        other = dict(t, entries=t["entries"] + np.uint32(1))  # a CPU whose estimates are 1 ulp higher
        sp.set_rsqrt_table(other)
        assert np.array_equal(sp.rsqrt_table()["entries"], other["entries"])
        n2, _ = normals()
        assert not np.array_equal(n2.view(np.uint32), base_n.view(np.uint32))
    finally:
        sp.set_rsqrt_table(None)
    assert np.array_equal(sp.rsqrt_table()["entries"], t["entries"])
    n3, _ = normals()
    assert np.array_equal(n3.view(np.uint32), base_n.view(np.uint32))


def test_rsqrt_table_override_rejects_tables_too_big_for_lds():
    # 2 << bits entries are copied to LDS by every kernel: more than 13 bits cannot fit next to the
    # traversal stacks, so sp_rsqrt_table_set refuses it up front with SP_ERR_ARG
    import simplepath_amd as sp
    from simplepath_amd import _abi

    big = {"entries": np.zeros(2 << 14, dtype=np.uint32), "bits": 14, "zero_result": 0x7f800000,
           "denorm_result": 0x7f800000}
    try:
        sp.set_rsqrt_table(big)
        raise AssertionError("expected SP_ERR_ARG")
    except sp.SimplePathError as e:
        assert e.code == _abi.SP_ERR_ARG and "LDS" in str(e)
    finally:
        sp.set_rsqrt_table(None)


def test_rsqrt_table_override_concurrent_readers(scene_dir):
    # scenes built on one thread while another installs and removes tables: every build sees one
    # complete table (the override is swapped as a whole, never modified in place)
    import os
    import threading

    import simplepath_amd as sp

    path = os.path.join(scene_dir, "bunny.sp")
    t = sp.rsqrt_table()
    stop = threading.Event()

    def writer():
        # bounded: a slow box must not turn this into an install storm (each install used to be
        # kept forever; now equal tables are reused, see test_rsqrt_table_set_is_bounded)
        for _ in range(20000):
            if stop.is_set():
                break
            sp.set_rsqrt_table(t)
            sp.set_rsqrt_table(None)

    th = threading.Thread(target=writer)
    th.start()
    try:
        base = None
        for _ in range(6):
            scene = sp.Scene.from_file(path)  # owns the arrays desc() points into
            d = scene.desc()
            n = np.ctypeslib.as_array(d.normals, shape=(d.info.num_vertices, 3)).copy()
            base = n if base is None else base
            assert np.array_equal(n.view(np.uint32), base.view(np.uint32))  # same table, either way
    finally:
        stop.set()
        th.join()
        sp.set_rsqrt_table(None)


def _rss_bytes():
    with open("/proc/self/statm") as f:
        return int(f.read().split()[1]) * os.sysconf("SC_PAGE_SIZE")


def test_rsqrt_table_set_is_bounded():
    # sp_rsqrt_table_set keeps every DISTINCT installed table alive (readers hold raw pointers), but
    # re-installing an equal table reuses the kept copy: 10 000 installs of two tables must not grow
    # the process (each copy is 8-32 KB, so a leak would be 80-320 MB)
    import simplepath_amd as sp

    t = sp.rsqrt_table()
    other = dict(t, entries=t["entries"] + np.uint32(1))
    try:
        for _ in range(200):  # warm-up: both tables installed once, allocator settled
            sp.set_rsqrt_table(t)
            sp.set_rsqrt_table(other)
        before = _rss_bytes()
        for i in range(10000):
            sp.set_rsqrt_table(t if i & 1 else other)
        grown = _rss_bytes() - before
        assert grown < 50 * 2**20, grown
        assert np.array_equal(sp.rsqrt_table()["entries"], t["entries"])  # the last one installed
    finally:
        sp.set_rsqrt_table(None)
    assert np.array_equal(sp.rsqrt_table()["entries"], t["entries"])


def test_grouped_twist_matches_libstdcxx(tmp_path):
    # the device's 4-word grouped twist (sp_twist4.h, used with the lane-blocked state layout)
    # compiled for the host: 5 consecutive generations x 3 seeds x 4 lane positions, every word
    # against std::mt19937_64 itself
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "twist4_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(root, "simplepath_amd", "csrc", "common"),
                    os.path.join(root, "tests", "cpp", "twist4_check.cpp"), "-o", exe], check=True,
                   timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatching" in r.stdout
