#!/usr/bin/env python3
"""TEST INFRASTRUCTURE: golden tiles of the full-size bunny.sp, lucy.sp, elf.sp and material_spheres.sp configs, rendered by the
reference itself (oracle/_ref/libsp_ref.so = the reference's Scene / BVHAccelerator / integrators
compiled from /root/reference, driven by main.cpp:86-103's per-pixel loop).

BASELINE.json configs[3] (lucy.sp, 1920x1080 @ 256 spp, DirectLighting) and configs[4] (elf.sp,
4096x4096 @ 1024 spp, IterativeRRNEE with max_depth 16) exist to stress a deep BVH and long
divergent paths; full frames are far beyond a CPU test budget, so a fixed, seeded subset of
tiles is rendered at the config's spp:

  1. every k-th tile of the frame is probed at 1 spp with the reference;
  2. tiles are picked from the probe: silhouettes (a mix of environment-only pixels and geometry),
     the highest-contrast all-geometry tiles (drapery folds, floor contact and shadows), and
     random tiles (seeded);
     For bunny.sp (configs[2], the headline frame) the slowest tiles are added: every tile of the
     frame is timed on the reference at 16 spp (the smaller of two runs), one thread per tile (8 worker
     processes), and
     the slowest whole tiles are taken -- the bunnies' undersides against the glossy floor, where
     the deepest traversals and most of the glossy estimates sit;
  3. those tiles are rendered at the config's spp and stored with the mesh generator's
     parameters and the SHA-256 of the generated mesh file, so a test can prove it rebuilt the
     same scene before comparing, and with this CPU's RSQRTSS table: the reference normalises
     with RSQRTSS (math/Math.h:205), whose outputs differ between CPU vendors, so its image is
     this CPU's; a test on another machine installs the table (sp_rsqrt_table_set) first.

Run in the build container (the reference sources are needed for oracle/_ref):
    python tests/golden/gen_full_scale.py            # both scenes
    python tests/golden/gen_full_scale.py --scene elf
Outputs tests/golden/{bunny,lucy,elf,spheres}_full_tiles.npz.  lucy takes ~10 min of 8 cores (28.05 M
triangle parse + reference BVH build dominate), elf ~5 min, bunny ~5 min (the per-tile timing).
"""
from __future__ import annotations

import argparse
import ctypes as C
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

REF_LIB = os.path.join(ROOT, "oracle", "_ref", "libsp_ref.so")
GOLDEN = os.path.join(ROOT, "tests", "golden")

# BASELINE.json configs: scene writer kwargs, frame, spp, integrator (SP_INTEGRATOR_*), picks
CONFIGS = {
    # configs[2], the north-star frame: four bunnies (clearcoat, lambertian, glossy) on a glossy plane
    "bunny": dict(writer="write_bunny_scene", kw={}, file="bunny.sp", mesh="ply_files/bunny/reconstruction/bun_zipper.ply",
                  w=1920, h=1080, spp=256, integrator=6, probe_step=5, picks=(8, 8, 8), seed=6, slow=8, slow_spp=16),
    "lucy": dict(writer="write_lucy_scene", kw=dict(n=1529), file="lucy.sp", mesh="ply_files/lucy_1529.ply",
                 w=1920, h=1080, spp=256, integrator=6, probe_step=5, picks=(12, 10, 10), seed=3),
    "elf": dict(writer="write_elf_scene", kw=dict(n=290, max_depth=16), file="elf.sp",
                mesh="stl_files/elf/nude-body_290.stl", w=4096, h=4096, spp=1024, integrator=5, probe_step=11,
                picks=(10, 8, 8), seed=4),
    # configs[1]: analytic spheres lit only by the 4096x2048 image-based environment light (the
    # Distribution2D tables at twice the map resolution, 8192-entry CDFs); "mesh" is the map
    "spheres": dict(writer="write_material_spheres_scene", kw={}, file="material_spheres_ibl.sp",
                    mesh="clarens_night_02_4k.pfm", w=1024, h=1024, spp=64, integrator=6, probe_step=7,
                    picks=(10, 8, 8), seed=5),
}


def sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for b in iter(lambda: fh.read(1 << 24), b""):
            h.update(b)
    return h.hexdigest()


def host_cpu() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def ref_lib():
    L = C.CDLL(REF_LIB)
    L.ref_scene_create.restype = C.c_void_p
    L.ref_scene_create.argtypes = [C.c_char_p, C.c_int, C.c_int]
    L.ref_scene_free.argtypes = [C.c_void_p]
    L.ref_render_tiles.restype = C.c_int
    L.ref_render_tiles.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.POINTER(C.c_int32), C.c_int64, C.c_int,
                                   C.POINTER(C.c_float)]
    L.ref_last_error.restype = C.c_char_p
    return L


def render(L, sc, integrator, spp, ids, threads):
    ids = np.ascontiguousarray(ids, dtype=np.int32)
    out = np.zeros((ids.size, 64, 3), dtype=np.float32)
    rc = L.ref_render_tiles(sc, integrator, spp, ids.ctypes.data_as(C.POINTER(C.c_int32)), ids.size, threads,
                            out.ctypes.data_as(C.POINTER(C.c_float)))
    assert rc == 0, L.ref_last_error()
    return out


def inside_mask(tile: int, w: int, h: int) -> np.ndarray:
    """Lanes (Morton order, base/Tile.h) of a tile that fall inside the image."""
    tw = (w + 7) // 8
    x0, y0 = (tile % tw) * 8, (tile // tw) * 8
    m = np.arange(64)
    x = np.zeros(64, dtype=np.int64)
    y = np.zeros(64, dtype=np.int64)
    for b in range(3):
        x |= ((m >> (2 * b)) & 1) << b
        y |= ((m >> (2 * b + 1)) & 1) << b
    return (x0 + x < w) & (y0 + y < h)


def strip_blocks(text: str, block: str) -> str:
    """The scene text without its top-level `block { ... }` entries (e.g. every sphere)."""
    out, i = [], 0
    lines = text.splitlines(keepends=True)
    while i < len(lines):
        if lines[i].strip() == block + " {":
            depth = 0
            while True:
                depth += lines[i].count("{") - lines[i].count("}")
                i += 1
                if depth == 0:
                    break
            continue
        out.append(lines[i])
        i += 1
    return "".join(out)


def pick_tiles(probe: np.ndarray, ids: np.ndarray, env, w: int, h: int, picks, seed: int, env_probe=None):
    """Silhouette, high-contrast and random tiles from a 1-spp probe (see module docstring)."""
    rng = np.random.default_rng(seed)
    n_sil, n_con, n_rnd = picks
    full = np.array([inside_mask(int(t), w, h).all() for t in ids])
    if env is None:  # image light: an escaped camera ray's radiance varies -- take pixels a spheres-free probe matches
        is_env = np.zeros(probe.shape[:2], dtype=bool) if env_probe is None else np.all(probe == env_probe, axis=-1)
    else:
        is_env = np.all(probe == env[None, None, :], axis=-1)  # camera ray escaped: L = the light's radiance
    n_env = is_env.sum(axis=1)
    lum = probe @ np.array([0.2126, 0.7152, 0.0722], dtype=np.float32)
    contrast = lum.std(axis=1)
    chosen, kinds = [], []
    sil = np.flatnonzero(full & (n_env > 8) & (n_env < 56))
    for i in rng.choice(sil, size=min(n_sil, sil.size), replace=False):
        chosen.append(int(ids[i]))
        kinds.append("silhouette")
    geo = np.flatnonzero(full & (n_env == 0))
    geo = geo[np.argsort(-contrast[geo], kind="stable")]
    geo = [i for i in geo if int(ids[i]) not in chosen]
    for i in geo[:n_con]:
        chosen.append(int(ids[i]))
        kinds.append("contrast")
    rest = np.array([i for i in range(ids.size) if int(ids[i]) not in chosen])
    for i in rng.choice(rest, size=min(n_rnd, rest.size), replace=False):
        chosen.append(int(ids[i]))
        kinds.append("random")
    return np.array(chosen, dtype=np.int32), np.array(kinds)


def _time_tiles_worker(job):
    """One worker process: each tile of `ids` rendered alone on one thread, wall time per tile."""
    path, w, h, integ, spp, ids = job
    L = ref_lib()
    sc = L.ref_scene_create(path.encode(), w, h)
    assert sc, L.ref_last_error()
    out = np.zeros((1, 64, 3), dtype=np.float32)
    t = np.zeros(len(ids))
    for k, tile in enumerate(ids):
        one = np.array([tile], dtype=np.int32)
        best = float("inf")
        for _ in range(2):  # the smaller of two runs: a tile's cost, not a scheduling hiccup
            t0 = time.perf_counter()
            rc = L.ref_render_tiles(sc, integ, spp, one.ctypes.data_as(C.POINTER(C.c_int32)), 1, 1,
                                    out.ctypes.data_as(C.POINTER(C.c_float)))
            best = min(best, time.perf_counter() - t0)
            assert rc == 0
        t[k] = best
    L.ref_scene_free(sc)
    return t


def slowest_tiles(path, w, h, integ, spp, n_pick, exclude, procs):
    """The n_pick slowest whole tiles of the frame on the reference (one thread per tile)."""
    import multiprocessing as mp
    import simplepath_amd as sp
    n = sp.TileScheduler(w, h).get_num_tiles()
    ids = np.arange(n, dtype=np.int32)
    parts = [ids[k::procs] for k in range(procs)]
    with mp.get_context("fork").Pool(procs) as pool:
        times = pool.map(_time_tiles_worker, [(path, w, h, integ, spp, p) for p in parts])
    t = np.zeros(n)
    for p, tp in zip(parts, times):
        t[p] = tp
    full = np.array([inside_mask(int(i), w, h).all() for i in ids])
    order = [int(i) for i in np.argsort(-t, kind="stable") if full[i] and int(i) not in exclude]
    picked = np.array(order[:n_pick], dtype=np.int32)
    return picked, t[picked], float(np.mean(t))


def generate(name: str, workdir: str, threads: int) -> str:
    import simplepath_amd as sp
    from simplepath_amd import scenes

    cfg = CONFIGS[name]
    t0 = time.time()
    path = getattr(scenes, cfg["writer"])(workdir, **cfg["kw"])
    mesh = os.path.join(workdir, cfg["mesh"])
    digest = sha256(mesh)
    print(f"[{name}] scene written ({time.time() - t0:.0f} s), mesh sha256 {digest[:16]}", flush=True)
    w, h, spp, integ = cfg["w"], cfg["h"], cfg["spp"], cfg["integrator"]

    # BVH depths of both builds (host only), recorded for the device tests
    s = sp.Scene.from_file(path)
    s.set_resolution(w, h)
    depth_ref = s.bvh_build_info(1)
    depth_sah = s.bvh_build_info(0)
    del s
    print(f"[{name}] host BVH: reference {depth_ref}, SAH {depth_sah} ({time.time() - t0:.0f} s)", flush=True)

    L = ref_lib()
    sc = L.ref_scene_create(path.encode(), w, h)
    assert sc, L.ref_last_error()
    print(f"[{name}] reference scene built ({time.time() - t0:.0f} s)", flush=True)
    n_tiles = sp.TileScheduler(w, h).get_num_tiles()
    probe_ids = np.arange(cfg["probe_step"] // 2, n_tiles, cfg["probe_step"], dtype=np.int32)
    probe = render(L, sc, integ, 1, probe_ids, threads)
    print(f"[{name}] probe: {probe_ids.size} tiles at 1 spp ({time.time() - t0:.0f} s)", flush=True)
    env, env_probe = None, None
    if name == "spheres":
        # the same probe with every sphere removed: pixels whose radiance it reproduces saw only the sky
        bare = os.path.join(workdir, "material_spheres_sky_only.sp")
        with open(path) as fh:
            text = fh.read()
        with open(bare, "w") as fh:
            fh.write(strip_blocks(text, "sphere"))
        sc0 = L.ref_scene_create(bare.encode(), w, h)
        assert sc0, L.ref_last_error()
        env_probe = render(L, sc0, integ, 1, probe_ids, threads)
        L.ref_scene_free(sc0)
    else:
        # an escaped camera ray sees the environment light's radiance (bunny.sp has none: 0)
        env = np.array({"lucy": [1.0, 1.0, 1.3], "elf": [0.75, 0.75, 0.75], "bunny": [0.0, 0.0, 0.0]}[name],
                       dtype=np.float32)
    ids, kinds = pick_tiles(probe, probe_ids, env, w, h, cfg["picks"], cfg["seed"], env_probe)
    extra = {}
    if cfg.get("slow"):
        slow, slow_t, mean_t = slowest_tiles(path, w, h, integ, cfg["slow_spp"], cfg["slow"], set(ids.tolist()),
                                             max(1, threads))
        ids = np.concatenate([ids, slow]).astype(np.int32)
        kinds = np.concatenate([kinds, np.array(["slowest"] * slow.size)])
        extra = dict(slow_tile_s=slow_t, mean_tile_s=mean_t, slow_spp=cfg["slow_spp"])
        print(f"[{name}] slowest tiles {slow.tolist()} ({slow_t.min() / mean_t:.1f}-{slow_t.max() / mean_t:.1f}x "
              f"the mean at {cfg['slow_spp']} spp, {time.time() - t0:.0f} s)", flush=True)
    t1 = time.time()
    out = render(L, sc, integ, spp, ids, threads)
    print(f"[{name}] {ids.size} tiles at {spp} spp ({time.time() - t1:.0f} s)", flush=True)
    L.ref_scene_free(sc)
    rs = sp.rsqrt_table()  # the reference ran with this host's RSQRTSS
    dst = os.path.join(GOLDEN, f"{name}_full_tiles.npz")
    np.savez_compressed(dst, tile_ids=ids, kinds=kinds, radiance=out, width=w, height=h, spp=spp, integrator=integ,
                        writer=cfg["writer"], writer_kw=repr(cfg["kw"]), scene_file=cfg["file"],
                        mesh_file=cfg["mesh"], mesh_sha256=digest,
                        bvh_ref=json.dumps(depth_ref), bvh_sah=json.dumps(depth_sah),
                        rsqrt_entries=rs["entries"], rsqrt_bits=rs["bits"], rsqrt_zero=rs["zero_result"],
                        rsqrt_denorm=rs["denorm_result"], host_cpu=host_cpu(),
                        generator="tests/golden/gen_full_scale.py (oracle/_ref = reference sources)", **extra)
    print(f"[{name}] wrote {dst} ({time.time() - t0:.0f} s total)", flush=True)
    return dst


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", choices=["bunny", "lucy", "elf", "spheres", "all"], default="all")
    ap.add_argument("--workdir", default=os.path.join("/tmp", "sp_full_scale"))
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    a = ap.parse_args()
    if not os.path.exists(REF_LIB):
        sys.exit("oracle/_ref/libsp_ref.so is missing: run oracle/build_ref.sh (needs /root/reference)")
    for name in (["bunny", "spheres", "elf", "lucy"] if a.scene == "all" else [a.scene]):
        generate(name, a.workdir, a.threads)


if __name__ == "__main__":
    main()
