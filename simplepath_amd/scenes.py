"""Benchmark / test workloads: the reference's scene descriptions and synthetic meshes.

The reference's scenes (scenes/bunny.sp, example_scene.sp, scenes/material_spheres.sp ...) name
PLY/STL/PFM assets that are not part of the repository (Stanford bunny `bun_zipper.ply`, lucy,
an HDR environment map).  There is no network here, so the meshes are generated: a closed,
smooth, star-shaped "bunny-like" surface on a cube-sphere grid with the same vertex/face counts
class (~35k vertices, ~69.5k near-uniform triangles) and the same bounding box as bun_zipper.ply, written in the same PLY layout
(binary_little_endian, float x y z confidence intensity, `list uchar int vertex_indices`).  The
scene parameters (camera, materials, transforms, lights) are those of the reference files.
"""
from __future__ import annotations

import os

import numpy as np

# bounding box of the Stanford bunny reconstruction bun_zipper.ply
_BUNNY_LO = np.array([-0.0946899, 0.0329874, -0.0618736])
_BUNNY_HI = np.array([0.0610398, 0.187321, 0.0587997])


def _bunny_radius(d: np.ndarray) -> np.ndarray:
    """Radial profile r(direction) of the synthetic bunny: an ellipsoidal body with head, ears and tail lobes."""
    lobes = [  # centre direction, width, amplitude
        ((0.55, 0.35, 0.0), 0.35, 0.55),    # head (forward, up)
        ((0.35, 0.85, 0.18), 0.05, 0.95),   # ear 1
        ((0.30, 0.88, -0.22), 0.05, 0.90),  # ear 2
        ((-0.95, 0.1, 0.0), 0.08, 0.25),    # tail
        ((0.2, -0.9, 0.0), 0.4, -0.15),     # flattened belly
    ]
    r = np.full(d.shape[0], 1.0)
    for c, w, a in lobes:
        c = np.asarray(c, dtype=np.float64)
        c = c / np.linalg.norm(c)
        dist2 = np.sum((d - c) ** 2, axis=1)
        r += a * np.exp(-dist2 / w)
    # gentle high-frequency ripples so the surface is not a smooth ellipsoid
    r += 0.015 * np.sin(23.0 * d[:, 0]) * np.cos(19.0 * d[:, 1]) * np.sin(17.0 * d[:, 2])
    return r


def bunny_mesh(n: int = 76):
    """Closed star-shaped surface on an equal-angle cube-sphere grid: 6*n*n quads -> 12*n*n
    triangles (n = 76: 34658 vertices, 69312 triangles; bun_zipper.ply: 35947 / 69451).  Like a
    scanned mesh its triangles are of near-uniform size: no parameterisation poles, whose fans of
    sliver triangles with overlapping boxes would make BVH traversal unrepresentatively costly."""
    t = np.tan(np.linspace(-np.pi / 4, np.pi / 4, n + 1))
    uu, vv = np.meshgrid(t, t, indexing="ij")
    pts, quads = [], []
    base = 0
    for axis in range(3):
        for sign in (1.0, -1.0):
            q = np.empty((n + 1, n + 1, 3))
            a1, a2 = (axis + 1) % 3, (axis + 2) % 3
            q[..., axis] = sign
            q[..., a1] = uu
            q[..., a2] = vv
            pts.append(q.reshape(-1, 3))
            i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
            v00 = base + i * (n + 1) + j
            v10, v01, v11 = v00 + (n + 1), v00 + 1, v00 + n + 2
            # (u, v, axis) is right-handed; flip for the negative faces so normals point outward
            if sign > 0:
                quads.append(np.stack([v00, v10, v11, v01], -1).reshape(-1, 4))
            else:
                quads.append(np.stack([v00, v01, v11, v10], -1).reshape(-1, 4))
            base += (n + 1) * (n + 1)
    d = np.concatenate(pts)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    key = np.round(d * 1e6).astype(np.int64)
    _, first, inverse = np.unique(key, axis=0, return_index=True, return_inverse=True)
    inverse = inverse.reshape(-1)
    d = d[first]
    qd = inverse[np.concatenate(quads)]
    f = np.concatenate([qd[:, [0, 1, 2]], qd[:, [0, 2, 3]]]).astype(np.int32)
    p = d * _bunny_radius(d)[:, None] * np.array([1.25, 1.0, 0.8])
    lo, hi = p.min(axis=0), p.max(axis=0)
    p = _BUNNY_LO + (p - lo) / (hi - lo) * (_BUNNY_HI - _BUNNY_LO)
    return p.astype(np.float32), f


def _cube_sphere(n: int):
    """Unit-sphere vertices and outward triangles on an equal-angle cube-sphere grid (12 n^2 triangles)."""
    t = np.tan(np.linspace(-np.pi / 4, np.pi / 4, n + 1))
    uu, vv = np.meshgrid(t, t, indexing="ij")
    pts, quads, base = [], [], 0
    for axis in range(3):
        for sign in (1.0, -1.0):
            q = np.empty((n + 1, n + 1, 3))
            q[..., axis] = sign
            q[..., (axis + 1) % 3] = uu
            q[..., (axis + 2) % 3] = vv
            pts.append(q.reshape(-1, 3))
            i, j = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
            v00 = base + i * (n + 1) + j
            v10, v01, v11 = v00 + (n + 1), v00 + 1, v00 + n + 2
            order = [v00, v10, v11, v01] if sign > 0 else [v00, v01, v11, v10]
            quads.append(np.stack(order, -1).reshape(-1, 4))
            base += (n + 1) * (n + 1)
    d = np.concatenate(pts)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    _, first, inverse = np.unique(np.round(d * 1e6).astype(np.int64), axis=0, return_index=True, return_inverse=True)
    qd = inverse.reshape(-1)[np.concatenate(quads)]
    return d[first], np.concatenate([qd[:, [0, 1, 2]], qd[:, [0, 2, 3]]]).astype(np.int32)


def bunny_scan_mesh(n_body: int = 70, n_ear: int = 22):
    """A harder, scan-like bunny (robustness workload, not the headline): the body without its ear
    lobes and with stronger surface relief, plus two separate cupped ears (closed shells whose
    front is pressed in: concave, tilted back over the head and body), so the mesh has the
    overhangs, creases and self-shadowing that the star-shaped stand-in lacks.  58800 + 2 x 5808
    = 70416 triangles in the bun_zipper.ply bounding box."""
    d, f = _cube_sphere(n_body)
    r = np.full(d.shape[0], 1.0)
    for c, w, a in [((0.55, 0.35, 0.0), 0.35, 0.55), ((-0.95, 0.1, 0.0), 0.08, 0.25), ((0.2, -0.9, 0.0), 0.4, -0.15)]:
        c = np.asarray(c) / np.linalg.norm(c)
        r += a * np.exp(-np.sum((d - c) ** 2, axis=1) / w)
    r += 0.04 * np.sin(31.0 * d[:, 0] + 1.0) * np.cos(27.0 * d[:, 1]) * np.sin(23.0 * d[:, 2] + 0.5)
    r += 0.02 * np.sin(57.0 * d[:, 0] * d[:, 1] + 61.0 * d[:, 2])
    scale = np.array([1.25, 1.0, 0.8])
    parts_v, parts_f, nv = [d * r[:, None] * scale], [f], d.shape[0]
    e, ef = _cube_sphere(n_ear)
    for side in (1.0, -1.0):
        base_dir = np.array([0.35, 0.85, 0.2 * side])
        base_dir /= np.linalg.norm(base_dir)
        rb = 1.0 + 0.55 * np.exp(-np.sum((base_dir - np.array([0.844, 0.537, 0.0])) ** 2) / 0.35)
        base = base_dir * rb * scale * 0.92
        # cupped shell: the +z half is pressed through the centre plane (a concave dish)
        q = e.copy()
        q[:, 2] = np.where(q[:, 2] > 0.0, -0.35 * q[:, 2], q[:, 2])
        q = q * np.array([0.16, 0.55, 0.12])
        axis = np.array([-0.45, 1.0, 0.25 * side])
        axis /= np.linalg.norm(axis)
        side_v = np.cross(axis, np.array([0.0, 0.0, 1.0]))
        side_v /= np.linalg.norm(side_v)
        front = np.cross(side_v, axis)
        rot = np.stack([side_v, axis, front], axis=1)  # ear x -> side, y -> axis, z (cup) -> front
        parts_v.append(q @ rot.T + base + axis * 0.5)
        parts_f.append(ef + nv)
        nv += e.shape[0]
    p = np.concatenate(parts_v)
    lo, hi = p.min(axis=0), p.max(axis=0)
    p = _BUNNY_LO + (p - lo) / (hi - lo) * (_BUNNY_HI - _BUNNY_LO)
    return p.astype(np.float32), np.concatenate(parts_f).astype(np.int32)


def write_bunny_scan_scene(directory: str) -> str:
    """scenes/bunny.sp with bunny_scan_mesh() in place of the star-shaped stand-in."""
    os.makedirs(directory, exist_ok=True)
    rel = os.path.join("ply_files", "bunny", "reconstruction", "bun_scan.ply")
    path = os.path.join(directory, rel)
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        v, f = bunny_scan_mesh()
        tmp = path + ".tmp%d" % os.getpid()
        write_ply(tmp, v, f)
        os.replace(tmp, path)
    out = os.path.join(directory, "bunny_scan.sp")
    with open(out, "w") as fh:
        fh.write(bunny_sp(rel))
    return out


def write_ply(path: str, verts: np.ndarray, faces: np.ndarray) -> None:
    """binary_little_endian PLY in the layout of bun_zipper.ply."""
    nv, nf = verts.shape[0], faces.shape[0]
    header = ("ply\nformat binary_little_endian 1.0\ncomment synthetic stand-in for bun_zipper.ply\n"
              f"element vertex {nv}\nproperty float x\nproperty float y\nproperty float z\n"
              "property float confidence\nproperty float intensity\n"
              f"element face {nf}\nproperty list uchar int vertex_indices\nend_header\n").encode()
    vrec = np.zeros(nv, dtype=[("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("c", "<f4"), ("i", "<f4")])
    vrec["x"], vrec["y"], vrec["z"] = verts[:, 0], verts[:, 1], verts[:, 2]
    vrec["c"], vrec["i"] = 1.0, 0.5
    frec = np.zeros(nf, dtype=[("n", "u1"), ("a", "<i4"), ("b", "<i4"), ("c", "<i4")])
    frec["n"] = 3
    frec["a"], frec["b"], frec["c"] = faces[:, 0], faces[:, 1], faces[:, 2]
    with open(path, "wb") as fh:
        fh.write(header)
        fh.write(vrec.tobytes())
        fh.write(frec.tobytes())


def ensure_bunny_ply(directory: str) -> str:
    rel = os.path.join("ply_files", "bunny", "reconstruction", "bun_zipper.ply")
    path = os.path.join(directory, rel)
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        v, f = bunny_mesh()
        tmp = path + ".tmp%d" % os.getpid()
        write_ply(tmp, v, f)
        os.replace(tmp, path)
    return rel


# scenes/bunny.sp of the reference: four bunnies (two clearcoat, lambertian, glossy), a glossy
# plane and a sphere light; 1000x600 as written (the benchmark overrides the resolution).
def bunny_sp(ply_rel: str) -> str:
    mats = [
        ("material_lambertian", "material_lambertian", {"diffuse": "0.1 0.8 0.8"}),
        ("material_lambertian", "material_lambertian_base", {"diffuse": "0.1 0.2 0.8"}),
        ("material_glossy", "material_glossy_base", {"diffuse": "0.8 0.2 0.8", "ior": "1.8", "roughness": "0.25"}),
        ("material_glossy", "material_glossy", {"diffuse": "0.8 0.2 0.2", "ior": "1.8", "roughness": "0.75"}),
        ("material_glossy", "material_glossy_plane", {"diffuse": "0.6 0.6 0.6", "ior": "1.8", "roughness": "0.01"}),
        ("material_clearcoat", "material_lambertian_clearcoat",
         {"base": '"material_lambertian_base"', "ior": "1.5", "color": "1.0 0.8 0.8"}),
        ("material_clearcoat", "material_glossy_clearcoat",
         {"base": '"material_glossy_base"', "ior": "1.3", "color": "1.0 1.0 1.0"}),
    ]
    out = ["version: 1", "", "scene_parameters {", '    output_file_name: "image.pfm"',
           "    width: 1000", "    height: 600", "}", "",
           "perspective_camera {", "    origin: 0.0 2.0 5.0", "    look_at: -0.25 1.0 0.0", "    fov: 45", "}", ""]
    for kind, name, attrs in mats:
        out.append(kind + " {")
        out.append(f'    name: "{name}"')
        for k, v in attrs.items():
            out.append(f"    {k}: {v}")
        out += ["}", ""]
    for tx, mat in [(2.25, "material_glossy_clearcoat"), (0.75, "material_lambertian_clearcoat"),
                    (-0.75, "material_lambertian"), (-2.25, "material_glossy")]:
        out += ["mesh {", f'    file: "{ply_rel}"', f"    translate: {tx} 0.0 0.0",
                "    scale: 10.0 10.0 10.0", f'    material: "{mat}"', "}", ""]
    out += ["plane {", '    material: "material_glossy_plane"', "    translate: 0.0 0.329874 0.0", "}", "",
            "sphere_light {", "    translate: 0.0 3.0 0.0", "    scale: 0.5 0.5 0.5",
            "    radiance: 10.0 10.0 10.0", "}", ""]
    return "\n".join(out)


def write_bunny_scene(directory: str) -> str:
    os.makedirs(directory, exist_ok=True)
    rel = ensure_bunny_ply(directory)
    path = os.path.join(directory, "bunny.sp")
    with open(path, "w") as fh:
        fh.write(bunny_sp(rel))
    return path


# scenes/material_spheres.sp with its image environment light replaced by a uniform
# environment_light plus a sphere light: a cheaper variant used by most parity tests.
def spheres_sp(env_radiance: str = "1.0 1.0 1.0", with_sphere_light: bool = True) -> str:
    s = """version: 1

scene_parameters {
    output_file_name: "spheres.pfm"
    width: 450
    height: 1500
}

perspective_camera {
    origin: 0.0 0.0 10.0
    look_at: 0.0 0.0 0.0
    fov: 45
}

material_lambertian {
    name: "material_lambertian"
    diffuse: 0.1 0.8 0.8
}

material_lambertian {
    name: "material_lambertian_base"
    diffuse: 0.1 0.2 0.8
}

material_glossy {
    name: "material_glossy_base"
    diffuse: 0.8 0.2 0.8
    ior: 1.8
    roughness: 0.25
}

material_glossy {
    name: "material_glossy"
    diffuse: 0.8 0.2 0.2
    ior: 1.8
    roughness: 0.75
}

material_glossy {
    name: "material_glossy_plane"
    diffuse: 0.6 0.6 0.6
    ior: 1.8
    roughness: 0.01
}

material_clearcoat {
    name: "material_lambertian_clearcoat"
    base: "material_lambertian_base"
    ior: 1.5
    color: 1.0 0.8 0.8
}

material_clearcoat {
    name: "material_glossy_clearcoat"
    base: "material_glossy_base"
    ior: 1.3
    color: 1.0 1.0 1.0
}

sphere {
    translate: 0.0 3.0 0.0
    material: "material_glossy_clearcoat"
}

sphere {
    translate: 0.0 1.0 0.0
    material: "material_lambertian_clearcoat"
}

sphere {
    translate: 0.0 -1.0 0.0
    material: "material_lambertian"
}

sphere {
    translate: 0.0 -3.0 0.0
    material: "material_glossy"
}

plane {
    material: "material_glossy_plane"
    rotate: 1 0 0 90
    translate: 0.0 0.0 -1.0
}

environment_light {
    rotate: 0.0 1.0 0.0 45.0
    radiance: %s
}
""" % env_radiance
    if with_sphere_light:
        s += """
sphere_light {
    translate: 3.0 4.0 6.0
    scale: 0.5 0.5 0.5
    radiance: 20.0 20.0 20.0
}
"""
    return s


def write_spheres_scene(directory: str, with_sphere_light: bool = True) -> str:
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, "material_spheres.sp")
    with open(path, "w") as fh:
        fh.write(spheres_sp(with_sphere_light=with_sphere_light))
    return path


# ---------------------------------------------------------------- image environment light
def night_sky_image(width: int = 4096, height: int = 2048, seed: int = 2) -> np.ndarray:
    """Synthetic stand-in for clarens_night_02_4k.pfm (not in the reference repository): a
    lat-long HDR night scene, img[y, x] in Image(x, y) order (y = 0 is theta = 0, straight up).
    Dim sky gradient, a bright moon, a row of street lamps near the horizon whose cores exceed
    the scene's max_radiance (100), a dark ground, and a few adversarial texels: +inf (handled by
    ImageBasedEnvironmentLight::modify_image), negative values (Distribution1D takes abs) and
    fully black rows (zero-integral conditional distributions)."""
    rng = np.random.default_rng(seed)
    v = (np.arange(height) + 0.5) / height
    u = (np.arange(width) + 0.5) / width
    theta = (np.pi * v)[:, None]
    phi = (2.0 * np.pi * u)[None, :]
    up = np.cos(theta)
    sky = np.where(up > 0, 0.02 + 0.08 * (1.0 - up) ** 3, 0.004 + 0.002 * np.sin(7 * phi) ** 2)
    img = np.stack([sky * 0.6, sky * 0.7, sky * 1.2], axis=-1) * np.ones((height, width, 1))
    # stars
    n_stars = width * height // 4000
    sy = rng.integers(0, height // 2, n_stars)
    sx = rng.integers(0, width, n_stars)
    img[sy, sx] += rng.uniform(0.5, 4.0, (n_stars, 1))
    # moon: a disc of radiance ~ 40
    d = np.array([np.sin(0.7) * np.cos(2.0), np.cos(0.7), np.sin(0.7) * np.sin(2.0)])
    dirs = np.stack([np.sin(theta) * np.cos(phi), np.cos(theta) * np.ones_like(phi), np.sin(theta) * np.sin(phi)], -1)
    cosang = dirs @ d
    img[cosang > np.cos(0.03)] = (40.0, 38.0, 30.0)
    # street lamps just above the horizon: cores far above max_radiance, halos around them
    for k in range(9):
        lc = np.array([np.sin(1.45) * np.cos(0.3 + 0.7 * k), np.cos(1.45), np.sin(1.45) * np.sin(0.3 + 0.7 * k)])
        c = dirs @ lc
        img += (c > np.cos(0.05))[..., None] * np.array([6.0, 4.0, 1.5])
        img[c > np.cos(0.008)] = (900.0 + 50 * k, 600.0, 250.0)
    img = img.astype(np.float32)
    img[height // 3, width // 5] = (np.inf, 1.0, 1.0)
    img[height // 2 + 3, width // 7] = (-0.5, -0.25, 0.1)
    img[height - 1, :] = 0.0
    img[height - 2, :] = 0.0
    return img


def write_pfm(path: str, img: np.ndarray) -> None:
    """Image/Image.cpp:40 write_pfm layout: little-endian, rows bottom-up (img[y, x] = img(x, y))."""
    h, w, _ = img.shape
    with open(path, "wb") as fh:
        fh.write(f"PF\n{w} {h}\n-1\n".encode())
        fh.write(np.ascontiguousarray(img[::-1].astype("<f4")).tobytes())


def material_spheres_sp(image: str = "clarens_night_02_4k.pfm") -> str:
    """scenes/material_spheres.sp verbatim: analytic spheres lit only by the image-based
    environment light (rotate 45 deg about y, max_radiance 100)."""
    s = spheres_sp(with_sphere_light=False)
    head = s[: s.index("environment_light {")]
    return head + """environment_light {
    rotate: 0.0 1.0 0.0 45.0
    radiance: 1.0 1.0 1.0
    max_radiance: 100
    image: "%s"
}
""" % image


def write_material_spheres_scene(directory: str, width: int = 4096, height: int = 2048,
                                 image: str = "clarens_night_02_4k.pfm",
                                 name: str = "material_spheres_ibl.sp") -> str:
    os.makedirs(directory, exist_ok=True)
    pfm = os.path.join(directory, image)
    if not os.path.exists(pfm):
        write_pfm(pfm, night_sky_image(width, height))
    path = os.path.join(directory, name)
    with open(path, "w") as fh:
        fh.write(material_spheres_sp(image))
    return path


# ---------------------------------------------------------------- lucy.sp / elf.sp
def cube_sphere(n: int):
    """Welded cube-sphere grid: unit directions (V, 3) float64 and triangles (12 n^2, 3) int32,
    outward winding.  Vertices are welded by their integer lattice position on the cube surface
    (cheap at tens of millions of triangles)."""
    keys, quads = [], []
    i, j = np.meshgrid(np.arange(n + 1), np.arange(n + 1), indexing="ij")
    i, j = i.ravel(), j.ravel()
    qi, qj = np.meshgrid(np.arange(n), np.arange(n), indexing="ij")
    q00 = (qi * (n + 1) + qj).ravel()
    base = 0
    lat = []
    for axis in range(3):
        for sign in (1, -1):
            a1, a2 = (axis + 1) % 3, (axis + 2) % 3
            c = np.empty((i.size, 3), dtype=np.int64)
            c[:, axis] = n if sign > 0 else 0
            c[:, a1] = i
            c[:, a2] = j
            lat.append(c)
            v00, v10, v01, v11 = q00 + base, q00 + base + (n + 1), q00 + base + 1, q00 + base + n + 2
            if sign > 0:
                quads.append(np.stack([v00, v10, v11, v01], -1))
            else:
                quads.append(np.stack([v00, v01, v11, v10], -1))
            base += i.size
    lat = np.concatenate(lat)
    key = (lat[:, 0] * (n + 1) + lat[:, 1]) * (n + 1) + lat[:, 2]
    uniq, first, inverse = np.unique(key, return_index=True, return_inverse=True)
    lat = lat[first]
    t = np.tan((lat / n * 2.0 - 1.0) * (np.pi / 4))  # equal-angle grid
    d = t / np.linalg.norm(t, axis=1, keepdims=True)
    q = inverse.reshape(-1)[np.concatenate(quads)]
    f = np.concatenate([q[:, [0, 1, 2]], q[:, [0, 2, 3]]]).astype(np.int32)
    return d, f


def _lobes(d: np.ndarray, lobes, ripples) -> np.ndarray:
    r = np.ones(d.shape[0])
    for c, w, a in lobes:
        c = np.asarray(c, dtype=np.float64)
        c = c / np.linalg.norm(c)
        r += a * np.exp(-np.sum((d - c) ** 2, axis=1) / w)
    for amp, fx, fy, fz in ripples:
        r += amp * np.sin(fx * d[:, 0] + 0.3) * np.sin(fy * d[:, 1] + 0.7) * np.sin(fz * d[:, 2] + 1.1)
    return r


def lucy_mesh(n: int = 1529):
    """Stand-in for the Stanford lucy.ply (14.0 M vertices, 28.06 M triangles; not in the
    reference repository): n = 1529 gives 14.03 M vertices / 28.05 M triangles.  A tall winged
    figure (radial lobes for head, wings, arms and robe) with drapery-like ripples at several
    frequencies, so the BVH is deep and boxes overlap like a scanned statue's.  Coordinates are
    in lucy.ply's frame: lucy.sp rotates it by -90 deg about x, stands it on the plane at
    y = -605.893 and frames it from (690.756, 500, -2000)."""
    d, f = cube_sphere(n)
    lobes = [((0.0, 0.0, 1.0), 0.05, 0.35),      # head (up = +z in the file frame)
             ((0.9, 0.3, 0.6), 0.10, 0.9),       # wing
             ((-0.9, 0.3, 0.6), 0.10, 0.9),      # wing
             ((0.6, -0.6, 0.1), 0.06, 0.35),     # arm
             ((-0.5, -0.7, 0.3), 0.06, 0.3),     # arm
             ((0.0, 0.0, -1.0), 0.4, 0.45)]      # robe
    ripples = [(0.02, 37.0, 29.0, 41.0), (0.008, 131.0, 97.0, 113.0), (0.003, 401.0, 367.0, 389.0)]
    p = d * _lobes(d, lobes, ripples)[:, None] * np.array([0.45, 0.3, 1.0])
    lo, hi = p.min(axis=0), p.max(axis=0)
    box_lo = np.array([690.756 - 420.0, -192.627 - 260.0, -605.893])
    box_hi = np.array([690.756 + 420.0, -192.627 + 260.0, -605.893 + 1610.0])
    p = box_lo + (p - lo) / (hi - lo) * (box_hi - box_lo)
    return p.astype(np.float32), f


def elf_mesh(n: int = 290):
    """Stand-in for stl_files/elf/nude-body.stl (not in the reference repository): a standing
    figure, 1.0 M triangles at n = 290, feet on elf.sp's plane (y = -42.7188), centred on its
    camera axis (x = -1.795, y = -0.034) at z = 13.84."""
    d, f = cube_sphere(n)
    lobes = [((0.0, 1.0, 0.0), 0.04, 0.3),       # head
             ((0.7, 0.45, 0.0), 0.05, 0.5),      # arms
             ((-0.7, 0.45, 0.0), 0.05, 0.5),
             ((0.25, -1.0, 0.0), 0.03, 0.45),    # legs
             ((-0.25, -1.0, 0.0), 0.03, 0.45)]
    ripples = [(0.01, 23.0, 31.0, 19.0), (0.004, 89.0, 71.0, 97.0)]
    p = d * _lobes(d, lobes, ripples)[:, None] * np.array([0.35, 1.0, 0.2])
    lo, hi = p.min(axis=0), p.max(axis=0)
    box_lo = np.array([-1.79536 - 18.0, -42.7188, 13.8378 - 8.0])
    box_hi = np.array([-1.79536 + 18.0, 42.7, 13.8378 + 8.0])
    p = box_lo + (p - lo) / (hi - lo) * (box_hi - box_lo)
    return p.astype(np.float32), f


def write_stl(path: str, verts: np.ndarray, faces: np.ndarray) -> None:
    """Binary STL (base/STLReader.cpp:46 layout): 80-byte header, count, then per triangle the
    unit face normal, three vertices and a 2-byte attribute count."""
    tri = verts[faces].astype(np.float32)
    nrm = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]).astype(np.float64)
    ln = np.linalg.norm(nrm, axis=1, keepdims=True)
    nrm = np.where(ln > 0, nrm / np.where(ln > 0, ln, 1.0), 0.0).astype(np.float32)
    rec = np.zeros(faces.shape[0], dtype=[("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")])
    rec["n"], rec["v"] = nrm, tri
    with open(path, "wb") as fh:
        fh.write(b"synthetic stand-in for nude-body.stl".ljust(80, b" "))
        fh.write(np.uint32(faces.shape[0]).tobytes())
        fh.write(rec.tobytes())


_FIGURE_MATERIALS = """material_glossy {
    name: "material_glossy_base"
    diffuse: 0.7 0.7 0.7
    ior: 1.3
    roughness: 0.75
}

material_glossy {
    name: "material_glossy_plane"
    diffuse: 0.4 0.1 0.1
    ior: 1.8
    roughness: 0.01
}

material_clearcoat {
    name: "material_glossy_clearcoat"
    base: "material_glossy_base"
    ior: 1.5
    color: 1.0 1.0 1.0
}
"""


def lucy_sp(ply_rel: str) -> str:
    """scenes/lucy.sp of the reference (mesh path pointing at the synthetic PLY)."""
    return f"""version: 1

scene_parameters {{
    output_file_name: "image.pfm"
    width: 1350
    height: 2000
}}

perspective_camera {{
    origin: 690.756 500.0 -2000.0
    look_at: 690.756 200.0 192.627
    fov: 45
}}

{_FIGURE_MATERIALS}
mesh {{
    file: "{ply_rel}"
    rotate: 1.0 0.0 0.0 -90.0
    material: "material_glossy_clearcoat"
}}

plane {{
    material: "material_glossy_plane"
    translate: 0.0 -605.893 0.0
}}

environment_light {{
    rotate: 0.0 1.0 0.0 45.0
    radiance: 1.0 1.0 1.3
}}
"""


def elf_sp(stl_rel: str, max_depth: int | None = None) -> str:
    """scenes/elf.sp of the reference; `max_depth` adds a scene_parameters max_depth (the
    BASELINE config renders it with max-depth 16).  The reference file writes the camera's
    look_at as "-1.79536, -0.0338669, 13.8378": under its parser (operator>> on floats) the comma
    fails the stream, so y becomes 0, z is left uninitialised (undefined) and the rest of the
    camera block is skipped.  The intended coordinates are written here instead."""
    md = "" if max_depth is None else f"\n    max_depth: {max_depth}"
    return f"""version: 1

scene_parameters {{
    output_file_name: "image.pfm"
    width: 1350
    height: 2000{md}
}}

perspective_camera {{
    origin: -1.79536 -0.0338669 130.0
    look_at: -1.79536 -0.0338669 13.8378
    fov: 45
}}

{_FIGURE_MATERIALS}
mesh {{
    file: "{stl_rel}"
    material: "material_glossy_clearcoat"
}}

plane {{
    material: "material_glossy_plane"
    translate: 0.0 -42.7188 0.0
}}

environment_light {{
    rotate: 0.0 1.0 0.0 45.0
    radiance: 0.75 0.75 0.75
}}
"""


def _write_once(path: str, writer) -> None:
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        tmp = path + ".tmp%d" % os.getpid()
        writer(tmp)
        os.replace(tmp, path)


def write_lucy_scene(directory: str, n: int = 1529, name: str = "lucy.sp") -> str:
    rel = os.path.join("ply_files", f"lucy_{n}.ply")
    _write_once(os.path.join(directory, rel), lambda p: write_ply(p, *lucy_mesh(n)))
    path = os.path.join(directory, name)
    with open(path, "w") as fh:
        fh.write(lucy_sp(rel))
    return path


def write_elf_scene(directory: str, n: int = 290, max_depth: int | None = 16, name: str = "elf.sp") -> str:
    rel = os.path.join("stl_files", "elf", f"nude-body_{n}.stl")
    _write_once(os.path.join(directory, rel), lambda p: write_stl(p, *elf_mesh(n)))
    path = os.path.join(directory, name)
    with open(path, "w") as fh:
        fh.write(elf_sp(rel, max_depth))
    return path


def closed_room_sp(max_depth: int = 40) -> str:
    """A camera inside a closed box of six inward-facing lambertian planes with a clearcoat
    ball and a sphere light: no path escapes, so the recursive integrators reach max_depth."""
    walls = [("0.0 -2.0 0.0", None), ("0.0 2.0 0.0", "1 0 0 180"), ("-2.0 0.0 0.0", "0 0 1 -90"),
             ("2.0 0.0 0.0", "0 0 1 90"), ("0.0 0.0 -6.0", "1 0 0 90"), ("0.0 0.0 2.0", "1 0 0 -90")]
    planes = ""
    for t, r in walls:
        planes += "plane {\n    material: \"wall\"\n    translate: %s\n" % t
        if r:
            planes += "    rotate: %s\n" % r
        planes += "}\n\n"
    return f"""version: 1

scene_parameters {{
    output_file_name: "room.pfm"
    width: 16
    height: 16
    max_depth: {max_depth}
}}

perspective_camera {{
    origin: 0.0 0.0 0.0
    look_at: 0.0 0.0 -1.0
    fov: 60
}}

material_lambertian {{
    name: "wall"
    diffuse: 0.9 0.85 0.8
}}

material_glossy {{
    name: "ball_base"
    diffuse: 0.8 0.3 0.3
    ior: 1.5
    roughness: 0.3
}}

material_clearcoat {{
    name: "ball"
    base: "ball_base"
    ior: 1.5
    color: 1.0 1.0 1.0
}}

{planes}sphere {{
    translate: 0.0 -1.0 -4.0
    material: "ball"
}}

sphere_light {{
    translate: 0.0 1.5 -3.0
    scale: 0.5 0.5 0.5
    radiance: 5.0 5.0 5.0
}}
"""


def write_closed_room_scene(directory: str, max_depth: int = 40, name: str = "closed_room.sp") -> str:
    os.makedirs(directory, exist_ok=True)
    path = os.path.join(directory, name)
    with open(path, "w") as fh:
        fh.write(closed_room_sp(max_depth))
    return path


# ---------------------------------------------------------------- degenerate BVH (stackless walk)
def wedge_strip_mesh(ratio: float = 1.9, lo_exp: int = -80, hi_exp: int = 135):
    """A strip of wedge triangles whose sizes form a geometric series, x_i = ratio^i from about
    6e-23 to 5e37: triangle i spans x in [x_i, 1.25 x_i] and y in [-x_i / 2, x_i / 2] on the
    z = 0 plane (smaller ones would have a zero cross product in float and be dropped as
    degenerate by the loader).  The reference's median split (shapes/BVHAccelerator.h:173:
    midpoint of the bounds on the longest axis) peels only the largest triangle off at almost
    every level, so its recursion nests 172 levels deep -- more than any LDS stack budget
    (tests/test_gpu_parity.py: the device walks it without a stack)."""
    i = np.arange(lo_exp, hi_exp + 1, dtype=np.float64)
    x = (ratio ** i).astype(np.float32).astype(np.float64)
    v = np.zeros((3 * x.size, 3), dtype=np.float32)
    v[0::3, 0], v[0::3, 1] = x, -0.5 * x
    v[1::3, 0], v[1::3, 1] = 1.25 * x, -0.5 * x
    v[2::3, 0], v[2::3, 1] = x, 0.5 * x
    f = np.arange(3 * x.size, dtype=np.int32).reshape(-1, 3)
    return v, f


def wedge_strip_sp(ply_rel: str, max_depth: int = 3) -> str:
    """The wedge strip seen from above its origin, a lambertian plane under it, a sphere light
    and an environment light."""
    return f"""version: 1

scene_parameters {{
    output_file_name: "strip.pfm"
    width: 64
    height: 48
    max_depth: {max_depth}
}}

perspective_camera {{
    origin: 0.6 0.0 2.0
    look_at: 0.6 0.0 0.0
    fov: 50
}}

material_lambertian {{
    name: "strip"
    diffuse: 0.8 0.6 0.3
}}

material_glossy {{
    name: "floor"
    diffuse: 0.3 0.3 0.6
    ior: 1.5
    roughness: 0.3
}}

mesh {{
    file: "{ply_rel}"
    material: "strip"
}}

plane {{
    material: "floor"
    rotate: 1.0 0.0 0.0 90.0
    translate: 0.0 0.0 -0.25
}}

sphere_light {{
    translate: 0.5 0.5 1.5
    scale: 0.2 0.2 0.2
    radiance: 20.0 20.0 20.0
}}

environment_light {{
    radiance: 0.2 0.2 0.3
}}
"""


def write_wedge_strip_scene(directory: str, name: str = "wedge_strip.sp", max_depth: int = 3) -> str:
    rel = os.path.join("ply_files", "wedge_strip.ply")
    _write_once(os.path.join(directory, rel), lambda p: write_ply(p, *wedge_strip_mesh()))
    path = os.path.join(directory, name)
    with open(path, "w") as fh:
        fh.write(wedge_strip_sp(rel, max_depth))
    return path
