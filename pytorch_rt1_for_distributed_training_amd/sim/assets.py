"""Procedural simulator assets: block meshes (OBJ), block / workspace URDFs, and loaders for both.

Behavioural spec: the reference ships hand-made Blender meshes and one URDF per coloured block under
``language_table/environments/assets/{blocks,suction}`` and a workspace URDF, loaded by pybullet
(``language_table/environments/language_table.py:556-563,659-661,738-760``, ``blocks.py:86-110``).  pybullet is
not importable here; this module GENERATES an equivalent asset tree from the
planar simulator's own block footprints (``sim.world._shape_mask``: moon / cube / star / pentagon at the block
radius, the goal pole as a disc), so that the geometry the renderer draws, the geometry the meshes describe and the
contact radii the physics uses are one definition.  The URDF fields follow the reference's block files (mass 0.01 kg,
lateral friction 0.5, rolling friction 1e-4, a mesh for visual + collision, an RGBA material).

    paths = write_assets("/tmp/lt_assets")      # {"red_moon": ".../blocks/red_moon.urdf", ..., "workspace": ...}
    spec = load_urdf(paths["red_moon"])         # UrdfBody(name, mass, lateral_friction, rgba, mesh, scale)
    verts, faces = load_obj(spec.mesh)
    env = LanguageTable(asset_root="/tmp/lt_assets")   # the world takes block sizes / colours from these files

No file of the reference is read or reproduced: meshes are extruded polygons computed here.
"""
from __future__ import annotations

import dataclasses
import math
import os
import xml.etree.ElementTree as ET
from typing import Dict, List, Sequence, Tuple

import numpy as np

from . import board
from .world import BLOCK_RADIUS, POLE_RADIUS

BLOCK_HEIGHT = 0.0381          # 1.5 in blocks
POLE_HEIGHT = 0.1
BLOCK_MASS = 0.01
LATERAL_FRICTION = 0.5
ROLLING_FRICTION = 1e-4
SHAPES = tuple(board.SHAPES) + ("pole",)


# ---------------------------------------------------------------- 2-D footprints (counter-clockwise polygons)
def footprint(shape: str, r: float = BLOCK_RADIUS, n: int = 48) -> np.ndarray:
    """Counter-clockwise outline [P, 2] (metres, block frame) of a block's footprint, matching the renderer's
    ``_shape_mask`` for the same radius."""
    if shape == "cube":
        h = 0.78 * r
        return np.array([[-h, -h], [h, -h], [h, h], [-h, h]])
    if shape == "pentagon":
        a = 2 * math.pi * np.arange(5) / 5                                  # vertices on the mask's sector bounds
        return np.stack([r * np.cos(a), r * np.sin(a)], -1)
    if shape == "star":
        # the mask's outline: radius r * (1 - 0.55 a), a = 0 at the tips (sector centres) .. 1 between them
        m = 10 * max(2, n // 10)
        phi = 2 * math.pi * np.arange(m) / m
        sector = 2 * math.pi / 5
        a = np.abs(np.mod(phi, sector) - sector / 2) / (sector / 2)
        rad = r * (1.0 - 0.55 * a)
        return np.stack([rad * np.cos(phi), rad * np.sin(phi)], -1)
    if shape == "moon":
        # disc(0, r) minus disc((0.55 r, 0), 0.8 r): the outer arc, then the inner arc back
        c, rin = 0.55 * r, 0.8 * r
        # intersection points of the two circles
        xi = (r * r - rin * rin + c * c) / (2 * c)
        yi = math.sqrt(max(r * r - xi * xi, 0.0))
        t0 = math.atan2(yi, xi)
        outer = np.linspace(t0, 2 * math.pi - t0, n)
        pts = [np.stack([r * np.cos(outer), r * np.sin(outer)], -1)]
        # the bite's arc inside the disc, from the lower intersection through (c - rin, 0) to the upper one
        u0 = math.atan2(-yi, xi - c) % (2 * math.pi)                        # ~270 deg about the bite centre
        u1 = math.atan2(yi, xi - c)                                         # ~90 deg
        inner = np.linspace(u0, u1, n)[1:-1]
        pts.append(np.stack([c + rin * np.cos(inner), rin * np.sin(inner)], -1))
        return np.concatenate(pts, 0)
    if shape == "pole":
        a = 2 * math.pi * np.arange(n) / n
        return np.stack([r * np.cos(a), r * np.sin(a)], -1)
    raise ValueError(f"unknown shape {shape!r}")


def polygon_area(p: np.ndarray) -> float:
    x, y = p[:, 0], p[:, 1]
    return 0.5 * float(np.dot(x, np.roll(y, -1)) - np.dot(y, np.roll(x, -1)))


def _ear_clip(p: np.ndarray) -> List[Tuple[int, int, int]]:
    """Triangulate a simple counter-clockwise polygon (O(P^2) ear clipping)."""
    idx = list(range(len(p)))
    tris = []

    def cross(o, a, b):
        return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0])

    guard = 0
    while len(idx) > 3 and guard < 10 * len(p) * len(p):
        guard += 1
        m = len(idx)
        for k in range(m):
            i0, i1, i2 = idx[(k - 1) % m], idx[k], idx[(k + 1) % m]
            a, b, c = p[i0], p[i1], p[i2]
            if cross(a, b, c) <= 1e-18:                                     # reflex or degenerate corner
                continue
            inside = False
            for j in idx:
                if j in (i0, i1, i2):
                    continue
                q = p[j]
                if cross(a, b, q) >= 0 and cross(b, c, q) >= 0 and cross(c, a, q) >= 0:
                    inside = True
                    break
            if inside:
                continue
            tris.append((i0, i1, i2))
            idx.pop(k)
            break
        else:
            raise ValueError("polygon is not simple")
    tris.append(tuple(idx))
    return tris


def extrude(poly: np.ndarray, height: float) -> Tuple[np.ndarray, np.ndarray]:
    """Closed prism mesh of a counter-clockwise polygon: vertices [2P, 3], outward triangles [T, 3] (0-based).
    z runs from 0 (table) to ``height``."""
    P = len(poly)
    v = np.concatenate([np.c_[poly, np.zeros(P)], np.c_[poly, np.full(P, height)]], 0)
    caps = _ear_clip(poly)
    faces = [(c, b, a) for a, b, c in caps]                                  # bottom faces down
    faces += [(a + P, b + P, c + P) for a, b, c in caps]                     # top faces up
    for i in range(P):
        j = (i + 1) % P
        faces += [(i, j, j + P), (i, j + P, i + P)]                          # side quads, outward for CCW
    return v, np.asarray(faces, np.int64)


def mesh_volume(v: np.ndarray, f: np.ndarray) -> float:
    """Signed volume of a closed, outward-oriented triangle mesh (divergence theorem)."""
    a, b, c = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    return float(np.einsum("ij,ij->i", a, np.cross(b, c)).sum() / 6.0)


# ---------------------------------------------------------------- OBJ
def obj_text(v: np.ndarray, f: np.ndarray, name: str) -> str:
    lines = [f"# rt1-mi355x procedural mesh: {name}", f"o {name}"]
    lines += [f"v {x:.6f} {y:.6f} {z:.6f}" for x, y, z in v]
    lines += [f"f {a + 1} {b + 1} {c + 1}" for a, b, c in f]
    return "\n".join(lines) + "\n"


def load_obj(path: str) -> Tuple[np.ndarray, np.ndarray]:
    """Vertices [V, 3] and 0-based triangles [F, 3] of an OBJ file (v / f records; polygons are fanned)."""
    vs, fs = [], []
    with open(path) as fh:
        for line in fh:
            t = line.split()
            if not t:
                continue
            if t[0] == "v":
                vs.append([float(x) for x in t[1:4]])
            elif t[0] == "f":
                ids = [int(x.split("/")[0]) for x in t[1:]]
                ids = [i - 1 if i > 0 else len(vs) + i for i in ids]
                for k in range(1, len(ids) - 1):
                    fs.append([ids[0], ids[k], ids[k + 1]])
    return np.asarray(vs, np.float64), np.asarray(fs, np.int64)


# ---------------------------------------------------------------- URDF
@dataclasses.dataclass
class UrdfBody:
    name: str
    mass: float
    lateral_friction: float
    rolling_friction: float
    rgba: Tuple[float, float, float, float]
    mesh: str                     # absolute path of the visual / collision mesh ("" for primitive boxes)
    scale: Tuple[float, float, float]
    box: Tuple[float, float, float] = (0.0, 0.0, 0.0)


def _rgba(color: str) -> Tuple[float, float, float, float]:
    r, g, b = board.RGB[color]
    return (round(r / 255.0, 4), round(g / 255.0, 4), round(b / 255.0, 4), 1.0)


def urdf_text(name: str, geometry: ET.Element, rgba, mass: float = BLOCK_MASS) -> str:
    robot = ET.Element("robot", name=name)
    link = ET.SubElement(robot, "link", name="baseLink")
    contact = ET.SubElement(link, "contact")
    ET.SubElement(contact, "lateral_friction", value=f"{LATERAL_FRICTION}")
    ET.SubElement(contact, "rolling_friction", value=f"{ROLLING_FRICTION}")
    inertial = ET.SubElement(link, "inertial")
    ET.SubElement(inertial, "origin", rpy="0 0 0", xyz="0 0 0")
    ET.SubElement(inertial, "mass", value=f"{mass}")
    ET.SubElement(inertial, "inertia", ixx="1", ixy="0", ixz="0", iyy="1", iyz="0", izz="1")
    for tag in ("visual", "collision"):
        el = ET.SubElement(link, tag)
        ET.SubElement(el, "origin", rpy="0 0 0", xyz="0 0 0")
        geom = ET.SubElement(el, "geometry")
        geom.append(geometry)
        if tag == "visual":
            mat = ET.SubElement(el, "material", name=name)
            ET.SubElement(mat, "color", rgba=" ".join(f"{c:g}" for c in rgba))
    ET.indent(robot)
    return '<?xml version="1.0" ?>\n' + ET.tostring(robot, encoding="unicode") + "\n"


def load_urdf(path: str) -> UrdfBody:
    """The single-link URDF fields the simulator uses: mass, friction, colour, mesh (resolved next to the file)."""
    root = ET.parse(path).getroot()
    link = root.find("link")
    mass = float(link.find("inertial/mass").get("value"))
    contact = link.find("contact")
    lat = float(contact.find("lateral_friction").get("value")) if contact is not None else 0.5
    rol = float(contact.find("rolling_friction").get("value")) if contact is not None else 0.0
    color = link.find("visual/material/color")
    rgba = tuple(float(x) for x in color.get("rgba").split()) if color is not None else (1.0, 1.0, 1.0, 1.0)
    mesh_el = link.find("visual/geometry/mesh")
    box_el = link.find("visual/geometry/box")
    mesh, scale, box = "", (1.0, 1.0, 1.0), (0.0, 0.0, 0.0)
    if mesh_el is not None:
        mesh = os.path.join(os.path.dirname(os.path.abspath(path)), mesh_el.get("filename"))
        scale = tuple(float(x) for x in mesh_el.get("scale", "1 1 1").split())
    if box_el is not None:
        box = tuple(float(x) for x in box_el.get("size").split())
    return UrdfBody(root.get("name"), mass, lat, rol, rgba, mesh, scale, box)


# ---------------------------------------------------------------- the asset tree
def write_assets(root: str, blocks: Sequence[str] = None) -> Dict[str, str]:
    """Write meshes + URDFs for ``blocks`` (default: every block the simulator knows) and the workspace under
    ``root``; returns {block name: URDF path, "workspace": ..., "plane": OBJ path} like the reference's
    ``_get_urdf_paths``."""
    blocks = list(blocks) if blocks is not None else board.all_block_names()
    bdir = os.path.join(root, "blocks")
    os.makedirs(bdir, exist_ok=True)
    paths: Dict[str, str] = {}
    meshes = {}
    for name in blocks:
        color, shape = board.color_shape(name)
        if shape not in meshes:
            r, h = (POLE_RADIUS, POLE_HEIGHT) if shape == "pole" else (BLOCK_RADIUS, BLOCK_HEIGHT)
            v, f = extrude(footprint(shape, r), h)
            with open(os.path.join(bdir, f"{shape}.obj"), "w") as fh:
                fh.write(obj_text(v, f, shape))
            meshes[shape] = f"{shape}.obj"
        geom = ET.Element("mesh", filename=meshes[shape], scale="1.0 1.0 1.0")
        p = os.path.join(bdir, f"{name}.urdf")
        with open(p, "w") as fh:
            fh.write(urdf_text(f"{name}.urdf", geom, _rgba(color)))
        paths[name] = p
    # the workspace: a thin static board over the workspace bounds (mass 0 = fixed in URDF convention)
    sx, sy = board.X_MAX - board.X_MIN + 2 * board.WORKSPACE_BOUNDS_BUFFER, board.Y_MAX - board.Y_MIN + \
        2 * board.WORKSPACE_BOUNDS_BUFFER
    geom = ET.Element("box", size=f"{sx:.4f} {sy:.4f} 0.01")
    p = os.path.join(root, "workspace.urdf")
    with open(p, "w") as fh:
        fh.write(urdf_text("workspace.urdf", geom, (0.2, 0.2, 0.2, 1.0), mass=0.0))
    paths["workspace"] = p
    v = np.array([[-5, -5, 0], [5, -5, 0], [5, 5, 0], [-5, 5, 0]], np.float64)
    f = np.array([[0, 1, 2], [0, 2, 3]])
    p = os.path.join(root, "plane.obj")
    with open(p, "w") as fh:
        fh.write(obj_text(v, f, "plane"))
    paths["plane"] = p
    return paths


def footprint_radius(mesh_path: str) -> float:
    """Largest horizontal distance of a mesh vertex from the block axis (the contact radius it implies)."""
    v, _ = load_obj(mesh_path)
    return float(np.hypot(v[:, 0], v[:, 1]).max())
