"""Procedural simulator assets (sim/assets.py): block meshes are closed prisms of the renderer's footprints, URDFs
round-trip through the loader, and the contact radii the meshes imply are the physics' radii.  Parity with the
reference's Blender meshes is unpinned (pybullet is not importable; the reference's asset files are not read)."""
import math

import numpy as np
import pytest

from pytorch_rt1_for_distributed_training_amd.sim import assets, board, world


def _point_in_poly(poly, pts):
    x, y = pts[:, 0][:, None], pts[:, 1][:, None]
    x0, y0 = poly[:, 0][None], poly[:, 1][None]
    x1, y1 = np.roll(poly[:, 0], -1)[None], np.roll(poly[:, 1], -1)[None]
    cond = (y0 > y) != (y1 > y)
    xint = x0 + (y - y0) * (x1 - x0) / np.where(y1 == y0, 1e-30, y1 - y0)
    return (cond & (x < xint)).sum(1) % 2 == 1


@pytest.mark.parametrize("shape", assets.SHAPES)
def test_footprint_agrees_with_render_mask(shape):
    r = world.POLE_RADIUS if shape == "pole" else world.BLOCK_RADIUS
    poly = assets.footprint(shape, r, n=96)
    rng = np.random.default_rng(0)
    pts = rng.uniform(-1.1 * r, 1.1 * r, (6000, 2))
    inside = _point_in_poly(poly, pts)
    mask = world._shape_mask(shape if shape != "pole" else "disc", pts[:, 0], pts[:, 1], r)
    agree = (inside == mask).mean()
    assert agree > 0.985, agree


@pytest.mark.parametrize("shape", assets.SHAPES)
def test_extruded_mesh_is_closed_and_outward(shape):
    r = world.POLE_RADIUS if shape == "pole" else world.BLOCK_RADIUS
    poly = assets.footprint(shape, r)
    h = assets.BLOCK_HEIGHT
    v, f = assets.extrude(poly, h)
    # every undirected edge is shared by exactly two triangles, with opposite orientations
    edges = {}
    for a, b, c in f:
        for e in ((a, b), (b, c), (c, a)):
            edges[e] = edges.get(e, 0) + 1
    for (a, b), n in edges.items():
        assert n == 1 and edges.get((b, a)) == 1
    assert math.isclose(assets.mesh_volume(v, f), assets.polygon_area(poly) * h, rel_tol=1e-9)


def test_write_and_load_asset_tree(tmp_path):
    paths = assets.write_assets(str(tmp_path))
    assert set(board.all_block_names()) | {"workspace", "plane"} == set(paths)
    for name in board.all_block_names():
        body = assets.load_urdf(paths[name])
        color, shape = board.color_shape(name)
        assert body.name == f"{name}.urdf"
        assert body.mass == assets.BLOCK_MASS and body.lateral_friction == assets.LATERAL_FRICTION
        assert body.rgba[:3] == tuple(round(c / 255.0, 4) for c in board.RGB[color])
        v, f = assets.load_obj(body.mesh)
        assert v.shape[1] == 3 and f.shape[1] == 3 and f.max() < len(v)
        want = world.POLE_RADIUS if shape == "pole" else world.BLOCK_RADIUS
        rad = assets.footprint_radius(body.mesh)
        outer = 0.78 * math.sqrt(2) * want if shape == "cube" else want         # the cube's corners reach past r
        assert abs(rad - outer) < 1e-6                                           # OBJ keeps 1 um
    ws = assets.load_urdf(paths["workspace"])
    assert ws.mass == 0.0 and ws.box[0] > board.X_MAX - board.X_MIN and ws.box[1] > board.Y_MAX - board.Y_MIN
    pv, pf = assets.load_obj(paths["plane"])
    assert pv.shape == (4, 3) and pf.shape == (2, 3)
