"""Planar quasi-static pushing world + pinhole renderer for the Language-Table board.

The reference simulates the board with pybullet (xArm6 + cylinder effector, URDF blocks,
``stepSimulation`` x sim_hz/10 per control step, TinyRenderer camera, ``language_table.py:579-646``).
pybullet is not part of this stack, so the board is modelled directly in 2-D, which is what every task
reward and oracle reads anyway (block xy + yaw, effector xy):

* the effector is a disc that tracks its commanded xy target in ``substeps`` straight-line moves per control
  step (the reference's IK tracking, without arm dynamics);
* blocks are rigid footprints with a collision radius; contacts are resolved by iterative position
  projection (effector pushes blocks, blocks push blocks), i.e. quasi-static pushing with full friction:
  a block moves only while it is pushed; an off-centre push also turns the block (yaw), as a real push does;
* blocks stay on the board (the board's rim);
* the camera is the reference's (pose ``(0.75, 0, 0.5)``, Euler ``(pi/5, pi, -pi/2)``, fx = 0.803 W,
  180 x 320): every pixel's ray is intersected with the table plane once, and each frame paints the block
  footprints (moon / cube / star / pentagon / pole) and the effector into that table image.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import board

BLOCK_RADIUS = 0.0175          # collision radius of a block footprint (m)
POLE_RADIUS = 0.012
EFFECTOR_RADIUS = 0.011
OFF_TABLE = np.array([5.0, 5.0])
_CIRCUM = {"cube": 0.78 * math.sqrt(2.0)}   # footprint circumradius / size parameter r (1 for the round shapes)
RIM = 0.03                     # how far past the workspace bounds a block may be pushed


def _rot_from_euler(roll, pitch, yaw):
    cr, sr, cp, sp, cy, sy = math.cos(roll), math.sin(roll), math.cos(pitch), math.sin(pitch), math.cos(yaw), \
        math.sin(yaw)
    rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    return rz @ ry @ rx


class Camera:
    """Pinhole camera of the reference (``calc_camera_params``): look along R.z, image-up along -R.y."""

    def __init__(self, pose=board.CAMERA_POSE, euler=board.CAMERA_ORIENTATION, height=board.IMAGE_HEIGHT,
                 width=board.IMAGE_WIDTH, focal=board.FOCAL_PX):
        self.eye = np.asarray(pose, np.float64)
        r = _rot_from_euler(*euler)
        fwd = r @ np.array([0.0, 0.0, 1.0])
        up = r @ np.array([0.0, -1.0, 0.0])
        right = np.cross(fwd, up)
        right /= np.linalg.norm(right)
        up = np.cross(right, fwd)
        self.fwd, self.up, self.right = fwd, up, right
        self.h, self.w, self.f = height, width, focal

    def table_points(self) -> np.ndarray:
        """World xy hit by each pixel's ray on the table plane z = 0 (NaN where the ray misses it)."""
        py, px = np.mgrid[0:self.h, 0:self.w].astype(np.float64)
        d = (self.fwd[None, None] * self.f + self.right[None, None] * (px[..., None] + 0.5 - self.w / 2.0)
             + self.up[None, None] * (self.h / 2.0 - py[..., None] - 0.5))
        t = -self.eye[2] / d[..., 2]
        xy = self.eye[None, None, :2] + t[..., None] * d[..., :2]
        xy[t <= 0] = np.nan
        return xy

    def pixel_to_table(self, row: float, col: float) -> np.ndarray:
        """Table point (x, y) seen at pixel centre (row, col) -- the reference's ``image_xy_to_view_ray`` +
        ``ray_to_plane_test`` (``utils_pybullet.py:158-196``); NaN when the ray misses the table."""
        d = self.fwd * self.f + self.right * (col + 0.5 - self.w / 2.0) + self.up * (self.h / 2.0 - row - 0.5)
        if d[2] >= 0:
            return np.array([np.nan, np.nan])
        t = -self.eye[2] / d[2]
        return self.eye[:2] + t * d[:2]

    def project(self, xyz) -> np.ndarray:
        """World point(s) -> (row, col) pixel coordinates."""
        p = np.atleast_2d(np.asarray(xyz, np.float64)) - self.eye
        z = p @ self.fwd
        col = (p @ self.right) * self.f / z + self.w / 2.0
        row = self.h / 2.0 - (p @ self.up) * self.f / z
        return np.stack([row, col], -1)


def _shape_mask(shape: str, lx: np.ndarray, ly: np.ndarray, r: float) -> np.ndarray:
    """Footprint membership of block-local points (metres), block frame = yaw-aligned."""
    if shape == "cube":
        return np.maximum(np.abs(lx), np.abs(ly)) <= 0.78 * r
    rho = np.hypot(lx, ly)
    phi = np.arctan2(ly, lx)
    if shape == "pentagon":
        sector = 2 * math.pi / 5
        a = np.mod(phi, sector) - sector / 2
        return rho * np.cos(a) <= r * math.cos(sector / 2)
    if shape == "star":
        sector = 2 * math.pi / 5
        a = np.abs(np.mod(phi, sector) - sector / 2) / (sector / 2)      # 0 at a tip .. 1 between tips
        return rho <= r * (1.0 - 0.55 * a)
    if shape == "moon":
        return (rho <= r) & (np.hypot(lx - 0.55 * r, ly) > 0.8 * r)
    return rho <= r                                                        # pole / fallback: disc


class PlanarWorld:
    """Block + effector state, quasi-static contact resolution, rendering."""

    def __init__(self, names: Sequence[str] = None, substeps: int = 10, iterations: int = 6,
                 camera: Optional[Camera] = None):
        self.names: List[str] = list(names or board.all_block_names())
        self.index = {n: i for i, n in enumerate(self.names)}
        n = len(self.names)
        self.pos = np.tile(OFF_TABLE, (n, 1)).astype(np.float64)
        self.yaw = np.zeros(n)
        self.active = np.zeros(n, bool)
        self.radius = np.array([POLE_RADIUS if nm.endswith("pole") else BLOCK_RADIUS for nm in self.names])
        self.color = np.array([board.RGB.get(board.color_shape(nm)[0], (128, 128, 128)) for nm in self.names],
                              np.uint8)
        self.bodies: Dict[str, object] = {}
        self.effector = np.array([board.CENTER_X, board.CENTER_Y])
        self.effector_target = self.effector.copy()
        self.substeps, self.iterations = substeps, iterations
        self.camera = camera or Camera()
        self._xy = self.camera.table_points()
        self._base = self._table_image()

    def load_assets(self, paths: Dict[str, str]):
        """Take block geometry and colour from URDF / OBJ assets (``sim.assets.write_assets`` output, the
        reference's ``_get_urdf_paths`` + ``load_urdf``, ``language_table.py:738-760``): each block's contact
        radius is its mesh's footprint radius, its paint colour the URDF material.  Blocks without a URDF keep
        the built-in geometry."""
        from . import assets
        for name, path in paths.items():
            if name not in self.index:
                continue
            body = assets.load_urdf(path)
            i = self.index[name]
            if body.mesh:
                # the footprint's circumradius over the shape's circumradius at unit size = the block's size
                # (contact disc and painted footprint scale together; the generated tree reproduces the defaults)
                shape = board.color_shape(name)[1]
                self.radius[i] = assets.footprint_radius(body.mesh) * body.scale[0] / _CIRCUM.get(shape, 1.0)
            self.color[i] = np.round(np.asarray(body.rgba[:3]) * 255.0).astype(np.uint8)
            self.bodies[name] = body
        return self

    # ------------------------------------------------------------------ state
    def place(self, name: str, xy, yaw: float = 0.0, active: bool = True):
        i = self.index[name]
        self.pos[i] = xy
        self.yaw[i] = yaw
        self.active[i] = active

    def remove_all(self):
        self.pos[:] = OFF_TABLE
        self.active[:] = False

    def get_state(self) -> Dict[str, np.ndarray]:
        return {"pos": self.pos.copy(), "yaw": self.yaw.copy(), "active": self.active.copy(),
                "effector": self.effector.copy(), "effector_target": self.effector_target.copy()}

    def set_state(self, s: Dict[str, np.ndarray]):
        self.pos, self.yaw, self.active = s["pos"].copy(), s["yaw"].copy(), s["active"].copy()
        self.effector, self.effector_target = s["effector"].copy(), s["effector_target"].copy()

    # ------------------------------------------------------------------ dynamics
    def set_effector_target(self, xy):
        self.effector_target = np.clip(np.asarray(xy, np.float64), board.WORKSPACE_BOUNDS[0],
                                       board.WORKSPACE_BOUNDS[1])

    def step(self):
        """One control step: the effector moves to its target in ``substeps`` moves, contacts resolved after each."""
        start = self.effector.copy()
        for k in range(1, self.substeps + 1):
            self.effector = start + (self.effector_target - start) * (k / self.substeps)
            self.resolve()

    def settle(self):
        for _ in range(4):
            self.resolve()

    def resolve(self):
        idx = np.flatnonzero(self.active)
        if idx.size == 0:
            return
        lo = board.WORKSPACE_BOUNDS[0] - RIM
        hi = board.WORKSPACE_BOUNDS[1] + RIM
        for _ in range(self.iterations):
            moved = False
            # effector -> blocks
            d = self.pos[idx] - self.effector
            dist = np.linalg.norm(d, axis=1)
            pen = self.radius[idx] + EFFECTOR_RADIUS - dist
            for j in np.flatnonzero(pen > 1e-9):
                i = idx[j]
                nrm = d[j] / dist[j] if dist[j] > 1e-9 else np.array([1.0, 0.0])
                self.pos[i] += nrm * pen[j]
                # off-centre push turns the block: torque ~ lateral offset of the contact w.r.t. the push
                push = self.effector_target - self.effector
                if np.linalg.norm(push) > 1e-9:
                    pd = push / np.linalg.norm(push)
                    lateral = pd[0] * (-nrm[1]) + pd[1] * nrm[0]
                    self.yaw[i] += 2.0 * lateral * pen[j] / self.radius[i]
                moved = True
            # block <-> block
            if idx.size > 1:
                p = self.pos[idx]
                diff = p[:, None, :] - p[None, :, :]
                dd = np.linalg.norm(diff, axis=-1)
                rr = self.radius[idx][:, None] + self.radius[idx][None, :]
                over = np.triu((rr - dd) > 1e-9, 1)
                for a, b in zip(*np.nonzero(over)):
                    ia, ib = idx[a], idx[b]
                    v = self.pos[ia] - self.pos[ib]
                    n = np.linalg.norm(v)
                    v = v / n if n > 1e-9 else np.array([0.0, 1.0])
                    corr = 0.5 * (rr[a, b] - n)
                    self.pos[ia] += v * corr
                    self.pos[ib] -= v * corr
                    moved = True
            self.pos[idx] = np.clip(self.pos[idx], lo, hi)
            if not moved:
                break
        self.yaw = np.mod(self.yaw + math.pi, 2 * math.pi) - math.pi

    # ------------------------------------------------------------------ rendering
    def _table_image(self) -> np.ndarray:
        xy = self._xy
        img = np.empty(xy.shape[:2] + (3,), np.uint8)
        img[:] = (92, 92, 96)                                               # floor / background
        ok = ~np.isnan(xy[..., 0])
        x, y = np.where(ok, xy[..., 0], 0), np.where(ok, xy[..., 1], 0)
        lo, hi = board.WORKSPACE_BOUNDS[0] - 0.04, board.WORKSPACE_BOUNDS[1] + 0.04
        on_board = ok & (x >= lo[0]) & (x <= hi[0]) & (y >= lo[1]) & (y <= hi[1])
        img[on_board] = (222, 214, 196)                                     # board surface
        rim = on_board & ~((x >= lo[0] + 0.012) & (x <= hi[0] - 0.012) & (y >= lo[1] + 0.012) & (y <= hi[1] - 0.012))
        img[rim] = (170, 160, 140)
        return img

    def render(self) -> np.ndarray:
        img = self._base.copy()
        xy = self._xy
        for i in np.flatnonzero(self.active):
            name = self.names[i]
            r = self.radius[i]
            dx = xy[..., 0] - self.pos[i, 0]
            dy = xy[..., 1] - self.pos[i, 1]
            near = np.abs(dx) < 1.2 * r
            near &= np.abs(dy) < 1.2 * r
            if not near.any():
                continue
            c, s = math.cos(-self.yaw[i]), math.sin(-self.yaw[i])
            lx = c * dx[near] - s * dy[near]
            ly = s * dx[near] + c * dy[near]
            shape = name.split("_")[1]
            m = _shape_mask(shape, lx, ly, r)
            rows, cols = np.nonzero(near)
            img[rows[m], cols[m]] = self.color[i]
        de = np.hypot(xy[..., 0] - self.effector[0], xy[..., 1] - self.effector[1])
        img[de <= EFFECTOR_RADIUS] = (40, 40, 44)
        img[(de > EFFECTOR_RADIUS) & (de <= EFFECTOR_RADIUS + 0.003)] = (235, 235, 235)
        return img
