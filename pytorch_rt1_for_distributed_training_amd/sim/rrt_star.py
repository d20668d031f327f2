"""RRT* shortest collision-free 2-D paths among disc obstacles.

Behavioural spec: ``language_table/environments/oracles/rrt_star.py:25-357`` -- the planner the reference's
push oracle (``push_oracle_rrt_slowdown.py:201-262``, ``:467-500``) runs to route a block (and the effector) around
the other blocks inside the workspace box, with a goal-sampling bias, a fixed step length, a rewiring radius and
an iteration cap; on failure it falls back to the direct segment [goal, start].

This is an independent, array-based implementation:
  * the tree lives in preallocated numpy arrays (xy, parent, cost), so nearest / near-neighbour queries are one
    vectorised distance computation instead of per-node Python loops;
  * collision checks are exact segment-vs-inflated-disc distance tests plus the workspace box (inflated by
    ``delta``), evaluated for all obstacles at once;
  * rewiring propagates cost changes to descendants through the parent array (no child lists);
  * randomness comes from a caller-supplied ``np.random.Generator`` -> plans are reproducible per seed.
Returned paths run goal -> start, like the reference's ``extract_path``.
"""
from __future__ import annotations

import dataclasses
from typing import List, Optional, Sequence, Tuple

import numpy as np


@dataclasses.dataclass
class Plan:
    path: List[Tuple[float, float]]      # goal ... start
    success: bool
    tree_xy: np.ndarray                  # [n, 2] explored vertices (for plotting)
    tree_parent: np.ndarray              # [n] parent index (-1 at the root)


def _seg_disc_dist(p0: np.ndarray, p1: np.ndarray, centres: np.ndarray) -> np.ndarray:
    """Distance from segment p0-p1 to each centre [k, 2]."""
    d = p1 - p0
    dd = float(d @ d)
    if dd < 1e-18:
        return np.linalg.norm(centres - p0, axis=1)
    t = np.clip(((centres - p0) @ d) / dd, 0.0, 1.0)
    proj = p0 + t[:, None] * d
    return np.linalg.norm(centres - proj, axis=1)


class RRTStar:
    """RRT* in a box [x_range] x [y_range] with disc obstacles (x, y, diameter) inflated by ``delta``."""

    def __init__(self, start, goal, obstacles: Sequence[Tuple[float, float, float]], x_range, y_range,
                 delta: float, step_len: float, goal_sample_rate: float, search_radius: float, iter_max: int,
                 rng: Optional[np.random.Generator] = None):
        self.start = np.asarray(start, np.float64)
        self.goal = np.asarray(goal, np.float64)
        obs = np.asarray(obstacles, np.float64).reshape(-1, 3)
        self.centres = obs[:, :2]
        self.radii = obs[:, 2] + delta           # the reference inflates each disc by delta
        self.x_range, self.y_range = tuple(x_range), tuple(y_range)
        self.delta = float(delta)
        self.step_len = float(step_len)
        self.goal_rate = float(goal_sample_rate)
        self.search_radius = float(search_radius)
        self.iter_max = int(iter_max)
        self.rng = rng if rng is not None else np.random.default_rng(0)
        n = self.iter_max + 2
        self.xy = np.zeros((n, 2))
        self.parent = np.full(n, -1, np.int64)
        self.cost = np.zeros(n)
        self.n = 0

    # ------------------------------------------------------------------ geometry
    def in_obstacle(self, p: np.ndarray) -> bool:
        if len(self.centres) and np.any(np.linalg.norm(self.centres - p, axis=1) <= self.radii):
            return True
        (x0, x1), (y0, y1) = self.x_range, self.y_range
        d = self.delta
        return not (x0 + d <= p[0] <= x1 - d and y0 + d <= p[1] <= y1 - d)

    def collides(self, a: np.ndarray, b: np.ndarray) -> bool:
        if self.in_obstacle(a) or self.in_obstacle(b):
            return True
        if len(self.centres):
            return bool(np.any(_seg_disc_dist(a, b, self.centres) <= self.radii))
        return False

    # ------------------------------------------------------------------ tree
    def _add(self, p, parent: int, cost: float) -> int:
        i = self.n
        self.xy[i] = p
        self.parent[i] = parent
        self.cost[i] = cost
        self.n += 1
        return i

    def _sample(self) -> np.ndarray:
        if self.rng.random() < self.goal_rate:
            return self.goal
        d = self.delta
        return np.array([self.rng.uniform(self.x_range[0] + d, self.x_range[1] - d),
                         self.rng.uniform(self.y_range[0] + d, self.y_range[1] - d)])

    def _near(self, p: np.ndarray) -> np.ndarray:
        n = self.n + 1
        r = min(self.search_radius * np.sqrt(np.log(n) / n), self.step_len)
        d = np.linalg.norm(self.xy[:self.n] - p, axis=1)
        return np.nonzero(d <= r)[0]

    def _propagate(self, root: int, delta_cost: float):
        """Shift the cost of every descendant of ``root`` by ``delta_cost`` (after a rewire)."""
        frontier = np.array([root])
        while frontier.size:
            kids = np.nonzero(np.isin(self.parent[:self.n], frontier))[0]
            self.cost[kids] += delta_cost
            frontier = kids

    def plan(self) -> Plan:
        self._add(self.start, -1, 0.0)
        if self.in_obstacle(self.start):
            return Plan([tuple(self.goal), tuple(self.start)], False, self.xy[:self.n].copy(),
                        self.parent[:self.n].copy())
        for _ in range(self.iter_max):
            q = self._sample()
            dists = np.linalg.norm(self.xy[:self.n] - q, axis=1)
            i_near = int(np.argmin(dists))
            p_near = self.xy[i_near]
            d = dists[i_near]
            if d < 1e-12:
                continue
            p_new = p_near + (q - p_near) * (min(self.step_len, d) / d)
            if self.collides(p_near, p_new):
                continue
            near = self._near(p_new)
            # choose the cheapest collision-free parent among the neighbours
            best, best_cost = i_near, self.cost[i_near] + np.linalg.norm(p_new - p_near)
            if near.size:
                cand = self.cost[near] + np.linalg.norm(self.xy[near] - p_new, axis=1)
                for j in near[np.argsort(cand)]:
                    c = self.cost[j] + np.linalg.norm(self.xy[j] - p_new)
                    if c >= best_cost:
                        break
                    if not self.collides(self.xy[j], p_new):
                        best, best_cost = int(j), c
                        break
            k = self._add(p_new, best, best_cost)
            # rewire neighbours through the new vertex when that is shorter
            for j in near:
                if j == best:
                    continue
                c = best_cost + np.linalg.norm(self.xy[j] - p_new)
                if c < self.cost[j] - 1e-12 and not self.collides(p_new, self.xy[j]):
                    delta_c = c - self.cost[j]
                    self.parent[j] = k
                    self.cost[j] = c
                    self._propagate(int(j), delta_c)
        return self._extract()

    def _extract(self) -> Plan:
        xy = self.xy[:self.n]
        d = np.linalg.norm(xy - self.goal, axis=1)
        cand = np.nonzero(d <= self.step_len)[0]
        best, best_cost = -1, np.inf
        for j in cand[np.argsort(self.cost[cand] + d[cand])]:
            if not self.collides(xy[j], self.goal):
                best, best_cost = int(j), self.cost[j] + d[j]
                break
        if best < 0:
            return Plan([tuple(self.goal), tuple(self.start)], False, xy.copy(), self.parent[:self.n].copy())
        path = [tuple(self.goal)]
        j = best
        while j >= 0:
            path.append(tuple(xy[j]))
            j = int(self.parent[j])
        return Plan(path, True, xy.copy(), self.parent[:self.n].copy())


def shortest_path(xy_start, xy_goal, x_range, y_range, obstacle_xy, obstacle_widths, delta: float,
                  step_length: float, goal_sample_rate: float, search_radius: float, iter_max: int,
                  boundary_width: float = 0.01, rng: Optional[np.random.Generator] = None,
                  raise_on_failure: bool = False, shortcut: bool = True):
    """(path goal->start, success) -- the contract of the reference's ``get_shortest_path_no_collisions``
    (``rrt_star.py:25-87``): the box walls are ``boundary_width`` thick, and a failed search returns the
    direct segment so the caller can "just try it" and replan later.  ``shortcut`` (not in the reference)
    straightens the tree path by line-of-sight jumps."""
    obstacles = [(float(x), float(y), float(w)) for (x, y), w in zip(obstacle_xy, obstacle_widths)]
    # walls of thickness boundary_width sit on the range edges: shrink the free box by it
    xr = (x_range[0] + boundary_width, x_range[1])
    yr = (y_range[0] + boundary_width, y_range[1])
    planner = RRTStar(xy_start, xy_goal, obstacles, xr, yr, delta, step_length, goal_sample_rate, search_radius,
                      iter_max, rng)
    plan = planner.plan()
    if not plan.success and raise_on_failure:
        raise ValueError("RRT*: no collision-free path found")
    path = plan.path
    if plan.success and shortcut:
        path = shortcut_path(path, planner.collides, step_length)
    return path, plan.success


def shortcut_path(path, collides, max_seg: float):
    """Greedy line-of-sight shortcutting of a goal->start path (keeps the endpoints; segments are re-split to
    at most ``max_seg`` so the oracle still gets closely spaced subgoals).  With the RRT* budget the oracle
    uses, raw paths are 10-30 % longer than needed; this removes most of that."""
    pts = [np.asarray(p, np.float64) for p in path]
    out = [pts[0]]
    i = 0
    while i < len(pts) - 1:
        j = len(pts) - 1
        while j > i + 1 and collides(pts[i], pts[j]):
            j -= 1
        out.append(pts[j])
        i = j
    res = [tuple(out[0])]
    for a, b in zip(out[:-1], out[1:]):
        k = max(1, int(np.ceil(np.linalg.norm(b - a) / max_seg)))
        res.extend(tuple(a + (b - a) * (t / k)) for t in range(1, k + 1))
    return res


def path_length(path: Sequence[Tuple[float, float]]) -> float:
    p = np.asarray(path, np.float64)
    return float(np.linalg.norm(np.diff(p, axis=0), axis=1).sum()) if len(p) > 1 else 0.0


def filter_subgoals(path: Sequence[Tuple[float, float]], min_distance: float) -> List[np.ndarray]:
    """start->goal waypoints at least ``min_distance`` apart, always ending at the goal
    (``push_oracle_rrt_slowdown.py:79-92``)."""
    pts = [np.asarray(p, np.float64) for p in reversed(list(path))]   # start ... goal
    if not pts:
        return []
    out = [pts[0]]
    for p in pts[1:-1]:
        if np.linalg.norm(p - out[-1]) >= min_distance:
            out.append(p)
    out.append(pts[-1])
    return out[1:] if len(out) > 1 else out


def render_plan(plan: Plan, start, goal, obstacles, x_range, y_range, size: int = 256) -> np.ndarray:
    """RGB uint8 debug image of a plan (``oracles/plot.py`` role, no matplotlib): obstacles grey, tree edges
    light blue, the path red, start green, goal blue."""
    img = np.full((size, size, 3), 255, np.uint8)
    sx = (size - 1) / (x_range[1] - x_range[0])
    sy = (size - 1) / (y_range[1] - y_range[0])

    def px(p):
        return int(round((p[1] - y_range[0]) * sy)), int(round((p[0] - x_range[0]) * sx))   # (col, row)

    yy, xx = np.mgrid[0:size, 0:size]
    wx = x_range[0] + yy / sx
    wy = y_range[0] + xx / sy
    for (ox, oy, w) in obstacles:
        img[(wx - ox) ** 2 + (wy - oy) ** 2 <= w ** 2] = (150, 150, 150)

    def line(a, b, color):
        (c0, r0), (c1, r1) = px(a), px(b)
        n = max(abs(c1 - c0), abs(r1 - r0), 1)
        t = np.linspace(0.0, 1.0, n + 1)
        cs = np.clip(np.round(c0 + (c1 - c0) * t).astype(int), 0, size - 1)
        rs = np.clip(np.round(r0 + (r1 - r0) * t).astype(int), 0, size - 1)
        img[rs, cs] = color

    for j in range(1, len(plan.tree_xy)):
        if plan.tree_parent[j] >= 0:
            line(plan.tree_xy[plan.tree_parent[j]], plan.tree_xy[j], (170, 200, 240))
    for a, b in zip(plan.path[:-1], plan.path[1:]):
        line(a, b, (220, 30, 30))
    for p, color in ((start, (30, 160, 60)), (goal, (40, 60, 220))):
        c, r = px(p)
        img[max(r - 2, 0):r + 3, max(c - 2, 0):c + 3] = color
    return img
