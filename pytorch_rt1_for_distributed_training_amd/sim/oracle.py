"""Scripted push oracle for the planar Language-Table board.

Reference: ``language_table/environments/oracles/oriented_push_oracle.py:44-240`` (a move-behind / approach /
push state machine) and the RRT* push oracle the eval driver uses to reject start boards it cannot solve
(``push_oracle_rrt_slowdown.py``, ``main_rt1.py:162-172``).  The planar world has no obstacle-dependent
dynamics worth an RRT search, so one state machine serves both roles:

  move_to_pre_block: go to 5 cm behind the block on the block->target line, orbiting the block on a 4 cm
                     clearance circle when the straight path would touch it;
  move_to_block:     approach to 3 cm behind it;
  push_block:        push through a point 1 cm behind it; fall back to move_to_pre_block whenever the
                     effector drifts off the push line.
Speeds are per-second (0.3 / 0.35 m/s) scaled by the env's control frequency, as in the reference.
``plan_succeeds`` rolls the oracle out on a copy of the env state: the eval-time "can the oracle solve it"
check.

``RRTPushOracle`` adds the reference's obstacle awareness on top of the same state machine: an RRT* route for the
block around the other blocks (``sim/rrt_star.py``), an RRT* effector approach, per-subgoal slowdown and replanning.
"""
from __future__ import annotations

import numpy as np

from . import board, rrt_star


class PushOracle:
    def __init__(self, env, action_noise_std: float = 0.0, seed: int = 0):
        self._env = env
        self._noise = action_noise_std
        self._rs = np.random.RandomState(seed)
        self.phase = "move_to_pre_block"

    def reset(self):
        self.phase = "move_to_pre_block"

    def action(self) -> np.ndarray:
        env = self._env
        block, target = env.oracle_target
        w = env.world
        xy_block = w.pos[w.index[block]]
        xy_ee = w.effector_target
        if target is None or env.is_point_task:  # point tasks: go to the block
            return self._limit(xy_block - xy_ee, 0.35)
        delta, speed = self._push_toward(xy_block, target, xy_ee)
        if self._noise:
            delta = delta + self._rs.randn(2) * self._noise
        return self._limit(delta, speed)

    def _pre_block_step(self, xy_ee, pre, xy_block, speed):
        return _orbit(xy_ee, pre, xy_block, speed / self._env.get_control_frequency())

    def _push_toward(self, xy_block, target, xy_ee):
        """(delta, speed) of the move-behind / approach / push state machine for pushing the block at
        ``xy_block`` towards ``target``."""
        to_target = target - xy_block
        dist = np.linalg.norm(to_target)
        if dist < 1e-6:
            return np.zeros(2), 0.35
        u = to_target / dist
        lo, hi = board.WORKSPACE_BOUNDS
        pre = np.clip(xy_block - u * 0.05, lo, hi)    # the effector cannot leave the workspace
        nxt = np.clip(xy_block - u * 0.03, lo, hi)
        touch = xy_block - u * 0.01
        speed = 0.35
        delta = np.zeros(2)
        if self.phase == "move_to_pre_block":
            speed = 0.3
            delta = pre - xy_ee
            if np.linalg.norm(delta) < 0.004:
                self.phase = "move_to_block"
            else:
                delta = self._pre_block_step(xy_ee, pre, xy_block, speed)
        if self.phase == "move_to_block":
            delta = nxt - xy_ee
            if np.linalg.norm(delta) < 0.004:
                self.phase = "push_block"
        if self.phase == "push_block":
            off_line = np.linalg.norm((xy_ee - xy_block) - np.dot(xy_ee - xy_block, u) * u)
            if off_line > 0.02:
                self.phase = "move_to_pre_block"
            delta = touch - xy_ee
        return delta, speed

    def _limit(self, delta, speed) -> np.ndarray:
        max_step = speed / self._env.get_control_frequency()
        n = np.linalg.norm(delta)
        if n > max_step:
            delta = delta / n * max_step
        return np.asarray(delta, np.float32)


class RRTPushOracle(PushOracle):
    """Obstacle-aware push oracle (``push_oracle_rrt_slowdown.py:95-731``): RRT* routes the block around the
    other blocks (``sim.rrt_star``), the block is pushed subgoal by subgoal (advance within 2.5 cm), the
    effector's approach to the pre-push point is planned around the blocks too, pushes slow down near each
    subgoal (0.2-0.6x inside 2-10 cm), and a failed plan is retried every ``replan_every`` steps while the
    oracle pushes straight at the target.  For relative-location targets that sit next to a block the plan
    backs off along the block->target line (1.1-1.5x) and appends the true target."""

    SUBGOAL_ADVANCE = 0.025
    EE_SUBGOAL_ADVANCE = 0.01
    X_RANGE = (board.X_MIN - 0.04, board.X_MAX + 0.04)
    Y_RANGE = (board.Y_MIN - 0.04, board.Y_MAX + 0.04)

    def __init__(self, env, action_noise_std: float = 0.0, seed: int = 0, replan_every: int = 10,
                 use_ee_planner: bool = True, slowdown_freespace: bool = False, iter_max: int = 1024,
                 ee_iter_max: int = 512):
        super().__init__(env, action_noise_std, seed)
        self._rng = np.random.default_rng(seed)
        self._replan_every = replan_every
        self._use_ee = use_ee_planner
        self._slow_free = slowdown_freespace
        self._iter_max, self._ee_iter_max = iter_max, ee_iter_max
        self.reset()

    def reset(self):
        super().reset()
        self._subgoals = None
        self._need_replan = False
        self._counter = 0
        self._ee_plan = None
        self._ee_goal = None
        self.plan_success = None

    # ------------------------------------------------------------------ planning
    def _obstacles(self, exclude):
        w = self._env.world
        keep = [i for i in range(len(w.names)) if w.active[i] and
                all(np.linalg.norm(w.pos[i] - e) > 1e-5 for e in exclude)]
        return w.pos[keep].copy(), 2 * w.radius[keep]

    def _plan_block(self, xy_block, target):
        obs_xy, obs_w = self._obstacles([xy_block, target])
        kw = dict(x_range=self.X_RANGE, y_range=self.Y_RANGE, obstacle_xy=obs_xy, obstacle_widths=obs_w,
                  delta=0.015, step_length=0.05, goal_sample_rate=0.1, search_radius=0.5,
                  iter_max=self._iter_max, rng=self._rng)
        path, ok = rrt_star.shortest_path(xy_block, target, **kw)
        if not ok and len(obs_xy):
            # target next to a block (block-to-block-relative tasks): back off along block -> target
            d = np.linalg.norm(obs_xy - target, axis=1)
            j = int(np.argmin(d))
            if d[j] < 0.12:
                for scale in (1.1, 1.2, 1.3, 1.4, 1.5):
                    alt = obs_xy[j] + (target - obs_xy[j]) * scale
                    p2, ok = rrt_star.shortest_path(xy_block, alt, **kw)
                    if ok:
                        path = [tuple(target)] + list(p2)
                        break
        self._need_replan = not ok
        self.plan_success = ok
        self._subgoals = rrt_star.filter_subgoals(path, self.SUBGOAL_ADVANCE)

    def _pre_block_step(self, xy_ee, pre, xy_block, speed):
        step = speed / self._env.get_control_frequency()
        if not self._use_ee:
            return super()._pre_block_step(xy_ee, pre, xy_block, speed)
        # replan the effector route when the pre-push point moved (slight contacts shift it)
        if self._ee_goal is None or np.linalg.norm(self._ee_goal - pre) > 0.01:
            self._ee_goal = pre.copy()
            obs_xy, _ = self._obstacles([])
            blocked = len(obs_xy) and np.any(rrt_star._seg_disc_dist(xy_ee, pre, obs_xy) < 0.03)
            self._ee_plan = None
            if blocked:
                path, ok = rrt_star.shortest_path(
                    xy_ee, pre, self.X_RANGE, self.Y_RANGE, obs_xy, [0.02] * len(obs_xy), delta=0.01,
                    step_length=0.025, goal_sample_rate=0.1, search_radius=0.5, iter_max=self._ee_iter_max,
                    rng=self._rng)
                if ok:
                    self._ee_plan = rrt_star.filter_subgoals(path, self.EE_SUBGOAL_ADVANCE)
        if self._ee_plan:
            while len(self._ee_plan) > 1 and np.linalg.norm(self._ee_plan[0] - xy_ee) < self.EE_SUBGOAL_ADVANCE:
                self._ee_plan.pop(0)
            if len(self._ee_plan) > 1:        # the planned route already clears every block: go straight
                d = self._ee_plan[0] - xy_ee
                n = np.linalg.norm(d)
                return d if n <= step else d / n * step
            self._ee_plan = None
        return _orbit(xy_ee, pre, xy_block, step)

    # ------------------------------------------------------------------ control
    def action(self) -> np.ndarray:
        env = self._env
        block, target = env.oracle_target
        if target is None or env.is_point_task:
            return super().action()
        w = env.world
        xy_block = w.pos[w.index[block]].copy()
        xy_ee = w.effector_target
        if self._subgoals is None:
            self._plan_block(xy_block, target)
        self._counter += 1
        if self._need_replan and self._counter % self._replan_every == 0:
            self._plan_block(xy_block, target)
        self._subgoals[-1] = np.asarray(target, np.float64)   # a block target may have moved
        while len(self._subgoals) > 1 and np.linalg.norm(xy_block - self._subgoals[0]) <= self.SUBGOAL_ADVANCE:
            self._subgoals.pop(0)
        sub = self._subgoals[0]
        free = self.phase == "move_to_pre_block"
        delta, speed = self._push_toward(xy_block, sub, xy_ee)
        if self._noise:
            delta = delta + self._rs.randn(2) * self._noise
        max_step = speed / env.get_control_frequency()
        if not free or self._slow_free:
            dist = np.linalg.norm(sub - xy_block)
            for thresh, slow in ((0.02, 0.2), (0.04, 0.3), (0.06, 0.4), (0.08, 0.5), (0.1, 0.6)):
                if dist < thresh:
                    max_step *= slow
                    break
        n = np.linalg.norm(delta)
        if n > max_step:
            delta = delta / n * max_step
        return np.asarray(delta, np.float32)


def _orbit(ee, goal, block, step, clear: float = 0.04):
    """Step towards ``goal`` without touching the block: inside the clearance circle, move along it (the
    shorter way round) while pushing back out to the clearance radius."""
    d = goal - ee
    n = np.linalg.norm(d)
    if n < 1e-9:
        return d
    move = d / n * min(n, step)
    r = ee - block
    rn = np.linalg.norm(r)
    if np.linalg.norm(ee + move - block) >= clear or rn < 1e-9:
        return move
    g = goal - block
    diff = (np.arctan2(g[1], g[0]) - np.arctan2(r[1], r[0]) + np.pi) % (2 * np.pi) - np.pi
    tangent = np.sign(diff) * np.array([-r[1], r[0]]) / rn
    return tangent * min(step, abs(diff) * clear) + r / rn * max(0.0, clear - rn)


def plan_succeeds(env, max_steps: int = 80, oracle_cls=None) -> bool:
    """Roll the oracle out from the env's current state and restore it; True if the task gets solved."""
    saved = env.get_state()
    rc = env._reward_calculator
    zone = getattr(rc, "_in_reward_zone_steps", 0)
    oracle = (oracle_cls or PushOracle)(env)
    ok = False
    try:
        for _ in range(max_steps):
            _, _, done, _ = env.step(oracle.action())
            if done:
                ok = True
                break
    finally:
        env.set_state(saved)
        if rc is not None:
            rc._in_reward_zone_steps = zone
    return ok
