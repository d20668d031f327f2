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
"""
from __future__ import annotations

import numpy as np


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
            delta = xy_block - xy_ee
            return self._limit(delta, 0.35)
        to_target = target - xy_block
        dist = np.linalg.norm(to_target)
        if dist < 1e-6:
            return np.zeros(2, np.float32)
        u = to_target / dist
        pre = xy_block - u * 0.05
        nxt = xy_block - u * 0.03
        touch = xy_block - u * 0.01
        speed = 0.35
        if self.phase == "move_to_pre_block":
            speed = 0.3
            delta = pre - xy_ee
            if np.linalg.norm(delta) < 0.004:
                self.phase = "move_to_block"
            else:
                delta = _orbit(xy_ee, pre, xy_block, speed / self._env.get_control_frequency())
        if self.phase == "move_to_block":
            delta = nxt - xy_ee
            if np.linalg.norm(delta) < 0.004:
                self.phase = "push_block"
        if self.phase == "push_block":
            off_line = np.linalg.norm((xy_ee - xy_block) - np.dot(xy_ee - xy_block, u) * u)
            if off_line > 0.02:
                self.phase = "move_to_pre_block"
            delta = touch - xy_ee
        if self._noise:
            delta = delta + self._rs.randn(2) * self._noise
        return self._limit(delta, speed)

    def _limit(self, delta, speed) -> np.ndarray:
        max_step = speed / self._env.get_control_frequency()
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


def plan_succeeds(env, max_steps: int = 80) -> bool:
    """Roll the oracle out from the env's current state and restore it; True if the task gets solved."""
    saved = env.get_state()
    rc = env._reward_calculator
    zone = getattr(rc, "_in_reward_zone_steps", 0)
    oracle = PushOracle(env)
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
