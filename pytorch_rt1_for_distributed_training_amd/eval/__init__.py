"""Closed-loop evaluation: RT-1 policy wrapper, env wrappers, rollout loop."""
from .envs import (CentralCropResize, History, SimEnvAdapter, ToyPushEnv, make_language_table_env,  # noqa: F401
                   make_sim_env)
from .policy import RT1Policy  # noqa: F401
from .rollout import evaluate, save_gif  # noqa: F401
