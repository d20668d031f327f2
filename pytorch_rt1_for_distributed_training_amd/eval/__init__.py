"""Closed-loop evaluation: RT-1 policy wrapper, env wrappers, rollout loop."""
from .envs import CentralCropResize, History, ToyPushEnv, make_language_table_env  # noqa: F401
from .policy import RT1Policy  # noqa: F401
from .rollout import evaluate, save_gif  # noqa: F401
